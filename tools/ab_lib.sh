#!/bin/bash
# bench A/B: the default library vs each tools/_ab/*.so (SO_LIB_PATH), 4K and 1080p.
cd "$GRAFT_REPO_ROOT" || exit 1
shopt -s nullglob
for cfg in ${CFGS:-4k 1080p}; do
 for rep in $(seq ${REPS:-1}); do
  for lib in "" tools/_ab/*.so; do
    SO_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --kernel-reps 10 > gpurun_out/ab_$cfg.log 2>&1 || { tail -3 gpurun_out/ab_$cfg.log; exit 1; }
    echo "$cfg lib=${lib:-default} $(grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*' gpurun_out/ab_$cfg.log | tr '\n' ' ')"
  done
 done
done
