#!/bin/bash
# Interleaved A/B of the default library against tools/_ab/*.so (SO_LIB_PATH) on the configs in
# CFGS, REPS rounds: one bench line per (round, library, config), ms per step and per-frame us.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
shopt -s nullglob
T=${TAG:-ab}
for rep in $(seq ${REPS:-3}); do
 for cfg in ${CFGS:-4k}; do
  for lib in "" tools/_ab/*.so; do
    SO_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-records --no-parity --config $cfg \
        --kernel-reps 10 --detail-out '' ${BENCH_ARGS} > gpurun_out/${T}_run.log 2>&1 || { tail -3 gpurun_out/${T}_run.log; exit 1; }
    echo "$rep $cfg lib=${lib:-default} $(tail -1 gpurun_out/${T}_run.log | grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${T}.log
  done
 done
done
