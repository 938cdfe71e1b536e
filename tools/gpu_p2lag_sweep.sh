#!/bin/bash
# configs[4]'s pass-2 lag (tile rows between a row's pass 1 and its pass 2 in the merged
# two-pass schedule): an SO_AB build reads SO_P2LAG; interleaved with the default library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lag in default ${LAGS:-14 20 32 40}; do
    if [ $lag = default ]; then lib=""; else lib=tools/_ab/ab_env.so; fi
    SO_LIB_PATH=$lib SO_P2LAG=$([ $lag = default ] || echo $lag) timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie \
        --no-records --no-parity --config 4k_rc2pass --kernel-reps 10 --detail-out '' > gpurun_out/p2lag_run.log 2>&1 \
        || { tail -3 gpurun_out/p2lag_run.log; exit 1; }
    echo "$rep lag=$lag $(tail -1 gpurun_out/p2lag_run.log | grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/p2lag.log
  done
done
