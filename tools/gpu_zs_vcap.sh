cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
 for cfg in 4k 1080p; do
  for zs in 0.5 0.0; do
   SO_ZERO_SKIP_SHARE=$zs timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-records --no-parity --config $cfg --kernel-reps 10 --detail-out '' > gpurun_out/zs_run.log 2>&1 || { tail -3 gpurun_out/zs_run.log; exit 1; }
   echo "$rep $cfg share=$zs $(tail -1 gpurun_out/zs_run.log | grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*\|"kernel": "[^"]*"' | tr '\n' ' ')" | tee -a gpurun_out/zs.log
  done
 done
done
CFGS="4k_vbs" REPS=2 TAG=vcap bash tools/gpu_ab_interleave.sh
