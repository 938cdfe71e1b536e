#!/bin/bash
# tools/gpu_traffic.sh over every record config (PMC traffic + VALU issue counters), one call;
# tools/traffic_json.py reduces each config on the box (the raw counter CSVs exceed what gpurun
# copies back), and the merged profiles/pmc_me_traffic.json comes back as
# gpurun_out/pmc_me_traffic.json.
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r06c}
for cfg in ${CFGS:-4k 1080p 4k_vbs 4k_rc2pass 4k_noise 4k_lowtex}; do
  bash tools/gpu_traffic.sh $T $cfg || exit $?
  python3 tools/traffic_json.py gpurun_out/traffic $T $cfg > gpurun_out/traffic_json_$cfg.log 2>&1 || exit $?
  rm -rf gpurun_out/traffic/${T}_${cfg}_*
done
cp profiles/pmc_me_traffic.json gpurun_out/pmc_me_traffic.json
rm -rf gpurun_out/traffic
