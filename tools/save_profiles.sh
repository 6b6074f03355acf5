#!/bin/bash
# copy the judged evidence of the last tools/gpu_round.sh (+ pmc_traffic.sh) call from
# gpurun_out/ into profiles/ (tracked).  Usage: tools/save_profiles.sh r1
set -e
cd "$(dirname "$0")/.."
R=${1:-r1}
[ -f gpurun_out/prof/run_kernel_stats.csv ] && cp gpurun_out/prof/run_kernel_stats.csv profiles/${R}_bench_kernel_stats.csv
[ -f gpurun_out/bench.log ] && grep -v amdgpu.ids gpurun_out/bench.log > profiles/${R}_bench.log
[ -f gpurun_out/phase.log ] && grep -v amdgpu.ids gpurun_out/phase.log > profiles/${R}_phase_profile.txt
if [ -f gpurun_out/traffic/traffic.json ]; then
  python3 - "$R" <<'PY'
import json, sys
r = sys.argv[1]
t = json.load(open("gpurun_out/traffic/traffic.json"))
json.dump(t, open(f"profiles/{r}_traffic.json", "w"), indent=1)
PY
  [ -f gpurun_out/traffic/traffic_cfg3.json ] && cp gpurun_out/traffic/traffic_cfg3.json profiles/${R}_traffic_cfg3.json
  mkdir -p profiles/${R}_pmc_traffic
  cp gpurun_out/traffic/fetch/*counter_collection.csv gpurun_out/traffic/write/*counter_collection.csv profiles/${R}_pmc_traffic/
fi
ls -la profiles/
