#!/bin/bash
# rocprofv3 kernel trace of the headline run only, then the two PMC traffic passes
set -o pipefail
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --kernel-timing 1 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 > "$R/gpurun_out/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && bash tools/pmc_traffic.sh
