#!/bin/bash
# rocprofv3 kernel statistics of the bench's cfg5 encode legs (zlib / lz4 / zstd / bitshuffle)
set -o pipefail
mkdir -p gpurun_out
R="$(pwd)"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/encprof" -o enc -- \
  python3 "$R/bench.py" --headline 0 --steps 3 --warmup 1 --cpu-seconds 0 --cfg3 0 --cfg1 0 --cfg5 1 --cfg4-full 0 --f2 0 --e2e 0 --lz4 0 --zstd 0 --bshuf 0 --cfg5w 0 --cfg4 0 \
  > "$R/gpurun_out/enc_prof.log" 2>&1
rc=$?; echo "enc rocprof rc=$rc"; tail -1 "$R/gpurun_out/enc_prof.log"
exit $rc
