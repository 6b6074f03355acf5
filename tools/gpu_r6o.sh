#!/bin/bash
# round 6: cfg3 step anatomy (kernel trace of 3 steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3
cd /tmp && export TMPDIR=/tmp
OFF="--cpu-seconds 0 --f2 0 --e2e 0 --cfg5 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3 -o c3 -- \
    python3 $R/bench.py --steps 3 --warmup 1 --headline 0 $OFF --cfg3 1 > $R/gpurun_out/c3.log 2>&1
rc=$?; echo "cfg3 trace rc=$rc"; tail -c 600 $R/gpurun_out/c3.log; [ $rc -eq 0 ] || exit $rc
