#!/bin/bash
# configs[4] sharded write: per-kernel split (rocprofv3 kernel trace + stats) of the aligned
# request alone, then of the aligned + (100,100)-offset requests (the offset one = the
# difference), cfg5 steps = 3 each after one warm-up
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
OFF="--headline 0 --cfg3 0 --cfg1 0 --cfg5 0 --cfg4 0 --cfg4-full 0 --cpu-seconds 0"
for v in full full,offset_100_100; do
  d=$R/gpurun_out/cfg5w_${v/,/_}
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --cfg5-steps 3 --cfg5w-variants $v $OFF > $d.log 2>&1
  rc=$?; echo "cfg5w $v rc=$rc"; grep -v amdgpu.ids $d.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
