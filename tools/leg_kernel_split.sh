#!/bin/bash
# Per-kernel time split of one cfg3 step and one cfg4 step:
# rocprofv3 --kernel-trace --stats over the legs alone (headline off), summaries into
# gpurun_out/legsplit/{cfg3,cfg4}/ .  Then the FETCH/WRITE passes of both legs
# (tools/traffic_parse.py names every kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/legsplit
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
OFF="--cpu-seconds 0 --f2 0 --e2e 0 --cfg5 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg3 0"
for leg in cfg3 cfg4; do
  if [ $leg = cfg3 ]; then A="--headline 0 $OFF --cfg3 1"; else A="--headline 0 $OFF --cfg4 1 --cfg4-steps 1"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$leg -o $leg -- \
    python3 $R/bench.py --steps 1 --warmup 1 $A > $OUT/$leg.log 2>&1
  rc=$?; echo "$leg trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for leg in cfg3 cfg4; do
  n=${leg#cfg}
  if [ $leg = cfg3 ]; then A="--headline 0 $OFF --cfg3 1"; else A="--headline 0 $OFF --cfg4 1 --cfg4-steps 1"; fi
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch$n -o fetch -- \
    python3 $R/bench.py --steps 1 --warmup 1 $A > $OUT/fetch$n.log 2>&1
  rc=$?; echo "$leg fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write$n -o write -- \
    python3 $R/bench.py --steps 1 --warmup 1 $A > $OUT/write$n.log 2>&1
  rc=$?; echo "$leg write rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/traffic_parse.py $OUT ${RND:-r4} $leg > $OUT/traffic_$leg.json || exit 1
done
