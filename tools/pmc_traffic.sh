#!/bin/bash
# HBM traffic: two separate --pmc passes (FETCH_SIZE, WRITE_SIZE; they do not fit one
# TCC pass) over the headline bench workload, then over the cfg3 leg alone, no tracing
# domains.  Writes gpurun_out/traffic/traffic.json and traffic_cfg3.json
# (tools/save_profiles.sh copies them to profiles/, where bench.py reads them).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RND=${RND:-r2}
OUT=$R/gpurun_out/traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
OFF="--cpu-seconds 0 --f2 0 --e2e 0 --cfg5 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0"
ARGS="--steps 1 --warmup 1 --cfg3 0 $OFF"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
  python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
  python3 $R/bench.py $ARGS > $OUT/write.log 2>&1
rc=$?; echo "write pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/traffic_parse.py $OUT $RND > $OUT/traffic.json && cat $OUT/traffic.json || exit 1
[ "${CFG3:-1}" = "1" ] || exit 0
A3="--steps 1 --warmup 1 --headline 0 --cfg3 1 $OFF"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch3 -o fetch -- \
  python3 $R/bench.py $A3 > $OUT/fetch3.log 2>&1
rc=$?; echo "cfg3 fetch pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write3 -o write -- \
  python3 $R/bench.py $A3 > $OUT/write3.log 2>&1
rc=$?; echo "cfg3 write pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/traffic_parse.py $OUT $RND cfg3 > $OUT/traffic_cfg3.json && cat $OUT/traffic_cfg3.json
