#!/bin/bash
# HBM traffic of the headline inflate launch: two separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE; they do not fit one TCC pass) over the bench workload, no tracing domains.
# Writes gpurun_out/traffic/traffic.json (copy to profiles/ to have bench.py report it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --cpu-seconds 0 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --cfg5w 0 --cfg4 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
  python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
  python3 $R/bench.py $ARGS > $OUT/write.log 2>&1
rc=$?; echo "write pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/traffic_parse.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
