#!/bin/bash
# inflate2 tuning sweep: HSDS_INFLATE_TUNE="W,rounds,over16" over the headline legs (F1, F2)
set -o pipefail
mkdir -p gpurun_out
for t in ${TUNES:-"384,4,1" "256,4,1" "192,8,1" "512,4,1" "384,4,0" "384,4,2" "384,8,1"}; do
  HSDS_INFLATE_TUNE=$t timeout -k 10 120 python bench.py --steps 4 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 > gpurun_out/tune_$t.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "tune $t rc=$rc"; tail -3 gpurun_out/tune_$t.log; exit $rc; }
  grep -v amdgpu.ids gpurun_out/tune_$t.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', 'F1', d['value'], d['roofline']['kernel_ms'], '| F2', d['f2']['value'], d['f2']['inflate_kernel_ms'])"
done
