#!/bin/bash
# A/B of builds on the lz4 leg: LZ parity tests gate each lib, then bench (F1 + lz4)
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "lz4 or other_blosc" \
    --timeout 200 --timeout-method thread > gpurun_out/abl_$(basename $lib).log 2>&1
  rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/abl_$(basename $lib).log)"; [ $rc -eq 0 ] || exit $rc
  HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 \
    > gpurun_out/ablb_$(basename $lib).log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -3 gpurun_out/ablb_$(basename $lib).log; exit $rc; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/ablb_$(basename $lib).log').read().strip().splitlines()[-1]); print('$lib', 'LZ4', d['lz4']['value'], 'GB/s', d['lz4']['lz_kernel_ms'], 'ms')"
done
