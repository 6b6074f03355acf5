#!/bin/bash
# LZ parity tests + the bench's lz4 leg only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "lz4 or other_blosc" --timeout 200 --timeout-method thread \
  > gpurun_out/lzq_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/lzq_tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 > gpurun_out/lzq_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lzq_bench.log; exit $rc; }
python -c "
import json; d=json.loads(open('gpurun_out/lzq_bench.log').read().strip().splitlines()[-1]); print('F1', d['value'], 'LZ4', d['lz4'])"
