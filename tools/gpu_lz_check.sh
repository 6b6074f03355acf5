#!/bin/bash
# codec parity on the GPU (incl. lz4 / blosclz), then a bench run with the lz4 leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/lz_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/lz_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds 3 --e2e 0 --cfg3 0 --cfg5 0 > gpurun_out/lz_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/lz_bench.log | tail -2
exit $rc
