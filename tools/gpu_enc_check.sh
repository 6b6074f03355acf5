#!/bin/bash
# GPU parity of the encode paths (zlib + lz4) and the DN write side
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_datanode.py tests/test_gpu_codec.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/enc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/enc_tests.log | tail -12
exit $rc
