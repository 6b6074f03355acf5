#!/bin/bash
# GPU parity tests, then the headline legs of the bench (F1 + F2) only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_quick.log | tail -2
exit $rc
