#!/bin/bash
# one iteration: GPU parity tests, phase profile (HZ_PROFILE build), headline bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
HZ_PROF_LZ=0 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_quick.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('F1', d['value'], 'GB/s', d['roofline']['kernel_ms'], 'ms frac', d['roofline']['frac'], '| F2', d['f2']['value'], d['f2']['inflate_kernel_ms'])"
exit $rc
