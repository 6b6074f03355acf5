#!/bin/bash
# one GPU call: parity tests, phase profile, headline bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -3
exit $rc
