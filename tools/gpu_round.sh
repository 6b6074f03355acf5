#!/bin/bash
# one GPU call: parity tests, phase profile, headline bench, rocprofv3 kernel trace
# (each step time-limited; the script stops at the first failing step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
if [ "${HZ_PHASE:-1}" = "1" ]; then
  timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
  rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -3
[ $rc -eq 0 ] || exit $rc
if [ "${HZ_ROCPROF:-1}" = "1" ]; then
  R="$(pwd)"; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --kernel-timing 1 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 > "$R/gpurun_out/bench_prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/bench_prof.log" | tail -1
fi
exit $rc
