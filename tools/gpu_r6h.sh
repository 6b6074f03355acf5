#!/bin/bash
# round 6: root pieces placed straight from the decoded chunks (PLAN_DIRECT): plan / selection
# tests, then the read legs (cfg1, cfg3, cfg4) without the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_selection.py tests/test_gpu_paged.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_sel_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_sel_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --headline 0 --f2 0 --e2e 0 --lz4 0 --bshuf 0 --zstd 0 --cfg5 0 --cfg5w 0 --cfg4-full 0 --copy-ceiling 0 --cpu-seconds 0 > gpurun_out/bench_read.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_read.log; [ $rc -eq 0 ] || exit $rc
