#!/bin/bash
# round 6 final check on the final tree: GPU tests, smoke, a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_final.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench_final.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
