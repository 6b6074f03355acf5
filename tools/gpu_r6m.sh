#!/bin/bash
# round 6: the 32-byte record groups as the default build -- GPU tests, smoke, the driver's bench
# command and the HBM traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
RND=r6 bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1; rc=$?; grep bytes_per_launch gpurun_out/traffic/traffic.json; [ $rc -eq 0 ] || exit $rc
