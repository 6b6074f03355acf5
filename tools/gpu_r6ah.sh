#!/bin/bash
# round 6: the shipped build with non-temporal record loads -- GPU tests, traffic passes, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
RND=r6 bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1; rc=$?; grep bytes_per_launch gpurun_out/traffic/traffic.json; [ $rc -eq 0 ] || exit $rc
