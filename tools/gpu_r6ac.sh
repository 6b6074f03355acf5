#!/bin/bash
# round 6: longest streams first (HZ2_LPT) -- GPU tests, A/B, tail profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh abtmp/lpt0.so abtmp/lpt1.so abtmp/lpt0.so abtmp/lpt1.so abtmp/lpt0.so abtmp/lpt1.so || exit 1
timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail.log 2>&1 || { tail gpurun_out/tail.log; exit 1; }
grep busy gpurun_out/tail.log
