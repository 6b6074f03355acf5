#!/bin/bash
# one GPU call of evidence for the current build: the given GPU tests, the inflate phase
# profile (HZ_PROFILE build), SQ counter passes at the bench configuration and the HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE).  Usage: tools/gpu_evidence.sh "<pytest files>" [tag]
set -o pipefail
TAG=${2:-r3}
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest $1 -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ev_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ev_tests.log; [ $rc -eq 0 ] || exit $rc
fi
HZ_PROF_LZ=0 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sq_bench.sh sq_$TAG || exit 1
for d in gpurun_out/sq_$TAG/p*; do python3 tools/pmc_sum.py $d; done
CFG3=${CFG3:-0} RND=$TAG bash tools/pmc_traffic.sh
