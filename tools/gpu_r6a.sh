#!/bin/bash
# round 6: GPU tests of the tree, header / table-build marginal cost A/B, lone-chunk phase profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh abtmp/base.so abtmp/hdr2.so abtmp/tb2.so abtmp/base.so abtmp/hdr2.so abtmp/tb2.so || exit 1
HZ_PROF_LONE=1 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase_lone.log 2>&1
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase_lone.log; [ $rc -eq 0 ] || exit $rc
bash tools/cfg5w_split.sh
