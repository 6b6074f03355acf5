#!/bin/bash
# round 6: phase profile of the current build (batch F1, F2 with one wavefront per stream)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HZ_PROF_F2W1=1 HZ_PROF_LZ=0 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase_r6.log 2>&1
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase_r6.log; exit $rc
