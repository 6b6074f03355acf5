#!/bin/bash
# round 5: F1 and F2 (one wave per stream) phase profiles of the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HZ_PROF_F2W1=1 HZ_PROF_LZ=0 HZ_PROF_LIB=$GRAFT_REPO_ROOT/abtmp/prof_fuse.so timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_f2.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ph_f2.log; exit $rc
