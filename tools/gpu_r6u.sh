#!/bin/bash
# round 6: phase shares of the zstd decoder after the literal change (HZ_PROFILE build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HZ_PROF_ZSTD=1 HZ_PROF_LZ=0 HZ_PROF_N1=64 HZ_PROF_N2=16 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase_zstd.log 2>&1 || { tail gpurun_out/phase_zstd.log; exit 1; }
grep -v amdgpu gpurun_out/phase_zstd.log | tail -30
