#!/bin/bash
# round 5: phase profiles and SQ passes of the fused (in-tree) and unfused builds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in fuse nofuse; do
  HZ_PROF_LZ=0 HZ_PROF_LIB=$GRAFT_REPO_ROOT/abtmp/prof_$v.so timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_$v.log 2>&1
  rc=$?; echo "== $v"; grep -v amdgpu gpurun_out/ph_$v.log | head -20; [ $rc -eq 0 ] || exit $rc
done
bash tools/sq_passes.sh F1 sqf || exit 1
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/nofuse.so bash tools/sq_passes.sh F1 sqn || exit 1
python tools/pmc_sum.py gpurun_out/sqf > gpurun_out/sqf.txt 2>&1; python tools/pmc_sum.py gpurun_out/sqn > gpurun_out/sqn.txt 2>&1
cat gpurun_out/sqf.txt gpurun_out/sqn.txt | grep -v "0 dispatches"
