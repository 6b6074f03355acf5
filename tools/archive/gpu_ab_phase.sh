#!/bin/bash
# A/B of abtmp/base.so against the in-tree library (F1 / F2 legs) plus the phase profile
# of the in-tree HZ_PROFILE build (tools/libhsds_prof.so), after the codec GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh abtmp/base.so hsds_amd/libhsds_amd.so || exit 1
HZ_PROF_LZ=0 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_new.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ph_new.log; exit $rc
