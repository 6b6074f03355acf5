#!/bin/bash
# round 5: fused A+E -- parity, A/B against the unfused build, phase profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/f3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f3_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/fuse.so abtmp/fuse_w3.so abtmp/fuse.so abtmp/fuse_w3.so || exit 1
exit 0
rc=$?; grep -v amdgpu gpurun_out/ph_fuse.log | head -20; exit $rc
