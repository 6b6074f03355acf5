#!/bin/bash
# round 5: fused A+E (HZ2_FUSE) -- GPU parity of the in-tree build, then F1/F2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/f1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f1_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/nofuse.so abtmp/fuse.so abtmp/nofuse.so abtmp/fuse.so
