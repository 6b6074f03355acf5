#!/bin/bash
# round 5: A/B of inflate builds after the codec GPU tests of one of them
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/lbf.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_pipe.py > gpurun_out/f6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f6_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/fc16.so abtmp/lb3.so abtmp/lbf.so abtmp/fc16.so abtmp/lb3.so abtmp/lbf.so
