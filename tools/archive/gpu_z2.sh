#!/bin/bash
# round 5: zstd wave priority A/B and the shuffled streams' warm-up (W2) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/w2_1024.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_pipe.py > gpurun_out/z2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/z2_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/w2_0.so abtmp/w2_1024.so abtmp/w2_1280.so abtmp/w2_0.so abtmp/w2_1024.so abtmp/w2_1280.so || exit 1
tools/ab_dec.sh abtmp/zs0.so abtmp/zs16.so abtmp/zs32.so abtmp/zs64.so abtmp/zs0.so abtmp/zs16.so abtmp/zs32.so
