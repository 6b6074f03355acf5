#!/bin/bash
# round 5: skewed parse lane ranges -- encode parity (GPU streams = emulator), cfg5 writer A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/enc_skew.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/e1_tests.log 2>&1
rc=$?; tail -2 gpurun_out/e1_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_enc5.sh abtmp/enc_noskew.so abtmp/enc_skew.so abtmp/enc_noskew.so abtmp/enc_skew.so
