#!/bin/bash
# round 5: bitshuffle decoder wave priority A/B (bitshuffle GPU tests of one variant first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/bs128.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "bshuf or bitshuffle or lz" --timeout 200 --timeout-method thread > gpurun_out/z4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/z4_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_dec.sh abtmp/bs0.so abtmp/bs64.so abtmp/bs128.so abtmp/bs192.so abtmp/bs0.so abtmp/bs64.so abtmp/bs128.so abtmp/bs192.so
