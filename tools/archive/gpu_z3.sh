#!/bin/bash
# round 5: LZ4 / BloscLZ wave priority A/B (lz GPU tests of one variant first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/lz32.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "lz or blosclz or codec" --timeout 200 --timeout-method thread > gpurun_out/z3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/z3_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_dec.sh abtmp/lz0.so abtmp/lz16.so abtmp/lz32.so abtmp/lz0.so abtmp/lz16.so abtmp/lz32.so
