#!/bin/bash
# round 5: non-temporal emission stores -- parity of the variant, F1/F2 A/B, traffic A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/nt.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py > gpurun_out/f5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f5_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/base.so abtmp/nt.so abtmp/base.so abtmp/nt.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/base.so abtmp/nt.so
