#!/bin/bash
# round 5: wave priority by remaining input (HZ2_PRIO_ABS KiB per level) against by output fraction
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/pabs24.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py > gpurun_out/f6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f6_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/base.so abtmp/pabs16.so abtmp/pabs24.so abtmp/pabs32.so abtmp/pabs40.so abtmp/base.so abtmp/pabs16.so abtmp/pabs24.so abtmp/pabs32.so abtmp/pabs40.so
