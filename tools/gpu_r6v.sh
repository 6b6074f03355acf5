#!/bin/bash
# round 6: the zstd FSE walk with the stage dwords read alongside the table entries
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_datanode.py tests/test_gpu_encode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_zstd.sh abtmp/zwalk2.so abtmp/zwalk4.so abtmp/zwalk2.so abtmp/zwalk4.so || exit 1
