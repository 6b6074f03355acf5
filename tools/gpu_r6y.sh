#!/bin/bash
# round 6: the parse staging's adler sums by byte dot products -- encode tests, encoder A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_write.py tests/test_gpu_datanode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_enc5.sh abtmp/enc_old.so abtmp/enc_dot.so abtmp/enc_old.so abtmp/enc_dot.so || exit 1
