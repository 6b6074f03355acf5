#!/bin/bash
# round 6: Huffman literal streams of the zstd decoder on every lane -- GPU tests, then the
# zstd decode leg A/B (one lane per stream vs all lanes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_zstd.sh abtmp/zser.so abtmp/zpar.so abtmp/zser.so abtmp/zpar.so || exit 1
