#!/bin/bash
# round 6: eight wavefronts per stream in the window pipeline -- pipe tests, lone-chunk latency
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_pipe.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_pipe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/lone_ab.py > gpurun_out/lone8.txt 2>gpurun_out/lone8.err || { tail -3 gpurun_out/lone8.err; exit 1; }
cat gpurun_out/lone8.txt
