#!/bin/bash
# round 5: one-pass decoder for NW = 1 only -- parity (pipe + codec), F1/F2 A/B, latency
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/f4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f4_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/fuse.so abtmp/split.so || exit 1
timeout -k 10 300 python tools/latency.py > gpurun_out/latency_split.json 2> gpurun_out/latency_split.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/latency_split.json'))
for f in ('F1','F2'): print(f, {k:v for k,v in d[f].items()})
"
