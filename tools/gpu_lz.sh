#!/bin/bash
# LZ iteration on the GPU box: LZ / bitshuffle GPU tests, LZ phase profile, lz4 + bshuf bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "lz or bshuf or blosclz or codec or splits" --timeout 200 --timeout-method thread > gpurun_out/gpu_lz.log 2>&1
rc=$?; echo "lz tests rc=$rc"; tail -2 gpurun_out/gpu_lz.log; [ $rc -eq 0 ] || exit $rc
HZ_PROF_N1=64 HZ_PROF_N2=16 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_lz.log 2>&1 || exit $?
grep -A4 "^LZ4" gpurun_out/ph_lz.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --zstd 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 > gpurun_out/b_lz.log 2>&1 || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/b_lz.log').read().strip().splitlines()[-1]); print('F1', d['value'], 'lz4', json.dumps(d.get('lz4'))[:200]); print('bshuf', json.dumps(d.get('bshuf'))[:200])"
