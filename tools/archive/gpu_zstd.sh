#!/bin/bash
# zstd iteration on the GPU box: zstd GPU tests, phase profile (HZ_PROFILE build in
# abtmp/prof_cur.so), zstd bench leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "zstd" --timeout 200 --timeout-method thread > gpurun_out/gpu_zstd.log 2>&1
rc=$?; echo "zstd tests rc=$rc"; tail -2 gpurun_out/gpu_zstd.log; [ $rc -eq 0 ] || exit $rc
HZ_PROF_LIB=$(realpath abtmp/prof_cur.so) HZ_PROF_LZ=0 HZ_PROF_ZSTD=1 HZ_PROF_N1=64 HZ_PROF_N2=16 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_zs.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ph_zs.log | tail -10
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 > gpurun_out/b_zs.log 2>&1 || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/b_zs.log').read().strip().splitlines()[-1]); print(json.dumps(d.get('zstd'))[:600])"
