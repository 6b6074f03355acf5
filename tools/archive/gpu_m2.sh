#!/bin/bash
# A/B of the resolve variants in abtmp/ + their phase profiles (F1 / F2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "$@" || exit 1
for l in "$@"; do
  p=${l/lib_/prof_}
  HZ_PROF_LIB=$(realpath $p) HZ_PROF_LZ=0 timeout -k 10 200 python tools/phase_profile.py > gpurun_out/ph_$(basename $p).log 2>&1 || exit 1
  echo "== $p"; grep -v amdgpu gpurun_out/ph_$(basename $p).log
done
