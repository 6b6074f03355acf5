#!/bin/bash
# correctness gate + A/B timing of candidate builds: every lib must pass the GPU
# codec/encode tests (bit-exact) before its timing counts.  tools/ab_check.sh a.so b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_encode.py \
    tests/test_gpu_selection.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abt_$(basename $lib).log 2>&1
  rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/abt_$(basename $lib).log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab.sh "$@"
