#!/bin/bash
# A/B of the encoder (parse/huffman/emit kernels) across builds: encode-parity tests
# gate each lib, then tools/deflate_profile.py times 512 x 1 MiB chunks.
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/abe_$(basename $lib).log 2>&1
  rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/abe_$(basename $lib).log)"; [ $rc -eq 0 ] || exit $rc
  HZ_PROF_LIB=$(realpath $lib) HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python tools/deflate_profile.py 2>&1 | grep -v amdgpu.ids | head -1
done
