#!/bin/bash
# Huffman-kernel timing variants: per-kernel rocprof stats of tools/deflate_profile.py
# (512 x 1 MiB, level 4) for each abtmp/*.so given; the first gated by the encode tests.
set -o pipefail
mkdir -p gpurun_out
R="$(pwd)"
for lib in "$@"; do
  n=$(basename $lib .so)
  if [ "${GATE:-0}" = 1 ]; then
    HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_write.py -m gpu -x -q \
      --timeout 200 --timeout-method thread > gpurun_out/h1_t_$n.log 2>&1
    rc=$?; echo "$n tests rc=$rc $(tail -n 1 gpurun_out/h1_t_$n.log)"; [ $rc -eq 0 ] || exit $rc
  fi
  (cd /tmp && export TMPDIR=/tmp && HZ_PROF_LIB=$R/$lib HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/$lib timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/h1/$n" -o k -- \
    python3 "$R/tools/deflate_profile.py" > "$R/gpurun_out/h1_$n.log" 2>&1)
  rc=$?; echo "$n rc=$rc $(grep encode $R/gpurun_out/h1_$n.log)"; [ $rc -eq 0 ] || exit $rc
  f=$(ls $R/gpurun_out/h1/$n/*kernel_stats.csv | head -n 1)
  grep -E "huff_kernel|emit_kernel|parse_kernel" "$f" | cut -d, -f1-5
done
