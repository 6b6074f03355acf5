#!/bin/bash
R="$(pwd)"; cd /tmp && export TMPDIR=/tmp
for L in cp8 nofl nolit none; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/abtmp/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/lzattr_$L" -o t -- \
    python3 "$R/bench.py" --headline 0 --steps 2 --warmup 1 --cpu-seconds 0 --cfg3 0 --cfg1 0 --cfg5 1 --cfg4-full 0 --f2 0 --e2e 0 --lz4 0 --zstd 0 --bshuf 0 --cfg5w 0 --cfg4 0 > "$R/gpurun_out/lzattr_$L.log" 2>&1
  echo "$L rc=$?"
done
exit 0
