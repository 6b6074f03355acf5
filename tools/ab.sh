#!/bin/bash
# A/B timing of several builds of the library on one box: tools/ab.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 \
    > gpurun_out/ab_$(basename $lib).log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/ab_$(basename $lib).log; exit $rc; }
  python - "$lib" gpurun_out/ab_$(basename $lib).log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} F1 {d['value']:7.2f} GB/s kernel {d['roofline']['kernel_ms']:8.2f} ms   F2 {d['f2']['value']:6.2f} GB/s kernel {d['f2']['inflate_kernel_ms']:8.2f} ms")
PY
done
