#!/bin/bash
# cfg5 encode legs only (zlib / lz4 / zstd / bitshuffle writers) for several builds:
# tools/ab_enc5.sh a.so b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --headline 0 --steps 3 --warmup 1 \
    --cpu-seconds 0 --f2 0 --e2e 0 --cfg3 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 \
    --copy-ceiling 0 > gpurun_out/abe_$(basename $lib).log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/abe_$(basename $lib).log; exit $rc; }
  python - $lib gpurun_out/abe_$(basename $lib).log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)["legs"]["cfg5"]
print(f"{sys.argv[1]:20s} zlib {d['value']:6.2f} GB/s ({d['deflate_kernel_ms']:7.2f} ms)  lz4 {d['lz4_encode']['value']:6.2f}  "
      f"zstd {d['zstd_encode']['value']:6.2f}  bshuf {d['bshuf_encode']['value']:6.2f}  size {d['size_vs_libz']} "
      f"first {d['size_vs_libz_first_column']}")
PY
done
