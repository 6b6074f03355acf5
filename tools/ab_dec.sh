#!/bin/bash
# A/B of the lz4 / zstd / bitshuffle decode legs for several builds: tools/ab_dec.sh a.so b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 \
    --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --copy-ceiling 0 > gpurun_out/abd_$(basename $lib).log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/abd_$(basename $lib).log; exit $rc; }
  python - $lib gpurun_out/abd_$(basename $lib).log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
d = d.get("legs", d)
print(f"{sys.argv[1]:20s} lz4 {d['lz4']['value']:7.2f} ({d['lz4']['lz_kernel_ms']:6.2f} ms)  zstd {d['zstd']['value']:6.2f} ({d['zstd']['zstd_kernel_ms']:6.2f} ms)  bshuf {d['bshuf']['value']:7.2f}")
PY
done
