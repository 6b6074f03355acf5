#!/bin/bash
# cfg5 encode (time + size against libz) for several parse chain depths:
# tools/ab_chain.sh 4 8 16 ...   (HSDS_DEFLATE_CHAIN development override)
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  HSDS_DEFLATE_CHAIN=$c timeout -k 10 300 python bench.py --headline 0 --steps 3 --warmup 1 --cpu-seconds 0 \
    --cfg3 0 --cfg1 0 --cfg5 1 --cfg4-full 0 > gpurun_out/abc_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "chain $c rc=$rc"; tail -5 gpurun_out/abc_$c.log; exit $rc; }
  python - $c gpurun_out/abc_$c.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["legs"]["cfg5"]
print(f"chain {sys.argv[1]:>4s}: {d['value']:6.2f} GB/s slab, deflate {d['deflate_kernel_ms']:7.2f} ms, "
      f"size_vs_libz {d['size_vs_libz']:.4f}, first column {d['size_vs_libz_first_column']:.4f}")
PY
done
