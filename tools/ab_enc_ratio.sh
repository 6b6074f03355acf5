#!/bin/bash
# cfg5 encode time and size against libz for parse variants:
# tools/ab_enc_ratio.sh LIB:CHAIN:FAR ...  (LIB: a .so path or "cur"; CHAIN 0 = the level's;
# FAR 1 = far ring at L4; HSDS_DEFLATE_CHAIN / HSDS_DEFLATE_FAR development overrides)
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r lib chain far <<< "$spec"
  envs=()
  [ "$lib" != "cur" ] && envs+=(HSDS_AMD_DEV=1 HSDS_AMD_LIB="$lib")
  [ "$chain" != "0" ] && envs+=(HSDS_DEFLATE_CHAIN="$chain")
  [ "$far" = "1" ] && envs+=(HSDS_DEFLATE_FAR=1)
  tag=$(echo "$spec" | tr '/:' '__')
  env "${envs[@]}" timeout -k 10 300 python bench.py --headline 0 --steps 3 --warmup 1 --cpu-seconds 0 \
    --cfg3 0 --cfg1 0 --cfg5 1 --cfg4-full 0 --f2 0 --e2e 0 --lz4 0 --zstd 0 --bshuf 0 --cfg5w 0 --cfg4 0 > gpurun_out/aber_$tag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -5 gpurun_out/aber_$tag.log; exit $rc; }
  python - "$spec" gpurun_out/aber_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["legs"]["cfg5"]
print(f"{sys.argv[1]:>24s}: {d['value']:6.2f} GB/s slab, deflate {d['deflate_kernel_ms']:7.2f} ms, "
      f"size_vs_libz {d['size_vs_libz']:.4f}, first column {d['size_vs_libz_first_column']:.4f}")
PY
done
