#!/bin/bash
# A/B of the LZ legs (lz4, bitshuffle) for several builds: tools/ab_lz.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 --f2 0 --cfg3 0 --cfg5 0 --zstd 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 \
    > gpurun_out/ablz_$(basename $lib).log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/ablz_$(basename $lib).log; exit 1; }
  python - "$lib" gpurun_out/ablz_$(basename $lib).log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:32s} lz4 {d['lz4']['value']:7.2f} GB/s ({d['lz4']['lz_kernel_ms']:.2f} ms)  bshuf {d['bshuf']['value']:7.2f} GB/s")
PY
done
