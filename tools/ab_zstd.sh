#!/bin/bash
# A/B of the Blosc-zstd decode leg for several builds: tools/ab_zstd.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath $lib) timeout -k 10 400 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 1 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --copy-ceiling 0 \
    > gpurun_out/abz_$(basename $lib).log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/abz_$(basename $lib).log; exit $rc; }
  python - "$lib" gpurun_out/abz_$(basename $lib).log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:30s} zstd {d['zstd']['value']:7.2f} GB/s kernel {d['zstd']['zstd_kernel_ms']:8.2f} ms")
PY
done
