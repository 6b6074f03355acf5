#!/bin/bash
# A/B of inflate window tunings on one build via HSDS_INFLATE_TUNE ("W,rounds,over16"):
# each tuning first passes the GPU codec tests (bit-exact), then bench.py times F1/F2.
#   tools/ab_tune.sh 384,4,1 256,4,1 ...
set -o pipefail
mkdir -p gpurun_out
for t in "$@"; do
  tag=${t//,/_}
  HSDS_INFLATE_TUNE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/abt_$tag.log 2>&1
  rc=$?; echo "$t tests rc=$rc $(tail -1 gpurun_out/abt_$tag.log)"; [ $rc -eq 0 ] || exit $rc
  HSDS_INFLATE_TUNE=$t timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 \
    > gpurun_out/ab_$tag.log 2>gpurun_out/ab_$tag.err
  rc=$?; grep -m1 "tune override" gpurun_out/ab_$tag.err; [ $rc -eq 0 ] || { echo "$t rc=$rc"; tail -5 gpurun_out/ab_$tag.err; exit $rc; }
  python - "$t" gpurun_out/ab_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:24s} F1 {d['value']:7.2f} GB/s kernel {d['roofline']['kernel_ms']:8.2f} ms   F2 {d['f2']['value']:6.2f} GB/s kernel {d['f2']['inflate_kernel_ms']:8.2f} ms")
PY
done
