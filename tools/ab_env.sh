#!/bin/bash
# A/B of one library under environment settings: tools/ab_env.sh "ENV1=.." "ENV2=.." ...
# ("-" = no extra environment); headline legs (F1, F2) of the bench per setting
set -o pipefail
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 \
    > gpurun_out/abenv_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$e] rc=$rc"; tail -5 gpurun_out/abenv_$i.log; exit $rc; }
  python - "$e" gpurun_out/abenv_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"[{sys.argv[1]:30s}] F1 {d['value']:7.2f} GB/s kernel {d['roofline']['kernel_ms']:8.2f} ms   F2 {d['f2']['value']:6.2f} GB/s kernel {d['f2']['inflate_kernel_ms']:8.2f} ms  step {d['f2'].get('ms_per_step', 0)}")
PY
done
