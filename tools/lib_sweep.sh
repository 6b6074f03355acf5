#!/bin/bash
# time the F1/F2 headline with alternative library builds: tools/lib_sweep.sh lib1.so lib2.so ...
mkdir -p gpurun_out
for lib in "$@"; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --e2e 0 --cfg3 0 --cfg5 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 > gpurun_out/sweep.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/sweep.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/sweep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'F1', d['value'], d['roofline']['kernel_ms'], 'ms | F2', d['f2']['value'], d['f2']['inflate_kernel_ms'])"
done
