#!/bin/bash
# round 5: one pass in the window pipeline (lone-chunk latency) and priority-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base fusepipe; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/$v.so timeout -k 10 300 python tools/latency.py > gpurun_out/lat_$v.json 2> gpurun_out/lat_$v.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/lat_$v.json'))
print('$v', 'F1', d['F1']['device_one_chunk_kernel_ms_4wave'], d['F1']['device_one_chunk_kernel_ms_2wave'], 'F2', d['F2']['device_one_chunk_kernel_ms_4wave'], d['F2']['device_one_chunk_kernel_ms_2wave'])"
done
tools/ab.sh abtmp/base.so abtmp/p32.so abtmp/p48.so abtmp/base.so abtmp/p32.so abtmp/p48.so
