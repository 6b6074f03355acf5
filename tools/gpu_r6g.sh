#!/bin/bash
# round 6: lone-chunk latency against the bit ring's refill rate (RS 12 / TICKN 5 = cur,
# RS 16 / TICKN 8, RS 24 / TICKN 12): does phase A of a lone stream wait on its refills?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/lone_ab.txt
for lib in cur rs16 rs24; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath abtmp/$lib.so) timeout -k 10 120 python tools/lone_ab.py >> gpurun_out/lone_ab.txt 2>gpurun_out/lone_ab.err || { tail -5 gpurun_out/lone_ab.err; exit 1; }
done
cat gpurun_out/lone_ab.txt
bash tools/ab.sh abtmp/cur.so abtmp/rs16.so || exit 1
