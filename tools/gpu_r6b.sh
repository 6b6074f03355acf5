#!/bin/bash
# round 6: parallel dynamic-header build + adler32 by dot products (new) against the round-5
# kernel (base) and new with the round-5 header (hdr1): bench A/B and lone-chunk latency
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/base.so abtmp/new.so abtmp/hdr1.so abtmp/base.so abtmp/new.so abtmp/hdr1.so || exit 1
for lib in base new hdr1; do
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$(realpath abtmp/$lib.so) timeout -k 10 120 python tools/lone_ab.py >> gpurun_out/lone_ab.txt 2>gpurun_out/lone_ab.err || { tail -5 gpurun_out/lone_ab.err; exit 1; }
done
cat gpurun_out/lone_ab.txt
