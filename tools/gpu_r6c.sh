#!/bin/bash
# round 6: lean warm-up loop + v_bfrev table fill (cur) against afac266 (r6a) and cur without the
# warm-up loop (warm0); then warm-up length sweep on the in-tree build (codec tests first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/r6a.so abtmp/cur.so abtmp/warm0.so abtmp/r6a.so abtmp/cur.so abtmp/warm0.so || exit 1
bash tools/ab_tune.sh 768,4,1 1024,4,1 640,4,1 1280,4,1 || exit 1
