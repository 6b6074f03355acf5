#!/bin/bash
# round 5: A/B of the inflate source-map
# fill cap (HZ2_FILLCAP 8 / 16 / 24 / 32; builds by tools/ablib.sh, abtmp/ must travel), F1 and F2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tools/ab.sh abtmp/fc16.so abtmp/fc8.so abtmp/fc24.so abtmp/fc32.so abtmp/fc16.so
