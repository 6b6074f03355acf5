#!/bin/bash
# round 6: wave priority step (KiB of remaining input per level) for F2's 1 MiB streams
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur3.so abtmp/pa80.so abtmp/pa136.so abtmp/pa200.so abtmp/cur3.so abtmp/pa80.so abtmp/pa136.so abtmp/pa200.so || exit 1
