#!/bin/bash
# round 6: match-record staging group size (RGRP 2 / 4 / 8 records per store) -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur.so abtmp/rg4.so abtmp/rg4os8m0.so abtmp/rg8.so abtmp/cur.so abtmp/rg4.so abtmp/rg4os8m0.so abtmp/rg8.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/cur.so abtmp/rg4.so abtmp/rg4os8m0.so abtmp/rg8.so 2>&1 | tee gpurun_out/rgrp_traffic.txt
