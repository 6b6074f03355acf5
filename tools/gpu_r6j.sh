#!/bin/bash
# round 6: RGRP 4 (32-byte record stores) at 16 waves per CU: the bit ring shrunk to 8 words
# (refill every 3 or 2 tokens) to pay for the larger record staging -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur.so abtmp/rg4rs8t3.so abtmp/rg4rs8t2.so abtmp/rs8t3.so abtmp/cur.so abtmp/rg4rs8t3.so abtmp/rg4rs8t2.so abtmp/rs8t3.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/rg4rs8t3.so abtmp/rs8t3.so 2>&1 | tee gpurun_out/rgrp2_traffic.txt
