#!/bin/bash
# round 6: literal/length LUT root 9 (frees ~1 KiB of LDS per wave) and with it 32-byte
# record stores (RGRP 4) at 16 waves per CU -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur.so abtmp/lr9.so abtmp/lr9rg4.so abtmp/cur.so abtmp/lr9.so abtmp/lr9rg4.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/lr9.so abtmp/lr9rg4.so 2>&1 | tee gpurun_out/lr9_traffic.txt
