#!/bin/bash
# round 6: 32-byte record groups whose last record is stored from registers (HZ2_RLAST: the
# LDS stage holds 3 records per lane), paid for by the ring mirror or 8-byte literal staging
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur.so abtmp/rl4m0.so abtmp/rl4os8.so abtmp/rl2.so abtmp/lr9rg4.so abtmp/cur.so abtmp/rl4m0.so abtmp/rl4os8.so abtmp/rl2.so abtmp/lr9rg4.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/rl4m0.so abtmp/rl4os8.so 2>&1 | tee gpurun_out/rlast_traffic.txt
