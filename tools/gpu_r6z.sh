#!/bin/bash
# round 6: zstd writer's backward sequence batch (ZE_SEQB 8 / 16 / 32)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_enc5.sh abtmp/zsb8.so abtmp/zsb16.so abtmp/zsb32.so abtmp/zsb8.so abtmp/zsb16.so abtmp/zsb32.so || exit 1
