#!/bin/bash
# round 6: zstd literal warm-up bits (ZW_HUF_WARM 48 / 64 / 96 / 160)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_zstd.sh abtmp/zw48.so abtmp/zw64.so abtmp/zw96.so abtmp/zw160.so abtmp/zw48.so abtmp/zw64.so abtmp/zw96.so abtmp/zw160.so || exit 1
