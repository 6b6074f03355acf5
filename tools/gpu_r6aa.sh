#!/bin/bash
# round 6: deflate emit walk, 8 / 16 token dwords per batch of loads
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_enc5.sh abtmp/wb8.so abtmp/wb16.so abtmp/wb8.so abtmp/wb16.so || exit 1
