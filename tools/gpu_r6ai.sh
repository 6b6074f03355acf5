#!/bin/bash
# round 6: matches per lane per resolve batch (HZ2_MPL 4 / 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/mpl4.so abtmp/mpl3.so abtmp/mpl4.so abtmp/mpl3.so abtmp/mpl4.so abtmp/mpl3.so || exit 1
