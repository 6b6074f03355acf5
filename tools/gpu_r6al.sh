#!/bin/bash
# round 6: matches per lane per resolve batch 3 / 2 -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/mpl3b.so abtmp/mpl2.so abtmp/mpl3b.so abtmp/mpl2.so abtmp/mpl3b.so abtmp/mpl2.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/mpl3b.so abtmp/mpl2.so 2>&1 | tail -2
