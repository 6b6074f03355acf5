#!/bin/bash
# round 6: M's record loads non-temporal (HZ2_NTREC) -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/base5.so abtmp/ntrec.so abtmp/base5.so abtmp/ntrec.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/base5.so abtmp/ntrec.so 2>&1 | tail -2
