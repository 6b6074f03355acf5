#!/bin/bash
# round 6: M's loads non-temporal (records HZ2_NTREC, gathers HZ2_NTGATH) -- speed and traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/base5.so abtmp/ntrec.so abtmp/ntgath.so abtmp/ntboth.so abtmp/base5.so abtmp/ntrec.so abtmp/ntgath.so abtmp/ntboth.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/ntgath.so abtmp/ntboth.so 2>&1 | tail -2
