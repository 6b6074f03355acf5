#!/bin/bash
# round 6: M's record loads non-temporal, three more pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/base5.so abtmp/ntrec.so abtmp/base5.so abtmp/ntrec.so abtmp/base5.so abtmp/ntrec.so || exit 1
