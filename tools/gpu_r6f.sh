#!/bin/bash
# round 6: lane-end bookkeeping out of phase A's token loop + mul24 in the long fill (estop)
# against the warm-up commit (cur) and estop with HZ2_ESTOP=0 (estop0: the mul24 only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/cur.so abtmp/estop.so abtmp/estop0.so abtmp/cur.so abtmp/estop.so abtmp/estop0.so || exit 1
