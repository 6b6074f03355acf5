#!/bin/bash
# round 6: non-temporal bitstream A/B, then FETCH_SIZE / WRITE_SIZE of inflate2_kernel on the
# shipped one-pass build with phases compiled out (abtmp/*.so from tools/ablib.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab.sh abtmp/base.so abtmp/ntbits.so abtmp/base.so abtmp/ntbits.so || exit 1
bash tools/pmc_traffic_ab.sh abtmp/base.so abtmp/nom_noemit.so abtmp/nom_noemitrec.so abtmp/nom.so abtmp/noemitrec.so abtmp/nomstore.so abtmp/nofar.so abtmp/nolitload.so abtmp/ntbits.so 2>&1 | tee gpurun_out/attr6.txt
