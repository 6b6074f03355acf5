#!/bin/bash
# round 5, Huffman build in registers: full GPU tests + bench + headline rocprof on the
# in-tree build, cfg5 writer A/B against the lane-0 build, encoder kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HZ_PHASE=0 bash tools/gpu_round.sh || exit 1
bash tools/ab_enc5.sh abtmp/hreg0.so hsds_amd/libhsds_amd.so abtmp/hreg0.so hsds_amd/libhsds_amd.so || exit 1
bash tools/enc_prof.sh || exit 1
echo "h2 done"
