#!/bin/bash
# round-5 evidence for the current build, one GPU call: GPU tests, inflate phase profile,
# full bench, rocprofv3 kernel stats of the headline, inflate SQ passes, HBM traffic passes
# (headline + cfg3), DN latency, encoder SQ passes; each step time-limited, stop at the first
# failure
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh || exit 1
bash tools/gpu_sq_bench.sh sq_r5 || exit 1
for d in gpurun_out/sq_r5/p*; do python3 tools/pmc_sum.py $d; done > gpurun_out/sq_r5/summary.txt
CFG3=1 RND=r5 bash tools/pmc_traffic.sh || exit 1
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.json 2> gpurun_out/latency.err || exit 1
bash tools/sq_encode.sh sq_enc_r5 || exit 1
echo "r5 evidence done"
