#!/bin/bash
# round-5 final evidence for the current build, one GPU call: GPU tests, phase profiles (F1,
# F2 one-wave), full bench, rocprofv3 kernel stats of the headline, inflate SQ passes, HBM
# traffic (headline + cfg3), latency, tail profile, encoder SQ passes; stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HZ_PROF_LIB=$GRAFT_REPO_ROOT/abtmp/prof_fuse.so
HZ_PHASE=0 bash tools/gpu_round.sh || exit 1
HZ_PROF_F2W1=1 HZ_PROF_LZ=0 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/phase.log
bash tools/gpu_sq_bench.sh sq_r5 || exit 1
for d in gpurun_out/sq_r5/p*; do [ -d $d ] && python3 tools/pmc_sum.py $d; done > gpurun_out/sq_r5/summary.txt
CFG3=1 RND=r5 bash tools/pmc_traffic.sh || exit 1
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.json 2> gpurun_out/latency.err || exit 1
timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/tail.log
bash tools/sq_encode.sh sq_enc_r5 || exit 1
echo "r5 final evidence done"
