#!/bin/bash
# round 6 evidence, part 2: HBM traffic (FETCH_SIZE / WRITE_SIZE passes, headline + cfg3), SQ
# counters, phase and tail profiles, encoder kernel stats and SQ, traffic attribution of the
# shipped build by compiling phases out
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_enc_tests.log 2>&1
rc=$?; echo "encode tests rc=$rc"; tail -2 gpurun_out/gpu_enc_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_enc5.sh abtmp/attr_base.so abtmp/zseq.so abtmp/attr_base.so abtmp/zseq.so || exit 1
bash tools/ab.sh abtmp/r5.so abtmp/attr_base.so abtmp/r5.so abtmp/attr_base.so || exit 1
RND=r6 bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1; rc=$?; tail -4 gpurun_out/traffic.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sq_bench.sh sq_r6 > gpurun_out/sq_r6.log 2>&1 || { tail gpurun_out/sq_r6.log; exit 1; }
python3 tools/pmc_sum.py gpurun_out/sq_r6 inflate2_kernel > gpurun_out/sq_r6_summary.txt; cat gpurun_out/sq_r6_summary.txt
HZ_PROF_F2W1=1 HZ_PROF_LZ=0 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1 || { tail gpurun_out/phase.log; exit 1; }
HZ_PROF_LONE=1 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase_lone.log 2>&1 || { tail gpurun_out/phase_lone.log; exit 1; }
timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail.log 2>&1 || { tail gpurun_out/tail.log; exit 1; }
cat gpurun_out/tail.log | grep -v amdgpu
bash tools/enc_prof.sh || exit 1
bash tools/sq_encode.sh sq_enc_r6 > /dev/null 2>&1 || exit 1
bash tools/pmc_traffic_ab.sh abtmp/attr_base.so abtmp/nom_noemit.so abtmp/nom_noemitrec.so abtmp/nom.so abtmp/nomstore.so abtmp/nofar.so abtmp/nolitload.so 2>&1 | tee gpurun_out/attr6.txt
