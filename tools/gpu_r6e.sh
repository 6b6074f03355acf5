#!/bin/bash
# round 6: GPU tests; inflate SQ counters of the current build; encoder lane-skew A/B (cfg5 legs
# and parse SQ counters); the sharded-write leg with the view-free cache hits
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh abtmp/cur.so abtmp/fill2.so abtmp/cur.so abtmp/fill2.so || exit 1
bash tools/gpu_sq_bench.sh sq_r6 > gpurun_out/sq_r6.log 2>&1 || { tail gpurun_out/sq_r6.log; exit 1; }
python3 tools/pmc_sum.py gpurun_out/sq_r6 inflate2_kernel
bash tools/ab_enc5.sh abtmp/cur.so abtmp/skew2.so abtmp/cur.so abtmp/skew2.so || exit 1
bash tools/sq_encode.sh sq_enc_cur abtmp/cur.so > /dev/null 2>&1 || exit 1
bash tools/sq_encode.sh sq_enc_skew2 abtmp/skew2.so > /dev/null 2>&1 || exit 1
grep -A17 "parse_kernel" gpurun_out/sq_enc_cur/summary.txt | grep "LDS_BANK\|LDS_IDX\|INSTS_VALU"
grep -A17 "parse_kernel" gpurun_out/sq_enc_skew2/summary.txt | grep "LDS_BANK\|LDS_IDX\|INSTS_VALU"
timeout -k 10 500 python bench.py --headline 0 --steps 1 --warmup 1 --cfg5-steps 3 --cfg3 0 --cfg1 0 --cfg5 0 --cfg4 0 --cfg4-full 0 --cpu-seconds 0 > gpurun_out/cfg5w.log 2>&1
rc=$?; echo "cfg5w rc=$rc"; grep "^{" gpurun_out/cfg5w.log; exit $rc
