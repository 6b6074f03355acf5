#!/bin/bash
# round 6 final evidence on the shipped build: GPU tests, smoke, the driver's bench command,
# headline rocprof stats, latency, SQ counters, phase / lone / tail profiles, encoder stats,
# the cfg3 step's kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
R="$(pwd)"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --kernel-timing 1 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 > "$R/gpurun_out/bench_prof.log" 2>&1)
rc=$?; echo "rocprof rc=$rc"; grep "inflate2_kernel" gpurun_out/prof/run_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/latency.py > gpurun_out/latency.json 2>gpurun_out/latency.err
rc=$?; echo "latency rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sq_bench.sh sq_r6 > gpurun_out/sq_r6.log 2>&1 || { tail gpurun_out/sq_r6.log; exit 1; }
python3 tools/pmc_sum.py gpurun_out/sq_r6 inflate2_kernel > gpurun_out/sq_r6_summary.txt; echo "sq ok"
HZ_PROF_F2W1=1 HZ_PROF_LZ=0 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1 || { tail gpurun_out/phase.log; exit 1; }
HZ_PROF_LONE=1 timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase_lone.log 2>&1 || { tail gpurun_out/phase_lone.log; exit 1; }
timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail.log 2>&1 || { tail gpurun_out/tail.log; exit 1; }
echo "profiles ok"
bash tools/enc_prof.sh || exit 1
bash tools/gpu_r6o.sh || exit 1
