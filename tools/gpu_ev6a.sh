#!/bin/bash
# round 6 evidence, part 1: GPU tests, smoke, the driver's bench command, headline rocprof stats,
# latency; then the warm-up length for lone chunks (window pipeline) via HSDS_INFLATE_TUNE
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
R="$(pwd)"; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --kernel-timing 1 --f2 0 --e2e 0 --cfg3 0 --cfg5 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 > "$R/gpurun_out/bench_prof.log" 2>&1)
rc=$?; echo "rocprof rc=$rc"; grep "inflate2_kernel" gpurun_out/prof/run_kernel_stats.csv | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/latency.py > gpurun_out/latency.json 2>gpurun_out/latency.err
rc=$?; echo "latency rc=$rc"; cat gpurun_out/latency.json; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/lone_ab.txt
for t in 512,4,1 768,4,1 1024,4,1; do
  HSDS_INFLATE_TUNE=$t timeout -k 10 120 python tools/lone_ab.py >> gpurun_out/lone_ab.txt 2>gpurun_out/lone_ab.err || { tail -3 gpurun_out/lone_ab.err; exit 1; }
done
cat gpurun_out/lone_ab.txt
