set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/g5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g5_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g5prof -o g5 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --headline 0 --f2 0 --e2e 0 --cfg3 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --copy-ceiling 0 > $GRAFT_REPO_ROOT/gpurun_out/g5_bench.log 2>&1
rc=$?; grep '^{' $GRAFT_REPO_ROOT/gpurun_out/g5_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); z=d['legs']['cfg5']['zstd_encode']; print({k: z[k] for k in ('value','encode_ms','size_vs_libblosc_zstd')})"
f=$(find $GRAFT_REPO_ROOT/gpurun_out/g5prof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-5
exit $rc
