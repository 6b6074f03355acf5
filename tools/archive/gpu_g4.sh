set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/g4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 6 --headline 0 --f2 0 --e2e 0 --cfg3 0 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --copy-ceiling 0 > gpurun_out/g4_bench.log 2>&1
rc=$?; tail -2 gpurun_out/g4_bench.log | cut -c1-3000; exit $rc
