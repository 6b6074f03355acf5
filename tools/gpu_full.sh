# full GPU suite, then the bench legs whose host code changed (cfg3 / cfg5 CPU baselines)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests.log 2>&1
rc=$?; tail -3 gpurun_out/full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 6 --headline 0 --f2 0 --e2e 0 --cfg3 1 --lz4 0 --zstd 0 --bshuf 0 --cfg1 0 --cfg5 0 --cfg5w 0 --cfg4 0 --cfg4-full 0 --copy-ceiling 0 > gpurun_out/cfg3_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/cfg3_bench.log | tail -1 | cut -c1-1500; exit $rc
