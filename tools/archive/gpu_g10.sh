set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batcher.py > gpurun_out/g10_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g10_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.json 2> gpurun_out/latency.err; rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/latency.json')); print({k: v['ms'] for k, v in d['batcher_F1_concurrent_requests'].items()})"
exit $rc
