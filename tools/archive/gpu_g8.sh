set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/g8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g8_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/st4only.so abtmp/st16.so abtmp/st4only.so abtmp/st16.so
