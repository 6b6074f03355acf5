set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/g3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g3_tests.log; [ $rc -eq 0 ] || exit $rc
HSDS_AMD_DEV=1 HSDS_AMD_LIB=$GRAFT_REPO_ROOT/abtmp/rec4s.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_codec.py > gpurun_out/g3_tests_s.log 2>&1
rc=$?; tail -3 gpurun_out/g3_tests_s.log; [ $rc -eq 0 ] || exit $rc
tools/ab.sh abtmp/rec8.so abtmp/rec4s.so abtmp/rec4t.so abtmp/rec8.so abtmp/rec4s.so abtmp/rec4t.so
bash tools/pmc_traffic_ab.sh abtmp/rec4t.so
