set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/enc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/deflate_profile.py 2>&1 | grep -v amdgpu.ids; [ $? -eq 0 ] || exit 1
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/eprof -o run -- python3 $R/tools/deflate_profile.py > $R/gpurun_out/eprof.log 2>&1; rc=$?
cut -d, -f1-4 $R/gpurun_out/eprof/run_kernel_stats.csv | head -12
exit $rc
