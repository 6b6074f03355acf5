#!/bin/bash
# GPU parity tests only (each test file bounded; stops at the first failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
