#!/bin/bash
# round 6: PUT_Chunk batch with the decode statuses checked at the dirty-flag wait
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
HSDS_PROFILE_CFG5W=1 timeout -k 10 900 python bench.py --steps 20 --warmup 5 --headline 0 --cfg5 0 --cfg4-full 0 --cfg3 0 --cfg4 0 --cfg1 0 --cpu-seconds 0 > gpurun_out/legs.log 2> gpurun_out/legs.err
rc=$?; echo "legs rc=$rc"; python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/legs.log") if l.startswith("{")][-1])["legs"]
w = d["cfg5_sharded_write"]
print("cfg5w", w["full"]["value"], w["full"]["ms_per_step"], w["offset_100_100"]["value"], w["offset_100_100"]["ms_per_step"],
      w["full"]["sample_check"], w["offset_100_100"]["sample_check"])
PY
[ $rc -eq 0 ] || exit $rc
