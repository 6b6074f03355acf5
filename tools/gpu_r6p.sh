#!/bin/bash
# round 6: host hot spots of the configs[4] sharded write (cProfile of two steps per variant)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSDS_PROFILE_CFG5W=1 timeout -k 10 600 python bench.py --steps 1 --warmup 1 --cfg5-steps 3 --headline 0 --cfg3 0 --cfg1 0 --cfg5 0 --cfg4 0 --cfg4-full 0 --cpu-seconds 0 > gpurun_out/cfg5w_prof.log 2> gpurun_out/cfg5w_prof.err
rc=$?; echo "rc=$rc"; tail -c 800 gpurun_out/cfg5w_prof.log; [ $rc -eq 0 ] || exit $rc
