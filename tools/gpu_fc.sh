#!/bin/bash
# round 5: parity tests + bench of the shipped build, then an A/B of the inflate source-map
# fill cap (HZ2_FILLCAP 8 / 12 / 16 / 24 / 32), F1 and F2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HZ_PHASE=0 HZ_ROCPROF=0 bash tools/gpu_round.sh || exit $?
tools/ab.sh abtmp/fc16.so abtmp/fc8.so abtmp/fc24.so abtmp/fc32.so abtmp/fc16.so abtmp/fc12.so
