#!/bin/bash
# experiment build of the engine: tools/ablib.sh NAME [-DFLAG ...] -> abtmp/NAME.so
# (abtmp/ is in .gpurunignore so that round-end pushes carry no scratch builds: drop that
# line while A/B builds must travel to the GPU box, and delete abtmp/ afterwards)
set -e
cd "$(dirname "$0")/.."
mkdir -p abtmp
N=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value "$@" \
  -o abtmp/$N.so hsds_amd/csrc/engine.hip
echo "abtmp/$N.so"
