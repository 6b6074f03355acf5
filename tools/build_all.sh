#!/bin/bash
# local build of every native artefact (fails loudly)
set -e
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()" > /tmp/build.log 2>&1 || { cat /tmp/build.log; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -DHZ_PROFILE \
  -o tools/libhsds_prof.so hsds_amd/csrc/engine.hip
echo "build ok"
