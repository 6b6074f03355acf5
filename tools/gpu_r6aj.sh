#!/bin/bash
# round 6: MPL 3 as the default -- full GPU tests, smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh
