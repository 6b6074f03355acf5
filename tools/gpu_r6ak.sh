#!/bin/bash
# round 6: HBM traffic passes of the final build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RND=r6 bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1; rc=$?; grep bytes_per_launch gpurun_out/traffic/traffic.json; [ $rc -eq 0 ] || exit $rc
