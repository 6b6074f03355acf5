#!/bin/bash
# round 6: phase shares of the deflate encoder (parse staging / chains / parse)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/enc_phase.py > gpurun_out/enc_phase.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/enc_phase.log | tail -12; exit $rc
