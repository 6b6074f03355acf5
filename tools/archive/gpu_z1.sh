#!/bin/bash
# round 5: zstd wave priority A/B (zstd GPU tests of one variant first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
true
tools/ab_dec.sh abtmp/zs0.so abtmp/zs16.so abtmp/zs32.so abtmp/zs64.so abtmp/zs0.so abtmp/zs16.so abtmp/zs32.so
