#!/bin/bash
# round 6: fill cap and priority step re-swept on the record-group build
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/cur4.so abtmp/fc12.so abtmp/fc24.so abtmp/pa32.so abtmp/pa48.so abtmp/cur4.so abtmp/fc12.so abtmp/fc24.so abtmp/pa32.so abtmp/pa48.so || exit 1
