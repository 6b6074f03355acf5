#!/bin/bash
# round 6: M's span of 1280 bytes (fits the LDS the record groups left; more spills)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh abtmp/cur4.so abtmp/span1280.so abtmp/cur4.so abtmp/span1280.so || exit 1
