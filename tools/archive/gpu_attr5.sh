#!/bin/bash
# round 5 traffic attribution: WRITE/FETCH calibration of the access widths, then
# FETCH_SIZE / WRITE_SIZE of inflate2_kernel with phases compiled out (abtmp/*.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/wcal_run.sh > gpurun_out/wcal.txt 2>&1; rc=$?; cat gpurun_out/wcal.txt; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic_ab.sh abtmp/base.so abtmp/nom_nostore.so abtmp/nom_noring.so abtmp/nom.so abtmp/nomstore.so abtmp/nofar.so abtmp/nolitload.so abtmp/nofar_nomstore.so 2>&1 | tee gpurun_out/attr5.txt
grep -h "pmc_run done" gpurun_out/pmc_tab/*.WRITE_SIZE.log
