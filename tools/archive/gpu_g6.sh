set -o pipefail
cd $GRAFT_REPO_ROOT
tools/ab.sh abtmp/base.so abtmp/g4.so abtmp/g4o8nm.so abtmp/nm.so abtmp/base.so abtmp/g4o8nm.so
bash tools/pmc_traffic_ab.sh abtmp/g4.so abtmp/g4o8nm.so
