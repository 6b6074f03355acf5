set -o pipefail
cd $GRAFT_REPO_ROOT
tools/ab.sh abtmp/base.so abtmp/p4.so abtmp/p2.so abtmp/base.so abtmp/p4.so
HZ_PROF_LIB=$GRAFT_REPO_ROOT/abtmp/prof_base.so timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail_base.txt 2>&1; rc=$?; grep -E "^F[12]" gpurun_out/tail_base.txt; [ $rc -eq 0 ] || exit $rc
HZ_PROF_LIB=$GRAFT_REPO_ROOT/abtmp/prof_p4.so timeout -k 10 300 python tools/tail_profile.py > gpurun_out/tail_p4.txt 2>&1; rc=$?; grep -E "^F[12]" gpurun_out/tail_p4.txt; exit $rc
