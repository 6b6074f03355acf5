set -o pipefail
bash tools/ab_encode.sh abtmp/enc_rle.so || exit 1
for v in head rle head rle; do HZ_PROF_LIB=abtmp/enc_$v.so HSDS_AMD_DEV=1 HSDS_AMD_LIB=abtmp/enc_$v.so timeout -k 10 200 python tools/deflate_profile.py 2>&1 | grep -v amdgpu | head -1 || exit 1; done
CFG3=1 bash tools/gpu_evidence.sh "" r3f
