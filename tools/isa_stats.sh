#!/bin/bash
# resource usage of every kernel (VGPR / SGPR / LDS / scratch / occupancy) from the gfx950 ISA
set -e
cd "$(dirname "$0")/.."
D=$(mktemp -d /tmp/isa.XXXX)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-value ${HZ_FLAGS} -save-temps=obj \
  -c -o $D/engine.o hsds_amd/csrc/engine.hip
S=$(ls $D/*gfx950*.s)
awk '/^\t\.amdhsa_kernel /{k=$2; sub(/^_ZN12_GLOBAL__N_1[0-9]+/, "", k); sub(/E.*/, "", k)}
     /^; (NumVgprs|NumSgprs|ScratchSize|LDSByteSize|Occupancy):/{printf "%-22s %s\n", k, $0}' $S
echo "ISA: $S"
