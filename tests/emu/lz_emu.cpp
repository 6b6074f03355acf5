// CPU emulation driver for hsds_amd/csrc/lz_wave.h (TEST INFRASTRUCTURE ONLY).
// Runs the exact single-source wave algorithm (uniform parse + per-lane resolve with
// LANE_LOOP iterating the 64 lanes in order) on one Blosc split.  Never used by the
// product.
#include <stdlib.h>
#include "../../hsds_amd/csrc/lz_wave.h"

extern "C" int emu_lz_stream(const uint8_t* src, uint32_t src_len, uint8_t* dst, uint32_t dst_len, uint32_t fmt) {
  lz::Shared* ls = (lz::Shared*)calloc(1, sizeof(lz::Shared));
  hz::StreamJob job = {src, src_len, dst, dst_len, 1u, nullptr};
  int r = lz::lz_stream(*ls, job, fmt);
  free(ls);
  return r;
}

extern "C" int emu_lz_shared_bytes() { return (int)sizeof(lz::Shared); }
