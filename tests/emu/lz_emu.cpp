// CPU emulation driver for hsds_amd/csrc/lz_wave.h (TEST INFRASTRUCTURE ONLY).
// Runs the exact single-source wave algorithm (per-lane header walks, shared resolve
// with LANE_LOOP iterating the 64 lanes in order) on up to 64 Blosc splits at once.
// Never used by the product.
#include <stdlib.h>
#include "../../hsds_amd/csrc/lz_wave.h"

// n <= 64 splits; status[i] receives each split's status
extern "C" int emu_lz_group(const uint8_t* const* src, const uint32_t* src_len, uint8_t* const* dst,
                            const uint32_t* dst_len, const uint32_t* fmt, int n, int32_t* status) {
  if (n < 0 || n > 64) return -6;
  lz::Shared* ls = (lz::Shared*)calloc(1, sizeof(lz::Shared));
  lz::Stage* st_ = (lz::Stage*)calloc(1, sizeof(lz::Stage));
  for (int b = 0; b < n; b += lz::GROUP) {       // one wavefront per GROUP splits
    for (int i = 0; i < lz::GROUP; i++) {
      lz::LaneJob j = {nullptr, nullptr, 0u, 0u, 0u, 0u};
      if (b + i < n) j = {src[b + i], dst[b + i], src_len[b + i], dst_len[b + i], fmt[b + i], 1u};
      ls->job[i] = j;
    }
    lz::lz_group<true>(*ls, st_);
    for (int i = 0; i < lz::GROUP && b + i < n; i++) status[b + i] = ls->m_st[i];
  }
  free(ls);
  free(st_);
  return 0;
}

extern "C" int emu_lz_stream(const uint8_t* src, uint32_t src_len, uint8_t* dst, uint32_t dst_len, uint32_t fmt) {
  int32_t st = 0;
  emu_lz_group(&src, &src_len, &dst, &dst_len, &fmt, 1, &st);
  return st;
}

extern "C" int emu_lz_shared_bytes() { return (int)sizeof(lz::Shared); }
