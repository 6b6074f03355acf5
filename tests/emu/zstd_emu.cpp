// CPU emulation driver for hsds_amd/csrc/zstd_lane.h (TEST INFRASTRUCTURE ONLY): the
// per-lane zstd frame decoder run on CPU for one split.  Never used by the product.
#include <stdlib.h>
#include "../../hsds_amd/csrc/zstd_lane.h"
#include "../../hsds_amd/csrc/zstd_wave.h"

extern "C" int emu_zstd_frame(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap) {
  zs::Tables* t = (zs::Tables*)calloc(1, sizeof(zs::Tables));
  const int r = zs::frame(*t, src, n, dst, cap);
  free(t);
  return r;
}

// the wavefront decoder (zstd_wave.h) with LANE_LOOP iterating the 64 lanes
extern "C" int emu_zstd_frame_wave(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap) {
  zw::Shared* ls = (zw::Shared*)calloc(1, sizeof(zw::Shared));
  const int r = zw::frame(*ls, src, n, dst, cap);
  free(ls);
  return r;
}

extern "C" int emu_zstd_wave_shared_bytes() { return (int)sizeof(zw::Shared); }
