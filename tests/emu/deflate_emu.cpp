// CPU emulation driver for hsds_amd/csrc/deflate_wave.h (TEST INFRASTRUCTURE ONLY).
// Runs the exact single-source wave encoder with LANE_LOOP iterating the 64 lanes
// in order, so its orchestration is checked against libz inflate on CPU.  Never
// used by the product.
#include <stdlib.h>
#include "../../hsds_amd/csrc/deflate_wave.h"

// dst: 4-byte aligned, cap + 8 bytes writable.  Returns compressed bytes or -1.
extern "C" int64_t emu_deflate(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level,
                               int chain_override) {
  hd::Shared* sh = (hd::Shared*)calloc(1, sizeof(hd::Shared));
  hd::Tune tune = hd::tune_for_level(level);
  if (chain_override > 0) tune.chain = (uint32_t)chain_override;
  hd::EncJob job = {src, n, (uint32_t*)dst, cap, level, 1u, 0u, 0u};
  const int64_t r = hd::deflate_stream(*sh, job, tune);
  free(sh);
  return r;
}

extern "C" int emu_deflate_shared_bytes() { return (int)sizeof(hd::Shared); }

// gather mode: the stream is bytes [off, off + n) of the byte-shuffled block at src
extern "C" int64_t emu_deflate_shuffled(const uint8_t* block, uint32_t n, uint8_t* dst, uint32_t cap, int level,
                                        uint32_t ts, uint32_t neb, uint32_t off) {
  hd::Shared* sh = (hd::Shared*)calloc(1, sizeof(hd::Shared));
  hd::Tune tune = hd::tune_for_level(level);
  hd::EncJob job = {block, n, (uint32_t*)dst, cap, level, ts, neb, off};
  const int64_t r = hd::deflate_stream(*sh, job, tune);
  free(sh);
  return r;
}
