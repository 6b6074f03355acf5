// CPU emulation driver for hsds_amd/csrc/bshuf.h (TEST INFRASTRUCTURE ONLY): runs the
// single-source bitshuffle+LZ4 chunk decoder with LANE_LOOP iterating the 64 lanes.
#include <stdlib.h>
#include "../../hsds_amd/csrc/bshuf.h"

// returns the chunk status (0 or a negative HSDS_ERR_*)
extern "C" int emu_bshuf_chunk(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t chunk_bytes, uint32_t es) {
  bs::Shared* sh = (bs::Shared*)calloc(1, sizeof(bs::Shared));
  uint8_t* stg = (uint8_t*)malloc(chunk_bytes ? chunk_bytes : 1);
  const int st = bs::chunk(*sh, src, n, dst, stg, chunk_bytes, es);
  free(stg);
  free(sh);
  return st;
}

// the inverse transposition alone (cnt % 8 == 0)
extern "C" void emu_bshuf_untrans(const uint8_t* in, uint8_t* out, uint32_t cnt, uint32_t es) {
  bs::untrans_block(in, out, cnt, es);
}

// the forward transposition of the write path (cnt % 8 == 0): every row byte q
extern "C" void emu_bshuf_trans(const uint8_t* in, uint8_t* out, uint32_t cnt, uint32_t es) {
  for (uint32_t q = 0; q < cnt / 8u; q++) bs::trans_group(in, out, q, cnt / 8u, es);
}
