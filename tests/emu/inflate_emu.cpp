// CPU emulation driver for hsds_amd/csrc/inflate_wave.h (TEST INFRASTRUCTURE ONLY).
// Runs the exact single-source wave algorithm with LANE_LOOP iterating the 64
// lanes in order, so the kernel's orchestration (speculation, sync, rounds) is
// checked against libz on CPU.  Never used by the product.
#include <stdlib.h>
#include "../../hsds_amd/csrc/inflate_wave.h"

extern "C" int emu_inflate(const uint8_t* src, uint32_t src_len, uint8_t* dst, uint32_t dst_len,
                           uint32_t L0, uint32_t W, uint32_t adapt, uint32_t C, int max_rounds, uint64_t* stats_out) {
  hz::Shared* sh = (hz::Shared*)calloc(1, sizeof(hz::Shared));
  hz::Stats st = {};
  hz::StreamJob job = {src, src_len, dst, dst_len, 1u, nullptr};
  hz::Tune tune = {L0, W > (uint32_t)hz::WMAX ? (uint32_t)hz::WMAX : W, adapt, C > (uint32_t)hz::CMAX ? (uint32_t)hz::CMAX : C, max_rounds};
  int r = hz::inflate_stream<hz::Stats>(*sh, job, tune, &st);
  if (stats_out) {
    stats_out[0] = st.windows; stats_out[1] = st.lanes_valid; stats_out[2] = st.tokens;
    stats_out[3] = st.matches; stats_out[4] = st.match_bytes; stats_out[5] = st.lit_bytes;
    stats_out[6] = st.rounds; stats_out[7] = st.blocks; stats_out[8] = st.stored;
    stats_out[9] = st.steps_max; stats_out[10] = st.steps_sum; stats_out[11] = st.repairs; stats_out[12] = st.hops; stats_out[13] = st.maxhops;
  }
  free(sh);
  return r;
}

extern "C" int emu_shared_bytes() { return (int)sizeof(hz::Shared); }

// token dump for analysis: returns number of tokens written (len<<16|dist or literal)
#include <zlib.h>
