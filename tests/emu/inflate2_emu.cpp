// CPU emulation driver for hsds_amd/csrc/inflate2.h (TEST INFRASTRUCTURE ONLY).
// Runs the single-source two-pass wave decoder with LANE_LOOP iterating the 64 lanes in
// order, so its orchestration (segments, sync, repairs, emit, match-ring resolve, fused
// unshuffle) is checked against libz on CPU.  Never used by the product.
#include <stdlib.h>
#include <string.h>
#include <thread>
#include "../../hsds_amd/csrc/inflate2.h"

// perm_n > 1: the output is written through the byte-unshuffle map of perm_n-byte elements
// (dst holds the unshuffled bytes), as the engine does for F2 chunks.
// dst_off: the stream's output starts dst_off bytes into dst (dst has dst_len + dst_off + 8
// bytes; the bytes around the output must stay untouched)
// nwaves == 2, 4 or 8: the window pipeline of inflate2w_kernel -- one thread per emulated
// wavefront, sharing a hz2::Ctl and the previous window's wavefront's LDS tables; all must
// return the same status
// Tune::spin_max of the emulated pipeline (0: hz2::SPIN_MAX); tests set it tiny to force the
// pipeline's wait timeouts and so its one-wavefront fallback
static uint32_t g_spin_max = 0;
extern "C" void emu_set_spin_max(uint32_t v) { g_spin_max = v; }

template <int NW>
static int run_pipe(hz2::Shared* sh0, const hz2::Job& job, const hz2::Tune& tune, uint8_t* ring0, hz2::Stats& st) {
  hz2::Shared* sh[NW];
  uint8_t* ring[NW];
  hz2::Stats sts[NW] = {};
  int rs[NW] = {};
  sh[0] = sh0; ring[0] = ring0;
  for (int w = 1; w < NW; w++) {
    sh[w] = (hz2::Shared*)calloc(1, sizeof(hz2::Shared));
    ring[w] = (uint8_t*)malloc(hz2::SCRATCH_BYTES);
  }
  hz2::Ctl ctl;
  memset(&ctl, 0, sizeof(ctl));
  hz2::ctl_reset(&ctl, 0);
  std::thread t[NW];
  for (int w = 1; w < NW; w++)
    t[w] = std::thread([&, w]() {
      rs[w] = hz2::inflate_stream_pipe<hz2::Stats, NW>(*sh[w], job, tune, ring[w], &sts[w], nullptr,
                                                       hz2::Pipe{&ctl, sh[(w + NW - 1) % NW], (uint32_t)w});
    });
  rs[0] = hz2::inflate_stream_pipe<hz2::Stats, NW>(*sh[0], job, tune, ring[0], &sts[0], nullptr,
                                                   hz2::Pipe{&ctl, sh[NW - 1], 0u});
  int r = rs[0];
  for (int w = 1; w < NW; w++) {
    t[w].join();
    if (rs[w] != r) r = -100;          // the wavefronts disagree: a pipeline bug
  }
  for (int w = 0; w < NW; w++) {
    uint64_t* a = (uint64_t*)&st;
    const uint64_t* b = (const uint64_t*)&sts[w];
    for (size_t i = 0; i < sizeof(st) / 8; i++) a[i] += b[i];
  }
  for (int w = 1; w < NW; w++) {
    free(ring[w]);
    free(sh[w]);
  }
  return r;
}

static int run_stream(hz2::Shared* sh, const hz2::Job& job, const hz2::Tune& tune, uint8_t* ring, hz2::Stats& st,
                      int nwaves) {
  if (nwaves >= 8) return run_pipe<8>(sh, job, tune, ring, st);
  if (nwaves >= 4) return run_pipe<4>(sh, job, tune, ring, st);
  if (nwaves == 2) return run_pipe<2>(sh, job, tune, ring, st);
  return hz2::inflate_stream<hz2::Stats, 1>(*sh, job, tune, ring, &st);
}

extern "C" int emu_inflate2_nw(const uint8_t* src, uint32_t src_len, uint8_t* dst, uint32_t dst_len, uint32_t W,
                               int max_rounds, uint32_t over16, uint32_t perm_n, uint32_t dst_off, uint64_t* stats_out,
                               int nwaves) {
  hz2::Shared* sh = (hz2::Shared*)calloc(1, sizeof(hz2::Shared));
  uint8_t* ring = (uint8_t*)malloc(hz2::SCRATCH_BYTES);
  hz2::Stats st = {};
  // perm_n > 1: the engine's pipeline for shuffled chunks -- inflate into staging, then the
  // byte unshuffle (unshuffle_kernel) into dst
  const uint32_t n = perm_n < 1 ? 1 : perm_n;
  uint8_t* stage = n > 1 ? (uint8_t*)malloc(dst_len + 16) : nullptr;
  hz2::Job job = {src, src_len, n > 1 ? stage + (dst_off & 15u) : dst + dst_off, dst_len, 1u, nullptr, hz2::perm_make(1, 1, 0)};
  hz2::Tune tune = {W, max_rounds, over16, g_spin_max};
  int r = run_stream(sh, job, tune, ring, st, nwaves);
  if (n > 1) {
    if (r == 0) {
      const uint8_t* in = stage + (dst_off & 15u);
      const uint32_t cnt = dst_len / n, body = cnt * n;
      for (uint32_t q = 0; q < dst_len; q++) dst[dst_off + q] = q >= body ? in[q] : in[(q % n) * cnt + q / n];
    }
    free(stage);
  }
  if (stats_out) {
    const uint64_t v[] = {st.windows, st.blocks, st.stored, st.tokens, st.matches, st.lanes_valid, st.repairs,
                          st.repair_lanes, st.cuts, st.batches, st.hops, st.steps_a, st.steps_e, st.extra_windows, st.fill_max, st.fill_sum, st.span_sum, st.src_in, st.src_far[0], st.src_far[1], st.src_far[2], st.src_far[3], st.hangs};
    for (int i = 0; i < 23; i++) stats_out[i] = v[i];
  }
  free(ring);
  free(sh);
  return r;
}

extern "C" int emu_inflate2(const uint8_t* src, uint32_t src_len, uint8_t* dst, uint32_t dst_len, uint32_t W,
                            int max_rounds, uint32_t over16, uint32_t perm_n, uint32_t dst_off, uint64_t* stats_out) {
  return emu_inflate2_nw(src, src_len, dst, dst_len, W, max_rounds, over16, perm_n, dst_off, stats_out, 1);
}

extern "C" int emu2_shared_bytes() { return (int)sizeof(hz2::Shared); }
