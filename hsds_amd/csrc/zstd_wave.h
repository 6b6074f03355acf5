// zstd_wave.h -- Zstandard (RFC 8878) split decoder, one wavefront per Blosc split.
//
// Same format work as zstd_lane.h (whose table builders it reuses), arranged for a
// wavefront (DESIGN.md "zstd"):
//   * decode tables (FSE, Huffman) live in LDS and are read by broadcast;
//   * the 4 Huffman literal streams of a block are decoded by lanes 0-3 at once, into
//     the END of the split's output span (the literal area);
//   * the sequence bitstream is staged into LDS 2 KiB at a time and walked by uniform
//     code (the FSE chain is serial), NSEQ sequences per window;
//   * a window's output bytes are resolved by all 64 lanes like lz_wave.h: literal bytes
//     from the literal area, match bytes by the periodic extension m - d + (k mod d).
//     The write frontier can catch up with the literal area near a block's end, so the
//     lanes work in iterations of 64 x 16 bytes: every lane loads, the wave syncs, every
//     lane stores; a match chain that leaves the current iteration reads the (final)
//     output instead of following the chain into bytes that may have been overwritten.
//
// Single source: tests/emu/zstd_emu.cpp runs the same code on CPU.
#pragma once
#include "zstd_lane.h"

#if HZ_GPU
#define LZ_LANE0_ZW if (threadIdx.x == 0)
#else
#define LZ_LANE0_ZW
#endif

namespace zw {

constexpr int NSEQ = 128;
constexpr int STG = 1024;                 // staged sequence-bitstream bytes

struct Shared {
  zs::Tables t;
  uint32_t s_out[NSEQ + 1];               // output offset of each window sequence; [n] = window end
  uint32_t s_lit[NSEQ];                   // literal bytes
  uint32_t s_src[NSEQ];                   // literal-area index of the first literal
  uint32_t s_off[NSEQ];                   // match distance (0: none)
  uint32_t stage[STG / 4 + 4];
  int32_t u_err;
};

// a uniform value: held in a scalar register on the GPU (the sequence decode is serial
// and runs on the scalar unit instead of 64 copies of it on the vector unit)
HZ_HD uint32_t uni(uint32_t v) {
#if HZ_GPU
  return __builtin_amdgcn_readfirstlane(v);
#else
  return v;
#endif
}
HZ_HD uint32_t ub8(const zs::In& in, uint32_t i) { return uni(zs::b8(in, i)); }
// an FSE entry {sym, nb, base} as one word: sym | nb << 8 | base << 16
HZ_HD uint32_t fse_word(const zs::Fse& e) { return uni((uint32_t)e.sym | ((uint32_t)e.nb << 8) | ((uint32_t)e.base << 16)); }

// staged backward bitstream of the sequences (uniform): the input bytes are staged into
// LDS STG bytes at a time, and the bits are read from a 64-bit register window over
// the stage (refilled with three LDS words every ~57 bits).  A sequence bitstream is
// shorter than a block (128 KiB), so bit positions fit 32 bits.
struct SBits {
  zs::In in;
  uint32_t lo, n;     // stream = input bytes [lo, lo + n)
  int32_t pos;        // bits left (negative after reading past the start: an error)
  int32_t sb;         // first stream byte in the stage (-1: none)
  int32_t wbit;       // stream bit of window bit 0 (a byte boundary; -1: none)
  uint64_t win;
};

#if HZ_GPU
__device__
#else
static
#endif
inline void sb_stage(Shared& ls, SBits& b, int32_t first) {
  WAVE_SYNC();
  LANE_LOOP {
    for (uint32_t k0 = 0; k0 < (uint32_t)STG / 4u + 4u; k0 += 64u) {   // uniform trip count
      const uint32_t k = k0 + (uint32_t)lane;
      uint32_t v = 0;
      for (uint32_t i = 0; i < 4u; i++) {
        const int32_t bi = first + 4 * (int32_t)k + (int32_t)i;
        v |= (bi >= 0 && bi < (int32_t)b.n ? zs::b8(b.in, b.lo + (uint32_t)bi) : 0u) << (8 * i);
      }
      if (k < (uint32_t)STG / 4u + 4u) ls.stage[k] = v;
    }
  }
  WAVE_SYNC();
  b.sb = (int32_t)uni((uint32_t)first);
}

#if HZ_GPU
__device__
#else
static
#endif
inline void sb_refill(Shared& ls, SBits& b) {
  int32_t by = (b.pos - 57) >> 3;            // window bytes [by, by + 8) hold >= 57 bits below pos
  if (by < 0) by = 0;
  if (b.sb < 0 || by < b.sb || by + 8 > b.sb + STG) {
    const int32_t f = by + 8 - STG;
    sb_stage(ls, b, f < 0 ? 0 : f);
  }
  const uint32_t r = (uint32_t)(by - b.sb), wi = r >> 2, sh = (r & 3u) * 8u;
  const uint64_t lo = (uint64_t)uni(ls.stage[wi]) | ((uint64_t)uni(ls.stage[wi + 1]) << 32);
  const uint64_t hi = uni(ls.stage[wi + 2]);
  b.win = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
  b.wbit = (int32_t)uni((uint32_t)(by * 8));
}

// the next k (<= 32) bits, most significant first; bits before the start read as 0
#if HZ_GPU
__device__
#else
static
#endif
inline uint32_t sb_read(Shared& ls, SBits& b, uint32_t k) {
  if (!k) return 0;
  const int32_t np = b.pos - (int32_t)k;
  const int32_t lo_bit = np < 0 ? 0 : np;
  if (b.wbit < 0 || lo_bit < b.wbit || b.pos > b.wbit + 64) sb_refill(ls, b);
  const uint64_t mask = (1ull << k) - 1ull;
  uint32_t v = (uint32_t)((b.win >> (uint32_t)(lo_bit - b.wbit)) & mask);
  if (np < 0) v = (uint32_t)(((uint64_t)v << (-np)) & mask);
  b.pos = (int32_t)uni((uint32_t)np);
  return v;
}

// largest k <= hi with s_out[k] <= p
HZ_HD uint32_t find_seq(const Shared& ls, uint32_t hi, uint32_t p) {
  uint32_t lo = 0;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (ls.s_out[mid] <= p) lo = mid; else hi = mid - 1u;
  }
  return lo;
}

// resolve and store the window's output [wb, we) (nseq sequences in the LDS table)
#if HZ_GPU
__device__
#else
static
#endif
inline void resolve(Shared& ls, hz_gu8* dst, uint32_t dmis, hz_gu8* lit, uint32_t wb, uint32_t we, uint32_t nseq,
                    HzProf* prof) {
  (void)prof;
  const uint32_t g0 = (wb + dmis) >> 4, g1 = (we + dmis + 15u) >> 4;
  for (uint32_t it = g0; it < g1; it += 64u) {
    const uint32_t ia = it * 16u;
    const uint32_t it_lo = ia > wb + dmis ? ia - dmis : wb;     // first window byte of the iteration
    LANE_VAR(uint32_t, have);
    LANE_VAR(uint32_t, w0);
    LANE_VAR(uint32_t, w1);
    LANE_VAR(uint32_t, w2);
    LANE_VAR(uint32_t, w3);
    LANE_LOOP {
      const uint32_t g = it + (uint32_t)lane;
      uint32_t hv = 0, ww[4] = {0u, 0u, 0u, 0u};
      if (g < g1) {
        const uint32_t a0 = g * 16u;
        const uint32_t pb = a0 > wb + dmis ? a0 - dmis : wb;
        uint32_t t = find_seq(ls, nseq - 1u, pb);
        uint32_t t_end = t + 1u < nseq ? ls.s_out[t + 1u] : we;
        hz_gu8* sp[16];
        HZ_UNROLL
        for (uint32_t k = 0; k < 16u; k++) {
          const uint32_t ak = a0 + k;
          sp[k] = dst;
          if (ak < wb + dmis || ak >= we + dmis) continue;
          const uint32_t p = ak - dmis;
          while (p >= t_end) { t++; t_end = t + 1u < nseq ? ls.s_out[t + 1u] : we; }
          uint32_t q = p, u = t;
          for (;;) {
            const uint32_t ub = ls.s_out[u], rel = q - ub, nl = ls.s_lit[u];
            if (rel < nl) { sp[k] = lit + ls.s_src[u] + rel; break; }
            const uint32_t m = ub + nl, d = ls.s_off[u], kk = q - m;
            const uint32_t q2 = m - d + (kk < d ? kk : kk % d);
            if (q2 < it_lo) { sp[k] = dst + q2; break; }     // final output (earlier window / iteration)
            u = find_seq(ls, u, q2);
            q = q2;
          }
          hv |= 1u << k;
        }
        HZ_T(6);
        HZ_UNROLL
        for (uint32_t k = 0; k < 16u; k++) ww[k >> 2] |= (uint32_t)*sp[k] << (8u * (k & 3u));
      }
      LV(have) = hv;
      LV(w0) = ww[0]; LV(w1) = ww[1]; LV(w2) = ww[2]; LV(w3) = ww[3];
    }
    HZ_T(7);
    WAVE_SYNC_GLOBAL();       // every load of the iteration before any store
    LANE_LOOP {
      const uint32_t g = it + (uint32_t)lane;
      if (g < g1) {
        const uint32_t a0 = g * 16u;
        const uint32_t ww[4] = {LV(w0), LV(w1), LV(w2), LV(w3)};
        for (uint32_t i = 0; i < 4u; i++) {
          const uint32_t hm = (LV(have) >> (4u * i)) & 15u;
          if (hm == 15u) *(hz_gu32*)(dst + (a0 + 4u * i - dmis)) = ww[i];
          else if (hm)
            for (uint32_t k = 0; k < 4u; k++)
              if (hm & (1u << k)) dst[a0 + 4u * i + k - dmis] = (uint8_t)(ww[i] >> (8u * k));
        }
      }
    }
    WAVE_SYNC_GLOBAL();
    HZ_T(3);
  }
}

// one compressed block at input [at, at + n); output from op; returns the new op or < 0 (uniform)
#if HZ_GPU
__device__
#else
static
#endif
inline int64_t block(Shared& ls, const zs::In& in, uint32_t at, uint32_t n, hz_gu8* dst, uint32_t dmis, uint32_t op,
                     uint32_t cap, HzProf* prof) {
  (void)prof;
  zs::Tables& t = ls.t;
  HZ_T(1);
  if (n < 1) return zs::E_DATA;
  const uint32_t h0 = ub8(in, at), lt = h0 & 3u, sf = (h0 >> 2) & 3u;
  uint32_t rsz, csz = 0, hl, ns = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { rsz = h0 >> 3; hl = 1; }
    else if (sf == 1) { if (n < 2) return zs::E_DATA; rsz = (h0 >> 4) | (ub8(in, at + 1) << 4); hl = 2; }
    else { if (n < 3) return zs::E_DATA; rsz = (h0 >> 4) | (ub8(in, at + 1) << 4) | (ub8(in, at + 2) << 12); hl = 3; }
  } else {
    hl = sf < 2 ? 3u : sf == 2 ? 4u : 5u;
    if (n < hl) return zs::E_DATA;
    uint64_t v = 0;
    for (int i = (int)hl - 1; i >= 0; i--) v = (v << 8) | ub8(in, at + (uint32_t)i);
    const uint32_t bits = sf < 2 ? 10u : sf == 2 ? 14u : 18u;
    rsz = (uint32_t)((v >> 4) & ((1u << bits) - 1u));
    csz = (uint32_t)((v >> (4 + bits)) & ((1u << bits) - 1u));
    ns = sf == 0 ? 1u : 4u;
  }
  if (rsz > (1u << 17) || rsz > cap - op) return zs::E_DATA;
  const uint32_t lbase = cap - rsz;
  hz_gu8* lit = dst + lbase;
  uint32_t q = hl;
  if (lt == 0) {
    if (q + rsz > n) return zs::E_TRUNC;
    LANE_LOOP { for (uint32_t i = (uint32_t)lane; i < rsz; i += 64u) lit[i] = (uint8_t)zs::b8(in, at + q + i); }
    q += rsz;
  } else if (lt == 1) {
    if (q + 1 > n) return zs::E_TRUNC;
    const uint8_t c = (uint8_t)ub8(in, at + q);
    LANE_LOOP { for (uint32_t i = (uint32_t)lane; i < rsz; i += 64u) lit[i] = c; }
    q += 1;
  } else {
    if (q + csz > n) return zs::E_TRUNC;
    int64_t tsz = 0;
    if (lt == 2) {
      HZ_T(4);
      WAVE_SYNC();
      tsz = (int64_t)(int32_t)uni((uint32_t)zs::huf_tree(t, in, at + q, csz));
      WAVE_SYNC();
      if (tsz < 0) return zs::E_DATA;
    } else if (!uni(t.have_huf)) {
      return zs::E_DATA;
    }
    const uint32_t s0 = at + q + (uint32_t)tsz, ssz = csz - (uint32_t)tsz;
    HZ_T(1);
    if (ns == 1) {
      LANE_LOOP { if (lane == 0) ls.u_err = zs::huf_stream(t, in, s0, ssz, lit, rsz); }
    } else {
      if (ssz < 6) return zs::E_DATA;
      const uint32_t l1 = ub8(in, s0) | (ub8(in, s0 + 1) << 8), l2 = ub8(in, s0 + 2) | (ub8(in, s0 + 3) << 8),
                     l3 = ub8(in, s0 + 4) | (ub8(in, s0 + 5) << 8);
      if (l1 + l2 + l3 + 6 > ssz) return zs::E_DATA;
      const uint32_t l4 = ssz - 6 - l1 - l2 - l3;
      const uint32_t seg = (rsz + 3) / 4;
      if (rsz < 3 * seg) return zs::E_DATA;
      const uint32_t p1 = s0 + 6;
      LANE_LOOP { if (lane == 0) ls.u_err = 0; }
      WAVE_SYNC();
      LANE_LOOP {
        if (lane < 4) {                       // the 4 streams in parallel
          const uint32_t off = lane == 0 ? 0u : lane == 1 ? l1 : lane == 2 ? l1 + l2 : l1 + l2 + l3;
          const uint32_t len = lane == 0 ? l1 : lane == 1 ? l2 : lane == 2 ? l3 : l4;
          const uint32_t cnt = lane == 3 ? rsz - 3 * seg : seg;
          if (zs::huf_stream(t, in, p1 + off, len, lit + (uint32_t)lane * seg, cnt)) ls.u_err = -1;
        }
      }
    }
    WAVE_SYNC();
    if (uni((uint32_t)ls.u_err)) return zs::E_DATA;
    q += csz;
  }
  WAVE_SYNC_GLOBAL();         // literals visible to every lane
  // ---- sequences ----
  if (q >= n) return zs::E_TRUNC;
  uint32_t nseq = ub8(in, at + q++);
  if (nseq >= 128) {
    if (nseq < 255) { if (q >= n) return zs::E_TRUNC; nseq = ((nseq - 128) << 8) + ub8(in, at + q++); }
    else { if (q + 1 >= n) return zs::E_TRUNC; nseq = ub8(in, at + q) + (ub8(in, at + q + 1) << 8) + 0x7F00; q += 2; }
  }
  uint32_t lp = 0;
  SBits b;
  uint32_t sll = 0, sof = 0, sml = 0;
  uint32_t rep0 = uni(t.rep[0]), rep1 = uni(t.rep[1]), rep2 = uni(t.rep[2]);
  if (nseq > 0) {
    if (q >= n) return zs::E_TRUNC;
    const uint32_t modes = ub8(in, at + q++);
    if (modes & 3) return zs::E_DATA;
    HZ_T(5);
    WAVE_SYNC();
    int64_t u = (int32_t)uni((uint32_t)zs::seq_table(t, t.ll, t.ll_al, (modes >> 6) & 3, in, at + q, n - q, 0, 35, 9));
    if (u < 0) return zs::E_DATA;
    q += (uint32_t)u;
    u = (int32_t)uni((uint32_t)zs::seq_table(t, t.of, t.of_al, (modes >> 4) & 3, in, at + q, n - q, 1, 31, 8));
    if (u < 0) return zs::E_DATA;
    q += (uint32_t)u;
    u = (int32_t)uni((uint32_t)zs::seq_table(t, t.ml, t.ml_al, (modes >> 2) & 3, in, at + q, n - q, 2, 52, 9));
    if (u < 0) return zs::E_DATA;
    q += (uint32_t)u;
    t.have_seq = 1;
    WAVE_SYNC();
    if (n - q == 0 || ub8(in, at + n - 1) == 0) return zs::E_DATA;
    b.in = in; b.lo = at + q; b.n = n - q; b.sb = -1; b.wbit = -1; b.win = 0;
    b.pos = 8 * (int32_t)(b.n - 1) + (int32_t)zs::hib(ub8(in, at + n - 1));
    const uint32_t lal = uni(t.ll_al), oal = uni(t.of_al), mal = uni(t.ml_al);
    const uint32_t v = sb_read(ls, b, lal + oal + mal);      // LL, OF, ML initial states
    sll = v >> (oal + mal); sof = (v >> mal) & ((1u << oal) - 1u); sml = v & ((1u << mal) - 1u);
  }
  uint32_t k = 0;
  for (;;) {
    HZ_T(2);
    // ---- decode up to NSEQ sequences (uniform, scalar) ----
    const uint32_t wb = op;
    uint32_t ns_w = 0;
    while (k < nseq && ns_w < (uint32_t)NSEQ - 1u) {
      const uint32_t ell = fse_word(t.ll[sll]), eof = fse_word(t.of[sof]), eml = fse_word(t.ml[sml]);
      const uint32_t llc = ell & 255u, ofc = eof & 255u, mlc = eml & 255u;
      if (llc > 35 || mlc > 52 || ofc > 31) return zs::E_DATA;
      // extra bits: offset, then match length, then literal length
      const uint32_t ofv = (1u << ofc) + sb_read(ls, b, ofc);
      const uint32_t mlb = zs::ml_bits(mlc), llb = zs::ll_bits(llc);
      const uint32_t vx = sb_read(ls, b, mlb + llb);
      const uint32_t ml = zs::ml_base(mlc) + (vx >> llb);
      const uint32_t ll = zs::ll_base(llc) + (vx & ((1u << llb) - 1u));
      uint32_t off;
      if (ofv > 3) {
        off = ofv - 3;
        rep2 = rep1; rep1 = rep0; rep0 = off;
      } else {
        const uint32_t idx = ofv - 1u + (ll == 0 ? 1u : 0u);
        if (idx == 0) off = rep0;
        else {
          off = idx == 3 ? rep0 - 1u : idx == 1 ? rep1 : rep2;
          if (idx != 1) rep2 = rep1;
          rep1 = rep0; rep0 = off;
        }
      }
      if (k + 1 < nseq) {       // state updates: LL, then ML, then OF
        const uint32_t nl = (ell >> 8) & 255u, nm = (eml >> 8) & 255u, no = (eof >> 8) & 255u;
        const uint32_t vs = sb_read(ls, b, nl + nm + no);
        sll = (ell >> 16) + (vs >> (nm + no));
        sml = (eml >> 16) + ((vs >> no) & ((1u << nm) - 1u));
        sof = (eof >> 16) + (vs & ((1u << no) - 1u));
      }
      if (ll > rsz - lp) return zs::E_DATA;
      if ((uint64_t)op + ml + (rsz - lp) > cap) return zs::E_SIZE;
      if (off == 0 || (uint64_t)off > (uint64_t)op + ll) return zs::E_DATA;
      // every lane stores the same words: a lane-0 branch would make the loop divergent
      // and push its uniform state into vector registers
      ls.s_out[ns_w] = op; ls.s_lit[ns_w] = ll; ls.s_src[ns_w] = lp; ls.s_off[ns_w] = off;
      ns_w++;
      op += ll + ml; lp += ll;
      k++;
    }
    const int last = k >= nseq;
    if (last) {
      if (nseq > 0 && b.pos != 0) return zs::E_DATA;
      WAVE_SYNC();
      LZ_LANE0_ZW { t.rep[0] = rep0; t.rep[1] = rep1; t.rep[2] = rep2; }
      const uint32_t rest = rsz - lp;
      if ((uint64_t)op + rest > cap) return zs::E_SIZE;
      if (rest) {
        LZ_LANE0_ZW { ls.s_out[ns_w] = op; ls.s_lit[ns_w] = rest; ls.s_src[ns_w] = lp; ls.s_off[ns_w] = 0; }
        ns_w++;
        op += rest; lp += rest;
      }
    }
    WAVE_SYNC();
    HZ_T(3);
    if (ns_w) resolve(ls, dst, dmis, lit, wb, op, ns_w, prof);
    if (last) break;
  }
  HZ_T(0);
  return (int64_t)op;
}

// Decode one zstd frame (src, n) into exactly cap bytes at dst.  Returns OK or < 0 (uniform).
#if HZ_GPU
__device__
#else
static
#endif
inline int frame(Shared& ls, const uint8_t* src, uint32_t n, uint8_t* dstp, uint32_t cap, HzProf* prof = nullptr) {
  zs::In in = {src, n};
  hz_gu8* dst = HZ_GLOBAL(hz_gu8*, dstp);
  const uint32_t dmis = (uint32_t)(((uintptr_t)dstp) & 3u);
  zs::Tables& t = ls.t;
  if (n < 5) return zs::E_TRUNC;
  if ((ub8(in, 0) | ub8(in, 1) << 8 | ub8(in, 2) << 16 | ub8(in, 3) << 24) != 0xFD2FB528u) return zs::E_DATA;
  const uint32_t fhd = ub8(in, 4);
  const uint32_t fcsf = fhd >> 6, single = (fhd >> 5) & 1u, cks = (fhd >> 2) & 1u, didf = fhd & 3u;
  if (fhd & 8u) return zs::E_DATA;
  if (didf) return zs::E_UNSUP;
  uint32_t q = 5 + (single ? 0u : 1u);
  const uint32_t fcsb = fcsf == 0 ? (single ? 1u : 0u) : fcsf == 1 ? 2u : fcsf == 2 ? 4u : 8u;
  if (q + fcsb > n) return zs::E_TRUNC;
  int64_t fcs = -1;
  if (fcsb) {
    uint64_t v = 0;
    for (int i = (int)fcsb - 1; i >= 0; i--) v = (v << 8) | ub8(in, q + (uint32_t)i);
    fcs = (int64_t)(fcsb == 2 ? v + 256 : v);
  }
  q += fcsb;
  WAVE_SYNC();
  LZ_LANE0_ZW {
    t.have_seq = 0; t.have_huf = 0;
    t.rep[0] = 1; t.rep[1] = 4; t.rep[2] = 8;
  }
  WAVE_SYNC();
  uint32_t op = 0;
  for (;;) {
    if (q + 3 > n) return zs::E_TRUNC;
    const uint32_t bh = ub8(in, q) | (ub8(in, q + 1) << 8) | (ub8(in, q + 2) << 16);
    q += 3;
    const uint32_t last = bh & 1u, type = (bh >> 1) & 3u, bsz = bh >> 3;
    if (type == 3 || bsz > (1u << 17)) return zs::E_DATA;
    if (type == 0) {
      if (q + bsz > n) return zs::E_TRUNC;
      if (bsz > cap - op) return zs::E_SIZE;
      LANE_LOOP { for (uint32_t i = (uint32_t)lane; i < bsz; i += 64u) dst[op + i] = (uint8_t)zs::b8(in, q + i); }
      op += bsz; q += bsz;
    } else if (type == 1) {
      if (q + 1 > n) return zs::E_TRUNC;
      if (bsz > cap - op) return zs::E_SIZE;
      const uint8_t c = (uint8_t)ub8(in, q);
      LANE_LOOP { for (uint32_t i = (uint32_t)lane; i < bsz; i += 64u) dst[op + i] = c; }
      op += bsz; q += 1;
    } else {
      if (q + bsz > n) return zs::E_TRUNC;
      const int64_t o2 = block(ls, in, q, bsz, dst, dmis, op, cap, prof);
      if (o2 < 0) return (int)o2;
      op = (uint32_t)o2; q += bsz;
    }
    WAVE_SYNC_GLOBAL();
    if (last) break;
  }
  if (fcs >= 0 && fcs != (int64_t)op) return zs::E_SIZE;
  if (op != cap) return zs::E_SIZE;
  if (cks) {
    if (q + 4 > n) return zs::E_TRUNC;
    const uint32_t want = ub8(in, q) | ub8(in, q + 1) << 8 | ub8(in, q + 2) << 16 | ub8(in, q + 3) << 24;
    if ((uint32_t)zs::xxh64(dst, op) != want) return zs::E_DATA;
  }
  return zs::OK;
}

}  // namespace zw
