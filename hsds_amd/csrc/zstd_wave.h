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

#ifndef ZW_WALK4
#define ZW_WALK4 0                    // FSE walk: four stage dwords read with the table entries
                                      // (one LDS round trip per sequence; measured slower: bench
                                      // zstd 63.1 -> 57.0 GB/s, the 4 reads cost more than the wait)
#endif
#ifndef ZW_HUF_PAR
#define ZW_HUF_PAR 1                  // Huffman literal streams on every lane (0: one lane per stream)
#endif
#ifndef ZW_PRIO_KB
#define ZW_PRIO_KB 32                 // wave priority: one level per 32 KiB of the split's input left (0: off)
#endif
namespace zw {

constexpr int NSEQ = 128;
constexpr int STG = 864;                  // staged sequence-bitstream bytes
constexpr int32_t SB_NONE = -(1 << 30);

// one window sequence.  The FSE walk stores {LL entry, OF entry, ML entry, bit position}
// (packed entries, below); the lane pass turns it into {out, lit, src, off}.
enum : uint32_t { SQ_OUT = 0, SQ_LIT = 1, SQ_SRC = 2, SQ_OFF = 3 };

// The wavefront's tables.  Same members as zs::Tables (the builders are shared), but the
// Huffman table, the table-description scratch and the sequence window share one LDS
// region: the Huffman table is dead once the literals are decoded (a treeless literals
// section rebuilds it from the kept weights), the scratch once the tables are built.
// 9.8 KB of LDS: four one-wavefront workgroups per SIMD.
struct WTables {
  zs::Fse ll[512], of[256], ml[512];
  zs::Fse hw[64];                          // Huffman weights table (accuracy <= 6)
  uint32_t ll_al, of_al, ml_al, have_seq, huf_bits, have_huf, huf_nw;
  uint32_t rep[3];
  uint8_t w[256];                          // Huffman weights (kept for treeless sections)
  union {
    zs::Huf huf[1 << 11];                  // the literals section
    struct { int16_t norm[256]; uint16_t next[256]; };        // table descriptions
    struct {                               // the sequences section
      alignas(16) uint32_t seq[NSEQ + 1][4];   // out: output offset; lit: literal bytes; src:
                                               // literal-area index of the first literal; off:
                                               // match distance (0: none)
      alignas(16) uint8_t ib[1024];            // resolve: the iteration's output bytes
      uint16_t pm[64];                         // resolve: each lane's bytes still pending
      uint32_t stage[STG / 4 + 4];
    };
  };
};

struct Shared {
  WTables t;
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
HZ_HD uint64_t uni64(uint64_t v) { return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v); }
HZ_HD uint32_t ub8(const zs::In& in, uint32_t i) { return uni(zs::b8(in, i)); }
// A sequence-table entry, repacked in place once its table is built:
//   bits 0..15 state baseline, 16..19 state bits, 20..24 extra bits of the code, 25..31 code
// so the serial FSE walk learns everything it needs from one LDS dword per table.
static_assert(sizeof(zs::Fse) == 4, "an FSE entry is one dword");
HZ_HD uint32_t sq_pack(const zs::Fse& e, uint32_t which) {
  const uint32_t c = e.sym;
  const uint32_t eb = which == 0 ? zs::ll_bits(c) : which == 1 ? c : zs::ml_bits(c);
  return (uint32_t)e.base | ((uint32_t)e.nb << 16) | (eb << 20) | (c << 25);
}
HZ_HD uint32_t sq_base(uint32_t e) { return e & 0xffffu; }
HZ_HD uint32_t sq_nb(uint32_t e) { return (e >> 16) & 15u; }
HZ_HD uint32_t sq_eb(uint32_t e) { return (e >> 20) & 31u; }
HZ_HD uint32_t sq_code(uint32_t e) { return e >> 25; }

// The predefined distributions' tables (RFC 8878 3.1.1.3.2.2), built at compile time in
// the packed form and copied into LDS when a block selects them: built at run time, the
// compiler folds the whole construction into constants that then occupy vector
// registers for the kernel's lifetime.
struct PreTab { uint32_t e[64]; };
constexpr PreTab pre_build(uint32_t which) {
  PreTab r{};
  const uint32_t al = which == 1u ? 5u : 6u, size = 1u << al, maxsym = which == 0u ? 35u : which == 1u ? 28u : 52u;
  uint8_t sym[64] = {};
  uint32_t next[53] = {};
  int32_t high = (int32_t)size - 1;
  for (uint32_t s = 0; s <= maxsym; s++) {
    const int16_t nv = zs::def_norm(which, s);
    if (nv == -1) { sym[high--] = (uint8_t)s; next[s] = 1u; }
    else next[s] = (uint32_t)nv;
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3u, mask = size - 1u;
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= maxsym; s++)
    for (int32_t i = 0; i < zs::def_norm(which, s); i++) {
      sym[pos] = (uint8_t)s;
      do pos = (pos + step) & mask; while ((int32_t)pos > high);
    }
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t c = sym[u], ns = next[c]++;
    const uint32_t nb = al - zs::hib(ns), base = (ns << nb) - size;
    const uint32_t eb = which == 0u ? zs::ll_bits(c) : which == 1u ? c : zs::ml_bits(c);
    r.e[u] = base | (nb << 16) | (eb << 20) | (c << 25);
  }
  return r;
}
#if HZ_GPU
__constant__ PreTab zw_pre[3] = {pre_build(0u), pre_build(1u), pre_build(2u)};
#else
static constexpr PreTab zw_pre[3] = {pre_build(0u), pre_build(1u), pre_build(2u)};
#endif

// a lane-uniform value kept in a vector register (the compiler would otherwise move each
// LDS result to a scalar register before using it)
HZ_HD uint32_t vdiv(uint32_t v) {
#if HZ_GPU
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
#else
  return v;
#endif
}
// bits [o, o + w) of x (w < 32)
HZ_HD uint32_t ubfe(uint32_t x, uint32_t o, uint32_t w) {
#if HZ_GPU
  return __builtin_amdgcn_ubfe(x, o, w);
#else
  return w ? (x >> o) & ((1u << w) - 1u) : 0u;
#endif
}
// the low 32 bits of (hi:lo) >> s, s < 32
HZ_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
#if HZ_GPU
  return __builtin_amdgcn_alignbit(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

HZ_HD uint32_t fse_word(const zs::Fse* tab, uint32_t i) {
#if HZ_GPU
  return ((const uint32_t*)tab)[i];          // one LDS dword read (callers make it uniform)
#else
  uint32_t v;
  memcpy(&v, tab + i, 4);
  return v;
#endif
}

// staged backward bitstream of the sequences (uniform): the input bytes are staged into
// LDS STG bytes at a time, and the bits are read from a 64-bit register window over
// the stage (refilled with three LDS words every ~57 bits).  A sequence bitstream is
// shorter than a block (128 KiB), so bit positions fit 32 bits.
struct SBits {
  zs::In in;
  uint32_t lo, n;     // stream = input bytes [lo, lo + n)
  int32_t pos;        // bits left (negative after reading past the start: an error)
  int32_t sb;         // stream byte of stage byte 0 (SB_NONE: nothing staged)
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
  // the stage starts at the dword-aligned address at or below stream byte `first`;
  // stage byte 0 is stream byte s0 (up to 3 bytes before `first`, possibly before the
  // stream's start).  Bytes outside the stream read as 0.
  const int32_t s0 = first - (int32_t)(((uintptr_t)b.in.p + b.lo + (uint32_t)first) & 3u);
  LANE_LOOP {
    constexpr uint32_t NWD = (uint32_t)STG / 4u + 4u, NJ = (NWD + 63u) / 64u;
    uint32_t v[NJ];
#if HZ_GPU
    // one aligned dword load per word, all issued before any is used (a word outside
    // the stream loads the word holding `first`), so a lane's loads share one latency
    hz_gcu8* bp = HZ_GLOBAL(hz_gcu8*, b.in.p) + b.lo;
    HZ_UNROLL
    for (uint32_t j = 0; j < NJ; j++) {
      const int32_t sk = s0 + 4 * (int32_t)(j * 64u + (uint32_t)lane);
      v[j] = *(hz_gcu32*)(bp + (sk + 4 > 0 && sk < (int32_t)b.n ? sk : s0));
    }
    HZ_UNROLL
    for (uint32_t j = 0; j < NJ; j++) {
      const int32_t sk = s0 + 4 * (int32_t)(j * 64u + (uint32_t)lane);     // stream byte of word k
      uint32_t w = v[j];
      if (sk < 0) w &= ~hz::bmask((uint32_t)(-sk) * 8u);
      if (sk + 4 > (int32_t)b.n) w &= hz::bmask((uint32_t)((int32_t)b.n - sk) * 8u);
      v[j] = sk + 4 > 0 && sk < (int32_t)b.n ? w : 0u;
    }
#else
    for (uint32_t j = 0; j < NJ; j++) {
      const int32_t sk = s0 + 4 * (int32_t)(j * 64u + (uint32_t)lane);     // stream byte of word k
      uint32_t w = 0;
      for (int32_t i = 0; i < 4; i++) {
        const int32_t bi = sk + i;
        if (bi >= 0 && bi < (int32_t)b.n) w |= zs::b8(b.in, b.lo + (uint32_t)bi) << (8 * i);
      }
      v[j] = w;
    }
#endif
    HZ_UNROLL
    for (uint32_t j = 0; j < NJ; j++) {
      const uint32_t k = j * 64u + (uint32_t)lane;
      if (k < NWD) ls.t.stage[k] = v[j];
    }
  }
  WAVE_SYNC();
  b.sb = (int32_t)uni((uint32_t)s0);
}

#if HZ_GPU
__device__
#else
static
#endif
inline void sb_refill(Shared& ls, SBits& b) {
  int32_t by = (b.pos - 57) >> 3;            // window bytes [by, by + 8) hold >= 57 bits below pos
  if (by < 0) by = 0;
  if (by < b.sb || by + 8 > b.sb + STG) {                 // (SB_NONE fails the second test)
    const int32_t f = by + 8 - STG;
    sb_stage(ls, b, f < 0 ? 0 : f);
  }
  const uint32_t r = (uint32_t)(by - b.sb), wi = r >> 2, sh = (r & 3u) * 8u;
  const uint64_t lo = (uint64_t)uni(ls.t.stage[wi]) | ((uint64_t)uni(ls.t.stage[wi + 1]) << 32);
  const uint64_t hi = uni(ls.t.stage[wi + 2]);
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

// largest k <= hi with seq[k].out <= p
HZ_HD uint32_t find_seq(const Shared& ls, uint32_t hi, uint32_t p) {
  uint32_t lo = 0;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (ls.t.seq[mid][SQ_OUT] <= p) lo = mid; else hi = mid - 1u;
  }
  return lo;
}
// resolve and store the window's output [wb, we) (nseq sequences in the LDS table);
// literals are at dst + lbase.  An iteration covers 64 x 16 output bytes:
//   (1) every lane finds its 16 bytes' sources: a literal, a byte of the final output
//       (an earlier window or iteration), or -- a match source inside the iteration -- a
//       pending byte; the first two are loaded (all loads of a lane together) into the
//       LDS byte buffer;
//   (2) rounds: a pending byte whose source is no longer pending copies it (the lowest
//       pending byte's source always precedes it, so every round makes progress; a
//       chain of in-iteration matches takes one round per link);
//   (3) the buffer is stored.
#if HZ_GPU
__device__
#else
static
#endif
inline void resolve(Shared& ls, hz_gu8* dst, uint32_t dmis, uint32_t lbase, uint32_t wb, uint32_t we, uint32_t nseq,
                    HzProf* prof) {
  (void)prof;
  WTables& T = ls.t;
  struct Src { uint32_t v[16]; };
  const uint32_t g0 = (wb + dmis) >> 4, g1 = (we + dmis + 15u) >> 4;
  for (uint32_t it = g0; it < g1; it += 64u) {
    const uint32_t ia = it * 16u;
    const uint32_t it_lo = ia > wb + dmis ? ia - dmis : wb;     // first window byte of the iteration
    LANE_VAR(uint32_t, have);
    LANE_VAR(uint32_t, pend);
    LANE_VAR(Src, so);
    LANE_LOOP {
      const uint32_t g = it + (uint32_t)lane;
      uint32_t hv = 0, pv = 0, ww[4] = {0u, 0u, 0u, 0u};
      Src& S = LV(so);
      if (g < g1) {
        const uint32_t a0 = g * 16u;
        const uint32_t pb = a0 > wb + dmis ? a0 - dmis : wb;
        // the lane's current sequence t, its record in registers
        uint32_t t = find_seq(ls, nseq - 1u, pb);
        uint32_t r_out = T.seq[t][SQ_OUT], r_lit = T.seq[t][SQ_LIT], r_src = T.seq[t][SQ_SRC], r_off = T.seq[t][SQ_OFF];
        uint32_t t_end = t + 1u < nseq ? T.seq[t + 1u][SQ_OUT] : we;
        uint32_t mq = ~0u;            // the previous byte's match source (same sequence), else ~0
        HZ_UNROLL
        for (uint32_t k = 0; k < 16u; k++) {
          const uint32_t ak = a0 + k;
          S.v[k] = 0;
          if (ak < wb + dmis || ak >= we + dmis) continue;
          const uint32_t p = ak - dmis;
          if (p >= t_end) {
            do { t++; t_end = t + 1u < nseq ? T.seq[t + 1u][SQ_OUT] : we; } while (p >= t_end);
            r_out = T.seq[t][SQ_OUT]; r_lit = T.seq[t][SQ_LIT]; r_src = T.seq[t][SQ_SRC]; r_off = T.seq[t][SQ_OFF];
            mq = ~0u;
          }
          const uint32_t rel = p - r_out;
          hv |= 1u << k;
          if (rel < r_lit) {
            S.v[k] = lbase + r_src + rel;
            mq = ~0u;
          } else {
            // match byte: the periodic extension m - d + (k mod d), stepped from the
            // previous byte's source when there is one (no division)
            const uint32_t m = r_out + r_lit, kk = p - m;
            const uint32_t q2 = mq != ~0u ? (mq + 1u == m ? m - r_off : mq + 1u)
                                          : m - r_off + (kk < r_off ? kk : kk % r_off);
            mq = q2;
            if (q2 < it_lo) S.v[k] = q2;                         // final output
            else { S.v[k] = q2 + dmis - ia; pv |= 1u << k; }     // a byte of this iteration
          }
        }
        HZ_T(6);
        const uint32_t ld = hv & ~pv;
        HZ_UNROLL
        for (uint32_t k = 0; k < 16u; k++) {
          const uint32_t v = dst[(ld >> k) & 1u ? S.v[k] : 0u];
          ww[k >> 2] |= ((ld >> k) & 1u ? v : 0u) << (8u * (k & 3u));
        }
      }
      uint32_t* ibw = (uint32_t*)(T.ib + 16u * (uint32_t)lane);
      ibw[0] = ww[0]; ibw[1] = ww[1]; ibw[2] = ww[2]; ibw[3] = ww[3];
      T.pm[lane] = (uint16_t)pv;
      LV(have) = hv;
      LV(pend) = pv;
    }
    HZ_T(7);
    WAVE_SYNC();
    for (;;) {
      if (!WAVE_BALLOT(LV(pend) != 0u)) break;
      LANE_VAR(uint32_t, done);
      LANE_VAR(uint32_t, v0);
      LANE_VAR(uint32_t, v1);
      LANE_VAR(uint32_t, v2);
      LANE_VAR(uint32_t, v3);
      LANE_LOOP {
        const uint32_t pv = LV(pend);
        uint32_t dn = 0, vv[4] = {0u, 0u, 0u, 0u};
        const Src& S = LV(so);
        HZ_UNROLL
        for (uint32_t k = 0; k < 16u; k++) {
          if ((pv >> k) & 1u) {
            const uint32_t sx = S.v[k];
            if (!((T.pm[sx >> 4] >> (sx & 15u)) & 1u)) {
              dn |= 1u << k;
              vv[k >> 2] |= (uint32_t)T.ib[sx] << (8u * (k & 3u));
            }
          }
        }
        LV(done) = dn;
        LV(v0) = vv[0]; LV(v1) = vv[1]; LV(v2) = vv[2]; LV(v3) = vv[3];
      }
      WAVE_SYNC();
      LANE_LOOP {
        const uint32_t dn = LV(done);
        if (dn) {
          const uint32_t vv[4] = {LV(v0), LV(v1), LV(v2), LV(v3)};
          uint32_t* ibw = (uint32_t*)(T.ib + 16u * (uint32_t)lane);
          HZ_UNROLL
          for (uint32_t i = 0; i < 4u; i++) {
            const uint32_t bm = (dn >> (4u * i)) & 15u;
            if (bm) {
              const uint32_t m = ((bm & 1u) ? 0xffu : 0u) | ((bm & 2u) ? 0xff00u : 0u) | ((bm & 4u) ? 0xff0000u : 0u) |
                                 ((bm & 8u) ? 0xff000000u : 0u);
              ibw[i] = (ibw[i] & ~m) | (vv[i] & m);
            }
          }
          LV(pend) &= ~dn;
          T.pm[lane] = (uint16_t)LV(pend);
        }
      }
      WAVE_SYNC();
    }
    HZ_T(3);
    LANE_LOOP {
      const uint32_t g = it + (uint32_t)lane;
      if (g < g1) {
        const uint32_t a0 = g * 16u;
        const uint32_t* ibw = (const uint32_t*)(T.ib + 16u * (uint32_t)lane);
        const uint32_t ww[4] = {ibw[0], ibw[1], ibw[2], ibw[3]};
        for (uint32_t i = 0; i < 4u; i++) {
          const uint32_t hm = (LV(have) >> (4u * i)) & 15u;
          if (hm == 15u) *(hz_gu32*)(dst + (a0 + 4u * i - dmis)) = ww[i];
          else if (hm)
            for (uint32_t k = 0; k < 4u; k++)
              if (hm & (1u << k)) dst[a0 + 4u * i + k - dmis] = (uint8_t)(ww[i] >> (8u * k));
        }
      }
    }
    WAVE_SYNC_GLOBAL();       // this iteration's output final before the next one reads it
    HZ_T(9);
  }
}

// ---- the lane pass over a window's sequences ----------------------------------------
// Repeat offsets (RFC 8878 3.1.1.5) as functions of the previous three offsets R: slot s
// of the result is R[src_s] + v_s (src_s < 3) or the constant v_s (src_s == 3).  The
// offset a sequence uses is slot 0 after its own step, so a window's offsets are an
// inclusive prefix composition of the steps, a log-depth scan across the lanes.
struct RepFn { uint32_t src, v0, v1, v2; };   // src: 2 bits per slot
HZ_HD RepFn rep_id() { return RepFn{0u | 1u << 2 | 2u << 4, 0u, 0u, 0u}; }
HZ_HD RepFn rep_step(uint32_t ofv, uint32_t ll) {
  if (ofv > 3u) return RepFn{3u | 0u << 2 | 1u << 4, ofv - 3u, 0u, 0u};        // new offset pushed
  const uint32_t idx = ofv - 1u + (ll == 0u ? 1u : 0u);
  if (idx == 0u) return rep_id();                                             // R0, history unchanged
  if (idx == 1u) return RepFn{1u | 0u << 2 | 2u << 4, 0u, 0u, 0u};            // R1 to the front
  if (idx == 2u) return RepFn{2u | 0u << 2 | 1u << 4, 0u, 0u, 0u};            // R2 to the front
  return RepFn{0u | 0u << 2 | 1u << 4, 0xffffffffu, 0u, 0u};                  // R0 - 1 pushed
}
// slot s of f's values, by masks (a select chain on the index becomes a scratch array)
HZ_HD uint32_t rep_sel(const RepFn& f, uint32_t s) {
  return (f.v0 & (0u - (uint32_t)(s == 0u))) | (f.v1 & (0u - (uint32_t)(s == 1u))) | (f.v2 & (0u - (uint32_t)(s == 2u)));
}
// f after g
HZ_HD RepFn rep_compose(const RepFn& f, const RepFn& g) {
  const uint32_t f0 = f.src & 3u, f1 = (f.src >> 2) & 3u, f2 = (f.src >> 4) & 3u;
  const uint32_t g0 = f0 == 3u ? 3u : (g.src >> (2u * f0)) & 3u;
  const uint32_t g1 = f1 == 3u ? 3u : (g.src >> (2u * f1)) & 3u;
  const uint32_t g2 = f2 == 3u ? 3u : (g.src >> (2u * f2)) & 3u;
  RepFn h;
  h.src = g0 | (g1 << 2) | (g2 << 4);
  h.v0 = f.v0 + (f0 == 3u ? 0u : rep_sel(g, f0));
  h.v1 = f.v1 + (f1 == 3u ? 0u : rep_sel(g, f1));
  h.v2 = f.v2 + (f2 == 3u ? 0u : rep_sel(g, f2));
  return h;
}
HZ_HD uint32_t rep_apply(const RepFn& f, uint32_t s, uint32_t r0, uint32_t r1, uint32_t r2) {
  const uint32_t fs = (f.src >> (2u * s)) & 3u;
  const uint32_t rv = (r0 & (0u - (uint32_t)(fs == 0u))) | (r1 & (0u - (uint32_t)(fs == 1u))) | (r2 & (0u - (uint32_t)(fs == 2u)));
  return rv + rep_sel(f, s);
}

// aligned dword j of the sequence stream (stream byte x is in dword (x + aoff) >> 2);
// bytes outside the stream read as 0, and j is clamped into the stream's words
HZ_HD uint32_t stream_word(const SBits& b, uint32_t aoff, int32_t j) {
  const int32_t sk = 4 * j - (int32_t)aoff;                // stream byte of the dword's byte 0
  const bool any = sk + 4 > 0 && sk < (int32_t)b.n;
#if HZ_GPU
  const int32_t jc = any ? j : 0;                          // word 0 holds stream byte 0
  uint32_t w = *(hz_gcu32*)(HZ_GLOBAL(hz_gcu8*, b.in.p) + b.lo - aoff + 4 * jc);
  if (sk < 0) w &= ~hz::bmask((uint32_t)(-sk) * 8u);
  if (sk + 4 > (int32_t)b.n) w &= hz::bmask((uint32_t)((int32_t)b.n - sk) * 8u);
  return any ? w : 0u;
#else
  uint32_t w = 0;
  for (int32_t i = 0; i < 4; i++)
    if (sk + i >= 0 && sk + i < (int32_t)b.n) w |= zs::b8(b.in, b.lo + (uint32_t)(sk + i)) << (8 * i);
  (void)any;
  return w;
#endif
}

struct SeqLane { uint32_t ll, ml; RepFn f; };
// one sequence from its walk record {LL entry, OF entry, ML entry, bit position}: the
// extra bits lie below the position (offset on top, then match length, then literal
// length) and are read straight from the input
HZ_HD SeqLane seq_decode(const uint32_t* rec, const SBits& b, uint32_t aoff) {
  const uint32_t eL = rec[0], eO = rec[1], eM = rec[2];
  const uint32_t llc = sq_code(eL), ofc = sq_code(eO), mlc = sq_code(eM);
  const uint32_t llb = sq_eb(eL), mlb = sq_eb(eM), ofb = sq_eb(eO);
  const int32_t q = (int32_t)rec[3] - (int32_t)(llb + mlb + ofb) + 8 * (int32_t)aoff;
  const int32_t j = q >> 5;
  const uint32_t r = (uint32_t)(q - 32 * j);
  const uint32_t w0 = stream_word(b, aoff, j), w1 = stream_word(b, aoff, j + 1), w2 = stream_word(b, aoff, j + 2);
  const uint64_t lo64 = (uint64_t)w0 | ((uint64_t)w1 << 32);
  auto field = [&](uint32_t o, uint32_t w) -> uint32_t {
    const uint64_t v = o >= 64u ? (uint64_t)(w2 >> (o - 64u)) : o ? (lo64 >> o) | ((uint64_t)w2 << (64u - o)) : lo64;
    return (uint32_t)v & hz::bmask(w);
  };
  SeqLane d;
  d.ll = zs::ll_base(llc) + field(r, llb);
  d.ml = zs::ml_base(mlc) + field(r + llb, mlb);
  d.f = rep_step((1u << ofc) + field(r + llb + mlb, ofb), d.ll);
  return d;
}

// the window's n walk records -> {out, lit, src, off}; op, lp and the offset history
// advance past them.  Returns 0 or the status of the first failing sequence (uniform).
#if HZ_GPU
__device__
#else
static
#endif
inline int seq_lanes(Shared& ls, const SBits& b, uint32_t n, uint32_t rsz, uint32_t cap, uint32_t& op, uint32_t& lp,
                     uint32_t& r0, uint32_t& r1, uint32_t& r2) {
  const uint32_t aoff = (uint32_t)(((uintptr_t)b.in.p + b.lo) & 3u);
  for (uint32_t c = 0; c < n; c += 64u) {
#if HZ_GPU
    const int lane = HZ_LANE_ID();
    const uint32_t i = c + (uint32_t)lane;
    const bool valid = i < n;
    SeqLane d;
    if (valid) {
      uint32_t rec[4] = {ls.t.seq[i][0], ls.t.seq[i][1], ls.t.seq[i][2], ls.t.seq[i][3]};
      d = seq_decode(rec, b, aoff);
    } else {
      d.ll = 0; d.ml = 0; d.f = rep_id();
    }
    RepFn F = d.f;
    HZ_UNROLL
    for (int o = 1; o < 64; o <<= 1) {
      RepFn g;
      g.src = __shfl_up(F.src, o, 64); g.v0 = __shfl_up(F.v0, o, 64);
      g.v1 = __shfl_up(F.v1, o, 64); g.v2 = __shfl_up(F.v2, o, 64);
      if (lane >= o) F = rep_compose(F, g);
    }
    const uint32_t off = rep_apply(F, 0u, r0, r1, r2);
    const uint32_t tot = d.ll + d.ml;
    const uint32_t ox = hz::wave_excl_scan(tot, lane), lx = hz::wave_excl_scan(d.ll, lane);
    const uint32_t opi = op + ox, lpi = lp + lx;
    const int code = !valid ? 0
                     : d.ll > rsz - lpi ? zs::E_DATA
                     : (uint64_t)opi + d.ml + (rsz - lpi) > cap ? zs::E_SIZE
                     : off == 0u || (uint64_t)off > (uint64_t)opi + d.ll ? zs::E_DATA : 0;
    const uint64_t bad = (uint64_t)__ballot(code != 0);
    if (bad) return __builtin_amdgcn_readlane(code, (int)__builtin_ctzll(bad));
    if (valid) {
      ls.t.seq[i][SQ_OUT] = opi; ls.t.seq[i][SQ_LIT] = d.ll; ls.t.seq[i][SQ_SRC] = lpi; ls.t.seq[i][SQ_OFF] = off;
    }
    RepFn L;                                    // the whole chunk's composition (lane 63)
    L.src = uni(__builtin_amdgcn_readlane(F.src, 63)); L.v0 = uni(__builtin_amdgcn_readlane(F.v0, 63));
    L.v1 = uni(__builtin_amdgcn_readlane(F.v1, 63)); L.v2 = uni(__builtin_amdgcn_readlane(F.v2, 63));
    const uint32_t n0 = rep_apply(L, 0u, r0, r1, r2), n1 = rep_apply(L, 1u, r0, r1, r2), n2 = rep_apply(L, 2u, r0, r1, r2);
    r0 = uni(n0); r1 = uni(n1); r2 = uni(n2);
    op = uni(op + (uint32_t)__builtin_amdgcn_readlane(ox + tot, 63));
    lp = uni(lp + (uint32_t)__builtin_amdgcn_readlane(lx + d.ll, 63));
#else
    SeqLane d[64];
    RepFn F[64];
    for (int lane = 0; lane < 64; lane++) {
      const uint32_t i = c + (uint32_t)lane;
      if (i < n) d[lane] = seq_decode(ls.t.seq[i], b, aoff);
      else { d[lane].ll = 0; d[lane].ml = 0; d[lane].f = rep_id(); }
      F[lane] = d[lane].f;
    }
    for (int o = 1; o < 64; o <<= 1) {         // the same log-depth scan as the wavefront's
      RepFn g[64];
      for (int lane = 0; lane < 64; lane++) g[lane] = F[lane];
      for (int lane = o; lane < 64; lane++) F[lane] = rep_compose(g[lane], g[lane - o]);
    }
    uint32_t ox = 0, lx = 0;
    for (int lane = 0; lane < 64; lane++) {
      const uint32_t i = c + (uint32_t)lane;
      if (i >= n) break;
      const uint32_t off = rep_apply(F[lane], 0u, r0, r1, r2);
      const uint32_t opi = op + ox, lpi = lp + lx;
      if (d[lane].ll > rsz - lpi) return zs::E_DATA;
      if ((uint64_t)opi + d[lane].ml + (rsz - lpi) > cap) return zs::E_SIZE;
      if (off == 0u || (uint64_t)off > (uint64_t)opi + d[lane].ll) return zs::E_DATA;
      ls.t.seq[i][SQ_OUT] = opi; ls.t.seq[i][SQ_LIT] = d[lane].ll; ls.t.seq[i][SQ_SRC] = lpi; ls.t.seq[i][SQ_OFF] = off;
      ox += d[lane].ll + d[lane].ml; lx += d[lane].ll;
    }
    const RepFn& L = F[63];
    const uint32_t n0 = rep_apply(L, 0u, r0, r1, r2), n1 = rep_apply(L, 1u, r0, r1, r2), n2 = rep_apply(L, 2u, r0, r1, r2);
    r0 = n0; r1 = n1; r2 = n2;
    op += ox; lp += lx;
#endif
  }
  return 0;
}

// repack a freshly built sequence table (sq_pack): every lane converts its own entries
#if HZ_GPU
__device__
#else
static
#endif
inline void sq_convert(zs::Fse* tab, uint32_t al, uint32_t which) {
  WAVE_SYNC();
  LANE_LOOP {
    for (uint32_t u = (uint32_t)lane; u < (1u << al); u += 64u) {
      const uint32_t w = sq_pack(tab[u], which);
#if HZ_GPU
      *(uint32_t*)(tab + u) = w;
#else
      memcpy(tab + u, &w, 4);
#endif
    }
  }
  WAVE_SYNC();
}

// one sequence table of the block header: bytes used or < 0 (uniform)
#if HZ_GPU
__device__
#else
static
#endif
inline int64_t seq_table_w(Shared& ls, zs::Fse* tab, uint32_t& al, uint32_t mode, const zs::In& in, uint32_t at,
                           uint32_t n, uint32_t which, uint32_t maxsym, uint32_t maxal) {
  WTables& t = ls.t;
  if (mode == 0u) {
    WAVE_SYNC();
    LANE_LOOP {
      const uint32_t size = which == 1u ? 32u : 64u;
      if ((uint32_t)lane < size) {
        const uint32_t w = zw_pre[which].e[lane];
#if HZ_GPU
        *(uint32_t*)(tab + lane) = w;
#else
        memcpy(tab + lane, &w, 4);
#endif
      }
    }
    WAVE_SYNC();
    LZ_LANE0_ZW { al = which == 1u ? 5u : 6u; }
    WAVE_SYNC();
    return 0;
  }
  WAVE_SYNC();
  const int64_t u = (int32_t)uni((uint32_t)zs::seq_table(t, tab, al, mode, in, at, n, which, maxsym, maxal));
  if (u < 0) return u;
  if (mode != 3u) sq_convert(tab, uni(al), which);
  return u;
}

// ---- the Huffman literal streams on every lane (round 6) ----------------------------
// A stream's bits are cut into G equal ranges, one per lane (G = 16 per stream for four
// streams, 64 for one).  Lane j decodes from W bits above its range (any bit position:
// Huffman codes resynchronise within a few symbols) down to the first symbol boundary at
// or below its range top (s), then counts the symbols whose boundaries lie in its range
// down to the first boundary below it (e).  Lane 0 starts at the stream's top, so its
// chain is the true one; lane j's is true when its s equals lane j - 1's e, and a lane
// where they differ decodes its range again from there (repair rounds, wave-uniform, at
// most G).  The counts' prefix sums place every lane's symbols, which it decodes a second
// time into the literal area.  The stream must end exactly at its first bit and hold the
// section's count of symbols, as huf_stream checks.
#ifndef ZW_HUF_WARM
#define ZW_HUF_WARM 96                // warm-up bits above a lane's range
#endif
#if HZ_GPU
#define ZW_MEM __device__ __forceinline__
#else
#define ZW_MEM inline
#endif
struct HufRd {                        // a backward reader: four dwords in registers (huf_stream)
  hz_gcu8* base;
  uint32_t a;
  int32_t pos, top;
  uint32_t W0, W1, W2, W3;
  ZW_MEM uint32_t dw(int32_t k) const {
    if (k > 0) return *(hz_gcu32*)(base + 4 * k);
    if (k < 0) return 0u;
    return *(hz_gcu32*)base & ~hz::bmask(8u * a);
  }
  ZW_MEM void init(int32_t p) {
    pos = p;
    top = (p - 1) >> 5;
    W0 = dw(top); W1 = dw(top - 1); W2 = dw(top - 2); W3 = dw(top - 3);
  }
  template <class TT>
  ZW_MEM uint32_t step(const TT& t, uint32_t hb, uint32_t mask) {
    const uint64_t win = ((uint64_t)W0 << 32) | W1;
    const uint32_t rel = (uint32_t)(pos - (int32_t)hb - 32 * (top - 1));
    const zs::Huf e = t.huf[(uint32_t)(win >> rel) & mask];
    pos -= e.nb;
    if (pos <= 32 * top) {
      W0 = W1; W1 = W2; W2 = W3;
      W3 = dw(top - 4);
      top--;
    }
    return e.sym;
  }
};

// lane `lane`'s stream of the section: its bytes [at, at + n), its symbols go to out[0, cnt)
struct HufLane {
  uint32_t at, n, cnt;
  hz_gu8* out;
};

// the streams' symbols; returns 0 or -1 (uniform)
#if HZ_GPU
__device__ inline int huf_streams_wave(const WTables& t, const zs::In& in, const HufLane& L, uint32_t G) {
  const uint32_t lane = threadIdx.x, j = lane % G;
  int bad = (L.n == 0u || L.at + L.n > in.n) ? 1 : 0;
  const uint32_t last = bad ? 1u : zs::b8(in, L.at + L.n - 1u);
  bad |= last == 0u ? 1 : 0;
  HufRd r;
  r.a = (uint32_t)(((uintptr_t)in.p + L.at) & 3u);
  r.base = HZ_GLOBAL(hz_gcu8*, in.p + L.at - r.a);
  const int32_t start = 8 * (int32_t)r.a;
  const int32_t ptop = bad ? start : 8 * (int32_t)(L.n - 1u) + (int32_t)zs::hib(last) + start;
  const int64_t span = ptop - start;
  const int32_t pj = start + (int32_t)(span - span * (int64_t)j / (int64_t)G);
  const int32_t pj1 = start + (int32_t)(span - span * (int64_t)(j + 1u) / (int64_t)G);
  const uint32_t hb = t.huf_bits, mask = (1u << hb) - 1u;
  // pass 1: warm-up, then the range's symbols counted
  const int32_t b0 = j == 0u ? ptop : (pj + ZW_HUF_WARM < ptop ? pj + ZW_HUF_WARM : ptop);
  r.init(b0);
  while (r.pos > pj) (void)r.step(t, hb, mask);
  int32_t s = r.pos, e;
  uint32_t n = 0;
  while (r.pos > pj1) { (void)r.step(t, hb, mask); n++; }
  e = r.pos;
  // repair rounds: a lane whose first boundary is not its predecessor's end decodes again
  for (uint32_t round = 0; round < G; round++) {
    const int32_t ep = __shfl_up(e, 1, 64);
    const bool fix = j > 0u && ep != s;
    if (!__ballot(fix)) break;
    if (fix) {
      s = ep;
      r.init(ep);
      n = 0;
      while (r.pos > pj1) { (void)r.step(t, hb, mask); n++; }
      e = r.pos;
    }
  }
  // placement: prefix sums of the counts inside each group of G lanes
  uint32_t inc = n;
  for (uint32_t o = 1; o < G; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (j >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, (int)(lane - j + G - 1u), 64);
  bad |= (total != L.cnt || (j == G - 1u && e != start)) ? 1 : 0;
  if (__ballot(bad != 0)) return -1;
  // pass 2: the lane's symbols into place
  r.init(s);
  hz_gu8* const o = L.out + (inc - n);
  for (uint32_t k = 0; k < n; k++) o[k] = (uint8_t)r.step(t, hb, mask);
  return 0;
}
#else
static inline int huf_streams_wave(const WTables& t, const zs::In& in, const HufLane* L, uint32_t G) {
  int32_t S[64], E[64], PJ[64], PJ1[64], START[64];
  uint32_t N[64];
  HufRd R[64];
  int bad = 0;
  const uint32_t hb = t.huf_bits, mask = (1u << hb) - 1u;
  for (uint32_t lane = 0; lane < 64; lane++) {
    const uint32_t j = lane % G;
    int lb = (L[lane].n == 0u || L[lane].at + L[lane].n > in.n) ? 1 : 0;
    const uint32_t last = lb ? 1u : zs::b8(in, L[lane].at + L[lane].n - 1u);
    lb |= last == 0u ? 1 : 0;
    bad |= lb;
    HufRd& r = R[lane];
    r.a = (uint32_t)(((uintptr_t)in.p + L[lane].at) & 3u);
    r.base = in.p + L[lane].at - r.a;
    const int32_t start = 8 * (int32_t)r.a;
    const int32_t ptop = lb ? start : 8 * (int32_t)(L[lane].n - 1u) + (int32_t)zs::hib(last) + start;
    const int64_t span = ptop - start;
    PJ[lane] = start + (int32_t)(span - span * (int64_t)j / (int64_t)G);
    PJ1[lane] = start + (int32_t)(span - span * (int64_t)(j + 1u) / (int64_t)G);
    START[lane] = start;
    const int32_t b0 = j == 0u ? ptop : (PJ[lane] + ZW_HUF_WARM < ptop ? PJ[lane] + ZW_HUF_WARM : ptop);
    r.init(b0);
    while (r.pos > PJ[lane]) (void)r.step(t, hb, mask);
    S[lane] = r.pos;
    N[lane] = 0;
    while (r.pos > PJ1[lane]) { (void)r.step(t, hb, mask); N[lane]++; }
    E[lane] = r.pos;
  }
  for (uint32_t round = 0; round < G; round++) {
    int32_t EP[64];
    bool any = false, fix[64];
    for (uint32_t lane = 0; lane < 64; lane++) EP[lane] = lane ? E[lane - 1] : E[0];
    for (uint32_t lane = 0; lane < 64; lane++) { fix[lane] = lane % G > 0u && EP[lane] != S[lane]; any |= fix[lane]; }
    if (!any) break;
    for (uint32_t lane = 0; lane < 64; lane++) {
      if (!fix[lane]) continue;
      HufRd& r = R[lane];
      S[lane] = EP[lane];
      r.init(EP[lane]);
      N[lane] = 0;
      while (r.pos > PJ1[lane]) { (void)r.step(t, hb, mask); N[lane]++; }
      E[lane] = r.pos;
    }
  }
  uint32_t X[64];
  for (uint32_t g0 = 0; g0 < 64; g0 += G) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < G; k++) { X[g0 + k] = acc; acc += N[g0 + k]; }
    bad |= (acc != L[g0].cnt || E[g0 + G - 1u] != START[g0 + G - 1u]) ? 1 : 0;
  }
  if (bad) return -1;
  for (uint32_t lane = 0; lane < 64; lane++) {
    HufRd& r = R[lane];
    r.init(S[lane]);
    for (uint32_t k = 0; k < N[lane]; k++) L[lane].out[X[lane] + k] = (uint8_t)r.step(t, hb, mask);
  }
  return 0;
}
#endif

// one compressed block at input [at, at + n); output from op; returns the new op or < 0 (uniform)
#if HZ_GPU
__device__
#else
static
#endif
inline int64_t block(Shared& ls, const zs::In& in, uint32_t at, uint32_t n, hz_gu8* dst, uint32_t dmis, uint32_t op,
                     uint32_t cap, HzProf* prof) {
  (void)prof;
  WTables& t = ls.t;
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
    } else {
      // treeless: the previous table, rebuilt from its weights (the sequences section
      // reused its LDS)
      if (!uni(t.have_huf)) return zs::E_DATA;
      WAVE_SYNC();
      zs::huf_fill(t, uni(t.huf_nw), uni(t.huf_bits));
      WAVE_SYNC();
    }
    const uint32_t s0 = at + q + (uint32_t)tsz, ssz = csz - (uint32_t)tsz;
    HZ_T(1);
#if ZW_HUF_PAR
    {
      // every lane on a stream: 64 on a single stream, 16 on each of four
      uint32_t l1 = ssz, l2 = 0, l3 = 0, l4 = 0, seg = rsz, p1 = s0;
      if (ns != 1) {
        if (ssz < 6) return zs::E_DATA;
        l1 = ub8(in, s0) | (ub8(in, s0 + 1) << 8); l2 = ub8(in, s0 + 2) | (ub8(in, s0 + 3) << 8);
        l3 = ub8(in, s0 + 4) | (ub8(in, s0 + 5) << 8);
        if (l1 + l2 + l3 + 6 > ssz) return zs::E_DATA;
        l4 = ssz - 6 - l1 - l2 - l3;
        seg = (rsz + 3) / 4;
        if (rsz < 3 * seg) return zs::E_DATA;
        p1 = s0 + 6;
      }
      const uint32_t G = ns == 1 ? 64u : 16u;
      WAVE_SYNC();
#if HZ_GPU
      HufLane hl;
      {
        const uint32_t st = threadIdx.x / G;
        const uint32_t off = st == 0 ? 0u : st == 1 ? l1 : st == 2 ? l1 + l2 : l1 + l2 + l3;
        hl.at = p1 + off;
        hl.n = ns == 1 ? ssz : st == 0 ? l1 : st == 1 ? l2 : st == 2 ? l3 : l4;
        hl.cnt = ns == 1 ? rsz : st == 3 ? rsz - 3 * seg : seg;
        hl.out = lit + st * seg;
      }
      const int herr = huf_streams_wave(t, in, hl, G);
#else
      HufLane hl[64];
      for (uint32_t lane = 0; lane < 64; lane++) {
        const uint32_t st = lane / G;
        const uint32_t off = st == 0 ? 0u : st == 1 ? l1 : st == 2 ? l1 + l2 : l1 + l2 + l3;
        hl[lane].at = p1 + off;
        hl[lane].n = ns == 1 ? ssz : st == 0 ? l1 : st == 1 ? l2 : st == 2 ? l3 : l4;
        hl[lane].cnt = ns == 1 ? rsz : st == 3 ? rsz - 3 * seg : seg;
        hl[lane].out = lit + st * seg;
      }
      const int herr = huf_streams_wave(t, in, hl, G);
#endif
      WAVE_SYNC();
      if (herr) return zs::E_DATA;
    }
#else
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
#endif
    q += csz;
  }
  WAVE_SYNC_GLOBAL();         // literals visible to every lane
  q = uni(q);
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
    // per table: mode 0 copies the compile-time predefined table; modes 1 (RLE) and 2
    // (FSE description) build it and repack it; mode 3 (repeat) keeps the packed table
    const int64_t ul = seq_table_w(ls, t.ll, t.ll_al, (modes >> 6) & 3u, in, at + q, n - q, 0u, 35u, 9u);
    if (ul < 0) return zs::E_DATA;
    q += (uint32_t)ul;
    const int64_t uo = seq_table_w(ls, t.of, t.of_al, (modes >> 4) & 3u, in, at + q, n - q, 1u, 31u, 8u);
    if (uo < 0) return zs::E_DATA;
    q += (uint32_t)uo;
    const int64_t um = seq_table_w(ls, t.ml, t.ml_al, (modes >> 2) & 3u, in, at + q, n - q, 2u, 52u, 9u);
    if (um < 0) return zs::E_DATA;
    q += (uint32_t)um;
    q = uni(q);
    t.have_seq = 1;
    WAVE_SYNC();
    if (n - q == 0 || ub8(in, at + n - 1) == 0) return zs::E_DATA;
    b.in = in; b.lo = at + q; b.n = n - q; b.sb = SB_NONE; b.wbit = -1; b.win = 0;
    b.pos = 8 * (int32_t)(b.n - 1) + (int32_t)zs::hib(ub8(in, at + n - 1));
    const uint32_t lal = uni(t.ll_al), oal = uni(t.of_al), mal = uni(t.ml_al);
    const uint32_t v = sb_read(ls, b, lal + oal + mal);      // LL, OF, ML initial states
    sll = v >> (oal + mal); sof = (v >> mal) & ((1u << oal) - 1u); sml = v & ((1u << mal) - 1u);
  }
  uint32_t k = 0;
  for (;;) {
    HZ_T(2);
    op = uni(op); lp = uni(lp); k = uni(k);
    rep0 = uni(rep0); rep1 = uni(rep1); rep2 = uni(rep2);
    const uint32_t wb = op;
    uint32_t ns_w = 0;
    // ---- (1) the serial FSE walk, in vector registers (lane-uniform values: LDS results
    // feed the next addresses with no scalar moves): per sequence one LDS dword from each
    // table, then the two stage dwords holding the state bits.  It records the three
    // entries and the bit position of the sequence's extra bits, skips those bits and
    // takes the next states ----
    {
      const uint32_t kend = uni(nseq - k < (uint32_t)NSEQ - 1u ? nseq : k + (uint32_t)NSEQ - 1u);
      uint32_t vl = vdiv(sll), vo = vdiv(sof), vm = vdiv(sml);
      int32_t vpos = (int32_t)vdiv((uint32_t)b.pos);
      while (k < kend) {
        int32_t sb = b.sb;
        if ((int32_t)uni((uint32_t)vpos) - 8 * sb < 128 && sb > 0) {   // the state bits may leave the stage
          b.pos = (int32_t)uni((uint32_t)vpos);
          const int32_t f = ((b.pos + 7) >> 3) - STG;
          sb_stage(ls, b, f < 0 ? 0 : f);
          sb = b.sb;
        }
#if ZW_WALK4
        // the four stage dwords below the position are read with the table entries (they
        // depend on the position only): the sequence's extra and state bits (<= 89) lie in
        // them, so one LDS round trip per sequence instead of two dependent ones
        const int32_t xs = vpos - 8 * sb;                            // stage bit (exclusive top)
        const int32_t jt = (xs - 1) >> 5, j0 = jt - 3 < 0 ? 0 : jt - 3;
        const uint32_t w0 = ls.t.stage[j0], w1 = ls.t.stage[j0 + 1], w2 = ls.t.stage[j0 + 2], w3 = ls.t.stage[j0 + 3];
#endif
        const uint32_t eL = fse_word(t.ll, vl), eO = fse_word(t.of, vo), eM = fse_word(t.ml, vm);
        const uint32_t xb = sq_eb(eL) + sq_eb(eO) + sq_eb(eM);
        const uint32_t nL = sq_nb(eL), nM = sq_nb(eM), nO = sq_nb(eO);
        const uint32_t nsb = k + 1u < nseq ? nL + nM + nO : 0u;   // state updates: LL, ML, OF
        int32_t lo = vpos - 8 * sb - (int32_t)(xb + nsb);           // stage bit of the state bits
        lo = lo < 0 ? 0 : lo;                                        // (< 0 only past the stream start)
#if ZW_WALK4
        const uint32_t d = (uint32_t)((lo >> 5) - j0);              // 0..3 (3: the bits lie in w3)
        const uint32_t lw = d == 0u ? w0 : d == 1u ? w1 : d == 2u ? w2 : w3;
        const uint32_t hw = d == 0u ? w1 : d == 1u ? w2 : d == 2u ? w3 : 0u;
        const uint32_t fld = ubfe(funnel(hw, lw, (uint32_t)lo & 31u), 0u, nsb);
#else
        const uint32_t j = (uint32_t)lo >> 5;
        const uint32_t fld = ubfe(funnel(ls.t.stage[j + 1u], ls.t.stage[j], (uint32_t)lo & 31u), 0u, nsb);
#endif
        ls.t.seq[ns_w][0] = eL; ls.t.seq[ns_w][1] = eO; ls.t.seq[ns_w][2] = eM; ls.t.seq[ns_w][3] = (uint32_t)vpos;
        vl = sq_base(eL) + (fld >> (nM + nO));
        vm = sq_base(eM) + ubfe(fld, nO, nM);
        vo = sq_base(eO) + ubfe(fld, 0u, nO);
        vpos -= (int32_t)(xb + nsb);
        ns_w++;
        k++;
      }
      sll = uni(vl); sof = uni(vo); sml = uni(vm);
      b.pos = (int32_t)uni((uint32_t)vpos);
      ns_w = uni(ns_w); k = uni(k);
    }
    HZ_T(8);
    WAVE_SYNC();
    // ---- (2) the lanes: extra bits, lengths, repeat offsets and positions of the window's
    // sequences, 64 at a time (the offset history is a prefix composition) ----
    {
      const int st = seq_lanes(ls, b, ns_w, rsz, cap, op, lp, rep0, rep1, rep2);
      if (st) return st;
    }
    HZ_T(2);
    const int last = k >= nseq;
    if (last) {
      if (nseq > 0 && b.pos != 0) return zs::E_DATA;
      WAVE_SYNC();
      LZ_LANE0_ZW { t.rep[0] = rep0; t.rep[1] = rep1; t.rep[2] = rep2; }
      const uint32_t rest = rsz - lp;
      if ((uint64_t)op + rest > cap) return zs::E_SIZE;
      if (rest) {
        LZ_LANE0_ZW { ls.t.seq[ns_w][SQ_OUT] = op; ls.t.seq[ns_w][SQ_LIT] = rest; ls.t.seq[ns_w][SQ_SRC] = lp; ls.t.seq[ns_w][SQ_OFF] = 0; }
        ns_w++;
        op += rest; lp += rest;
      }
    }
    WAVE_SYNC();
    HZ_T(9);
    if (ns_w) resolve(ls, dst, dmis, lbase, wb, op, ns_w, prof);
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
  WTables& t = ls.t;
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
    // the frame walk is uniform: re-assert it at each block (a lane loop's exit value can
    // otherwise make the compiler treat the loop-carried state as divergent)
    q = uni(q); op = uni(op);
#if HZ_GPU && ZW_PRIO_KB
    {
      // wave priority by the split's remaining input (inflate2.h HZ2_PRIO_ABS): the waves with
      // the most work left get the SIMD's issue slots (A/B round 5, bench zstd leg: off 52.4,
      // 16 KiB 51.8, 32 KiB 54.0, 64 KiB 53.8 GB/s)
      const uint32_t lv = (n > q ? (n - q) >> 10 : 0u) / (uint32_t)ZW_PRIO_KB;
      if (lv >= 3u) __builtin_amdgcn_s_setprio(3);
      else if (lv == 2u) __builtin_amdgcn_s_setprio(2);
      else if (lv == 1u) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
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
