// lz_wave.h -- decoder for the byte-aligned LZ77 codecs a Blosc1 frame can carry
// besides zlib:
//   * codec 1, "lz4" / "lz4hc": LZ4 block format (lz4 1.9.x LZ4_decompress_safe, which
//     c-blosc 1.21 calls from lz4_wrap_decompress for every split);
//   * codec 0, "blosclz": c-blosc 1.21's BloscLZ (blosclz_decompress).
// The reference reaches both through storUtil._uncompress -> numcodecs Blosc.decode
// (hsds/util/storUtil.py:195-208) and writes them through storUtil._compress with
// cname = the dataset's compressor (storUtil.py:255-262, dsetUtil.py:38-44).
//
// Algorithm (DESIGN.md "LZ4 / BloscLZ"):
//   One wavefront decodes GROUP (8) splits at once, in rounds.
//   * Parse: lane i < GROUP walks the sequence headers of ITS split (literal length,
//     literal source, match distance, match length) for up to GK sequences, reading the
//     input through an 8-byte register window.  This serial, latency-bound walk runs on
//     GROUP splits in parallel instead of one lane walking one split.
//   * Resolve: the round's output of the GROUP splits is cut into 16-byte destination
//     groups that the 64 lanes share.  Every output byte is a pure function of its
//     split's sequence table: a literal byte is read from the input; a match byte at
//     offset k into a match of distance d starting at m is the byte at
//     m - d + (k mod d) (the periodic extension of an overlapping copy), which lies in
//     an earlier sequence of the round or before it (already stored).  Bytes are
//     stored as aligned dwords.
//
// Single source, like inflate_wave.h: tests/emu/lz_emu.cpp runs the same code on CPU.
#pragma once
#include "inflate_wave.h"

#ifndef LZ_PRIO_KB
#define LZ_PRIO_KB 16                 // wave priority: one level per 16 KiB of the group's largest input left (0: off)
#endif
namespace lz {

#ifndef LZ_GK
#define LZ_GK 32
#endif
constexpr int GK = LZ_GK;                           // sequences per split per round
#ifndef LZ_GROUP
#define LZ_GROUP 8
#endif
// splits per wavefront: lanes [0, GROUP) walk headers, all 64 lanes resolve.  A batch
// has only ~8 splits per 1 MiB chunk, so a small group keeps enough wavefronts per CU
// to hide the resolve's LDS and memory latency (MI355X A/B, 4096 x 1 MiB lz4 chunks:
// GROUP 64 / 16 / 8 / 4 -> 23 / 62 / 79 / 67 GB/s; GK 16 / 32 / 64 -> 77 / 79 / 79).
constexpr int GROUP = LZ_GROUP;
constexpr uint32_t FMT_BLOSCLZ = 0, FMT_LZ4 = 1;    // Blosc1 codec numbers (flags >> 5)
#ifndef LZ_SW
#define LZ_SW 128
#endif
constexpr uint32_t SW = LZ_SW;                      // staged input dwords per split per round

// one split per lane
struct LaneJob {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t src_len, dst_len;
  uint32_t fmt, valid;
};

// KR: sequences per split per round (lz_kernel GK; the bitshuffle decoder's 8 KiB blocks
// take fewer)
template <int KR>
struct SharedT {
  static constexpr int K = KR;
  uint32_t t_out[KR][GROUP];   // [k][split]: output offset of the split's k-th sequence this round
  uint32_t t_lit[KR][GROUP];   // literal bytes
  uint32_t t_src[KR][GROUP];   // input offset of the literals
  uint32_t t_off[KR][GROUP];   // match distance (0: literals only)
  LaneJob job[GROUP];
  uint32_t m_lo[GROUP], m_hi[GROUP], m_nk[GROUP];   // round output [lo, hi) and sequence count
  int32_t m_st[GROUP];                               // per-split status
  uint32_t gpre[GROUP + 1];                          // exclusive prefix of 16-byte groups per split
  alignas(16) uint8_t ib[1024];                      // resolve: the iteration's output bytes
  uint16_t pm[64];                                   // resolve: each lane's bytes still pending
};
using Shared = SharedT<GK>;

// the parse's LDS stage (lz_kernel; the bitshuffle decoder's small blocks run without:
// its 4 KB would cost that kernel a wave per SIMD)
struct Stage {
  uint32_t stg[GROUP][SW];                           // staged input of each split
  uint32_t sbeg[GROUP];                              // its base offset (~0: none)
};

// per-lane input window: 8 bytes at a dword-aligned position of the split
// Each round the wave stages SW dwords of every split's input from its parse position
// into LDS (all 64 lanes, one memory latency); the header walk refills its window from
// there (an LDS latency) and from global memory only past the staged bytes.
struct ByteRd {
  hz_gcu8* base;      // split start rounded down to 4 bytes
  uint32_t lo, hi;    // valid byte range in base coordinates
  uint32_t bpos;      // base offset of buf
  uint64_t buf;
  const uint32_t* stg;  // this split's stage (LDS): dwords at base offsets sb + 4k, k < SW
  uint32_t sb;
};

HZ_HD uint32_t rd_byte(ByteRd& r, uint32_t pos) {
  const uint32_t ap = pos + r.lo;
  if (ap - r.bpos >= 8u) {
    r.bpos = ap & ~3u;
    const uint32_t rel = r.bpos - r.sb;
    if (rel + 8u <= 4u * SW) {
      r.buf = (uint64_t)r.stg[rel >> 2] | ((uint64_t)r.stg[(rel >> 2) + 1u] << 32);
    } else {
      r.buf = (uint64_t)hz::load_word(r.base, r.bpos >> 2, r.lo, r.hi) |
              ((uint64_t)hz::load_word(r.base, (r.bpos >> 2) + 1u, r.lo, r.hi) << 32);
    }
  }
  return (uint32_t)(r.buf >> (8u * (ap - r.bpos))) & 0xffu;
}

struct PState { uint32_t ip, op, done; };

#define LZ_NEED(pos) if ((pos) >= iend) return hz::ST_TRUNC;

// One LZ4 sequence (LZ4_decompress_safe rules; oracle.c orc_lz4_decode).  1: parsed
// (ps.done set after the last one), < 0: status.
HZ_HD int parse_lz4(ByteRd& r, PState& ps, uint32_t iend, uint32_t oend, uint32_t& lit, uint32_t& lsrc,
                    uint32_t& off, uint32_t& ml) {
  uint32_t x = ps.ip;
  LZ_NEED(x);
  const uint32_t t = rd_byte(r, x); x++;
  lit = t >> 4;
  if (lit == 15) {
    uint32_t b;
    do { LZ_NEED(x); b = rd_byte(r, x); x++; lit += b; } while (b == 255 && lit < 0x7fffffffu);
  }
  lsrc = x;
  if (lit > iend - x) return hz::ST_TRUNC;
  if (lit > oend - ps.op) return hz::ST_SIZE;
  x += lit;
  // a literal run reaching oend - MFLIMIT (12) or iend - 8 is the last sequence and
  // must end exactly at iend
  if (ps.op + lit + 12u > oend || x + 8u > iend) {
    if (x != iend) return hz::ST_DATA;
    off = 0; ml = 0; ps.ip = x; ps.done = 1;
    return 1;
  }
  off = rd_byte(r, x);
  off |= rd_byte(r, x + 1u) << 8;
  x += 2;
  ml = t & 15u;
  if (ml == 15) {
    uint32_t b;
    do { LZ_NEED(x); b = rd_byte(r, x); x++; ml += b; } while (b == 255 && ml < 0x7fffffffu);
  }
  ml += 4;
  const uint32_t oe = ps.op + lit;
  if (off == 0 || off > oe) return hz::ST_DATA;
  if (ml > oend - oe || oe + ml + 5u > oend) return hz::ST_DATA;   // LASTLITERALS
  ps.ip = x;
  return 1;
}

// One BloscLZ item (c-blosc 1.21 blosclz_decompress; oracle.c orc_blosclz_decode)
HZ_HD int parse_blosclz(ByteRd& r, PState& ps, uint32_t iend, uint32_t oend, uint32_t& lit, uint32_t& lsrc,
                        uint32_t& off, uint32_t& ml) {
  uint32_t x = ps.ip;
  LZ_NEED(x);
  uint32_t c = rd_byte(r, x); x++;
  if (ps.ip == 0) c &= 31u;
  lit = 0; lsrc = 0; off = 0; ml = 0;
  if (c >= 32) {
    ml = (c >> 5) - 1u;
    const uint32_t ofs = (c & 31u) << 8;
    uint32_t code;
    if (ml == 6) {
      do { LZ_NEED(x); code = rd_byte(r, x); x++; ml += code; } while (code == 255 && ml < 0x7fffffffu);
    }
    LZ_NEED(x);
    code = rd_byte(r, x); x++;
    ml += 3;
    off = ofs + code + 1u;
    if (code == 255 && ofs == (31u << 8)) {
      LZ_NEED(x + 1u);
      off = ((rd_byte(r, x) << 8) | rd_byte(r, x + 1u)) + 8192u;
      x += 2;
    }
    if (ml > oend - ps.op) return hz::ST_SIZE;
    if (off > ps.op) return hz::ST_DATA;
  } else {
    lit = c + 1u;
    lsrc = x;
    if (lit > oend - ps.op) return hz::ST_SIZE;
    if (lit > iend - x) return hz::ST_TRUNC;
    x += lit;
  }
  ps.ip = x;
  if (x >= iend) ps.done = 1;
  return 1;
}
#undef LZ_NEED

// largest k <= hi with t_out[k][s] <= p (non-decreasing in k, t_out[0][s] <= p)
template <class SH>
HZ_HD uint32_t find_seq(const SH& ls, uint32_t s, uint32_t hi, uint32_t p) {
  uint32_t lo = 0;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (ls.t_out[mid][s] <= p) lo = mid; else hi = mid - 1u;
  }
  return lo;
}

// largest s < GROUP with gpre[s] <= g
template <class SH>
HZ_HD uint32_t find_split(const SH& ls, uint32_t g) {
  uint32_t lo = 0, hi = GROUP - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (ls.gpre[mid] <= g) lo = mid; else hi = mid - 1u;
  }
  return lo;
}

// Decode the splits in ls.job[0..GROUP) (valid ones); statuses land in ls.m_st.
// Forced inline: lz_kernel and bshuf_kernel both call it, and an outlined call costs
// lz_kernel 92 -> 165 VGPRs (5 -> 3 waves/SIMD) and a scratch spill.
template <bool STAGE, class SH>
#if HZ_GPU
__device__ __attribute__((always_inline))
#else
static
#endif
inline void lz_group(SH& ls, Stage* stage, HzProf* prof = nullptr) {
  (void)prof;
  LANE_VAR(PState, ps);
  LANE_VAR(ByteRd, rd);
  LANE_VAR(int, active);
  LANE_VAR(uint32_t, gc);
  LANE_LOOP {
    LV(active) = 0;
    LV(gc) = 0;
    if (lane >= GROUP) continue;
    const LaneJob j = ls.job[lane];
    const uint32_t a = (uint32_t)(((uintptr_t)j.src) & 3u);
    LV(ps).ip = 0; LV(ps).op = 0; LV(ps).done = 0;
    LV(rd).base = HZ_GLOBAL(hz_gcu8*, j.src - a);
    LV(rd).lo = a; LV(rd).hi = a + j.src_len;
    LV(rd).bpos = 0x80000000u; LV(rd).buf = 0;
    LV(rd).stg = STAGE ? stage->stg[lane] : nullptr; LV(rd).sb = 0x80000000u;
    LV(active) = j.valid != 0;
    ls.m_st[lane] = hz::ST_OK;
    if (j.valid && j.src_len == 0) { ls.m_st[lane] = hz::ST_TRUNC; LV(active) = 0; }
  }
  WAVE_SYNC();
  for (;;) {
    if (!WAVE_BALLOT(LV(active))) break;
#if HZ_GPU && LZ_PRIO_KB
    if constexpr (STAGE) {          // (lz_kernel; the bitshuffle decoder sets its own per chunk)
      // wave priority by the group's largest remaining input (inflate2.h HZ2_PRIO_ABS): the
      // waves with the most work left get the SIMD's issue slots (A/B round 5, bench lz4 leg:
      // off 148.1, 16 KiB 158.7, 32 KiB 156.5 GB/s)
      uint32_t rem = 0;
HZ_UNROLL
      for (int l = 0; l < GROUP; l++) {
        const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)(LV(active) ? LV(rd).hi - (LV(ps).ip + LV(rd).lo) : 0u), l);
        rem = r > rem ? r : rem;
      }
      const uint32_t lv = (rem >> 10) / (uint32_t)LZ_PRIO_KB;
      if (lv >= 3u) __builtin_amdgcn_s_setprio(3);
      else if (lv == 2u) __builtin_amdgcn_s_setprio(2);
      else if (lv == 1u) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    HZ_T(1);
    // ---- stage: SW dwords of every active split's input from its parse position ----
    if constexpr (STAGE) {
    LANE_LOOP {
      if (lane < GROUP) stage->sbeg[lane] = LV(active) ? ((LV(ps).ip + LV(rd).lo) & ~3u) : ~0u;
    }
    WAVE_SYNC();
    LANE_LOOP {
      constexpr uint32_t LPS = 64u / GROUP;          // lanes per split
      static_assert(64 % GROUP == 0 && SW % (64u / GROUP) == 0, "stage: whole dwords per lane");
      const uint32_t s = (uint32_t)lane / LPS, part = (uint32_t)lane % LPS, b0 = stage->sbeg[s];
      if (b0 != ~0u) {
        const LaneJob j = ls.job[s];
        const uint32_t a = (uint32_t)(((uintptr_t)j.src) & 3u), hi = a + j.src_len;
        hz_gcu8* base = HZ_GLOBAL(hz_gcu8*, j.src - a);
        uint32_t v[SW / LPS];
        HZ_UNROLL
        for (uint32_t i = 0; i < SW / LPS; i++) {      // every load issued before any is used
          const uint32_t o = b0 + 4u * (part + LPS * i);
#if HZ_GPU
          v[i] = *(hz_gcu32*)(base + (o < hi ? o : b0));
#else
          v[i] = hz::load_word(base, o >> 2, a, hi);
#endif
        }
        HZ_UNROLL
        for (uint32_t i = 0; i < SW / LPS; i++)
          stage->stg[s][part + LPS * i] = b0 + 4u * (part + LPS * i) < hi ? v[i] : 0u;
      }
    }
    WAVE_SYNC();
    }
    // ---- parse: every lane walks up to GK sequence headers of its own split ----
    LANE_LOOP {
      if (STAGE && lane < GROUP) LV(rd).sb = stage->sbeg[lane];
      if (lane >= GROUP) continue;
      const LaneJob j = ls.job[lane];
      const uint32_t op0 = LV(ps).op;
      uint32_t k = 0;
      if (LV(active)) {
        for (; k < (uint32_t)SH::K && !LV(ps).done; k++) {
          uint32_t lit, lsrc, off, ml;
          const int r = j.fmt == FMT_LZ4 ? parse_lz4(LV(rd), LV(ps), j.src_len, j.dst_len, lit, lsrc, off, ml)
                                         : parse_blosclz(LV(rd), LV(ps), j.src_len, j.dst_len, lit, lsrc, off, ml);
          if (r < 0) { ls.m_st[lane] = r; LV(active) = 0; break; }
          ls.t_out[k][lane] = LV(ps).op;
          ls.t_lit[k][lane] = lit;
          ls.t_src[k][lane] = lsrc;
          ls.t_off[k][lane] = off;
          LV(ps).op += lit + ml;
        }
      }
      const uint32_t hi = LV(active) ? LV(ps).op : op0;
      ls.m_lo[lane] = op0;
      ls.m_hi[lane] = hi;
      ls.m_nk[lane] = LV(active) ? k : 0u;
      const uint32_t dmis = (uint32_t)(((uintptr_t)j.dst) & 3u);
      LV(gc) = hi > op0 ? ((hi + dmis + 15u) >> 4) - ((op0 + dmis) >> 4) : 0u;
    }
    HZ_T(2);
    // ---- groups of all splits, exclusive prefix ----
    {
      LANE_VAR(uint32_t, gx);
#if HZ_GPU
      gx = hz::wave_excl_scan(gc, (int)threadIdx.x);
#else
      { uint32_t acc = 0; for (int lane = 0; lane < 64; lane++) { gx[lane] = acc; acc += gc[lane]; } }
#endif
      LANE_LOOP {
        if (lane < GROUP) ls.gpre[lane] = LV(gx);
        if (lane == GROUP - 1) ls.gpre[GROUP] = LV(gx) + LV(gc);
      }
    }
    WAVE_SYNC();
    const uint32_t total = ls.gpre[GROUP];
    // ---- resolve: 16-byte destination groups shared by all lanes, 64 per iteration ----
    // (1) each byte's source: a literal of the input, a byte stored before this iteration
    //     (an earlier round or iteration: final), or a byte of this iteration (pending);
    //     the first two are loaded, together, into the LDS byte buffer;
    // (2) rounds: a pending byte copies its source once that is no longer pending (the
    //     lowest pending byte's source always precedes it, so every round makes progress);
    // (3) the buffer is stored, and the iteration's bytes are final for the next one.
    struct Src { uint32_t v[16]; };          // bit 31: from the input, else from dst / the buffer
    for (uint32_t it = 0; it < total; it += 64u) {
      LANE_VAR(uint32_t, have);
      LANE_VAR(uint32_t, pend);
      LANE_VAR(uint32_t, gsplit);
      LANE_VAR(Src, so);
      LANE_LOOP {
        const uint32_t g = it + (uint32_t)lane;
        uint32_t hv = 0, pv = 0, ww[4] = {0u, 0u, 0u, 0u}, s = 0;
        Src& S = LV(so);
        if (g < total) {
          s = find_split(ls, g);
          const LaneJob j = ls.job[s];
          hz_gcu8* src = HZ_GLOBAL(hz_gcu8*, j.src);
          hz_gcu8* dst = HZ_GLOBAL(hz_gcu8*, j.dst);
          const uint32_t dmis = (uint32_t)(((uintptr_t)j.dst) & 3u);
          const uint32_t wb = ls.m_lo[s], we = ls.m_hi[s], nk = ls.m_nk[s], gp = ls.gpre[s];
          const uint32_t gw = (wb + dmis) >> 4;                        // the round's first group of the split
          const uint32_t a0 = (gw + (g - gp)) * 16u;                   // dst - dmis offset of the group
          const uint32_t pb = a0 > wb + dmis ? a0 - dmis : wb;         // first window byte in it
          // the split's first byte in this iteration: sources below it are final
          const uint32_t it_lo = gp >= it ? wb : (gw + (it - gp)) * 16u - dmis;
          uint32_t t = find_seq(ls, s, nk - 1u, pb);
          uint32_t r_out = ls.t_out[t][s], r_lit = ls.t_lit[t][s], r_src = ls.t_src[t][s], r_off = ls.t_off[t][s];
          uint32_t t_end = t + 1u < nk ? ls.t_out[t + 1u][s] : we;
          uint32_t mq = ~0u;            // the previous byte's match source (same sequence), else ~0
          HZ_UNROLL
          for (uint32_t k = 0; k < 16u; k++) {
            const uint32_t ak = a0 + k;
            S.v[k] = 0;
            if (ak < wb + dmis || ak >= we + dmis) continue;
            const uint32_t p = ak - dmis;
            if (p >= t_end) {
              do { t++; t_end = t + 1u < nk ? ls.t_out[t + 1u][s] : we; } while (p >= t_end);
              r_out = ls.t_out[t][s]; r_lit = ls.t_lit[t][s]; r_src = ls.t_src[t][s]; r_off = ls.t_off[t][s];
              mq = ~0u;
            }
            hv |= 1u << k;
            const uint32_t rel = p - r_out;
            if (rel < r_lit) {
              S.v[k] = 0x80000000u | (r_src + rel);
              mq = ~0u;
            } else {
              // the periodic extension m - d + (k mod d), stepped from the previous byte's
              // source when there is one (no division)
              const uint32_t m = r_out + r_lit, kk = p - m;
              const uint32_t q2 = mq != ~0u ? (mq + 1u == m ? m - r_off : mq + 1u)
                                            : m - r_off + (kk < r_off ? kk : kk % r_off);
              mq = q2;
              if (q2 < it_lo) {
                S.v[k] = q2;
              } else {                  // its group, relative to the iteration
                S.v[k] = (gp + ((q2 + dmis) >> 4) - gw - it) * 16u + ((q2 + dmis) & 15u);
                pv |= 1u << k;
              }
            }
          }
          const uint32_t ld = hv & ~pv;
          HZ_UNROLL
          for (uint32_t k = 0; k < 16u; k++) {
            const uint32_t x = S.v[k];
            const uint64_t la = (uint64_t)(uintptr_t)src + (x & 0x7fffffffu), da = (uint64_t)(uintptr_t)dst + x;
            const uint32_t v = *HZ_GLOBAL(hz_gcu8*, (uintptr_t)((ld >> k) & 1u ? ((x >> 31) ? la : da)
                                                                            : (uint64_t)(uintptr_t)dst));
            ww[k >> 2] |= ((ld >> k) & 1u ? v : 0u) << (8u * (k & 3u));
          }
        }
        uint32_t* ibw = (uint32_t*)(ls.ib + 16u * (uint32_t)lane);
        ibw[0] = ww[0]; ibw[1] = ww[1]; ibw[2] = ww[2]; ibw[3] = ww[3];
        ls.pm[lane] = (uint16_t)pv;
        LV(have) = hv;
        LV(pend) = pv;
        LV(gsplit) = s;
      }
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
              if (!((ls.pm[sx >> 4] >> (sx & 15u)) & 1u)) {
                dn |= 1u << k;
                vv[k >> 2] |= (uint32_t)ls.ib[sx] << (8u * (k & 3u));
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
            uint32_t* ibw = (uint32_t*)(ls.ib + 16u * (uint32_t)lane);
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
            ls.pm[lane] = (uint16_t)LV(pend);
          }
        }
        WAVE_SYNC();
      }
      LANE_LOOP {
        const uint32_t g = it + (uint32_t)lane;
        if (g < total && LV(have)) {
          const uint32_t s = LV(gsplit);
          const LaneJob j = ls.job[s];
          hz_gu8* dst = HZ_GLOBAL(hz_gu8*, j.dst);
          const uint32_t dmis = (uint32_t)(((uintptr_t)j.dst) & 3u);
          const uint32_t a0 = (((ls.m_lo[s] + dmis) >> 4) + (g - ls.gpre[s])) * 16u;
          const uint32_t* ibw = (const uint32_t*)(ls.ib + 16u * (uint32_t)lane);
          for (uint32_t i = 0; i < 4u; i++) {
            const uint32_t w = ibw[i];
            const uint32_t hm = (LV(have) >> (4u * i)) & 15u;
            if (hm == 15u) {
              *(hz_gu32*)(dst + (a0 + 4u * i - dmis)) = w;
            } else if (hm) {
              for (uint32_t k = 0; k < 4u; k++)
                if (hm & (1u << k)) dst[a0 + 4u * i + k - dmis] = (uint8_t)(w >> (8u * k));
            }
          }
        }
      }
      WAVE_SYNC_GLOBAL();       // this iteration's output final before the next one reads it
    }
    HZ_T(0);
    LANE_LOOP {
      if (lane < GROUP && LV(active) && LV(ps).done) {
        if (LV(ps).op != ls.job[lane].dst_len) ls.m_st[lane] = hz::ST_SIZE;
        LV(active) = 0;
      }
    }
  }
  WAVE_SYNC();
}

}  // namespace lz
