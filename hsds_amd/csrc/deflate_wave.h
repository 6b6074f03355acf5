// deflate_wave.h -- wavefront zlib (RFC 1950/1951) encoder, split into phases.
//
// Replaces, for the HSDS data-node write path, the zlib deflate that the reference
// reaches through storUtil._compress (hsds/util/storUtil.py:238-281):
// numcodecs Blosc(cname="zlib", clevel, shuffle).encode -> c-blosc 1.21
// zlib_wrap_compress -> compress2(level) once per Blosc split.  The compressed bytes
// need not equal libz's (any valid deflate is accepted); the
// stream must inflate to the input through libz, c-blosc and the reference's
// _uncompress, and its size should stay within a few percent of zlib's level.
//
// A stream is cut into segments of SEG input bytes; every segment becomes one
// deflate block (dynamic Huffman, fixed Huffman or stored, whichever is smallest)
// with exact bit packing (no flush markers).  The work is split into phases so that
// each runs at the occupancy its LDS footprint allows (DESIGN.md "Deflate encoder"):
//
//   P  parse_stream   one wavefront per stream, segments in order (the hash head
//                     table and the input ring carry over, matches reach WIN bytes
//                     behind the segment).  Per segment:
//                     - exact hash chains: positions are inserted 64 at a time, the
//                       64 (hash, lane) keys are bitonic-sorted across the wave, so
//                       every position learns its true predecessor with the same
//                       3-byte hash and the last position of every run updates head;
//                     - lane-parallel greedy LZ77 parse: lane l owns an equal 1/64
//                       share of the segment (matches truncated at its end), chain
//                       depth / nice length from the level;
//                     - tokens (16-bit slots) and symbol frequencies go to HBM;
//                     - adler32 as per-lane (sum b, sum pos*b), combined at the end.
//   H  huff_segment   one wavefront per segment: bitonic sort of the symbols by
//                     frequency in LDS, in-place minimum-redundancy code lengths
//                     (Moffat & Katajainen), Kraft-exact limiting to 15 / 7 bits,
//                     canonical codes, the RFC 1951 3.2.7 code-length header, the
//                     block type and its exact size in bits.
//   L  (engine.hip)   per chunk: stream sizes -> c-blosc frame layout -> the
//                     absolute bit position of every block in the destination.
//   E  emit_segment   one wavefront per segment: lanes count their tokens' bits, a
//                     wave prefix sum places them, lanes OR them into LDS staging,
//                     the block is stored at its bit position with whole-word
//                     stores (the two edge words it shares with its neighbours by
//                     atomic OR into words L zeroed).
//
// SINGLE SOURCE for two drivers exactly like inflate_wave.h: the HIP kernels
// (engine.hip) and the CPU emulation (tests/emu/deflate_emu.cpp, test only).
#pragma once
#include "inflate_wave.h"

namespace hd {

constexpr int WAVE = 64;
constexpr int SEG = 8192;                   // input bytes per deflate block
constexpr int RING = 2 * SEG;               // LDS input ring: window + current segment
constexpr int RWORDS = RING / 4;
constexpr int LOOK = 4;                     // bytes staged past the segment end (hashes)
constexpr uint32_t WIN = SEG - 2 * LOOK;    // farthest match source before the segment
constexpr uint32_t FARW = 32768;            // zlib window: with a far ring, matches reach this far
                                            // (candidates past the LDS ring come from HBM)
#ifndef HD_HBITS
#define HD_HBITS 11
#endif
#ifndef HD_SKEW
#define HD_SKEW 1                           // skewed lane ranges (lane_start)
#endif
constexpr int HBITS = HD_HBITS;
constexpr int HSIZE = 1 << HBITS;
constexpr int LANE_MAX = SEG / WAVE + (HD_SKEW == 2 ? 6 : 4);   // input bytes per lane (a full segment; lane_start's skew)
constexpr int TSLOTS = LANE_MAX;            // 16-bit token slots per lane
constexpr int SEG_TOK = TSLOTS * WAVE;      // token slots per segment in HBM
constexpr int STAGE_WORDS = SEG / 4 + 24;   // a block is never emitted above its stored size
constexpr int NLL = 286, ND = 30, NCL = 19;
constexpr int NSYM = NLL + ND;
constexpr uint32_t ADLER_MOD = 65521;
constexpr uint32_t KEY_NONE = 0xffffffffu;

struct Tune {
  uint32_t chain;    // hash-chain candidates tried per position
  uint32_t nice;     // stop searching at this match length
  uint32_t too_far;  // length-3 matches farther than this are not taken (zlib TOO_FAR)
  uint32_t stored;   // 1: level 0, stored blocks only
  uint32_t far;       // 1: chains continue through the HBM far ring (32 KiB window; zlib
                      // levels >= 6, where ratio outweighs the parse time it costs)
};

#if HZ_GPU
__host__ __device__
#endif
inline uint32_t far_level(int level) { return level >= 6 ? 1u : 0u; }

HZ_HD Tune tune_for_level(int level) {
  Tune t;
  t.too_far = 4096;
  t.stored = level <= 0 ? 1u : 0u;
  // measured on the cfg5 slab (chain 4, L4): the far ring left the ratio unchanged (1.0018
  // vs libz L4) and cost 45 % more parse time; deeper chains gain ratio only with it
  t.far = far_level(level);
  switch (level) {
    case 1: t.chain = 1; t.nice = 8; break;
    case 2: t.chain = 2; t.nice = 16; break;
    case 3: t.chain = 2; t.nice = 32; break;
    case 4: case 5: t.chain = 4; t.nice = 32; break;
    case 6: t.chain = 8; t.nice = 64; break;
    case 7: t.chain = 16; t.nice = 128; break;
    case 8: t.chain = 32; t.nice = 258; break;
    default: t.chain = 64; t.nice = 258; break;
  }
  return t;
}

// zlib FLG byte for a level (deflate.c level_flags, FCHECK so that CMF*256+FLG is a
// multiple of 31); CMF = 0x78 (deflate, 32 KiB window).
HZ_HD uint32_t zlib_flg(int level) {
  const uint32_t lf = level < 2 ? 0u : level < 6 ? 1u : level == 6 ? 2u : 3u;
  const uint32_t f = lf << 6;
  return f | (31u - ((0x78u * 256u + f) % 31u)) % 31u;
}

// length 3..258 -> literal/length symbol offset (0..28) and extra bits
HZ_HD void len_sym(uint32_t len, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
  const uint32_t x = len - 3u;
  if (len == 258u) { sym = 28; eb = 0; ev = 0; return; }
  if (x < 8u) { sym = x; eb = 0; ev = 0; return; }
  const uint32_t msb = 31u - (uint32_t)__builtin_clz(x);
  eb = msb - 2u;
  sym = 4u * (msb - 1u) + ((x >> eb) & 3u);
  ev = x & ((1u << eb) - 1u);
}
// distance 1..32768 -> distance symbol (0..29) and extra bits
HZ_HD void dist_sym(uint32_t dist, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
  const uint32_t x = dist - 1u;
  if (x < 4u) { sym = x; eb = 0; ev = 0; return; }
  const uint32_t msb = 31u - (uint32_t)__builtin_clz(x);
  eb = msb - 1u;
  sym = 2u * msb + ((x >> eb) & 1u);
  ev = x & ((1u << eb) - 1u);
}
HZ_HD uint32_t len_extra_bits(uint32_t k) { return (k < 8u || k == 28u) ? 0u : (k - 4u) / 4u; }
HZ_HD uint32_t dist_extra_bits(uint32_t s) { return s < 4u ? 0u : (s - 2u) / 2u; }
HZ_HD uint32_t fixed_ll_len(uint32_t s) { return s < 144u ? 8u : s < 256u ? 9u : s < 280u ? 7u : 8u; }
HZ_HD uint32_t cl_extra_bits(uint32_t sym) { return sym == 16u ? 2u : sym == 17u ? 3u : sym == 18u ? 7u : 0u; }
HZ_HD uint32_t rev16(uint32_t code, uint32_t len) {
#if HZ_GPU
  return len ? __builtin_bitreverse32(code) >> (32u - len) : 0u;     // one v_bfrev_b32
#else
  uint32_t r = 0;
  for (uint32_t i = 0; i < len; i++) { r = (r << 1) | (code & 1u); code >>= 1; }
  return r;
#endif
}

HZ_HD void lds_add(uint32_t* p, uint32_t v) {
#if HZ_GPU
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
// LDS exchange: returns *p and stores v.  On gfx950 the lanes of one ds_wrxchg_rtn_b32
// that hit the same address are applied in ascending lane order (measured over 12.8 M
// lanes at 0..11 hash bits, tools/lds_xchg_order.hip), which is the CPU emulation's
// sequential lane order.
HZ_HD uint32_t lds_xchg(uint32_t* p, uint32_t v) {
#if HZ_GPU
  return atomicExch(p, v);
#else
  const uint32_t o = *p;
  *p = v;
  return o;
#endif
}
HZ_HD void lds_or(uint32_t* p, uint32_t v) {
#if HZ_GPU
  atomicOr(p, v);
#else
  *p |= v;
#endif
}
HZ_HD void glb_or(uint32_t* p, uint32_t v) {
#if HZ_GPU
  atomicOr(p, v);
#else
  *p |= v;
#endif
}

// ---- per-segment records in HBM (phase outputs) ------------------------------
struct SegParse {            // P -> H, E
  uint32_t freq[NSYM];       // literal/length 0..285 | distance 286..315 (EOB not counted)
  uint16_t nslot[WAVE];      // token slots used per lane
};
struct SegCode {             // H -> L, E
  uint32_t tab[NSYM];        // (reversed code << 4) | length, literal/length then distance
  uint32_t cl[NCL + 1];      // code-length code, same packing
  uint16_t rle[NSYM];        // code-length sequence: symbol | extra << 8
  uint32_t nrle, hlit, hdist, hclen;
  uint32_t btype;            // 0 stored, 1 fixed, 2 dynamic
  uint32_t bits;             // exact block bits for fixed / dynamic, 3-bit header included
};
struct SegOut {              // L -> E
  uint64_t bitpos;           // bit position of the block in the destination buffer
  uint32_t item;             // EncItem slot of the stream
  uint32_t seg;              // segment index in the stream
  uint32_t flags;            // bit 0: emit, bit 1: final block (+ padding + adler32)
  uint32_t adler;
};

struct EncJob {
  const uint8_t* src;   // stream input (any alignment); with ts > 1 the Blosc block base
  uint32_t len;         // input bytes
  int level;
  uint32_t ts;          // > 1: the stream is bytes [off, off + len) of the byte-shuffled block
  uint32_t neb;         //      (c-blosc shuffle: plane-major, neb elements per plane, tail as-is)
  uint32_t off;
};

HZ_HD uint32_t nsegments(uint32_t len) { return len ? (len + SEG - 1) / SEG : 1u; }

// byte k of a byte-shuffled Blosc block (c-blosc shuffle(): plane j holds byte j of
// every element; the bs % ts tail bytes follow unchanged)
HZ_HD uint32_t shuffled_src_index(uint32_t k, uint32_t ts, uint32_t neb) {
  return k < neb * ts ? (k % neb) * ts + k / neb : k;
}

// 4 stream bytes [p, p + 4) & the valid range [p, hi) (zeros beyond), from global
HZ_HD uint32_t load_stream_word(const EncJob& job, uint32_t p, uint32_t hi) {
  uint32_t v = 0;
  if (job.ts > 1u) {                          // gather from the unshuffled block
    hz_gcu8* const bsrc = HZ_GLOBAL(hz_gcu8*, job.src);
    for (uint32_t b = 0; b < 4u; b++)
      if (p + b < hi) v |= (uint32_t)bsrc[shuffled_src_index(job.off + p + b, job.ts, job.neb)] << (8u * b);
    return v;
  }
  hz_gcu8* const gsrc = HZ_GLOBAL(hz_gcu8*, (uintptr_t)job.src & ~(uintptr_t)3);
  const uint32_t sa = (uint32_t)((uintptr_t)job.src & 3u);
  const uint32_t a = p + sa;                  // byte offset from the aligned base
  const uint32_t lo = sa, hh = sa + hi;       // valid bytes [lo, hh) of the aligned base
  const uint32_t w0 = hz::load_word(gsrc, a >> 2, lo, hh);
  v = w0;
  if (a & 3u) {
    const uint32_t w1 = hz::load_word(gsrc, (a >> 2) + 1u, lo, hh);
    const uint32_t s = (a & 3u) * 8u;
    v = (w0 >> s) | (w1 << (32u - s));
  }
  return v;
}

// Lane l's range of a segment of seglen bytes: [lane_start(l), lane_start(l + 1)), R =
// ceil(seglen / 64) bytes each with the start skewed by 4 floor(l / 2) bytes.  Unskewed, the
// lanes start 128 bytes apart, so their input-ring words (and their 16-bit predecessor links)
// sit in one LDS bank -- and stay near it as the lanes advance at similar rates; skewed, the
// first ring words of the 64 lanes fall in 64 banks.  A range grows by at most 4 bytes.
HZ_HD uint32_t lane_start(uint32_t l, uint32_t seglen) {
  const uint32_t R = (seglen + (uint32_t)WAVE - 1u) / (uint32_t)WAVE;
#if HD_SKEW == 2
  // ds_read_b32 banks are (a / 4) mod 32 per 32-lane group: 4 l bytes put lane l's ring word
  // in bank l, and 2 more bytes for lanes 16-31 of each group put its 16-bit link (bank
  // (p / 2) mod 32 = 2 l + 1) apart from lane l - 16's
  const uint32_t a = l * R + 4u * l + 2u * ((l >> 4) & 1u);
#elif HD_SKEW
  const uint32_t a = l * R + 4u * (l >> 1);
#else
  const uint32_t a = l * R;
#endif
  return a < seglen ? a : seglen;
}

// token slot s of lane `lane` inside one segment's SEG_TOK slots: pairs of a lane
// share one dword, lanes interleaved so that a wave's k-th slots are contiguous
HZ_HD uint32_t tslot(uint32_t s, int lane) { return ((s >> 1) * (uint32_t)WAVE + (uint32_t)lane) * 2u + (s & 1u); }

// ============================================================================
// P: parse
// ============================================================================
struct ParseShared {
  uint32_t ring[RWORDS];                 // input bytes, position p at byte p % RING
  uint16_t prev[SEG];                    // (predecessor position) & 0xffff per segment position
  // latest position per hash (32-bit: the exchange target).  The greedy parse never reads
  // the heads, so the symbol counts live in entries [0, NSYM) during it, with those heads
  // saved in registers (40 KiB in all: 4 parse waves per CU)
  union {
    uint32_t head[HSIZE];
    uint32_t freq[NSYM];
  };
};
// The parse's symbol counts, with one dummy entry per lane (a literal counts its absent
// distance there): the LDS applies same-address atomics one after the other, and with one
// dummy shared by all lanes every count instruction serialised on it (2/3 of the parse's
// LDS cycles were bank conflicts, profiles/r5_sq_encode.txt; per-lane dummies: deflate
// 125.5 -> 121.1 ms on the cfg5 slab).  HD_NREP > 1 spreads the counts over replicas, lane l
// adding to replica l % HD_NREP (odd multiples of 4 dwords apart: different banks); measured
// 122.1 ms at 4 and 6 replicas, so one set stays.  (An XOR bank swizzle of the ring and the
// prev[] links -- the lanes start 128 bytes apart, one bank -- measured 130 ms: its address
// arithmetic costs more than the conflicts.)
#ifndef HD_WALKB
#define HD_WALKB 8                          // the emit walk's token dwords per batch of loads
#endif
#ifndef HD_ADLER_DOT
#define HD_ADLER_DOT 1                      // the staging's adler sums by byte dot products
#endif
#ifndef HD_NREP
#define HD_NREP 1
#endif
constexpr uint32_t NREP = HD_NREP;
constexpr uint32_t CSTR0 = (((uint32_t)NSYM + ((uint32_t)WAVE + NREP - 1u) / NREP) + 3u) & ~3u;
constexpr uint32_t CSTR = (CSTR0 / 4u) % 2u ? CSTR0 : CSTR0 + 4u;   // entries per replica
constexpr uint32_t CENT = NREP * CSTR;                               // head entries the counts take
constexpr uint32_t NSAVE = (CENT + (uint32_t)WAVE - 1u) / (uint32_t)WAVE;   // head entries saved per lane
static_assert(CENT <= (uint32_t)HSIZE, "count replicas fit the head table");

// bytes [p, p + 4) from the two words a, b they span: {b, a} >> 8 (p & 3) (v_alignbyte)
HZ_HD uint32_t funnel(uint32_t a, uint32_t b, uint32_t p) {
#if HZ_GPU
  return __builtin_amdgcn_alignbyte(b, a, p & 3u);
#else
  const uint32_t s = (p & 3u) * 8u;
  return s ? (a >> s) | (b << (32u - s)) : a;
#endif
}
// c + the dot product of the four bytes of a and of b (v_dot4_u32_u8)
HZ_HD uint32_t dot4(uint32_t a, uint32_t b, uint32_t c) {
#if HZ_GPU
  return __builtin_amdgcn_udot4(a, b, c, false);
#else
  for (uint32_t i = 0; i < 32u; i += 8u) c += ((a >> i) & 255u) * ((b >> i) & 255u);
  return c;
#endif
}
HZ_HD uint32_t rd32(const ParseShared& sh, uint32_t p) {
  const uint32_t w = (p >> 2) & (uint32_t)(RWORDS - 1);
  return funnel(sh.ring[w], sh.ring[(w + 1u) & (uint32_t)(RWORDS - 1)], p);
}
HZ_HD uint32_t rd8(const ParseShared& sh, uint32_t p) {
  return (sh.ring[(p >> 2) & (uint32_t)(RWORDS - 1)] >> ((p & 3u) * 8u)) & 0xffu;
}
HZ_HD uint32_t hash3(uint32_t w) { return ((w & 0xffffffu) * 0x9E3779B1u) >> (32 - HBITS); }

HZ_HD uint32_t match_len(const ParseShared& sh, uint32_t q, uint32_t p, uint32_t maxl) {
  uint32_t L = 0;
  while (L < maxl) {
    const uint32_t x = rd32(sh, q + L) ^ rd32(sh, p + L);
    if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
    L += 4u;
  }
  return L < maxl ? L : maxl;
}

}  // namespace hd

namespace hd {
// far candidate q (before the LDS ring): its bytes from the stream in HBM, the current
// position's from the ring (q + maxl <= p, so stream bytes past the end are never compared)
HZ_HD uint32_t match_len_far(const ParseShared& sh, const EncJob& job, uint32_t q, uint32_t p, uint32_t maxl) {
  uint32_t L = 0;
  while (L < maxl) {
    const uint32_t x = load_stream_word(job, q + L, job.len) ^ rd32(sh, p + L);
    if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
    L += 4u;
  }
  return L < maxl ? L : maxl;
}
}  // namespace hd

// ---- wave-collective helpers for the encoder ---------------------------------
#if HZ_GPU
namespace hd {
// lane i <- lane i ^ j.  DPP inside a row (no LDS round trip): quad_perm for j = 1,
// 2; for j = 4, 8 two row shifts, each writing the banks (groups of 4 lanes) whose
// partner lies in its direction.  j = 16, 32 cross rows: ds_bpermute.
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int j) {
  switch (j) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    case 4: {
      const int r = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x104, 0xF, 0x5, false);   // row_shl:4
      return (uint32_t)__builtin_amdgcn_update_dpp(r, (int)v, 0x114, 0xF, 0xA, false);     // row_shr:4
    }
    case 8: {
      const int r = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x108, 0xF, 0x3, false);   // row_shl:8
      return (uint32_t)__builtin_amdgcn_update_dpp(r, (int)v, 0x118, 0xF, 0xC, false);     // row_shr:8
    }
    default: return __shfl_xor(v, j, 64);
  }
}
__device__ __forceinline__ uint32_t wave_sort64(uint32_t key, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t o = lane_xor(key, j);
      const bool lower = (lane & j) == 0;
      const bool asc = (lane & k) == 0;
      const uint32_t mn = o < key ? o : key, mx = o < key ? key : o;
      key = (lower == asc) ? mn : mx;
    }
  }
  return key;
}
}  // namespace hd
#define HD_SORT64(var) var = hd::wave_sort64(var, (int)threadIdx.x)
#define HD_NEIGHBOURS(prv, nxt, var)                   \
  do {                                                 \
    prv = __shfl_up(var, 1, 64);                       \
    nxt = __shfl_down(var, 1, 64);                     \
    if (threadIdx.x == 0) prv = hd::KEY_NONE;          \
    if (threadIdx.x == 63) nxt = hd::KEY_NONE;         \
  } while (0)
#else
#define HD_SORT64(var)                                                      \
  do {                                                                      \
    for (int _i = 1; _i < 64; _i++) {                                       \
      uint32_t _k = var[_i]; int _j = _i - 1;                               \
      while (_j >= 0 && var[_j] > _k) { var[_j + 1] = var[_j]; _j--; }       \
      var[_j + 1] = _k;                                                     \
    }                                                                       \
  } while (0)
#define HD_NEIGHBOURS(prv, nxt, var)                                        \
  do {                                                                      \
    for (int _l = 0; _l < 64; _l++) {                                       \
      prv[_l] = _l ? var[_l - 1] : hd::KEY_NONE;                            \
      nxt[_l] = _l < 63 ? var[_l + 1] : hd::KEY_NONE;                       \
    }                                                                       \
  } while (0)
#endif

namespace hd {

// parse_stream runs as a one-wavefront workgroup, and the LDS executes a wave's
// instructions in order: a cross-lane LDS hand-off only needs the compiler not to move or
// cache LDS accesses across it (wavefront-scope fences), not the s_waitcnt vmcnt(0) of
// __syncthreads, which would also wait for the token stores and the staging prefetch
#if HZ_GPU
#define HD_LDS_SYNC()                                           \
  do {                                                          \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");      \
    __builtin_amdgcn_wave_barrier();                            \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");      \
  } while (0)
#else
#define HD_LDS_SYNC() do {} while (0)
#endif

// the ring words of a segment's staging range [s0, hi) a lane prefetches (word k = lane +
// 64 u), for a contiguous 4-byte aligned stream (job.ts <= 1): whole aligned dwords, the
// bytes past hi are masked when the words are staged (a dword never crosses a page)
constexpr uint32_t PF_WORDS = ((uint32_t)SEG + (uint32_t)LOOK + 3u) / 4u / (uint32_t)WAVE + 1u;
HZ_HD void stage_fetch(const EncJob& job, uint32_t s0, uint32_t hi, int lane, uint32_t* pf) {
  hz_gcu32* const w = HZ_GLOBAL(hz_gcu32*, job.src);
  const uint32_t nw = (hi - s0 + 3u) / 4u;
  HZ_UNROLL
  for (uint32_t u = 0; u < PF_WORDS; u++) {
    const uint32_t k = (uint32_t)lane + u * (uint32_t)WAVE;
    pf[u] = k < nw ? w[(s0 >> 2) + k] : 0u;
  }
}

// branch-free symbol codes for the counts (len 3..258, dist 1..32768)
HZ_HD uint32_t len_code(uint32_t len) {
  const uint32_t x = len - 3u;
  const uint32_t msb = 31u - (uint32_t)__builtin_clz(x | 1u);
  const uint32_t eb = msb >= 2u ? msb - 2u : 0u;
  const uint32_t c = x < 8u ? x : 4u * (msb - 1u) + ((x >> eb) & 3u);
  return len == 258u ? 28u : c;
}
HZ_HD uint32_t dist_code(uint32_t dist) {
  const uint32_t x = dist - 1u;
  const uint32_t msb = 31u - (uint32_t)__builtin_clz(x | 1u);
  const uint32_t eb = msb >= 1u ? msb - 1u : 0u;
  return x < 4u ? x : 2u * msb + ((x >> eb) & 1u);
}

// One lane's greedy parse of stream bytes [pos, end) (its share of the segment at s0):
// tokens into its slots of gtok, symbol counts into the head entries [0, NSYM) (and a
// dummy entry NSYM that literal tokens count their absent distance into).  Returns the
// number of 16-bit slots written.  FAR: candidates before the LDS ring come from the HBM
// far ring and the stream in HBM; without it every candidate lies in the ring, and the
// per-token work is straight-line except the chain walk and the match extension.
template <bool FAR>
HZ_HD uint32_t parse_range(ParseShared& sh, const EncJob& job, const Tune& tune, hz_gu16* gfar, hz_gu8* gtok,
                           int lane, uint32_t s0, uint32_t pos, uint32_t end, uint32_t lo_pos) {
  uint32_t ns = 0;
  uint32_t pend = 0, npend = 0;    // slot pairs (2k, 2k + 1) of a lane are stored as one dword
  while (pos < end) {
    uint32_t best = 0, bd = 0;
    const uint32_t maxl = end - pos < 258u ? end - pos : 258u;
    const uint32_t cur = rd32(sh, pos);
    uint32_t c16 = sh.prev[pos - s0];
    const uint32_t maxd = FAR ? (pos < FARW ? pos : FARW) : pos - lo_pos;
    const uint32_t chain = maxl >= 3u ? tune.chain : 0u;
    for (uint32_t depth = 0; depth < chain; depth++) {
      const uint32_t d = (pos - c16) & 0xffffu;
      if (d == 0u || d > maxd) break;
      const uint32_t q = pos - d;
      uint32_t x;
      bool near = true;
      if (FAR) {
        near = q >= lo_pos;
        // the next candidate's load is independent of this compare: issue it now
        c16 = q >= s0 ? (uint32_t)sh.prev[q - s0] : (uint32_t)gfar[q & (FARW - 1u)];
        x = (near ? rd32(sh, q) : load_stream_word(job, q, job.len)) ^ cur;
      } else {
        // (d <= maxd keeps q inside the ring; a candidate before the segment ends the chain)
        const uint32_t pv = sh.prev[q >= s0 ? q - s0 : 0u];
        x = rd32(sh, q) ^ cur;
        c16 = q >= s0 ? pv : pos;
      }
      const uint32_t L0 = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4u;
      // only a candidate that can beat `best` is measured in full
      const bool cand = L0 >= 3u && (L0 > best || (L0 == 4u && best >= 4u));
      uint32_t L = L0;
      if (cand && L0 == 4u && maxl > 4u)
        L = 4u + (near ? match_len(sh, q + 4u, pos + 4u, maxl - 4u)
                       : match_len_far(sh, job, q + 4u, pos + 4u, maxl - 4u));
      L = L < maxl ? L : maxl;
      const bool better = cand && L > best;
      best = better ? L : best;
      bd = better ? d : bd;
      if (better && (L >= tune.nice || L == maxl)) break;
    }
    if (best == 3u && bd > tune.too_far) best = 0;
    const bool m = best >= 3u;
    const uint32_t lit = cur & 0xffu;
    const uint32_t t0 = m ? (0x8000u | (best - 3u)) : lit;
    const uint32_t t1 = bd - 1u;
    // counts (sh.freq aliases sh.head; the dummy entry NSYM is restored with the heads)
    {
      const uint32_t rb = ((uint32_t)lane % NREP) * CSTR;
      lds_add(&sh.head[rb + (m ? 257u + len_code(best) : lit)], 1u);
      lds_add(&sh.head[rb + (m ? (uint32_t)NLL + dist_code(bd) : (uint32_t)NSYM + (uint32_t)lane / NREP)], 1u);
    }
    pos += m ? best : 1u;
    // a pending slot pairs with t0; a match without one stores (t0, t1)
    if (npend || m)
      *(hz_gu32*)(gtok + (size_t)tslot(ns & ~1u, lane) * 2u) = npend ? (pend | (t0 << 16)) : (t0 | (t1 << 16));
    pend = npend ? t1 : t0;
    npend = (npend + (m ? 2u : 1u)) & 1u;
    ns += m ? 2u : 1u;
  }
  if (npend) *(hz_gu32*)(gtok + (size_t)tslot(ns - 1u, lane) * 2u) = pend;
  return ns;
}

// Parse one stream into per-segment tokens and frequencies.  sp / tok: this
// stream's first segment record / token block (SEG_TOK slots per segment).
// Returns the adler32 of the stream input.
//
// far (used when tune.far): this wave's ring of FARW predecessor entries in HBM.  Every segment's chain
// links go there after its parse, so a chain that leaves the segment goes on into earlier
// ones and matches reach FARW (zlib's 32 KiB window) instead of the LDS ring's WIN; a far
// candidate's bytes are read from the stream in HBM.
HZ_HD uint32_t parse_stream(ParseShared& sh, const EncJob& job, const Tune& tune, SegParse* sp, uint16_t* tok,
                            HzProf* prof = nullptr, uint16_t* far = nullptr) {
  (void)prof;
  hz_gu16* const gfar = tune.far ? HZ_GLOBAL(hz_gu16*, far) : nullptr;
  const uint32_t n = job.len;
  const uint32_t nseg = nsegments(n);
  LANE_VAR(uint64_t, as1);           // adler partial sums: S1 = sum b, S2 = sum pos * b
  LANE_VAR(uint64_t, as2);
  LANE_LOOP {
    LV(as1) = 0; LV(as2) = 0;
    for (int h = lane; h < HSIZE; h += WAVE) sh.head[h] = 0xffffffffu;
  }
  HD_LDS_SYNC();

#if HZ_GPU
  uint32_t pf[PF_WORDS];
  const bool pf_ok = job.ts <= 1u && ((uintptr_t)job.src & 3u) == 0u;
#endif
  for (uint32_t seg = 0; seg < nseg; seg++) {
    const uint32_t s0 = seg * (uint32_t)SEG;
    const uint32_t s1 = s0 + (uint32_t)SEG < n ? s0 + (uint32_t)SEG : n;
    const uint32_t seglen = s1 - s0;
    const uint32_t stage_hi = s1 + (uint32_t)LOOK < n ? s1 + (uint32_t)LOOK : n;
    SegParse* const out = sp + seg;
    hz_gu8* const gtok = HZ_GLOBAL(hz_gu8*, tok + (size_t)seg * SEG_TOK);

    // ---- stage the segment (+ lookahead) into the ring, adler sums ----
    HZ_T(1);
    LANE_LOOP {
      const uint32_t nw = (stage_hi - s0 + 3u) / 4u;
      // byte sums of the word at p: S1 += bytes below s1, S2 += their positions * bytes
#if HD_ADLER_DOT
      // (byte dot products: sum b and sum (p + k) b of the word's bytes below s1 -- one
      // 32 x 32 -> 64 multiply per word instead of four 64-bit ones, round 6)
#define HD_ADLER_WORD(p, v)                                                    \
      {                                                                        \
        const uint32_t w_ = (p) + 4u <= s1 ? (v) : (p) >= s1 ? 0u : (v) & hz::bmask(8u * (s1 - (p))); \
        const uint32_t sb_ = hd::dot4(w_, 0x01010101u, 0u);                   \
        LV(as1) += sb_;                                                        \
        LV(as2) += (uint64_t)(p) * sb_ + hd::dot4(w_, 0x03020100u, 0u);       \
      }
#else
#define HD_ADLER_WORD(p, v)                                                    \
      for (uint32_t b = 0; b < 4u; b++) {                                      \
        const uint32_t q = (p) + b;                                            \
        if (q < s1) {                                                          \
          const uint32_t byte = ((v) >> (8u * b)) & 0xffu;                     \
          LV(as1) += byte;                                                     \
          LV(as2) += (uint64_t)q * byte;                                       \
        }                                                                      \
      }
#endif
#if HZ_GPU
      if (pf_ok) {
        // the words were fetched into registers while the previous segment was parsed
        if (seg == 0) stage_fetch(job, s0, stage_hi, lane, pf);
        HZ_UNROLL
        for (uint32_t u = 0; u < PF_WORDS; u++) {
          const uint32_t k = (uint32_t)lane + u * (uint32_t)WAVE;
          const uint32_t p = s0 + 4u * k;           // stream position of ring word
          if (k < nw) {
            const uint32_t v = stage_hi - p >= 4u ? pf[u] : pf[u] & ((1u << (8u * (stage_hi - p))) - 1u);
            sh.ring[(p >> 2) & (uint32_t)(RWORDS - 1)] = v;
            HD_ADLER_WORD(p, v)
          }
        }
      } else
#endif
      for (uint32_t k = (uint32_t)lane; k < nw; k += WAVE) {
        const uint32_t p = s0 + 4u * k;             // stream position of ring word
        const uint32_t v = load_stream_word(job, p, stage_hi);
        sh.ring[(p >> 2) & (uint32_t)(RWORDS - 1)] = v;
        HD_ADLER_WORD(p, v)
      }
#undef HD_ADLER_WORD
#if HZ_GPU
      // the next segment's words: their loads complete under this segment's chains and parse
      if (pf_ok && seg + 1u < nseg) {
        const uint32_t t0 = s1, t1 = t0 + (uint32_t)SEG < n ? t0 + (uint32_t)SEG : n;
        stage_fetch(job, t0, t1 + (uint32_t)LOOK < n ? t1 + (uint32_t)LOOK : n, lane, pf);
      }
#endif
    }
    HD_LDS_SYNC();

    const uint32_t lo_pos = s0 > WIN ? s0 - WIN : 0u;   // farthest match source in the LDS ring
    if (!tune.stored) {
      // ---- exact hash chains, 64 positions per step: one exchange on the head table
      // gives every position the latest earlier position with its hash (lanes of one
      // exchange apply in lane order, so a position sees the lower lanes of its step) ----
      HZ_T(2);
      for (uint32_t g = s0; g < s1; g += WAVE) {
        LANE_LOOP {
          const uint32_t p = g + (uint32_t)lane;
          if (p < s1 && p + 2u < n) sh.prev[p - s0] = (uint16_t)lds_xchg(&sh.head[hash3(rd32(sh, p))], p);
        }
      }
    }
    // the symbol counts (NREP replicas) take head entries [0, CENT) for the parse
#if HZ_GPU
    uint32_t hk[NSAVE];                  // (per lane: LV(hk)[u])
#else
    uint32_t hk[64][NSAVE];
#endif
    HD_LDS_SYNC();
    LANE_LOOP {
HZ_UNROLL
      for (uint32_t u = 0; u < NSAVE; u++) {
        const uint32_t k = (uint32_t)lane + u * (uint32_t)WAVE;
        LV(hk)[u] = k < CENT ? sh.head[k] : 0u;
      }
      for (uint32_t k = (uint32_t)lane; k < CENT; k += WAVE) sh.head[k] = 0;
    }
    HD_LDS_SYNC();

    // ---- lane-parallel greedy parse, tokens to HBM ----
    HZ_T(3);
    LANE_LOOP {
      const uint32_t a0 = lane_start((uint32_t)lane, seglen), a1 = lane_start((uint32_t)lane + 1u, seglen);
      uint32_t pos = s0 + a0;
      const uint32_t end = s0 + a1;
      const uint32_t ns = tune.stored ? 0u
                          : gfar ? parse_range<true>(sh, job, tune, gfar, gtok, lane, s0, pos, end, lo_pos)
                                 : parse_range<false>(sh, job, tune, gfar, gtok, lane, s0, pos, end, lo_pos);
      out->nslot[lane] = (uint16_t)ns;
    }
    HD_LDS_SYNC();
    LANE_LOOP {
      for (int s = lane; s < NSYM; s += WAVE) {
        uint32_t c = 0;
HZ_UNROLL
        for (uint32_t r = 0; r < NREP; r++) c += sh.head[r * CSTR + (uint32_t)s];
        out->freq[s] = c;
      }
    }
    HD_LDS_SYNC();
    LANE_LOOP {
HZ_UNROLL
      for (uint32_t u = 0; u < NSAVE; u++) {
        const uint32_t k = (uint32_t)lane + u * (uint32_t)WAVE;
        if (k < CENT) sh.head[k] = LV(hk)[u];
      }
      // the segment's chain links join the far ring once the segment is parsed (written
      // earlier, they would overwrite links FARW back that this parse still follows)
      if (gfar)
        for (uint32_t i = (uint32_t)lane; i < seglen; i += WAVE) gfar[(s0 + i) & (FARW - 1u)] = sh.prev[i];
    }
    if (gfar) WAVE_SYNC_GLOBAL();
    else HD_LDS_SYNC();
  }
  HZ_T(9);
  uint64_t S1, S2;
#if HZ_GPU
  S1 = hz::wave_sum64(as1);
  S2 = hz::wave_sum64(as2);
#else
  S1 = 0; S2 = 0;
  for (int l = 0; l < 64; l++) { S1 += as1[l]; S2 += as2[l]; }
#endif
  // adler32 = B << 16 | A with A = 1 + sum b, B = n + n * sum b - sum pos * b (mod 65521)
  const uint64_t A = (1u + S1) % ADLER_MOD;
  const uint64_t nm = (uint64_t)n % ADLER_MOD;
  const uint64_t B = (nm + nm * (S1 % ADLER_MOD) + (uint64_t)ADLER_MOD * ADLER_MOD - S2 % ADLER_MOD) % ADLER_MOD;
  return (uint32_t)((B << 16) | A);
}

// ============================================================================
// H: Huffman codes + block choice for one segment
// ============================================================================
struct HuffShared {
  uint32_t freq[NSYM];                   // patched (>= 2 codes per tree)
  uint32_t clf[NCL + 1];
  uint32_t keys[512];                    // sort scratch (freq << 9 | symbol)
  uint32_t work[NLL];                    // minimum-redundancy scratch
  uint8_t len_ll[NLL + 2];
  uint8_t len_d[ND + 2];
  uint8_t len_cl[NCL + 1];
  uint16_t code_ll[NLL];
  uint16_t code_d[ND];
  uint16_t code_cl[NCL + 1];
  uint16_t rle[NSYM];
  uint32_t nrle, hlit, hdist, hclen, hdr_bits, cnt;
  uint32_t bl_count[17];
  uint32_t next_code[17];
};

#ifndef HD_HUFF_X2
#define HD_HUFF_X2 0   // timing experiments only: bit 1/2/4 runs the sort / parents / counts twice
#endif
#ifndef HD_HUFF_REG
#define HD_HUFF_REG 1  // GPU: phases 1 and 3 by the whole wave (huff_parents_wave, huff_counts_wave)
#endif

// Serial part of the Huffman build (lane 0): keys[0..n) are sorted ascending by
// (frequency, symbol).  Minimum-redundancy lengths in place (Moffat & Katajainen
// 1995) and Kraft-exact limiting to maxbits give the code count per length
// (bl_count) and the first canonical code per length (next_code, RFC 1951 3.2.2);
// the lanes then assign lengths and codes (HD_BUILD_HUFF).
HZ_HD void huff_parents_serial(HuffShared& sh, int n) {
  uint32_t* A = sh.work;
  for (int i = 0; i < n; i++) A[i] = sh.keys[i] >> 9;
  // phase 1: parents, left to right
  A[0] += A[1];
  int root = 0, leaf = 2;
  for (int next = 1; next < n - 1; next++) {
    if (leaf >= n || A[root] < A[leaf]) { A[next] = A[root]; A[root++] = (uint32_t)next; }
    else A[next] = A[leaf++];
    if (leaf >= n || (root < next && A[root] < A[leaf])) { A[next] += A[root]; A[root++] = (uint32_t)next; }
    else A[next] += A[leaf++];
  }
}

// Phase 2 (all lanes): the depth of every internal node by pointer jumping.  After
// phase 1 A[i] (i < n - 2) is the parent of internal node i (parents lie to the right)
// and n - 2 is the root.  Each word packs pointer | depth-so-far << 16; ceil(log2 n)
// rounds of (d += d[p], p = p[p]) leave every node pointing at the root with its depth,
// the value the serial right-to-left pass A[i] = A[A[i]] + 1 computes.
#define HD_HUFF_DEPTHS(sh, NN)                                                           \
  do {                                                                                    \
    const int _n = (NN);                                                                  \
    uint32_t* const _A = (sh).work;                                                       \
    LANE_LOOP {                                                                           \
      for (int _i = lane; _i < _n - 1; _i += 64)                                          \
        _A[_i] = _i == _n - 2 ? (uint32_t)_i : (_A[_i] | (1u << 16));                     \
    }                                                                                     \
    WAVE_SYNC();                                                                          \
    for (int _s = 1; _s < _n; _s <<= 1) {                                                 \
      LANE_VAR(uint32_t, _v0); LANE_VAR(uint32_t, _v1); LANE_VAR(uint32_t, _v2);          \
      LANE_VAR(uint32_t, _v3); LANE_VAR(uint32_t, _v4);                                   \
      LANE_LOOP {                                                                         \
        uint32_t _t[5];                                                                   \
        HZ_UNROLL for (int _k = 0; _k < 5; _k++) {                                        \
          const int _i = lane + 64 * _k;                                                  \
          uint32_t _x = 0;                                                                \
          if (_i < _n - 1) {                                                              \
            const uint32_t _a = _A[_i], _b = _A[_a & 0xffffu];                            \
            _x = (_b & 0xffffu) | (((_a >> 16) + (_b >> 16)) << 16);                      \
          }                                                                               \
          _t[_k] = _x;                                                                    \
        }                                                                                 \
        LV(_v0) = _t[0]; LV(_v1) = _t[1]; LV(_v2) = _t[2]; LV(_v3) = _t[3]; LV(_v4) = _t[4]; \
      }                                                                                   \
      WAVE_SYNC();                                                                        \
      LANE_LOOP {                                                                         \
        const uint32_t _t[5] = {LV(_v0), LV(_v1), LV(_v2), LV(_v3), LV(_v4)};             \
        HZ_UNROLL for (int _k = 0; _k < 5; _k++) {                                        \
          const int _i = lane + 64 * _k;                                                  \
          if (_i < _n - 1) _A[_i] = _t[_k];                                               \
        }                                                                                 \
      }                                                                                   \
      WAVE_SYNC();                                                                        \
    }                                                                                     \
    LANE_LOOP { for (int _i = lane; _i < _n - 1; _i += 64) _A[_i] >>= 16; }               \
    WAVE_SYNC();                                                                          \
  } while (0)

// Serial phase 3 (lane 0): leaf depths -> counts per length, the length limit and the
// first canonical code per length.
HZ_HD void huff_counts_serial(HuffShared& sh, int n, int maxbits) {
  uint32_t* A = sh.work;
  for (int l = 0; l <= 16; l++) sh.bl_count[l] = 0;
  // phase 3: leaf depths -> counts per length
  {
    int avbl = 1, used = 0, dpth = 0;
    int root = n - 2;
    while (avbl > 0) {
      while (root >= 0 && (int)A[root] == dpth) { used++; root--; }
      while (avbl > used) { sh.bl_count[dpth > 16 ? 16 : dpth]++; avbl--; }
      avbl = 2 * used;
      dpth++;
      used = 0;
    }
  }
  // limit to maxbits keeping the code complete: fold longer codes onto maxbits, then
  // while the Kraft sum exceeds 1 move one maxbits code and split a shorter leaf
  for (int l = maxbits + 1; l <= 16; l++) { sh.bl_count[maxbits] += sh.bl_count[l]; sh.bl_count[l] = 0; }
  {
    uint32_t total = 0;
    for (int l = maxbits; l > 0; l--) total += sh.bl_count[l] << (maxbits - l);
    while (total != (1u << maxbits)) {
      sh.bl_count[maxbits]--;
      for (int l = maxbits - 1; l > 0; l--) {
        if (sh.bl_count[l]) { sh.bl_count[l]--; sh.bl_count[l + 1] += 2u; break; }
      }
      total--;
    }
  }
  // lengths and canonical codes: by all lanes (HD_BUILD_HUFF), from bl_count
  {
    uint32_t code = 0;
    sh.bl_count[0] = 0;
    for (int l = 1; l <= 15; l++) {
      code = (code + sh.bl_count[l - 1]) << 1;
      sh.next_code[l] = code;
    }
  }
}

#if HZ_GPU && HD_HUFF_REG
// Phases 1 and 3 on the GPU with the whole wave in lock step (round 5).  Lane 0 alone spent
// 45 % (phase 1) and 17 % (phase 3) of huff_kernel's time in dependent LDS round trips.
//
// Phase 1, the same two queues (leaves ascending, internal nodes in creation order) and the
// same tie rule as huff_parents_serial, but each queue's current 64-entry chunk sits in a
// register across the lanes, read by v_readlane and written by a lane select at wave-uniform
// indices: wl = the leaf weights of chunk leaf >> 6, iw = the internal weights being written
// (chunk next >> 6), ir = those of chunk root >> 6 once next has left it, pw = the parents of
// chunk root >> 6.  A chunk goes to LDS only when its cursor leaves it: internal weights into
// work[] (read back into ir), parents over them (their weights are dead by then), so work[]
// ends as huff_parents_serial leaves it for every node but the root.
__device__ __forceinline__ uint32_t rdl(uint32_t v, int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); }
__device__ __forceinline__ uint32_t wrl(uint32_t v, int i, uint32_t old) {
  return HZ_LANE_ID() == i ? v : old;
}
__device__ __forceinline__ void huff_parents_wave(HuffShared& sh, int n_) {
  const int lane = HZ_LANE_ID();
  const int n = __builtin_amdgcn_readfirstlane(n_);
  uint32_t* A = sh.work;
  auto leaf_chunk = [&](int c) -> uint32_t {
    const int i = 64 * c + lane;
    return i < n ? sh.keys[i] >> 9 : 0u;
  };
  uint32_t wl = leaf_chunk(0), iw = 0, ir = 0, pw = 0;
  iw = wrl(rdl(wl, 0) + rdl(wl, 1), 0, iw);
  int root = 0, leaf = 2;
  auto take_leaf = [&]() -> uint32_t {
    const uint32_t w = rdl(wl, leaf & 63);
    leaf++;
    if ((leaf & 63) == 0) wl = leaf_chunk(leaf >> 6);
    return w;
  };
  for (int next = 1; next < n - 1; next++) {
    if ((next & 63) == 0) {               // next leaves its chunk: keep it for root, store it
      if ((root >> 6) == (next >> 6) - 1) ir = iw;
      A[next - 64 + lane] = iw;
      iw = 0;
    }
    auto take_root = [&]() -> uint32_t {
      const uint32_t w = rdl((root >> 6) == (next >> 6) ? iw : ir, root & 63);
      pw = wrl((uint32_t)next, root & 63, pw);
      root++;
      if ((root & 63) == 0) {             // root leaves its chunk: its parents are final
        A[root - 64 + lane] = pw;
        if ((root >> 6) < (next >> 6)) ir = root + lane < NLL ? A[root + lane] : 0u;
      }
      return w;
    };
    const uint32_t iv1 = rdl((root >> 6) == (next >> 6) ? iw : ir, root & 63);
    const uint32_t lv1 = leaf < n ? rdl(wl, leaf & 63) : 0u;
    uint32_t w = (leaf >= n || iv1 < lv1) ? take_root() : take_leaf();
    const uint32_t iv2 = rdl((root >> 6) == (next >> 6) ? iw : ir, root & 63);
    const uint32_t lv2 = leaf < n ? rdl(wl, leaf & 63) : 0u;
    w += (leaf >= n || (root < next && iv2 < lv2)) ? take_root() : take_leaf();
    iw = wrl(w, next & 63, iw);
  }
  if (64 * (root >> 6) + lane < root) A[64 * (root >> 6) + lane] = pw;
}

// Phase 3 from a histogram: H[d] internal nodes at depth d (d >= 16 pooled) give
// bl_count[d] = 2 H[d - 1] - H[d] leaves (the serial walk's avbl - used), the pooled
// 2 H[15] + H[>= 16] at 16; then the fold onto maxbits, the Kraft fix-up and next_code as
// huff_counts_serial, with bl_count[l] in lane l.
__device__ __forceinline__ void huff_counts_wave(HuffShared& sh, int n_, int maxbits) {
  const int lane = HZ_LANE_ID();
  const int n = __builtin_amdgcn_readfirstlane(n_);
  const uint32_t* A = sh.work;
  uint32_t hv = 0;                        // H[lane] for lane <= 16
  uint32_t d[5];
  HZ_UNROLL for (int k = 0; k < 5; k++) {
    const int i = 64 * k + lane;
    d[k] = i < n - 1 ? (A[i] > 16u ? 16u : A[i]) : 99u;
  }
  HZ_UNROLL for (int k = 0; k < 5; k++) {
    if (64 * k >= n - 1) break;
    for (int t = 0; t <= 16; t++) {
      const uint32_t c = (uint32_t)__builtin_popcountll(__ballot(d[k] == (uint32_t)t));
      if (lane == t) hv += c;
    }
  }
  const uint32_t hprev = (uint32_t)__shfl_up((int)hv, 1, 64);
  uint32_t b = lane == 0 ? 0u : lane < 16 ? 2u * hprev - hv : lane == 16 ? 2u * hprev + hv : 0u;
  // fold the lengths above maxbits onto maxbits
  uint32_t over = lane > maxbits ? b : 0u;
  over = hz::wave_sum(over);
  if (lane > maxbits) b = 0;
  if (lane == maxbits) b += over;
  uint32_t kr = (lane >= 1 && lane <= maxbits) ? b << (maxbits - lane) : 0u;
  uint32_t total = __builtin_amdgcn_readfirstlane(hz::wave_sum(kr));
  while (total != (1u << maxbits)) {
    const uint64_t m = __ballot(lane >= 1 && lane < maxbits && b != 0u);
    const int l = m ? 63 - __builtin_clzll(m) : 0;
    if (lane == maxbits) b -= 1u;
    if (l && lane == l) b -= 1u;
    if (l && lane == l + 1) b += 2u;
    total--;
  }
  uint32_t code = 0, nc = 0;
  for (int l = 1; l <= 15; l++) {
    code = (code + (l > 1 ? rdl(b, l - 1) : 0u)) << 1;
    nc = wrl(code, l, nc);
  }
  if (lane <= 16) { sh.bl_count[lane] = b; sh.next_code[lane] = nc; }
}

// The code lengths and canonical codes with bl_count / next_code in registers: a symbol of
// rank r (from the most frequent) gets length 1 + #{l < 15 : bl_count[1] + .. + bl_count[l] <= r},
// the serial walk's result; codes by ballots per length as before, the running next_code[L]
// in lane L instead of one LDS read-modify-write per length.
__device__ __forceinline__ void huff_lens_wave(HuffShared& sh, int n_, uint8_t* lens) {
  const int lane = HZ_LANE_ID();
  const int n = __builtin_amdgcn_readfirstlane(n_);
  const uint32_t cum = hz::wave_incl_scan_dpp(lane <= 16 ? sh.bl_count[lane] : 0u);
  uint32_t cs[15];
  HZ_UNROLL for (int l = 1; l < 15; l++) cs[l] = rdl(cum, l);
  for (int i = lane; i < n; i += 64) {
    const uint32_t r = (uint32_t)(n - 1 - i);
    uint32_t len = 1;
    HZ_UNROLL for (int l = 1; l < 15; l++) len += cs[l] <= r ? 1u : 0u;
    lens[sh.keys[i] & 511u] = (uint8_t)len;
  }
}
__device__ __forceinline__ void huff_codes_wave(HuffShared& sh, int nsym, int maxbits, const uint8_t* lens,
                                                uint16_t* codes) {
  const int lane = HZ_LANE_ID();
  uint32_t ncv = lane <= 15 ? sh.next_code[lane] : 0u;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int c = 0; c < nsym; c += 64) {
    const uint32_t ln = c + lane < nsym ? (uint32_t)lens[c + lane] : 0u;
    uint32_t code = 0;
    for (int L = 1; L <= maxbits; L++) {
      const uint64_t m = __ballot(ln == (uint32_t)L);
      if (!m) continue;
      if (ln == (uint32_t)L) code = rev16(rdl(ncv, L) + hz::popc64(m & below), (uint32_t)L);
      if (lane == L) ncv += hz::popc64(m);
    }
    if (c + lane < nsym) codes[c + lane] = (uint16_t)code;
  }
}
#endif

#if HZ_GPU && HD_HUFF_REG
#define HD_HUFF_PARENTS(sh, NN) hd::huff_parents_wave(sh, NN)
#define HD_HUFF_COUNTS(sh, NN, MB) hd::huff_counts_wave(sh, NN, MB)
#define HD_HUFF_LENS(sh, LENS) hd::huff_lens_wave(sh, (int)(sh).cnt, LENS)
#define HD_HUFF_CODES(sh, N, MB, LENS, CODES) hd::huff_codes_wave(sh, N, MB, LENS, CODES)
#else
#define HD_HUFF_PARENTS(sh, NN) LANE_LOOP { if (lane == 0) hd::huff_parents_serial(sh, NN); }
#define HD_HUFF_COUNTS(sh, NN, MB) LANE_LOOP { if (lane == 0) hd::huff_counts_serial(sh, NN, MB); }
#define HD_HUFF_LENS(sh, LENS) HD_HUFF_LENS_SERIAL(sh, LENS)
#define HD_HUFF_CODES(sh, N, MB, LENS, CODES) HD_HUFF_CODES_SERIAL(sh, N, MB, LENS, CODES)
#endif
// cooperative Huffman build for FREQ[0..N) limited to MAXBITS (NP: power of two >= N)
#define HD_BUILD_HUFF(sh, FREQ, N, NP, MAXBITS, LENS, CODES)                                    \
  do {                                                                                          \
    LANE_LOOP { if (lane == 0) (sh).cnt = 0; }                                                  \
    WAVE_SYNC();                                                                                \
    LANE_LOOP {                                                                                 \
      uint32_t _c = 0;                                                                          \
      for (int _s = lane; _s < (N); _s += 64) { (LENS)[_s] = 0; _c += (FREQ)[_s] ? 1u : 0u; }  \
      if (_c) hd::lds_add(&(sh).cnt, _c);                                                       \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
    LANE_LOOP {                                                                                 \
      if (lane == 0 && (sh).cnt < 2u) {                                                         \
        /* zlib build_tree: force two codes so that one bit is always sent */                  \
        if (!(FREQ)[0]) { (FREQ)[0] = 1; (sh).cnt++; }                                          \
        if ((sh).cnt < 2u && !(FREQ)[1]) { (FREQ)[1] = 1; (sh).cnt++; }                         \
      }                                                                                         \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
    LANE_LOOP {                                                                                 \
      for (int _s = lane; _s < (NP); _s += 64)                                                  \
        (sh).keys[_s] = (_s < (N) && (FREQ)[_s]) ? (((FREQ)[_s] << 9) | (uint32_t)_s) : hd::KEY_NONE; \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
    for (int _x2 = 0; _x2 < ((HD_HUFF_X2 & 1) ? 2 : 1); _x2++)                                 \
    for (int _k = 2; _k <= (NP); _k <<= 1) {                                                    \
      for (int _j = _k >> 1; _j > 0; _j >>= 1) {                                                \
        LANE_LOOP {                                                                             \
          for (int _t = lane; _t < (NP) / 2; _t += 64) {                                        \
            const int _i = ((_t & ~(_j - 1)) << 1) | (_t & (_j - 1));                           \
            const int _l = _i | _j;                                                             \
            const uint32_t _a = (sh).keys[_i], _b = (sh).keys[_l];                              \
            if ((_a > _b) == ((_i & _k) == 0)) { (sh).keys[_i] = _b; (sh).keys[_l] = _a; }      \
          }                                                                                     \
        }                                                                                       \
        WAVE_SYNC();                                                                            \
      }                                                                                         \
    }                                                                                           \
    for (int _x2 = 0; _x2 < ((HD_HUFF_X2 & 2) ? 2 : 1); _x2++) {                               \
      HD_HUFF_PARENTS(sh, (int)(sh).cnt);                                                       \
      WAVE_SYNC();                                                                              \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
    HD_HUFF_DEPTHS(sh, (int)(sh).cnt);                                                          \
    for (int _x2 = 0; _x2 < ((HD_HUFF_X2 & 4) ? 2 : 1); _x2++) {                               \
      HD_HUFF_COUNTS(sh, (int)(sh).cnt, (MAXBITS));                                             \
      WAVE_SYNC();                                                                              \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
    /* lengths: the most frequent symbols (end of keys) get the shortest codes */              \
    HD_HUFF_LENS(sh, LENS);                                                                     \
    WAVE_SYNC();                                                                                \
    /* canonical codes: rank within a length by ballots, 64 symbols at a time */               \
    HD_HUFF_CODES(sh, N, MAXBITS, LENS, CODES);                                                 \
  } while (0)

// the serial forms (CPU emulation, HD_HUFF_REG=0) of huff_lens_wave / huff_codes_wave
#define HD_HUFF_LENS_SERIAL(sh, LENS)                                                           \
  do {                                                                                          \
    LANE_LOOP {                                                                                 \
      const int _n = (int)(sh).cnt;                                                             \
      for (int _i = lane; _i < _n; _i += 64) {                                                  \
        const uint32_t _r = (uint32_t)(_n - 1 - _i);                                            \
        uint32_t _l = 1, _acc = (sh).bl_count[1];                                               \
        while (_acc <= _r && _l < 15u) { _l++; _acc += (sh).bl_count[_l]; }                     \
        (LENS)[(sh).keys[_i] & 511u] = (uint8_t)_l;                                             \
      }                                                                                         \
    }                                                                                           \
  } while (0)
#define HD_HUFF_CODES_SERIAL(sh, N, MAXBITS, LENS, CODES)                                       \
  do {                                                                                          \
    for (int _c = 0; _c < (N); _c += 64) {                                                      \
      LANE_VAR(uint32_t, _ln);                                                                  \
      LANE_LOOP {                                                                               \
        LV(_ln) = _c + lane < (N) ? (uint32_t)(LENS)[_c + lane] : 0u;                           \
        if (_c + lane < (N)) (CODES)[_c + lane] = 0;                                            \
      }                                                                                         \
      for (uint32_t _L = 1; _L <= (uint32_t)(MAXBITS); _L++) {                                  \
        const uint64_t _m = WAVE_BALLOT(LV(_ln) == _L);                                         \
        if (!_m) continue;                                                                      \
        LANE_LOOP {                                                                             \
          if (LV(_ln) == _L) {                                                                  \
            const uint64_t _below = lane ? (_m & ((~0ull) >> (64 - lane))) : 0ull;              \
            (CODES)[_c + lane] = (uint16_t)hd::rev16((sh).next_code[_L] + hz::popc64(_below), _L); \
          }                                                                                     \
        }                                                                                       \
        WAVE_SYNC();                                                                            \
        LANE_LOOP { if (lane == 0) (sh).next_code[_L] += hz::popc64(_m); }                      \
        WAVE_SYNC();                                                                            \
      }                                                                                         \
    }                                                                                           \
  } while (0)


// ---- the code-length sequence (RFC 1951 3.2.7) of len_ll[0..hlit) ++ len_d[0..hdist), run-length
// coded with symbols 16/17/18, built by all lanes (a lane-0 loop through round 3) ----
// length i of the combined literal/length + distance sequence
HZ_HD uint32_t rle_len(const HuffShared& sh, uint32_t i, uint32_t hlit) {
  return i < hlit ? sh.len_ll[i] : sh.len_d[i - hlit];
}
// code-length symbols build_rle emits for a run of R copies of v
HZ_HD uint32_t rle_count(uint32_t v, uint32_t R) {
  if (v == 0u) {
    const uint32_t q = R / 138u, rem = R % 138u;
    return rem >= 11u ? q + 1u : q + (rem >= 3u ? 1u : rem);
  }
  const uint32_t rem = R - 1u, q = rem / 6u, rr = rem % 6u;
  return 1u + q + (rr >= 3u ? 1u : rr);
}
// the symbols of that run at rle[nr..], in build_rle's order, counted into clf
HZ_HD void rle_emit(HuffShared& sh, uint32_t v, uint32_t run, uint32_t nr) {
  if (v == 0u) {
    while (run >= 11u) {
      const uint32_t r = run > 138u ? 138u : run;
      sh.rle[nr++] = (uint16_t)(18u | ((r - 11u) << 8)); lds_add(&sh.clf[18], 1u);
      run -= r;
    }
    if (run >= 3u) { sh.rle[nr++] = (uint16_t)(17u | ((run - 3u) << 8)); lds_add(&sh.clf[17], 1u); run = 0; }
    while (run) { sh.rle[nr++] = 0; lds_add(&sh.clf[0], 1u); run--; }
  } else {
    sh.rle[nr++] = (uint16_t)v; lds_add(&sh.clf[v], 1u);
    run--;
    while (run >= 3u) {
      const uint32_t r = run > 6u ? 6u : run;
      sh.rle[nr++] = (uint16_t)(16u | ((r - 3u) << 8)); lds_add(&sh.clf[16], 1u);
      run -= r;
    }
    while (run) { sh.rle[nr++] = (uint16_t)v; lds_add(&sh.clf[v], 1u); run--; }
  }
}
// the first run start after position i (starts: bit i & 63 of sm[i >> 6]), or tot
HZ_HD uint32_t rle_next_start(const uint64_t* sm, uint32_t i, uint32_t tot) {
  const uint32_t k = i >> 6;
  uint64_t w = sm[k] & ~((2ull << (i & 63u)) - 1ull);
  if (w) return 64u * k + (uint32_t)__builtin_ctzll(w);
  for (uint32_t j = k + 1u; j < 5u; j++)
    if (sm[j]) return 64u * j + (uint32_t)__builtin_ctzll(sm[j]);
  return tot;
}
#if HZ_GPU
#define HD_WAVE_MAX(v, out)                                                                  \
  do {                                                                                       \
    uint32_t _m = (v);                                                                       \
    for (int _o = 32; _o > 0; _o >>= 1) { const uint32_t _y = __shfl_xor(_m, _o, 64); _m = _y > _m ? _y : _m; } \
    out = _m;                                                                                \
  } while (0)
#define HD_WAVE_SCAN(v, off, sum) do { off = hz::wave_excl_scan(v, (int)threadIdx.x); sum = hz::wave_sum(v); } while (0)
#else
#define HD_WAVE_MAX(v, out) do { out = 0; for (int _l = 0; _l < 64; _l++) out = (v)[_l] > out ? (v)[_l] : out; } while (0)
#define HD_WAVE_SCAN(v, off, sum) do { sum = 0; for (int _l = 0; _l < 64; _l++) { (off)[_l] = sum; sum += (v)[_l]; } } while (0)
#endif
// hlit / hdist (one past the last nonzero length), the run starts by ballot, each run's
// symbol count, a wave scan for the offsets, and each run's symbols by its starting lane
#define HD_BUILD_RLE(sh)                                                                     \
  do {                                                                                       \
    LANE_VAR(uint32_t, _hl);                                                                 \
    LANE_VAR(uint32_t, _hd);                                                                 \
    LANE_LOOP {                                                                              \
      uint32_t _a = 257u, _b = 1u;                                                           \
      for (int _s = lane; _s < NLL; _s += WAVE) if (_s >= 257 && (sh).len_ll[_s]) _a = (uint32_t)_s + 1u; \
      for (int _s = lane; _s < ND; _s += WAVE) if ((sh).len_d[_s]) _b = (uint32_t)_s + 1u;   \
      LV(_hl) = _a;                                                                          \
      LV(_hd) = _b;                                                                          \
      if (lane <= NCL) (sh).clf[lane] = 0;                                                   \
    }                                                                                        \
    uint32_t _hlit, _hdist;                                                                  \
    HD_WAVE_MAX(_hl, _hlit);                                                                 \
    HD_WAVE_MAX(_hd, _hdist);                                                                \
    WAVE_SYNC();                                                                             \
    const uint32_t _tot = _hlit + _hdist;                                                    \
    uint64_t _sm[5];                                                                         \
    for (uint32_t _k = 0; _k < 5u; _k++)                                                     \
      _sm[_k] = WAVE_BALLOT(64u * _k + (uint32_t)lane < _tot &&                              \
                            (64u * _k + (uint32_t)lane == 0u ||                              \
                             hd::rle_len((sh), 64u * _k + (uint32_t)lane, _hlit) !=          \
                                 hd::rle_len((sh), 64u * _k + (uint32_t)lane - 1u, _hlit))); \
    uint32_t _base = 0;                                                                      \
    for (uint32_t _k = 0; _k < 5u; _k++) {                                                   \
      LANE_VAR(uint32_t, _cn);                                                               \
      LANE_VAR(uint32_t, _rv);                                                               \
      LANE_VAR(uint32_t, _rr);                                                               \
      LANE_VAR(uint32_t, _of);                                                               \
      uint32_t _sum;                                                                         \
      LANE_LOOP {                                                                            \
        const uint32_t _i = 64u * _k + (uint32_t)lane;                                       \
        uint32_t _c = 0, _v = 0, _r = 0;                                                     \
        if ((_sm[_k] >> lane) & 1ull) {                                                      \
          _r = hd::rle_next_start(_sm, _i, _tot) - _i;                                       \
          _v = hd::rle_len((sh), _i, _hlit);                                                 \
          _c = hd::rle_count(_v, _r);                                                        \
        }                                                                                    \
        LV(_cn) = _c;                                                                        \
        LV(_rv) = _v;                                                                        \
        LV(_rr) = _r;                                                                        \
      }                                                                                      \
      HD_WAVE_SCAN(_cn, _of, _sum);                                                          \
      LANE_LOOP { if (LV(_cn)) hd::rle_emit((sh), LV(_rv), LV(_rr), _base + LV(_of)); }      \
      _base += _sum;                                                                         \
    }                                                                                        \
    LANE_LOOP { if (lane == 0) { (sh).nrle = _base; (sh).hlit = _hlit; (sh).hdist = _hdist; } } \
    WAVE_SYNC();                                                                             \
  } while (0)

// dynamic block header size in bits (after the code-length code is built): the run-length
// coded lengths summed by all lanes, HCLEN on lane 0
#define HD_HEADER_BITS(sh)                                                                   \
  do {                                                                                       \
    LANE_VAR(uint32_t, _hb);                                                                 \
    LANE_LOOP {                                                                              \
      uint32_t _b = 0;                                                                       \
      for (uint32_t _i = (uint32_t)lane; _i < (sh).nrle; _i += WAVE) {                       \
        const uint32_t _sym = (sh).rle[_i] & 0xffu;                                          \
        _b += (sh).len_cl[_sym] + cl_extra_bits(_sym);                                       \
      }                                                                                      \
      LV(_hb) = _b;                                                                          \
    }                                                                                        \
    uint32_t _tot;                                                                           \
    LANE_VAR(uint32_t, _ho);                                                                 \
    HD_WAVE_SCAN(_hb, _ho, _tot);                                                            \
    (void)_ho;                                                                               \
    LANE_LOOP {                                                                              \
      if (lane == 0) {                                                                       \
        uint32_t _hc = 4;                                                                    \
        for (uint32_t _i = 0; _i < (uint32_t)NCL; _i++) if ((sh).len_cl[hz::cl_order(_i)]) _hc = _i + 1 > 4u ? _i + 1 : 4u; \
        (sh).hclen = _hc;                                                                    \
        (sh).hdr_bits = 3u + 5u + 5u + 4u + 3u * _hc + _tot;                                 \
      }                                                                                      \
    }                                                                                        \
  } while (0)

// Worst-case bits of a stored block (3-bit header, up to 7 padding bits, LEN/NLEN)
HZ_HD uint64_t stored_bits_max(uint32_t seglen) { return 3u + 7u + 32u + 8ull * seglen; }

HZ_HD void huff_segment(HuffShared& sh, const SegParse* sp, SegCode* sc, uint32_t seglen, int stored_only) {
  LANE_LOOP {
    for (int s = lane; s < NSYM; s += WAVE) sh.freq[s] = sp->freq[s];
    if (lane == 0) { sh.freq[256] = 1; sh.nrle = 0; sh.hlit = 257; sh.hdist = 1; sh.hclen = 4; }
  }
  WAVE_SYNC();
  uint64_t dyn_bits = ~0ull, fix_bits = ~0ull;
  if (!stored_only) {
    // data bits of both codes from the true frequencies (before the >= 2-code patch)
    LANE_VAR(uint64_t, fb);
    LANE_LOOP {
      uint64_t f = 0;
      for (int s = lane; s < NSYM; s += WAVE) {
        const uint64_t c = sh.freq[s];
        if (!c) continue;
        if (s < NLL) f += c * (fixed_ll_len((uint32_t)s) + (s > 256 ? len_extra_bits((uint32_t)s - 257u) : 0u));
        else f += c * (5u + dist_extra_bits((uint32_t)(s - NLL)));
      }
      LV(fb) = f;
    }
#if HZ_GPU
    fix_bits = 3u + hz::wave_sum64(fb);
#else
    fix_bits = 3u;
    for (int l = 0; l < 64; l++) fix_bits += fb[l];
#endif
    HD_BUILD_HUFF(sh, sh.freq, NLL, 512, 15, sh.len_ll, sh.code_ll);
    HD_BUILD_HUFF(sh, (sh.freq + NLL), ND, 32, 15, sh.len_d, sh.code_d);
    HD_BUILD_RLE(sh);
    WAVE_SYNC();
    HD_BUILD_HUFF(sh, sh.clf, NCL, 32, 7, sh.len_cl, sh.code_cl);
    HD_HEADER_BITS(sh);
    WAVE_SYNC();
    LANE_VAR(uint64_t, db);
    LANE_LOOP {
      uint64_t d = 0;
      for (int s = lane; s < NSYM; s += WAVE) {
        const uint64_t c = sp->freq[s] + (s == 256 ? 1u : 0u);   // true counts, no phantom codes
        if (!c) continue;
        if (s < NLL) d += c * (sh.len_ll[s] + (s > 256 ? len_extra_bits((uint32_t)s - 257u) : 0u));
        else d += c * (sh.len_d[s - NLL] + dist_extra_bits((uint32_t)(s - NLL)));
      }
      LV(db) = d;
    }
#if HZ_GPU
    dyn_bits = sh.hdr_bits + hz::wave_sum64(db);
#else
    dyn_bits = sh.hdr_bits;
    for (int l = 0; l < 64; l++) dyn_bits += db[l];
#endif
  }
  const uint64_t st_bits = stored_bits_max(seglen);
  uint32_t btype;
  if (dyn_bits <= fix_bits && dyn_bits < st_bits) btype = 2;
  else if (fix_bits < st_bits) btype = 1;
  else btype = 0;
  LANE_LOOP {
    if (btype == 2) {
      for (int s = lane; s < NSYM; s += WAVE)
        sc->tab[s] = s < NLL ? ((uint32_t)sh.code_ll[s] << 4) | sh.len_ll[s]
                             : ((uint32_t)sh.code_d[s - NLL] << 4) | sh.len_d[s - NLL];
      if (lane <= NCL) sc->cl[lane] = lane < NCL ? ((uint32_t)sh.code_cl[lane] << 4) | sh.len_cl[lane] : 0u;
      for (int i = lane; i < (int)sh.nrle; i += WAVE) sc->rle[i] = sh.rle[i];
    } else if (btype == 1) {
      // fixed code (RFC 1951 3.2.6): canonical codes of the fixed lengths
      for (int s = lane; s < NSYM; s += WAVE) {
        uint32_t code, len;
        if (s < NLL) {
          len = fixed_ll_len((uint32_t)s);
          code = s < 144 ? 0x30u + (uint32_t)s : s < 256 ? 0x190u + (uint32_t)(s - 144)
                 : s < 280 ? (uint32_t)(s - 256) : 0xc0u + (uint32_t)(s - 280);
        } else {
          len = 5;
          code = (uint32_t)(s - NLL);
        }
        sc->tab[s] = (rev16(code, len) << 4) | len;
      }
    }
    if (lane == 0) {
      sc->btype = btype;
      sc->bits = btype == 2 ? (uint32_t)dyn_bits : btype == 1 ? (uint32_t)fix_bits : 0u;
      sc->nrle = sh.nrle;
      sc->hlit = sh.hlit;
      sc->hdist = sh.hdist;
      sc->hclen = sh.hclen;
    }
  }
  WAVE_SYNC_GLOBAL();
}

// Exact stream layout from the segment codes: relative bit position of every block
// (segbit[s], from the start of the zlib stream) and the stream size in bytes
// (2-byte header, blocks, byte padding, adler32).
HZ_HD uint64_t stream_layout(const SegCode* sc, uint32_t len, uint64_t* segbit) {
  const uint32_t nseg = nsegments(len);
  uint64_t b = 16;
  for (uint32_t s = 0; s < nseg; s++) {
    if (segbit) segbit[s] = b;
    const uint32_t s0 = s * (uint32_t)SEG;
    const uint32_t seglen = len - s0 < (uint32_t)SEG ? len - s0 : (uint32_t)SEG;
    if (sc[s].btype == 0) b = ((b + 3u + 7u) & ~7ull) + 32u + 8ull * seglen;
    else b += sc[s].bits;
  }
  b = (b + 7u) & ~7ull;
  return b / 8u + 4u;
}

// ============================================================================
// E: emission of one block at its bit position
// ============================================================================
struct EmitShared {
  uint32_t tab[NSYM];
  uint32_t cl[NCL + 1];
  uint16_t rle[NSYM];
  uint32_t stage[STAGE_WORDS];           // block bits starting at bit (bitpos & 31) of word 0
};

// serial bit writer into the staging words (one lane at a time)
struct BitW {
  uint64_t acc;
  uint32_t nacc;   // bits in acc
  uint32_t word;   // staging word acc starts at
};
HZ_HD void bw_init(BitW& w, uint32_t bitpos) { w.acc = 0; w.nacc = bitpos & 31u; w.word = bitpos >> 5; }
HZ_HD void bw_put(uint32_t* stage, BitW& w, uint32_t v, uint32_t n) {
  w.acc |= (uint64_t)v << w.nacc;
  w.nacc += n;
  if (w.nacc >= 32u) {
    lds_or(&stage[w.word], (uint32_t)w.acc);
    w.word++;
    w.acc >>= 32;
    w.nacc -= 32u;
  }
}
HZ_HD void bw_flush(uint32_t* stage, BitW& w) {
  if (w.nacc) lds_or(&stage[w.word], (uint32_t)w.acc);
}

// bits of one token (t: first slot, dv: distance slot of a match)
HZ_HD uint32_t tok_bits(const EmitShared& sh, uint32_t t, uint32_t dv) {
  if (!(t & 0x8000u)) return sh.tab[t] & 15u;
  uint32_t ls, eb, ev, ds, deb, dev;
  len_sym((t & 0x7fffu) + 3u, ls, eb, ev);
  dist_sym(dv + 1u, ds, deb, dev);
  return (sh.tab[257u + ls] & 15u) + eb + (sh.tab[NLL + ds] & 15u) + deb;
}

// f(t, dv) for each token of one lane's slots in order (t: the first slot, dv: the
// distance slot of a match, else 0).  The slot dwords are loaded 8 at a time, one memory
// latency per 16 slots instead of one per dependent load.
template <class F>
HZ_HD void walk_tokens(hz_gcu8* gtok, int lane, uint32_t ns, F&& f) {
  constexpr uint32_t NB = HD_WALKB;  // token dwords per batch of loads
  uint32_t mt = 0;                 // a match's first slot waiting for its distance slot
  const uint32_t nd = (ns + 1u) / 2u;
  for (uint32_t j0 = 0; j0 < nd; j0 += NB) {
    uint32_t d[NB];
    HZ_UNROLL
    for (uint32_t u = 0; u < NB; u++) {
      const uint32_t j = j0 + u;
      d[u] = j < nd ? *(hz_gcu32*)(gtok + (size_t)(j * (uint32_t)WAVE + (uint32_t)lane) * 4u) : 0u;
    }
    HZ_UNROLL
    for (uint32_t u = 0; u < 2u * NB; u++) {
      if (2u * j0 + u < ns) {
        const uint32_t v = (u & 1u) ? d[u >> 1] >> 16 : d[u >> 1] & 0xffffu;
        const bool call = mt || !(v & 0x8000u);
        const uint32_t ft = mt ? mt : v, fd = mt ? v : 0u;
        mt = mt ? 0u : (v & 0x8000u) ? v : 0u;
        if (call) f(ft, fd);
      }
    }
  }
}

// dst: the destination buffer as 32-bit words (bit positions are relative to it).
// The first and the last word touched are shared with neighbours: atomic OR into
// words the layout phase zeroed; every other word is owned and stored whole.
HZ_HD void emit_segment(EmitShared& sh, const SegOut& so, const SegCode* sc, const SegParse* sp,
                        const uint16_t* tok, const EncJob& job, uint32_t* dst) {
  const uint32_t s0 = so.seg * (uint32_t)SEG;
  const uint32_t seglen = job.len - s0 < (uint32_t)SEG ? job.len - s0 : (uint32_t)SEG;
  const uint32_t last = (so.flags >> 1) & 1u;
  const uint32_t btype = sc->btype;
  const uint32_t off0 = (uint32_t)(so.bitpos & 31u);
  hz_gcu8* const gtok = HZ_GLOBAL(hz_gcu8*, tok);
  LANE_LOOP {
    for (int w = lane; w < STAGE_WORDS; w += WAVE) sh.stage[w] = 0;
    if (btype) for (int s = lane; s < NSYM; s += WAVE) sh.tab[s] = sc->tab[s];
    if (btype == 2) {
      if (lane <= NCL) sh.cl[lane] = sc->cl[lane];
      for (int i = lane; i < (int)sc->nrle; i += WAVE) sh.rle[i] = sc->rle[i];
    }
  }
  WAVE_SYNC();
  uint32_t total;   // bits in the staging words, from bit 0 of word 0
  if (btype == 0) {
    const uint32_t b0 = (off0 + 3u + 7u) >> 3;      // byte of LEN after the padded header
    LANE_LOOP {
      if (lane == 0) {
        BitW w;
        bw_init(w, off0);
        bw_put(sh.stage, w, last, 3);
        bw_flush(sh.stage, w);
      }
      uint8_t* sb = (uint8_t*)sh.stage;
      if (lane < 4) {
        const uint32_t v = (lane < 2) ? seglen : (~seglen & 0xffffu);
        sb[b0 + (uint32_t)lane] = (uint8_t)((lane & 1) ? (v >> 8) : v);
      }
      const uint32_t nw = (seglen + 3u) / 4u;
      for (uint32_t k = (uint32_t)lane; k < nw; k += WAVE) {
        const uint32_t v = load_stream_word(job, s0 + 4u * k, s0 + seglen);
        for (uint32_t b = 0; b < 4u && 4u * k + b < seglen; b++) sb[b0 + 4u + 4u * k + b] = (uint8_t)(v >> (8u * b));
      }
    }
    total = (b0 + 4u + seglen) * 8u;
  } else {
    LANE_VAR(uint32_t, nb);
    LANE_VAR(uint32_t, hb);
    // block header: 3 bits, and for a dynamic block HLIT / HDIST / HCLEN, the code-length
    // code lengths (3 bits each) and the run-length coded code lengths -- written by all
    // lanes at their bit offsets (a serial lane-0 writer spent ~300 LDS atomics per block)
    uint32_t hbits_all = 3;
    LANE_LOOP {
      if (lane == 0) {
        BitW w;
        bw_init(w, off0);
        bw_put(sh.stage, w, last | (btype << 1), 3);
        if (btype == 2) {
          bw_put(sh.stage, w, sc->hlit - 257u, 5);
          bw_put(sh.stage, w, sc->hdist - 1u, 5);
          bw_put(sh.stage, w, sc->hclen - 4u, 4);
        }
        bw_flush(sh.stage, w);
      }
      if (btype == 2 && (uint32_t)lane < sc->hclen) {
        BitW w;
        bw_init(w, off0 + 17u + 3u * (uint32_t)lane);
        bw_put(sh.stage, w, sh.cl[hz::cl_order((uint32_t)lane)] & 15u, 3);
        bw_flush(sh.stage, w);
      }
    }
    if (btype == 2) {
      uint32_t base = off0 + 17u + 3u * sc->hclen;
      const uint32_t nrle = sc->nrle;
      for (uint32_t c0 = 0; c0 < nrle; c0 += WAVE) {
        LANE_VAR(uint32_t, rb);
        LANE_LOOP {
          const uint32_t i = c0 + (uint32_t)lane;
          uint32_t b = 0;
          if (i < nrle) {
            const uint32_t e = sh.rle[i];
            b = (sh.cl[e & 0xffu] & 15u) + cl_extra_bits(e & 0xffu);
          }
          LV(rb) = b;
        }
        LANE_VAR(uint32_t, ro);
        uint32_t chunk_bits;
#if HZ_GPU
        ro = hz::wave_excl_scan(rb, (int)threadIdx.x);
        chunk_bits = hz::wave_sum(rb);
#else
        chunk_bits = 0;
        for (int l = 0; l < 64; l++) { ro[l] = chunk_bits; chunk_bits += rb[l]; }
#endif
        LANE_LOOP {
          const uint32_t i = c0 + (uint32_t)lane;
          if (i < nrle) {
            const uint32_t e = sh.rle[i];
            const uint32_t sym = e & 0xffu;
            const uint32_t c = sh.cl[sym];
            BitW w;
            bw_init(w, base + LV(ro));
            bw_put(sh.stage, w, c >> 4, c & 15u);
            const uint32_t xb = cl_extra_bits(sym);
            if (xb) bw_put(sh.stage, w, e >> 8, xb);
            bw_flush(sh.stage, w);
          }
        }
        base += chunk_bits;
      }
      hbits_all = base - off0;
    }
    LANE_LOOP {
      LV(hb) = lane == 0 ? hbits_all : 0u;
      // pass 1: bits of this lane's tokens
      uint32_t bits = 0;
      walk_tokens(gtok, lane, sp->nslot[lane], [&](uint32_t t, uint32_t dv) { bits += tok_bits(sh, t, dv); });
      if (lane == WAVE - 1) bits += sh.tab[256] & 15u;
      LV(nb) = bits;
    }
    WAVE_SYNC();
    LANE_VAR(uint32_t, off);
    uint32_t hdr_bits;
#if HZ_GPU
    hdr_bits = __shfl(hb, 0, 64);
    off = hz::wave_excl_scan(nb, (int)threadIdx.x);
    const uint32_t sum_bits = hz::wave_sum(nb);
#else
    hdr_bits = hb[0];
    uint32_t sum_bits = 0;
    for (int l = 0; l < 64; l++) { off[l] = sum_bits; sum_bits += nb[l]; }
#endif
    // pass 2: write
    LANE_LOOP {
      BitW w;
      bw_init(w, off0 + hdr_bits + LV(off));
      walk_tokens(gtok, lane, sp->nslot[lane], [&](uint32_t t, uint32_t dv) {
        if (t & 0x8000u) {
          uint32_t ls, eb, ev, ds, deb, dev;
          len_sym((t & 0x7fffu) + 3u, ls, eb, ev);
          dist_sym(dv + 1u, ds, deb, dev);
          const uint32_t cl = sh.tab[257u + ls], cd = sh.tab[NLL + ds];
          // code + extra bits in one put each (<= 20 and <= 28 bits)
          bw_put(sh.stage, w, (cl >> 4) | (ev << (cl & 15u)), (cl & 15u) + eb);
          bw_put(sh.stage, w, (cd >> 4) | (dev << (cd & 15u)), (cd & 15u) + deb);
        } else {
          const uint32_t c = sh.tab[t];
          bw_put(sh.stage, w, c >> 4, c & 15u);
        }
      });
      if (lane == WAVE - 1) bw_put(sh.stage, w, sh.tab[256] >> 4, sh.tab[256] & 15u);
      bw_flush(sh.stage, w);
    }
    total = off0 + hdr_bits + sum_bits;
  }
  WAVE_SYNC();
  if (last) {   // byte padding, then adler32 big-endian
    total = (total + 7u) & ~7u;
    LANE_LOOP {
      if (lane < 4) {
        uint8_t* sb = (uint8_t*)sh.stage;
        sb[total / 8u + (uint32_t)lane] = (uint8_t)(so.adler >> (24 - 8 * lane));
      }
    }
    total += 32u;
    WAVE_SYNC();
  }
  // store: words [w0, w0 + nw) of dst; the first and the last by atomic OR
  const uint64_t w0 = so.bitpos >> 5;
  const uint32_t nw = (total + 31u) / 32u;
  hz_gu32* const gd = HZ_GLOBAL(hz_gu32*, dst + w0);
  LANE_LOOP {
    for (uint32_t k = (uint32_t)lane; k < nw; k += WAVE) {
      const uint32_t v = sh.stage[k];
      if (k == 0 || k == nw - 1u) glb_or(dst + w0 + k, v);
      else gd[k] = v;
    }
  }
  WAVE_SYNC_GLOBAL();
}

}  // namespace hd
