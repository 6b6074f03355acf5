// deflate_wave.h -- one-wavefront-per-stream zlib (RFC 1950/1951) encoder.
//
// Replaces, for the HSDS data-node write path, the zlib deflate that the reference
// reaches through storUtil._compress (hsds/util/storUtil.py:238-281):
// numcodecs Blosc(cname="zlib", clevel, shuffle).encode -> c-blosc 1.21
// zlib_wrap_compress -> compress2(level) once per Blosc split.  The compressed bytes
// need not equal libz's (any valid deflate is accepted); the
// stream must inflate to the input through libz, c-blosc and the reference's
// _uncompress, and its size should stay within a few percent of zlib's level.
//
// Algorithm (DESIGN.md "Deflate encoder"):
//   The stream is cut into segments of SEG input bytes; each segment becomes one
//   deflate block (dynamic Huffman, fixed Huffman or stored, whichever is
//   smallest).  Matches may reach WIN bytes behind the segment start, which an LDS
//   input ring holds.  Per segment:
//   1. Hash chains, exact: positions are inserted 64 at a time; the 64 (hash, lane)
//      keys are bitonic-sorted across the wave, so every position learns its true
//      predecessor with the same 3-byte hash (an earlier lane of the same group or
//      the head table) and the last position of every hash run updates the head.
//   2. LZ77 parse, lane-parallel: lane l owns an equal 1/64 share of the segment and
//      parses it greedily (chain depth and nice length from the level), matches
//      truncated at its share's end.  Tokens go to LDS as 16-bit slots, symbol
//      frequencies to LDS counters.
//   3. Huffman code lengths: symbols bitonic-sorted by frequency in LDS, then the
//      in-place minimum-redundancy algorithm (Moffat & Katajainen) and Kraft-exact
//      length limiting to 15 (7 for the code-length code), canonical codes.
//   4. Emission: every lane counts its tokens' bits, a wave prefix sum places them,
//      every lane ORs its bits into an LDS staging buffer, full words are flushed
//      to the output with coalesced stores and the partial word carries over.
//   adler32 is accumulated per lane as (sum b, sum pos*b) and combined once.
//
// SINGLE SOURCE for two drivers exactly like inflate_wave.h: the HIP kernel
// (engine.hip) and the CPU emulation (tests/emu/deflate_emu.cpp, test only).
#pragma once
#include "inflate_wave.h"

namespace hd {

constexpr int WAVE = 64;
constexpr int SEG = 8192;                   // input bytes per deflate block
constexpr int RING = 2 * SEG;               // LDS input ring: window + current segment
constexpr uint32_t RMASK = RING - 1;
constexpr int RWORDS = RING / 4;
constexpr int LOOK = 4;                     // bytes staged past the segment end (hashes)
constexpr uint32_t WIN = SEG - 2 * LOOK;    // farthest match source before the segment
constexpr int HBITS = 12;
constexpr int HSIZE = 1 << HBITS;
constexpr int LANE_MAX = SEG / WAVE;        // input bytes per lane (a full segment)
constexpr int TSLOTS = LANE_MAX;            // 16-bit token slots per lane
constexpr int STAGE_WORDS = SEG / 4 + 16;   // a block is never emitted above its stored size
constexpr int NLL = 286, ND = 30, NCL = 19;
constexpr int NSYM = NLL + ND;
constexpr uint32_t ADLER_MOD = 65521;
constexpr uint32_t KEY_NONE = 0xffffffffu;

// result codes of deflate_stream (>= 0: compressed bytes)
constexpr int64_t R_OVERFLOW = -1;          // output would exceed the capacity

struct Tune {
  uint32_t chain;    // hash-chain candidates tried per position
  uint32_t nice;     // stop searching at this match length
  uint32_t too_far;  // length-3 matches farther than this are not taken (zlib TOO_FAR)
  uint32_t stored;   // 1: level 0, stored blocks only
};

HZ_HD Tune tune_for_level(int level) {
  Tune t;
  t.too_far = 4096;
  t.stored = level <= 0 ? 1u : 0u;
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
HZ_HD uint32_t rev16(uint32_t code, uint32_t len) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < len; i++) { r = (r << 1) | (code & 1u); code >>= 1; }
  return r;
}

struct Shared {
  uint32_t ring[RWORDS];                 // input bytes, position p at byte p & RMASK
  uint16_t prev[SEG];                    // (predecessor position) & 0xffff per segment position
  uint16_t head[HSIZE];                  // (latest position) & 0xffff per hash
  uint32_t tokw[TSLOTS / 2 * WAVE];      // 16-bit token slots, lane-interleaved pairs
  uint32_t stage[STAGE_WORDS];           // output bits of the block being emitted
  uint32_t freq[NSYM];                   // literal/length 0..285 | distance 286..315
  uint32_t clf[NCL + 1];                 // code-length code frequencies
  uint32_t keys[512];                    // sort scratch (freq << 9 | symbol)
  uint32_t work[NLL];                    // minimum-redundancy scratch
  uint8_t len_ll[NLL + 2];
  uint8_t len_d[ND + 2];
  uint8_t len_cl[NCL + 1];
  uint16_t code_ll[NLL];
  uint16_t code_d[ND];
  uint16_t code_cl[NCL + 1];
  uint16_t rle[NSYM];                    // code-length sequence: symbol | extra << 8
  uint32_t nrle, hlit, hdist, hclen, hdr_bits, cnt;
  uint32_t btype;                        // 0 stored, 1 fixed, 2 dynamic
  uint32_t bl_count[17];
  uint32_t next_code[17];
};

// token slot s of lane `lane` (u16), pairs of a lane share one dword
HZ_HD uint32_t tslot(uint32_t s, int lane) { return ((s >> 1) * (uint32_t)WAVE + (uint32_t)lane) * 2u + (s & 1u); }
HZ_HD uint32_t tok_get(const Shared& sh, uint32_t s, int lane) {
  return ((const uint16_t*)sh.tokw)[tslot(s, lane)];
}
HZ_HD void tok_put(Shared& sh, uint32_t s, int lane, uint32_t v) {
  ((uint16_t*)sh.tokw)[tslot(s, lane)] = (uint16_t)v;
}

// 4 input bytes at stream position p (little-endian), ring wrap-around included
HZ_HD uint32_t rd32(const Shared& sh, uint32_t p) {
  const uint32_t w = (p >> 2) & (uint32_t)(RWORDS - 1);
  const uint32_t a = sh.ring[w];
  const uint32_t b = sh.ring[(w + 1u) & (uint32_t)(RWORDS - 1)];
  const uint32_t s = (p & 3u) * 8u;
  return s ? (a >> s) | (b << (32u - s)) : a;
}
HZ_HD uint32_t rd8(const Shared& sh, uint32_t p) {
  return (sh.ring[(p >> 2) & (uint32_t)(RWORDS - 1)] >> ((p & 3u) * 8u)) & 0xffu;
}
HZ_HD uint32_t hash3(uint32_t w) { return ((w & 0xffffffu) * 0x9E3779B1u) >> (32 - HBITS); }

HZ_HD uint32_t match_len(const Shared& sh, uint32_t q, uint32_t p, uint32_t maxl) {
  uint32_t L = 0;
  while (L < maxl) {
    const uint32_t x = rd32(sh, q + L) ^ rd32(sh, p + L);
    if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
    L += 4u;
  }
  return L < maxl ? L : maxl;
}

HZ_HD void lds_add(uint32_t* p, uint32_t v) {
#if HZ_GPU
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
HZ_HD void lds_or(uint32_t* p, uint32_t v) {
#if HZ_GPU
  atomicOr(p, v);
#else
  *p |= v;
#endif
}

// serial bit writer into the staging words (one lane at a time)
struct BitW {
  uint64_t acc;
  uint32_t nacc;   // bits in acc
  uint32_t word;   // staging word acc starts at
};
HZ_HD void bw_init(BitW& w, uint32_t bitpos) { w.acc = 0; w.nacc = bitpos & 31u; w.word = bitpos >> 5; }
HZ_HD void bw_put(Shared& sh, BitW& w, uint32_t v, uint32_t n) {
  w.acc |= (uint64_t)v << w.nacc;
  w.nacc += n;
  if (w.nacc >= 32u) {
    lds_or(&sh.stage[w.word], (uint32_t)w.acc);
    w.word++;
    w.acc >>= 32;
    w.nacc -= 32u;
  }
}
HZ_HD void bw_flush(Shared& sh, BitW& w) {
  if (w.nacc) lds_or(&sh.stage[w.word], (uint32_t)w.acc);
}

}  // namespace hd

// ---- wave-collective helpers for the encoder ---------------------------------
#if HZ_GPU
namespace hd {
__device__ __forceinline__ uint32_t wave_sort64(uint32_t key, int lane) {
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t o = __shfl_xor(key, j, 64);
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
#define HD_WAVE_SUM64(v) hz::wave_sum64(v)
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

struct EncJob {
  const uint8_t* src;   // stream input (any alignment); with ts > 1 the Blosc block base
  uint32_t len;         // input bytes
  uint32_t* dst;        // output, 4-byte aligned, cap + 8 bytes writable
  uint32_t cap;         // max output bytes
  int level;
  uint32_t ts;          // > 1: the stream is bytes [off, off + len) of the byte-shuffled block
  uint32_t neb;         //      (c-blosc shuffle: plane-major, neb elements per plane, tail as-is)
  uint32_t off;
};

// byte k of a byte-shuffled Blosc block (c-blosc shuffle(): plane j holds byte j of
// every element; the bs % ts tail bytes follow unchanged)
HZ_HD uint32_t shuffled_src_index(uint32_t k, uint32_t ts, uint32_t neb) {
  return k < neb * ts ? (k % neb) * ts + k / neb : k;
}

// ---------------------------------------------------------------------------
// Huffman code lengths for freq[0..n) limited to maxbits, written to lens[], and
// bit-reversed canonical codes to codes[].  Cooperative (all lanes call it).  At
// least two symbols get a code (zlib build_tree's rule), so every code is complete.
// ---------------------------------------------------------------------------
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
    LANE_LOOP {                                                                                 \
      if (lane == 0) hd::huff_lengths_serial(sh, (int)(sh).cnt, (MAXBITS), (LENS), (CODES), (N)); \
    }                                                                                           \
    WAVE_SYNC();                                                                                \
  } while (0)

// Serial part of the Huffman build (lane 0): keys[0..n) are sorted ascending by
// (frequency, symbol).  Minimum-redundancy lengths in place (Moffat & Katajainen
// 1995), Kraft-exact limiting to maxbits, lengths assigned longest-first to the
// least frequent symbols, then canonical codes (RFC 1951 3.2.2), bit-reversed.
HZ_HD void huff_lengths_serial(Shared& sh, int n, int maxbits, uint8_t* lens, uint16_t* codes, int nsym) {
  uint32_t* A = sh.work;
  for (int i = 0; i < n; i++) A[i] = sh.keys[i] >> 9;
  for (int l = 0; l <= 16; l++) sh.bl_count[l] = 0;
  // phase 1: parents, left to right
  A[0] += A[1];
  int root = 0, leaf = 2;
  for (int next = 1; next < n - 1; next++) {
    if (leaf >= n || A[root] < A[leaf]) { A[next] = A[root]; A[root++] = (uint32_t)next; }
    else A[next] = A[leaf++];
    if (leaf >= n || (root < next && A[root] < A[leaf])) { A[next] += A[root]; A[root++] = (uint32_t)next; }
    else A[next] += A[leaf++];
  }
  // phase 2: internal node depths, right to left
  A[n - 2] = 0;
  for (int next = n - 3; next >= 0; next--) A[next] = A[A[next]] + 1u;
  // phase 3: leaf depths -> counts per length
  {
    int avbl = 1, used = 0, dpth = 0;
    root = n - 2;
    int next = n - 1;
    while (avbl > 0) {
      while (root >= 0 && (int)A[root] == dpth) { used++; root--; }
      while (avbl > used) {
        sh.bl_count[dpth > 16 ? 16 : dpth]++;
        (void)next; next--;
        avbl--;
      }
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
  // lengths: the most frequent symbols (end of keys) get the shortest codes
  {
    int j = n;
    for (int l = 1; l <= maxbits; l++) {
      for (uint32_t c = sh.bl_count[l]; c > 0; c--) lens[sh.keys[--j] & 511u] = (uint8_t)l;
    }
  }
  // canonical codes
  {
    uint32_t code = 0;
    sh.bl_count[0] = 0;
    for (int l = 1; l <= 15; l++) {
      code = (code + sh.bl_count[l - 1]) << 1;
      sh.next_code[l] = code;
    }
    for (int s = 0; s < nsym; s++) {
      const uint32_t l = lens[s];
      codes[s] = l ? (uint16_t)rev16(sh.next_code[l]++, l) : (uint16_t)0;
    }
  }
}

HZ_HD void set_fixed_codes(Shared& sh) {
  for (int l = 0; l <= 16; l++) sh.bl_count[l] = 0;
  for (uint32_t s = 0; s < 288u; s++) sh.bl_count[fixed_ll_len(s)]++;
  uint32_t code = 0;
  sh.bl_count[0] = 0;
  for (int l = 1; l <= 15; l++) { code = (code + sh.bl_count[l - 1]) << 1; sh.next_code[l] = code; }
  for (uint32_t s = 0; s < (uint32_t)NLL; s++) {
    const uint32_t l = fixed_ll_len(s);
    sh.len_ll[s] = (uint8_t)l;
    sh.code_ll[s] = (uint16_t)rev16(sh.next_code[l]++, l);
  }
  for (uint32_t s = 0; s < (uint32_t)ND; s++) { sh.len_d[s] = 5; sh.code_d[s] = (uint16_t)rev16(s, 5); }
}

// code-length sequence (RFC 1951 3.2.7) of len_ll[0..hlit) ++ len_d[0..hdist),
// run-length coded with symbols 16/17/18; lane 0
HZ_HD void build_rle(Shared& sh) {
  uint32_t hlit = 257, hdist = 1;
  for (uint32_t s = 257; s < (uint32_t)NLL; s++) if (sh.len_ll[s]) hlit = s + 1;
  for (uint32_t s = 0; s < (uint32_t)ND; s++) if (sh.len_d[s]) hdist = s + 1;
  sh.hlit = hlit;
  sh.hdist = hdist;
  for (int i = 0; i <= NCL; i++) sh.clf[i] = 0;
  const uint32_t total = hlit + hdist;
  uint32_t nr = 0, i = 0;
  while (i < total) {
    const uint32_t v = i < hlit ? sh.len_ll[i] : sh.len_d[i - hlit];
    uint32_t run = 1;
    while (i + run < total && (i + run < hlit ? sh.len_ll[i + run] : sh.len_d[i + run - hlit]) == v) run++;
    i += run;
    if (v == 0) {
      while (run >= 11u) {
        const uint32_t r = run > 138u ? 138u : run;
        sh.rle[nr++] = (uint16_t)(18u | ((r - 11u) << 8)); sh.clf[18]++;
        run -= r;
      }
      if (run >= 3u) { sh.rle[nr++] = (uint16_t)(17u | ((run - 3u) << 8)); sh.clf[17]++; run = 0; }
      while (run) { sh.rle[nr++] = 0; sh.clf[0]++; run--; }
    } else {
      sh.rle[nr++] = (uint16_t)v; sh.clf[v]++;
      run--;
      while (run >= 3u) {
        const uint32_t r = run > 6u ? 6u : run;
        sh.rle[nr++] = (uint16_t)(16u | ((r - 3u) << 8)); sh.clf[16]++;
        run -= r;
      }
      while (run) { sh.rle[nr++] = (uint16_t)v; sh.clf[v]++; run--; }
    }
  }
  sh.nrle = nr;
}

HZ_HD uint32_t cl_extra_bits(uint32_t sym) { return sym == 16u ? 2u : sym == 17u ? 3u : sym == 18u ? 7u : 0u; }

// dynamic block header size in bits (after the code-length code is built); lane 0
HZ_HD uint32_t dyn_header_bits(Shared& sh) {
  uint32_t hclen = 4;
  for (uint32_t i = 0; i < (uint32_t)NCL; i++) if (sh.len_cl[hz::cl_order(i)]) hclen = i + 1 > 4u ? i + 1 : 4u;
  sh.hclen = hclen;
  uint32_t bits = 3u + 5u + 5u + 4u + 3u * hclen;
  for (uint32_t i = 0; i < sh.nrle; i++) {
    const uint32_t sym = sh.rle[i] & 0xffu;
    bits += sh.len_cl[sym] + cl_extra_bits(sym);
  }
  return bits;
}

// ---------------------------------------------------------------------------
// one zlib stream.  Returns compressed bytes, or R_OVERFLOW when the output would
// exceed job.cap (the caller then stores the input raw, as c-blosc does).
// ---------------------------------------------------------------------------
HZ_HD int64_t deflate_stream(Shared& sh, const EncJob& job, const Tune& tune, HzProf* prof = nullptr) {
  (void)prof;
  const uint32_t n = job.len;
  hz_gcu8* const gsrc = HZ_GLOBAL(hz_gcu8*, (uintptr_t)job.src & ~(uintptr_t)3);
  const uint32_t sa = (uint32_t)((uintptr_t)job.src & 3u);
  hz_gu32* const gdst = HZ_GLOBAL(hz_gu32*, job.dst);
  const uint32_t nseg = n ? (n + SEG - 1) / SEG : 1u;

  LANE_VAR(uint64_t, as1);           // adler partial sums: S1 = sum b, S2 = sum pos * b
  LANE_VAR(uint64_t, as2);
  LANE_LOOP {
    LV(as1) = 0; LV(as2) = 0;
    for (int h = lane; h < HSIZE; h += WAVE) sh.head[h] = 0xffffu;
  }
  uint32_t carry = 0x78u | (zlib_flg(job.level) << 8);   // zlib header
  uint32_t carry_bits = 16;
  uint32_t out_words = 0;
  bool overflow = false;
  WAVE_SYNC();

  for (uint32_t seg = 0; seg < nseg && !overflow; seg++) {
    const uint32_t s0 = seg * (uint32_t)SEG;
    const uint32_t s1 = s0 + (uint32_t)SEG < n ? s0 + (uint32_t)SEG : n;
    const uint32_t seglen = s1 - s0;
    const uint32_t stage_hi = s1 + (uint32_t)LOOK < n ? s1 + (uint32_t)LOOK : n;
    const bool last = seg + 1 == nseg;

    // ---- 1. stage the segment (+ lookahead) into the ring, adler sums ----
    HZ_T(1);
    LANE_LOOP {
      const uint32_t nw = (stage_hi - s0 + 3u) / 4u;
      for (uint32_t k = (uint32_t)lane; k < nw; k += WAVE) {
        const uint32_t p = s0 + 4u * k;             // stream position of ring word
        uint32_t v = 0;
        if (job.ts > 1u) {                          // gather from the unshuffled block
          hz_gcu8* const bsrc = HZ_GLOBAL(hz_gcu8*, job.src);
          for (uint32_t b = 0; b < 4u; b++)
            if (p + b < stage_hi) v |= (uint32_t)bsrc[shuffled_src_index(job.off + p + b, job.ts, job.neb)] << (8u * b);
        } else {
          const uint32_t a = p + sa;                  // byte offset from the aligned base
          const uint32_t lo = sa, hi = sa + stage_hi; // valid bytes [lo, hi) of the aligned base
          const uint32_t w0 = hz::load_word(gsrc, a >> 2, lo, hi);
          v = w0;
          if (a & 3u) {
            const uint32_t w1 = hz::load_word(gsrc, (a >> 2) + 1u, lo, hi);
            const uint32_t s = (a & 3u) * 8u;
            v = (w0 >> s) | (w1 << (32u - s));
          }
        }
        sh.ring[(p >> 2) & (uint32_t)(RWORDS - 1)] = v;
        for (uint32_t b = 0; b < 4u; b++) {
          const uint32_t q = p + b;
          if (q < s1) {
            const uint32_t byte = (v >> (8u * b)) & 0xffu;
            LV(as1) += byte;
            LV(as2) += (uint64_t)q * byte;
          }
        }
      }
      for (int s = lane; s < NSYM; s += WAVE) sh.freq[s] = 0;
    }
    WAVE_SYNC();

    const uint32_t lo_pos = s0 > WIN ? s0 - WIN : 0u;   // farthest match source
    if (!tune.stored) {
      // ---- 2. exact hash chains, 64 positions per step ----
      HZ_T(2);
      for (uint32_t g = s0; g < s1; g += WAVE) {
        LANE_VAR(uint32_t, key);
        LANE_VAR(uint32_t, kp);
        LANE_VAR(uint32_t, kn);
        LANE_LOOP {
          const uint32_t p = g + (uint32_t)lane;
          LV(key) = KEY_NONE;
          if (p < s1 && p + 2u < n) LV(key) = (hash3(rd32(sh, p)) << 6) | (uint32_t)lane;
        }
        HD_SORT64(key);
        HD_NEIGHBOURS(kp, kn, key);
        LANE_LOOP {
          const uint32_t k = LV(key);
          if (k != KEY_NONE) {
            const uint32_t h = k >> 6;
            const uint32_t pos = g + (k & 63u);
            const uint32_t pk = LV(kp);
            const uint32_t pv = (pk != KEY_NONE && (pk >> 6) == h) ? ((g + (pk & 63u)) & 0xffffu) : sh.head[h];
            sh.prev[pos - s0] = (uint16_t)pv;
          }
        }
        WAVE_SYNC();
        LANE_LOOP {
          const uint32_t k = LV(key), nk = LV(kn);
          if (k != KEY_NONE && (nk == KEY_NONE || (nk >> 6) != (k >> 6)))
            sh.head[k >> 6] = (uint16_t)((g + (k & 63u)) & 0xffffu);
        }
        WAVE_SYNC();
      }
    }

    // ---- 3. lane-parallel greedy parse ----
    HZ_T(3);
    LANE_VAR(uint32_t, nslot);
    LANE_LOOP {
      const uint32_t R = (seglen + WAVE - 1) / WAVE;
      const uint32_t a0 = (uint32_t)lane * R < seglen ? (uint32_t)lane * R : seglen;
      const uint32_t a1 = a0 + R < seglen ? a0 + R : seglen;
      uint32_t pos = s0 + a0;
      const uint32_t end = s0 + a1;
      uint32_t ns = 0;
      if (!tune.stored) {
        while (pos < end) {
          uint32_t best = 0, bd = 0;
          const uint32_t maxl = end - pos < 258u ? end - pos : 258u;
          if (maxl >= 3u) {
            uint32_t c16 = sh.prev[pos - s0];
            for (uint32_t depth = 0; depth < tune.chain; depth++) {
              const uint32_t d = (pos - c16) & 0xffffu;
              if (d == 0u || d > pos - lo_pos) break;
              const uint32_t q = pos - d;
              // cheap reject: the byte that would extend the best match
              if (best == 0u || rd8(sh, q + best) == rd8(sh, pos + best)) {
                const uint32_t L = match_len(sh, q, pos, maxl);
                if (L > best) { best = L; bd = d; if (L >= tune.nice || L == maxl) break; }
              }
              if (q < s0) break;
              c16 = sh.prev[q - s0];
            }
            if (best == 3u && bd > tune.too_far) best = 0;
          }
          if (best >= 3u) {
            uint32_t ls, eb, ev, ds, deb, dev;
            len_sym(best, ls, eb, ev);
            dist_sym(bd, ds, deb, dev);
            tok_put(sh, ns++, lane, 0x8000u | (best - 3u));
            tok_put(sh, ns++, lane, bd - 1u);
            lds_add(&sh.freq[257u + ls], 1u);
            lds_add(&sh.freq[NLL + ds], 1u);
            pos += best;
          } else {
            const uint32_t lit = rd8(sh, pos);
            tok_put(sh, ns++, lane, lit);
            lds_add(&sh.freq[lit], 1u);
            pos++;
          }
        }
      }
      LV(nslot) = ns;
    }
    WAVE_SYNC();

    // ---- 4. block type and codes ----
    HZ_T(4);
    LANE_LOOP { if (lane == 0) sh.freq[256] = 1; }
    WAVE_SYNC();
    uint64_t dyn_bits = ~0ull, fix_bits = ~0ull;
    if (!tune.stored) {
      HD_BUILD_HUFF(sh, sh.freq, NLL, 512, 15, sh.len_ll, sh.code_ll);
      HD_BUILD_HUFF(sh, (sh.freq + NLL), ND, 32, 15, sh.len_d, sh.code_d);
      HZ_T(5);
      LANE_LOOP { if (lane == 0) build_rle(sh); }
      WAVE_SYNC();
      HD_BUILD_HUFF(sh, sh.clf, NCL, 32, 7, sh.len_cl, sh.code_cl);
      LANE_LOOP { if (lane == 0) sh.hdr_bits = dyn_header_bits(sh); }
      WAVE_SYNC();
      HZ_T(10);
      // data bits under the dynamic and the fixed code
      LANE_VAR(uint64_t, db);
      LANE_VAR(uint64_t, fb);
      LANE_LOOP {
        uint64_t d = 0, f = 0;
        for (int s = lane; s < NSYM; s += WAVE) {
          const uint64_t c = sh.freq[s];
          if (!c) continue;
          if (s < NLL) {
            const uint32_t e = s > 256 ? len_extra_bits((uint32_t)s - 257u) : 0u;
            d += c * (sh.len_ll[s] + e);
            f += c * (fixed_ll_len((uint32_t)s) + e);
          } else {
            const uint32_t e = dist_extra_bits((uint32_t)(s - NLL));
            d += c * (sh.len_d[s - NLL] + e);
            f += c * (5u + e);
          }
        }
        LV(db) = d;
        LV(fb) = f;
      }
#if HZ_GPU
      dyn_bits = HD_WAVE_SUM64(db);
      fix_bits = HD_WAVE_SUM64(fb);
#else
      dyn_bits = 0; fix_bits = 0;
      for (int l = 0; l < 64; l++) { dyn_bits += db[l]; fix_bits += fb[l]; }
#endif
      dyn_bits += sh.hdr_bits;
      fix_bits += 3u;
    }
    const uint64_t hdr_end = (carry_bits + 3u + 7u) & ~7u;
    const uint64_t stored_bits = hdr_end - carry_bits + 32u + 8ull * seglen;
    uint32_t btype;
    if (dyn_bits <= fix_bits && dyn_bits < stored_bits) btype = 2;
    else if (fix_bits < stored_bits) btype = 1;
    else btype = 0;

    // ---- 5. emission into the staging words ----
    HZ_T(6);
    LANE_LOOP {
      for (int w = lane; w < STAGE_WORDS; w += WAVE) sh.stage[w] = w == 0 ? carry : 0u;
      if (lane == 0 && btype == 1) set_fixed_codes(sh);
    }
    WAVE_SYNC();
    uint32_t total_bits;
    if (btype == 0) {
      const uint32_t b0 = (uint32_t)(hdr_end >> 3);
      LANE_LOOP {
        if (lane == 0) {
          BitW w;
          bw_init(w, carry_bits);
          bw_put(sh, w, last ? 1u : 0u, 3);
          bw_flush(sh, w);
        }
        uint8_t* sb = (uint8_t*)sh.stage;
        if (lane < 4) {
          const uint32_t v = (lane < 2) ? seglen : (~seglen & 0xffffu);
          sb[b0 + (uint32_t)lane] = (uint8_t)((lane & 1) ? (v >> 8) : v);
        }
        for (uint32_t i = (uint32_t)lane; i < seglen; i += WAVE) sb[b0 + 4u + i] = (uint8_t)rd8(sh, s0 + i);
      }
      total_bits = (b0 + 4u + seglen) * 8u;
    } else {
      uint32_t hdr = 3;
      if (btype == 2) hdr = sh.hdr_bits;
      // header: lane 0 (while the other lanes count their token bits)
      LANE_VAR(uint32_t, nb);
      LANE_LOOP {
        if (lane == 0) {
          BitW w;
          bw_init(w, carry_bits);
          bw_put(sh, w, (last ? 1u : 0u) | (btype << 1), 3);
          if (btype == 2) {
            bw_put(sh, w, sh.hlit - 257u, 5);
            bw_put(sh, w, sh.hdist - 1u, 5);
            bw_put(sh, w, sh.hclen - 4u, 4);
            for (uint32_t i = 0; i < sh.hclen; i++) bw_put(sh, w, sh.len_cl[hz::cl_order(i)], 3);
            for (uint32_t i = 0; i < sh.nrle; i++) {
              const uint32_t e = sh.rle[i];
              const uint32_t sym = e & 0xffu;
              bw_put(sh, w, sh.code_cl[sym], sh.len_cl[sym]);
              const uint32_t xb = cl_extra_bits(sym);
              if (xb) bw_put(sh, w, e >> 8, xb);
            }
          }
          bw_flush(sh, w);
        }
        uint32_t bits = 0;
        const uint32_t ns = LV(nslot);
        for (uint32_t s = 0; s < ns; s++) {
          const uint32_t t = tok_get(sh, s, lane);
          if (t & 0x8000u) {
            const uint32_t d = tok_get(sh, ++s, lane) + 1u;
            uint32_t ls, eb, ev, ds, deb, dev;
            len_sym((t & 0x7fffu) + 3u, ls, eb, ev);
            dist_sym(d, ds, deb, dev);
            bits += sh.len_ll[257u + ls] + eb + sh.len_d[ds] + deb;
          } else {
            bits += sh.len_ll[t];
          }
        }
        if (lane == WAVE - 1) bits += sh.len_ll[256];
        LV(nb) = bits;
      }
      WAVE_SYNC();
      HZ_T(7);
      LANE_VAR(uint32_t, off);
#if HZ_GPU
      off = hz::wave_excl_scan(nb, (int)threadIdx.x);
      const uint32_t sum_bits = hz::wave_sum(nb);
#else
      uint32_t sum_bits = 0;
      for (int l = 0; l < 64; l++) { off[l] = sum_bits; sum_bits += nb[l]; }
#endif
      LANE_LOOP {
        BitW w;
        bw_init(w, carry_bits + hdr + LV(off));
        const uint32_t ns = LV(nslot);
        for (uint32_t s = 0; s < ns; s++) {
          const uint32_t t = tok_get(sh, s, lane);
          if (t & 0x8000u) {
            const uint32_t d = tok_get(sh, ++s, lane) + 1u;
            uint32_t ls, eb, ev, ds, deb, dev;
            len_sym((t & 0x7fffu) + 3u, ls, eb, ev);
            dist_sym(d, ds, deb, dev);
            bw_put(sh, w, sh.code_ll[257u + ls], sh.len_ll[257u + ls]);
            if (eb) bw_put(sh, w, ev, eb);
            bw_put(sh, w, sh.code_d[ds], sh.len_d[ds]);
            if (deb) bw_put(sh, w, dev, deb);
          } else {
            bw_put(sh, w, sh.code_ll[t], sh.len_ll[t]);
          }
        }
        if (lane == WAVE - 1) bw_put(sh, w, sh.code_ll[256], sh.len_ll[256]);
        bw_flush(sh, w);
      }
      total_bits = carry_bits + hdr + sum_bits;
    }
    WAVE_SYNC();

    // ---- 6. flush full words, carry the partial one ----
    HZ_T(8);
    const uint32_t full = total_bits >> 5;
    if ((out_words + full) * 4ull > (uint64_t)job.cap + 4u) {   // dst holds cap + 8 bytes
      overflow = true;
    } else {
      LANE_LOOP {
        for (uint32_t w = (uint32_t)lane; w < full; w += WAVE) gdst[out_words + w] = sh.stage[w];
      }
      carry = sh.stage[full];
      carry_bits = total_bits & 31u;
      out_words += full;
    }
    WAVE_SYNC();
  }
  if (overflow) return R_OVERFLOW;

  // ---- trailer: byte align, adler32 big-endian ----
  HZ_T(9);
  uint64_t S1, S2;
#if HZ_GPU
  S1 = HD_WAVE_SUM64(as1);
  S2 = HD_WAVE_SUM64(as2);
#else
  S1 = 0; S2 = 0;
  for (int l = 0; l < 64; l++) { S1 += as1[l]; S2 += as2[l]; }
#endif
  const uint64_t A = (1u + S1) % ADLER_MOD;
  const uint64_t B = ((uint64_t)n % ADLER_MOD + ((uint64_t)n % ADLER_MOD) * (S1 % ADLER_MOD) + ADLER_MOD * ADLER_MOD -
                      S2 % ADLER_MOD) % ADLER_MOD;
  const uint32_t adler = (uint32_t)((B << 16) | A);
  const uint32_t be = (adler >> 24) | ((adler >> 8) & 0xff00u) | ((adler << 8) & 0xff0000u) | (adler << 24);
  carry_bits = (carry_bits + 7u) & ~7u;
  if (carry_bits == 32u) {   // byte alignment completed a word
    const uint64_t end = (uint64_t)out_words * 4u + 8u;
    if (end > job.cap) return R_OVERFLOW;
    LANE_LOOP { if (lane == 0) gdst[out_words] = carry; }
    out_words++;
    carry = 0;
    carry_bits = 0;
  }
  const uint64_t total_bytes = (uint64_t)out_words * 4u + (carry_bits + 32u) / 8u;
  if (total_bytes > job.cap) return R_OVERFLOW;
  const uint32_t w0 = carry_bits ? (carry & ((1u << carry_bits) - 1u)) | (be << carry_bits) : be;
  const uint32_t w1 = carry_bits ? be >> (32u - carry_bits) : 0u;
  LANE_LOOP {
    if (lane == 0) {
      gdst[out_words] = w0;
      if (carry_bits) gdst[out_words + 1u] = w1;
    }
  }
  WAVE_SYNC_GLOBAL();
  return (int64_t)total_bytes;
}

}  // namespace hd
