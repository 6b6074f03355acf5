// inflate_wave.h -- one-wavefront-per-stream zlib (RFC 1950/1951) decoder.
//
// Replaces, for the HSDS data-node hot path, the zlib inflate that the reference
// reaches through storUtil._uncompress (hsds/util/storUtil.py:209-220, CPython
// zlib.decompress) and through c-blosc's zlib_wrap_decompress for every Blosc split
// (storUtil.py:195-208).  Output must be bit-identical to libz; errors map to the
// same "500" outcome (corrupt data, truncated stream, adler32 mismatch).
//
// Algorithm (see DESIGN.md "Inflate"):
//   The 64 lanes of a wavefront cooperate on ONE deflate stream.  Inside a Huffman
//   block the bitstream window [win_start, win_start + 64*L) is cut into 64 segments
//   of L bits.  Phase A: lane i speculatively decodes tokens starting W bits before
//   its segment (lane 0 starts exactly at the known token boundary), marking every
//   token start in an LDS bitmap and storing tokens in LDS.  Phase B: lane i is
//   "synced" when the exit position of lane i-1 (first token start at or after the
//   end of segment i-1) is one of lane i's marked token starts; from there on its
//   decode is the true decode (Huffman self-synchronisation).  The longest synced
//   prefix of lanes is accepted.  Phase C: output offsets by a wave prefix sum,
//   literals written, LZ77 matches resolved in rounds against a frontier F (all
//   output below F is final), adler32 accumulated per lane as position-weighted
//   sums and combined once per stream.
//
// The file is SINGLE SOURCE for two drivers:
//   * HIP (gfx950):  every lane is a real SIMT lane, LANE_LOOP is one iteration.
//   * CPU emulation (tests/emu): LANE_LOOP iterates lanes 0..63 in order, so the
//     same orchestration (including every cross-lane step) is unit-tested on CPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HZ_GPU 1
#define HZ_HD __device__ __forceinline__
// global (address space 1) pointers: plain global_load/global_store that only
// count on vmcnt, instead of flat accesses that also hold up every LDS wait
typedef __attribute__((address_space(1))) uint8_t hz_gu8;
typedef __attribute__((address_space(1))) const uint8_t hz_gcu8;
typedef __attribute__((address_space(1))) uint32_t hz_gu32;
typedef __attribute__((address_space(1))) const uint32_t hz_gcu32;
typedef __attribute__((address_space(1))) uint16_t hz_gu16;
#define HZ_GLOBAL(T, p) ((T)(uintptr_t)(p))
#define HZ_UNROLL _Pragma("unroll")
#define LANE_VAR(T, name) T name
#define LV(name) name
// the lane index within the wavefront (a workgroup may hold two: inflate2w_kernel)
#define HZ_LANE_ID() ((int)(threadIdx.x & 63u))
#define LANE_LOOP for (int lane = HZ_LANE_ID(), _once = 1; _once; _once = 0)
#if defined(HZ_LIGHT_SYNC)
// one-wavefront workgroups: the LDS executes a wave's instructions in order, so
// cross-lane LDS hand-offs only need the compiler not to move or cache memory
// accesses across this point (wavefront-scope acquire/release fences), not the
// s_waitcnt vmcnt(0) lgkmcnt(0) + s_barrier of __syncthreads
#define WAVE_SYNC()                                              \
  do {                                                           \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");       \
    __builtin_amdgcn_wave_barrier();                             \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");       \
  } while (0)
#else
#define WAVE_SYNC() __syncthreads()
#endif
#define WAVE_SYNC_GLOBAL() \
  do { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); __syncthreads(); \
       __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); } while (0)
#else
#include <string.h>
#include <stdio.h>
#define HZ_GPU 0
#define HZ_HD static inline
typedef uint8_t hz_gu8;
typedef const uint8_t hz_gcu8;
typedef uint32_t hz_gu32;
typedef const uint32_t hz_gcu32;
typedef uint16_t hz_gu16;
#define HZ_GLOBAL(T, p) ((T)(p))
#define HZ_UNROLL
#define LANE_VAR(T, name) T name[64]
#define LV(name) name[lane]
#define LANE_LOOP for (int lane = 0; lane < 64; lane++)
#define WAVE_SYNC() do {} while (0)
#define WAVE_SYNC_GLOBAL() do {} while (0)
#endif

#if HZ_GPU && defined(HZ_PROFILE)
__device__ unsigned long long hz_prof[16];
__device__ unsigned long long hz_tail[8];
struct HzProf { uint64_t acc[16]; uint64_t last; int cur; };
#define HZ_T(slot)                                                                          \
  do { if (prof) { const uint64_t _now = __builtin_amdgcn_s_memtime();                      \
       prof->acc[prof->cur] += _now - prof->last; prof->last = _now; prof->cur = (slot); } } while (0)
#else
struct HzProf { int unused; };
#define HZ_T(slot) do {} while (0)
#endif

namespace hz {

constexpr int WAVE = 64;
constexpr int LL_ROOT = 10;
constexpr int D_ROOT = 8;
// second-level entries (codes longer than the root).  Sized at or above zlib's exact
// worst cases (ENOUGH: 286 symbols / root 10 -> 308 extra entries; 30 symbols /
// root 8 -> at most 3 x 128), so every complete code fits and no slow path exists.
// Window sizes (LMAX, SCAP, SLOTS) are set so that sizeof(Shared) = 20480 B: eight
// wavefronts per CU (A/B on MI355X: 7 -> 8 waves/CU gave F1 +7 %, F2 +14 %; smaller
// windows at 9-10 waves/CU lost more to per-window overhead than they gained).
#ifndef HZ_LL_SUB
#define HZ_LL_SUB 320
#endif
constexpr int LL_SUB = HZ_LL_SUB;
constexpr int D_SUB = 384;
#ifndef HZ_SLOTS
#define HZ_SLOTS 50
#endif
constexpr int SLOTS = HZ_SLOTS;           // 16-bit token slots per lane per window (a match takes two)
#ifndef HZ_LMAX
#define HZ_LMAX 288
#endif
constexpr int LMAX = HZ_LMAX;           // max segment length (bits)
constexpr int LMIN = 64;
constexpr uint32_t ADAPT_FILL16 = 11; // adaptive L aims at this many 16ths of SLOTS token slots per segment
#ifndef HZ_SCAP
#define HZ_SCAP 4608
#endif
constexpr int SCAP = HZ_SCAP;           // window output bytes resolved in LDS
#ifndef HZ_CMAX
#define HZ_CMAX 256
#endif
constexpr int CMAX = HZ_CMAX;
#ifndef HZ_SCAP_FILL8
#define HZ_SCAP_FILL8 7                 // adaptive L aims at this many 8ths of SCAP output bytes per window
#endif           // max continuation bits into the next segment
constexpr int OVR = 64;             // bitmap bits past the last token start
constexpr int BM_WORDS = (LMAX + CMAX + OVR) / 32 + 1;
// staged input dwords: window (64 L) + warm-up (<= L) + alignment + overrun/peek
constexpr int WMAX = 1024;
constexpr int IN_WORDS = (WAVE * LMAX + WMAX + CMAX + 256) / 32 + 8;
constexpr uint32_t ADLER_MOD = 65521;

// status codes (include/hsds_amd.h)
constexpr int ST_OK = 0;
constexpr int ST_FRAME = -1;
constexpr int ST_DATA = -2;
constexpr int ST_TRUNC = -3;
constexpr int ST_SIZE = -4;
constexpr int ST_UNSUP = -5;

// 16-bit decode-table entry: bits 0-3 code length, bits 4-15 symbol (literal/length
// table: 0-255 literal, 256 end of block, 257-285 length, anything else invalid;
// distance table: 0-29, anything else invalid).  Code length 0 marks a pointer to a
// second-level table: bits 4-12 its offset after the root entries, 13-15 its index
// bits.  Length / distance bases and extra-bit counts are computed from the symbol.
constexpr uint32_t SYM_BAD = 0xfffu;
HZ_HD uint16_t ent_sym(uint32_t len, uint32_t sym) { return (uint16_t)(len | (sym << 4)); }
HZ_HD uint16_t ent_sub(uint32_t off, uint32_t sb) { return (uint16_t)((off << 4) | (sb << 13)); }
// "rich" symbol entries (inflate2.h): the length / distance base and extra bits come from
// the table instead of per-token arithmetic.
//  literal/length (kind 1): bits 0-3 code length, 4-6 extra bits x (7: literal / EOB /
//    invalid), 7-15 value v (literal byte, 256 = EOB, 257 = invalid, or the length base)
//  distance (kind 2): bits 0-3 code length, 4-7 extra bits, 8-10 b, 11 one, 12 invalid:
//    distance = (b << extra) + one + extra value
// Subtable links keep ent_sub's layout (code length field 0).
HZ_HD uint16_t ent_rich(int kind, uint32_t len, uint32_t sym) {
  if (kind == 1) {
    if (sym <= 256u) return (uint16_t)(len | (7u << 4) | (sym << 7));
    if (sym > 285u) return (uint16_t)(len | (7u << 4) | (257u << 7));
    const uint32_t q = sym - 257u;
    const uint32_t x = (q < 8u || q == 28u) ? 0u : (q - 4u) >> 2;
    const uint32_t base = q < 8u ? q + 3u : q == 28u ? 258u : ((4u | (q & 3u)) << x) + 3u;
    return (uint16_t)(len | (x << 4) | (base << 7));
  }
  if (sym >= 30u) return (uint16_t)(len | (1u << 12));
  const uint32_t x = sym < 4u ? 0u : (sym - 2u) >> 1;
  const uint32_t b = sym < 4u ? sym + 1u : 2u | (sym & 1u);
  const uint32_t one = sym < 4u ? 0u : 1u;
  return (uint16_t)(len | (x << 4) | (b << 8) | (one << 11));
}

// tokens (decoder result): literal = byte; match = 0x80000000 | len<<16 | (dist-1); EOB / ERR
constexpr uint32_t T_MATCH = 0x80000000u;
constexpr uint32_t T_EOB = 0x100u;        // == its stored slot value S_EOB
constexpr uint32_t T_ERR = 0x101u;        // == S_ERR
// stored token slots (16 bit): literal byte, S_EOB, S_ERR, or a match as two slots
// 0x8000 | (len - 3) followed by (dist - 1).  A lane's token k sits at slot
// k + popcount(match mask of tokens < k).
constexpr uint32_t S_EOB = 0x100u, S_ERR = 0x101u, S_MATCH = 0x8000u;


struct Shared {
  uint16_t lut_ll[(1 << LL_ROOT) + LL_SUB];
  uint16_t lut_d[(1 << D_ROOT) + D_SUB];
  uint16_t tb_first[16];
  uint16_t tb_offs[17];
  uint16_t tb_next[16];
  // token slots, lane-interleaved in pairs: slot s of lane l is half (s & 1) of dword
  // (s >> 1) * 64 + l, so lanes reading any slots hit distinct banks
  union {
    uint16_t tok[SLOTS * WAVE];
    uint32_t tokw[SLOTS / 2 * WAVE];
  };
  // The window's decode state (input staging, token-start bitmaps, per-lane exit /
  // sync / repair flags) is dead once phase C starts building the byte reference
  // map, and is rebuilt by the next window's staging / phase A: the two share LDS.
  union {
    struct {
      union {
        uint32_t bitmap[WAVE][BM_WORDS];
        struct {                         // Huffman table build scratch (dead while windows run)
          uint16_t sorted_ll[288];
          uint16_t sorted_d[32];
          uint16_t cnt_ll[16];
          uint16_t cnt_d[16];
          uint16_t cnt_cl[16];
          uint16_t sorted_cl[20];
          uint8_t lens[320 + 32];
        };
      };
      uint32_t in32[IN_WORDS + 4];
      uint32_t exitpos[WAVE];
      uint32_t syncpos[WAVE];
      uint32_t flag[WAVE];
      uint32_t flag2[WAVE];
    };
    uint16_t ref[SCAP];
  };
  uint32_t contpos[WAVE];
  uint32_t obase[WAVE + 1];
  uint16_t tcur_l[WAVE];
  uint16_t tend_l[WAVE];
  // uniform scalars published by lane 0
  int32_t u_status;
  uint32_t u_pos;
  uint32_t u_nlen, u_ndist;
  uint32_t u_stage_base;
  uint32_t u_stored_len;
};

HZ_HD uint32_t bmask(uint32_t n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1u); }

HZ_HD uint32_t popc32(uint32_t x) {
#if HZ_GPU
  return __popc(x);
#else
  return (uint32_t)__builtin_popcount(x);
#endif
}

// RFC 1951 order of the code-length code lengths, packed 5 bits per entry
HZ_HD uint32_t cl_order(uint32_t i) {
  // 16,17,18,0,8,7,9,6,10,5,11,4 | 12,3,13,2,14,1,15
  const uint64_t lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 | 9ull << 30 |
                      6ull << 35 | 10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
  const uint64_t hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 | 15ull << 30;
  return (uint32_t)((i < 12 ? lo >> (5 * i) : hi >> (5 * (i - 12))) & 31u);
}

HZ_HD uint32_t popc64(uint64_t x) {
#if HZ_GPU
  return (uint32_t)__popcll(x);
#else
  return (uint32_t)__builtin_popcountll(x);
#endif
}

HZ_HD void atomicAdd_lds(uint16_t* p, int v) {
#if HZ_GPU
  // 16-bit counters live in LDS: add to the containing aligned dword
  uint32_t* w = (uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
  atomicAdd(w, (uint32_t)v << (((uintptr_t)p & 2) * 8));
#else
  *p = (uint16_t)(*p + v);
#endif
}

HZ_HD uint32_t rev_bits(uint32_t v, int n) {
  uint32_t r = 0;
  for (int i = 0; i < n; i++) { r = (r << 1) | (v & 1u); v >>= 1; }
  return r;
}

// ---- LDS bit access ---------------------------------------------------------
// Bit positions are relative to the 4-byte aligned base of the stream, so every
// staged dword load is aligned.  peek64 returns >= 64 valid bits at `pos`.
HZ_HD uint64_t peek64(const Shared* sh, uint32_t pos) {
  uint32_t w = pos - sh->u_stage_base;
  uint32_t i = w >> 5, s = w & 31u;
  uint64_t lo = (uint64_t)sh->in32[i] | ((uint64_t)sh->in32[i + 1] << 32);
  uint64_t hi = sh->in32[i + 2];
  return s ? ((lo >> s) | (hi << (64 - s))) : lo;
}

HZ_HD uint32_t lookup_ll(const Shared* sh, uint64_t bits) {
  uint32_t e = sh->lut_ll[bits & ((1u << LL_ROOT) - 1)];
  if (!(e & 15u)) e = sh->lut_ll[(1u << LL_ROOT) + ((e >> 4) & 511u) + ((uint32_t)(bits >> LL_ROOT) & bmask(e >> 13))];
  return e;
}
HZ_HD uint32_t lookup_d(const Shared* sh, uint64_t bits) {
  uint32_t e = sh->lut_d[bits & ((1u << D_ROOT) - 1)];
  if (!(e & 15u)) e = sh->lut_d[(1u << D_ROOT) + ((e >> 4) & 511u) + ((uint32_t)(bits >> D_ROOT) & bmask(e >> 13))];
  return e;
}

// ---- register bit reader over the staged window ------------------------------
// bb holds `avail` (>= 32 after fill) bits starting at bit position `pos`; the next
// staged dword is prefetched into `nxt` so a refill never waits on LDS.
struct BitRd {
  uint64_t bb;
  uint32_t avail;
  uint32_t widx;
  uint32_t nxt;
  uint32_t pos;
};

HZ_HD void br_init(const Shared* sh, BitRd& r, uint32_t p, uint32_t stage_base) {
  const uint32_t w = p - stage_base, i = w >> 5, s = w & 31u;
  const uint64_t lo = (uint64_t)sh->in32[i] | ((uint64_t)sh->in32[i + 1] << 32);
  r.bb = lo >> s;
  r.avail = 64u - s;
  r.widx = i + 2u;
  r.nxt = sh->in32[i + 2];
  r.pos = p;
}

HZ_HD void br_fill(const Shared* sh, BitRd& r) {
  // branch-free: always read the next staged word, keep it only when used
  const uint32_t need = r.avail < 32u;
  const uint64_t add = (uint64_t)r.nxt << (r.avail & 31u);
  r.bb |= need ? add : 0ull;
  r.avail += need ? 32u : 0u;
  r.widx += need;
  const uint32_t nn = sh->in32[r.widx];
  r.nxt = need ? nn : r.nxt;
}

HZ_HD void br_drop(BitRd& r, uint32_t n) { r.bb >>= n; r.avail -= n; r.pos += n; }

// decode one token at r.pos and advance past it.  Invalid codes advance by their
// table length (any deterministic advance keeps speculative decoders consistent;
// a real error stops the stream at the ERR token's start).
HZ_HD uint32_t next_token(const Shared* sh, BitRd& r) {
  br_fill(sh, r);
  const uint32_t e = lookup_ll(sh, r.bb);
  const uint32_t nb = e & 15u, p = e >> 4;
  // RFC 1951 3.2.5 length codes: symbol 257+s, s < 8 -> 3+s, s == 28 -> 258,
  // otherwise ((4 | s&3) << x) + 3 with x = (s-4)/4 extra bits
  const uint32_t s = p - 257u;
  const int islen = s < 29u;
  const uint32_t xb = (islen && s >= 8u && s < 28u) ? (s - 4u) >> 2 : 0u;
  const uint32_t base = s < 8u ? s + 3u : s == 28u ? 258u : ((4u | (s & 3u)) << xb) + 3u;
  const uint32_t len = base + ((uint32_t)(r.bb >> nb) & bmask(xb));
  br_drop(r, nb + xb);
  uint32_t tok = p <= 256u ? p : T_ERR;     // literal byte or T_EOB (= 256)
  if (islen) {
    br_fill(sh, r);
    const uint32_t ed = lookup_d(sh, r.bb);
    const uint32_t nd = ed & 15u, d = ed >> 4;
    // distance codes: d < 4 -> d+1, otherwise ((2 | d&1) << x) + 1 with x = d/2-1
    const int ok = d < 30u;
    const uint32_t xd = (ok && d >= 2u) ? (d - 2u) >> 1 : 0u;
    const uint32_t dist = (d < 4u ? d + 1u : ((2u | (d & 1u)) << xd) + 1u) + ((uint32_t)(r.bb >> nd) & bmask(xd));
    br_drop(r, ok ? nd + xd : nd);
    tok = ok ? (T_MATCH | (len << 16) | (dist - 1u)) : T_ERR;
  }
  return tok;
}

HZ_HD uint32_t tok_idx(uint32_t s, int lane) { return ((s >> 1) * (uint32_t)WAVE + (uint32_t)lane) * 2u + (s & 1u); }
HZ_HD uint32_t tok_at(const Shared* sh, uint32_t s, int lane) { return sh->tok[tok_idx(s, lane)]; }
// store decoder token tokv at slot ns of `lane`; returns the slots used (1 or 2)
HZ_HD uint32_t put_tok(Shared* sh, int lane, uint32_t ns, uint32_t tokv) {
  const uint32_t m = tokv & T_MATCH;
  const uint32_t i0 = tok_idx(ns, lane);
  sh->tok[i0] = (uint16_t)(m ? (S_MATCH | (((tokv >> 16) & 0x1ffu) - 3u)) : tokv);
  if (m) sh->tok[i0 + ((ns & 1u) ? 2u * (uint32_t)WAVE - 1u : 1u)] = (uint16_t)(tokv & 0x7fffu);
  return m ? 2u : 1u;
}
// token at slot t of lane j: v = the slot, d = distance of a match (the next slot + 1);
// two independent dword reads instead of two dependent 16-bit ones
HZ_HD void tok_pair(const Shared* sh, uint32_t t, int j, uint32_t& v, uint32_t& d) {
  const uint32_t q = t >> 1;
  const uint32_t q1 = q + 1u < (uint32_t)(SLOTS / 2) ? q + 1u : q;
  const uint32_t w0 = sh->tokw[q * (uint32_t)WAVE + (uint32_t)j];
  const uint32_t w1 = sh->tokw[q1 * (uint32_t)WAVE + (uint32_t)j];
  v = (t & 1u) ? (w0 >> 16) : (w0 & 0xffffu);
  d = ((t & 1u) ? (w1 & 0xffffu) : (w0 >> 16)) + 1u;
}
// slot of token k of a lane whose match mask is mb
HZ_HD uint32_t tok_slot(uint64_t mb, uint32_t k) { return k + popc64(k >= 64u ? mb : mb & ((1ull << k) - 1ull)); }

HZ_HD void mark_bit(Shared* sh, int lane, uint32_t rel) {
  if (rel < (uint32_t)(BM_WORDS * 32)) sh->bitmap[lane][rel >> 5] |= 1u << (rel & 31u);
}

// relative bit position of the k-th (0-based) mark of a lane
HZ_HD uint32_t nth_mark(const Shared* sh, int lane, uint32_t k) {
  uint32_t c = 0;
  for (uint32_t w = 0; w < (uint32_t)BM_WORDS; w++) {
    uint32_t m = sh->bitmap[lane][w];
    const uint32_t pc = popc32(m);
    if (c + pc > k) {
      for (;;) {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        if (c == k) return w * 32u + b;
        c++;
        m &= m - 1u;
      }
    }
    c += pc;
  }
  return 0xffffffffu;
}

// ---- global memory helpers -------------------------------------------------
// aligned dword k of the stream's aligned base; bytes outside [lo, hi) are zero.
HZ_HD uint32_t load_word(hz_gcu8* base, uint32_t k, uint32_t lo, uint32_t hi) {
  uint32_t b0 = k * 4u;
  if (b0 >= hi || b0 + 4u <= lo) return 0u;
  uint32_t v = *(hz_gcu32*)(base + b0);
  if (b0 < lo) v &= ~bmask((lo - b0) * 8u);
  if (b0 + 4u > hi) v &= bmask((hi - b0) * 8u);
  return v;
}

}  // namespace hz

// ---- wave-collective helpers (the only places the two drivers differ) -------
#if HZ_GPU
#define WAVE_BALLOT(expr) \
  ([&]() { const int lane = HZ_LANE_ID(); (void)lane; return (uint64_t)__ballot((expr) ? 1 : 0); }())
namespace hz {
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane) {
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}
// inclusive prefix sum over the 64 lanes by DPP (no LDS round trip): shifts of 1, 2, 4, 8
// lanes inside each row of 16, then each row's last lane broadcast to the rows after it
// (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3)
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
// exclusive prefix maximum over the lanes (lane 0: 0)
__device__ __forceinline__ uint32_t wave_excl_max(uint32_t v, int lane) {
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x = y > x ? y : x;
  }
  const uint32_t e = __shfl_up(x, 1, 64);
  return lane ? e : 0u;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) { uint32_t y = __shfl_xor(v, o, 64); v = y < v ? y : v; }
  return v;
}
}  // namespace hz
#define WAVE_EXCL_SCAN(arr_or_var, out) out = hz::wave_excl_scan(arr_or_var, lane)
#define WAVE_SUM(v) hz::wave_sum(v)
#else
#define WAVE_BALLOT(expr)                                          \
  ([&]() {                                                         \
    uint64_t _m = 0;                                               \
    for (int lane = 0; lane < 64; lane++) if (expr) _m |= 1ull << lane; \
    return _m;                                                     \
  }())
#endif

namespace hz {

// ---------------------------------------------------------------------------
// Cooperative Huffman table construction (RFC 1951 3.2.2 canonical codes).
// lens[0..n) -> cnt[16], sorted[], lut (root bits).  Returns ST_OK or ST_DATA
// following zlib inflate_table's rules: over-subscribed always fails; an
// incomplete code fails for the code-length code, and for the literal/length and
// distance codes unless it is a single code of length 1.  n == 0 (no codes,
// e.g. no distances) is accepted and every lookup then decodes as invalid.
// kind: 0 = code-length code, 1 = literal/length, 2 = distance.
// ---------------------------------------------------------------------------
struct TableArgs {
  const uint8_t* lens;
  int n;
  uint16_t* cnt;
  uint16_t* sorted;
  uint16_t* lut;
  int root;
  int kind;
  int nsub;     // second-level capacity after the 2^root root entries
  int rich;     // 1: ent_rich symbol entries (inflate2.h), 0: ent_sym
};

}  // namespace hz

#if HZ_GPU
#define HZ_UNIFORM(x) ((uint32_t)__builtin_amdgcn_readfirstlane((int)(x)))
// exclusive scan of the low 24 bits of lane variable v into o, total into t
#define HZ_SCAN_LOW24(v, o, t)                                \
  do {                                                        \
    o = hz::wave_excl_scan((v) & 0xffffffu, HZ_LANE_ID()); \
    t = hz::wave_sum((v) & 0xffffffu);                        \
  } while (0)
#else
#define HZ_UNIFORM(x) ((uint32_t)(x))
#define HZ_SCAN_LOW24(v, o, t)                                                              \
  do {                                                                                      \
    t = 0;                                                                                  \
    for (int _ln = 0; _ln < 64; _ln++) { o[_ln] = t; t += v[_ln] & 0xffffffu; }             \
  } while (0)
#endif

#ifndef HZ_TB_SYNC
#define HZ_TB_SYNC() WAVE_SYNC()
#endif
// Table build as a macro-free function per driver is awkward because it needs
// ballots; it is written once in the SIMT style below.
#define HZ_BUILD_TABLE(sh, A, status_out)                                               \
  do {                                                                                  \
    /* counts: LDS atomics over all lanes */                                          \
    LANE_LOOP { if (lane < 16) (A).cnt[lane] = 0; }                                     \
    HZ_TB_SYNC();                                                                        \
    LANE_LOOP {                                                                         \
      for (int s = lane; s < (A).n; s += 64) {                                          \
        const int l = (A).lens[s];                                                      \
        if (l) hz::atomicAdd_lds(&(A).cnt[l], 1);                                       \
      }                                                                                 \
    }                                                                                   \
    HZ_TB_SYNC();                                                                        \
    /* validity (zlib inflate_table rules), first code and offset per length */        \
    LANE_LOOP {                                                                         \
      if (lane == 0) {                                                                  \
        int left = 1, maxl = 0, bad = 0;                                                \
        for (int l = 1; l <= 15; l++) {                                                 \
          left <<= 1; left -= (A).cnt[l];                                               \
          if ((A).cnt[l]) maxl = l;                                                     \
          if (left < 0) bad = 1;                                                        \
        }                                                                               \
        if (!bad && maxl > 0 && left > 0 && ((A).kind == 0 || maxl != 1)) bad = 1;      \
        if ((A).kind == 0 && maxl == 0) bad = 1;                                        \
        int code = 0, off = 0;                                                          \
        for (int l = 1; l <= 15; l++) {                                                 \
          code = (code + (l > 1 ? (A).cnt[l - 1] : 0)) << 1;                            \
          (sh).tb_first[l] = (uint16_t)code;                                            \
          (sh).tb_offs[l] = (uint16_t)off;                                              \
          (sh).tb_next[l] = (uint16_t)off;                                              \
          off += (A).cnt[l];                                                            \
        }                                                                               \
        (sh).tb_offs[16] = (uint16_t)off;                                               \
        (sh).u_status = bad ? hz::ST_DATA : hz::ST_OK;                                  \
      }                                                                                 \
    }                                                                                   \
    HZ_TB_SYNC();                                                                        \
    /* per-length counts, first codes and offsets, read once into wave-uniform registers */ \
    uint32_t _cn[16], _fc[16], _of[16];                                                 \
    _Pragma("unroll") for (int _q = 0; _q < 16; _q++) {                                 \
      _cn[_q] = HZ_UNIFORM(_q ? (A).cnt[_q] : 0);                                       \
      _fc[_q] = HZ_UNIFORM(_q ? (sh).tb_first[_q] : 0);                                 \
      _of[_q] = HZ_UNIFORM(_q ? (sh).tb_offs[_q] : 0);                                  \
    }                                                                                   \
    /* canonical order: ranks within a length via ballots, 64 symbols at a time; the  \
       running offset per length stays in registers (no LDS round trip per length) */  \
    {                                                                                   \
      uint32_t _nx[16];                                                                 \
      _Pragma("unroll") for (int _q = 0; _q < 16; _q++) _nx[_q] = _of[_q];              \
      for (int _c = 0; _c < (A).n; _c += 64) {                                          \
        LANE_VAR(int, _l);                                                              \
        LANE_LOOP { LV(_l) = _c + lane < (A).n ? (A).lens[_c + lane] : 0; }             \
        _Pragma("unroll") for (int L = 1; L <= 15; L++) {                               \
          if (!_cn[L]) continue;                                                        \
          const uint64_t m = WAVE_BALLOT(LV(_l) == L);                                  \
          if (!m) continue;                                                             \
          LANE_LOOP {                                                                   \
            if (LV(_l) == L) {                                                          \
              const uint64_t below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;      \
              (A).sorted[_nx[L] + hz::popc64(below)] = (uint16_t)(_c + lane);           \
            }                                                                           \
          }                                                                             \
          _nx[L] += (uint32_t)hz::popc64(m);                                            \
        }                                                                               \
      }                                                                                 \
    }                                                                                   \
    HZ_TB_SYNC();                                                                        \
    /* LUT fill: every root index tested against each length's canonical range (no   \
       loop-carried chain: a prefix-free code matches at most one length) */           \
    LANE_LOOP {                                                                         \
      for (int idx = lane; idx < (1 << (A).root); idx += 64) {                          \
        const uint32_t rc = hz::rev_bits((uint32_t)idx, (A).root);                      \
        uint32_t el = 1, es = hz::SYM_BAD;                                            \
        _Pragma("unroll") for (int len = 1; len <= 15; len++) {                         \
          if (len > (A).root) break;                                                    \
          const uint32_t d = (rc >> ((A).root - len)) - _fc[len];                       \
          if (d < _cn[len]) { el = (uint32_t)len; es = (A).sorted[_of[len] + d]; }      \
        }                                                                               \
        const uint32_t e = (A).rich ? hz::ent_rich((A).kind, el, es) : hz::ent_sym(el, es); \
        (A).lut[idx] = (uint16_t)e;                                                     \
      }                                                                                 \
    }                                                                                   \
    HZ_TB_SYNC();                                                                        \
    /* second level: one subtable per root prefix of longer codes.  Codes with the     \
       same prefix are contiguous in canonical order; the last of a run (the longest)  \
       sizes its subtable, and a scan over the runs places them */                      \
    const int _R = (A).root;                                                            \
    const int _k0 = (sh).tb_offs[_R + 1], _k1 = (sh).tb_offs[16];                       \
    if (_k1 > _k0) {                                                                    \
      uint32_t _used = 0;                                                               \
      for (int _b = _k0; _b < _k1; _b += 64) {                                          \
        LANE_VAR(uint32_t, _sz);                                                        \
        LANE_VAR(uint32_t, _pp);                                                        \
        LANE_VAR(uint32_t, _ox);                                                        \
        LANE_LOOP {                                                                     \
          const int k = _b + lane;                                                      \
          uint32_t sz = 0, p = 0;                                                       \
          if (k < _k1) {                                                                \
            const int l0 = (A).lens[(A).sorted[k]];                                     \
            p = (uint32_t)(((int)(sh).tb_first[l0] + (k - (int)(sh).tb_offs[l0])) >> (l0 - _R)); \
            int last = k + 1 == _k1;                                                    \
            if (!last) {                                                                \
              const int l1 = (A).lens[(A).sorted[k + 1]];                               \
              last = (uint32_t)(((int)(sh).tb_first[l1] + (k + 1 - (int)(sh).tb_offs[l1])) >> (l1 - _R)) != p; \
            }                                                                           \
            if (last) sz = (uint32_t)(l0 - _R);                                         \
            sz = last ? (1u << sz) | (sz << 24) : 0u;                                   \
          }                                                                             \
          LV(_sz) = sz; LV(_pp) = p;                                                    \
        }                                                                               \
        uint32_t _tot;                                                                  \
        HZ_SCAN_LOW24(_sz, _ox, _tot);                                                  \
        LANE_LOOP {                                                                     \
          if (LV(_sz))                                                                  \
            (A).lut[hz::rev_bits(LV(_pp), _R)] =                                        \
                hz::ent_sub(_used + LV(_ox), LV(_sz) >> 24);                             \
        }                                                                               \
        _used += _tot;                                                                  \
      }                                                                                 \
      /* <= nsub for every complete code (see LL_SUB/D_SUB); a table that would not    \
         fit is rejected before any subtable entry is written */                        \
      LANE_LOOP { if (lane == 0 && _used > (uint32_t)(A).nsub) (sh).u_status = hz::ST_DATA; } \
      HZ_TB_SYNC();                                                                      \
      /* fill subtables by symbol (zlib-style replication) */                           \
      LANE_LOOP {                                                                       \
        for (int k = _k0 + lane; k < _k1 && (sh).u_status == hz::ST_OK; k += 64) {      \
          const uint32_t sym = (A).sorted[k];                                           \
          const int len = (A).lens[sym];                                                \
          const int c = (int)(sh).tb_first[len] + (k - (int)(sh).tb_offs[len]);         \
          const int p = c >> (len - _R);                                                \
          const uint32_t re = (A).lut[hz::rev_bits((uint32_t)p, _R)];                   \
          if (re & 15u) continue;                                                       \
          const int sb = (int)(re >> 13), off = (1 << _R) + (int)((re >> 4) & 511u);    \
          const int tl = len - _R;                                                      \
          const uint32_t j0 = hz::rev_bits((uint32_t)(c & ((1 << tl) - 1)), tl);        \
          const uint16_t e = (A).rich ? hz::ent_rich((A).kind, (uint32_t)len, sym) : hz::ent_sym((uint32_t)len, sym); \
          for (int m = 0; m < (1 << (sb - tl)); m++) (A).lut[off + (j0 | (m << tl))] = e; \
        }                                                                               \
      }                                                                                 \
      HZ_TB_SYNC();                                                                      \
    }                                                                                   \
    status_out = (sh).u_status;                                                         \
  } while (0)

namespace hz {

// Work description for one zlib stream.
struct StreamJob {
  const uint8_t* src;   // stream bytes (any alignment)
  uint32_t src_len;
  uint8_t* dst;         // output
  uint32_t dst_len;     // expected size (exact) or capacity (exact == 0)
  uint32_t exact;       // 1: output must be exactly dst_len bytes
  uint32_t* out_len;    // optional: decoded length
};

// Tunables (runtime so that tests can sweep them)
struct Tune {
  uint32_t L0;     // initial segment bits
  uint32_t W;      // warm-up bits
  uint32_t adapt;  // 0: fixed L; 1: adapt L to the token density; n > 1: same, aiming at n/16 of SLOTS slots
  uint32_t C;      // continuation budget (bits)
  int max_rounds;  // repair rounds per window
};

// Statistics (emulator / diagnostics only)
struct Stats {
  uint64_t windows, lanes_valid, tokens, matches, match_bytes, lit_bytes, rounds, blocks, stored;
  uint64_t steps_max, steps_sum, repairs, hops, maxhops;
};

}  // namespace hz

// ===========================================================================
// The stream decoder.  `sh` is the wave's LDS block.  Returns a status code
// (uniform).  Written in SIMT style: code outside LANE_LOOP is uniform across the
// wave and runs redundantly on every lane; LANE_LOOP bodies never break/continue
// at their top level and never return.
// ===========================================================================
#define HZ_STAGE(sh, base_al, lo, hi, first_word, nwords)                          \
  do {                                                                              \
    WAVE_SYNC();                                                                    \
    LANE_LOOP {                                                                     \
      for (uint32_t _k = (uint32_t)lane; _k < (uint32_t)(nwords) + 4u; _k += 64)    \
        (sh).in32[_k] = _k < (uint32_t)(nwords)                                     \
                            ? hz::load_word((base_al), (first_word) + _k, (lo), (hi)) : 0u; \
    }                                                                               \
    (sh).u_stage_base = (first_word) * 32u;                                          \
    WAVE_SYNC();                                                                    \
  } while (0)

namespace hz {

template <class StatsT>
#if HZ_GPU
__device__
#else
static
#endif
int inflate_stream(Shared& sh, const StreamJob job, const Tune tune, StatsT* stats, HzProf* prof = nullptr) {
  (void)prof;
  // aligned base so that every staged dword load is aligned
  const uint32_t a = (uint32_t)(((uintptr_t)job.src) & 3u);
  hz_gcu8* base = HZ_GLOBAL(hz_gcu8*, job.src - a);
  const uint32_t lo = a, hi = a + job.src_len;   // valid byte range of the stream
  const uint32_t limit_bits = hi * 8u;
  const uint32_t dst_len = job.dst_len;
  hz_gu8* const dst = HZ_GLOBAL(hz_gu8*, job.dst);

  LANE_VAR(uint32_t, s1);   // adler32 partial sums: S1 = sum b, S2 = sum pos*b (mod 65521)
  LANE_VAR(uint32_t, s2);
  LANE_LOOP { LV(s1) = 0; LV(s2) = 0; }

  // ---- zlib header (RFC 1950) ----
  if (job.src_len < 2) return ST_TRUNC;
  HZ_STAGE(sh, base, lo, hi, 0u, 2u);
  {
    uint32_t hdr16 = (uint32_t)(peek64(&sh, lo * 8u) & 0xffffu);
    uint32_t cmf = hdr16 & 0xff, flg = hdr16 >> 8;
    if ((cmf & 0x0f) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0) return ST_DATA;
    if (flg & 0x20) return ST_DATA;  // preset dictionary: Z_NEED_DICT
  }
  uint32_t pos = lo * 8u + 16u;
  uint32_t out = 0;
  uint32_t L = tune.L0 < (uint32_t)LMIN ? (uint32_t)LMIN : tune.L0 > (uint32_t)LMAX ? (uint32_t)LMAX : tune.L0;

  for (;;) {  // ---- deflate blocks ----
    HZ_T(1);
    HZ_STAGE(sh, base, lo, hi, pos >> 5, 128u);
    if (pos + 3u > limit_bits) return ST_TRUNC;
    const uint32_t h3 = (uint32_t)(peek64(&sh, pos) & 7u);
    pos += 3;
    const uint32_t bfinal = h3 & 1u, btype = h3 >> 1;
    if (stats) stats->blocks++;
    if (btype == 3) return ST_DATA;
    if (btype == 0) {
      // ---- stored block ----
      pos = (pos + 7u) & ~7u;
      if (pos + 32u > limit_bits) return ST_TRUNC;
      const uint32_t ln = (uint32_t)(peek64(&sh, pos) & 0xffffffffu);
      const uint32_t len = ln & 0xffffu, nlen = ln >> 16;
      if ((len ^ 0xffffu) != nlen) return ST_DATA;
      pos += 32u;
      if (pos + len * 8u > limit_bits) return ST_TRUNC;
      if (out + len > dst_len) return ST_SIZE;
      const uint32_t sb = pos >> 3;  // byte index relative to the aligned base
      LANE_LOOP {
        uint32_t a1 = LV(s1), a2 = LV(s2);
        for (uint32_t i = (uint32_t)lane; i < len; i += 64) {
          const uint32_t b = base[sb + i];
          dst[out + i] = (uint8_t)b;
          a1 += b;
          a2 = (uint32_t)((a2 + (uint64_t)((out + i) % ADLER_MOD) * b) % ADLER_MOD);
        }
        LV(s1) = a1 % ADLER_MOD; LV(s2) = a2;
      }
      out += len;
      pos += len * 8u;
      if (stats) stats->stored++;
      WAVE_SYNC_GLOBAL();
      if (bfinal) break;
      continue;
    }
    // ---- Huffman code lengths ----
    HZ_T(2);
    uint32_t nlen = 288, ndist = 32;
    if (btype == 1) {
      LANE_LOOP {
        for (int s = lane; s < 320; s += 64)
          sh.lens[s] = s >= 288 ? 5 : s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      }
      WAVE_SYNC();
    } else {
      // dynamic header (RFC 1951 3.2.7): lane 0 decodes it serially from the staged
      // input with a register bit reader and a 7-bit code-length lookup table
      LANE_LOOP {
        if (lane == 0) {
          int st = ST_OK;
          BitRd r;
          br_init(&sh, r, pos, sh.u_stage_base);
          br_fill(&sh, r);
          const uint32_t hlit = (uint32_t)(r.bb & 31u) + 257u, hdist = (uint32_t)((r.bb >> 5) & 31u) + 1u;
          const uint32_t hclen = (uint32_t)((r.bb >> 10) & 15u) + 4u;
          br_drop(r, 14);
          if (hlit > 286 || hdist > 30) st = ST_DATA;
          uint16_t* cl = sh.sorted_cl;               // code-length code lengths (19)
          for (int i = 0; i < 19; i++) cl[i] = 0;
          for (uint32_t i = 0; i < hclen; i++) {
            br_fill(&sh, r);
            cl[cl_order(i)] = (uint16_t)(r.bb & 7u);
            br_drop(r, 3);
          }
          uint16_t* cnt = sh.cnt_cl;
          for (int l = 0; l < 16; l++) cnt[l] = 0;
          for (int i = 0; i < 19; i++) cnt[cl[i]]++;
          cnt[0] = 0;
          int left = 1, maxl = 0;
          for (int l = 1; l <= 7; l++) {
            left <<= 1; left -= cnt[l];
            if (cnt[l]) maxl = l;
            if (left < 0) st = ST_DATA;
          }
          if (left > 0 || maxl == 0) st = ST_DATA;  // code-length code must be complete
          // 7-bit LUT (sym | len << 8) in the distance table's space (rebuilt below)
          uint16_t* clut = sh.lut_d;
          if (st == ST_OK) {
            uint32_t next[8];
            uint32_t code = 0;
            for (int l = 1; l <= 7; l++) { code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1; next[l] = code; }
            for (int i = 0; i < 19; i++) {
              const uint32_t l = cl[i];
              if (!l) continue;
              const uint32_t rc = rev_bits(next[l]++, (int)l);
              for (uint32_t k = rc; k < 128u; k += 1u << l) clut[k] = (uint16_t)(i | (l << 8));
            }
          }
          const uint32_t total = hlit + hdist;
          uint32_t n = 0;
          const uint32_t stage_end = sh.u_stage_base + 128u * 32u;
          while (st == ST_OK && n < total) {
            if (r.pos + 64u > stage_end) { st = ST_DATA; break; }   // header longer than any valid one
            br_fill(&sh, r);
            const uint32_t e = clut[r.bb & 127u];
            const uint32_t sym = e & 0xffu, l = e >> 8;
            br_drop(r, l);
            if (sym < 16) { sh.lens[n++] = (uint8_t)sym; continue; }
            uint32_t rep, val = 0;
            if (sym == 16) {
              if (n == 0) { st = ST_DATA; break; }
              val = sh.lens[n - 1]; rep = 3 + (uint32_t)(r.bb & 3u); br_drop(r, 2);
            } else if (sym == 17) { rep = 3 + (uint32_t)(r.bb & 7u); br_drop(r, 3); }
            else { rep = 11 + (uint32_t)(r.bb & 127u); br_drop(r, 7); }
            if (n + rep > total) { st = ST_DATA; break; }
            for (uint32_t k = 0; k < rep; k++) sh.lens[n++] = (uint8_t)val;
          }
          if (st == ST_OK && r.pos > limit_bits) st = ST_TRUNC;
          if (st == ST_OK && sh.lens[256] == 0) st = ST_DATA;  // missing end-of-block code
          if (st == ST_OK) {
            for (int i = (int)hdist - 1; i >= 0; i--) sh.lens[288 + i] = sh.lens[hlit + i];
            for (uint32_t i = hlit; i < 288; i++) sh.lens[i] = 0;
            for (uint32_t i = 288 + hdist; i < 320; i++) sh.lens[i] = 0;
          }
#if !HZ_GPU && defined(HZ_DEBUG)
          { unsigned long long hsh = 0; for (uint32_t i = 0; i < 320; i++) hsh = hsh * 31 + sh.lens[i];
            printf("HDR pos=%u end=%u hlit=%u hdist=%u st=%d hash=%llu\n", pos, r.pos, hlit, hdist, st, hsh); }
#endif
          sh.u_status = st;
          sh.u_pos = r.pos;
          sh.u_nlen = hlit;
          sh.u_ndist = hdist;
        }
      }
      WAVE_SYNC();
      const int hst = sh.u_status;
      if (hst != ST_OK) return hst;
      pos = sh.u_pos;
      nlen = sh.u_nlen;
      ndist = sh.u_ndist;
    }
    {
      int bst = ST_OK;
      TableArgs tll = {sh.lens, (int)nlen, sh.cnt_ll, sh.sorted_ll, sh.lut_ll, LL_ROOT, 1, LL_SUB};
      HZ_T(3);
      HZ_BUILD_TABLE(sh, tll, bst);
      if (bst != ST_OK) return bst;
      TableArgs td = {sh.lens + 288, (int)ndist, sh.cnt_d, sh.sorted_d, sh.lut_d, D_ROOT, 2, D_SUB};
      HZ_BUILD_TABLE(sh, td, bst);
      if (bst != ST_OK) return bst;
    }

    // ---- windows over the Huffman block ----
    for (;;) {
      if (stats) stats->windows++;
      HZ_T(4);
      const uint32_t win_start = pos;
      // a continuation never runs past its successor's segment: phase B counts a
      // lane's valid tokens from the point where its predecessor met its marks
      const uint32_t W = tune.W, C = tune.C < L ? tune.C : L;
      {
        const uint32_t first_bit = win_start >= W ? win_start - W : 0u;
        const uint32_t words = (64u * L + W + C + 256u) / 32u + 3u;
        HZ_STAGE(sh, base, lo, hi, first_bit >> 5, words);
      }

      HZ_T(5);
      // -------- Phase A: speculative decode of 64 segments --------
      // lane i decodes from (segment start - W); tokens whose start lies inside its
      // own segment [ss, ss+L) are stored and their start bits marked.
      const uint32_t stage_base = ((win_start >= W ? win_start - W : 0u) >> 5) * 32u;
      LANE_VAR(uint32_t, seg_start);
      LANE_VAR(uint32_t, ntok);      // tokens stored
      LANE_VAR(uint32_t, nslot);     // slots they use
      LANE_VAR(uint64_t, mbits);     // bit k: token k is a match (two slots)
      LANE_VAR(int, storing);
      LANE_VAR(uint32_t, nsteps);
      LANE_LOOP {
        const uint32_t ss = win_start + (uint32_t)lane * L;
        const uint32_t se = ss + L;
        const uint32_t p0 = (lane > 0 && ss - win_start > W) ? ss - W : win_start;
        int st = p0 >= ss;
        uint32_t nt = 0, ns = 0, steps = 0;
        uint64_t mb = 0;
        for (int w = 0; w < BM_WORDS; w++) sh.bitmap[lane][w] = 0;
        uint32_t mw_idx = 0, mw = 0;  // bitmap word cached in a register (monotonic positions)
        BitRd r;
        br_init(&sh, r, p0, stage_base);
        while (r.pos < se) {
          if (!st && r.pos >= ss) st = 1;
          if (st && ns + 2u > (uint32_t)SLOTS) break;
          const uint32_t tp = r.pos;
          const uint32_t tokv = next_token(&sh, r);
          steps++;
          if (st) {
            const uint32_t rel = tp - ss, wi = rel >> 5;
            if (wi != mw_idx) { sh.bitmap[lane][mw_idx] |= mw; mw = 0; mw_idx = wi; }
            mw |= 1u << (rel & 31u);
            const uint32_t w = put_tok(&sh, lane, ns, tokv);
            mb |= (uint64_t)(w - 1u) << nt;
            ns += w;
            nt++;
          }
        }
        if (st) {
          sh.bitmap[lane][mw_idx] |= mw;
          mark_bit(&sh, lane, r.pos - ss);   // exit boundary (start of the next token)
        }
        LV(seg_start) = ss;
        LV(ntok) = nt;
        LV(nslot) = ns;
        LV(mbits) = mb;
        LV(storing) = st;
        LV(nsteps) = steps;
        sh.exitpos[lane] = r.pos;
        sh.syncpos[lane] = 0xffffffffu;
      }
      WAVE_SYNC();

      HZ_T(6);
      // -------- Phase A': continuation --------
      // lane i keeps decoding from its exit until it reaches a token start that
      // lane i+1 marked (then both decodes coincide from there on), for at most C
      // bits into segment i+1.  Tokens decoded here belong to lane i.
      LANE_LOOP {
        const uint32_t ss = LV(seg_start);
        uint32_t nt = LV(ntok), ns = LV(nslot), steps = 0;
        uint64_t mb = LV(mbits);
        uint32_t pend = sh.exitpos[lane];
        if (lane < 63 && LV(storing)) {
          const uint32_t ssn = ss + L;
          BitRd r;
          br_init(&sh, r, pend, stage_base);
          uint32_t nw_idx = 0xffffffffu, nw = 0;     // cached word of lane+1's bitmap
          uint32_t mw_idx = (r.pos - ss) >> 5, mw = 0;
          for (;;) {
            const uint32_t reln = r.pos - ssn;
            if (r.pos >= ssn && reln < (uint32_t)(BM_WORDS * 32)) {
              if ((reln >> 5) != nw_idx) { nw_idx = reln >> 5; nw = sh.bitmap[lane + 1][nw_idx]; }
              if ((nw >> (reln & 31u)) & 1u) { sh.syncpos[lane + 1] = r.pos; break; }
            }
            if (r.pos >= ssn + C || ns + 2u > (uint32_t)SLOTS) break;
            const uint32_t rel = r.pos - ss, wi = rel >> 5;
            const uint32_t tokv = next_token(&sh, r);
            steps++;
            if (wi != mw_idx) { sh.bitmap[lane][mw_idx] |= mw; mw = 0; mw_idx = wi; }
            mw |= 1u << (rel & 31u);
            const uint32_t w = put_tok(&sh, lane, ns, tokv);
            mb |= (uint64_t)(w - 1u) << nt;
            ns += w;
            nt++;
          }
          if (mw_idx < (uint32_t)BM_WORDS) sh.bitmap[lane][mw_idx] |= mw;
          pend = r.pos;
          mark_bit(&sh, lane, pend - ss);     // final boundary of this lane's decode
        }
        LV(ntok) = nt;
        LV(nslot) = ns;
        LV(mbits) = mb;
        LV(nsteps) += steps;
        sh.contpos[lane] = pend;
      }
      WAVE_SYNC();
      HZ_T(7);
      // -------- repair rounds --------
      // A lane whose predecessor's continuation never met one of its marks is
      // "failed": its speculative path had not merged with the true path.  It
      // re-decodes its segment from the predecessor's final position (a true token
      // boundary once the predecessor is valid) and continues into its successor.
      LANE_VAR(int, failed);
      LANE_LOOP {
        LV(failed) = lane > 0 && sh.syncpos[lane] == 0xffffffffu;
        sh.flag[lane] = (uint32_t)LV(failed);
      }
      WAVE_SYNC();
#if !HZ_GPU
      uint32_t rsteps[64] = {0};
#endif
      for (int round = 0; round < tune.max_rounds; round++) {
        const uint64_t fm = WAVE_BALLOT(LV(failed));
        if (!fm) break;
        if (stats) stats->repairs++;
        LANE_LOOP {
          const int redo = LV(failed) && !sh.flag[lane - 1 < 0 ? 0 : lane - 1] &&
                           sh.contpos[lane - 1 < 0 ? 0 : lane - 1] >= LV(seg_start);
          const int next_failed = lane < 63 ? (int)sh.flag[lane + 1] : 1;
          uint32_t steps = 0;
          if (redo) {
            // re-decode from the predecessor's true exit; as soon as the true path
            // lands on a token start of this lane's own speculative path, the rest
            // of that path (tokens, continuation, successor sync) is already right:
            // splice it in instead of decoding it again
            const uint32_t ss = LV(seg_start), se = ss + L;
            const uint32_t old_nt = LV(ntok), old_ns = LV(nslot);
            const uint64_t old_mb = LV(mbits);
            const uint32_t start = sh.contpos[lane - 1];
            const uint32_t old_sync_next = lane < 63 ? sh.syncpos[lane + 1] : 0xffffffffu;
            if (lane < 63 && !next_failed) sh.syncpos[lane + 1] = 0xffffffffu;
            uint32_t cw = (start - ss) >> 5;          // bitmap word being rewritten
            uint32_t oldc = 0;                        // old marks below word cw
            for (uint32_t w = 0; w < cw && w < (uint32_t)BM_WORDS; w++) {
              oldc += popc32(sh.bitmap[lane][w]);
              sh.bitmap[lane][w] = 0;
            }
            uint32_t ow = cw < (uint32_t)BM_WORDS ? sh.bitmap[lane][cw] : 0u;   // its old marks
            uint32_t mw = 0;                          // its new marks
            uint32_t nt = 0, ns = 0;
            uint64_t mb = 0;
            int merged = 0, nomerge = 0;
            BitRd r;
            br_init(&sh, r, start, stage_base);
            uint32_t nw_idx = 0xffffffffu, nw = 0;
            for (;;) {
              const uint32_t rel = r.pos - ss, wi = rel >> 5;
              if (wi != cw) {
                oldc += popc32(ow);
                if (cw < (uint32_t)BM_WORDS) sh.bitmap[lane][cw] = mw;
                for (uint32_t w = cw + 1; w < wi && w < (uint32_t)BM_WORDS; w++) {
                  oldc += popc32(sh.bitmap[lane][w]);
                  sh.bitmap[lane][w] = 0;
                }
                cw = wi; mw = 0;
                ow = wi < (uint32_t)BM_WORDS ? sh.bitmap[lane][wi] : 0u;
              }
              const uint32_t jcur = oldc + popc32(ow & bmask(rel & 31u));   // old tokens before here
              const uint32_t scur = jcur <= old_nt ? tok_slot(old_mb, jcur) : old_ns;   // their slots
              if (((ow >> (rel & 31u)) & 1u) && !nomerge && jcur <= old_nt) {
                // ns <= scur: new tokens only ever overwrote old slots below scur
                sh.bitmap[lane][cw] = mw | (ow & ~bmask(rel & 31u));
                if (ns < scur) {
                  for (uint32_t t = scur; t < old_ns; t++) sh.tok[tok_idx(ns + t - scur, lane)] = sh.tok[tok_idx(t, lane)];
                }
                mb |= (old_mb >> jcur) << nt;
                ns += old_ns - scur;
                nt += old_nt - jcur;
                merged = 1;
                break;
              }
              if (r.pos >= se) {                      // continuation into the successor
                if (lane == 63 || next_failed) break;
                const uint32_t reln = r.pos - se;
                if (reln < (uint32_t)(BM_WORDS * 32)) {
                  if ((reln >> 5) != nw_idx) { nw_idx = reln >> 5; nw = sh.bitmap[lane + 1][nw_idx]; }
                  if ((nw >> (reln & 31u)) & 1u) { sh.syncpos[lane + 1] = r.pos; break; }
                }
                if (r.pos >= se + C) break;
              }
              if (ns + 2u > (uint32_t)SLOTS) break;
              const uint32_t tokv = next_token(&sh, r);
              steps++;
              mw |= 1u << (rel & 31u);
              const uint32_t w = (tokv & T_MATCH) ? 2u : 1u;
              if (ns + w > scur) nomerge = 1;         // would overwrite a possibly needed old slot
              put_tok(&sh, lane, ns, tokv);
              mb |= (uint64_t)(w - 1u) << nt;
              ns += w;
              nt++;
            }
#if !HZ_GPU && defined(HZ_DEBUG)
            if (!merged) printf("NOMERGE lane=%d L=%u start=%u end=%u old_nt=%u nt=%u nomerge=%d next_failed=%d oldc=%u se=%u\n", lane, L, start - ss, r.pos - ss, old_nt, nt, nomerge, next_failed, oldc, se - ss);
#endif
            if (merged) {
              if (lane < 63) sh.syncpos[lane + 1] = old_sync_next;   // the old continuation stands
            } else {
              // final boundary mark; old marks at or after it are stale
              const uint32_t rel = r.pos - ss;
              if (cw < (uint32_t)BM_WORDS) sh.bitmap[lane][cw] = mw;
              for (uint32_t w = cw + 1; w < (uint32_t)BM_WORDS; w++) sh.bitmap[lane][w] = 0;
              mark_bit(&sh, lane, rel);
              sh.contpos[lane] = r.pos;
            }
            sh.syncpos[lane] = start;                 // whole token list is valid
            LV(ntok) = nt;
            LV(nslot) = ns;
            LV(mbits) = mb;
            if (stats) { stats->matches++; stats->match_bytes += (uint64_t)merged; }
          }
          LV(nsteps) += steps;
#if !HZ_GPU
          rsteps[lane] = steps;
#endif
          sh.flag2[lane] = (uint32_t)redo;
        }
        WAVE_SYNC();
#if !HZ_GPU
        if (stats) { uint32_t mx = 0; for (int l = 0; l < 64; l++) mx = rsteps[l] > mx ? rsteps[l] : mx; stats->lit_bytes += mx; }
#endif
        LANE_LOOP {
          if (sh.flag2[lane]) LV(failed) = 0;
          else if (lane > 0 && sh.flag2[lane - 1] && sh.syncpos[lane] == 0xffffffffu) LV(failed) = 1;
        }
        WAVE_SYNC();
        LANE_LOOP { sh.flag[lane] = (uint32_t)LV(failed); }
        WAVE_SYNC();
      }
      if (stats) {
#if !HZ_GPU
        uint32_t mx = 0; uint64_t sm = 0;
        for (int lane = 0; lane < 64; lane++) { mx = nsteps[lane] > mx ? nsteps[lane] : mx; sm += nsteps[lane]; }
        stats->steps_max += mx; stats->steps_sum += sm;
#endif
      }

      HZ_T(8);
      // -------- Phase B: validity --------
      LANE_VAR(uint32_t, tok_first);
      LANE_VAR(uint32_t, tok_end);
      LANE_VAR(int, endk);       // 0 none, 1 EOB, 2 ERR inside the valid range
      LANE_LOOP {
        uint32_t tf = 0;
        int ok = lane == 0;
        if (lane > 0 && sh.syncpos[lane] != 0xffffffffu && !LV(failed)) {
          ok = 1;
          const uint32_t sp = sh.syncpos[lane];
          const uint32_t rel = sp >= LV(seg_start) ? sp - LV(seg_start) : 0u;
          uint32_t c = 0;
          for (uint32_t w = 0; w < (rel >> 5); w++) c += popc32(sh.bitmap[lane][w]);
          c += popc32(sh.bitmap[lane][rel >> 5] & bmask(rel & 31u));
          tf = c;
        }
        uint32_t te = LV(ntok);
        int ek = 0;
        if (ok) {
          uint32_t sl = tok_slot(LV(mbits), tf);
          for (uint32_t t = tf; t < te; t++) {
            const uint32_t v = tok_at(&sh, sl, lane);
            if (v == S_EOB || v == S_ERR) { ek = v == S_EOB ? 1 : 2; te = t; break; }
            sl += (v & S_MATCH) ? 2u : 1u;
          }
        }
        LV(tok_first) = ok ? tf : 0xffffffffu;
        LV(tok_end) = te;
        LV(endk) = ek;
      }
      const uint64_t smask = WAVE_BALLOT(LV(tok_first) != 0xffffffffu);
      uint32_t V = 0;
      while (V < 64u && ((smask >> V) & 1ull)) V++;
      const uint64_t emask = WAVE_BALLOT(LV(endk) != 0) & (V >= 64 ? ~0ull : ((1ull << V) - 1ull));
      int end_lane = -1;
      for (uint32_t k = 0; k < V; k++) if ((emask >> k) & 1ull) { end_lane = (int)k; break; }
      if (end_lane >= 0) V = (uint32_t)end_lane + 1u;
      if (stats) stats->lanes_valid += V;

      HZ_T(9);
      // -------- Phase C: emit --------
      LANE_VAR(uint32_t, tcur);
      LANE_VAR(uint32_t, tend);
      LANE_VAR(uint32_t, olen);
      LANE_LOOP {
        uint32_t tf = LV(tok_first), te = LV(tok_end), ol = 0;
        if ((uint32_t)lane >= V) { tf = 0; te = 0; }
        if (lane == end_lane) {
          sh.u_status = LV(endk);
          // bit position after the EOB token = the mark following token te
          sh.u_pos = nth_mark(&sh, lane, te + 1u) + LV(seg_start);
        }
        const uint32_t sf = tok_slot(LV(mbits), tf);
        uint32_t sl = sf;
        for (uint32_t t = tf; t < te; t++) {
          const uint32_t v = tok_at(&sh, sl, lane);
          const uint32_t m = v & S_MATCH;
          ol += m ? (v & 0xffu) + 3u : 1u;
          sl += m ? 2u : 1u;
        }
        LV(tcur) = sf; LV(tend) = sl; LV(olen) = ol;
      }
      WAVE_SYNC();
      if (end_lane >= 0 && sh.u_status == 2) {
        return sh.u_pos + 64u > limit_bits ? ST_TRUNC : ST_DATA;
      }
      HZ_T(10);
      // output offsets; the window keeps only what fits the LDS reference map
      LANE_VAR(uint32_t, obase);
#if HZ_GPU
      obase = wave_excl_scan(olen, HZ_LANE_ID());
#else
      { uint32_t acc = 0; for (int lane = 0; lane < 64; lane++) { obase[lane] = acc; acc += olen[lane]; } }
#endif
      uint32_t npos;
      {
        const uint64_t over = WAVE_BALLOT((uint32_t)lane < V && LV(obase) + LV(olen) > (uint32_t)SCAP);
        uint32_t k = 0;
        while (k < V && !((over >> k) & 1ull)) k++;
        if (k < V) {
          if (k == 0) {
            // lane 0 alone overflows: keep its first tokens that fit (>= 1 token)
            LANE_LOOP {
              if (lane == 0) {
                uint32_t sl = LV(tcur), t = 0, acc = 0;     // lane 0's tokens start at token 0
                while (sl < LV(tend)) {
                  const uint32_t v = tok_at(&sh, sl, lane);
                  const uint32_t m = v & S_MATCH;
                  const uint32_t n = m ? (v & 0xffu) + 3u : 1u;
                  if (acc + n > (uint32_t)SCAP) break;
                  acc += n; sl += m ? 2u : 1u; t++;
                }
                LV(tend) = sl; LV(olen) = acc;
                sh.u_pos = win_start + nth_mark(&sh, lane, t);
              }
            }
            WAVE_SYNC();
            npos = sh.u_pos;
            V = 1;
          } else {
            V = k;
            npos = sh.contpos[k - 1];
          }
          end_lane = -1;                 // an EOB beyond the cut is met again next window
          LANE_LOOP { if ((uint32_t)lane >= V) { LV(tcur) = 0; LV(tend) = 0; LV(olen) = 0; } }
        } else {
          npos = end_lane >= 0 ? sh.u_pos : sh.contpos[V - 1];
        }
      }
      uint32_t wtotal = 0, ntok_valid = 0;
#if HZ_GPU
      wtotal = wave_sum(olen);
      ntok_valid = wave_sum(tend - tcur);
#else
      for (int lane = 0; lane < 64; lane++) { wtotal += olen[lane]; ntok_valid += tend[lane] - tcur[lane]; }
#endif
      if (stats) stats->tokens += ntok_valid;
      if (out + wtotal > dst_len) return ST_SIZE;
      if (npos > limit_bits) return ST_TRUNC;

      // ---- byte-level source map in LDS ----
      // ref[r] for window byte r: 0x4000|b literal, r' < 0x4000 internal reference,
      // 0x8000|(x-1) the byte x positions before the window (final in dst).
      const uint32_t wbeg = out;
      // publish per-lane token ranges so that any lane can walk any lane's tokens
      LANE_LOOP {
        sh.obase[lane] = LV(obase);
        sh.tcur_l[lane] = (uint16_t)LV(tcur);
        sh.tend_l[lane] = (uint16_t)LV(tend);
        if (lane == 63) sh.obase[64] = wtotal;
      }
      WAVE_SYNC();
      LANE_VAR(int, lerr);
      LANE_LOOP {
        // lane w produces the references of output bytes [w*B, (w+1)*B): balanced
        // whatever the token / output distribution across the owning lanes
        int err = 0;
        const uint32_t B = (wtotal + 63u) >> 6;
        const uint32_t x0 = (uint32_t)lane * B;
        const uint32_t x1 = x0 + B < wtotal ? x0 + B : wtotal;
        if (x0 < x1) {
          int lo_j = 0, hi_j = 63;                 // owner: largest j with obase[j] <= x0
          while (lo_j < hi_j) {
            const int mid = (lo_j + hi_j + 1) >> 1;
            if (sh.obase[mid] <= x0) lo_j = mid; else hi_j = mid - 1;
          }
          int j = lo_j;
          uint32_t t = sh.tcur_l[j], q = sh.obase[j];     // t: slot of lane j
          uint32_t v, d;
          tok_pair(&sh, t, j, v, d);
          uint32_t m = v & S_MATCH;
          uint32_t n = m ? (v & 0xffu) + 3u : 1u;
          while (q + n <= x0) {                    // token of lane j containing x0
            q += n; t += m ? 2u : 1u;
            tok_pair(&sh, t, j, v, d);
            m = v & S_MATCH;
            n = m ? (v & 0xffu) + 3u : 1u;
          }
          d = m ? d : 1u;
          uint32_t jj = m ? (x0 - q) % d : 0u;
          int32_t base = (int32_t)q - (int32_t)d;
          uint32_t tend_j = sh.tend_l[j];
          if (m && d > wbeg + q) err = 1;
          for (uint32_t x = x0; x < x1 && !err; x++) {
            if (x == q + n) {                      // next token (possibly of the next lane)
              q = x; t += m ? 2u : 1u;
              while (t >= tend_j) { j++; t = sh.tcur_l[j]; tend_j = sh.tend_l[j]; }
              tok_pair(&sh, t, j, v, d);
              m = v & S_MATCH;
              n = m ? (v & 0xffu) + 3u : 1u;
              d = m ? d : 1u;
              base = (int32_t)q - (int32_t)d;
              jj = 0;
              if (m && d > wbeg + q) { err = 1; break; }
            }
            const int32_t srcq = base + (int32_t)jj;
            const uint32_t rv = !m ? (0x4000u | v)
                              : srcq >= 0 ? (uint32_t)srcq : (0x8000u | (uint32_t)(-srcq - 1));
            sh.ref[x] = (uint16_t)rv;
            jj++;
            jj = jj == d ? 0u : jj;
          }
        }
        LV(lerr) = err;
      }
      WAVE_SYNC();
      if (WAVE_BALLOT(LV(lerr))) return ST_DATA;
      if (stats) stats->rounds++;
      HZ_T(11);
      // chase: references strictly decrease, so every chain ends in a literal or an
      // external byte; resolved values are written back (benign races: every stored
      // value is a valid ancestor of the position)
      LANE_LOOP {
        for (uint32_t r = (uint32_t)lane; r < wtotal; r += 64) {
          uint32_t v = sh.ref[r];
          uint32_t hops = 0;
          while (v < 0x4000u) { v = sh.ref[v]; hops++; }
          sh.ref[r] = (uint16_t)v;
          if (stats) { stats->hops += hops; if (hops > stats->maxhops) stats->maxhops = hops; }
        }
      }
      WAVE_SYNC();
      // external bytes: gather from dst, 8 independent loads in flight per lane
      LANE_LOOP {
        for (uint32_t r0 = (uint32_t)lane; r0 < wtotal; r0 += 64u * 8u) {
          uint32_t v[8], b[8];
HZ_UNROLL
          for (int k = 0; k < 8; k++) {
            const uint32_t r = r0 + 64u * (uint32_t)k;
            v[k] = r < wtotal ? sh.ref[r] : 0x4000u;
          }
HZ_UNROLL
          for (int k = 0; k < 8; k++) b[k] = (v[k] & 0x8000u) ? (uint32_t)dst[wbeg - (v[k] & 0x7fffu) - 1u] : v[k];
HZ_UNROLL
          for (int k = 0; k < 8; k++) {
            const uint32_t r = r0 + 64u * (uint32_t)k;
            if (r < wtotal && (v[k] & 0x8000u)) sh.ref[r] = (uint16_t)b[k];
          }
        }
      }
      WAVE_SYNC();
      HZ_T(12);
      // flush: 4-byte stores (byte stores at the unaligned head / tail) + adler sums
      LANE_LOOP {
        uint32_t b1 = 0, b2 = 0;                  // sum b, sum r*b over this lane's bytes
        const uint32_t head = (uint32_t)((4u - (((uintptr_t)(dst + wbeg)) & 3u)) & 3u);
        const uint32_t h = head < wtotal ? head : wtotal;
        if ((uint32_t)lane < h) {
          const uint32_t bv = sh.ref[lane] & 0xffu;
          dst[wbeg + lane] = (uint8_t)bv;
          b1 += bv; b2 += (uint32_t)lane * bv;
        }
        for (uint32_t r = h + 4u * (uint32_t)lane; r < wtotal; r += 256u) {
          const uint32_t n = wtotal - r < 4u ? wtotal - r : 4u;
          uint32_t w = 0;
          for (uint32_t k = 0; k < n; k++) {
            const uint32_t bv = sh.ref[r + k] & 0xffu;
            w |= bv << (8u * k);
            b1 += bv; b2 += (r + k) * bv;
          }
          if (n == 4u) *(hz_gu32*)(dst + wbeg + r) = w;
          else for (uint32_t k = 0; k < n; k++) dst[wbeg + r + k] = (uint8_t)(w >> (8u * k));
        }
        LV(s1) = (LV(s1) + b1) % ADLER_MOD;
        LV(s2) = (uint32_t)((LV(s2) + (uint64_t)(wbeg % ADLER_MOD) * b1 + b2) % ADLER_MOD);
      }
      WAVE_SYNC_GLOBAL();
      if (stats) stats->lit_bytes += 0;
      HZ_T(14);
      out += wtotal;
      pos = npos;
      if (end_lane >= 0) break;        // EOB: the next block header follows
      // next segment length: about half of SLOTS token slots per segment (room for the
      // continuation) and an expected window output of about 3/4 of the LDS map
      if (tune.adapt) {
        const uint32_t used = npos - win_start;
        const uint32_t bpt16 = ntok_valid ? (used * 16u) / ntok_valid : 16u * 8u;   // bits/token x16
        const uint32_t fill16 = tune.adapt > 1u ? tune.adapt : ADAPT_FILL16;   // of SLOTS, /16
        uint32_t target = (bpt16 * (uint32_t)SLOTS * fill16) / (16u * 16u);   // bpt16: bits per slot
        if (wtotal && used) {
          const uint64_t lim = ((uint64_t)SCAP * HZ_SCAP_FILL8 / 8u) * used / ((uint64_t)wtotal * 64u);
          if (lim < target) target = (uint32_t)lim;
        }
        L = target < (uint32_t)LMIN ? (uint32_t)LMIN : target > (uint32_t)LMAX ? (uint32_t)LMAX : target;
      }
    }
    if (bfinal) break;
  }
  // ---- trailer: adler32 (big-endian) after byte alignment ----
  HZ_T(15);
  pos = (pos + 7u) & ~7u;
  if (pos + 32u > limit_bits) return ST_TRUNC;
  HZ_STAGE(sh, base, lo, hi, pos >> 5, 4u);
  const uint32_t t32 = (uint32_t)(peek64(&sh, pos) & 0xffffffffu);
  const uint32_t want = (t32 >> 24) | ((t32 >> 8) & 0xff00u) | ((t32 << 8) & 0xff0000u) | (t32 << 24);
  uint64_t S1 = 0, S2 = 0;
#if HZ_GPU
  S1 = wave_sum64((uint64_t)s1);
  S2 = wave_sum64((uint64_t)s2);
#else
  for (int lane = 0; lane < 64; lane++) { S1 += s1[lane]; S2 += s2[lane]; }
#endif
  const uint32_t A = (uint32_t)((1u + S1) % ADLER_MOD);
  const uint32_t B = (uint32_t)(((uint64_t)(out % ADLER_MOD) * A + ADLER_MOD - (S2 % ADLER_MOD)) % ADLER_MOD);
  if (((B << 16) | A) != want) return ST_DATA;
  if (job.exact && out != dst_len) return ST_SIZE;
  if (job.out_len) *job.out_len = out;
  return ST_OK;
}

}  // namespace hz
