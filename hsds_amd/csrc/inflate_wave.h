// inflate_wave.h -- shared pieces of the zlib (RFC 1950/1951) decoder in inflate2.h.
//
// The decoder itself (inflate2.h, inflate2_stream.inc) replaces, for the HSDS data-node hot
// path, the zlib inflate that the reference reaches through storUtil._uncompress
// (hsds/util/storUtil.py:209-220, CPython zlib.decompress) and through c-blosc's
// zlib_wrap_decompress for every Blosc split (storUtil.py:195-208).  This header holds what
// it shares with the other wave kernels:
//   * the single-source SIMT conventions (LANE_LOOP, LANE_VAR, WAVE_BALLOT, wave scans):
//     HIP (gfx950) runs every lane as a real SIMT lane and LANE_LOOP is one iteration; the
//     CPU emulation (tests/emu) iterates lanes 0..63 in order, so every cross-lane step is
//     unit-tested on CPU;
//   * status codes, the 16-bit decode-table entry formats (ent_sym / ent_sub / ent_rich);
//   * the cooperative canonical-Huffman table build (HZ_BUILD_TABLE, zlib inflate_table's
//     acceptance rules) and the global-memory word loader.
// (The round-1 decoder that lived here -- LDS-staged windows, token slots -- was retired in
// round 6; inflate2.h replaced it in round 2.)
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
#ifndef HZ_LL_ROOT
#define HZ_LL_ROOT 10
#endif
constexpr int LL_ROOT = HZ_LL_ROOT;
static_assert(LL_ROOT == 9 || LL_ROOT == 10, "literal/length root: 9 or 10 bits");
constexpr int D_ROOT = 8;
// second-level entries (codes longer than the root).  Sized at or above zlib's exact
// worst cases (ENOUGH: 286 symbols / root 10 -> 308 extra entries; 30 symbols /
// root 8 -> at most 3 x 128), so every complete code fits and no slow path exists.
#ifndef HZ_LL_SUB
#define HZ_LL_SUB (HZ_LL_ROOT == 9 ? 352 : 320)     // zlib ENOUGH_LENS - 2^root: 340 / 308
#endif
constexpr int LL_SUB = HZ_LL_SUB;
constexpr int D_SUB = 384;
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

// position of code-length symbol s in that order (the inverse of cl_order), s < 19
HZ_HD uint32_t cl_pos(uint32_t s) {
  // 0:3 1:17 2:15 3:13 4:11 5:9 6:7 7:5 8:4 9:6 10:8 11:10 | 12:12 13:14 14:16 15:18 16:0 17:1 18:2
  const uint64_t lo = 3ull | 17ull << 5 | 15ull << 10 | 13ull << 15 | 11ull << 20 | 9ull << 25 | 7ull << 30 |
                      5ull << 35 | 4ull << 40 | 6ull << 45 | 8ull << 50 | 10ull << 55;
  const uint64_t hi = 12ull | 14ull << 5 | 16ull << 10 | 18ull << 15 | 0ull << 20 | 1ull << 25 | 2ull << 30;
  return (uint32_t)((s < 12 ? lo >> (5 * s) : hi >> (5 * (s - 12))) & 31u);
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

// the low n bits of v reversed (n <= 32): v_bfrev_b32 and a shift on the GPU
HZ_HD uint32_t rev_bits(uint32_t v, int n) {
#if HZ_GPU
  return n > 0 ? __builtin_bitreverse32(v) >> (32 - n) : 0u;
#else
  uint32_t r = 0;
  for (int i = 0; i < n; i++) { r = (r << 1) | (v & 1u); v >>= 1; }
  return r;
#endif
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
// (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3).  row_bcast exists on
// GFX9 (CDNA) only: the engine is built for gfx950 alone, and any other target stops here
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "wave_incl_scan_dpp: row_bcast DPP controls are GFX9 / CDNA only (build with --offload-arch=gfx950)"
#endif
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
        uint32_t el = 1, si = 0xffffu;     /* the code's length and its rank in sorted[] */ \
        _Pragma("unroll") for (int len = 1; len <= 15; len++) {                         \
          if (len > (A).root) break;                                                    \
          const uint32_t d = (rc >> ((A).root - len)) - _fc[len];                       \
          const bool hit = d < _cn[len];                                                \
          el = hit ? (uint32_t)len : el;                                                \
          si = hit ? _of[len] + d : si;                                                 \
        }                                                                               \
        const uint32_t es = si != 0xffffu ? (uint32_t)(A).sorted[si] : hz::SYM_BAD;     \
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
