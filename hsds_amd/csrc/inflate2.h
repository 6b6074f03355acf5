// inflate2.h -- two-pass, long-segment zlib (RFC 1950/1951) decoder, one wavefront per stream.
//
// Replaces, for the HSDS data-node hot path, the zlib inflate that the reference reaches
// through storUtil._uncompress (hsds/util/storUtil.py:209-220, CPython zlib.decompress) and
// through c-blosc's zlib_wrap_decompress for every Blosc split (storUtil.py:195-208).  Output
// is bit-identical to libz; corrupt / truncated streams and adler32 mismatches fail (the
// reference's HTTPInternalServerError).
//
// Design (DESIGN.md "The inflate kernel"): a Huffman block is cut into 64 segments of L bits,
// L sized from the previous block so that one window covers the whole block (L is thousands
// of bits, not hundreds).  Per window:
//   A   lane i decodes from W bits before its segment (warm-up: Huffman codes
//       self-synchronise) to the first token start at or past the next segment, recording
//       its first K token starts with the output / match / literal counts reached there;
//   A'  lane i keeps decoding into segment i+1 until it lands on one of lane i+1's recorded
//       starts ("sync": from there both decodes coincide) -- no token storage at all;
//   R   a lane its predecessor never met is re-decoded from the predecessor's exit;
//   P   wave prefix sums of the synced output / match / literal counts give every lane its
//       output offset, its slots in the wave's match ring and its offset in the window's
//       literal stream;
//   E   every valid lane decodes its exact range again.  Nothing goes to dst: literal bytes
//       go to the literal stream, matches to the match ring as (position, length, distance)
//       records, both staged per lane in LDS and stored in whole groups;
//   M   the window's output is written span by span (SPAN bytes / <= 256 matches): a
//       source map of the span's match bytes (distance to an equal earlier byte, the
//       periodic extension of overlapping copies), pointer jumping until every match byte's
//       source is a literal of the span or a final byte before it, one gather per byte slot
//       (literal stream or dst), in-span sources from LDS, and the span's aligned dwords
//       stored from LDS.  Every output byte is written once.
// Shuffled streams (F2, Blosc typesize > 1) are inflated plain into a staging buffer and
// unshuffled afterwards by unshuffle_kernel (engine.hip); Job.perm must be the identity.
// adler32 is accumulated as per-lane (sum b, sum pos*b) pairs by M's gather and the
// stored-block copy.
//
// SINGLE SOURCE for the HIP kernel and the CPU emulation (tests/emu/inflate2_emu.cpp), like
// inflate_wave.h whose helpers (table build, LUT format, load_word) it reuses.
#pragma once
#include "inflate_wave.h"
#if !defined(__HIPCC__) && !defined(__HIP__)
#include <sched.h>
#endif
// the table builder's hand-offs are wavefront-scope here (two wavefronts of one workgroup
// build tables independently)
#undef HZ_TB_SYNC
#define HZ_TB_SYNC() HZ2_LSYNC()

namespace hz2 {

using hz::WAVE;
using hz::LL_ROOT;
using hz::D_ROOT;
using hz::LL_SUB;
using hz::D_SUB;
using hz::ST_OK;
using hz::ST_DATA;
using hz::ST_TRUNC;
using hz::ST_SIZE;
using hz::T_EOB;
using hz::T_ERR;
using hz::T_MATCH;
using hz::ADLER_MOD;

// one decode pass (HZ2_FUSE = 1): phases A, A' and R emit every token they count -- literal
// bytes and match records -- into the lane's own fixed region of the scratch (lane s:
// records [s MCAP_LANE, ...), literals [s LCAP_LANE, ...), numbered from the lane's first
// recorded start), so phase E's second decode is gone.  A lane's valid range is a suffix
// of what it emitted (from the record its predecessor met); phase M maps a window record
// or literal rank to its lane's region with a wave-uniform cursor over the lanes' ranges.
// The recorded starts live in registers (the LDS holds the staging instead).  0: phase E
// decodes every valid range again into the window-ordered ring (rounds 2-5)
#ifndef HZ2_FUSE
#define HZ2_FUSE 1
#endif
#ifndef HZ2_K
#define HZ2_K 8
#endif
constexpr int K = HZ2_K;                  // recorded token starts per lane
constexpr uint32_t LMIN = 64;
constexpr uint32_t LMAX = 1u << 16;       // segment bits (lane output stays well inside u32)
constexpr uint32_t MCAP_LANE = 256;       // matches per lane per window (ring bound)
constexpr uint32_t RING = MCAP_LANE * WAVE;   // match ring entries per wave
constexpr uint32_t RING_BYTES = RING * 8u;
constexpr uint32_t LCAP_LANE = 1024;      // literals per lane per window (literal stream bound)
constexpr uint32_t LIT_BYTES = LCAP_LANE * WAVE;
constexpr uint32_t SCRATCH_BYTES = RING_BYTES + LIT_BYTES;   // per resident wave: match ring, literal stream
#ifndef HZ2_SPAN
#define HZ2_SPAN 1024
#endif
constexpr uint32_t SPAN = HZ2_SPAN;       // resolve batch: output bytes covered by the source map
constexpr uint32_t MPL = 4;               // resolve: matches per lane per batch
static_assert(MPL == 4, "sel4 selects among four per-lane matches");
constexpr uint32_t SPL = SPAN / WAVE;     // resolve: span bytes per lane
static_assert(SPL <= 24, "resolve slots per lane");
constexpr uint32_t RGP = SPL;              // resolve: byte slots per lane (q = lane + 64 i)
// Every hand-off inside one stream's decode is wavefront-scope (HZ2_LSYNC for LDS,
// HZ2_GSYNC for the wave's own global stores read back by its later loads): no s_barrier,
// no s_waitcnt vmcnt(0) -- loads in flight (the next span's records) stay in flight, and
// two wavefronts of one workgroup can decode two windows of a stream independently
// (inflate2w_kernel); their hand-offs are workgroup-scope release / acquire on Ctl.
// phase E: match records are staged per lane and stored as whole aligned 32-byte groups
// (16-byte stores of each lane's own records, scattered over 64 lanes, cost about 4x their
// bytes in HBM writes plus L2 fills: measured, profiles/r2_traffic_attribution.txt)
#ifndef HZ2_RGRP
#define HZ2_RGRP 2
#endif
constexpr uint32_t RGRP = HZ2_RGRP;
static_assert(RGRP == 2 || RGRP == 4 || RGRP == 8, "RGRP: 2, 4 or 8 records");
// bit ring (phases A .. E): RS stream words per lane in LDS, refilled a quad at a time at
// wave-uniform ticks; a token reads at most 48 bits, so a window advances at most 1.5
// words per token
#ifndef HZ2_RS
#define HZ2_RS 12
#endif
constexpr uint32_t RS = HZ2_RS;           // ring words per lane (a multiple of 4)
#ifndef HZ2_MIRROR
#define HZ2_MIRROR 1                      // a copy of ring slot 0 after slot RS - 1 (no wrap select)
#endif
// phase E literal staging: bytes per lane, stored whole (16: one 16-byte store per 16 literals)
#ifndef HZ2_OS
#define HZ2_OS 16
#endif
constexpr uint32_t OS = HZ2_OS;
static_assert(OS == 4 || OS == 8 || OS == 16, "OS: 4, 8 or 16 bytes");
// span stores: 16 bytes per lane where the span's dwords allow (1: on)
#ifndef HZ2_ST16
#define HZ2_ST16 1
#endif
// wave priority by stream progress (s_setprio at every window start): HZ2_PRIO levels, the
// highest for a stream's first 1/HZ2_PRIO; 0 = off (A/B round 5, 4096 chunks: F1 26.0 ->
// 25.5 ms, F2 38.2 -> 35.9 ms; waves busy F1 0.897 -> 0.961, F2 0.83 -> 0.87)
#ifndef HZ2_PRIO
#define HZ2_PRIO 4
#endif
#ifndef HZ2_TICKN
#define HZ2_TICKN (HZ2_RS >= 16 ? 8 : 5)
#endif
constexpr uint32_t TICKN = HZ2_TICKN;     // tokens between ring refills
static_assert(RS % 4 == 0 && RS >= 8, "RS: whole quads");
// ring words a lane needs at a tick: TICKN tokens move the window at most
// (31 + 48 (TICKN - 1)) / 32 words before the last one, which reads words c+3 and c+4
constexpr uint32_t NEED = (31u + 48u * (TICKN - 1u)) / 32u + 5u;
static_assert(NEED <= RS, "ring too small for TICKN");
constexpr uint32_t SYNC_NONE = 0xfeu;     // predecessor ended (EOB / ERR / CUT): lane beyond the window
constexpr uint32_t SYNC_FAIL = 0xffu;     // predecessor never met this lane's recorded path
constexpr uint32_t END_NONE = 0, END_EOB = 1, END_ERR = 2, END_CUT = 3;

// record: bits 0-9 token start relative to the segment, 10-21 output bytes, 22-26 matches,
// 27-31 literals (cumulative from the lane's first record: the first record lies within 48
// bits of the segment start, and K - 1 <= 15 tokens of <= 48 bits / <= 258 bytes follow)
static_assert(K >= 1 && K <= 16, "record fields hold K <= 16 tokens");
HZ_HD uint32_t rec_pack(uint32_t rel, uint32_t o, uint32_t m, uint32_t l) { return rel | (o << 10) | (m << 22) | (l << 27); }
HZ_HD uint32_t rec_rel(uint32_t r) { return r & 0x3ffu; }
HZ_HD uint32_t rec_out(uint32_t r) { return (r >> 10) & 0xfffu; }
HZ_HD uint32_t rec_mat(uint32_t r) { return (r >> 22) & 31u; }
HZ_HD uint32_t rec_lit(uint32_t r) { return r >> 27; }

struct alignas(16) Shared {
  uint16_t lut_ll[(1 << LL_ROOT) + LL_SUB];
  uint16_t lut_d[(1 << D_ROOT) + D_SUB];
  uint16_t tb_first[16];
  uint16_t tb_offs[17];
  uint16_t tb_next[16];
  union {
    struct {                      // Huffman table build scratch (dead while windows run)
      uint16_t sorted_ll[288];
      uint16_t sorted_d[32];
      uint16_t cnt_ll[16];
      uint16_t cnt_d[16];
      uint16_t cnt_cl[16];
      uint16_t sorted_cl[20];
      uint8_t lens[320 + 32];
    };
    struct {                      // phases A .. E
#if HZ2_MIRROR
      uint32_t bring[RS + 1][WAVE];   // each lane's bit ring: stream word j in slot j % RS (word-major:
                                      // lanes hit distinct banks); slot RS mirrors slot 0
#else
      uint32_t bring[RS][WAVE];       // each lane's bit ring: stream word j in slot j % RS (word-major:
                                      // lanes hit distinct banks)
#endif
      union {
        uint32_t hbits[256];          // dynamic block header: 8192 stream bits from the header's quad
        uint32_t rec[K][WAVE];        // phases A .. R: recorded token starts (lane-interleaved)
        struct {                      // phase E
          alignas(16) uint8_t ostage[WAVE][OS];     // each lane's current OS bytes of the literal stream
          uint64_t rstage[WAVE][RGRP];              // each lane's current group of match records
        };
      };
    };
    struct {                      // phase M
      uint16_t smap[SPAN + 2];    // batch byte -> distance to its source (0: literal); [SPAN] stays 0
      alignas(16) uint32_t sbuf[SPAN / 4 + 4];   // the batch's aligned dwords, assembled in LDS
#if HZ2_FUSE
      // lane s's share of the window (written after the prefix sums): its first window
      // record mb[s] and literal rank lb[s], the region index minus the window index of its
      // records (rdl) and literals (ldl), the window position minus the region position of
      // its records (odl), and the end of its literal ranks (le)
      uint32_t mb[WAVE], rdl[WAVE], odl[WAVE], lb[WAVE], le[WAVE], ldl[WAVE];
#endif
    };
  };
  uint32_t wnext[8];              // NW == 1: the next window's start (WinState), kept in LDS across E and M
  uint8_t syncw[WAVE];            // record index where the predecessor met this lane / SYNC_*
  uint32_t endp[WAVE];            // lane's exclusive end (token boundary)
  uint8_t nrec[WAVE];
  int32_t u_status;
  uint32_t u_pos;
  uint32_t u_nlen, u_ndist;
};

struct Tune {
  uint32_t W;          // warm-up bits before a segment
  int max_rounds;      // repair rounds per window
  uint32_t over16;     // segment over-provisioning against the previous block size, in 16ths
  uint32_t spin_max;   // window pipeline: polls (s_sleep 2 each) before a wait gives up (0: SPIN_MAX)
};

// a wait of the window pipeline gave up (internal: the stream is then decoded again by one
// wavefront, inflate_stream_pipe; never reported as a chunk status)
constexpr int ST_HANG = -8;

// Output address map: stream byte x -> dst offset.  n == 1: x + x0.  Otherwise the HDF5 /
// Blosc byte unshuffle of a span of N elements of n bytes (`body` = N * n; tail bytes stay),
// evaluated at X = x0 + x (x0 places a Blosc plane split inside its block).
struct Perm {
  uint32_t n, N, body, magic, x0;
};

HZ_HD uint32_t umulhi32(uint32_t a, uint32_t b) {
#if HZ_GPU
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

HZ_HD uint32_t perm_at(const Perm& p, uint32_t x) {
  const uint32_t X = x + p.x0;
  if (p.n == 1u || X >= p.body) return X;
  uint32_t q = umulhi32(X, p.magic);     // X / N or one more
  uint32_t r = X - q * p.N;
  if ((int32_t)r < 0) { q--; r += p.N; }
  return r * p.n + q;
}

HZ_HD Perm perm_make(uint32_t n, uint32_t N, uint32_t x0) {
  Perm p;
  p.n = n < 1u ? 1u : n;
  p.N = N < 1u ? 1u : N;
  p.body = p.n == 1u ? 0u : p.N * p.n;
  p.magic = p.N <= 1u ? 0xffffffffu : (uint32_t)(((1ull << 32) + p.N - 1u) / p.N);
  p.x0 = x0;
  return p;
}

// ---- bit reader straight from the stream in global memory --------------------------------
// Words move through a 4-word shift register q (q0 next) refilled from the quad f, which was
// loaded when the previous quad became current: a quad load has a whole quad of tokens
// (~10) to arrive before the rotation that consumes it, and loads are unconditional (the
// address is clamped to the stream's last quad) so the load writes f directly.  bb holds
// `avail` (>= 32 after a fill) bits from bit position `pos` (relative to the 16-byte aligned
// stream base).  Bits past the stream end are whatever the clamped loads return: the decode
// of the true path never reads them (a token reaching past the end ends the window beyond
// limit_bits, which fails as truncated); speculative lanes may.
//
// Epoch refills (HZ2_EPOCH > 0).  A wave has ONE vmcnt counter for all 64 lanes, so a lane
// that waits for its own prefetched quad waits for every load issued before it -- including
// the quads other lanes issued one token earlier: with a per-lane refill, some lane refills
// at almost every token and the whole wave pays a memory latency per token.  With epochs,
// loads are issued only at wave-uniform epoch boundaries (every HZ2_EPOCH wave iterations)
// into a third quad h; the next boundary first moves h into f (its load had a whole epoch
// to land) and then issues the next one, so the waits inside an epoch are gone.  A lane that
// runs dry inside an epoch takes h at once (a wait, but rare: q + f hold up to 8 words).
#ifndef HZ2_EPOCH
#define HZ2_EPOCH 8
#endif
// HZ2_ALIGNBIT: the current two stream words (lo, hi) and a bit offset sh < 32 in lo, so at
// least 33 bits are always there: a peek is one funnel shift (v_alignbit_b32) and a drop adds
// to sh, taking the next word when it crosses 32 -- instead of a 64-bit bit buffer shifted
// on every drop and refilled before every symbol
#ifndef HZ2_ALIGNBIT
#define HZ2_ALIGNBIT 1
#endif
struct GRd {
#if HZ2_ALIGNBIT
  uint32_t lo, hi, sh;
#else
  uint64_t bb;
  uint32_t avail;
#endif
  uint32_t pos;
  uint32_t qa;         // dword index of the next quad to load (epochs: into h, else into f)
  uint32_t qn;         // words left in q
  uint32_t q0, q1, q2, q3;
  uint32_t f0, f1, f2, f3;
#if HZ2_EPOCH
  uint32_t fh;         // bit 0: f holds a quad; bit 1: h holds an issued load
  uint32_t h0, h1, h2, h3;
#endif
};

struct Src {
  hz_gcu8* base;       // 16-byte aligned base
  uint32_t lo, hi;     // valid byte range relative to base
  uint32_t last;       // dword index of the last quad holding stream bytes
};

HZ_HD uint32_t gword(const Src& s, uint32_t k) { return hz::load_word(s.base, k, s.lo, s.hi); }

// quad qa (clamped to the stream's last quad: an aligned 16-byte block holding a stream
// byte never crosses a page, so the load is always safe)
HZ_HD void g_quad(const Src& s, uint32_t qa, uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3) {
  const uint32_t b0 = (qa < s.last ? qa : s.last) * 4u;
#if HZ_GPU
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
  const u32x4 v = *(gu32x4*)(s.base + b0);
  a0 = v.x; a1 = v.y; a2 = v.z; a3 = v.w;
#else
  uint8_t t[16] = {0};
  for (uint32_t i = 0; i < 16u && b0 + i < s.hi; i++) t[i] = s.base[b0 + i];
  memcpy(&a0, t, 4); memcpy(&a1, t + 4, 4); memcpy(&a2, t + 8, 4); memcpy(&a3, t + 12, 4);
#endif
}

// vmcnt(0) as an instruction the compiler's wait pass sees: the rare refill paths below
// drain their load INSIDE their branch, so no register of the common path is left
// "possibly pending" at the merge (a pending register there makes the compiler put an
// s_waitcnt vmcnt(0) on the common path -- one full memory latency per token for the wave,
// waiting on the epoch prefetch as well)
#if HZ_GPU && !defined(HZ2_NOVMWAIT)
#define HZ2_VMWAIT() __builtin_amdgcn_s_waitcnt(0x0F70)
#else
#define HZ2_VMWAIT() do { } while (0)
#endif

#if HZ2_EPOCH
HZ_HD uint32_t g_take(const Src& s, GRd& r) {
  const uint32_t w = r.q0;
  r.q0 = r.q1; r.q1 = r.q2; r.q2 = r.q3;
  if (--r.qn == 0u) {
    // stream order is q, f, h, then quad qa
    if (r.fh & 1u) {
      r.q0 = r.f0; r.q1 = r.f1; r.q2 = r.f2; r.q3 = r.f3;
      r.fh &= ~1u;
    } else if (r.fh & 2u) {
      HZ2_VMWAIT();
      r.q0 = r.h0; r.q1 = r.h1; r.q2 = r.h2; r.q3 = r.h3;
      r.fh &= ~2u;
    } else {
      g_quad(s, r.qa, r.q0, r.q1, r.q2, r.q3);
      HZ2_VMWAIT();
      r.qa += 4u;
    }
    r.qn = 4u;
  }
  return w;
}

// wave-uniform epoch boundary: h (issued an epoch ago) moves into an empty f, and an empty h
// is issued
HZ_HD void g_epoch(const Src& s, GRd& r) {
  if ((r.fh & 3u) == 2u) {
    r.f0 = r.h0; r.f1 = r.h1; r.f2 = r.h2; r.f3 = r.h3;
    r.fh = 1u;
  }
  if (!(r.fh & 2u)) {
    g_quad(s, r.qa, r.h0, r.h1, r.h2, r.h3);
    r.qa += 4u;
    r.fh |= 2u;
  }
}

HZ_HD void g_init(const Src& s, GRd& r, uint32_t p) {
  const uint32_t k = p >> 5, qa = k & ~3u, qi = k & 3u;
  uint32_t a0, a1, a2, a3;
  g_quad(s, qa, a0, a1, a2, a3);
  g_quad(s, qa + 4u, r.f0, r.f1, r.f2, r.f3);
  g_quad(s, qa + 8u, r.h0, r.h1, r.h2, r.h3);
  r.fh = 3u;
  r.qa = qa + 12u;
  // shift register starts at word qi of the quad
  r.q0 = qi == 0u ? a0 : qi == 1u ? a1 : qi == 2u ? a2 : a3;
  r.q1 = qi == 0u ? a1 : qi == 1u ? a2 : a3;
  r.q2 = qi == 0u ? a2 : a3;
  r.q3 = a3;
  r.qn = 4u - qi;
  const uint32_t sh = p & 31u;
  const uint32_t w0 = g_take(s, r);
  const uint32_t w1 = g_take(s, r);
#if HZ2_ALIGNBIT
  r.lo = w0; r.hi = w1; r.sh = sh;
#else
  r.bb = (((uint64_t)w1 << 32) | w0) >> sh;
  r.avail = 64u - sh;
#endif
  r.pos = p;
}
#else
HZ_HD void g_epoch(const Src&, GRd&) {}

HZ_HD uint32_t g_take(const Src& s, GRd& r) {
  const uint32_t w = r.q0;
  r.q0 = r.q1; r.q1 = r.q2; r.q2 = r.q3;
  if (--r.qn == 0u) {
    r.q0 = r.f0; r.q1 = r.f1; r.q2 = r.f2; r.q3 = r.f3;
    r.qn = 4u;
  }
  // the refill load sits in a block of its own, after the block whose q <- f copies retire
  // f's old values: the load can then write f's registers directly (in one block with the
  // copies it lands in other registers, and the copy into f waits for the load)
  if (r.qn == 4u) {
    r.qa += 4u;
    g_quad(s, r.qa, r.f0, r.f1, r.f2, r.f3);
  }
  return w;
}

HZ_HD void g_init(const Src& s, GRd& r, uint32_t p) {
  const uint32_t k = p >> 5, qa = k & ~3u, qi = k & 3u;
  uint32_t a0, a1, a2, a3;
  g_quad(s, qa, a0, a1, a2, a3);
  // shift register starts at word qi of the quad
  r.q0 = qi == 0u ? a0 : qi == 1u ? a1 : qi == 2u ? a2 : a3;
  r.q1 = qi == 0u ? a1 : qi == 1u ? a2 : a3;
  r.q2 = qi == 0u ? a2 : a3;
  r.q3 = a3;
  r.qn = 4u - qi;
  r.qa = qa + 4u;
  g_quad(s, r.qa, r.f0, r.f1, r.f2, r.f3);
  const uint32_t sh = p & 31u;
  const uint32_t w0 = g_take(s, r);
  const uint32_t w1 = g_take(s, r);
#if HZ2_ALIGNBIT
  r.lo = w0; r.hi = w1; r.sh = sh;
#else
  r.bb = (((uint64_t)w1 << 32) | w0) >> sh;
  r.avail = 64u - sh;
#endif
  r.pos = p;
}
#endif

#if HZ2_ALIGNBIT
HZ_HD void g_fill(const Src&, GRd&) {}      // >= 33 bits are always there

// the 32 stream bits from r.pos
HZ_HD uint32_t g_peek(const GRd& r) {
#if HZ_GPU
  return __builtin_amdgcn_alignbit(r.hi, r.lo, r.sh);
#else
  return (uint32_t)((((uint64_t)r.hi << 32) | r.lo) >> r.sh);
#endif
}

// n <= 32
HZ_HD void g_drop(const Src& s, GRd& r, uint32_t n) {
  r.pos += n;
  r.sh += n;
  if (r.sh >= 32u) {
    r.sh -= 32u;
    r.lo = r.hi;
    r.hi = g_take(s, r);
  }
}
#else
HZ_HD void g_fill(const Src& s, GRd& r) {
  if (r.avail < 32u) {
    r.bb |= (uint64_t)g_take(s, r) << r.avail;
    r.avail += 32u;
  }
}

HZ_HD uint32_t g_peek(const GRd& r) { return (uint32_t)r.bb; }

HZ_HD void g_drop(const Src&, GRd& r, uint32_t n) { r.bb >>= n; r.avail -= n; r.pos += n; }
#endif

HZ_HD uint32_t lookup_ll(const Shared* sh, uint64_t bits) {
  uint32_t e = sh->lut_ll[bits & ((1u << LL_ROOT) - 1)];
  if (!(e & 15u)) e = sh->lut_ll[(1u << LL_ROOT) + ((e >> 4) & 511u) + ((uint32_t)(bits >> LL_ROOT) & hz::bmask(e >> 13))];
  return e;
}
HZ_HD uint32_t lookup_d(const Shared* sh, uint64_t bits) {
  uint32_t e = sh->lut_d[bits & ((1u << D_ROOT) - 1)];
  if (!(e & 15u)) e = sh->lut_d[(1u << D_ROOT) + ((e >> 4) & 511u) + ((uint32_t)(bits >> D_ROOT) & hz::bmask(e >> 13))];
  return e;
}

// one token at r.pos (hz::next_token over the global reader): literal byte, T_EOB, T_ERR, or
// T_MATCH | len << 16 | (dist - 1).  Invalid codes advance by their table length.
HZ_HD uint32_t next_token(const Shared* sh, const Src& s, GRd& r) {
  g_fill(s, r);
  const uint32_t bits = g_peek(r);
  const uint32_t e = lookup_ll(sh, bits);
  const uint32_t nb = e & 15u, p = e >> 4;
  const uint32_t q = p - 257u;
  const int islen = q < 29u;
  const uint32_t xb = (islen && q >= 8u && q < 28u) ? (q - 4u) >> 2 : 0u;
  const uint32_t base = q < 8u ? q + 3u : q == 28u ? 258u : ((4u | (q & 3u)) << xb) + 3u;
  const uint32_t len = base + ((bits >> nb) & hz::bmask(xb));
  g_drop(s, r, nb + xb);
  uint32_t tok = p <= 256u ? p : T_ERR;
  if (islen) {
    g_fill(s, r);
    const uint32_t dbits = g_peek(r);
    const uint32_t ed = lookup_d(sh, dbits);
    const uint32_t nd = ed & 15u, d = ed >> 4;
    const int ok = d < 30u;
    const uint32_t xd = (ok && d >= 2u) ? (d - 2u) >> 1 : 0u;
    const uint32_t dist = (d < 4u ? d + 1u : ((2u | (d & 1u)) << xd) + 1u) + ((dbits >> nd) & hz::bmask(xd));
    g_drop(s, r, ok ? nd + xd : nd);
    tok = ok ? (T_MATCH | (len << 16) | (dist - 1u)) : T_ERR;
  }
  return tok;
}

// ---- the bit ring reader (phases A, A', R, E) --------------------------------------------
// A lane's stream position is word c (of the 16-byte aligned base) plus sh bits.  The window
// w0..w2 holds words c..c+2 (>= 64 bits past the position whatever sh is, so a whole token
// -- at most 48 bits -- decodes from one window); n0 n1 are ring words c+3 c+4, read at the
// start of every token so the advance (by 0, 1 or 2 words) is a few masked merges, no branch.
// The ring holds words [wr - RS, wr).  It is refilled at wave-uniform ticks, every TICKN
// tokens: the quads that fit are loaded and written at once, so no load is ever in flight
// across a token (a load kept in flight in loop-carried registers makes the compiler copy
// them, and wait for the load, on every token).
struct BR {
  uint32_t w0, w1, w2, sh, c;
  uint32_t n0, n1;
  uint32_t wr;
  uint32_t slot;       // (c + 3) % RS, kept incrementally (no division per token)
  uint32_t wslot;      // wr % RS (a multiple of 4), kept incrementally
};

HZ_HD uint32_t br_pos(const BR& r) { return r.c * 32u + r.sh; }

// the quad of words at ring slot k (a multiple of 4: with RS % 4 == 0 the quad never wraps)
HZ_HD void br_put(Shared& sh, int lane, uint32_t k, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  sh.bring[k][lane] = a0;
  sh.bring[k + 1u][lane] = a1;
  sh.bring[k + 2u][lane] = a2;
  sh.bring[k + 3u][lane] = a3;
#if HZ2_MIRROR
  if (k == 0u) sh.bring[RS][lane] = a0;
#endif
}

// ring words c+3 and c+4 (slot (c+3) % RS and the next; the mirror covers the wrap)
HZ_HD void br_next(const Shared& sh, int lane, BR& r) {
  const uint32_t k = r.slot;
  r.n0 = sh.bring[k][lane];
#if HZ2_MIRROR
  r.n1 = sh.bring[k + 1u][lane];
#else
  r.n1 = sh.bring[k + 1u == RS ? 0u : k + 1u][lane];
#endif
}

HZ_HD uint32_t slot4(uint32_t k) { return k + 4u == RS ? 0u : k + 4u; }

// refill: the quads that fit (their slots hold only words below c+3, i.e. wr <= c + RS - 1),
// all loads issued before the first write.  Leaves wr in [c + RS, c + RS + 3]: every word a
// token reads within the next TICKN tokens is in the ring (NEED <= RS).  TICKN tokens read at
// most 48 TICKN bits, so two quads always restore the ring (and br_init needs two at most)
static_assert((48u * TICKN + 31u) / 32u <= 8u && RS - 8u + 3u <= 8u, "two quads per refill");
HZ_HD void br_fill(Shared& sh, int lane, const Src& S, BR& r) {
  if (r.wr + 1u > r.c + RS) return;
  const bool two = r.wr + 5u <= r.c + RS;              // room for a second quad
  uint32_t a[8];
  g_quad(S, r.wr, a[0], a[1], a[2], a[3]);
  if (two) g_quad(S, r.wr + 4u, a[4], a[5], a[6], a[7]);
  const uint32_t k1 = slot4(r.wslot);
  br_put(sh, lane, r.wslot, a[0], a[1], a[2], a[3]);
  if (two) br_put(sh, lane, k1, a[4], a[5], a[6], a[7]);
  r.wr += two ? 8u : 4u;
  r.wslot = two ? slot4(k1) : k1;
}

// position p: the window (words c .. c+2) from two quad loads and a full ring (from quad q)
HZ_HD void br_init(Shared& sh, int lane, const Src& S, BR& r, uint32_t p) {
  const uint32_t c = p >> 5, q = c & ~3u, i = c - q;
  uint32_t a[8];
  g_quad(S, q, a[0], a[1], a[2], a[3]);
  g_quad(S, q + 4u, a[4], a[5], a[6], a[7]);
  // words c, c+1, c+2 = a[i], a[i+1], a[i+2] (selects: no dynamically indexed array)
  r.w0 = i == 0u ? a[0] : i == 1u ? a[1] : i == 2u ? a[2] : a[3];
  r.w1 = i == 0u ? a[1] : i == 1u ? a[2] : i == 2u ? a[3] : a[4];
  r.w2 = i == 0u ? a[2] : i == 1u ? a[3] : i == 2u ? a[4] : a[5];
  r.sh = p & 31u;
  r.c = c;
  r.slot = (c + 3u) % RS;
  const uint32_t k0 = q % RS, k1 = slot4(k0);
  br_put(sh, lane, k0, a[0], a[1], a[2], a[3]);
  br_put(sh, lane, k1, a[4], a[5], a[6], a[7]);
  r.wr = q + 8u;
  r.wslot = slot4(k1);
  br_fill(sh, lane, S, r);
}

HZ_HD void br_tick(Shared& sh, int lane, const Src& S, BR& r) { br_fill(sh, lane, S, r); }

// advance by n <= 48 bits (n0 n1 must hold ring words c+3, c+4).  The window moves by
// k = 0, 1 or 2 words: two compares and three pairs of selects (v_cndmask) of SSA values
// (written as selects between fields of the reader, the compiler turns them into an indexed
// load of the struct -- a scratch copy)
HZ_HD void br_adv(BR& r, uint32_t n) {
  const uint32_t a0 = r.w0, a1 = r.w1, a2 = r.w2, a3 = r.n0, a4 = r.n1;
  const uint32_t t = r.sh + n;
  const uint32_t k = t >> 5;
  const bool k1 = t >= 32u, k2 = t >= 64u;
  r.w0 = k2 ? a2 : k1 ? a1 : a0;
  r.w1 = k2 ? a3 : k1 ? a2 : a1;
  r.w2 = k2 ? a4 : k1 ? a3 : a2;
  r.sh = t & 31u;
  r.c += k;
  const uint32_t s2 = r.slot + k, s3 = s2 - RS;      // (c + 3) % RS without a division
  r.slot = s3 < s2 ? s3 : s2;
}

HZ_HD uint32_t bfe32(uint32_t v, uint32_t off, uint32_t w) {
#if HZ_GPU
  return __builtin_amdgcn_ubfe(v, off, w);
#else
  return w ? (uint32_t)((v >> off) & ((1ull << w) - 1u)) : 0u;
#endif
}

HZ_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
#if HZ_GPU
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31u));
#endif
}

#if HZ_GPU && defined(HZ2_MARKS)
#define HZ2_MARK(s) asm volatile(";@@" s)
#else
#define HZ2_MARK(s) do { } while (0)
#endif
#if HZ_GPU
#define HZ2_HM __device__ __forceinline__
#else
#define HZ2_HM inline
#endif
// lane 0's reader over the dynamic header's bits in LDS (sh.hbits)
struct HR {
  const uint32_t* b;
  uint32_t p, base;
  HZ2_HM uint32_t peek() const { return funnel(b[(p >> 5) + 1u], b[p >> 5], p & 31u); }
  HZ2_HM void drop(uint32_t n) { p += n; }
  HZ2_HM uint32_t pos() const { return base + p; }
};
// the same reader with its current two words in registers and the next one loaded ahead:
// a symbol's peek is one funnel shift, and the only LDS read on the serial path of the
// code-length loop is the table lookup (a drop of <= 32 bits crosses at most one word)
struct HRR {
  const uint32_t* b;
  uint32_t p, base, w0, w1, w2, wi;
  HZ2_HM void init(const uint32_t* bits, uint32_t p0, uint32_t base0) {
    b = bits; p = p0; base = base0; wi = p0 >> 5;
    w0 = b[wi]; w1 = b[wi + 1u]; w2 = b[wi + 2u];
  }
  HZ2_HM uint32_t peek() const { return funnel(w1, w0, p & 31u); }
  HZ2_HM void drop(uint32_t n) {
    p += n;
    if ((p >> 5) != wi) { wi++; w0 = w1; w1 = w2; w2 = b[wi + 2u]; }
  }
  HZ2_HM uint32_t pos() const { return base + p; }
};

enum : uint32_t { TK_LIT = 0, TK_MATCH = 1, TK_EOB = 2, TK_ERR = 3 };
struct Tok {
  uint32_t n;      // bits
  uint32_t kind;   // TK_*
  uint32_t len;    // output bytes (1 for a literal)
  uint32_t v;      // literal byte, or the match distance
};

// one token at the reader's position, from the rich tables (hz::ent_rich): literal/length
// symbol, its extra bits, the distance symbol and its extra bits all from the 64-bit window.
// Branch-free but for the rare second-level lookups: the distance lookup is made for every
// token (a literal's is ignored) -- the wave waits for its slowest lane anyway, and a
// literal/match branch costs both paths plus the exec-mask bookkeeping on every token
HZ_HD Tok rtok(const Shared* sh, const BR& r) {
  const uint32_t lo = funnel(r.w1, r.w0, r.sh), hi = funnel(r.w2, r.w1, r.sh);
  uint32_t e = sh->lut_ll[lo & ((1u << LL_ROOT) - 1u)];
  if (!(e & 15u)) e = sh->lut_ll[(1u << LL_ROOT) + ((e >> 4) & 511u) + bfe32(lo, LL_ROOT, e >> 13)];
  const uint32_t nb = e & 15u, x = (e >> 4) & 7u, v = e >> 7;
  const bool lit = x == 7u;                     // literal, EOB or an invalid code
  const uint32_t s1 = nb + x;                   // < 32 for every entry
  const uint32_t dl = funnel(hi, lo, s1);
  // a literal looks up distance entry 0 -- the shortest code's, never a second-level pointer
  // -- so the second-level branch below does not depend on the literal / match split
  uint32_t ed = sh->lut_d[dl & (lit ? 0u : (1u << D_ROOT) - 1u)];
  if (!(ed & 15u)) ed = sh->lut_d[(1u << D_ROOT) + ((ed >> 4) & 511u) + bfe32(dl, D_ROOT, ed >> 13)];
  const uint32_t nd = ed & 15u, xd = (ed >> 4) & 15u;
  const bool derr = (ed >> 12) & 1u;
  const uint32_t dist = (((ed >> 8) & 7u) << xd) + ((ed >> 11) & 1u) + bfe32(dl, nd, xd);
  const uint32_t lk = v < 256u ? (uint32_t)TK_LIT : v == 256u ? (uint32_t)TK_EOB : (uint32_t)TK_ERR;
  const uint32_t mk = derr ? (uint32_t)TK_ERR : (uint32_t)TK_MATCH;
  Tok t;
  t.n = lit ? nb : s1 + nd + (derr ? 0u : xd);
  t.kind = lit ? lk : mk;
  t.len = lit ? 1u : v + bfe32(lo, nb, x);
  t.v = lit ? v : dist;
  return t;
}

// a[u] for a register array and a runtime u < MPL (no dynamic register indexing)
HZ_HD uint32_t sel4(const uint32_t* a, uint32_t u) { return u == 0u ? a[0] : u == 1u ? a[1] : u == 2u ? a[2] : a[3]; }
// a[j] of a lane's K recorded starts (registers) for a runtime j < K: masks OR-ed (a select
// chain is folded back into an indexed load, which puts the array in scratch)
HZ_HD uint32_t selk(const uint32_t* a, uint32_t j) {
  uint32_t v = 0;
HZ_UNROLL
  for (uint32_t i = 0; i < (uint32_t)K; i++) v |= a[i] & (0u - (uint32_t)(j == i));
  return v;
}
HZ_HD void setk(uint32_t* a, uint32_t j, uint32_t v, bool on) {
HZ_UNROLL
  for (uint32_t i = 0; i < (uint32_t)K; i++) a[i] = (on && j == i) ? v : a[i];
}
// a lane's MPL match records (absolute position, len << 16 | dist - 1): one reaches before
// the stream's first byte
HZ_HD bool rec_bad(const uint32_t* o, const uint32_t* w) {
  bool bad = false;
HZ_UNROLL
  for (uint32_t u = 0; u < MPL; u++) bad |= o[u] != 0xffffffffu && (w[u] & 0xffffu) + 1u > o[u];
  return bad;
}

HZ_HD uint32_t tok_len(uint32_t t) { return (t & T_MATCH) ? ((t >> 16) & 0x1ffu) : 1u; }

struct Job {
  const uint8_t* src;   // stream bytes (any alignment)
  uint32_t src_len;
  uint8_t* dst;         // base of the permuted output span
  uint32_t dst_len;     // expected stream output (exact) or capacity (exact == 0)
  uint32_t exact;
  uint32_t* out_len;    // optional decoded length
  Perm perm;
};

struct Stats {
  uint64_t windows, blocks, stored, tokens, matches, lanes_valid, repairs, repair_lanes, cuts, batches, hops;
  uint64_t steps_a, steps_e, extra_windows;
  uint64_t fill_max, fill_sum, span_sum;   // resolve: per-batch max lane source-map fill, total fill, spans
  uint64_t src_in, src_far[4];             // resolve: sources inside the batch; before it within 256/1536/4096/more
  uint64_t hangs;                          // window pipeline: waits that gave up (one-wavefront re-decode)
};

}  // namespace hz2

#if HZ_GPU
namespace hz2 {
__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v) { return hz::wave_excl_scan(v, HZ_LANE_ID()); }
}  // namespace hz2
// value of lane-variable v in lane i (uniform i: v_readlane, no LDS round trip as a
// ds_bpermute shuffle would take); LANE_ARR: a per-lane array
#define LV_AT(v, i) ((uint32_t)__builtin_amdgcn_readlane((int)(v), (int)(i)))
#define LANE_ARR(T, name, n) T name[n]
#define LVA_AT(arr, u, i) ((uint32_t)__builtin_amdgcn_readlane((int)hz2::sel4(arr, u), (int)(i)))
// a lane counter made wave-uniform (the first active lane's), for epoch boundaries
#define HZ2_UNI(v) ((uint32_t)__builtin_amdgcn_readfirstlane((int)(v)))
// LDS hand-off inside one wavefront: the LDS executes a wave's instructions in order, so
// only the compiler must not move or cache accesses across this point (no s_waitcnt, no
// s_barrier: loads in flight -- the next span's match records -- stay in flight)
#define HZ2_LSYNC()                                              \
  do {                                                           \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");       \
    __builtin_amdgcn_wave_barrier();                             \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");       \
  } while (0)
// wavefront-scope ordering of this wavefront's own global stores and later loads (no wait)
#define HZ2_GSYNC() HZ2_LSYNC()
#define HZ2_PAUSE() __builtin_amdgcn_s_sleep(2)
#define HZ2_WGBAR() __syncthreads()
namespace hz2 {
__device__ __forceinline__ uint32_t ctl_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ctl_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
}  // namespace hz2
#else
#define HZ2_UNI(v) (v)
#define LV_AT(v, i) ((v)[i])
#define LANE_ARR(T, name, n) T name[64][n]
#define LVA_AT(arr, u, i) ((arr)[i][u])
#define HZ2_LSYNC() do { } while (0)
#define HZ2_GSYNC() do { } while (0)
#define HZ2_PAUSE() sched_yield()
#define HZ2_WGBAR() hz2::emu_wgbar(pipe.ctl, NW)
namespace hz2 {
// CPU emulation: the two wavefronts are two threads
inline uint32_t ctl_ld(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void ctl_st(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
struct Ctl;
void emu_wgbar(Ctl* c, int n);
}  // namespace hz2
#endif

#if HZ2_EPOCH
#define HZ2_TICK(it) do { if ((HZ2_UNI(++(it)) % (uint32_t)HZ2_EPOCH) == 0u) hz2::g_epoch(S, r); } while (0)
#else
#define HZ2_TICK(it) do { ++(it); } while (0)
#endif
// ring reader tick (r: the lane's hz2::BR)
#define HZ2_RTICK(it) do { if ((HZ2_UNI(++(it)) % hz2::TICKN) == 0u) hz2::br_tick(sh, lane, S, r); } while (0)

namespace hz2 {

// rank of this lane among the set lanes of a ballot (v_mbcnt)
HZ_HD uint32_t lane_rank(uint64_t m, int lane) {
#if HZ_GPU
  (void)lane;
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
#else
  return hz::popc64(m & ((1ull << lane) - 1ull));
#endif
}

// ---- the window pipeline of two wavefronts on one stream (inflate2w_kernel) ---------------
enum : uint32_t { WK_NEWBLOCK = 0, WK_CONT = 1, WK_END = 2 };
struct WinState {                // a window's start
  uint32_t pos;                  // bit position (a block header for WK_NEWBLOCK, the trailer's byte for WK_END)
  uint32_t out;                  // output offset
  uint32_t kind;                 // WK_*
  uint32_t block_start, bfinal;  // WK_CONT: the block it continues
  uint32_t est;                  // WK_CONT: expected bits left in the block
  uint32_t prev_block_bits;      // the last Huffman block's size (next block's estimate)
};
constexpr int NW_MAX = 4;        // wavefronts per stream in the window pipeline
struct Ctl {                     // in LDS, shared by the workgroup's wavefronts
  uint32_t synced;               // the window whose start is in `next`
  uint32_t mdone;                // windows whose output is final
  uint32_t end_at;               // the WK_END window's index (~0u: not reached)
  int32_t err;                   // the first error (0: none)
  uint32_t item;                 // the work item both wavefronts decode
  uint32_t bar;                  // CPU emulation: barrier generation counter
  int32_t redo;                  // inflate_stream_pipe: status of the one-wavefront re-decode
  WinState next;
  uint64_t adler[NW_MAX][2];     // per wavefront: sum b, sum pos * b
};
struct Pipe {
  Ctl* ctl;
  const Shared* other;           // the previous window's wavefront's LDS (its block tables)
  uint32_t w;                    // this wavefront's index in the workgroup
};
constexpr uint32_t SPIN_MAX = 1u << 24;   // a wait that never ends fails the stream instead of hanging

HZ_HD void ctl_reset(Ctl* c, uint32_t item) {
  c->synced = 0; c->mdone = 0; c->end_at = ~0u; c->err = 0; c->item = item;
}
HZ_HD void atomic_min_err(Ctl* c, int st) {
#if HZ_GPU
  atomicCAS(&c->err, 0, st);
#else
  int32_t z = 0;
  __atomic_compare_exchange_n(&c->err, &z, st, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
#endif
}
#if !HZ_GPU
// the emulated wavefronts meet (generation barrier over Ctl::bar: the low 8 bits count
// arrivals, the rest is the generation)
inline void emu_wgbar(Ctl* c, int n) {
  const uint32_t v = __atomic_add_fetch(&c->bar, 1u, __ATOMIC_ACQ_REL);
  const uint32_t g = v & ~0xffu;
  if ((v & 0xffu) == (uint32_t)n) {
    __atomic_store_n(&c->bar, g + 0x100u, __ATOMIC_RELEASE);                          // the last: release
  } else {
    while ((__atomic_load_n(&c->bar, __ATOMIC_ACQUIRE) & ~0xffu) == g) sched_yield();  // wait
  }
}
#endif

// stream byte x is dst[x] (a shuffled chunk is inflated into staging and unshuffled after);
// ring_base: the wave's SCRATCH_BYTES (match ring, then the literal stream).
//
// The stream is decoded as a sequence of windows (a window = one pass of phases A .. M over
// one Huffman block or a part of it; a stored block is a window of its own).  A window's
// start (bit position, output offset, block state) is known once the previous window's
// sync phases (A, A', R, prefix sums) are done, and its resolve M needs every output byte
// before it.  NW = 1: one wavefront runs the windows in order.  NW = 2 (inflate2w_kernel):
// two wavefronts of one workgroup alternate windows -- wavefront w takes windows w, w + 2,
// ... -- handing the next window's start over as soon as their sync phases end, and
// waiting for the other's M before their own M, so one window's header, sync phases and
// emit run beside the other's resolve (pipe.ctl in LDS; a continuation window copies the
// block's tables from the other wavefront's LDS).
template <class StatsT, int NW>
#if HZ_GPU
__device__ __forceinline__
#else
static
#endif
int inflate_stream(Shared& sh, const Job job, const Tune tune, uint8_t* ring_base, StatsT* stats, HzProf* prof = nullptr,
                   Pipe pipe = Pipe{nullptr, nullptr, 0u}) {
  (void)prof;
  const uint32_t a = (uint32_t)(((uintptr_t)job.src) & 15u);
  const Src S = {HZ_GLOBAL(hz_gcu8*, job.src - a), a, a + job.src_len, ((a + job.src_len - 1u) >> 2) & ~3u};
  const uint32_t limit_bits = S.hi * 8u;
  const uint32_t dst_len = job.dst_len;
  hz_gu8* const dst = HZ_GLOBAL(hz_gu8*, job.dst);
  hz_gu32* const ring = HZ_GLOBAL(hz_gu32*, ring_base);
#if HZ_GPU
  typedef __attribute__((address_space(1))) uint64_t hz_gu64;
#else
  typedef uint64_t hz_gu64;
#endif
  hz_gu64* const ring64 = HZ_GLOBAL(hz_gu64*, ring_base);
  hz_gu8* const lits = HZ_GLOBAL(hz_gu8*, ring_base + RING_BYTES);
  if (job.perm.n > 1u) return ST_SIZE;      // no output map: shuffled streams are staged

  LANE_VAR(uint32_t, s1);     // adler32 partial sums of the bytes this lane wrote: sum b, sum pos*b
  LANE_VAR(uint32_t, s2);
  LANE_LOOP { LV(s1) = 0; LV(s2) = 0; }

  // ---- zlib header (RFC 1950) ----
  if (job.src_len < 2) return ST_TRUNC;
  {
    GRd r;
    g_init(S, r, S.lo * 8u);
    const uint64_t two = g_peek(r);
    const uint32_t cmf = (uint32_t)(two & 0xffu), flg = (uint32_t)((two >> 8) & 0xffu);
    if ((cmf & 0x0f) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0) return ST_DATA;
    if (flg & 0x20) return ST_DATA;   // preset dictionary: Z_NEED_DICT
  }
  (void)pipe;
  WinState cur;                        // the current window's start
  cur.pos = S.lo * 8u + 16u;
  cur.out = 0;
  cur.kind = WK_NEWBLOCK;
  cur.block_start = 0;
  cur.bfinal = 0;
  cur.est = 0;
  cur.prev_block_bits = 0;
  static_assert(NW >= 1 && NW <= NW_MAX, "wavefronts per stream");
  uint32_t k = NW > 1 ? pipe.w : 0u;   // window index
  static_assert(sizeof(WinState) <= sizeof(sh.wnext), "WinState in Shared::wnext");

  // the next window's start to whoever decodes it
  auto publish = [&](const WinState& nx) {
    if (NW > 1) {
      Ctl* c = pipe.ctl;
      c->next = nx;
      if (nx.kind == WK_END) ctl_st(&c->end_at, k + 1u);
      ctl_st(&c->synced, k + 1u);
    } else {
      // (in LDS: no register holds it across phases E and M)
      LANE_LOOP { if (lane == 0) memcpy(sh.wnext, &nx, sizeof(nx)); }
    }
  };
  // every wait is bounded; one that gives up is ST_HANG (not corrupt data: the caller
  // decodes the stream again with one wavefront)
  const uint32_t spin_max = tune.spin_max ? tune.spin_max : SPIN_MAX;
  (void)spin_max;
  // wait until every output byte before this window is final (the other wavefront's M)
  auto wait_output = [&]() -> int {
    if (NW > 1) {
      Ctl* c = pipe.ctl;
      for (uint32_t spin = 0;; spin++) {
        if (ctl_ld(&c->mdone) == k) return ST_OK;
        const int32_t e = (int32_t)ctl_ld((const uint32_t*)&c->err);
        if (e) return e;
        if (spin > spin_max) return ST_HANG;
        HZ2_PAUSE();
      }
    }
    return ST_OK;
  };
  auto output_done = [&]() {
    if (NW > 1) ctl_st(&pipe.ctl->mdone, k + 1u);
  };

  int fail = ST_OK;
  for (;; k += NW) {
    if (NW > 1) {
      // window k's start: published by the other wavefront's sync phases of window k - 1
      Ctl* c = pipe.ctl;
      int got = 0;
      for (uint32_t spin = 0;; spin++) {
        if (k == 0u) { got = 1; break; }             // window 0 starts at the stream's first block
        if (ctl_ld(&c->synced) == k) { cur = c->next; got = 1; break; }
        if (ctl_ld(&c->end_at) <= k) break;          // the stream ended before window k
        const int32_t e = (int32_t)ctl_ld((const uint32_t*)&c->err);
        if (e) { fail = e; break; }
        if (spin > spin_max) { fail = ST_HANG; break; }
        HZ2_PAUSE();
      }
      if (!got) break;
    } else if (k > 0) {
      HZ2_LSYNC();
      memcpy(&cur, sh.wnext, sizeof(cur));
    }
    if (cur.kind == WK_END) break;
    const int wst = [&]() -> int {
#if HZ_GPU && HZ2_PRIO
      // VALU issue on a SIMD goes to the higher priority, then the OLDER wave: with one
      // stream per wave the youngest waves finish last.  A wave's priority falls with its
      // stream's progress, so the waves that lag get the issue slots
      {
        const uint32_t q = cur.out < dst_len ? (uint32_t)(((uint64_t)cur.out * HZ2_PRIO) / dst_len) : HZ2_PRIO - 1u;
        const uint32_t pr = HZ2_UNI(HZ2_PRIO - 1u - q);
        if (pr >= 3u) __builtin_amdgcn_s_setprio(3);
        else if (pr == 2u) __builtin_amdgcn_s_setprio(2);
        else if (pr == 1u) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
#endif
      uint32_t pos = cur.pos, out = cur.out;
      uint32_t block_start = cur.block_start, bfinal = cur.bfinal, est = cur.est;
      int first_window = 0;
      if (cur.kind == WK_NEWBLOCK) {
      HZ_T(1);
      if (pos + 3u > limit_bits) return ST_TRUNC;
      uint32_t h3;
      {
        GRd r;
        g_init(S, r, pos);
        h3 = (uint32_t)(g_peek(r) & 7u);
      }
      block_start = pos;
      pos += 3;
      bfinal = h3 & 1u;
      const uint32_t btype = h3 >> 1;
      if (stats) stats->blocks++;
      if (btype == 3) return ST_DATA;
        if (btype == 0) {
        // ---- stored block: copied through the output map ----
        pos = (pos + 7u) & ~7u;
        if (pos + 32u > limit_bits) return ST_TRUNC;
        GRd r;
        g_init(S, r, pos);
        const uint32_t ln = (uint32_t)(g_peek(r) & 0xffffffffu);
        const uint32_t len = ln & 0xffffu, nlen = ln >> 16;
        if ((len ^ 0xffffu) != nlen) return ST_DATA;
        pos += 32u;
        if (pos + len * 8u > limit_bits) return ST_TRUNC;
        if (out + len > dst_len) return ST_SIZE;
        {
          WinState nx = cur;
          nx.pos = pos + len * 8u;
          nx.out = out + len;
          nx.kind = bfinal ? WK_END : WK_NEWBLOCK;
          publish(nx);
          const int wr = wait_output();
          if (wr != ST_OK) return wr;
        }
        const uint32_t sb = pos >> 3;
        LANE_LOOP {
          uint32_t a1 = LV(s1), a2 = LV(s2);
          for (uint32_t i = (uint32_t)lane; i < len; i += 64) {
            const uint32_t b = S.base[sb + i];
            dst[out + i] = (uint8_t)b;
            a1 += b;
            a2 = (uint32_t)((a2 + (uint64_t)((out + i) % ADLER_MOD) * b) % ADLER_MOD);
          }
          LV(s1) = a1 % ADLER_MOD; LV(s2) = a2;
        }
        if (stats) stats->stored++;
        HZ2_GSYNC();
        output_done();
        return ST_OK;
        }
      // ---- Huffman code lengths ----
      uint32_t nlen = 288, ndist = 32;
      if (btype == 1) {
        LANE_LOOP {
          for (int q = lane; q < 320; q += 64) sh.lens[q] = q >= 288 ? 5 : q < 144 ? 8 : q < 256 ? 9 : q < 280 ? 7 : 8;
        }
        HZ2_LSYNC();
      } else {
        // dynamic header (RFC 1951 3.2.7): the wave loads the 8192 stream bits from the header's
        // quad into LDS at once (a header is at most 14 + 19 x 3 + 320 x 14 bits), then lane 0
        // decodes it serially from LDS -- no global load latency per refill
        const uint32_t hq = (pos >> 5) & ~3u;
        LANE_LOOP {
          uint32_t a0, a1, a2, a3;
          g_quad(S, hq + 4u * (uint32_t)lane, a0, a1, a2, a3);
          sh.hbits[4 * lane] = a0; sh.hbits[4 * lane + 1] = a1; sh.hbits[4 * lane + 2] = a2; sh.hbits[4 * lane + 3] = a3;
        }
        HZ2_LSYNC();
        LANE_LOOP {
          if (lane == 0) {
            int st = ST_OK;
            HR r = {sh.hbits, pos - hq * 32u, hq * 32u};
            const uint32_t hlit = (r.peek() & 31u) + 257u, hdist = ((r.peek() >> 5) & 31u) + 1u;
            const uint32_t hclen = ((r.peek() >> 10) & 15u) + 4u;
            r.drop(14);
            if (hlit > 286 || hdist > 30) st = ST_DATA;
            uint16_t* cl = sh.sorted_cl;
            for (int i = 0; i < 19; i++) cl[i] = 0;
            for (uint32_t i = 0; i < hclen; i++) {
              cl[hz::cl_order(i)] = (uint16_t)(r.peek() & 7u);
              r.drop(3);
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
            if (left > 0 || maxl == 0) st = ST_DATA;   // code-length code must be complete
            uint16_t* clut = sh.lut_d;                   // 7-bit LUT (sym | len << 8), rebuilt below
            if (st == ST_OK) {
              uint16_t* next = sh.tb_next;                 // next code per length (LDS: no scratch)
              uint32_t code = 0;
              for (int l = 1; l <= 7; l++) { code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1; next[l] = (uint16_t)code; }
              for (int i = 0; i < 19; i++) {
                const uint32_t l = cl[i];
                if (!l) continue;
                const uint32_t rc = hz::rev_bits(next[l]++, (int)l);
                for (uint32_t k = rc; k < 128u; k += 1u << l) clut[k] = (uint16_t)(i | (l << 8));
              }
            }
            const uint32_t total = hlit + hdist;
            uint32_t n = 0, prevl = 0;
            HRR rr;
            rr.init(sh.hbits, r.p, r.base);
            while (st == ST_OK && n < total) {
              if (rr.pos() > limit_bits + 64u) { st = ST_TRUNC; break; }
              const uint32_t bits = rr.peek();
              const uint32_t e = clut[bits & 127u];
              const uint32_t sym = e & 0xffu, l = e >> 8;
              if (sym < 16) { rr.drop(l); sh.lens[n++] = (uint8_t)sym; prevl = sym; continue; }
              // a repeat: its extra bits follow the code in the same peek (7 + 7 bits)
              const uint32_t x = bits >> l;
              uint32_t rep, val = 0;
              if (sym == 16) {
                if (n == 0) { st = ST_DATA; break; }
                val = prevl; rep = 3 + (x & 3u); rr.drop(l + 2u);
              } else if (sym == 17) { rep = 3 + (x & 7u); rr.drop(l + 3u); }
              else { rep = 11 + (x & 127u); rr.drop(l + 7u); }
              if (n + rep > total) { st = ST_DATA; break; }
              for (uint32_t k = 0; k < rep; k++) sh.lens[n++] = (uint8_t)val;
              prevl = val;
            }
            r.p = rr.p;
            if (st == ST_OK && r.pos() > limit_bits) st = ST_TRUNC;
            if (st == ST_OK && sh.lens[256] == 0) st = ST_DATA;   // missing end-of-block code
            if (st == ST_OK) {
              for (int i = (int)hdist - 1; i >= 0; i--) sh.lens[288 + i] = sh.lens[hlit + i];
              for (uint32_t i = hlit; i < 288; i++) sh.lens[i] = 0;
              for (uint32_t i = 288 + hdist; i < 320; i++) sh.lens[i] = 0;
            }
            sh.u_status = st;
            sh.u_pos = r.pos();
            sh.u_nlen = hlit;
            sh.u_ndist = hdist;
          }
        }
        HZ2_LSYNC();
        const int hst = sh.u_status;
        if (hst != ST_OK) return hst;
        pos = sh.u_pos;
        nlen = sh.u_nlen;
        ndist = sh.u_ndist;
      }
      HZ_T(2);
      {
        int bst = ST_OK;
        hz::TableArgs tll = {sh.lens, (int)nlen, sh.cnt_ll, sh.sorted_ll, sh.lut_ll, LL_ROOT, 1, LL_SUB, 1};
        HZ_BUILD_TABLE(sh, tll, bst);
        if (bst != ST_OK) return bst;
        hz::TableArgs td = {sh.lens + 288, (int)ndist, sh.cnt_d, sh.sorted_d, sh.lut_d, D_ROOT, 2, D_SUB, 1};
        HZ_BUILD_TABLE(sh, td, bst);
        if (bst != ST_OK) return bst;
      }
      HZ2_LSYNC();

      est = cur.prev_block_bits ? cur.prev_block_bits : 200000u;
      {
        const uint32_t rem = limit_bits > pos ? limit_bits - pos : 0u;
        if (est > rem + 64u) est = rem + 64u;
      }
      est += (uint32_t)(((uint64_t)est * tune.over16) >> 4);
        first_window = 1;
      } else if (NW > 1) {
        // a continuation window: the block's tables are the previous window's wavefront's
        const Shared& o = *pipe.other;
        LANE_LOOP {
          for (uint32_t i = (uint32_t)lane; i < (uint32_t)((1 << LL_ROOT) + LL_SUB); i += 64u) sh.lut_ll[i] = o.lut_ll[i];
          for (uint32_t i = (uint32_t)lane; i < (uint32_t)((1 << D_ROOT) + D_SUB); i += 64u) sh.lut_d[i] = o.lut_d[i];
        }
        HZ2_LSYNC();
      }
      if (stats) { stats->windows++; if (!first_window) stats->extra_windows++; }
      const uint32_t ws = pos;
      uint32_t L = (est + 63u) >> 6;
      L = L < LMIN ? LMIN : L > LMAX ? LMAX : L;
      const uint32_t W = tune.W;

      HZ_T(3);
      // -------- phase A: warm-up + own segment, first K token starts recorded --------
      LANE_VAR(BR, rd);
      LANE_VAR(uint32_t, co);      // output bytes since the first record
      LANE_VAR(uint32_t, cm);      // matches since the first record
      LANE_VAR(uint32_t, cl);      // literals since the first record
      LANE_VAR(uint32_t, ek);      // END_*
      LANE_VAR(uint32_t, ea);      // position after the EOB token
#if HZ2_FUSE
      LANE_ARR(uint32_t, rcv, K);  // the lane's recorded starts
      LANE_ARR(uint32_t, nxr, K);  // its successor's (phase A')
      // lane s's successor's recorded starts into its registers (every lane active)
      auto fetch_succ = [&]() {
#if HZ_GPU
        const int sl = ((HZ_LANE_ID() + 1) & 63) << 2;
HZ_UNROLL
        for (uint32_t j = 0; j < (uint32_t)K; j++) nxr[j] = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)rcv[j]);
#else
        for (int s = 0; s < 63; s++)
          for (uint32_t j = 0; j < (uint32_t)K; j++) nxr[s][j] = rcv[s + 1][j];
#endif
      };
      // a counted token into the lane's region: the literal byte and the match record
      // (position = output bytes since the first record) are staged unconditionally -- the one
      // that does not apply sits in the slot the next literal / match overwrites -- and a
      // completed group of OS literals / RGRP records is stored whole
      auto emit = [&](int lane, const Tok& t, bool cnt, uint32_t o, uint32_t m, uint32_t l) {
        sh.ostage[lane][l & (OS - 1u)] = (uint8_t)t.v;
        sh.rstage[lane][m & (RGRP - 1u)] = (uint64_t)o | ((uint64_t)((t.len << 16) | (t.v - 1u)) << 32);
        if (cnt && t.kind == TK_LIT && ((l + 1u) & (OS - 1u)) == 0u) {
          hz_gu8* const p = lits + (uint32_t)lane * LCAP_LANE + (l + 1u - OS);
#if HZ_GPU
          if constexpr (OS == 16u) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(1))) u32x4 gu32x4;
            *(gu32x4*)p = *(const u32x4*)&sh.ostage[lane][0];
          } else if constexpr (OS == 8u) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(1))) u32x2 gu32x2;
            *(gu32x2*)p = *(const u32x2*)&sh.ostage[lane][0];
          } else {
            *(hz_gu32*)p = *(const uint32_t*)&sh.ostage[lane][0];
          }
#else
          memcpy(p, &sh.ostage[lane][0], OS);
#endif
        }
        if (cnt && t.kind == TK_MATCH && (m & (RGRP - 1u)) == RGRP - 1u) {
          hz_gu64* const p = ring64 + (uint32_t)lane * MCAP_LANE + (m & ~(RGRP - 1u));
#if HZ_GPU
          typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
          typedef __attribute__((address_space(1))) u64x2 gu64x2;
HZ_UNROLL
          for (uint32_t k = 0; k < RGRP; k += 2u) *(gu64x2*)(p + k) = *(const u64x2*)&sh.rstage[lane][k];
#else
          for (uint32_t k = 0; k < RGRP; k++) p[k] = sh.rstage[lane][k];
#endif
        }
      };
#endif
      LANE_LOOP {
        const uint32_t ss = ws + (uint32_t)lane * L, se = ss + L;
        const uint32_t p0 = (lane > 0 && ss - ws > W) ? ss - W : ws;
        BR r;
        br_init(sh, lane, S, r, p0);
        uint32_t steps = 0;
        uint32_t nr = 0, o = 0, m = 0, l = 0, e = END_NONE, after = 0;
#if HZ2_FUSE
HZ_UNROLL
        for (uint32_t j = 0; j < (uint32_t)K; j++) LV(rcv)[j] = 0u;
#endif
        // one loop for the warm-up (tokens before ss are decoded and dropped: whatever they
        // are, even invalid codes, which advance by their table length) and the segment.
        // Branch-free body: the only exit is at the top (a token that ends the lane sets e
        // and does not advance, so the next test fails)
        for (;;) {
          HZ2_MARK("A_TOP");
          const uint32_t tp = br_pos(r);
          if (tp >= se || e != END_NONE) break;
          br_next(sh, lane, r);
          const bool inseg = tp >= ss;
#if HZ2_FUSE
          {
            // the first K starts in the segment (registers; the select chain only runs while
            // some lane still records)
            const bool rk = inseg && nr < (uint32_t)K;
#if HZ_GPU
            if (WAVE_BALLOT(rk))
#endif
              setk(LV(rcv), nr, rec_pack(tp - ss, o, m, l), rk);
            nr += rk ? 1u : 0u;
          }
#else
          {
            // a record past the K-th (or in the warm-up) goes to the lane's endp word,
            // which phase A' overwrites
            const bool rk = inseg && nr < (uint32_t)K;
            uint32_t* rp = rk ? &sh.rec[nr < (uint32_t)K ? nr : 0u][lane] : &sh.endp[lane];
            *rp = rec_pack(tp - ss, o, m, l);
            nr += rk ? 1u : 0u;
          }
#endif
          const Tok t = rtok(&sh, r);
          const bool ismatch = t.kind == TK_MATCH, islit = t.kind == TK_LIT;
          const bool stop = inseg && (t.kind >= TK_EOB || (ismatch && m >= MCAP_LANE) || (islit && l >= LCAP_LANE));
          e = stop ? (t.kind == TK_EOB ? END_EOB : t.kind == TK_ERR ? END_ERR : END_CUT) : e;
          after = stop ? tp + t.n : after;
          const bool cnt = inseg && !stop;
#if HZ2_FUSE
          emit(lane, t, cnt, o, m, l);
#endif
          o += cnt ? t.len : 0u;
          m += (cnt && ismatch) ? 1u : 0u;
          l += (cnt && islit) ? 1u : 0u;
          br_adv(r, stop ? 0u : t.n);
          HZ2_RTICK(steps);
        }
        sh.nrec[lane] = nr;
        sh.syncw[lane] = lane == 0 ? 0u : SYNC_NONE;
        LV(rd) = r; LV(co) = o; LV(cm) = m; LV(cl) = l; LV(ek) = e; LV(ea) = after;
        if (stats) stats->steps_a += steps;
      }
      HZ2_LSYNC();

      HZ_T(4);
      // -------- phase A': continuation until lane+1's recorded path is met --------
      // (a lane that ended leaves its successor at SYNC_NONE)
      // (in the loop below: the successor's recorded starts at or past `rel` -- k, the first
      // of them -- are passed: none left ends the search; one at `rel` is the sync)
#if HZ2_FUSE
      // registers: every start compared at once (a runtime index would put them in scratch)
#define HZ2_SYNC_TEST(lane_)                                                                     \
      {                                                                                          \
        uint32_t nlt = 0, hit = SYNC_FAIL;                                                       \
        HZ_UNROLL for (uint32_t i = 0; i < (uint32_t)K; i++) {                                   \
          const uint32_t q = hz2::rec_rel(LV(nxr)[i]);                                           \
          nlt += (i < nrn && q < rel) ? 1u : 0u;                                                 \
          hit = (i < nrn && q == rel) ? i : hit;                                                 \
        }                                                                                        \
        k = nlt;                                                                                 \
        if (k >= nrn) break;                                                                     \
        if (hit != SYNC_FAIL) { res = hit; break; }                                              \
      }
#define HZ2_EMIT(lane_, t_, c_, o_, m_, l_) emit((lane_), (t_), (c_), (o_), (m_), (l_))
      fetch_succ();
#else
#define HZ2_SYNC_TEST(lane_)                                                                     \
      {                                                                                          \
        while (k < nrn && hz2::rec_rel(sh.rec[k][(lane_) + 1]) < rel) k++;                      \
        if (k >= nrn) break;                                                                     \
        if (hz2::rec_rel(sh.rec[k][(lane_) + 1]) == rel) { res = k; break; }                    \
      }
#define HZ2_EMIT(lane_, t_, c_, o_, m_, l_) do { } while (0)
#endif
#define HZ2_CONTINUE(lane_)                                                                      \
      do {                                                                                       \
        BR r = LV(rd);                                                                           \
        uint32_t o = LV(co), m = LV(cm), l = LV(cl), e = LV(ek), after = LV(ea);                 \
        uint32_t res = SYNC_NONE;                                                                \
        if (e == END_NONE && (lane_) < 63) {                                                     \
          /* A ticked at most TICKN - 1 tokens ago: refill now, so the tick counter can restart */ \
          hz2::br_tick(sh, lane, S, r);                                                          \
          const uint32_t base = ws + (uint32_t)((lane_) + 1) * L;                                \
          const uint32_t nrn = sh.nrec[(lane_) + 1];                                             \
          uint32_t k = 0, ct = 0;                                                                \
          res = SYNC_FAIL;                                                                       \
          for (;;) {                                                                             \
            const uint32_t tp = hz2::br_pos(r);                                                  \
            const uint32_t rel = tp - base;                                                      \
            HZ2_SYNC_TEST(lane_);                                                                \
            hz2::br_next(sh, lane, r);                                                           \
            const hz2::Tok t = hz2::rtok(&sh, r);                                                \
            if (t.kind >= hz2::TK_EOB) {                                                         \
              e = t.kind == hz2::TK_EOB ? END_EOB : END_ERR; after = tp + t.n; res = SYNC_NONE; break; \
            }                                                                                    \
            if ((t.kind == hz2::TK_MATCH && m >= MCAP_LANE) || (t.kind == hz2::TK_LIT && l >= LCAP_LANE)) { \
              e = END_CUT; res = SYNC_NONE; break;                                               \
            }                                                                                    \
            HZ2_EMIT(lane, t, true, o, m, l);                                                    \
            o += t.len;                                                                          \
            m += t.kind == hz2::TK_MATCH ? 1u : 0u;                                              \
            l += t.kind == hz2::TK_LIT ? 1u : 0u;                                                \
            hz2::br_adv(r, t.n);                                                                 \
            HZ2_RTICK(ct);                                                                       \
          }                                                                                      \
        }                                                                                        \
        if ((lane_) < 63) sh.syncw[(lane_) + 1] = res;                                           \
        sh.endp[lane_] = hz2::br_pos(r);                                                         \
        LV(rd) = r; LV(co) = o; LV(cm) = m; LV(cl) = l; LV(ek) = e; LV(ea) = after;              \
      } while (0)
      LANE_LOOP { HZ2_CONTINUE(lane); }
      HZ2_LSYNC();

      HZ_T(5);
      // -------- repair rounds --------
      // a lane whose predecessor exists but never met its path re-runs A + A' from the
      // predecessor's exit (a token boundary), recording its new path; its successor's sync
      // is recomputed.  Adjacent lanes are never redone in the same round.
      for (int round = 0; round < tune.max_rounds; round++) {
        const uint64_t redo_m = WAVE_BALLOT(lane > 0 && sh.syncw[lane] == SYNC_FAIL && sh.syncw[lane - 1] < (uint32_t)K);
        if (!redo_m) break;
        if (stats) { stats->repairs++; stats->repair_lanes += hz::popc64(redo_m); }
        LANE_LOOP {
          if ((redo_m >> lane) & 1ull) {
            const uint32_t ss = ws + (uint32_t)lane * L, se = ss + L;
            BR r;
            br_init(sh, lane, S, r, sh.endp[lane - 1]);
            uint32_t nr = 0, o = 0, m = 0, l = 0, e = END_NONE, after = 0, ct = 0;
            for (;;) {
              const uint32_t tp = br_pos(r);
              if (!(tp < se || nr == 0)) break;
              br_next(sh, lane, r);
#if HZ2_FUSE
              setk(LV(rcv), nr, rec_pack(tp - ss, o, m, l), nr < (uint32_t)K);
              nr += nr < (uint32_t)K ? 1u : 0u;
#else
              if (nr < (uint32_t)K) { sh.rec[nr][lane] = rec_pack(tp - ss, o, m, l); nr++; }
#endif
              const Tok t = rtok(&sh, r);
              if (t.kind >= TK_EOB) { e = t.kind == TK_EOB ? END_EOB : END_ERR; after = tp + t.n; break; }
              if ((t.kind == TK_MATCH && m >= MCAP_LANE) || (t.kind == TK_LIT && l >= LCAP_LANE)) { e = END_CUT; break; }
              HZ2_EMIT(lane, t, true, o, m, l);
              o += t.len;
              m += t.kind == TK_MATCH ? 1u : 0u;
              l += t.kind == TK_LIT ? 1u : 0u;
              br_adv(r, t.n);
              HZ2_RTICK(ct);
            }
            sh.nrec[lane] = nr;
            sh.syncw[lane] = 0;                       // its path starts at record 0
            LV(rd) = r; LV(co) = o; LV(cm) = m; LV(cl) = l; LV(ek) = e; LV(ea) = after;
          }
        }
        HZ2_LSYNC();
#if HZ2_FUSE
        fetch_succ();     // (a successor redone in an earlier round has new starts)
#endif
        LANE_LOOP {
          if ((redo_m >> lane) & 1ull) HZ2_CONTINUE(lane);
        }
        HZ2_LSYNC();
      }
#undef HZ2_CONTINUE
#undef HZ2_SYNC_TEST
#undef HZ2_EMIT

      HZ_T(6);
      // -------- validity, window end, prefix sums --------
      // lane i is valid when every lane before it is and lane i-1 met its path
      uint32_t V = 1;
      {
        const uint64_t okm = WAVE_BALLOT(lane == 0 || sh.syncw[lane] < (uint32_t)K);
        while (V < 64u && ((okm >> V) & 1ull)) V++;
      }
      LANE_VAR(uint32_t, wout);
      LANE_VAR(uint32_t, wmat);
      LANE_VAR(uint32_t, wlit);
      LANE_VAR(uint32_t, sbit);    // exact start bit of the lane's range
#if HZ2_FUSE
      LANE_VAR(uint32_t, srec);    // the record the lane's range starts at
#endif
      LANE_LOOP {
        uint32_t wo = 0, wm = 0, wl = 0, sb = 0;
        if ((uint32_t)lane < V) {
          const uint32_t k = sh.syncw[lane];
#if HZ2_FUSE
          const uint32_t rc = selk(LV(rcv), k);
          LV(srec) = rc;
#else
          const uint32_t rc = sh.rec[k][lane];
#endif
          wo = LV(co) - rec_out(rc);
          wm = LV(cm) - rec_mat(rc);
          wl = LV(cl) - rec_lit(rc);
          sb = ws + (uint32_t)lane * L + rec_rel(rc);
        }
        LV(wout) = wo; LV(wmat) = wm; LV(wlit) = wl; LV(sbit) = sb;
      }
      // the first valid lane that ended (EOB / ERR / CUT) closes the window
      int end_lane = -1;
      {
        const uint64_t em = WAVE_BALLOT((uint32_t)lane < V && LV(ek) != END_NONE);
        if (em) end_lane = (int)__builtin_ctzll(em);
      }
      if (end_lane >= 0) V = (uint32_t)end_lane + 1u;
      if (stats) stats->lanes_valid += V;
      uint32_t end_kind = END_NONE, npos = 0;
      LANE_LOOP {
        if ((uint32_t)lane >= V) { LV(wout) = 0; LV(wmat) = 0; LV(wlit) = 0; }
        if (lane == (end_lane >= 0 ? end_lane : (int)V - 1)) {
          sh.u_status = (int32_t)LV(ek);
          sh.u_pos = LV(ek) == END_EOB ? LV(ea) : sh.endp[lane];
          sh.u_nlen = sh.endp[lane];
        }
      }
      HZ2_LSYNC();
      end_kind = (uint32_t)sh.u_status;
      npos = sh.u_pos;
      if (end_kind == END_ERR) {
        // the first invalid code on the true path: a stream that ran out of input is
        // truncated, anything else is corrupt
        return sh.u_nlen + 64u > limit_bits ? ST_TRUNC : ST_DATA;
      }
      LANE_VAR(uint32_t, obase);
      LANE_VAR(uint32_t, mbase);
      LANE_VAR(uint32_t, lbase);
      uint32_t wtotal = 0, mtotal = 0, ltotal = 0;
#if HZ_GPU
      obase = wave_excl_scan32(wout);
      mbase = wave_excl_scan32(wmat);
      lbase = wave_excl_scan32(wlit);
      wtotal = hz::wave_sum(wout);
      mtotal = hz::wave_sum(wmat);
      ltotal = hz::wave_sum(wlit);
#else
      for (int lane = 0; lane < 64; lane++) {
        obase[lane] = wtotal; mbase[lane] = mtotal; lbase[lane] = ltotal;
        wtotal += wout[lane]; mtotal += wmat[lane]; ltotal += wlit[lane];
      }
#endif
      (void)ltotal;
      if (stats) stats->matches += mtotal;
      if (out + wtotal > dst_len) return ST_SIZE;
      if (npos > limit_bits) return ST_TRUNC;
#if HZ2_FUSE
      // the valid lanes' last, partial groups (the staging dies below: the maps overlay it)
      LANE_LOOP {
        if ((uint32_t)lane < V) {
          const uint32_t m = LV(cm), l = LV(cl);
          hz_gu64* const rp = ring64 + (uint32_t)lane * MCAP_LANE;
          hz_gu8* const lp = lits + (uint32_t)lane * LCAP_LANE;
          for (uint32_t k = m & ~(RGRP - 1u); k < m; k++) rp[k] = sh.rstage[lane][k & (RGRP - 1u)];
          for (uint32_t k = l & ~(OS - 1u); k < l; k++) lp[k] = sh.ostage[lane][k & (OS - 1u)];
        }
      }
      HZ2_LSYNC();
      LANE_LOOP {
        const uint32_t rc = (uint32_t)lane < V ? LV(srec) : 0u;
        sh.mb[lane] = LV(mbase);
        sh.rdl[lane] = (uint32_t)lane * MCAP_LANE + rec_mat(rc) - LV(mbase);
        sh.odl[lane] = out + LV(obase) - rec_out(rc);
        sh.lb[lane] = LV(lbase);
        sh.le[lane] = LV(lbase) + LV(wlit);
        sh.ldl[lane] = (uint32_t)lane * LCAP_LANE + rec_lit(rc) - LV(lbase);
      }
      HZ2_LSYNC();
#endif

      {  // the next window's start: the other wavefront may begin its sync phases now
        WinState nx;
        nx.pos = npos;
        nx.out = out + wtotal;
        nx.prev_block_bits = cur.prev_block_bits;
        nx.block_start = block_start;
        nx.bfinal = bfinal;
        nx.est = 0;
        if (end_kind == END_EOB) {
          nx.kind = bfinal ? WK_END : WK_NEWBLOCK;
          nx.prev_block_bits = npos - block_start;
        } else {
          nx.kind = WK_CONT;
          // the block goes on: the rest is estimated from what is left of the estimate
          const uint32_t used = npos - ws;
          uint32_t e2 = est > used ? est - used : 0u;
          const uint32_t floor_est = ((npos - block_start) >> 3) + 64u * LMIN;
          e2 = e2 < floor_est ? floor_est : e2;
          const uint32_t rem = limit_bits > npos ? limit_bits - npos : 0u;
          if (e2 > rem + 64u) e2 = rem + 64u;
          nx.est = e2;
        }
        publish(nx);
      }

      HZ_T(7);
#if !HZ2_FUSE
      // -------- phase E: exact decode of every valid range --------
      // Nothing goes to dst here: literal bytes go to the window's literal stream (lane i's
      // literals at lbase[i]..., staged 16 bytes at a time in LDS and stored whole), matches
      // to the match ring as (position, length, distance) records (staged per lane, stored as
      // aligned groups).  Phase M then writes every output byte of the window exactly once.
      LANE_VAR(int, lerr);
      LANE_LOOP {
        int err = 0;
        uint32_t steps = 0;
        if ((uint32_t)lane < V) {
          BR r;
          br_init(sh, lane, S, r, LV(sbit));
          const uint32_t stop = sh.endp[lane];
          uint32_t o = out + LV(obase), mi = LV(mbase);
          const uint32_t l0 = LV(lbase);
          uint32_t lk = l0;
          const uint32_t m0 = mi;                          // the lane's first record
          // branch-free body but for the two flushes: a token's literal byte and its match
          // record are both staged unconditionally -- the one that does not apply sits in the
          // slot the next literal / match overwrites (lk / mi do not move for it)
          while (br_pos(r) < stop && !err) {
            HZ2_MARK("E_TOP");
            br_next(sh, lane, r);
            const Tok tk = rtok(&sh, r);
            br_adv(r, tk.n);
            HZ2_RTICK(steps);
            const bool islit = tk.kind == TK_LIT, ismatch = tk.kind == TK_MATCH;
            // (E decodes ranges A verified: an EOB / invalid code or a distance past the
            // output start here is a bug, reported as corrupt data)
            err |= (!islit && (!ismatch || tk.v > o)) ? 1 : 0;
            sh.ostage[lane][lk & (OS - 1u)] = (uint8_t)tk.v;
#if !defined(HZ2_EXP_NOSTORE) && !defined(HZ2_EXP_NORING)
            sh.rstage[lane][mi & (RGRP - 1u)] = (uint64_t)o | ((uint64_t)((tk.len << 16) | (tk.v - 1u)) << 32);
#endif
            lk += islit ? 1u : 0u;
#ifndef HZ2_EXP_NOSTORE
            if (islit && !(lk & (OS - 1u))) {            // OS bytes of the literal stream complete
              const uint32_t g = lk - OS;
              if (g >= l0) {
#if HZ_GPU
                if constexpr (OS == 16u) {
                  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                  typedef __attribute__((address_space(1))) u32x4 gu32x4;
                  *(gu32x4*)(lits + g) = *(const u32x4*)&sh.ostage[lane][0];
                } else if constexpr (OS == 8u) {
                  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                  typedef __attribute__((address_space(1))) u32x2 gu32x2;
                  *(gu32x2*)(lits + g) = *(const u32x2*)&sh.ostage[lane][0];
                } else {
                  *(hz_gu32*)(lits + g) = *(const uint32_t*)&sh.ostage[lane][0];
                }
#else
                memcpy(lits + g, &sh.ostage[lane][0], OS);
#endif
              } else {                                   // the group starts in the previous lane's literals
                for (uint32_t k = l0; k < lk; k++) lits[k] = sh.ostage[lane][k & (OS - 1u)];
              }
            }
#endif
#if !defined(HZ2_EXP_NOSTORE) && !defined(HZ2_EXP_NORING)
            if (ismatch && (mi & (RGRP - 1u)) == RGRP - 1u) {
              const uint32_t g = mi & ~(RGRP - 1u);
              if (g >= m0) {                             // a whole group of this lane: stored at once
#if HZ_GPU
                typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
                typedef __attribute__((address_space(1))) u64x2 gu64x2;
HZ_UNROLL
                for (uint32_t k = 0; k < RGRP; k += 2u)
                  *(gu64x2*)(ring64 + g + k) = *(const u64x2*)&sh.rstage[lane][k];
#else
                for (uint32_t k = 0; k < RGRP; k++) ring64[g + k] = sh.rstage[lane][k];
#endif
              } else {                                   // the group starts in the previous lane's records
                for (uint32_t k = m0; k <= mi; k++) ring64[k] = sh.rstage[lane][k & (RGRP - 1u)];
              }
            }
#endif
            mi += ismatch ? 1u : 0u;
            o += islit ? 1u : ismatch ? tk.len : 0u;
          }
#if !defined(HZ2_EXP_NOSTORE) && !defined(HZ2_EXP_NORING)
          {                                            // the lane's last, partial group
            const uint32_t g = mi & ~(RGRP - 1u);
            for (uint32_t k = g > m0 ? g : m0; k < mi; k++) ring64[k] = sh.rstage[lane][k & (RGRP - 1u)];
          }
#endif
#ifndef HZ2_EXP_NOSTORE
          {                                            // the lane's last, partial 16 literal bytes
            const uint32_t g = lk & ~(OS - 1u);
            for (uint32_t k = g > l0 ? g : l0; k < lk; k++) lits[k] = sh.ostage[lane][k & (OS - 1u)];
          }
#endif
        }
        LV(lerr) = err;
        if (stats) stats->steps_e += steps;
      }
      if (WAVE_BALLOT(LV(lerr))) return ST_DATA;
#endif
      HZ2_GSYNC();

      {
        const int wr = wait_output();    // every byte before `out` final (the other wavefront's M)
        if (wr != ST_OK) return wr;
      }
      HZ_T(8);
      // -------- phase M: write the window's output, one span at a time --------
      // The window's output [out, out + wtotal) is cut into consecutive spans [F, F + span):
      // span = the frontier F up to the end of the last of the next <= 256 matches that fit
      // SPAN bytes (a span of literals only when no match fits).  Per span:
      //   1. smap[x - F] = distance from match byte x to an equal earlier byte (the periodic
      //      extension of an overlapping copy), literal bytes 0;
      //   2. pointer jumping: while a byte's source is a match byte of the span, add that
      //      byte's distance (rounds over all bytes, one LDS round trip each) -- after it every
      //      match byte's source is either before F (final in dst) or a literal of the span;
      //   3. every lane gathers its byte slots q = lane + 64 i at once: literals from the
      //      literal stream (rank among the span's literals by ballot), sources before F from
      //      dst; in-span sources (literals) then from LDS;
      //   4. the span's aligned dwords are stored from LDS, whole where they lie inside the
      //      span (and the stream), byte by byte at its edges.
      // Every output byte is written once, coalesced; E stored nothing to dst.
      // match bytes' adler sums: a1 < 2^32 and a2 < 2^64 for any window (< 2^24 bytes)
      LANE_VAR(uint32_t, ra1);
      LANE_VAR(uint64_t, ra2);
      LANE_LOOP { LV(ra1) = 0; LV(ra2) = 0; }
      LANE_ARR(uint32_t, ro, MPL);
      LANE_ARR(uint32_t, rw, MPL);
#if HZ2_FUSE
      // window records jb + lane + 64 u from their lanes' regions (positions made absolute):
      // rcur, the last lane whose first record is at or before jb, only grows; the lanes
      // whose records the MPL x 64 touch are walked from it (a batch spans a few)
      uint32_t rcur = 0;
      auto load_recs = [&](uint32_t jb, auto& xo, auto& xw) {
        // the lanes' shares into registers (one LDS round trip), walked by v_readlane
        LANE_VAR(uint32_t, vmb);
        LANE_VAR(uint32_t, vrd);
        LANE_VAR(uint32_t, vod);
        LANE_LOOP { LV(vmb) = sh.mb[lane]; LV(vrd) = sh.rdl[lane]; LV(vod) = sh.odl[lane]; }
        while (rcur < 63u && LV_AT(vmb, rcur + 1u) <= jb) rcur++;
        LANE_ARR(uint32_t, dr, MPL);
        LANE_ARR(uint32_t, dd, MPL);
        {
          const uint32_t r0 = LV_AT(vrd, rcur), o0 = LV_AT(vod, rcur);
          LANE_LOOP {
HZ_UNROLL
            for (uint32_t u = 0; u < MPL; u++) { LV(dr)[u] = r0; LV(dd)[u] = o0; }
          }
        }
        const uint32_t jl = jb + 64u * MPL;
        for (uint32_t s = rcur; s < 63u;) {
          const uint32_t b = LV_AT(vmb, s + 1u);
          if (b >= jl || b >= mtotal) break;
          s++;
          const uint32_t r1 = LV_AT(vrd, s), o1 = LV_AT(vod, s);
          LANE_LOOP {
HZ_UNROLL
            for (uint32_t u = 0; u < MPL; u++) {
              const bool in = jb + (uint32_t)lane + 64u * u >= b;
              LV(dr)[u] = in ? r1 : LV(dr)[u];
              LV(dd)[u] = in ? o1 : LV(dd)[u];
            }
          }
        }
        LANE_LOOP {
HZ_UNROLL
          for (uint32_t u = 0; u < MPL; u++) {
            // (unconditional loads: a record past the window reads slot 0)
            const uint32_t j = jb + (uint32_t)lane + 64u * u;
            const bool ok = j < mtotal;
            const uint64_t v = ring64[ok ? j + LV(dr)[u] : 0u];
            LV(xo)[u] = ok ? (uint32_t)v + LV(dd)[u] : 0xffffffffu;
            LV(xw)[u] = ok ? (uint32_t)(v >> 32) : 0u;
          }
        }
      };
      load_recs(0u, ro, rw);
      // literal ranks -> regions: the cursor lane lcur holds ranks up to lend (exclusive)
      uint32_t lcur = 0, lend = HZ2_UNI(sh.le[0]), lcd = HZ2_UNI(sh.ldl[0]);
#else
      LANE_LOOP {
HZ_UNROLL
        for (uint32_t u = 0; u < MPL; u++) {
          const uint32_t j = (uint32_t)lane + 64u * u;
          LV(ro)[u] = j < mtotal ? ring[2u * j] : 0xffffffffu;
          LV(rw)[u] = j < mtotal ? ring[2u * j + 1u] : 0u;
        }
      }
#endif
      LANE_LOOP { if (lane == 0) sh.smap[SPAN] = 0; }
      const uint32_t wend = out + wtotal;
      uint32_t F = out, L0 = 0;      // frontier and its rank in the literal stream
      // the dword that holds the frontier: the last one the previous span assembled (its
      // bytes before F are final: that span's own or its head), so only a window's first
      // span loads it
      uint32_t hcar = 0;
      bool hcar_ok = false;
#ifdef HZ2_EXP_NOM
      for (uint32_t b0 = 0; F < 0u;) {
#else
      for (uint32_t b0 = 0; F < wend;) {
#endif
        HZ_T(14);
        HZ2_MARK("M_BATCH");
        if (stats) stats->batches++;
#if HZ2_FUSE
        // (phase E's check, on the records' absolute positions: a distance past the stream start)
        if (WAVE_BALLOT(hz2::rec_bad(LV(ro), LV(rw)))) return ST_DATA;
#endif
        uint32_t nb = 0, open_ = 1;
HZ_UNROLL
        for (uint32_t u = 0; u < MPL; u++) {
          const uint64_t fit = WAVE_BALLOT(LV(ro)[u] != 0xffffffffu && LV(ro)[u] + (LV(rw)[u] >> 16) - F <= SPAN);
          const uint32_t k = ~fit ? (uint32_t)__builtin_ctzll(~fit) : 64u;   // leading fitting matches
          nb += open_ ? k : 0u;
          open_ = open_ && k == 64u;
        }
        uint32_t span;
        if (nb) {
          const uint32_t last_o = LVA_AT(ro, (nb - 1u) >> 6, (nb - 1u) & 63u);
          const uint32_t last_w = LVA_AT(rw, (nb - 1u) >> 6, (nb - 1u) & 63u);
          span = last_o + (last_w >> 16) - F;
        } else {
          const uint32_t nxt = b0 < mtotal ? LVA_AT(ro, 0u, 0u) : wend;
          span = nxt - F < SPAN ? nxt - F : SPAN;
        }
        // the span's first dword holds bytes before F (final): loaded now, merged below
        const uint32_t mis = (uint32_t)((uintptr_t)(job.dst + F) & 3u);
        const uint32_t xa = F - mis;                           // stream position of dword 0
        const uint32_t ndw = (span + mis + 3u) >> 2;
        const bool head = mis && (int32_t)xa >= 0 && xa + 4u <= dst_len;   // dword 0 loaded (whole-stored)
        // (the previous span's last dword; loaded only for a window's first span, and waited
        // for inside that branch: a load left pending at the merge makes the compiler wait
        // for it -- a memory latency -- on every span)
        uint32_t hl = hcar;
        if (head && !hcar_ok) {
          hl = *(hz_gu32*)(dst + xa);
          HZ2_VMWAIT();
        }
        const uint32_t hv = head ? hl : 0u;
        HZ_T(8);
        // the whole map is cleared (three 16-byte stores per lane): slots past the span read 0
        static_assert(SPAN % 256u == 0u, "smap clear: whole 8-byte stores per lane");
        LANE_LOOP {
#if HZ_GPU
          if constexpr (SPAN % 512u == 0u) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4* const zp = (u32x4*)&sh.smap[(SPAN / 64u) * (uint32_t)lane];
            const u32x4 z = {0u, 0u, 0u, 0u};
HZ_UNROLL
            for (uint32_t k = 0; k < SPAN / 512u; k++) zp[k] = z;
          } else {
            uint64_t* const zp = (uint64_t*)&sh.smap[(SPAN / 64u) * (uint32_t)lane];
HZ_UNROLL
            for (uint32_t k = 0; k < SPAN / 256u; k++) zp[k] = 0ull;
          }
#else
          memset(&sh.smap[(SPAN / 64u) * (uint32_t)lane], 0, SPAN / 32u);
#endif
        }
        HZ2_LSYNC();
        if (stats) {
          uint64_t mx = 0, sm = 0;
          for (int l = 0; l < 64; l++) {
            uint64_t f = 0;
            for (uint32_t u = 0; u < MPL; u++)
              if ((uint32_t)l + 64u * u < nb) f += LVA_AT(rw, u, l) >> 16;
            mx = f > mx ? f : mx;
            sm += f;
          }
          stats->fill_max += mx; stats->fill_sum += sm; stats->span_sum += span;
        }
        LANE_LOOP {
HZ_UNROLL
          for (uint32_t u = 0; u < MPL; u++) {
            if ((uint32_t)lane + 64u * u < nb) {
              const uint32_t o0 = LV(ro)[u] - F, ln = LV(rw)[u] >> 16, d = (LV(rw)[u] & 0xffffu) + 1u;
              // byte t copies o - d + (t mod d): distance d + d * floor(t / d).  Four bytes
              // per iteration (bytes past the match go to the junk entry SPAN + 1): the wave
              // runs as many iterations as its longest match needs
              uint32_t dist = d, jj = 0;
              for (uint32_t t0 = 0; t0 < ln; t0 += 4u) {
HZ_UNROLL
                for (uint32_t k = 0; k < 4u; k++) {
                  const uint32_t t = t0 + k;
                  sh.smap[t < ln ? o0 + t : SPAN + 1u] = (uint16_t)dist;
                  jj++;
                  const bool w = jj == d;
                  jj = w ? 0u : jj;
                  dist += w ? d : 0u;
                }
              }
            }
          }
        }
        HZ2_LSYNC();
        HZ_T(15);
        // prefetch the next batch's records
        LANE_ARR(uint32_t, no, MPL);
        LANE_ARR(uint32_t, nw, MPL);
#if HZ2_FUSE
        load_recs(b0 + nb, no, nw);
#else
        LANE_LOOP {
HZ_UNROLL
          for (uint32_t u = 0; u < MPL; u++) {
            const uint32_t j = b0 + nb + (uint32_t)lane + 64u * u;
            LV(no)[u] = j < mtotal ? ring[2u * j] : 0xffffffffu;
            LV(nw)[u] = j < mtotal ? ring[2u * j + 1u] : 0u;
          }
        }
#endif
        HZ_T(11);
        HZ2_MARK("M_JUMP");
        // 2. pointer jumping over the span's match bytes (branch-free per slot: a slot's
        // source index is min(q - d, SPAN), and smap[SPAN] stays 0, so literal slots (d = 0
        // reads smap[q] = 0), sources before F (q - d wraps) and slots past the span (d = 0)
        // never move; every slot's entry is written back each round)
        LANE_ARR(uint32_t, dq, RGP);
        LANE_LOOP {
HZ_UNROLL
          for (uint32_t i = 0; i < RGP; i++) LV(dq)[i] = sh.smap[(uint32_t)lane + 64u * i];
        }
        if (nb) {
          for (;;) {
            LANE_VAR(uint32_t, chg);
            LANE_LOOP {
              uint32_t d2[RGP];
HZ_UNROLL
              for (uint32_t i = 0; i < RGP; i++) {
                const uint32_t y = (uint32_t)lane + 64u * i - LV(dq)[i];
                d2[i] = sh.smap[y < SPAN ? y : SPAN];
              }
              uint32_t c = 0;
HZ_UNROLL
              for (uint32_t i = 0; i < RGP; i++) {
                c |= d2[i];
                LV(dq)[i] += d2[i];
              }
              LV(chg) = c;
              if (stats) for (uint32_t i = 0; i < RGP; i++) stats->hops += d2[i] != 0u;
            }
            if (stats) stats->tokens++;                // (emulator statistic: pointer-jumping rounds)
            if (!WAVE_BALLOT(LV(chg) != 0u)) break;
            HZ2_LSYNC();
            LANE_LOOP {
HZ_UNROLL
              for (uint32_t i = 0; i < RGP; i++) sh.smap[(uint32_t)lane + 64u * i] = (uint16_t)LV(dq)[i];
            }
            HZ2_LSYNC();
          }
        }
        HZ_T(12);
        HZ2_MARK("M_GATHER");
        // 3. gather, branch-free per slot: two byte loads each (a literal's from the literal
        // stream -- its rank among the span's literals by ballot -- and a source before F from
        // dst; the other load reads a harmless in-range byte) and a select; LDS byte writes of
        // slots that take no byte go to a junk byte past the span buffer
        constexpr uint32_t JUNK = (SPAN / 4u + 2u) * 4u - 1u;
        LANE_VAR(uint32_t, vm);                 // slots inside the span
        LANE_LOOP {
          const uint32_t nv = span > (uint32_t)lane ? ((span - 1u - (uint32_t)lane) >> 6) + 1u : 0u;
          LV(vm) = nv >= 32u ? ~0u : (1u << nv) - 1u;
        }
        // per-slot flags live as VGPR bit masks (bit i: slot i), not as per-slot predicates:
        // the compiler would keep 24 of those in SGPR pairs across the batch and spill them
        LANE_VAR(uint32_t, lb);                 // literal slots
        LANE_VAR(uint32_t, fb);                 // match bytes whose source lies before F
        LANE_LOOP { LV(lb) = 0; LV(fb) = 0; if (lane == 0) sh.sbuf[0] = hv; }
        HZ2_LSYNC();
        uint32_t lcnt = 0;                      // literals of the span so far (wave-uniform)
#if HZ2_FUSE
        LANE_VAR(uint32_t, vlb);                // the lanes' literal shares (registers, v_readlane)
        LANE_VAR(uint32_t, vle);
        LANE_VAR(uint32_t, vld);
        LANE_LOOP { LV(vlb) = sh.lb[lane]; LV(vle) = sh.le[lane]; LV(vld) = sh.ldl[lane]; }
#endif
        // two halves of GH slots: GH loaded bytes in flight per lane (all 24 spill)
        constexpr uint32_t GH = RGP / 2u;
HZ_UNROLL
        for (uint32_t h = 0; h < RGP; h += GH) {
          LANE_ARR(uint32_t, bv, GH);
HZ_UNROLL
          for (uint32_t k = 0; k < GH; k++) {
            const uint32_t i = h + k;
            const uint64_t bm = WAVE_BALLOT(((LV(vm) >> i) & 1u) && LV(dq)[i] == 0u);
#if HZ2_FUSE
            // the slot's literal ranks [R0, R1): region deltas by the cursor
            const uint32_t R0 = L0 + lcnt, R1 = R0 + (uint32_t)hz::popc64(bm);
            LANE_VAR(uint32_t, ldx);
            LANE_LOOP { LV(ldx) = lcd; }
            while (R1 > lend && lcur < 63u) {
              lcur++;
              const uint32_t b = LV_AT(vlb, lcur);
              lend = LV_AT(vle, lcur);
              lcd = LV_AT(vld, lcur);
              LANE_LOOP { LV(ldx) = R0 + hz2::lane_rank(bm, lane) >= b ? lcd : LV(ldx); }
            }
#endif
            LANE_LOOP {
              const uint32_t q = (uint32_t)lane + 64u * i, d = LV(dq)[i];
              const uint32_t isl = (LV(vm) >> i) & (d == 0u ? 1u : 0u);
              const uint32_t far = d > q ? 1u : 0u;      // (never for a slot past the span: d = 0)
              LV(lb) |= isl << i;
              LV(fb) |= far << i;
              // one load: the 64-bit address selected as an integer (a pointer select becomes
              // a branch), a harmless in-range byte of dst (F) for slots that take no byte
#ifdef HZ2_EXP_NOLITLOAD                  // (traffic attribution builds: outputs wrong)
              const uint64_t la = (uint64_t)(uintptr_t)lits;
#elif HZ2_FUSE
              const uint64_t la = (uint64_t)(uintptr_t)lits + (uint32_t)(R0 + hz2::lane_rank(bm, lane) + LV(ldx));
#else
              const uint64_t la = (uint64_t)(uintptr_t)lits + L0 + lcnt + hz2::lane_rank(bm, lane);
#endif
#ifdef HZ2_EXP_NOFAR
              const uint64_t da = (uint64_t)(uintptr_t)dst + F;
#else
              const uint64_t da = (uint64_t)(uintptr_t)dst + (far ? F + q - d : F);
#endif
              LV(bv)[k] = *HZ_GLOBAL(hz_gcu8*, (uintptr_t)(isl ? la : da));
              if (stats && far) stats->src_far[d - q <= 256u ? 0 : d - q <= 1536u ? 1 : d - q <= 4096u ? 2 : 3]++;
            }
            lcnt += (uint32_t)hz::popc64(bm);
          }
          LANE_LOOP {
            uint32_t a1 = 0, b2 = 0;       // adler: sum b, batch-relative sum (x - F) b
            uint8_t* const sb = (uint8_t*)sh.sbuf;
            const uint32_t tb = LV(lb) | LV(fb);
HZ_UNROLL
            for (uint32_t k = 0; k < GH; k++) {
              const uint32_t i = h + k;
              const uint32_t q = (uint32_t)lane + 64u * i, v = LV(bv)[k];
              const uint32_t tk = (tb >> i) & 1u;       // a literal or a byte from before F
              sb[tk ? q + mis : JUNK] = (uint8_t)v;
              a1 += tk * v;
              b2 += tk * (q * v);
            }
            LV(ra1) += a1;
            LV(ra2) += (uint64_t)F * a1 + b2;
          }
        }
        HZ2_LSYNC();
        // in-span sources: literals of the span, now in LDS
        LANE_LOOP {
          uint32_t a1 = 0, b2 = 0;
          uint8_t* const sb = (uint8_t*)sh.sbuf;
          const uint32_t ib = LV(vm) & ~(LV(lb) | LV(fb));
          uint32_t v[RGP];
HZ_UNROLL
          for (uint32_t i = 0; i < RGP; i++) {
            const uint32_t q = (uint32_t)lane + 64u * i;
            v[i] = sb[((ib >> i) & 1u) ? q - LV(dq)[i] + mis : JUNK];
          }
HZ_UNROLL
          for (uint32_t i = 0; i < RGP; i++) {
            const uint32_t q = (uint32_t)lane + 64u * i, inb = (ib >> i) & 1u;
            sb[inb ? q + mis : JUNK] = (uint8_t)v[i];
            a1 += inb * v[i];
            b2 += inb * (q * v[i]);
            if (stats && inb) stats->src_in++;
          }
          LV(ra1) += a1;
          LV(ra2) += (uint64_t)F * a1 + b2;
        }
        HZ2_LSYNC();
        HZ_T(13);
        HZ2_MARK("M_STORE");
        // 4. store: whole dwords inside the span (dword 0 also when its head was loaded) and
        // the stream; the span's edge bytes one by one.  HZ2_ST16: lane t takes dwords
        // 4t .. 4t+3 with one 16-byte store when all four lie inside (a 1 KiB span is one
        // store instruction); those lanes are a contiguous range [a, b] (only lane 0 can fail
        // at the head, and a prefix of lanes fits the span), and the few dwords outside it
        // -- [0, 4a) and [4b + 4, ndw) -- go dword by dword, one per lane
        {
          auto store_dword = [&](int lane, uint32_t k) {
            (void)lane;
            const uint32_t x0 = xa + 4u * k;
            const bool inside = (int32_t)x0 >= 0 && x0 + 4u <= dst_len && x0 + 4u <= F + span && (k > 0u || !mis || head);
#ifdef HZ2_EXP_NOMSTORE                   // (traffic attribution builds: outputs wrong)
            (void)inside;
#else
            if (inside) {
              *(hz_gu32*)(dst + x0) = sh.sbuf[k];
            } else {
              for (uint32_t b = 0; b < 4u; b++) {
                const uint32_t x = x0 + b;
                if (x >= F && x < F + span && x < dst_len) dst[x] = ((const uint8_t*)sh.sbuf)[4u * k + b];
              }
            }
#endif
          };
#if HZ2_ST16
          LANE_VAR(uint32_t, st4);
          LANE_LOOP {
            const uint32_t k0 = 4u * (uint32_t)lane, x0 = xa + 16u * (uint32_t)lane;
            LV(st4) = (k0 + 4u <= ndw && (int32_t)x0 >= 0 && x0 + 16u <= dst_len && x0 + 16u <= F + span &&
                       (lane > 0 || !mis || head)) ? 1u : 0u;
          }
          const uint64_t m4 = WAVE_BALLOT(LV(st4) != 0u);
          if (m4) {
            const uint32_t a = (uint32_t)__builtin_ctzll(m4), b = 63u - (uint32_t)__builtin_clzll(m4);
            LANE_LOOP {
#ifndef HZ2_EXP_NOMSTORE
              if (LV(st4)) {
                const uint32_t k0 = 4u * (uint32_t)lane;
#if HZ_GPU
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                typedef __attribute__((address_space(1))) u32x4 gu32x4;
                *(gu32x4*)(dst + (uint32_t)(xa + 4u * k0)) = *(const u32x4*)&sh.sbuf[k0];   // (xa may wrap: 32-bit sum)
#else
                memcpy(dst + (uint32_t)(xa + 4u * k0), &sh.sbuf[k0], 16);
#endif
              }
#endif
              const uint32_t lo = 4u * a, hi = 4u * b + 4u, nun = lo + (ndw - hi);
              for (uint32_t t = (uint32_t)lane; t < nun; t += 64u) store_dword(lane, t < lo ? t : hi + (t - lo));
            }
          } else
#endif
          {
            LANE_LOOP {
              for (uint32_t k = (uint32_t)lane; k < ndw; k += 64u) store_dword(lane, k);
            }
          }
        }
        hcar = sh.sbuf[ndw - 1u];
        hcar_ok = true;
        HZ2_GSYNC();      // this wave reads the stored dwords back as far sources
        LANE_LOOP {
HZ_UNROLL
          for (uint32_t u = 0; u < MPL; u++) { LV(ro)[u] = LV(no)[u]; LV(rw)[u] = LV(nw)[u]; }
        }
        HZ2_MARK("M_END");
        b0 += nb;
        F += span;
        L0 += lcnt;
      }
      LANE_LOOP {
        LV(s1) = (LV(s1) + LV(ra1) % ADLER_MOD) % ADLER_MOD;
        LV(s2) = (uint32_t)((LV(s2) + LV(ra2) % ADLER_MOD) % ADLER_MOD);
      }

      HZ_T(10);
      output_done();
      return ST_OK;
    }();
    if (wst != ST_OK) {
      fail = wst;
      if (NW > 1) atomic_min_err(pipe.ctl, wst);
      break;
    }
  }
  if (NW > 1) {
    // all wavefronts: every window done (or failed); the adler sums of all
    if (fail != ST_OK) atomic_min_err(pipe.ctl, fail);
    HZ2_WGBAR();
    const int32_t e = (int32_t)ctl_ld((const uint32_t*)&pipe.ctl->err);
    if (e) return e;
    cur = pipe.ctl->next;                 // the END state: trailer position and total output
  } else if (fail != ST_OK) {
    return fail;
  }
  uint32_t pos = cur.pos;
  const uint32_t out = cur.out;
  // ---- trailer: adler32 (big-endian) after byte alignment ----
  HZ_T(9);
  pos = (pos + 7u) & ~7u;
  if (pos + 32u > limit_bits) return ST_TRUNC;
  uint32_t t32;
  {
    GRd r;
    g_init(S, r, pos);
    t32 = (uint32_t)(g_peek(r) & 0xffffffffu);
  }
  const uint32_t want = (t32 >> 24) | ((t32 >> 8) & 0xff00u) | ((t32 << 8) & 0xff0000u) | (t32 << 24);
  uint64_t S1 = 0, S2 = 0;
#if HZ_GPU
  S1 = hz::wave_sum64((uint64_t)s1);
  S2 = hz::wave_sum64((uint64_t)s2);
#else
  for (int lane = 0; lane < 64; lane++) { S1 += s1[lane]; S2 += s2[lane]; }
#endif
  if (NW > 1) {
    // the wavefronts' partial sums, added up through LDS
    Ctl* c = pipe.ctl;
    c->adler[pipe.w][0] = S1;
    c->adler[pipe.w][1] = S2;
    HZ2_WGBAR();
    S1 = 0; S2 = 0;
    for (int i = 0; i < NW; i++) { S1 += c->adler[i][0]; S2 += c->adler[i][1]; }
  }
  const uint32_t A = (uint32_t)((1u + S1) % ADLER_MOD);
  const uint32_t B = (uint32_t)(((uint64_t)(out % ADLER_MOD) * A + ADLER_MOD - (S2 % ADLER_MOD)) % ADLER_MOD);
  if (((B << 16) | A) != want) return ST_DATA;
  if (job.exact && out != dst_len) return ST_SIZE;
  if (job.out_len) *job.out_len = out;
  return ST_OK;
}

// The window pipeline (NW > 1) with its timeout fallback.  A wait that gives up (ST_HANG:
// a neighbouring window that never finished) is no evidence of corrupt data, so the stream
// is decoded again by wavefront 0 alone (NW = 1, no waits), and every wavefront returns that
// decode's status.  All NW wavefronts of the workgroup call this together: the fallback path
// has a workgroup barrier.  (ST_HANG is uniform: inflate_stream<NW> returns Ctl::err, the
// first failure of any wavefront, to all of them.)
template <class StatsT, int NW>
#if HZ_GPU
__device__ __forceinline__
#else
static
#endif
int inflate_stream_pipe(Shared& sh, const Job job, const Tune tune, uint8_t* ring_base, StatsT* stats, HzProf* prof,
                        Pipe pipe) {
  int st = inflate_stream<StatsT, NW>(sh, job, tune, ring_base, stats, prof, pipe);
  if (st == ST_HANG) {
    if (stats) stats->hangs++;
    if (pipe.w == 0u) {
      const int r = inflate_stream<StatsT, 1>(sh, job, tune, ring_base, stats, prof);
      // (not in Ctl::err: the other wavefronts may still be reading that one)
      LANE_LOOP { if (lane == 0) ctl_st((uint32_t*)&pipe.ctl->redo, (uint32_t)r); }
    }
    HZ2_WGBAR();
    st = (int32_t)ctl_ld((const uint32_t*)&pipe.ctl->redo);
  }
  return st;
}

}  // namespace hz2
