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
// The recorded starts live in registers (the LDS holds the staging instead).  The two-pass
// form (phase E decodes every valid range again into the window-ordered ring, rounds 2-5)
// stays for the window pipeline (inflate_stream below)
#ifndef HZ2_FUSE
#define HZ2_FUSE 1                        // one pass for one wavefront per stream
#endif
#ifndef HZ2_FUSE_PIPE
#define HZ2_FUSE_PIPE 0                   // one pass in the window pipeline (NW > 1) as well
#endif
#ifndef HZ2_K
#define HZ2_K 8
#endif
constexpr int K = HZ2_K;                  // recorded token starts per lane (two-pass form, LDS)
#ifndef HZ2_K1
#define HZ2_K1 8
#endif
constexpr int K1 = HZ2_K1;                // recorded token starts per lane (one-pass form, registers)
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
// (round 6, two boxes, three pairs each, tools/gpu_r6ai.sh: 3 instead of 4 -- 6 fewer live
// registers in M, 22 VGPRs spilled instead of 24 -- F1 equal, F2 149.1 -> 152.0 GB/s)
#ifndef HZ2_MPL
#define HZ2_MPL 3
#endif
constexpr uint32_t MPL = HZ2_MPL;         // resolve: matches per lane per batch
#ifndef HZ2_FILLCAP
#define HZ2_FILLCAP 16
#endif
constexpr uint32_t FILL_CAP = HZ2_FILLCAP;
   // resolve: source-map bytes a lane fills per match (258: all)
static_assert(MPL >= 2 && MPL <= 4, "sel4 selects among up to four per-lane matches");
constexpr uint32_t SPL = SPAN / WAVE;     // resolve: span bytes per lane
static_assert(SPL <= 24, "resolve slots per lane");
constexpr uint32_t RGP = SPL;              // resolve: byte slots per lane (q = lane + 64 i)
// Every hand-off inside one stream's decode is wavefront-scope (HZ2_LSYNC for LDS,
// HZ2_GSYNC for the wave's own global stores read back by its later loads): no s_barrier,
// no s_waitcnt vmcnt(0) -- loads in flight (the next span's records) stay in flight, and
// two wavefronts of one workgroup can decode two windows of a stream independently
// (inflate2w_kernel); their hand-offs are workgroup-scope release / acquire on Ctl.
// phases A / E: match records are staged per lane and stored as whole aligned 32-byte groups
// (16-byte stores of each lane's own records, scattered over 64 lanes, cost about 4x their
// bytes in HBM writes plus L2 fills: measured, profiles/r2_traffic_attribution.txt).  Round 6
// A/B on one box (profiles/r6_ab_record_groups.txt): 16-byte groups 196.1-200.8 GB/s, 32-byte
// groups (last record from registers, no ring mirror: 16 waves per CU) 203.0-203.2, HBM traffic
// per launch 90.4 -> 77.8 GB; 32-byte groups staged whole cost the 16th wave (173 GB/s)
#ifndef HZ2_RGRP
#define HZ2_RGRP 4
#endif
constexpr uint32_t RGRP = HZ2_RGRP;
static_assert(RGRP == 2 || RGRP == 4 || RGRP == 8, "RGRP: 2, 4 or 8 records");
// the last record of a group is stored from registers with the staged ones (it completes
// the group), so the LDS stage holds RGRP - 1 records per lane (1: on)
#ifndef HZ2_RLAST
#define HZ2_RLAST 1
#endif
constexpr uint32_t RSTG = RGRP - (HZ2_RLAST ? 1u : 0u);    // staged records per lane
// bit ring (phases A .. E): RS stream words per lane in LDS, refilled a quad at a time at
// wave-uniform ticks; a token reads at most 48 bits, so a window advances at most 1.5
// words per token
#ifndef HZ2_RS
#define HZ2_RS 12
#endif
constexpr uint32_t RS = HZ2_RS;           // ring words per lane (a multiple of 4)
#ifndef HZ2_MIRROR
#define HZ2_MIRROR 0                      // a copy of ring slot 0 after slot RS - 1 (no wrap select;
                                          // its 256 bytes of LDS go to the record stage instead)
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
// wave priority by the stream's remaining work (s_setprio at every window start): HZ2_PRIO
// levels, one per HZ2_PRIO_ABS KiB of input left (the highest from 3 x 40 KiB up); 0 = off.
// A/B round 5, 4096 chunks: by output fraction (HZ2_PRIO_ABS 0) F1 26.0 -> 25.5 ms, F2 38.2 ->
// 35.9 ms, waves busy F1 0.897 -> 0.961, F2 0.83 -> 0.87; by remaining input, 40 KiB per level,
// F1 180.4 -> 183.0 GB/s, F2 115.1 -> 120.0 (16 / 24 / 32 / 64 / 128 KiB measured worse)
#ifndef HZ2_PRIO
#define HZ2_PRIO 4
#endif
#ifndef HZ2_PRIO_ABS
#define HZ2_PRIO_ABS 40
#endif
// M's record loads non-temporal: the records are read once, so their lines go first when L2
// evicts, and the output lines the far-source gathers read stay longer.  Three boxes (tools/
// gpu_r6ae.sh, gpu_r6af.sh, gpu_r6ag.sh): F1 +0 / +3 / -0.3 %, HBM traffic -3 % (FETCH 15.4 ->
// 14.6 GB per 2048 chunks).  The gathers' loads made non-temporal too lost 6-9 %.
#ifndef HZ2_NTREC
#define HZ2_NTREC 1
#endif
#ifndef HZ2_NTGATH
#define HZ2_NTGATH 0                      // M's gather loads non-temporal (experiment)
#endif
// phase A's warm-up decoded by a loop of its own (1) or inside the segment loop (0)
#ifndef HZ2_WARM2
#define HZ2_WARM2 1
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
static_assert(K >= 1 && K <= 16 && K1 >= 1 && K1 <= 16, "record fields hold K <= 16 tokens");
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
          uint64_t rstage[WAVE][RSTG];              // each lane's current group of match records
        };
      };
    };
    struct {                      // phase M
      uint16_t smap[SPAN + 2];    // batch byte -> distance to its source (0: literal); [SPAN] stays 0
      alignas(16) uint32_t sbuf[SPAN / 4 + 4];   // the batch's aligned dwords, assembled in LDS
      // one-pass decoder: lane s's share of the window (written after the prefix sums): its
      // first window record mb[s] and literal rank lb[s], the region index minus the window
      // index of its records (rdl) and literals (ldl), the window position minus the region
      // position of its records (odl), and the end of its literal ranks (le)
      uint32_t mb[WAVE], rdl[WAVE], odl[WAVE], lb[WAVE], le[WAVE], ldl[WAVE];
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

// the compressed stream is read once (A's warm-up overlaps aside): HZ2_NTBITS = 1 loads it
// non-temporally, so it does not push the match records and recent output out of L2
#ifndef HZ2_NTBITS
#define HZ2_NTBITS 0
#endif
// quad qa (clamped to the stream's last quad: an aligned 16-byte block holding a stream
// byte never crosses a page, so the load is always safe)
HZ_HD void g_quad(const Src& s, uint32_t qa, uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3) {
  const uint32_t b0 = (qa < s.last ? qa : s.last) * 4u;
#if HZ_GPU
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
#if HZ2_NTBITS
  const u32x4 v = __builtin_nontemporal_load((gu32x4*)(s.base + b0));
#else
  const u32x4 v = *(gu32x4*)(s.base + b0);
#endif
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
#if HZ2_RS > 12
// a larger ring (latency experiments: fewer ticks per token): as many quads as fit
constexpr uint32_t NQF = RS / 4u;
HZ_HD void br_fill(Shared& sh, int lane, const Src& S, BR& r) {
  uint32_t a[4 * NQF];
  bool f[NQF];
HZ_UNROLL
  for (uint32_t q = 0; q < NQF; q++) {
    f[q] = r.wr + 4u * q + 1u <= r.c + RS;
    if (f[q]) g_quad(S, r.wr + 4u * q, a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
  }
HZ_UNROLL
  for (uint32_t q = 0; q < NQF; q++) {
    if (f[q]) {
      br_put(sh, lane, r.wslot, a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
      r.wr += 4u;
      r.wslot = slot4(r.wslot);
    }
  }
}
#else
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
#endif

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

// lens[n .. n + rep) = val (a code-length run): bytes up to a dword boundary, then dwords
HZ2_HM void fill_run(uint8_t* p, uint32_t n, uint32_t rep, uint32_t val) {
  uint32_t i = n;
  const uint32_t e = n + rep;
  while (i < e && ((uintptr_t)(p + i) & 3u)) p[i++] = (uint8_t)val;
  const uint32_t w = val * 0x01010101u;
  for (; i + 4u <= e; i += 4u) *(uint32_t*)(p + i) = w;
  while (i < e) p[i++] = (uint8_t)val;
}

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

// a * b for a, b < 2^24 with a product < 2^32 (v_mul_u32_u24: full rate)
HZ_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if HZ_GPU
  return __umul24(a, b);
#else
  return a * b;
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

// a[u] for a register array and a runtime u < MPL (no dynamic register indexing)
HZ_HD uint32_t sel4(const uint32_t* a, uint32_t u) { return u == 0u ? a[0] : (u == 1u || MPL < 3u) ? a[1] : (u == 2u || MPL < 4u) ? a[MPL < 3u ? 1u : 2u] : a[MPL - 1u]; }
// a[j] of a lane's K recorded starts (registers) for a runtime j < K: masks OR-ed (a select
// chain is folded back into an indexed load, which puts the array in scratch)
template <int N>
HZ_HD uint32_t selk(const uint32_t* a, uint32_t j) {
  uint32_t v = 0;
HZ_UNROLL
  for (uint32_t i = 0; i < (uint32_t)N; i++) v |= a[i] & (0u - (uint32_t)(j == i));
  return v;
}
template <int N>
HZ_HD void setk(uint32_t* a, uint32_t j, uint32_t v, bool on) {
HZ_UNROLL
  for (uint32_t i = 0; i < (uint32_t)N; i++) a[i] = (on && j == i) ? v : a[i];
}
// a lane's batch records: one of the span's (index < nb) longer than FILL_CAP
HZ_HD bool has_long(const uint32_t* w, uint32_t lane, uint32_t nb) {
  bool r = false;
HZ_UNROLL
  for (uint32_t u = 0; u < MPL; u++) r |= lane + 64u * u < nb && (w[u] >> 16) > FILL_CAP;
  return r;
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
// (the counter is wave-uniform -- the lanes of a loop tick together -- and kept so: a scalar
// register, no per-token VALU increment and readfirstlane)
#define HZ2_RTICK(it) do { (it) = HZ2_UNI(it) + 1u; if ((it) % hz2::TICKN == 0u) hz2::br_tick(sh, lane, S, r); } while (0)

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
constexpr int NW_MAX = 8;        // wavefronts per stream in the window pipeline
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
// The stream decoder, compiled in its two forms (inflate2_stream.inc):
#define HZ2_ONEPASS 1
#define HZ2_STREAM_FN inflate_stream_1p
#include "inflate2_stream.inc"
#undef HZ2_STREAM_FN
#undef HZ2_ONEPASS
#define HZ2_ONEPASS 0
#define HZ2_STREAM_FN inflate_stream_2p
#include "inflate2_stream.inc"
#undef HZ2_STREAM_FN
#undef HZ2_ONEPASS

// one pass for one wavefront per stream (the batch path: phase E's second decode is work
// the wave would do itself); two passes for the window pipeline, whose critical path is the
// chain of the windows' sync phases -- there phase E runs beside the other wavefront's M, and
// emitting inside phase A would lengthen the chain (one F2 chunk on four wavefronts: 16.9 ms
// one-pass, 14.7 two-pass)
template <class StatsT, int NW>
#if HZ_GPU
__device__ __forceinline__
#else
static
#endif
int inflate_stream(Shared& sh, const Job job, const Tune tune, uint8_t* ring_base, StatsT* stats, HzProf* prof = nullptr,
                   Pipe pipe = Pipe{nullptr, nullptr, 0u}) {
  if constexpr ((NW == 1 && HZ2_FUSE) || (NW > 1 && HZ2_FUSE_PIPE))
    return inflate_stream_1p<StatsT, NW>(sh, job, tune, ring_base, stats, prof, pipe);
  else
    return inflate_stream_2p<StatsT, NW>(sh, job, tune, ring_base, stats, prof, pipe);
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
