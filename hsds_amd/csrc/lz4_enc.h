// lz4_enc.h -- LZ4 and BloscLZ block writers for the Blosc-lz4 / -lz4hc / -blosclz write path.
//
// storUtil._compress (hsds/util/storUtil.py:238-281) encodes with
// Blosc(cname=<the dataset's compressor>); for "lz4" / "lz4hc" c-blosc 1.21 calls
// lz4_wrap_compress once per split.  The compressed bytes need not equal lz4's (any
// valid block is accepted); the frame must decode to the input
// through c-blosc and the reference's _uncompress.
//
// The match finding is the deflate encoder's parse phase (deflate_wave.h P: exact hash
// chains over an 8 KiB window, lane-parallel greedy parse, tokens in HBM).  This file
// turns one split's token list into an LZ4 block, one wavefront per split (each lane
// keeps the token range the parse gave it; see lz4_block_wave), length-3 matches
// become literals, and the block end rules LZ4_decompress_safe enforces are kept (the
// last match starts at least MFLIMIT = 12 bytes before the end and ends at least
// LASTLITERALS = 5 bytes before it).  The walk runs twice: once for the size (frame
// layout), once to write.
//
// Single source: tests/emu/deflate_emu.cpp runs the same walk on CPU.
#pragma once
#include "deflate_wave.h"
#include "lz_wave.h"

namespace lze {

struct Out {
  hz_gu8* p;
  uint32_t n;
  int write;
};
HZ_HD void put(Out& o, uint32_t b) {
  if (o.write) o.p[o.n] = (uint8_t)b;
  o.n++;
}
HZ_HD void put_len(Out& o, uint32_t v) {
  while (v >= 255u) { put(o, 255u); v -= 255u; }
  put(o, v);
}

// the split's input bytes: direct (ts == 1) or gathered from the byte-shuffled block
struct InRd {
  lz::ByteRd r;
  hz_gcu8* blk;
  uint32_t ts, neb, off;
};
HZ_HD void in_init(InRd& in, const hd::EncJob& job) {
  const uint32_t a = (uint32_t)(((uintptr_t)job.src) & 3u);
  in.r.base = HZ_GLOBAL(hz_gcu8*, job.src - a);
  in.r.lo = a;
  in.r.hi = a + (job.ts > 1u ? job.off + job.len : job.len);
  in.r.bpos = 0x80000000u;
  in.r.stg = nullptr;
  in.r.sb = 0x80000000u;                    // no LDS stage: every refill from global memory
  in.r.buf = 0;
  in.blk = HZ_GLOBAL(hz_gcu8*, job.src);
  in.ts = job.ts; in.neb = job.neb; in.off = job.off;
}
HZ_HD uint32_t in_byte(InRd& in, uint32_t pos) {
  return in.ts > 1u ? (uint32_t)in.blk[hd::shuffled_src_index(in.off + pos, in.ts, in.neb)] : lz::rd_byte(in.r, pos);
}

// Literal runs of RUN_MIN bytes or more are not copied by the lane that owns their
// sequence (a run can span many lanes' token ranges, up to a whole incompressible
// block): the lane reserves the bytes and lists the run; the whole wave then copies
// the listed runs (flush_runs), 64 bytes per instruction, CP_UNR independent loads in
// flight per lane before their stores (one memory latency per 64 * CP_UNR bytes).
#ifndef HZ_RUN_MIN
#define HZ_RUN_MIN 32
#endif
constexpr uint32_t RUN_MIN = HZ_RUN_MIN;
constexpr uint32_t CP_UNR = 8;
constexpr uint32_t RUN_CAP = 8192u / RUN_MIN + 8u;   // > SEG / RUN_MIN + carried run + final run
struct CopyRun {
  hz_gu8* dst;
  uint32_t src, len;
};
struct CopyList {
  uint32_t n;
  CopyRun r[RUN_CAP];
};
HZ_HD bool defer_run(CopyList* cl, hz_gu8* dst, uint32_t src, uint32_t len) {
  if (!cl) return false;
#if HZ_GPU
  const uint32_t k = atomicAdd(&cl->n, 1u);
#else
  const uint32_t k = cl->n++;
#endif
  if (k >= RUN_CAP) return false;        // list full: the lane copies the run itself
  cl->r[k].dst = dst;
  cl->r[k].src = src;
  cl->r[k].len = len;
  return true;
}
#if HZ_GPU
__device__
#else
static
#endif
inline void flush_runs(CopyList* cl, const hd::EncJob& job) {
  WAVE_SYNC();
#ifdef HZ_EXP_NOFLUSH
  const uint32_t nr = 0;
#else
  const uint32_t nr = cl->n < RUN_CAP ? cl->n : RUN_CAP;
#endif
  hz_gcu8* s = HZ_GLOBAL(hz_gcu8*, job.src);
  for (uint32_t k = 0; k < nr; k++) {
    hz_gu8* const d = cl->r[k].dst;
    const uint32_t src = cl->r[k].src, len = cl->r[k].len;
    LANE_LOOP {
      for (uint32_t i0 = 0; i0 < len; i0 += 64u * CP_UNR) {
        uint8_t v[CP_UNR];
HZ_UNROLL
        for (uint32_t j = 0; j < CP_UNR; j++) {
          const uint32_t i = i0 + 64u * j + (uint32_t)lane;
          v[j] = i < len ? (job.ts > 1u ? s[hd::shuffled_src_index(job.off + src + i, job.ts, job.neb)] : s[src + i]) : 0;
        }
HZ_UNROLL
        for (uint32_t j = 0; j < CP_UNR; j++) {
          const uint32_t i = i0 + 64u * j + (uint32_t)lane;
          if (i < len) d[i] = v[j];
        }
      }
    }
  }
  WAVE_SYNC();
  LANE_LOOP { if (lane == 0) cl->n = 0; }
  WAVE_SYNC();
}

// literal bytes [l0, l1) of a direct (ts == 1) split to o, 32 bytes per round: the 9
// dwords covering a round are loaded together, so a round costs one memory latency
// (the byte reader's refills cost one per 4 - 8 bytes)
#ifndef HZ_LIT_ROUND
#define HZ_LIT_ROUND 32
#endif
HZ_HD void copy_lits(Out& o, const InRd& in, uint32_t l0, uint32_t l1) {
  constexpr uint32_t RB = HZ_LIT_ROUND, RW = RB / 4u;
  for (uint32_t p = l0; p < l1; p += RB) {
    const uint32_t ap = p + in.r.lo, w0 = ap >> 2, sh = (ap & 3u) * 8u;
    uint32_t dw[RW + 1];
HZ_UNROLL
    for (uint32_t k = 0; k <= RW; k++) dw[k] = hz::load_word(in.r.base, w0 + k, in.r.lo, in.r.hi);
    const uint32_t cnt = l1 - p < RB ? l1 - p : RB;
HZ_UNROLL
    for (uint32_t k = 0; k < RW; k++) {
      const uint32_t v = sh ? (dw[k] >> sh) | (dw[k + 1] << (32u - sh)) : dw[k];
HZ_UNROLL
      for (uint32_t b = 0; b < 4u; b++)
        if (4u * k + b < cnt) o.p[o.n + 4u * k + b] = (uint8_t)(v >> (8u * b));
    }
    o.n += cnt;
  }
}

// one sequence: literals [l0, l1), then a match (ml >= 4) of distance dist; ml == 0:
// the final literals-only sequence
HZ_HD void sequence(Out& o, InRd& in, uint32_t l0, uint32_t l1, uint32_t dist, uint32_t ml,
                    CopyList* cl = nullptr) {
  const uint32_t ll = l1 - l0;
  const uint32_t mc = ml ? (ml - 4u < 15u ? ml - 4u : 15u) : 0u;
  put(o, ((ll < 15u ? ll : 15u) << 4) | mc);
  if (ll >= 15u) put_len(o, ll - 15u);
  if (o.write) {
    if (ll >= RUN_MIN && defer_run(cl, o.p + o.n, l0, ll)) o.n += ll;
#ifdef HZ_EXP_NOLIT
    else o.n += ll;
#else
    else if (in.ts == 1u) copy_lits(o, in, l0, l1);
    else for (uint32_t p = l0; p < l1; p++) put(o, in_byte(in, p));
#endif
  } else {
    o.n += ll;
  }
  if (ml) {
    put(o, dist & 255u);
    put(o, dist >> 8);
    if (ml - 4u >= 15u) put_len(o, ml - 4u - 15u);
  }
}

HZ_HD uint32_t ext_len(uint32_t v) { return v >= 15u ? (v - 15u) / 255u + 1u : 0u; }
// bytes of a sequence with `run` literals and a match of ml bytes (ml == 0: none)
HZ_HD uint32_t seq_size(uint32_t run, uint32_t ml) { return 1u + ext_len(run) + run + (ml ? 2u + ext_len(ml - 4u) : 0u); }

// Walk lane `lane`'s parse tokens of one segment (input from p0): f(pos, len, dist)
// for every match of the parse, in order.  Token slots 2k, 2k+1 share the word
// (k * WAVE + lane); TB words are loaded per batch (independent loads in flight
// instead of one dependent load per token pair) and shifted through wv[0].
template <class F>
HZ_HD void lane_tokens(hz_gcu8* gtok, uint32_t ns, int lane, uint32_t p0, F&& f) {
  constexpr uint32_t TB = 8;
  hz_gcu32* gw = (hz_gcu32*)gtok;
  const uint32_t nw = (ns + 1u) >> 1;
  uint32_t pos = p0, tl = 0;
  bool want_dist = false;
  for (uint32_t w0 = 0; w0 < nw; w0 += TB) {
    uint32_t wv[TB];
#pragma unroll
    for (uint32_t i = 0; i < TB; i++)
      wv[i] = w0 + i < nw ? gw[(size_t)(w0 + i) * (uint32_t)hd::WAVE + (uint32_t)lane] : 0u;
    const uint32_t cnt = nw - w0 < TB ? nw - w0 : TB;
    for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t word = wv[0];
#pragma unroll
      for (uint32_t i = 0; i + 1 < TB; i++) wv[i] = wv[i + 1];
      const uint32_t s = 2u * (w0 + k);
      for (uint32_t h = 0; h < 2u && s + h < ns; h++) {
        const uint32_t t = h ? word >> 16 : word & 0xffffu;
        if (want_dist) {
          f(pos, tl, t + 1u);
          pos += tl;
          want_dist = false;
        } else if (t & 0x8000u) {
          tl = (t & 0x7fffu) + 3u;
          want_dist = true;
        } else {
          pos++;
        }
      }
    }
  }
}

// The matches an LZ4 block keeps: length-3 matches and matches breaking the block end
// rules (start within MFLIMIT = 12 bytes of the end, or ending within LASTLITERALS =
// 5) become literals / are shortened.  f(pos, ml, dist).
template <class F>
HZ_HD void lane_matches(hz_gcu8* gtok, uint32_t ns, int lane, uint32_t p0, uint32_t n, F&& f) {
  lane_tokens(gtok, ns, lane, p0, [&](uint32_t pos, uint32_t len, uint32_t dist) {
    if (len >= 4u && pos + 12u <= n) f(pos, pos + len + 5u > n ? n - 5u - pos : len, dist);   // ml >= 7 when cut
  });
}

// The LZ4 block of one split from its parse tokens (sp / tok: the split's first
// segment), one wavefront: the 64 lanes take the token ranges the parse gave them
// (an equal 1/64 of each segment).  A sequence belongs to the lane holding its match;
// its literal run may begin in earlier lanes or segments, so each lane's run-in
// length comes from a segmented scan (reset at every lane with a match), and lane
// output offsets from a prefix sum.  write == 0: returns the block size; write == 1:
// writes the block to out (and returns the size).
HZ_HD uint32_t lz4_block_wave(const hd::SegParse* sp, const uint16_t* tok, const hd::EncJob& job, uint8_t* out,
                              int write, CopyList* cl = nullptr) {
  const uint32_t n = job.len;
  const uint32_t nseg = hd::nsegments(n);
  uint32_t carry = 0;      // literals pending from earlier segments
  uint32_t base = 0;       // output bytes of earlier segments
  LANE_VAR(uint32_t, sv);  // scan value: literals carried past this lane
  LANE_VAR(uint32_t, sr);  // 1: the lane has a match (the scan resets)
  LANE_VAR(uint32_t, osz); // output bytes of the lane's sequences
  LANE_VAR(uint32_t, hh);  // literals before the lane's first match
  LANE_VAR(uint32_t, fml); // first match length
  LANE_VAR(uint32_t, rest);
  LANE_VAR(uint32_t, cin); // literal run entering the lane
  for (uint32_t sg = 0; sg < nseg; sg++) {
    const uint32_t s0 = sg * (uint32_t)hd::SEG;
    const uint32_t seglen = n - s0 < (uint32_t)hd::SEG ? n - s0 : (uint32_t)hd::SEG;
    hz_gcu8* const gtok = HZ_GLOBAL(hz_gcu8*, tok + (size_t)sg * hd::SEG_TOK);
    LANE_LOOP {
      const uint32_t a0 = hd::lane_start((uint32_t)lane, seglen), a1 = hd::lane_start((uint32_t)lane + 1u, seglen);
      uint32_t has = 0, h = 0, ml0 = 0, rs = 0, lit0 = s0 + a0;
      lane_matches(gtok, sp[sg].nslot[lane], lane, s0 + a0, n, [&](uint32_t pos, uint32_t ml, uint32_t) {
        if (!has) { has = 1; h = pos - lit0; ml0 = ml; } else { rs += seq_size(pos - lit0, ml); }
        lit0 = pos + ml;
      });
      LV(sr) = has;
      LV(sv) = has ? s0 + a1 - lit0 : a1 - a0;
      LV(hh) = h; LV(fml) = ml0; LV(rest) = rs;
    }
    // segmented exclusive scan of the carried literals, seeded with `carry`
    uint32_t seg_carry, seg_total;
#if HZ_GPU
    {
      const int lane = (int)threadIdx.x;
      uint32_t v = sv, r = sr;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t pv = __shfl_up(v, o, 64), pr = __shfl_up(r, o, 64);
        if (lane >= o && !r) { v += pv; r = pr; }
      }
      uint32_t ev = __shfl_up(v, 1, 64), er = __shfl_up(r, 1, 64);
      if (lane == 0) { ev = 0; er = 0; }
      cin = er ? ev : carry + ev;
      const uint32_t lv = __shfl(v, 63, 64), lr = __shfl(r, 63, 64);
      seg_carry = lr ? lv : carry + lv;
      osz = sr ? seq_size(cin + hh, fml) + rest : 0u;
      const uint32_t ox = hz::wave_excl_scan(osz, lane);
      seg_total = __shfl(ox + osz, 63, 64);
      osz = ox;               // from here on: the lane's output offset in the segment
    }
#else
    {
      uint32_t v = carry;
      for (int lane = 0; lane < 64; lane++) { cin[lane] = v; v = sr[lane] ? sv[lane] : v + sv[lane]; }
      seg_carry = v;
      uint32_t acc = 0;
      for (int lane = 0; lane < 64; lane++) {
        const uint32_t z = sr[lane] ? seq_size(cin[lane] + hh[lane], fml[lane]) + rest[lane] : 0u;
        osz[lane] = acc;
        acc += z;
      }
      seg_total = acc;
    }
#endif
    if (write) {
      LANE_LOOP {
        if (LV(sr)) {
          const uint32_t a0 = hd::lane_start((uint32_t)lane, seglen);
          Out o = {HZ_GLOBAL(hz_gu8*, out + base + LV(osz)), 0u, 1};
          InRd in;
          in_init(in, job);
          uint32_t lit0 = s0 + a0 - LV(cin);
          lane_matches(gtok, sp[sg].nslot[lane], lane, s0 + a0, n, [&](uint32_t pos, uint32_t ml, uint32_t dist) {
            sequence(o, in, lit0, pos, dist, ml, cl);
            lit0 = pos + ml;
          });
        }
      }
      WAVE_SYNC();
      if (cl) flush_runs(cl, job);
    }
    carry = seg_carry;
    base += seg_total;
  }
  // the final literals-only sequence
  if (write) {
    LANE_LOOP {
      if (lane == 0) {
        Out o = {HZ_GLOBAL(hz_gu8*, out + base), 0u, 1};
        InRd in;
        in_init(in, job);
        sequence(o, in, n - carry, n, 0u, 0u, cl);
      }
    }
    if (cl) flush_runs(cl, job);
  }
  return base + seq_size(carry, 0u);
}

// ---- BloscLZ (Blosc codec 0, c-blosc 1.21 blosclz_decompress's format) ----------
// items: c < 32 -> c + 1 literals; else a match of (c >> 5) + 2 bytes ((c >> 5) == 7:
// plus extension bytes), distance ((c & 31) << 8) + next byte + 1, or for distances
// from 8192 on (the parse reaches ~16 KiB back) c & 31 == 31, byte 255 and a 16-bit
// big-endian distance - 8192.
HZ_HD uint32_t blz_lit_size(uint32_t r) { return r + (r + 31u) / 32u; }
HZ_HD uint32_t blz_match_size(uint32_t len, uint32_t dist) {
  return 2u + (len >= 9u ? (len - 9u) / 255u + 1u : 0u) + (dist > 8191u ? 2u : 0u);
}
HZ_HD void blz_literals(Out& o, InRd& in, uint32_t l0, uint32_t l1) {
  for (uint32_t p = l0; p < l1; p += 32u) {
    const uint32_t k = l1 - p < 32u ? l1 - p : 32u;
    put(o, k - 1u);
    for (uint32_t i = 0; i < k; i++) put(o, in_byte(in, p + i));
  }
}
HZ_HD void blz_match(Out& o, uint32_t len, uint32_t dist) {
  const uint32_t cl = len - 2u < 7u ? len - 2u : 7u;
  const int far = dist > 8191u;                     // (31, 255) marks the 16-bit form
  put(o, (cl << 5) | (far ? 31u : (dist - 1u) >> 8));
  if (cl == 7u) put_len(o, len - 9u);
  if (far) {
    put(o, 255u);
    put(o, (dist - 8192u) >> 8);
    put(o, (dist - 8192u) & 255u);
  } else {
    put(o, (dist - 1u) & 255u);
  }
}

// The BloscLZ block of one split, one wavefront: a literal run is cut at lane
// boundaries (consecutive literal items are valid), so every lane's bytes follow
// from its own tokens and a prefix sum places them.
HZ_HD uint32_t blosclz_block_wave(const hd::SegParse* sp, const uint16_t* tok, const hd::EncJob& job, uint8_t* out,
                                  int write) {
  const uint32_t n = job.len;
  const uint32_t nseg = hd::nsegments(n);
  uint32_t base = 0;
  LANE_VAR(uint32_t, osz);
  for (uint32_t sg = 0; sg < nseg; sg++) {
    const uint32_t s0 = sg * (uint32_t)hd::SEG;
    const uint32_t seglen = n - s0 < (uint32_t)hd::SEG ? n - s0 : (uint32_t)hd::SEG;
    hz_gcu8* const gtok = HZ_GLOBAL(hz_gcu8*, tok + (size_t)sg * hd::SEG_TOK);
    LANE_LOOP {
      const uint32_t a0 = hd::lane_start((uint32_t)lane, seglen), a1 = hd::lane_start((uint32_t)lane + 1u, seglen);
      uint32_t lit0 = s0 + a0, sz = 0;
      lane_tokens(gtok, sp[sg].nslot[lane], lane, s0 + a0, [&](uint32_t pos, uint32_t len, uint32_t dist) {
        sz += blz_lit_size(pos - lit0) + blz_match_size(len, dist);
        lit0 = pos + len;
      });
      LV(osz) = sz + blz_lit_size(s0 + a1 - lit0);
    }
    uint32_t seg_total;
#if HZ_GPU
    {
      const uint32_t ox = hz::wave_excl_scan(osz, (int)threadIdx.x);
      seg_total = __shfl(ox + osz, 63, 64);
      osz = ox;
    }
#else
    {
      uint32_t acc = 0;
      for (int lane = 0; lane < 64; lane++) { const uint32_t z = osz[lane]; osz[lane] = acc; acc += z; }
      seg_total = acc;
    }
#endif
    if (write) {
      LANE_LOOP {
        const uint32_t a0 = hd::lane_start((uint32_t)lane, seglen), a1 = hd::lane_start((uint32_t)lane + 1u, seglen);
        Out o = {HZ_GLOBAL(hz_gu8*, out + base + LV(osz)), 0u, 1};
        InRd in;
        in_init(in, job);
        uint32_t lit0 = s0 + a0;
        lane_tokens(gtok, sp[sg].nslot[lane], lane, s0 + a0, [&](uint32_t pos, uint32_t len, uint32_t dist) {
          blz_literals(o, in, lit0, pos);
          blz_match(o, len, dist);
          lit0 = pos + len;
        });
        blz_literals(o, in, lit0, s0 + a1);
      }
      WAVE_SYNC();
    }
    base += seg_total;
  }
  return base;
}

}  // namespace lze
