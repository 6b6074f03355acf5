// lz4_enc.h -- LZ4 block writer for the Blosc-lz4 write path.
//
// storUtil._compress (hsds/util/storUtil.py:238-281) encodes with
// Blosc(cname=<the dataset's compressor>); for "lz4" / "lz4hc" c-blosc 1.21 calls
// lz4_wrap_compress once per split.  The compressed bytes need not equal lz4's (any
// valid block is accepted); the frame must decode to the input
// through c-blosc and the reference's _uncompress.
//
// The match finding is the deflate encoder's parse phase (deflate_wave.h P: exact hash
// chains over an 8 KiB window, lane-parallel greedy parse, tokens in HBM).  This file
// turns one split's token list into an LZ4 block: one lane per split walks the tokens
// in order (a serial, byte-granular walk over ~10^4 sequences, which the batch runs on
// thousands of splits at once), length-3 matches become literals, and the block end
// rules LZ4_decompress_safe enforces are kept (the last match starts at least MFLIMIT
// = 12 bytes before the end and ends at least LASTLITERALS = 5 bytes before it).
// The walk runs twice: once for the size (frame layout), once to write.
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
  in.r.buf = 0;
  in.blk = HZ_GLOBAL(hz_gcu8*, job.src);
  in.ts = job.ts; in.neb = job.neb; in.off = job.off;
}
HZ_HD uint32_t in_byte(InRd& in, uint32_t pos) {
  return in.ts > 1u ? (uint32_t)in.blk[hd::shuffled_src_index(in.off + pos, in.ts, in.neb)] : lz::rd_byte(in.r, pos);
}

// one sequence: literals [l0, l1), then a match (ml >= 4) of distance dist; ml == 0:
// the final literals-only sequence
HZ_HD void sequence(Out& o, InRd& in, uint32_t l0, uint32_t l1, uint32_t dist, uint32_t ml) {
  const uint32_t ll = l1 - l0;
  const uint32_t mc = ml ? (ml - 4u < 15u ? ml - 4u : 15u) : 0u;
  put(o, ((ll < 15u ? ll : 15u) << 4) | mc);
  if (ll >= 15u) put_len(o, ll - 15u);
  if (o.write) {
    for (uint32_t p = l0; p < l1; p++) put(o, in_byte(in, p));
  } else {
    o.n += ll;
  }
  if (ml) {
    put(o, dist & 255u);
    put(o, dist >> 8);
    if (ml - 4u >= 15u) put_len(o, ml - 4u - 15u);
  }
}

// The LZ4 block of one split from its parse tokens (sp / tok: the split's first
// segment).  Returns the block size; writes it to out when `write`.
HZ_HD uint32_t lz4_block(const hd::SegParse* sp, const uint16_t* tok, const hd::EncJob& job, uint8_t* out,
                         int write) {
  const uint32_t n = job.len;
  const uint32_t nseg = hd::nsegments(n);
  Out o = {HZ_GLOBAL(hz_gu8*, out), 0u, write};
  InRd in;
  in_init(in, job);
  uint32_t pos = 0, lit0 = 0;
  // the last sequence is held back: a match that continues it (no literals in
  // between, same distance) extends it, so runs longer than deflate's 258-byte
  // matches become one LZ4 match
  uint32_t q0 = 0, q1 = 0, qd = 0, qml = 0;
  int have_q = 0;
  for (uint32_t sg = 0; sg < nseg; sg++) {
    hz_gcu8* const gtok = HZ_GLOBAL(hz_gcu8*, tok + (size_t)sg * hd::SEG_TOK);
    for (int lane = 0; lane < hd::WAVE; lane++) {
      const uint32_t ns = sp[sg].nslot[lane];
      uint32_t pend = 0;
      bool have = false;
      for (uint32_t s = 0; s < ns; s++) {
        uint32_t t;
        if (!have) {
          const uint32_t pr = *(hz_gcu32*)(gtok + (size_t)hd::tslot(s, lane) * 2u);
          t = pr & 0xffffu; pend = pr >> 16; have = true;
        } else {
          t = pend; have = false;
        }
        if (!(t & 0x8000u)) { pos++; continue; }
        uint32_t dv;
        s++;
        if (!have) {
          const uint32_t pr = *(hz_gcu32*)(gtok + (size_t)hd::tslot(s, lane) * 2u);
          dv = pr & 0xffffu; pend = pr >> 16; have = true;
        } else {
          dv = pend; have = false;
        }
        const uint32_t len = (t & 0x7fffu) + 3u;
        if (len >= 4u && pos + 12u <= n) {
          const uint32_t ml = pos + len + 5u > n ? n - 5u - pos : len;   // >= 7 here
          if (have_q && lit0 == pos && q1 + qml == pos && qd == dv + 1u) {
            qml += ml;
          } else {
            if (have_q) sequence(o, in, q0, q1, qd, qml);
            q0 = lit0; q1 = pos; qd = dv + 1u; qml = ml; have_q = 1;
          }
          lit0 = pos + ml;
        }
        pos += len;
      }
    }
  }
  if (have_q) sequence(o, in, q0, q1, qd, qml);
  sequence(o, in, lit0, n, 0u, 0u);
  return o.n;
}

}  // namespace lze
