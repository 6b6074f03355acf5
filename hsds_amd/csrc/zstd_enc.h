// zstd_enc.h -- zstd (RFC 8878) block writer for Blosc-zstd objects, one lane per 8 KiB segment.
//
// Replaces, for the HSDS write path, the zstd encoder that the reference reaches through
// storUtil._compress (hsds/util/storUtil.py:238-281): numcodecs Blosc(cname="zstd") ->
// c-blosc 1.21 zstd_wrap_compress -> ZSTD_compressCCtx once per Blosc block.  The frame need
// not equal libzstd's bytes (any valid stream is accepted); it must
// decode to the block through libzstd / c-blosc and the reference's _uncompress.
//
// Format written (every choice is a legal RFC 8878 encoding):
//   frame    magic, Single_Segment header with the content size, no checksum, one block
//            per 8 KiB parse segment (the deflate encoder's P phase gives the matches);
//   block    Compressed_Block: Raw_Literals_Block (the literal bytes in order) + a
//            sequences section in Predefined_Mode for literal lengths, offsets and match
//            lengths (offsets as Offset_Value = offset + 3: no repeat codes); a block whose
//            content would not be smaller than the segment is a Raw_Block.
// A lane walks its segment's tokens forward (literal bytes) and backward (sequences are
// FSE-encoded from the last to the first, as ZSTD_encodeSequences does), so no sequence
// store is needed.
//
// SINGLE SOURCE for the HIP kernels (engine.hip) and the CPU emulation (tests/emu/deflate_emu.cpp).
#pragma once
#include "deflate_wave.h"
#include "zstd_lane.h"

namespace hze {

constexpr uint32_t ZCAP = (uint32_t)hd::SEG + 64u;   // scratch bytes per segment block
constexpr uint32_t MAXSYM = 53;

// FSE compression table of one predefined distribution (FSE_buildCTable)
struct CTab {
  uint16_t state[64];
  int32_t dnb[MAXSYM];        // deltaNbBits
  int32_t dfs[MAXSYM];        // deltaFindState
  uint32_t log;
};
struct Tabs {
  CTab ll, of, ml;
};

HZ_HD uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// which: 0 LL (36 codes, log 6), 1 OF (29, log 5), 2 ML (53, log 6)
HZ_HD void build(CTab& t, uint32_t which) {
  const uint32_t n = which == 0 ? 36u : which == 1 ? 29u : 53u;
  const uint32_t log = which == 1 ? 5u : 6u;
  const uint32_t size = 1u << log, mask = size - 1u, step = (size >> 1) + (size >> 3) + 3u;
  uint8_t sym[64];
  uint32_t cumul[MAXSYM + 1];
  uint32_t high = size - 1u;
  cumul[0] = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = zs::def_norm(which, s);
    if (c == -1) { cumul[s + 1] = cumul[s] + 1u; sym[high--] = (uint8_t)s; }
    else cumul[s + 1] = cumul[s] + (uint32_t)c;
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = zs::def_norm(which, s);
    for (int32_t k = 0; k < c; k++) {
      sym[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  }
  for (uint32_t u = 0; u < size; u++) t.state[cumul[sym[u]]++] = (uint16_t)(size + u);
  uint32_t total = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = zs::def_norm(which, s);
    if (c == 0) {
      t.dnb[s] = (int32_t)(((log + 1u) << 16) - size);
      t.dfs[s] = 0;
    } else if (c == -1 || c == 1) {
      t.dnb[s] = (int32_t)((log << 16) - size);
      t.dfs[s] = (int32_t)total - 1;
      total++;
    } else {
      const uint32_t maxb = log - hb32((uint32_t)c - 1u);
      const uint32_t minsp = (uint32_t)c << maxb;
      t.dnb[s] = (int32_t)((maxb << 16) - minsp);
      t.dfs[s] = (int32_t)total - c;
      total += (uint32_t)c;
    }
  }
  t.log = log;
}

HZ_HD void build_all(Tabs& T) {
  build(T.ll, 0);
  build(T.of, 1);
  build(T.ml, 2);
}

// literal length -> code (RFC 8878 3.1.1.3.2.1.1)
HZ_HD uint32_t ll_code(uint32_t v) {
  if (v < 16) return v;
  if (v >= 64) return hb32(v) + 19u;               // 64..127: 25 ... 65536: 35
  for (uint32_t c = 24; c > 16; c--) if (v >= zs::ll_base(c)) return c;
  return 16;
}
// match length (>= 3) -> code
HZ_HD uint32_t ml_code(uint32_t v) {
  if (v < 35) return v - 3u;
  if (v >= 131) return hb32(v - 3u) + 36u;         // 131..258: 43, 259..: 44 ...
  for (uint32_t c = 42; c > 32; c--) if (v >= zs::ml_base(c)) return c;
  return 32;
}

// forward bit writer, LSB first (BIT_CStream); stops writing past cap
struct BitW {
  uint64_t acc;
  uint32_t n;
  uint32_t pos, cap;
  uint8_t* out;
  int over;
};
HZ_HD void bw_add(BitW& w, uint32_t v, uint32_t nb) {
  w.acc |= (uint64_t)(v & (nb >= 32u ? 0xffffffffu : ((1u << nb) - 1u))) << w.n;
  w.n += nb;
  while (w.n >= 8u) {
    if (w.pos < w.cap) w.out[w.pos] = (uint8_t)w.acc;
    else w.over = 1;
    w.pos++;
    w.acc >>= 8;
    w.n -= 8u;
  }
}
HZ_HD void put8(uint8_t* out, uint32_t& p, uint32_t cap, uint32_t v, int& over) {
  if (p < cap) out[p] = (uint8_t)v;
  else over = 1;
  p++;
}

// FSE state of one table (FSE_CState)
HZ_HD uint32_t fse_init(const CTab& t, uint32_t s) {
  const uint32_t nbo = (uint32_t)((t.dnb[s] + (1 << 15)) >> 16);
  const uint32_t value = (nbo << 16) - (uint32_t)t.dnb[s];
  return t.state[(value >> nbo) + t.dfs[s]];
}
HZ_HD void fse_enc(BitW& w, const CTab& t, uint32_t& st, uint32_t s) {
  const uint32_t nbo = (uint32_t)((st + (uint32_t)t.dnb[s]) >> 16);
  bw_add(w, st, nbo);
  st = t.state[(st >> nbo) + t.dfs[s]];
}

// one sequence's codes and extra-bit values
struct Seq {
  uint32_t llc, llv, mlc, mlv, ofc, ofv;
};
HZ_HD Seq make_seq(uint32_t ll, uint32_t ml, uint32_t off) {
  Seq q;
  q.llc = ll_code(ll);
  q.llv = ll - zs::ll_base(q.llc);
  q.mlc = ml_code(ml);
  q.mlv = ml - zs::ml_base(q.mlc);
  const uint32_t ov = off + 3u;                    // Offset_Value: no repeat codes
  q.ofc = hb32(ov);
  q.ofv = ov - (1u << q.ofc);
  return q;
}

// the 3-byte block header
HZ_HD void block_header(uint8_t* out, uint32_t last, uint32_t type, uint32_t size) {
  const uint32_t h = last | (type << 1) | (size << 3);
  out[0] = (uint8_t)h;
  out[1] = (uint8_t)(h >> 8);
  out[2] = (uint8_t)(h >> 16);
}

// Writes segment `seg` of a stream as one zstd block (header included) at out (cap bytes
// of scratch, >= ZCAP).  tok / sp: the segment's parse tokens and counts; job / s0: the
// stream input (a raw block copies the segment from it).  Returns the block size.
HZ_HD uint32_t encode_segment(const Tabs& T, const uint16_t* tok, const hd::SegParse* sp, const hd::EncJob& job,
                              uint32_t s0, uint32_t seglen, uint32_t last, uint8_t* out, uint32_t cap) {
  hz_gcu8* const gt = HZ_GLOBAL(hz_gcu8*, tok);
  auto slot = [&](uint32_t k, uint32_t l) -> uint32_t {
    const uint32_t i = hd::tslot(k, (int)l);
    return (uint32_t)gt[2u * i] | ((uint32_t)gt[2u * i + 1u] << 8);
  };
  uint32_t nlit = 0, nseq = 0;
  for (uint32_t s = 0; s < 256u; s++) nlit += sp->freq[s];
  for (uint32_t s = 257; s < 286u; s++) nseq += sp->freq[s];
  int over = 0;
  uint32_t p = 3;
  // literals section header (Raw_Literals_Block)
  if (nlit < 32u) {
    put8(out, p, cap, nlit << 3, over);
  } else if (nlit < 4096u) {
    put8(out, p, cap, (1u << 2) | ((nlit & 15u) << 4), over);
    put8(out, p, cap, nlit >> 4, over);
  } else {
    put8(out, p, cap, (3u << 2) | ((nlit & 15u) << 4), over);
    put8(out, p, cap, (nlit >> 4) & 0xffu, over);
    put8(out, p, cap, nlit >> 12, over);
  }
  // literal bytes, forward over the lanes' token ranges
  for (uint32_t l = 0; l < (uint32_t)hd::WAVE && !over; l++) {
    const uint32_t ns = sp->nslot[l];
    for (uint32_t k = 0; k < ns;) {
      const uint32_t v = slot(k, l);
      if (v & 0x8000u) { k += 2; continue; }
      put8(out, p, cap, v, over);
      k++;
    }
  }
  // sequences section header
  if (nseq < 128u) {
    put8(out, p, cap, nseq, over);
  } else if (nseq < 0x7f00u) {
    put8(out, p, cap, (nseq >> 8) + 128u, over);
    put8(out, p, cap, nseq & 0xffu, over);
  } else {
    put8(out, p, cap, 255u, over);
    put8(out, p, cap, (nseq - 0x7f00u) & 0xffu, over);
    put8(out, p, cap, (nseq - 0x7f00u) >> 8, over);
  }
  if (nseq) {
    put8(out, p, cap, 0u, over);                     // Predefined_Mode x 3
    BitW w = {0, 0, p, cap, out, over};
    uint32_t sll = 0, sof = 0, sml = 0;
    // backward walk: a match's literal run is known once the walk reaches the match
    // before it (or the segment start), so each sequence is encoded one match late
    uint32_t have = 0, pml = 0, poff = 0, run = 0, first = 1;
    auto emit = [&](uint32_t ll, uint32_t ml, uint32_t off) {
      const Seq q = make_seq(ll, ml, off);
      if (first) {
        sml = fse_init(T.ml, q.mlc);
        sof = fse_init(T.of, q.ofc);
        sll = fse_init(T.ll, q.llc);
        first = 0;
      } else {
        fse_enc(w, T.of, sof, q.ofc);
        fse_enc(w, T.ml, sml, q.mlc);
        fse_enc(w, T.ll, sll, q.llc);
      }
      bw_add(w, q.llv, zs::ll_bits(q.llc));
      bw_add(w, q.mlv, zs::ml_bits(q.mlc));
      bw_add(w, q.ofv, q.ofc);
    };
    for (int32_t l = hd::WAVE - 1; l >= 0 && !w.over; l--) {
      int32_t k = (int32_t)sp->nslot[l] - 1;
      while (k >= 0) {
        const uint32_t v = slot((uint32_t)k, (uint32_t)l);
        if (k >= 1) {
          const uint32_t u = slot((uint32_t)k - 1u, (uint32_t)l);
          if (u & 0x8000u) {                         // (k-1, k): a match
            if (have) emit(run, pml, poff);
            have = 1;
            pml = (u & 0x7fffu) + 3u;
            poff = v + 1u;
            run = 0;
            k -= 2;
            continue;
          }
        }
        run++;                                       // a literal (trailing ones belong to no sequence)
        k--;
      }
    }
    if (have) emit(run, pml, poff);
    bw_add(w, sml, T.ml.log);
    bw_add(w, sof, T.of.log);
    bw_add(w, sll, T.ll.log);
    bw_add(w, 1u, 1u);                               // end mark
    if (w.n) bw_add(w, 0u, 8u - w.n);
    p = w.pos;
    over = w.over;
  }
  const uint32_t csize = p - 3u;
  if (over || csize >= seglen) {
    // Raw_Block: the segment's bytes
    block_header(out, last, 0u, seglen);
    for (uint32_t i = 0; i < seglen; i++) {
      const uint32_t q = s0 + i;
      out[3u + i] = (uint8_t)(hd::load_stream_word(job, q & ~3u, job.len) >> (8u * (q & 3u)));
    }
    return 3u + seglen;
  }
  block_header(out, last, 2u, csize);
  return p;
}

// frame header (Single_Segment, content size, no checksum / dictionary): bytes for n
HZ_HD uint32_t frame_header_size(uint32_t n) { return 4u + 1u + (n < 256u ? 1u : n < 65536u + 256u ? 2u : 4u); }
HZ_HD uint32_t frame_header(uint8_t* out, uint32_t n) {
  out[0] = 0x28; out[1] = 0xb5; out[2] = 0x2f; out[3] = 0xfd;
  if (n < 256u) {
    out[4] = 0x20; out[5] = (uint8_t)n;
    return 6;
  }
  if (n < 65536u + 256u) {
    const uint32_t v = n - 256u;
    out[4] = 0x60; out[5] = (uint8_t)v; out[6] = (uint8_t)(v >> 8);
    return 7;
  }
  out[4] = 0xa0;
  for (int i = 0; i < 4; i++) out[5 + i] = (uint8_t)(n >> (8 * i));
  return 9;
}

}  // namespace hze
