// lz_wave.h -- one-wavefront-per-stream decoder for the byte-aligned LZ77 codecs a
// Blosc1 frame can carry besides zlib:
//   * codec 1, "lz4" / "lz4hc": LZ4 block format (lz4 1.9.x LZ4_decompress_safe, which
//     c-blosc 1.21 calls from lz4_wrap_decompress for every split);
//   * codec 0, "blosclz": c-blosc 1.21's BloscLZ (blosclz_decompress).
// The reference reaches both through storUtil._uncompress -> numcodecs Blosc.decode
// (hsds/util/storUtil.py:195-208) and writes them through storUtil._compress with
// cname = the dataset's compressor (storUtil.py:255-262, dsetUtil.py:38-44).
//
// Algorithm (DESIGN.md "LZ4 / BloscLZ"):
//   A window is a run of up to NSEQ sequences (literal run + match).  Their headers are
//   parsed serially from a 4 KiB LDS stage of the input (uniform code: every lane
//   walks the same bytes), which fixes every sequence's absolute output offset.  Then
//   every output byte of the window is a pure function of the sequence table: a literal
//   byte is read from the input; a match byte at offset k into a match of distance d
//   starting at m is the byte at m - d + (k mod d) (the periodic extension of an
//   overlapping copy), which lies in an earlier sequence or before the window (already
//   stored), so each lane resolves its bytes independently in a few hops and stores
//   them as aligned dwords.  No LDS output buffer, no rounds.
//
// Single source, like inflate_wave.h: tests/emu/lz_emu.cpp runs the same code on CPU.
#pragma once
#include "inflate_wave.h"

namespace lz {

constexpr int NSEQ = 256;            // sequences per window
constexpr int STAGE_WORDS = 1024;    // 4 KiB input stage
constexpr uint32_t FMT_BLOSCLZ = 0, FMT_LZ4 = 1;   // Blosc1 codec numbers (flags >> 5)

struct Shared {
  uint32_t in32[STAGE_WORDS + 4];
  uint32_t s_out[NSEQ + 1];   // absolute output offset of each sequence; [nseq] = window end
  uint32_t s_lit[NSEQ];       // literal bytes
  uint32_t s_src[NSEQ];       // stream offset of the literals
  uint32_t s_off[NSEQ];       // match distance (0: literals only)
};

HZ_HD uint32_t sbyte(const Shared& ls, uint32_t idx) { return (ls.in32[idx >> 2] >> ((idx & 3u) * 8u)) & 0xffu; }

#if HZ_GPU
#define LZ_LANE0 if (threadIdx.x == 0)
#else
#define LZ_LANE0
#endif

// Decode one Blosc split.  Returns hz::ST_OK or an error status (uniform).
#if HZ_GPU
__device__
#else
static
#endif
inline int lz_stream(Shared& ls, const hz::StreamJob job, uint32_t fmt) {
  const uint32_t a = (uint32_t)(((uintptr_t)job.src) & 3u);
  hz_gcu8* base = HZ_GLOBAL(hz_gcu8*, job.src - a);
  hz_gcu8* src = HZ_GLOBAL(hz_gcu8*, job.src);
  hz_gu8* const dst = HZ_GLOBAL(hz_gu8*, job.dst);
  const uint32_t iend = job.src_len, oend = job.dst_len;
  const uint32_t dmis = (uint32_t)(((uintptr_t)job.dst) & 3u);
  uint32_t ip = 0, op = 0;
  int done = 0;
  if (iend == 0) return hz::ST_TRUNC;
  while (!done) {
    // ---- stage 4 KiB of input at ip (dword-aligned) ----
    const uint32_t w0 = (ip + a) >> 2;
    WAVE_SYNC();
    LANE_LOOP {
      for (uint32_t k = (uint32_t)lane; k < (uint32_t)STAGE_WORDS + 4u; k += 64)
        ls.in32[k] = k < (uint32_t)STAGE_WORDS ? hz::load_word(base, w0 + k, a, a + iend) : 0u;
    }
    WAVE_SYNC();
    // stream offsets [slo, shi) are in the stage; byte x is at stage index x - slo + sfix
    const uint32_t sfix = (ip + a) & 3u, slo = ip;
    const uint32_t shi = ip + (uint32_t)STAGE_WORDS * 4u - sfix;
    const uint32_t win_base = op;
    uint32_t nseq = 0;
    int err = hz::ST_OK;
    // ---- serial parse of sequence headers (uniform) ----
    // A window takes sequences while their first byte is staged; header bytes past
    // the stage (the tail of a window's last sequence, after a long literal run) are
    // read from the input directly.
    while (!done && nseq < (uint32_t)NSEQ && ip < shi) {
      uint32_t x = ip, lit = 0, lsrc = 0, off = 0, ml = 0;
#define LZ_NEED(pos) \
  if ((pos) >= iend) { err = hz::ST_TRUNC; break; }
#define LZ_B(pos) ((pos) < shi ? sbyte(ls, (pos) - slo + sfix) : (uint32_t)src[pos])
      int last = 0;
      do {
        if (fmt == FMT_LZ4) {
          LZ_NEED(x);
          const uint32_t t = LZ_B(x); x++;
          lit = t >> 4;
          if (lit == 15) {
            uint32_t b;
            do { LZ_NEED(x); b = LZ_B(x); x++; lit += b; } while (b == 255 && lit < 0x7fffffffu);
            if (err != hz::ST_OK) break;
          }
          lsrc = x;
          if (lit > iend - x) { err = hz::ST_TRUNC; break; }
          x += lit;
          const uint32_t oe = op + lit;
          if (lit > oend - op) { err = hz::ST_SIZE; break; }
          // LZ4_decompress_safe: a literal run that reaches oend - MFLIMIT (12) or
          // iend - 8 must be the last sequence and end exactly at iend
          if (oe + 12u > oend || x + 8u > iend) {
            if (x != iend) { err = hz::ST_DATA; break; }
            last = 1;
            break;
          }
          LZ_NEED(x + 1u);
          off = LZ_B(x) | (LZ_B(x + 1u) << 8); x += 2;
          ml = t & 15u;
          if (ml == 15) {
            uint32_t b;
            do { LZ_NEED(x); b = LZ_B(x); x++; ml += b; } while (b == 255 && ml < 0x7fffffffu);
            if (err != hz::ST_OK) break;
          }
          ml += 4;
          if (off == 0 || off > oe) { err = hz::ST_DATA; break; }
          if (ml > oend - oe || oe + ml + 5u > oend) { err = hz::ST_DATA; break; }   // LASTLITERALS
        } else {
          LZ_NEED(x);
          uint32_t c = LZ_B(x); x++;
          if (ip == 0) c &= 31u;
          if (c >= 32) {
            ml = (c >> 5) - 1u;
            const uint32_t ofs = (c & 31u) << 8;
            uint32_t code;
            if (ml == 6) {
              do { LZ_NEED(x); code = LZ_B(x); x++; ml += code; } while (code == 255 && ml < 0x7fffffffu);
              if (err != hz::ST_OK) break;
            }
            LZ_NEED(x);
            code = LZ_B(x); x++;
            ml += 3;
            off = ofs + code + 1u;
            if (code == 255 && ofs == (31u << 8)) {
              LZ_NEED(x + 1u);
              off = ((LZ_B(x) << 8) | LZ_B(x + 1u)) + 8192u;
              x += 2;
            }
            if (ml > oend - op) { err = hz::ST_SIZE; break; }
            if (off > op) { err = hz::ST_DATA; break; }
          } else {
            lit = c + 1u;
            lsrc = x;
            if (lit > oend - op) { err = hz::ST_SIZE; break; }
            if (lit > iend - x) { err = hz::ST_TRUNC; break; }
            x += lit;
          }
          if (x >= iend) last = 1;
        }
      } while (0);
#undef LZ_NEED
#undef LZ_B
      if (err != hz::ST_OK) return err;
      LZ_LANE0 {
        ls.s_out[nseq] = op;
        ls.s_lit[nseq] = lit;
        ls.s_src[nseq] = lsrc;
        ls.s_off[nseq] = off;
      }
      nseq++;
      op += lit + ml;
      ip = x;
      if (last) done = 1;
    }
    LZ_LANE0 { ls.s_out[nseq] = op; }
    WAVE_SYNC();
    // ---- resolve and store the window's bytes [win_base, op) ----
    const uint32_t wb = win_base, we = op;
    const uint32_t g0 = (wb + dmis) >> 2, g1 = (we + dmis + 3u) >> 2;
    LANE_LOOP {
      uint32_t s = 0;                              // cursor: sequence holding the current byte
      uint32_t s_beg = ls.s_out[0], s_end = ls.s_out[1];
      for (uint32_t g = g0 + (uint32_t)lane; g < g1; g += 64u) {
        uint32_t word = 0, have = 0;
        for (uint32_t k = 0; k < 4u; k++) {
          const uint32_t p = g * 4u + k - dmis;    // wraps below 0 for the first group
          if (g * 4u + k < wb + dmis || p >= we) continue;
          while (p >= s_end) { s++; s_beg = s_end; s_end = ls.s_out[s + 1]; }
          uint32_t q = p, t = s, tb = s_beg, v = 0;
          for (;;) {
            const uint32_t rel = q - tb, nl = ls.s_lit[t];
            if (rel < nl) { v = src[ls.s_src[t] + rel]; break; }
            const uint32_t m = tb + nl, d = ls.s_off[t], kk = q - m;
            const uint32_t q2 = m - d + (kk < d ? kk : kk % d);
            if (q2 < wb) { v = dst[q2]; break; }
            // q2 lies in an earlier (or this) sequence of the window: largest t2 <= t
            // with s_out[t2] <= q2
            uint32_t lo2 = 0, hi2 = t;
            while (lo2 < hi2) {
              const uint32_t mid = (lo2 + hi2 + 1u) >> 1;
              if (ls.s_out[mid] <= q2) lo2 = mid; else hi2 = mid - 1u;
            }
            q = q2; t = lo2; tb = ls.s_out[lo2];
          }
          word |= v << (8u * k);
          have |= 1u << k;
        }
        if (have == 15u) {
          *(hz_gu32*)(dst + (g * 4u - dmis)) = word;
        } else {
          for (uint32_t k = 0; k < 4u; k++)
            if (have & (1u << k)) dst[g * 4u + k - dmis] = (uint8_t)(word >> (8u * k));
        }
      }
    }
    WAVE_SYNC_GLOBAL();
  }
  if (op != oend) return hz::ST_SIZE;
  if (job.out_len) { LZ_LANE0 { *job.out_len = op; } }
  return hz::ST_OK;
}

}  // namespace lz
