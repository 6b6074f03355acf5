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
//   block    Compressed_Block: a Compressed_Literals_Block (the segment's own Huffman code,
//            limited to 11 bits, its weights FSE-compressed; 4 streams) -- or the literal
//            bytes raw when that is not smaller -- and a sequences section whose literal
//            length, offset and match length codes are FSE-coded with the FRAME's own
//            tables (FSE_Compressed_Mode: frame_tables from the code counts of all its
//            segments, count_segment; each block repeats the descriptions, so no block
//            depends on an earlier one being compressed); a code type with fewer than two
//            distinct codes in the frame uses the predefined table.  Offsets are sent as
//            Offset_Value = offset + 3 (no repeat codes).  A block whose content would not be
//            smaller than the segment is a Raw_Block.
// lit_section: one wavefront per segment builds the literals section (token walk per parse
// lane, the deflate encoder's cooperative Huffman build, weights + 4 streams).
// encode_segment: one lane per segment walks the tokens forward (raw literals when there
// is no literals section) and backward (sequences are FSE-encoded from the last to the
// first, as ZSTD_encodeSequences does), so no sequence store is needed.
//
// SINGLE SOURCE for the HIP kernels (engine.hip) and the CPU emulation (tests/emu/deflate_emu.cpp).
#pragma once
#include "deflate_wave.h"
#include "zstd_lane.h"

namespace hze {

constexpr uint32_t ZCAP = (uint32_t)hd::SEG + 64u;   // scratch bytes per segment block
constexpr uint32_t LCAP = (uint32_t)hd::SEG + 512u;  // scratch bytes per segment literals section
constexpr uint32_t HUF_MAXBITS = 11;
constexpr uint32_t STRM = ((uint32_t)hd::SEG / 4u * HUF_MAXBITS + 7u) / 8u + 16u;   // one Huffman stream, max
constexpr uint32_t MAXSYM = 53;

// FSE compression table of one predefined distribution (FSE_buildCTable)
struct CTab {
  uint16_t state[64];
  int32_t dnb[MAXSYM];        // deltaNbBits
  int32_t dfs[MAXSYM];        // deltaFindState
  uint32_t log;
};
// the three sequence tables a block is encoded with, and how its sequences section
// describes them: Symbol_Compression_Modes byte `mode` (0: all Predefined_Mode) followed by
// `dsize` bytes of FSE_Compressed_Mode descriptions (LL, then OF, then ML)
constexpr uint32_t DESC_MAX = 192;
struct Tabs {
  CTab ll, of, ml;
  uint32_t mode, dsize;
  uint8_t desc[DESC_MAX];
};
// code counts of a frame's sequences (the input of its FSE_Compressed_Mode tables)
struct SeqCounts {
  uint32_t ll[36], of[32], ml[53];
};
// table logs of the compressed-mode tables: every block carries its descriptions, so they
// stay short (RFC 8878 maxima: 9 / 8 / 9)
constexpr uint32_t LL_LOG = 6, OF_LOG = 5, ML_LOG = 6;

HZ_HD uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// FSE_buildCTable for normalized counts norm[0..n) (-1: a low-probability symbol) at `log`
HZ_HD void build_norm(CTab& t, const int16_t* norm, uint32_t n, uint32_t log) {
  const uint32_t size = 1u << log, mask = size - 1u, step = (size >> 1) + (size >> 3) + 3u;
  uint8_t sym[64];
  uint32_t cumul[MAXSYM + 1];
  uint32_t high = size - 1u;
  cumul[0] = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = norm[s];
    if (c == -1) { cumul[s + 1] = cumul[s] + 1u; sym[high--] = (uint8_t)s; }
    else cumul[s + 1] = cumul[s] + (uint32_t)c;
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = norm[s];
    for (int32_t k = 0; k < c; k++) {
      sym[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  }
  for (uint32_t u = 0; u < size; u++) t.state[cumul[sym[u]]++] = (uint16_t)(size + u);
  uint32_t total = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int32_t c = norm[s];
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
  // codes outside the distribution (s >= n) are absent, as a zero count is
  for (uint32_t s = n; s < MAXSYM; s++) {
    t.dnb[s] = (int32_t)(((log + 1u) << 16) - size);
    t.dfs[s] = 0;
  }
  t.log = log;
}

// a code with no state in table t (normalized count 0): encoding it would corrupt the
// sequences, so a block that needs one is written as a Raw_Block instead (encode_segment)
HZ_HD bool absent(const CTab& t, uint32_t s) {
  return s >= MAXSYM || t.dnb[s] == (int32_t)(((t.log + 1u) << 16) - (1u << t.log));
}

// which: 0 LL (36 codes, log 6), 1 OF (29, log 5), 2 ML (53, log 6): the predefined tables
HZ_HD void build(CTab& t, uint32_t which) {
  const uint32_t n = which == 0 ? 36u : which == 1 ? 29u : 53u;
  int16_t norm[MAXSYM];
  for (uint32_t s = 0; s < n; s++) norm[s] = zs::def_norm(which, s);
  build_norm(t, norm, n, which == 1 ? 5u : 6u);
}

HZ_HD void build_all(Tabs& T) {
  build(T.ll, 0);
  build(T.of, 1);
  build(T.ml, 2);
  T.mode = 0;
  T.dsize = 0;
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
// the sequences' bit writer: bits gather in a 64-bit register and leave as aligned
// dwords (the lane's scratch block is 4-byte aligned); pos is the byte position of acc's
// bit 0 (aligned)
struct BitD {
  uint64_t acc;
  uint32_t n;
  uint32_t pos, cap;
  uint8_t* out;
  int over;
};
// starts at byte p, keeping the bytes already written below p in its dword
HZ_HD void bd_init(BitD& w, uint8_t* out, uint32_t p, uint32_t cap, int over) {
  w.out = out; w.cap = cap; w.over = over;
  w.pos = p & ~3u; w.n = 8u * (p & 3u); w.acc = 0;
  for (uint32_t b = 0; b < (p & 3u); b++) w.acc |= (uint64_t)out[w.pos + b] << (8u * b);
}
HZ_HD void bw_add(BitD& w, uint32_t v, uint32_t nb) {
  w.acc |= (uint64_t)(v & (nb >= 32u ? 0xffffffffu : ((1u << nb) - 1u))) << w.n;
  w.n += nb;
  if (w.n >= 32u) {
    if (w.pos + 4u <= w.cap) *(uint32_t*)(w.out + w.pos) = (uint32_t)w.acc;
    else w.over = 1;
    w.pos += 4u;
    w.acc >>= 32;
    w.n -= 32u;
  }
}
// pads to a byte, writes the last bytes; returns the end position
HZ_HD uint32_t bd_finish(BitD& w) {
  if (w.n & 7u) bw_add(w, 0u, 8u - (w.n & 7u));
  for (uint32_t b = 0; b < w.n / 8u; b++) {
    if (w.pos + b < w.cap) w.out[w.pos + b] = (uint8_t)(w.acc >> (8u * b));
    else w.over = 1;
  }
  return w.pos + w.n / 8u;
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
template <class W>
HZ_HD void fse_enc(W& w, const CTab& t, uint32_t& st, uint32_t s) {
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

// literal length / match length codes by table below 64 / 131 (ll_code and ml_code search
// the baselines: lane-divergent loops that the whole wave runs), shared by a workgroup in LDS
struct CodeTabs {
  uint8_t ll[64];
  uint8_t ml[128];           // match length 3 + i
};
HZ_HD void code_tabs_fill(CodeTabs& t, uint32_t i0, uint32_t step) {
  for (uint32_t v = i0; v < 64u; v += step) t.ll[v] = (uint8_t)ll_code(v);
  for (uint32_t v = i0; v < 128u; v += step) t.ml[v] = (uint8_t)ml_code(v + 3u);
}
HZ_HD Seq make_seq_t(const CodeTabs& t, uint32_t ll, uint32_t ml, uint32_t off) {
  Seq q;
  q.llc = ll < 64u ? t.ll[ll] : hb32(ll) + 19u;
  q.llv = ll - zs::ll_base(q.llc);
  q.mlc = ml - 3u < 128u ? t.ml[ml - 3u] : hb32(ml - 3u) + 36u;
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

// Huffman-coded literals from this level on: on the cfg5 slab they cut the objects by 2 %
// (1.236 -> 1.211 of libblosc-zstd's size) for 2.5x the encode time (290 -> 724 ms), so
// the speed levels keep raw literals (the literal bytes of float data are near 8 bits of
// entropy; the sequences section is where libzstd gains)
#if HZ_GPU
__host__ __device__
#endif
inline uint32_t huff_lit_level(int level) { return level >= 6 ? 1u : 0u; }

// ---- literals section (Compressed_Literals_Block, 4 streams) ----------------------------
struct LitShared {
  hd::HuffShared hs;
  uint8_t lit[hd::SEG];
  uint8_t strm[4][STRM];
  uint8_t tree[132];                // Huffman_Tree_Description (header byte + FSE weights)
  uint8_t w[256];                   // Huffman weights (lane 0's serial build)
  CTab wt;                          // their FSE table
  uint16_t val[256];
  uint32_t cnt[hd::WAVE], base[hd::WAVE];
  uint32_t ssize[4];
  uint32_t nlit, tsize, ok, size;
};

// FSE_writeNCount (zstd fse_compress.c) of norm[0..n) at `log` into out; returns bytes
HZ_HD uint32_t write_ncount(uint8_t* out, const int16_t* norm, uint32_t n, uint32_t log) {
  uint32_t o = 0;
  const int32_t size = 1 << log;
  int32_t remaining = size + 1, threshold = size, nbits = (int32_t)log + 1;
  uint32_t bs = log - 5u;            // table log - FSE_MIN_TABLELOG, 4 bits
  int32_t bc = 4;
  uint32_t sym = 0;
  int prev0 = 0;
  while (sym < n && remaining > 1) {
    if (prev0) {
      uint32_t start = sym;
      while (sym < n && !norm[sym]) sym++;
      if (sym >= n) break;
      while (sym >= start + 24u) {
        start += 24u;
        bs += 0xffffu << bc;
        out[o++] = (uint8_t)bs; out[o++] = (uint8_t)(bs >> 8);
        bs >>= 16;
      }
      while (sym >= start + 3u) { start += 3u; bs += 3u << bc; bc += 2; }
      bs += (sym - start) << bc;
      bc += 2;
      if (bc > 16) { out[o++] = (uint8_t)bs; out[o++] = (uint8_t)(bs >> 8); bs >>= 16; bc -= 16; }
    }
    int32_t count = norm[sym++];
    const int32_t mx = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    count++;
    if (count >= threshold) count += mx;
    bs += (uint32_t)count << bc;
    bc += nbits;
    bc -= count < mx ? 1 : 0;
    prev0 = count == 1;
    while (remaining < threshold) { nbits--; threshold >>= 1; }
    if (bc > 16) { out[o++] = (uint8_t)bs; out[o++] = (uint8_t)(bs >> 8); bs >>= 16; bc -= 16; }
  }
  out[o++] = (uint8_t)bs;
  out[o++] = (uint8_t)(bs >> 8);
  o -= 2u - (uint32_t)((bc + 7) / 8);
  return o;
}

// normalized counts norm[0..n) at `log` for counts cnt[0..n) (total > 0): every present
// symbol gets at least one state, the rest in proportion, and the sum is exactly 2^log
// (any such distribution is a valid FSE_Compressed_Mode table; n <= 2^log)
HZ_HD void normalize(const uint32_t* cnt, uint32_t n, uint32_t log, int16_t* norm) {
  uint64_t total = 0;
  for (uint32_t k = 0; k < n; k++) total += cnt[k];
  const int32_t size = 1 << log;
  int32_t sum = 0;
  uint32_t big = 0;
  for (uint32_t k = 0; k < n; k++) {
    int32_t v = 0;
    if (cnt[k]) {
      v = (int32_t)(((uint64_t)cnt[k] * (uint32_t)size + total / 2u) / total);
      v = v < 1 ? 1 : v;
      if (cnt[k] > cnt[big]) big = k;
    }
    norm[k] = (int16_t)v;
    sum += v;
  }
  while (sum > size) {                 // rounding overshoot: take from the largest
    uint32_t m = 0;
    for (uint32_t k = 0; k < n; k++) if (norm[k] > norm[m]) m = k;
    norm[m]--;
    sum--;
  }
  norm[big] = (int16_t)(norm[big] + (size - sum));
}

// one code type's table: FSE_Compressed_Mode from the counts when at least two codes occur
// (the description is appended to T.desc), else the predefined one.  which: 0 LL, 1 OF, 2 ML
HZ_HD void frame_table(Tabs& T, CTab& t, const uint32_t* cnt, uint32_t n, uint32_t which, uint32_t log) {
  uint32_t maxs = 0, distinct = 0;
  for (uint32_t k = 0; k < n; k++) if (cnt[k]) { maxs = k; distinct++; }
  if (distinct < 2u) { build(t, which); return; }
  int16_t norm[MAXSYM];
  normalize(cnt, maxs + 1u, log, norm);
  build_norm(t, norm, maxs + 1u, log);
  uint8_t d[80];
  const uint32_t k = write_ncount(d, norm, maxs + 1u, log);
  if (T.dsize + k > DESC_MAX) { build(t, which); return; }   // (no room: the predefined table)
  for (uint32_t i = 0; i < k; i++) T.desc[T.dsize++] = d[i];
  T.mode |= 2u << (which == 0 ? 6u : which == 1 ? 4u : 2u);
}

// the tables of one frame (every block of it is encoded with them)
HZ_HD void frame_tables(Tabs& T, const SeqCounts& c) {
  T.mode = 0;
  T.dsize = 0;
  frame_table(T, T.ll, c.ll, 36u, 0u, LL_LOG);
  frame_table(T, T.of, c.of, 32u, 1u, OF_LOG);
  frame_table(T, T.ml, c.ml, 53u, 2u, ML_LOG);
}

// Huffman_Tree_Description of the code lengths len[0..256) into sh.tree (header byte
// = size of the FSE-compressed weights); values in sh.val.  Returns 0 when the weights
// cannot be FSE-described (a single weight value, or >= 128 bytes).
HZ_HD uint32_t huff_tree(LitShared& sh, const uint8_t* len) {
  uint32_t maxb = 0, last = 0;
  for (uint32_t s = 0; s < 256u; s++) if (len[s]) { maxb = len[s] > maxb ? len[s] : maxb; last = s; }
  // values (HUF_buildCTable): longest codes get the smallest values, symbol order within a length
  uint32_t nper[HUF_MAXBITS + 2] = {0}, vper[HUF_MAXBITS + 2] = {0};
  for (uint32_t s = 0; s < 256u; s++) if (len[s]) nper[len[s]]++;
  {
    uint32_t mn = 0;
    for (uint32_t b = maxb; b > 0; b--) { vper[b] = mn; mn += nper[b]; mn >>= 1; }
  }
  for (uint32_t s = 0; s < 256u; s++) sh.val[s] = len[s] ? (uint16_t)vper[len[s]]++ : (uint16_t)0;
  // weights of symbols 0 .. last-1 (the last symbol's weight is implied)
  uint8_t* const w = sh.w;
  uint32_t wc[HUF_MAXBITS + 2] = {0};
  for (uint32_t s = 0; s < last; s++) { w[s] = len[s] ? (uint8_t)(maxb + 1u - len[s]) : 0u; wc[w[s]]++; }
  uint32_t nw = last, distinct = 0, maxw = 0;
  for (uint32_t v = 0; v <= maxb; v++) if (wc[v]) { distinct++; maxw = v; }
  if (nw < 2u || distinct < 2u) return 0;
  // normalized weight counts at log 6 (any distribution summing to 64 with every used
  // value >= 1 is a valid description)
  const uint32_t LOG = 6;
  int16_t norm[HUF_MAXBITS + 2];
  int32_t sum = 0, big = 0;
  for (uint32_t v = 0; v <= maxw; v++) {
    int32_t c = wc[v] ? (int32_t)((wc[v] << LOG) / nw) : 0;
    if (wc[v] && c < 1) c = 1;
    norm[v] = (int16_t)c;
    sum += c;
    if (c > norm[big]) big = (int32_t)v;
  }
  while (sum > (1 << LOG)) {
    int32_t m = 0;
    for (uint32_t v = 0; v <= maxw; v++) if (norm[v] > norm[m]) m = (int32_t)v;
    norm[m]--;
    sum--;
  }
  norm[big] = (int16_t)(norm[big] + ((1 << LOG) - sum));
  CTab& t = sh.wt;
  build_norm(t, norm, maxw + 1u, LOG);
  uint32_t o = 1u + write_ncount(sh.tree + 1, norm, maxw + 1u, LOG);
  // two interleaved states, from the last weight back (FSE_compress_usingCTable)
  BitW bw = {0, 0, o, 131u, sh.tree, 0};
  uint32_t s1 = 0, s2 = 0;
  int32_t i = (int32_t)nw - 1;
  if (nw & 1u) {
    s1 = fse_init(t, w[i--]);
    s2 = fse_init(t, w[i--]);
    fse_enc(bw, t, s1, w[i--]);
  } else {
    s2 = fse_init(t, w[i--]);
    s1 = fse_init(t, w[i--]);
  }
  while (i >= 0) {
    fse_enc(bw, t, s2, w[i--]);
    fse_enc(bw, t, s1, w[i--]);
  }
  bw_add(bw, s2, LOG);
  bw_add(bw, s1, LOG);
  bw_add(bw, 1u, 1u);
  if (bw.n) bw_add(bw, 0u, 8u - bw.n);
  if (bw.over || bw.pos - 1u >= 128u) return 0;
  sh.tree[0] = (uint8_t)(bw.pos - 1u);
  return bw.pos;
}

// One wavefront: the segment's literals section into out (LCAP bytes); returns its size,
// or 0 when raw literals are not larger (encode_segment then writes them raw).
HZ_HD uint32_t lit_section(LitShared& sh, const uint16_t* tok, const hd::SegParse* sp, uint8_t* out) {
  const hz_gu16* const gt = HZ_GLOBAL(const hz_gu16*, tok);
  auto slot = [&](uint32_t k, uint32_t l) -> uint32_t { return gt[hd::tslot(k, (int)l)]; };
  // literal bytes in stream order: parse lane l's literals after those of lanes < l
  LANE_LOOP {
    uint32_t c = 0;
    const uint32_t ns = sp->nslot[lane];
    for (uint32_t k = 0; k < ns;) {
      if (slot(k, (uint32_t)lane) & 0x8000u) { k += 2; continue; }
      c++;
      k++;
    }
    sh.cnt[lane] = c;
  }
  WAVE_SYNC();
  LANE_LOOP {
    if (lane == 0) {
      uint32_t b = 0;
      for (int l = 0; l < hd::WAVE; l++) { sh.base[l] = b; b += sh.cnt[l]; }
      sh.nlit = b;
    }
  }
  WAVE_SYNC();
  const uint32_t nlit = sh.nlit;
  if (nlit < 64u) return 0;
  LANE_LOOP {
    uint32_t b = sh.base[lane];
    const uint32_t ns = sp->nslot[lane];
    for (uint32_t k = 0; k < ns;) {
      const uint32_t v = slot(k, (uint32_t)lane);
      if (v & 0x8000u) { k += 2; continue; }
      sh.lit[b++] = (uint8_t)v;
      k++;
    }
    for (int q = lane; q < 256; q += hd::WAVE) sh.hs.freq[q] = sp->freq[q];
  }
  WAVE_SYNC();
  HD_BUILD_HUFF(sh.hs, sh.hs.freq, 256, 256, (int)HUF_MAXBITS, sh.hs.len_ll, sh.hs.code_ll);
  LANE_LOOP {
    if (lane == 0) sh.tsize = huff_tree(sh, sh.hs.len_ll);
  }
  WAVE_SYNC();
  if (!sh.tsize) return 0;
  // four streams, each encoded from its last literal back (HUF_compress1X), lanes 0-3
  const uint32_t segsz = (nlit + 3u) / 4u;
  LANE_LOOP {
    if (lane < 4) {
      const uint32_t a = (uint32_t)lane * segsz, b = lane == 3 ? nlit : a + segsz;
      BitW bw = {0, 0, 0, STRM, sh.strm[lane], 0};
      for (uint32_t i = b; i > a; i--) {
        const uint32_t c = sh.lit[i - 1u];
        bw_add(bw, sh.val[c], sh.hs.len_ll[c]);
      }
      bw_add(bw, 1u, 1u);
      if (bw.n) bw_add(bw, 0u, 8u - bw.n);
      sh.ssize[lane] = bw.over ? 0xffffu + 1u : bw.pos;
    }
  }
  WAVE_SYNC();
  LANE_LOOP {
    if (lane == 0) {
      uint32_t ok = 1, csize = sh.tsize + 6u;
      for (int k = 0; k < 4; k++) { csize += sh.ssize[k]; ok &= sh.ssize[k] <= 0xffffu && (k == 3 || sh.ssize[k]); }
      const uint32_t hsz = (nlit < 1024u && csize < 1024u) ? 3u : 4u;
      const uint32_t rawsz = nlit + (nlit < 32u ? 1u : nlit < 4096u ? 2u : 3u);
      if (!ok || hsz + csize >= rawsz || csize >= (1u << 14)) {
        sh.size = 0;
      } else {
        // Literals_Section_Header: type 2, size format 1 (3 bytes, 10-bit sizes) or 2 (4 bytes)
        const uint32_t h = 2u | ((hsz == 3u ? 1u : 2u) << 2) | (nlit << 4) | (csize << (hsz == 3u ? 14u : 18u));
        for (uint32_t i = 0; i < hsz; i++) out[i] = (uint8_t)(h >> (8u * i));
        uint32_t o = hsz;
        for (uint32_t i = 0; i < sh.tsize; i++) out[o++] = sh.tree[i];
        for (int k = 0; k < 3; k++) { out[o++] = (uint8_t)sh.ssize[k]; out[o++] = (uint8_t)(sh.ssize[k] >> 8); }
        sh.base[0] = o;                                // where stream 0 starts
        sh.size = hsz + csize;
      }
    }
  }
  WAVE_SYNC();
  const uint32_t size = sh.size;
  if (!size) return 0;
  LANE_LOOP {
    uint32_t o = sh.base[0];
    for (int k = 0; k < 4; k++) {
      for (uint32_t i = (uint32_t)lane; i < sh.ssize[k]; i += hd::WAVE) out[o + i] = sh.strm[k][i];
      o += sh.ssize[k];
    }
  }
  WAVE_SYNC();
  return size;
}

// The 16-bit token slots of parse lane l (ns of them; slots 2w, 2w + 1 share the dword
// w * WAVE + l), forward or backward, loaded 8 dwords at a time: a batch costs one memory
// latency instead of one per slot (the block writes in between would otherwise keep the
// compiler from hoisting the loads).
// the lane's slots in order, NB dwords (2 NB slots) per batch of loads
template <uint32_t NB, class F>
HZ_HD void slots_fwd_n(hz_gcu32* gw, uint32_t ns, uint32_t l, F&& f) {
  const uint32_t nw = (ns + 1u) >> 1;
  for (uint32_t w0 = 0; w0 < nw; w0 += NB) {
    uint32_t wv[NB];
HZ_UNROLL
    for (uint32_t i = 0; i < NB; i++) wv[i] = w0 + i < nw ? gw[(size_t)(w0 + i) * (uint32_t)hd::WAVE + l] : 0u;
    const uint32_t cnt = nw - w0 < NB ? nw - w0 : NB;
    for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t word = wv[0];
HZ_UNROLL
      for (uint32_t i = 0; i + 1 < NB; i++) wv[i] = wv[i + 1];
      f(word & 0xffffu);
      if (2u * (w0 + k) + 1u < ns) f(word >> 16);
    }
  }
}
template <class F>
HZ_HD void slots_fwd(hz_gcu32* gw, uint32_t ns, uint32_t l, F&& f) {
  slots_fwd_n<8>(gw, ns, l, static_cast<F&&>(f));
}
template <class F>
HZ_HD void slots_bwd(hz_gcu32* gw, uint32_t ns, uint32_t l, F&& f) {
  uint32_t w1 = (ns + 1u) >> 1;
  while (w1 > 0) {
    const uint32_t cnt = w1 < 8u ? w1 : 8u;
    uint32_t wv[8];
HZ_UNROLL
    for (uint32_t i = 0; i < 8u; i++) wv[i] = i < cnt ? gw[(size_t)(w1 - 1u - i) * (uint32_t)hd::WAVE + l] : 0u;
    for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t word = wv[0];
HZ_UNROLL
      for (uint32_t i = 0; i + 1 < 8u; i++) wv[i] = wv[i + 1];
      if (2u * (w1 - 1u - k) + 1u < ns) f(word >> 16);
      f(word & 0xffffu);
    }
    w1 -= cnt;
  }
}

// The sequences of a segment, last to first: emit(literal run, match length, offset).  The
// backward walk knows a match's literal run once it reaches the match before it (or the
// segment start), so each sequence is emitted one match late.
template <class F>
HZ_HD void walk_sequences(hz_gcu32* gw, const hd::SegParse* sp, F&& emit) {
  uint32_t have = 0, pml = 0, poff = 0, run = 0;
  for (int32_t l = hd::WAVE - 1; l >= 0; l--) {
    // backward: slot k is held until slot k - 1 shows whether (k - 1, k) is a match
    uint32_t pend = 0, hold = 0;
    slots_bwd(gw, sp->nslot[l], (uint32_t)l, [&](uint32_t u) {
      if (!hold) { pend = u; hold = 1; return; }
      if (u & 0x8000u) {                           // (u, pend): a match
        if (have) emit(run, pml, poff);
        have = 1;
        pml = (u & 0x7fffu) + 3u;
        poff = pend + 1u;
        run = 0;
        hold = 0;
      } else {
        run++;                                     // pend: a literal (trailing ones belong to no sequence)
        pend = u;
      }
    });
    if (hold) run++;
  }
  if (have) emit(run, pml, poff);
}

// zstd_count_kernel's share of parse lane l in a segment's counts (the kernel's per-lane
// algorithm; count_segment_lanes below runs it lane by lane on the CPU): the lane walks its
// own token slots forward and adds (code index into SeqCounts: LL 0-35, OF 36-67, ML 68-120)
// the offset and match-length codes of its matches and the literal-length codes of all but
// its first match, whose literal run may begin in earlier lanes (first_run, after the scans)
struct LaneCount {
  uint32_t lits;     // literals in the lane's range
  uint32_t run;      // literals after its last match
  uint32_t lead;     // literals before its first match
  uint32_t hm;       // it has a match
};
template <class Add>
HZ_HD LaneCount lane_count(const CodeTabs& ct, hz_gcu32* gw, uint32_t ns, uint32_t l, Add&& add) {
  LaneCount r = {0u, 0u, 0u, 0u};
  uint32_t want_dist = 0, ml = 0;
  slots_fwd(gw, ns, l, [&](uint32_t v) {
    if (want_dist) {                               // (len | 0x8000, dist - 1): a match
      const Seq q = make_seq_t(ct, r.run, ml, v + 1u);
      if (r.hm) add(q.llc);
      else r.lead = r.run;
      add(36u + q.ofc);
      add(68u + q.mlc);
      r.hm = 1;
      r.run = 0;
      want_dist = 0;
    } else if (v & 0x8000u) {
      ml = (v & 0x7fffu) + 3u;
      want_dist = 1;
    } else {
      r.run++;
      r.lits++;
    }
  });
  return r;
}
// literal ordinal after the lane's last match (0: no match); L = literals before the lane
HZ_HD uint32_t lane_q(uint32_t L, const LaneCount& r) { return r.hm ? L + r.lits - r.run : 0u; }
// the literal run of the lane's first match: qprev = max lane_q over the earlier lanes
HZ_HD uint32_t first_run(uint32_t L, const LaneCount& r, uint32_t qprev) { return L + r.lead - qprev; }

#if !HZ_GPU
// zstd_count_kernel's algorithm for one segment on the CPU: lane_count for every parse lane,
// the kernel's add scan (L) and exclusive max scan (qprev) done serially
inline void count_segment_lanes(const CodeTabs& ct, const uint16_t* tok, const hd::SegParse* sp, SeqCounts& c) {
  hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, tok);
  uint32_t* const cw = (uint32_t*)&c;
  LaneCount lc[hd::WAVE];
  for (uint32_t l = 0; l < (uint32_t)hd::WAVE; l++) lc[l] = lane_count(ct, gw, sp->nslot[l], l, [&](uint32_t k) { cw[k]++; });
  uint32_t L = 0, qmax = 0;
  for (uint32_t l = 0; l < (uint32_t)hd::WAVE; l++) {
    if (lc[l].hm) cw[make_seq_t(ct, first_run(L, lc[l], qmax), 3u, 1u).llc]++;
    const uint32_t q = lane_q(L, lc[l]);
    qmax = q > qmax ? q : qmax;
    L += lc[l].lits;
  }
}
#endif

// adds a segment's sequence codes to c (the frame's counts)
HZ_HD void count_segment(const CodeTabs& ct, const uint16_t* tok, const hd::SegParse* sp, SeqCounts& c) {
  hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, tok);
  walk_sequences(gw, sp, [&](uint32_t ll, uint32_t ml, uint32_t off) {
    const Seq q = make_seq_t(ct, ll, ml, off);
    c.ll[q.llc]++;
    c.of[q.ofc]++;
    c.ml[q.mlc]++;
  });
}

// ---- the compact sequences of a segment (zstd_seq_kernel, round 6) ------------------------
// zstd_seg_kernel's lane per segment used to walk the 64 parse lanes' token slots itself --
// twice (literals forward, sequences backward), each load of its lane touching its own cache
// lines, 64 segments' slots per wave.  zstd_seq_kernel (one wave per segment, each lane on its
// own parse lane: coalesced rows) turns the slots into a compact sequence array in the same
// scratch -- a[i] = literal run | match length << 16, b[i] = offset - 1, in segment order --
// and writes the raw literals section's bytes into the block scratch (byte stores: no LDS copy
// of the literals, so that more waves per CU hide the token loads; 16 dwords per batch).
constexpr uint32_t SEQ_MAX = (uint32_t)hd::SEG / 3u + 1u;     // a match covers >= 3 input bytes
static_assert(SEQ_MAX * 6u <= (uint32_t)hd::SEG_TOK * 2u, "the compact sequences fit the segment's token slots");
HZ_HD uint32_t* seq_a(uint16_t* tok) { return (uint32_t*)tok; }
HZ_HD uint16_t* seq_b(uint16_t* tok) { return tok + 2u * SEQ_MAX; }
HZ_HD const uint32_t* seq_a(const uint16_t* tok) { return (const uint32_t*)tok; }
HZ_HD const uint16_t* seq_b(const uint16_t* tok) { return tok + 2u * SEQ_MAX; }
// the raw literals section header (Literals_Section_Header, Raw_Literals_Block) for n bytes
HZ_HD uint32_t lit_header(uint32_t n, uint8_t* h) {
  if (n < 32u) { h[0] = (uint8_t)(n << 3); return 1; }
  if (n < 4096u) { h[0] = (uint8_t)((1u << 2) | ((n & 15u) << 4)); h[1] = (uint8_t)(n >> 4); return 2; }
  h[0] = (uint8_t)((3u << 2) | ((n & 15u) << 4)); h[1] = (uint8_t)((n >> 4) & 0xffu); h[2] = (uint8_t)(n >> 12);
  return 3;
}
// parse lane l's part of the segment, pass 1: literals, the run after its last match, the run
// before its first match, whether it has one, its matches
struct LaneSeq {
  uint32_t lits, run, lead, hm, nm;
};
template <uint32_t NB = 8>
HZ_HD LaneSeq lane_seq_count(hz_gcu32* gw, uint32_t ns, uint32_t l) {
  LaneSeq r = {0u, 0u, 0u, 0u, 0u};
  uint32_t want_dist = 0;
  slots_fwd_n<NB>(gw, ns, l, [&](uint32_t v) {
    if (want_dist) {
      if (!r.hm) r.lead = r.run;
      r.hm = 1; r.nm++; r.run = 0; want_dist = 0;
    } else if (v & 0x8000u) {
      want_dist = 1;
    } else {
      r.run++; r.lits++;
    }
  });
  return r;
}
// pass 2: lit(k, byte) for the lane's k-th literal, seq(j, run, length, offset) for its j-th
// match (the first one's run = first, from the scans over the lanes)
template <uint32_t NB = 8, class Lit, class Sq>
HZ_HD void lane_seq_emit(hz_gcu32* gw, uint32_t ns, uint32_t l, uint32_t first, Lit&& lit, Sq&& sq) {
  uint32_t want_dist = 0, ml = 0, run = 0, k = 0, j = 0;
  slots_fwd_n<NB>(gw, ns, l, [&](uint32_t v) {
    if (want_dist) {
      sq(j, j ? run : first, ml, v + 1u);
      j++; run = 0; want_dist = 0;
    } else if (v & 0x8000u) {
      ml = (v & 0x7fffu) + 3u;
      want_dist = 1;
    } else {
      lit(k, v);
      k++; run++;
    }
  });
}
#if !HZ_GPU
// zstd_seq_kernel on the CPU: both passes lane by lane, the kernel's scans done serially; the
// raw literals (header included) into out + 3 when `raw` (the block scratch)
inline void extract_sequences(uint16_t* tok, const hd::SegParse* sp, uint8_t* out, int raw) {
  hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, tok);
  LaneSeq lc[hd::WAVE];
  uint32_t L[hd::WAVE], S[hd::WAVE], Q[hd::WAVE];
  uint32_t nlit = 0, nseq = 0, qmax = 0;
  for (uint32_t l = 0; l < (uint32_t)hd::WAVE; l++) {
    lc[l] = lane_seq_count(gw, sp->nslot[l], l);
    L[l] = nlit; S[l] = nseq; Q[l] = qmax;
    const uint32_t q = lc[l].hm ? nlit + lc[l].lits - lc[l].run : 0u;
    qmax = q > qmax ? q : qmax;
    nlit += lc[l].lits; nseq += lc[l].nm;
  }
  static thread_local uint32_t A[SEQ_MAX];
  static thread_local uint16_t B[SEQ_MAX];
  static thread_local uint8_t lbuf[hd::SEG + 16];
  for (uint32_t l = 0; l < (uint32_t)hd::WAVE; l++)
    lane_seq_emit(gw, sp->nslot[l], l, L[l] + lc[l].lead - Q[l],
                  [&](uint32_t k, uint32_t v) { lbuf[L[l] + k] = (uint8_t)v; },
                  [&](uint32_t j, uint32_t run, uint32_t ml, uint32_t off) {
                    A[S[l] + j] = run | (ml << 16); B[S[l] + j] = (uint16_t)(off - 1u); });
  memcpy(seq_a(tok), A, nseq * 4u);
  memcpy(seq_b(tok), B, nseq * 2u);
  if (raw) {
    const uint32_t h = lit_header(nlit, out + 3);
    memcpy(out + 3 + h, lbuf, nlit);
  }
}
#endif

// the compact sequences last to first (ZE_SEQB per batch: one memory latency per batch)
#ifndef ZE_SEQB
#define ZE_SEQB 32                      // bench zstd_encode 8 / 16 / 32: 31.9 / 32.2 / 32.6 GB/s of slab
#endif
template <class F>
HZ_HD void seqs_bwd(const uint32_t* A, const uint16_t* B, uint32_t n, F&& emit) {
  hz_gcu32* const ga = HZ_GLOBAL(hz_gcu32*, A);
  const hz_gu16* const gb = HZ_GLOBAL(const hz_gu16*, B);
  constexpr uint32_t NB = ZE_SEQB;
  uint32_t i1 = n;
  while (i1 > 0u) {
    const uint32_t cnt = i1 < NB ? i1 : NB;
    uint32_t av[NB], bv[NB];
HZ_UNROLL
    for (uint32_t i = 0; i < NB; i++) {
      const uint32_t k = i < cnt ? i1 - 1u - i : i1 - 1u;
      av[i] = ga[k];
      bv[i] = gb[k];
    }
    for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t a = av[0], b = bv[0];
HZ_UNROLL
      for (uint32_t i = 0; i + 1 < NB; i++) { av[i] = av[i + 1]; bv[i] = bv[i + 1]; }
      emit(a & 0xffffu, a >> 16, b + 1u);
    }
    i1 -= cnt;
  }
}

// Writes segment `seg` of a stream as one zstd block (header included) at out (cap bytes
// of scratch, >= ZCAP).  tok / sp: the segment's parse tokens and counts; job / s0: the
// stream input (a raw block copies the segment from it).  Returns the block size.
// seqs: tok holds the compact sequences (zstd_seq_kernel), and out + 3 the raw literals section
// unless lsize (the Huffman section in lsec)
HZ_HD uint32_t encode_segment(const Tabs& T, const CodeTabs& ct, const uint16_t* tok, const hd::SegParse* sp, const hd::EncJob& job,
                              uint32_t s0, uint32_t seglen, uint32_t last, uint8_t* out, uint32_t cap,
                              const uint8_t* lsec = nullptr, uint32_t lsize = 0, int seqs = 0) {
  hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, tok);
  uint32_t nlit = 0, nseq = 0;
  for (uint32_t s = 0; s < 256u; s++) nlit += sp->freq[s];
  for (uint32_t s = 257; s < 286u; s++) nseq += sp->freq[s];
  int over = 0;
  uint32_t p = 3;
  if (lsize) {
    // the Huffman-coded literals section (lit_section)
    for (uint32_t i = 0; i < lsize; i++) put8(out, p, cap, lsec[i], over);
  } else if (nlit < 32u) {
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
  // (gathered in a register and stored a dword at a time: the lane's scratch block is
  // 4-byte aligned; bytes already written below p in the first word are kept)
  if (!lsize && !over && seqs) {
    if (p + nlit > cap) over = 1;           // (zstd_seq_kernel wrote them)
    else p += nlit;
  } else if (!lsize && !over) {
    if (p + nlit > cap) {
      over = 1;
    } else {
      uint32_t acc = 0;
      for (uint32_t b = 0; b < (p & 3u); b++) acc |= (uint32_t)out[(p & ~3u) + b] << (8u * b);
      for (uint32_t l = 0; l < (uint32_t)hd::WAVE; l++) {
        uint32_t skip = 0;                             // the distance slot after a match length
        slots_fwd(gw, sp->nslot[l], l, [&](uint32_t v) {
          if (skip) { skip = 0; return; }
          if (v & 0x8000u) { skip = 1; return; }
          acc |= v << (8u * (p & 3u));
          p++;
          if (!(p & 3u)) { *(uint32_t*)(out + p - 4u) = acc; acc = 0; }
        });
      }
      for (uint32_t b = 0; b < (p & 3u); b++) out[(p & ~3u) + b] = (uint8_t)(acc >> (8u * b));
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
    put8(out, p, cap, T.mode, over);                 // Symbol_Compression_Modes
    for (uint32_t i = 0; i < T.dsize; i++) put8(out, p, cap, T.desc[i], over);
    BitD w;
    bd_init(w, out, p, cap, over);
    uint32_t sll = 0, sof = 0, sml = 0;
    uint32_t first = 1, bad = 0;
    auto emit = [&](uint32_t ll, uint32_t ml, uint32_t off) {
      const Seq q = make_seq_t(ct, ll, ml, off);
      bad |= (absent(T.ll, q.llc) || absent(T.of, q.ofc) || absent(T.ml, q.mlc)) ? 1u : 0u;
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
    if (seqs) seqs_bwd(seq_a(tok), seq_b(tok), nseq, emit);
    else walk_sequences(gw, sp, emit);
    bw_add(w, sml, T.ml.log);
    bw_add(w, sof, T.of.log);
    bw_add(w, sll, T.ll.log);
    bw_add(w, 1u, 1u);                               // end mark
    p = bd_finish(w);
    over = w.over || bad;
  }
  const uint32_t csize = p - 3u;
  if (over || csize >= seglen) {
    // Raw_Block: the segment's bytes
    block_header(out, last, 0u, seglen);
    // s0 is a multiple of the segment size: 8 aligned stream words per round, loaded together
    for (uint32_t i0 = 0; i0 < seglen; i0 += 32u) {
      uint32_t wv[8];
HZ_UNROLL
      for (uint32_t k = 0; k < 8u; k++) wv[k] = i0 + 4u * k < seglen ? hd::load_stream_word(job, s0 + i0 + 4u * k, job.len) : 0u;
HZ_UNROLL
      for (uint32_t k = 0; k < 32u; k++)
        if (i0 + k < seglen) out[3u + i0 + k] = (uint8_t)(wv[k >> 2] >> (8u * (k & 3u)));
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
