// zstd_lane.h -- Zstandard (RFC 8878) frame decoder, one lane per Blosc split.
//
// c-blosc 1.21 writes codec 4 ("zstd", dsetUtil.py:44) splits as single zstd frames
// (zstd_wrap_compress); the reference decodes them through storUtil._uncompress ->
// numcodecs Blosc.decode (storUtil.py:195-208).  zstd's sequence decoding is a serial
// chain of FSE state transitions, so each lane decodes one whole split; a batch holds
// thousands of splits, which run in parallel across the lanes of the chip.
//
// Memory: a lane's FSE / Huffman decode tables (ZTAB_BYTES) live in a global scratch
// slot it owns; literals are decoded into the END of the split's own output span
// (dst + cap - literals), which the block's output can only reach after reading them
// (the block ends at or before cap), so no literal buffer is needed.
//
// Single source: tests/emu/zstd_emu.cpp runs the same code on CPU.
#pragma once
#include "inflate_wave.h"

namespace zs {

struct Fse { uint8_t sym, nb; uint16_t base; };
struct Huf { uint8_t sym, nb; };

struct Tables {            // one per lane, in global memory
  Fse ll[512], of[256], ml[512];
  Fse hw[64];              // Huffman weights table (accuracy <= 6)
  Huf huf[1 << 11];
  uint32_t ll_al, of_al, ml_al, have_seq, huf_bits, have_huf, huf_nw;
  uint32_t rep[3];
  int16_t norm[256];       // scratch for table descriptions
  uint16_t next[256];
  uint8_t w[256];
};
constexpr size_t ZTAB_BYTES = (sizeof(Tables) + 255) & ~(size_t)255;

constexpr int OK = 0, E_DATA = -2, E_TRUNC = -3, E_SIZE = -4, E_UNSUP = -5;

// constexpr (host and device): also used to build the predefined tables at compile time
constexpr uint32_t hib(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v | 1u); }

// input bytes of the split (bounded)
struct In { const uint8_t* p; uint32_t n; };
HZ_HD uint32_t b8(const In& in, uint32_t i) { return i < in.n ? (uint32_t)((hz_gcu8*)HZ_GLOBAL(hz_gcu8*, in.p))[i] : 0u; }

// backward bitstream over input bytes [lo, lo + n): bits are consumed from the end
struct Bits { In in; uint32_t lo; int64_t pos; };   // pos: bits left above the start
HZ_HD int bits_init(Bits& b, const In& in, uint32_t lo, uint32_t n) {
  if (n == 0 || lo + n > in.n) return -1;
  const uint32_t last = b8(in, lo + n - 1);
  if (!last) return -1;
  b.in = in; b.lo = lo;
  b.pos = 8 * (int64_t)(n - 1) + hib(last);
  return 0;
}
// the next k (<= 32) bits, most significant first; bits before the start read as 0
HZ_HD uint32_t bits_read(Bits& b, uint32_t k) {
  if (!k) return 0;
  const int64_t np = b.pos - (int64_t)k;
  // gather the 5 bytes covering [np, pos) (at most 32 bits) as a little-endian window
  const int64_t lo_bit = np < 0 ? 0 : np;
  const int64_t byte0 = lo_bit >> 3;
  uint64_t w = 0;
  for (int i = 4; i >= 0; i--) {
    const int64_t bi = byte0 + i;
    w = (w << 8) | ((bi >= 0 && (bi << 3) < b.pos) ? b8(b.in, b.lo + (uint32_t)bi) : 0u);
  }
  uint32_t v = (uint32_t)((w >> (lo_bit & 7)) & ((k == 32) ? 0xffffffffull : ((1ull << k) - 1ull)));
  if (np < 0) v = (uint32_t)(((uint64_t)v << (-np)) & ((k == 32) ? 0xffffffffull : ((1ull << k) - 1ull)));
  // v holds bits [lo_bit, pos) aligned at lo_bit; when np < 0 the missing low bits are 0
  b.pos = np;
  return v;
}

// FSE table description (forward little-endian bits); returns bytes used or -1
template <class TT>
HZ_HD int64_t ncount(TT& t, const In& in, uint32_t at, uint32_t n, uint32_t& maxsym, uint32_t& al,
                     uint32_t maxal) {
  if (n < 1) return -1;
  uint64_t bp = 0;
  auto rd = [&](uint32_t k) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < k; i++) {
      const uint64_t q = bp + i;
      if ((q >> 3) < n) v |= ((b8(in, at + (uint32_t)(q >> 3)) >> (q & 7)) & 1u) << i;
    }
    return v;
  };
  const uint32_t log = rd(4) + 5u;
  bp = 4;
  if (log > maxal) return -1;
  al = log;
  int32_t remaining = (1 << log) + 1, threshold = 1 << log;
  uint32_t nbits = log + 1, s = 0;
  int prev0 = 0;
  while (remaining > 1 && s <= maxsym) {
    if (prev0) {
      uint32_t n0 = s;
      for (;;) {
        const uint32_t r = rd(2);
        bp += 2;
        n0 += r;
        if (r != 3u) break;
      }
      if (n0 > maxsym + 1u) return -1;
      while (s < n0) t.norm[s++] = 0;
      if (s > maxsym) break;
    }
    const int32_t mx = (2 * threshold - 1) - remaining;
    int32_t count;
    const uint32_t low = rd(nbits - 1u);
    if ((int32_t)low < mx) { count = (int32_t)low; bp += nbits - 1u; }
    else {
      count = (int32_t)rd(nbits);
      if (count >= threshold) count -= mx;
      bp += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    t.norm[s++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) { nbits--; threshold >>= 1; }
  }
  if (remaining != 1) return -1;
  maxsym = s - 1u;
  return (int64_t)((bp + 7) >> 3);
}

template <class TT>
HZ_HD int build_fse(TT& t, Fse* tab, uint32_t maxsym, uint32_t al) {
  const uint32_t size = 1u << al;
  int32_t high = (int32_t)size - 1;
  for (uint32_t s = 0; s <= maxsym; s++) {
    if (t.norm[s] == -1) { tab[high--].sym = (uint8_t)s; t.next[s] = 1; }
    else t.next[s] = (uint16_t)t.norm[s];
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3u, mask = size - 1u;
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= maxsym; s++)
    for (int32_t i = 0; i < t.norm[s]; i++) {
      tab[pos].sym = (uint8_t)s;
      do pos = (pos + step) & mask; while ((int32_t)pos > high);
    }
  if (pos != 0) return -1;
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t ns = t.next[tab[u].sym]++;
    const uint32_t nb = al - hib(ns);
    tab[u].nb = (uint8_t)nb;
    tab[u].base = (uint16_t)((ns << nb) - size);
  }
  return 0;
}

// predefined distributions (RFC 8878 3.1.1.3.2.2) and code baselines
constexpr int16_t def_norm(uint32_t which, uint32_t s) {
  // which: 0 LL (36 codes), 1 OF (29), 2 ML (53)
  if (which == 0) {
    const int16_t v[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
                           -1, -1, -1, -1};
    return v[s];
  }
  if (which == 1) {
    const int16_t v[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    return v[s];
  }
  return s == 0 ? 1 : s == 1 ? 4 : s == 2 ? 3 : s < 9 ? 2 : s < 46 ? 1 : -1;
}
// code -> baseline / extra bits (RFC 8878 3.1.1.3.2.1.1), from packed immediates: a
// local table would be read from memory on every sequence
constexpr uint32_t ll_bits(uint32_t c) {
  if (c < 16) return 0;
  if (c >= 25) return c - 19;                                   // 25: 6 bits ... 35: 16 bits
  return (uint32_t)((0x433221111ull >> (4 * (c - 16))) & 15u);   // 16..24: 1 1 1 1 2 2 3 3 4
}
HZ_HD uint32_t ll_base(uint32_t c) {
  if (c < 16) return c;
  if (c >= 25) return 1u << (c - 19);                           // 64, 128, ... 65536
  // 16..24: 16 18 20 22 24 28 32 40 48, 6 bits each
  const uint64_t v = 16ull | 18ull << 6 | 20ull << 12 | 22ull << 18 | 24ull << 24 | 28ull << 30 | 32ull << 36 |
                     40ull << 42 | 48ull << 48;
  return (uint32_t)((v >> (6 * (c - 16))) & 63u);
}
constexpr uint32_t ml_bits(uint32_t c) {
  if (c < 32) return 0;
  if (c >= 43) return c - 36;                                   // 43: 7 bits ... 52: 16 bits
  // 32..42: 1 1 1 1 2 2 3 3 4 4 5, 3 bits each
  const uint64_t v = 1ull | 1ull << 3 | 1ull << 6 | 1ull << 9 | 2ull << 12 | 2ull << 15 | 3ull << 18 | 3ull << 21 |
                     4ull << 24 | 4ull << 27 | 5ull << 30;
  return (uint32_t)((v >> (3 * (c - 32))) & 7u);
}
HZ_HD uint32_t ml_base(uint32_t c) {
  if (c < 32) return c + 3;
  if (c >= 43) return (1u << (c - 36)) + 3u;                    // 131, 259, ... 65539
  // 32..42: 35 37 39 41 43 47 51 59 67 | 83 99, 7 bits each
  if (c < 41) {
    const uint64_t v = 35ull | 37ull << 7 | 39ull << 14 | 41ull << 21 | 43ull << 28 | 47ull << 35 | 51ull << 42 |
                       59ull << 49 | 67ull << 56;
    return (uint32_t)((v >> (7 * (c - 32))) & 127u);
  }
  return c == 41 ? 83u : 99u;
}

// LL / OF / ML table: mode 0 predefined, 1 RLE, 2 FSE description, 3 repeat
template <class TT>
HZ_HD int64_t seq_table(TT& t, Fse* tab, uint32_t& al, uint32_t mode, const In& in, uint32_t at, uint32_t n,
                        uint32_t which, uint32_t maxsym, uint32_t maxal) {
  if (mode == 0) {
    const uint32_t defmax = which == 0 ? 35u : which == 1 ? 28u : 52u;
    for (uint32_t s = 0; s <= defmax; s++) t.norm[s] = def_norm(which, s);
    al = which == 1 ? 5u : 6u;
    return build_fse(t, tab, defmax, al) ? -1 : 0;
  }
  if (mode == 1) {
    if (n < 1 || b8(in, at) > maxsym) return -1;
    tab[0].sym = (uint8_t)b8(in, at); tab[0].nb = 0; tab[0].base = 0;
    al = 0;
    return 1;
  }
  if (mode == 2) {
    uint32_t ms = maxsym, l = 0;
    const int64_t used = ncount(t, in, at, n, ms, l, maxal);
    if (used < 0 || build_fse(t, tab, ms, l)) return -1;
    al = l;
    return used;
  }
  return t.have_seq ? 0 : -1;
}

template <class TT>
HZ_HD void huf_fill(TT& t, uint32_t nw, uint32_t maxb);

// Huffman tree description at `at`; returns bytes used or -1
template <class TT>
HZ_HD int64_t huf_tree(TT& t, const In& in, uint32_t at, uint32_t n) {
  if (n < 1) return -1;
  uint32_t nw = 0;
  int64_t used;
  const uint32_t h = b8(in, at);
  if (h >= 128) {
    nw = h - 127u;
    used = 1 + (nw + 1) / 2;
    if (used > n) return -1;
    for (uint32_t i = 0; i < nw; i++) {
      const uint32_t byte = b8(in, at + 1 + i / 2);
      t.w[i] = (uint8_t)((i & 1) ? (byte & 15u) : (byte >> 4));
    }
  } else {
    const uint32_t cs = h;
    used = 1 + (int64_t)cs;
    if (used > n || cs < 1) return -1;
    uint32_t ms = 255, al = 0;
    const int64_t u = ncount(t, in, at + 1, cs, ms, al, 6);
    if (u < 0) return -1;
    Fse* tab = t.hw;
    if (build_fse(t, tab, ms, al)) return -1;
    Bits b;
    if (bits_init(b, in, at + 1 + (uint32_t)u, cs - (uint32_t)u)) return -1;
    uint32_t s1 = bits_read(b, al), s2 = bits_read(b, al);
    for (;;) {
      if (nw >= 255) return -1;
      t.w[nw++] = tab[s1].sym;
      s1 = tab[s1].base + bits_read(b, tab[s1].nb);
      if (b.pos < 0) { t.w[nw++] = tab[s2].sym; break; }
      if (nw >= 255) return -1;
      t.w[nw++] = tab[s2].sym;
      s2 = tab[s2].base + bits_read(b, tab[s2].nb);
      if (b.pos < 0) { if (nw >= 255) return -1; t.w[nw++] = tab[s1].sym; break; }
    }
  }
  uint32_t total = 0;
  for (uint32_t i = 0; i < nw; i++) {
    if (t.w[i] > 11) return -1;
    if (t.w[i]) total += 1u << (t.w[i] - 1);
  }
  if (!total) return -1;
  const uint32_t maxb = hib(total) + 1;
  const uint32_t rest = (1u << maxb) - total;
  if (rest & (rest - 1)) return -1;
  t.w[nw++] = (uint8_t)(hib(rest) + 1);
  if (maxb > 11) return -1;
  t.huf_nw = nw;
  huf_fill(t, nw, maxb);
  return used;
}

// the decode table of weights w[0, nw) (max code length maxb): entries of symbol i fill
// 2^(w-1) consecutive slots in weight order
template <class TT>
HZ_HD void huf_fill(TT& t, uint32_t nw, uint32_t maxb) {
  uint32_t start[13];
  {
    uint32_t rank[13];
    for (int k = 0; k < 13; k++) rank[k] = 0;
    for (uint32_t i = 0; i < nw; i++) rank[t.w[i]]++;
    uint32_t nx = 0;
    for (uint32_t k = 1; k <= maxb; k++) { start[k] = nx; nx += rank[k] << (k - 1); }
  }
  for (uint32_t i = 0; i < nw; i++) {
    const uint32_t wi = t.w[i];
    if (!wi) continue;
    const uint32_t len = 1u << (wi - 1);
    for (uint32_t u = start[wi]; u < start[wi] + len; u++) { t.huf[u].sym = (uint8_t)i; t.huf[u].nb = (uint8_t)(maxb + 1 - wi); }
    start[wi] += len;
  }
  t.huf_bits = maxb;
  t.have_huf = 1;
}

// one Huffman literal stream (backward bitstream of n bytes at `at`) -> cnt symbols.
// The bits come from four aligned dwords held in registers (W0 the highest); when the
// top one is used up the others move up and the next lower dword is loaded, three
// dwords (~10 symbols) before it is needed, so the loads' latency is hidden.
template <class TT>
HZ_HD int huf_stream(const TT& t, const In& in, uint32_t at, uint32_t n, hz_gu8* out, uint32_t cnt) {
  if (n == 0 || at + n > in.n) return -1;
  const uint32_t last = b8(in, at + n - 1);
  if (!last) return -1;
  const uint32_t a = (uint32_t)(((uintptr_t)in.p + at) & 3u);
  hz_gcu8* base = HZ_GLOBAL(hz_gcu8*, in.p + at - a);     // stream byte i is base[a + i]
  // positions in base bits (stream bit s is base bit s + 8a); bits below the stream
  // start read as 0.  Dword k > 0 lies wholly in the stream (up to the top dword, whose
  // bytes above the stream are never peeked): its load is unconditional, so its use --
  // three dwords later -- is where the wait lands.
  auto dw = [&](int32_t k) -> uint32_t {
    if (k > 0) return *(hz_gcu32*)(base + 4 * k);
    if (k < 0) return 0u;
    return *(hz_gcu32*)base & ~hz::bmask(8u * a);
  };
  int32_t pos = 8 * (int32_t)(n - 1) + (int32_t)hib(last) + 8 * (int32_t)a;   // bits left, exclusive top
  int32_t top = (pos - 1) >> 5;                            // the dword holding bit pos - 1 (W0)
  uint32_t W0 = dw(top), W1 = dw(top - 1), W2 = dw(top - 2), W3 = dw(top - 3);
  const uint32_t hb = t.huf_bits;
  const uint32_t mask = (1u << hb) - 1u;
  for (uint32_t i = 0; i < cnt; i++) {
    // 32 top < pos <= 32 top + 32, so the hb <= 11 bits below pos are in W0:W1
    const uint64_t win = ((uint64_t)W0 << 32) | W1;      // base bits [32 (top - 1), 32 (top + 1))
    const uint32_t rel = (uint32_t)(pos - (int32_t)hb - 32 * (top - 1));
    const Huf e = t.huf[(uint32_t)(win >> rel) & mask];
    pos -= e.nb;
    out[i] = e.sym;
    if (pos <= 32 * top) {
      W0 = W1; W1 = W2; W2 = W3;
      W3 = dw(top - 4);
      top--;
    }
  }
  return pos == 8 * (int32_t)a ? 0 : -1;
}

// n bytes from s to d with d <= s (possibly overlapping): 16 loads issued together,
// then 16 stores, so a copy costs one memory latency per 16 bytes, not per byte
HZ_HD void copy_fwd(hz_gu8* d, hz_gu8* s, uint32_t n) {
  uint32_t i = 0;
  for (; i + 16u <= n; i += 16u) {
    uint8_t v[16];
    HZ_UNROLL
    for (int k = 0; k < 16; k++) v[k] = s[i + k];
    HZ_UNROLL
    for (int k = 0; k < 16; k++) d[i + k] = v[k];
  }
  for (; i < n; i++) d[i] = s[i];
}
// match of ml bytes at op, distance off: byte i comes from op - off + (i mod off),
// which is already final, so the loads of a 16-byte step are independent
HZ_HD void copy_match(hz_gu8* dst, uint32_t op, uint32_t off, uint32_t ml) {
  const uint32_t src = op - off;
  uint32_t i = 0, r = 0;                      // r = i mod off
  for (; i + 16u <= ml; i += 16u) {
    uint8_t v[16];
    HZ_UNROLL
    for (int k = 0; k < 16; k++) {
      v[k] = dst[src + r];
      r = r + 1u == off ? 0u : r + 1u;
    }
    HZ_UNROLL
    for (int k = 0; k < 16; k++) dst[op + i + k] = v[k];
  }
  for (; i < ml; i++) {
    dst[op + i] = dst[src + r];
    r = r + 1u == off ? 0u : r + 1u;
  }
}

// one compressed block at input [at, at + n); output from op; returns the new op or < 0
HZ_HD int64_t block(Tables& t, const In& in, uint32_t at, uint32_t n, hz_gu8* dst, uint32_t op, uint32_t cap) {
  if (n < 1) return E_DATA;
  const uint32_t h0 = b8(in, at), lt = h0 & 3u, sf = (h0 >> 2) & 3u;
  uint32_t rsz, csz = 0, hl, ns = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { rsz = h0 >> 3; hl = 1; }
    else if (sf == 1) { if (n < 2) return E_DATA; rsz = (h0 >> 4) | (b8(in, at + 1) << 4); hl = 2; }
    else { if (n < 3) return E_DATA; rsz = (h0 >> 4) | (b8(in, at + 1) << 4) | (b8(in, at + 2) << 12); hl = 3; }
  } else {
    hl = sf < 2 ? 3u : sf == 2 ? 4u : 5u;
    if (n < hl) return E_DATA;
    uint64_t v = 0;
    for (int i = (int)hl - 1; i >= 0; i--) v = (v << 8) | b8(in, at + (uint32_t)i);
    const uint32_t bits = sf < 2 ? 10u : sf == 2 ? 14u : 18u;
    rsz = (uint32_t)((v >> 4) & ((1u << bits) - 1u));
    csz = (uint32_t)((v >> (4 + bits)) & ((1u << bits) - 1u));
    ns = sf == 0 ? 1u : 4u;
  }
  if (rsz > (1u << 17) || rsz > cap - op) return E_DATA;
  // literals go to the end of the output span
  const uint32_t lbase = cap - rsz;
  hz_gu8* lit = dst + lbase;
  uint32_t q = hl;
  if (lt == 0) {
    if (q + rsz > n) return E_TRUNC;
    for (uint32_t i = 0; i < rsz; i++) lit[i] = (uint8_t)b8(in, at + q + i);
    q += rsz;
  } else if (lt == 1) {
    if (q + 1 > n) return E_TRUNC;
    const uint8_t c = (uint8_t)b8(in, at + q);
    for (uint32_t i = 0; i < rsz; i++) lit[i] = c;
    q += 1;
  } else {
    if (q + csz > n) return E_TRUNC;
    int64_t tsz = 0;
    if (lt == 2) { tsz = huf_tree(t, in, at + q, csz); if (tsz < 0) return E_DATA; }
    else if (!t.have_huf) return E_DATA;
    const uint32_t s0 = at + q + (uint32_t)tsz, ssz = csz - (uint32_t)tsz;
    if (ns == 1) {
      if (huf_stream(t, in, s0, ssz, lit, rsz)) return E_DATA;
    } else {
      if (ssz < 6) return E_DATA;
      const uint32_t l1 = b8(in, s0) | (b8(in, s0 + 1) << 8), l2 = b8(in, s0 + 2) | (b8(in, s0 + 3) << 8),
                     l3 = b8(in, s0 + 4) | (b8(in, s0 + 5) << 8);
      if (l1 + l2 + l3 + 6 > ssz) return E_DATA;
      const uint32_t l4 = ssz - 6 - l1 - l2 - l3;
      const uint32_t seg = (rsz + 3) / 4;
      if (rsz < 3 * seg) return E_DATA;
      const uint32_t p1 = s0 + 6;
      if (huf_stream(t, in, p1, l1, lit, seg) || huf_stream(t, in, p1 + l1, l2, lit + seg, seg) ||
          huf_stream(t, in, p1 + l1 + l2, l3, lit + 2 * seg, seg) ||
          huf_stream(t, in, p1 + l1 + l2 + l3, l4, lit + 3 * seg, rsz - 3 * seg))
        return E_DATA;
    }
    q += csz;
  }
  // sequences
  if (q >= n) return E_TRUNC;
  uint32_t nseq = b8(in, at + q++);
  if (nseq >= 128) {
    if (nseq < 255) { if (q >= n) return E_TRUNC; nseq = ((nseq - 128) << 8) + b8(in, at + q++); }
    else { if (q + 1 >= n) return E_TRUNC; nseq = b8(in, at + q) + (b8(in, at + q + 1) << 8) + 0x7F00; q += 2; }
  }
  uint32_t lp = 0;      // literals consumed
  if (nseq > 0) {
    if (q >= n) return E_TRUNC;
    const uint32_t modes = b8(in, at + q++);
    if (modes & 3) return E_DATA;
    int64_t u = seq_table(t, t.ll, t.ll_al, (modes >> 6) & 3, in, at + q, n - q, 0, 35, 9);
    if (u < 0) return E_DATA;
    q += (uint32_t)u;
    u = seq_table(t, t.of, t.of_al, (modes >> 4) & 3, in, at + q, n - q, 1, 31, 8);
    if (u < 0) return E_DATA;
    q += (uint32_t)u;
    u = seq_table(t, t.ml, t.ml_al, (modes >> 2) & 3, in, at + q, n - q, 2, 52, 9);
    if (u < 0) return E_DATA;
    q += (uint32_t)u;
    t.have_seq = 1;
    Bits b;
    if (bits_init(b, in, at + q, n - q)) return E_DATA;
    uint32_t sll = bits_read(b, t.ll_al), sof = bits_read(b, t.of_al), sml = bits_read(b, t.ml_al);
    for (uint32_t k = 0; k < nseq; k++) {
      const uint32_t llc = t.ll[sll].sym, ofc = t.of[sof].sym, mlc = t.ml[sml].sym;
      if (llc > 35 || mlc > 52 || ofc > 31) return E_DATA;
      const uint64_t ofv = (1ull << ofc) + bits_read(b, ofc);
      const uint32_t ml = ml_base(mlc) + bits_read(b, ml_bits(mlc));
      const uint32_t ll = ll_base(llc) + bits_read(b, ll_bits(llc));
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        t.rep[2] = t.rep[1]; t.rep[1] = t.rep[0]; t.rep[0] = (uint32_t)off;
      } else {
        const uint32_t idx = (uint32_t)ofv - 1u + (ll == 0 ? 1u : 0u);
        if (idx == 0) off = t.rep[0];
        else {
          off = idx == 3 ? (uint64_t)t.rep[0] - 1u : t.rep[idx];
          if (idx == 1) t.rep[1] = t.rep[0];
          else { t.rep[2] = t.rep[1]; t.rep[1] = t.rep[0]; }
          t.rep[0] = (uint32_t)off;
        }
      }
      if (k + 1 < nseq) {
        sll = t.ll[sll].base + bits_read(b, t.ll[sll].nb);
        sml = t.ml[sml].base + bits_read(b, t.ml[sml].nb);
        sof = t.of[sof].base + bits_read(b, t.of[sof].nb);
      }
      if (ll > rsz - lp) return E_DATA;
      // the block must still fit: then the copies never reach the unread literals
      // at the end of the span
      if ((uint64_t)op + ml + (rsz - lp) > cap) return E_SIZE;
      copy_fwd(dst + op, lit + lp, ll);          // forward: op <= lbase + lp
      op += ll; lp += ll;
      if (off == 0 || off > op) return E_DATA;
      copy_match(dst, op, (uint32_t)off, ml);
      op += ml;
    }
    if (b.pos != 0) return E_DATA;
  }
  const uint32_t rest = rsz - lp;
  if ((uint64_t)op + rest > cap) return E_SIZE;
  copy_fwd(dst + op, lit + lp, rest);
  return (int64_t)op + rest;
}

HZ_HD uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// XXH64 of the decoded split (the optional content checksum)
HZ_HD uint64_t xxh64(hz_gu8* p, uint32_t len) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                 P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  auto r64 = [&](uint32_t i) { uint64_t v = 0; for (int k = 7; k >= 0; k--) v = (v << 8) | p[i + k]; return v; };
  uint32_t i = 0;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= len; i += 32) {
      v1 = rotl(v1 + r64(i) * P2, 31) * P1;
      v2 = rotl(v2 + r64(i + 8) * P2, 31) * P1;
      v3 = rotl(v3 + r64(i + 16) * P2, 31) * P1;
      v4 = rotl(v4 + r64(i + 24) * P2, 31) * P1;
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = (h ^ (rotl(v1 * P2, 31) * P1)) * P1 + P4;
    h = (h ^ (rotl(v2 * P2, 31) * P1)) * P1 + P4;
    h = (h ^ (rotl(v3 * P2, 31) * P1)) * P1 + P4;
    h = (h ^ (rotl(v4 * P2, 31) * P1)) * P1 + P4;
  } else {
    h = P5;
  }
  h += len;
  for (; i + 8 <= len; i += 8) { h ^= rotl(r64(i) * P2, 31) * P1; h = rotl(h, 27) * P1 + P4; }
  if (i + 4 <= len) {
    const uint64_t v = (uint64_t)p[i] | (uint64_t)p[i + 1] << 8 | (uint64_t)p[i + 2] << 16 | (uint64_t)p[i + 3] << 24;
    h ^= v * P1; h = rotl(h, 23) * P2 + P3; i += 4;
  }
  for (; i < len; i++) { h ^= p[i] * P5; h = rotl(h, 11) * P1; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

// Decode one zstd frame (src, n) into exactly cap bytes at dst.  Returns OK or < 0.
HZ_HD int frame(Tables& t, const uint8_t* src, uint32_t n, uint8_t* dstp, uint32_t cap) {
  In in = {src, n};
  hz_gu8* dst = HZ_GLOBAL(hz_gu8*, dstp);
  if (n < 5) return E_TRUNC;
  if ((b8(in, 0) | b8(in, 1) << 8 | b8(in, 2) << 16 | b8(in, 3) << 24) != 0xFD2FB528u) return E_DATA;
  const uint32_t fhd = b8(in, 4);
  const uint32_t fcsf = fhd >> 6, single = (fhd >> 5) & 1u, cks = (fhd >> 2) & 1u, didf = fhd & 3u;
  if (fhd & 8u) return E_DATA;
  if (didf) return E_UNSUP;                  // dictionaries: never written by c-blosc
  uint32_t q = 5 + (single ? 0u : 1u);
  const uint32_t fcsb = fcsf == 0 ? (single ? 1u : 0u) : fcsf == 1 ? 2u : fcsf == 2 ? 4u : 8u;
  if (q + fcsb > n) return E_TRUNC;
  int64_t fcs = -1;
  if (fcsb) {
    uint64_t v = 0;
    for (int i = (int)fcsb - 1; i >= 0; i--) v = (v << 8) | b8(in, q + (uint32_t)i);
    fcs = (int64_t)(fcsb == 2 ? v + 256 : v);
  }
  q += fcsb;
  t.have_seq = 0; t.have_huf = 0;
  t.rep[0] = 1; t.rep[1] = 4; t.rep[2] = 8;
  uint32_t op = 0;
  for (;;) {
    if (q + 3 > n) return E_TRUNC;
    const uint32_t bh = b8(in, q) | (b8(in, q + 1) << 8) | (b8(in, q + 2) << 16);
    q += 3;
    const uint32_t last = bh & 1u, type = (bh >> 1) & 3u, bsz = bh >> 3;
    if (type == 3 || bsz > (1u << 17)) return E_DATA;
    if (type == 0) {
      if (q + bsz > n) return E_TRUNC;
      if (bsz > cap - op) return E_SIZE;
      for (uint32_t i = 0; i < bsz; i++) dst[op + i] = (uint8_t)b8(in, q + i);
      op += bsz; q += bsz;
    } else if (type == 1) {
      if (q + 1 > n) return E_TRUNC;
      if (bsz > cap - op) return E_SIZE;
      const uint8_t c = (uint8_t)b8(in, q);
      for (uint32_t i = 0; i < bsz; i++) dst[op + i] = c;
      op += bsz; q += 1;
    } else {
      if (q + bsz > n) return E_TRUNC;
      const int64_t o2 = block(t, in, q, bsz, dst, op, cap);
      if (o2 < 0) return (int)o2;
      op = (uint32_t)o2; q += bsz;
    }
    if (last) break;
  }
  if (fcs >= 0 && fcs != (int64_t)op) return E_SIZE;
  if (op != cap) return E_SIZE;
  if (cks) {
    if (q + 4 > n) return E_TRUNC;
    const uint32_t want = b8(in, q) | b8(in, q + 1) << 8 | b8(in, q + 2) << 16 | b8(in, q + 3) << 24;
    if ((uint32_t)xxh64(dst, op) != want) return E_DATA;
  }
  return OK;
}

}  // namespace zs
