/*
 * oracle.c -- CPU restatement of the HSDS data-node chunk codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (hsds_amd/) never links or calls it.
 *
 * What it restates (reference = /root/reference, HSDS 0.9.4):
 *   - _uncompress        hsds/util/storUtil.py:182-235   (orc_uncompress)
 *   - _compress          hsds/util/storUtil.py:238-281   (orc_blosc_encode_zlib)
 *   - _shuffle/_unshuffle (codec 1) storUtil.py:94-102,136-143 -> numcodecs.Shuffle
 *   - the Blosc1 frame codec that numcodecs vendors (c-blosc 1.21.x, third-party,
 *     not under /root/reference; pinned by numcodecs 0.12.1-0.15.1,
 *     requirements.txt:27 / pyproject.toml:46).  Frame rules were established
 *     against /opt/conda/lib/libblosc.so.1.21.0 (SURVEY.md section 8a row a3 and
 *     tests/golden/make_golden.py probes).
 *   - zlib inflate/deflate: the reference calls CPython zlib 1.2.11 and c-blosc's
 *     zlib_wrap_{compress,decompress}; this file calls the same system libz 1.2.11.
 *   - the other Blosc inner codecs the reference writes with cname = the dataset's
 *     compressor (storUtil.py:255-262): LZ4 block decode (lz4 1.9.x) and BloscLZ
 *     (c-blosc 1.21), restated from their published formats (orc_lz4_decode,
 *     orc_blosclz_decode), and zstd (orc_zstd_decode); snappy stays unsupported.
 *   - _unshuffle / _shuffle codec 2 (bitshuffle+LZ4 behind HSDS's 12-byte header,
 *     storUtil.py:103-131,144-174): orc_bitshuffle_decode / orc_bitshuffle_encode.
 *     bitshuffle 0.5.2 (requirements.txt:11) is absent; its bit transposition is
 *     pinned by tests/golden/bitshuffle_cases (imagecodecs' bitshuffle 0.3.5 core).
 *
 * Parity pinning: tests/test_oracle_golden.py checks every function here against the
 * golden vectors in tests/golden/ that were produced by the reference's own
 * storUtil._compress/_uncompress (run through tests/golden/refshim.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* status codes shared with include/hsds_amd.h */
#define ORC_OK 0
#define ORC_ERR_FRAME -1      /* malformed Blosc frame                       */
#define ORC_ERR_DATA -2       /* corrupt deflate stream / adler32 mismatch   */
#define ORC_ERR_TRUNC -3      /* stream ended before its end-of-stream       */
#define ORC_ERR_SIZE -4       /* output larger / smaller than expected       */
#define ORC_ERR_UNSUPPORTED -5/* other Blosc codec, bitshuffle, ...          */
#define ORC_ERR_ARG -6

static uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void wr32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* ---- byte shuffle (HDF5 / numcodecs Shuffle / c-blosc generic) ------------- */

/* numcodecs Shuffle(n).encode: out[b*count + i] = in[i*n + b]; trailing
 * (len % n) bytes are copied unchanged (c-blosc shuffle_generic does the same). */
void orc_shuffle(const uint8_t *src, int64_t len, int n, uint8_t *dst) {
  if (n <= 1) { memcpy(dst, src, (size_t)len); return; }
  int64_t count = len / n;
  for (int64_t i = 0; i < count; i++)
    for (int b = 0; b < n; b++) dst[(int64_t)b * count + i] = src[i * n + b];
  int64_t rem = len - count * n;
  if (rem) memcpy(dst + len - rem, src + len - rem, (size_t)rem);
}

/* numcodecs Shuffle(n).decode: out[i*n + b] = in[b*count + i] */
void orc_unshuffle(const uint8_t *src, int64_t len, int n, uint8_t *dst) {
  if (n <= 1) { memcpy(dst, src, (size_t)len); return; }
  int64_t count = len / n;
  for (int b = 0; b < n; b++)
    for (int64_t i = 0; i < count; i++) dst[i * n + b] = src[(int64_t)b * count + i];
  int64_t rem = len - count * n;
  if (rem) memcpy(dst + len - rem, src + len - rem, (size_t)rem);
}

/* ---- zlib (RFC 1950) stream decode ------------------------------------------
 * Mirrors CPython zlib.decompress (storUtil.py:214) for the F2 path and c-blosc's
 * zlib_wrap_decompress (libz uncompress) for Blosc splits: the stream must reach
 * Z_STREAM_END, adler32 is verified by libz, bytes after the stream are ignored.
 * Returns decoded length, or ORC_ERR_SIZE when the stream needs more than cap. */
int64_t orc_zlib_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t cap) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit(&zs) != Z_OK) return ORC_ERR_ARG;
  zs.next_in = (Bytef *)src;
  zs.avail_in = (uInt)srclen;
  zs.next_out = dst;
  zs.avail_out = (uInt)cap;
  int rc = inflate(&zs, Z_FINISH);
  int64_t out = (int64_t)zs.total_out;
  int64_t left_in = zs.avail_in;
  inflateEnd(&zs);
  if (rc == Z_STREAM_END) return out;
  if (rc == Z_DATA_ERROR || rc == Z_NEED_DICT || rc == Z_STREAM_ERROR || rc == Z_MEM_ERROR)
    return ORC_ERR_DATA;
  /* Z_BUF_ERROR: either out of output space or out of input */
  if (zs.avail_out == 0 && left_in > 0) return ORC_ERR_SIZE;
  if (left_in == 0) return ORC_ERR_TRUNC;
  return ORC_ERR_SIZE;
}

/* ---- LZ4 block decode (lz4 1.9.x LZ4_decompress_safe, third-party: the lz4 that
 * c-blosc 1.21 vendors and calls from lz4_wrap_decompress for codec 1, "lz4" and
 * "lz4hc").  Restated from the published block format: token (literal length high
 * nibble, match length - 4 low nibble, 15 = extended by bytes until one != 255),
 * literals, 16-bit little-endian offset, extended match length.  End-of-block rules of
 * the safe decoder: a literal run reaching oend - MFLIMIT(12) or iend - 8 must be the
 * last sequence and end exactly at iend; a match must end at least LASTLITERALS(5)
 * bytes before oend; offset 0 or an offset before the output start is corrupt.
 * Pinned by tests/golden/codec2_cases (frames written by libblosc 1.21.0's lz4).
 * Returns the decoded length or a negative status. */
int64_t orc_lz4_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  for (;;) {
    if (ip >= srclen) return ORC_ERR_TRUNC;
    unsigned t = src[ip++];
    int64_t lit = t >> 4;
    if (lit == 15) {
      unsigned b;
      do { if (ip >= srclen) return ORC_ERR_TRUNC; b = src[ip++]; lit += b; } while (b == 255);
    }
    if (lit > srclen - ip) return ORC_ERR_TRUNC;
    if (lit > cap - op) return ORC_ERR_SIZE;
    memcpy(dst + op, src + ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (op + 12 > cap || ip + 8 > srclen) {
      if (ip != srclen) return ORC_ERR_DATA;
      return op;
    }
    if (ip + 1 >= srclen) return ORC_ERR_TRUNC;
    int64_t off = src[ip] | (src[ip + 1] << 8);
    ip += 2;
    int64_t ml = t & 15;
    if (ml == 15) {
      unsigned b;
      do { if (ip >= srclen) return ORC_ERR_TRUNC; b = src[ip++]; ml += b; } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > op) return ORC_ERR_DATA;
    if (op + ml + 5 > cap) return ORC_ERR_DATA;
    for (int64_t k = 0; k < ml; k++) dst[op + k] = dst[op + k - off];   /* overlapping copy */
    op += ml;
  }
}

/* ---- BloscLZ decode (c-blosc 1.21 blosclz_decompress, third-party, in-tree in
 * c-blosc).  Control byte c (the first one masked to 5 bits): c < 32 -> c + 1 literal
 * bytes; else a match of (c >> 5) + 2 bytes (c >> 5 == 7: plus extension bytes until
 * one != 255), distance ((c & 31) << 8) + next byte + 1, or, when that byte is 255 and
 * c & 31 == 31, 8192 + a 16-bit big-endian distance.  The stream ends when the input
 * is exhausted after an item.  Pinned by tests/golden/codec2_cases (libblosc 1.21.0). */
int64_t orc_blosclz_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  if (srclen <= 0) return ORC_ERR_TRUNC;
  unsigned c = src[ip++] & 31u;
  for (;;) {
    if (c >= 32) {
      int64_t len = (c >> 5) - 1;
      int64_t dist = (int64_t)(c & 31u) << 8;
      unsigned code;
      if (len == 6) {
        do { if (ip >= srclen) return ORC_ERR_TRUNC; code = src[ip++]; len += code; } while (code == 255);
      }
      if (ip >= srclen) return ORC_ERR_TRUNC;
      code = src[ip++];
      len += 3;
      if (code == 255 && dist == (31 << 8)) {
        if (ip + 1 >= srclen) return ORC_ERR_TRUNC;
        dist = ((int64_t)src[ip] << 8 | src[ip + 1]) + 8192;
        ip += 2;
      } else {
        dist += code + 1;
      }
      if (len > cap - op) return ORC_ERR_SIZE;
      if (dist > op) return ORC_ERR_DATA;
      for (int64_t k = 0; k < len; k++) dst[op + k] = dst[op + k - dist];
      op += len;
    } else {
      int64_t n = (int64_t)c + 1;
      if (n > cap - op) return ORC_ERR_SIZE;
      if (n > srclen - ip) return ORC_ERR_TRUNC;
      memcpy(dst + op, src + ip, (size_t)n);
      op += n;
      ip += n;
    }
    if (ip >= srclen) return op;
    c = src[ip++];
  }
}

/* ---- Zstandard frame decode (RFC 8878; third-party: the zstd that c-blosc 1.21
 * vendors and calls from zstd_wrap_decompress for codec 4).  Restated from the RFC:
 * frame header, raw / RLE / compressed blocks, literals (raw, RLE, Huffman with 1 or
 * 4 streams, FSE-compressed or direct weights, treeless reuse), sequences (predefined,
 * RLE, FSE and repeat tables; three repeat offsets) and the optional XXH64 checksum.
 * Pinned by tests/golden/codec2_cases (zstd objects written by the reference's
 * _compress over libblosc 1.21.0).  Returns the decoded size or a negative status. */

typedef struct { uint8_t sym, nb; uint16_t base; } zfse_t;            /* FSE decode entry */
typedef struct { uint8_t sym, nb; } zhuf_t;                            /* Huffman decode entry */

/* backward bitstream (read from the last byte towards the first) */
typedef struct { const uint8_t *p; int64_t nbits; int64_t pos; } zbits_t;  /* pos: bits left */
static int zb_init(zbits_t *b, const uint8_t *p, int64_t n) {
  if (n <= 0 || p[n - 1] == 0) return -1;
  int hb = 7; while (!(p[n - 1] >> hb)) hb--;
  b->p = p; b->nbits = 8 * n; b->pos = 8 * (n - 1) + hb;   /* bits below the marker */
  return 0;
}
static uint64_t zb_read(zbits_t *b, int n) {   /* n <= 56; bits past the start read as 0 */
  uint64_t v = 0;
  for (int i = 0; i < n; i++) {
    b->pos--;
    int bit = 0;
    if (b->pos >= 0) bit = (b->p[b->pos >> 3] >> (b->pos & 7)) & 1;
    v = (v << 1) | (uint64_t)bit;
  }
  return v;
}
static int zb_overflow(const zbits_t *b) { return b->pos < 0; }

static int zhighbit(uint32_t v) { int r = 0; while (v >>= 1) r++; return r; }

/* FSE table description (NCount): returns bytes used, or -1 */
static int64_t z_ncount(const uint8_t *src, int64_t n, int16_t *norm, int *maxsym, int *al, int maxal) {
  if (n < 1) return -1;
  int64_t bitpos = 0;
#define ZRD(k) ({ uint32_t _v = 0; for (int _i = 0; _i < (k); _i++) { int64_t _q = bitpos + _i; \
    if ((_q >> 3) < n) _v |= (uint32_t)((src[_q >> 3] >> (_q & 7)) & 1) << _i; } _v; })
  int log = (int)ZRD(4) + 5;
  bitpos = 4;
  if (log > maxal) return -1;
  *al = log;
  int remaining = (1 << log) + 1, threshold = 1 << log, nbits = log + 1, s = 0, prev0 = 0;
  while (remaining > 1 && s <= *maxsym) {
    if (prev0) {
      int n0 = s;
      for (;;) {
        uint32_t r = ZRD(2); bitpos += 2;
        n0 += (int)r;
        if (r != 3) break;
      }
      if (n0 > *maxsym + 1) return -1;
      while (s < n0) norm[s++] = 0;
      if (s > *maxsym) break;
    }
    int maxv = (2 * threshold - 1) - remaining;
    int count;
    uint32_t low = ZRD(nbits - 1);
    if ((int)low < maxv) { count = (int)low; bitpos += nbits - 1; }
    else {
      count = (int)ZRD(nbits);
      if (count >= threshold) count -= maxv;
      bitpos += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[s++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) { nbits--; threshold >>= 1; }
  }
#undef ZRD
  if (remaining != 1) return -1;
  *maxsym = s - 1;
  return (bitpos + 7) >> 3;
}

static int z_build_fse(zfse_t *t, const int16_t *norm, int maxsym, int al) {
  const int size = 1 << al;
  int high = size - 1;
  uint16_t next[256];
  for (int s = 0; s <= maxsym; s++) {
    if (norm[s] == -1) { t[high--].sym = (uint8_t)s; next[s] = 1; }
    else next[s] = (uint16_t)norm[s];
  }
  const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  int pos = 0;
  for (int s = 0; s <= maxsym; s++) {
    for (int i = 0; i < norm[s]; i++) {
      t[pos].sym = (uint8_t)s;
      do pos = (pos + step) & mask; while (pos > high);
    }
  }
  if (pos != 0) return -1;
  for (int u = 0; u < size; u++) {
    const int s = t[u].sym;
    const uint32_t ns = next[s]++;
    const int nb = al - zhighbit(ns);
    t[u].nb = (uint8_t)nb;
    t[u].base = (uint16_t)((ns << nb) - size);
  }
  return 0;
}

static const int16_t z_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t z_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t z_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t z_ll_base[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40,
                                       48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t z_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                                      4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t z_ml_base[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26,
                                       27, 28, 29, 30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259,
                                       515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t z_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

typedef struct {
  zfse_t ll[512], of[256], ml[512];
  int ll_al, of_al, ml_al, have_tables;
  zhuf_t huf[1 << 11];
  int huf_bits, have_huf;
  uint32_t rep[3];
} zstate_t;

/* one of LL / OF / ML: mode 0 predefined, 1 RLE, 2 FSE, 3 repeat; returns bytes used */
static int64_t z_table(zfse_t *t, int *al, int mode, const uint8_t *p, int64_t n, const int16_t *def, int defmax,
                       int defal, int maxsym, int maxal, int have) {
  int16_t norm[256];
  if (mode == 0) { memcpy(norm, def, sizeof(int16_t) * (defmax + 1)); *al = defal; return z_build_fse(t, norm, defmax, defal) ? -1 : 0; }
  if (mode == 1) {
    if (n < 1 || p[0] > maxsym) return -1;
    t[0].sym = p[0]; t[0].nb = 0; t[0].base = 0; *al = 0;
    return 1;
  }
  if (mode == 2) {
    int ms = maxsym, l;
    int64_t used = z_ncount(p, n, norm, &ms, &l, maxal);
    if (used < 0 || z_build_fse(t, norm, ms, l)) return -1;
    *al = l;
    return used;
  }
  return have ? 0 : -1;
}

/* Huffman tree description; returns bytes used */
static int64_t z_huf_tree(zstate_t *z, const uint8_t *p, int64_t n) {
  uint8_t w[256];
  int nw = 0;
  if (n < 1) return -1;
  int64_t used;
  if (p[0] >= 128) {
    nw = p[0] - 127;
    used = 1 + (nw + 1) / 2;
    if (used > n) return -1;
    for (int i = 0; i < nw; i++) w[i] = (i & 1) ? (p[1 + i / 2] & 15) : (p[1 + i / 2] >> 4);
  } else {
    const int64_t cs = p[0];
    used = 1 + cs;
    if (used > n || cs < 1) return -1;
    int16_t norm[256];
    int ms = 255, al;
    int64_t u = z_ncount(p + 1, cs, norm, &ms, &al, 6);
    if (u < 0) return -1;
    zfse_t t[64];
    if (z_build_fse(t, norm, ms, al)) return -1;
    zbits_t b;
    if (zb_init(&b, p + 1 + u, cs - u)) return -1;
    uint32_t s1 = (uint32_t)zb_read(&b, al), s2 = (uint32_t)zb_read(&b, al);
    for (;;) {
      if (nw >= 255) return -1;
      w[nw++] = t[s1].sym;
      s1 = t[s1].base + (uint32_t)zb_read(&b, t[s1].nb);
      if (zb_overflow(&b)) { w[nw++] = t[s2].sym; break; }
      if (nw >= 255) return -1;
      w[nw++] = t[s2].sym;
      s2 = t[s2].base + (uint32_t)zb_read(&b, t[s2].nb);
      if (zb_overflow(&b)) { if (nw >= 255) return -1; w[nw++] = t[s1].sym; break; }
    }
  }
  /* last weight implied: the weight sum becomes a power of two */
  uint32_t total = 0;
  for (int i = 0; i < nw; i++) { if (w[i] > 11) return -1; if (w[i]) total += 1u << (w[i] - 1); }
  if (total == 0) return -1;
  const int maxb = zhighbit(total) + 1;
  const uint32_t rest = (1u << maxb) - total;
  if (rest & (rest - 1)) return -1;
  w[nw++] = (uint8_t)(zhighbit(rest) + 1);
  if (maxb > 11) return -1;
  /* decode table: weights ascending, symbols in order inside a weight */
  uint32_t rank[13] = {0}, start[13];
  for (int i = 0; i < nw; i++) rank[w[i]]++;
  uint32_t nxt = 0;
  for (int k = 1; k <= maxb; k++) { start[k] = nxt; nxt += rank[k] << (k - 1); }
  for (int i = 0; i < nw; i++) {
    if (!w[i]) continue;
    const uint32_t len = 1u << (w[i] - 1);
    for (uint32_t u = start[w[i]]; u < start[w[i]] + len; u++) { z->huf[u].sym = (uint8_t)i; z->huf[u].nb = (uint8_t)(maxb + 1 - w[i]); }
    start[w[i]] += len;
  }
  z->huf_bits = maxb;
  z->have_huf = 1;
  return used;
}

static int z_huf_stream(const zstate_t *z, const uint8_t *p, int64_t n, uint8_t *out, int64_t cnt) {
  zbits_t b;
  if (zb_init(&b, p, n)) return -1;
  for (int64_t i = 0; i < cnt; i++) {
    const int64_t save = b.pos;
    const uint32_t peek = (uint32_t)zb_read(&b, z->huf_bits);
    const zhuf_t e = z->huf[peek];
    b.pos = save - e.nb;
    out[i] = e.sym;
  }
  return b.pos == 0 ? 0 : -1;   /* every bit consumed */
}

static uint64_t xxh_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t xxh_rd64(const uint8_t *p) { uint64_t v = 0; for (int i = 7; i >= 0; i--) v = (v << 8) | p[i]; return v; }
static uint64_t orc_xxh64(const uint8_t *p, int64_t len) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                 P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  int64_t i = 0;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= len; i += 32) {
      v1 = xxh_rotl(v1 + xxh_rd64(p + i) * P2, 31) * P1;
      v2 = xxh_rotl(v2 + xxh_rd64(p + i + 8) * P2, 31) * P1;
      v3 = xxh_rotl(v3 + xxh_rd64(p + i + 16) * P2, 31) * P1;
      v4 = xxh_rotl(v4 + xxh_rd64(p + i + 24) * P2, 31) * P1;
    }
    h = xxh_rotl(v1, 1) + xxh_rotl(v2, 7) + xxh_rotl(v3, 12) + xxh_rotl(v4, 18);
    uint64_t vs[4] = {v1, v2, v3, v4};
    for (int k = 0; k < 4; k++) { h ^= xxh_rotl(vs[k] * P2, 31) * P1; h = h * P1 + P4; }
  } else {
    h = P5;
  }
  h += (uint64_t)len;
  for (; i + 8 <= len; i += 8) { h ^= xxh_rotl(xxh_rd64(p + i) * P2, 31) * P1; h = xxh_rotl(h, 27) * P1 + P4; }
  if (i + 4 <= len) {
    uint64_t v = (uint64_t)p[i] | (uint64_t)p[i + 1] << 8 | (uint64_t)p[i + 2] << 16 | (uint64_t)p[i + 3] << 24;
    h ^= v * P1; h = xxh_rotl(h, 23) * P2 + P3; i += 4;
  }
  for (; i < len; i++) { h ^= p[i] * P5; h = xxh_rotl(h, 11) * P1; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

static int64_t z_block(zstate_t *z, const uint8_t *p, int64_t n, uint8_t *dst, int64_t op, int64_t cap,
                       uint8_t *lit) {
  /* ---- literals section ---- */
  if (n < 1) return ORC_ERR_DATA;
  const int lt = p[0] & 3, sf = (p[0] >> 2) & 3;
  int64_t rsz, csz = 0, hl;
  int nstreams = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { rsz = p[0] >> 3; hl = 1; }
    else if (sf == 1) { if (n < 2) return ORC_ERR_DATA; rsz = (p[0] >> 4) | (p[1] << 4); hl = 2; }
    else { if (n < 3) return ORC_ERR_DATA; rsz = (p[0] >> 4) | (p[1] << 4) | ((int64_t)p[2] << 12); hl = 3; }
  } else {
    hl = sf < 2 ? 3 : sf == 2 ? 4 : 5;
    if (n < hl) return ORC_ERR_DATA;
    uint64_t v = 0;
    for (int i = (int)hl - 1; i >= 0; i--) v = (v << 8) | p[i];
    const int bits = sf < 2 ? 10 : sf == 2 ? 14 : 18;
    rsz = (int64_t)((v >> 4) & ((1u << bits) - 1));
    csz = (int64_t)((v >> (4 + bits)) & ((1u << bits) - 1));
    nstreams = sf == 0 ? 1 : 4;
  }
  if (rsz > (1 << 17)) return ORC_ERR_DATA;
  int64_t q = hl;
  if (lt == 0) { if (q + rsz > n) return ORC_ERR_TRUNC; memcpy(lit, p + q, (size_t)rsz); q += rsz; }
  else if (lt == 1) { if (q + 1 > n) return ORC_ERR_TRUNC; memset(lit, p[q], (size_t)rsz); q += 1; }
  else {
    if (q + csz > n) return ORC_ERR_TRUNC;
    const uint8_t *h = p + q;
    int64_t tsz = 0;
    if (lt == 2) { tsz = z_huf_tree(z, h, csz); if (tsz < 0) return ORC_ERR_DATA; }
    else if (!z->have_huf) return ORC_ERR_DATA;
    const uint8_t *s = h + tsz;
    const int64_t ssz = csz - tsz;
    if (nstreams == 1) {
      if (z_huf_stream(z, s, ssz, lit, rsz)) return ORC_ERR_DATA;
    } else {
      if (ssz < 6) return ORC_ERR_DATA;
      const int64_t l1 = s[0] | (s[1] << 8), l2 = s[2] | (s[3] << 8), l3 = s[4] | (s[5] << 8);
      const int64_t l4 = ssz - 6 - l1 - l2 - l3;
      if (l4 < 0) return ORC_ERR_DATA;
      const int64_t seg = (rsz + 3) / 4;
      if (rsz < 3 * seg) return ORC_ERR_DATA;
      const uint8_t *s1 = s + 6;
      if (z_huf_stream(z, s1, l1, lit, seg) || z_huf_stream(z, s1 + l1, l2, lit + seg, seg) ||
          z_huf_stream(z, s1 + l1 + l2, l3, lit + 2 * seg, seg) ||
          z_huf_stream(z, s1 + l1 + l2 + l3, l4, lit + 3 * seg, rsz - 3 * seg))
        return ORC_ERR_DATA;
    }
    q += csz;
  }
  /* ---- sequences section ---- */
  if (q >= n) return ORC_ERR_TRUNC;
  int64_t nseq = p[q++];
  if (nseq >= 128) {
    if (nseq < 255) { if (q >= n) return ORC_ERR_TRUNC; nseq = ((nseq - 128) << 8) + p[q++]; }
    else { if (q + 1 >= n) return ORC_ERR_TRUNC; nseq = p[q] + (p[q + 1] << 8) + 0x7F00; q += 2; }
  }
  int64_t lp = 0;
  if (nseq > 0) {
    if (q >= n) return ORC_ERR_TRUNC;
    const int modes = p[q++];
    if (modes & 3) return ORC_ERR_DATA;
    int64_t u;
    u = z_table(z->ll, &z->ll_al, (modes >> 6) & 3, p + q, n - q, z_ll_def, 35, 6, 35, 9, z->have_tables);
    if (u < 0) return ORC_ERR_DATA;
    q += u;
    u = z_table(z->of, &z->of_al, (modes >> 4) & 3, p + q, n - q, z_of_def, 28, 5, 31, 8, z->have_tables);
    if (u < 0) return ORC_ERR_DATA;
    q += u;
    u = z_table(z->ml, &z->ml_al, (modes >> 2) & 3, p + q, n - q, z_ml_def, 52, 6, 52, 9, z->have_tables);
    if (u < 0) return ORC_ERR_DATA;
    q += u;
    z->have_tables = 1;
    zbits_t b;
    if (zb_init(&b, p + q, n - q)) return ORC_ERR_DATA;
    uint32_t sll = (uint32_t)zb_read(&b, z->ll_al), sof = (uint32_t)zb_read(&b, z->of_al),
             sml = (uint32_t)zb_read(&b, z->ml_al);
    for (int64_t k = 0; k < nseq; k++) {
      const int llc = z->ll[sll].sym, ofc = z->of[sof].sym, mlc = z->ml[sml].sym;
      if (llc > 35 || mlc > 52 || ofc > 31) return ORC_ERR_DATA;
      const uint64_t ofv = (1ull << ofc) + zb_read(&b, ofc);
      const uint64_t ml = z_ml_base[mlc] + zb_read(&b, z_ml_bits[mlc]);
      const uint64_t ll = z_ll_base[llc] + zb_read(&b, z_ll_bits[llc]);
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; z->rep[0] = (uint32_t)off;
      } else {
        const int idx = (int)ofv - 1 + (ll == 0);   /* LL == 0 shifts the repeat index by one */
        if (idx == 0) off = z->rep[0];
        else {
          off = idx == 3 ? (uint64_t)z->rep[0] - 1 : z->rep[idx];
          if (idx == 1) { z->rep[1] = z->rep[0]; }
          else { z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; }
          z->rep[0] = (uint32_t)off;
        }
      }
      if (k + 1 < nseq) {
        sll = z->ll[sll].base + (uint32_t)zb_read(&b, z->ll[sll].nb);
        sml = z->ml[sml].base + (uint32_t)zb_read(&b, z->ml[sml].nb);
        sof = z->of[sof].base + (uint32_t)zb_read(&b, z->of[sof].nb);
      }
      if (lp + (int64_t)ll > rsz) return ORC_ERR_DATA;
      if (op + (int64_t)ll + (int64_t)ml > cap) return ORC_ERR_SIZE;
      memcpy(dst + op, lit + lp, (size_t)ll);
      op += (int64_t)ll; lp += (int64_t)ll;
      if (off == 0 || (int64_t)off > op) return ORC_ERR_DATA;
      for (uint64_t i = 0; i < ml; i++) dst[op + (int64_t)i] = dst[op + (int64_t)i - (int64_t)off];
      op += (int64_t)ml;
    }
    if (b.pos != 0) return ORC_ERR_DATA;
  }
  if (op + (rsz - lp) > cap) return ORC_ERR_SIZE;
  memcpy(dst + op, lit + lp, (size_t)(rsz - lp));
  return op + (rsz - lp);
}

int64_t orc_zstd_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t cap) {
  if (srclen < 5) return ORC_ERR_TRUNC;
  if (rd32(src) != 0xFD2FB528u) return ORC_ERR_DATA;
  const int fhd = src[4];
  const int fcsf = fhd >> 6, single = (fhd >> 5) & 1, cks = (fhd >> 2) & 1, didf = fhd & 3;
  if (fhd & 8) return ORC_ERR_DATA;
  int64_t q = 5 + (single ? 0 : 1);
  q += didf == 0 ? 0 : didf == 1 ? 1 : didf == 2 ? 2 : 4;
  if (didf) return ORC_ERR_UNSUPPORTED;                     /* dictionaries: not used by c-blosc */
  const int fcsb = fcsf == 0 ? (single ? 1 : 0) : fcsf == 1 ? 2 : fcsf == 2 ? 4 : 8;
  if (q + fcsb > srclen) return ORC_ERR_TRUNC;
  int64_t fcs = -1;
  if (fcsb) {
    uint64_t v = 0;
    for (int i = fcsb - 1; i >= 0; i--) v = (v << 8) | src[q + i];
    fcs = (int64_t)(fcsb == 2 ? v + 256 : v);
  }
  q += fcsb;
  zstate_t *z = (zstate_t *)calloc(1, sizeof(zstate_t));
  uint8_t *lit = (uint8_t *)malloc(1 << 17);
  z->rep[0] = 1; z->rep[1] = 4; z->rep[2] = 8;
  int64_t op = 0, r = 0;
  for (;;) {
    if (q + 3 > srclen) { r = ORC_ERR_TRUNC; break; }
    const uint32_t bh = src[q] | (src[q + 1] << 8) | (src[q + 2] << 16);
    q += 3;
    const int last = bh & 1, type = (bh >> 1) & 3;
    const int64_t bsz = bh >> 3;
    if (type == 3 || bsz > (1 << 17)) { r = ORC_ERR_DATA; break; }
    if (type == 0) {
      if (q + bsz > srclen) { r = ORC_ERR_TRUNC; break; }
      if (op + bsz > cap) { r = ORC_ERR_SIZE; break; }
      memcpy(dst + op, src + q, (size_t)bsz); op += bsz; q += bsz;
    } else if (type == 1) {
      if (q + 1 > srclen) { r = ORC_ERR_TRUNC; break; }
      if (op + bsz > cap) { r = ORC_ERR_SIZE; break; }
      memset(dst + op, src[q], (size_t)bsz); op += bsz; q += 1;
    } else {
      if (q + bsz > srclen) { r = ORC_ERR_TRUNC; break; }
      const int64_t o2 = z_block(z, src + q, bsz, dst, op, cap, lit);
      if (o2 < 0) { r = o2; break; }
      op = o2; q += bsz;
    }
    if (last) break;
  }
  if (r == 0 && fcs >= 0 && fcs != op) r = ORC_ERR_SIZE;
  if (r == 0 && cks) {
    if (q + 4 > srclen) r = ORC_ERR_TRUNC;
    else if ((uint32_t)orc_xxh64(dst, op) != rd32(src + q)) r = ORC_ERR_DATA;
  }
  free(lit);
  free(z);
  return r < 0 ? r : op;
}

/* ---- Blosc1 frame decode (c-blosc 1.21 blosc_decompress semantics) --------- */

int orc_is_blosc(const uint8_t *src, int64_t srclen) {
  /* numcodecs.blosc.cbuffer_metainfo(data)[0] > 0  (storUtil.py:195-196):
   * c-blosc reports typesize 0 when the version byte is > 2 (BLOSC_VERSION_FORMAT). */
  if (srclen < 4) return 0;
  if (src[0] > 2) return 0;
  return src[3] > 0;
}

/* nsplits rule established against libblosc 1.21.0: split into `typesize` streams
 * only if the frame does not carry 0x10 (dont-split), typesize <= 16
 * (MAX_SPLITS), blocksize/typesize >= 128 (MIN_BUFFERSIZE) and the block is not
 * the trailing leftover block. */
static int blosc_nsplits(int flags, int ts, int64_t blocksize, int leftover) {
  if (!(flags & 0x10) && ts <= 16 && blocksize / ts >= 128 && !leftover) return ts;
  return 1;
}

static void bshuf_untrans(const uint8_t *in, uint8_t *out, int64_t n, int64_t es);

int64_t orc_blosc_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t dstcap) {
  if (srclen < 16) return ORC_ERR_FRAME;
  int ver = src[0], verlz = src[1], flags = src[2], ts = src[3];
  int64_t nbytes = rd32(src + 4), bs = rd32(src + 8), cbytes = rd32(src + 12);
  if (ver != 2) return ORC_ERR_FRAME;
  if (cbytes > srclen || cbytes < 16) return ORC_ERR_FRAME;
  if (nbytes > dstcap) return ORC_ERR_SIZE;
  if (flags & 0x02) { /* memcpyed */
    if (nbytes + 16 > cbytes) return ORC_ERR_FRAME;
    memcpy(dst, src + 16, (size_t)nbytes);
    return nbytes;
  }
  int codec = (flags >> 5) & 7;   /* 0 blosclz, 1 lz4/lz4hc, 3 zlib, 4 zstd; 2 snappy unsupported */
  if (codec != 3 && codec != 1 && codec != 0 && codec != 4) return ORC_ERR_UNSUPPORTED;
  if (verlz != 1) return ORC_ERR_FRAME;
  if (nbytes == 0) return 0;
  if (bs <= 0 || ts <= 0 || bs > nbytes) return ORC_ERR_FRAME;
  int64_t nblocks = (nbytes + bs - 1) / bs;
  int64_t leftover = nbytes % bs;
  int64_t hdr = 16 + 4 * nblocks;
  if (hdr > cbytes) return ORC_ERR_FRAME;
  /* c-blosc 1.21 blosc_d: byte unshuffle when 0x01 and typesize > 1, else bit unshuffle
   * when 0x04 (any typesize) -- bitunshuffle() of format version 2: the block's
   * bsz / ts elements are untransposed (bshuf_trans_bit_elem inverse) when their count
   * is a multiple of 8, otherwise the block stays as decoded; tail bytes past the last
   * whole element stay as decoded.  Pinned against libblosc 1.21.0
   * (tests/golden/make_blosc_bitshuffle_golden.py). */
  int doshuffle = (flags & 0x01) && ts > 1;
  int dobit = !doshuffle && (flags & 0x04);
  uint8_t *tmp = (doshuffle || dobit) ? (uint8_t *)malloc((size_t)bs) : NULL;
  int64_t result = nbytes;
  for (int64_t b = 0; b < nblocks; b++) {
    int isleft = (b == nblocks - 1) && leftover;
    int64_t bsz = isleft ? leftover : bs;
    int nspl = blosc_nsplits(flags, ts, bs, isleft);
    int64_t neblock = bsz / nspl;
    int64_t p = (int32_t)rd32(src + 16 + 4 * b);
    if (p < hdr || p >= cbytes) { result = ORC_ERR_FRAME; break; }
    uint8_t *out = (doshuffle || dobit) ? tmp : dst + b * bs;
    for (int j = 0; j < nspl; j++) {
      if (p + 4 > cbytes) { result = ORC_ERR_FRAME; goto done; }
      int64_t cs = (int32_t)rd32(src + p);
      p += 4;
      if (cs < 0 || p + cs > cbytes) { result = ORC_ERR_FRAME; goto done; }
      if (cs == neblock) {
        memcpy(out + j * neblock, src + p, (size_t)neblock);
      } else {
        int64_t r = codec == 3 ? orc_zlib_decode(src + p, cs, out + j * neblock, neblock)
                  : codec == 1 ? orc_lz4_decode(src + p, cs, out + j * neblock, neblock)
                  : codec == 4 ? orc_zstd_decode(src + p, cs, out + j * neblock, neblock)
                               : orc_blosclz_decode(src + p, cs, out + j * neblock, neblock);
        if (r < 0) { result = r == ORC_ERR_SIZE ? ORC_ERR_SIZE : r; goto done; }
        if (r != neblock) { result = ORC_ERR_SIZE; goto done; }
      }
      p += cs;
    }
    if (doshuffle) orc_unshuffle(tmp, bsz, ts, dst + b * bs);
    if (dobit) {
      const int64_t ne = bsz / ts;
      if (ne % 8 == 0) {
        bshuf_untrans(tmp, dst + b * bs, ne, ts);
        memcpy(dst + b * bs + ne * ts, tmp + ne * ts, (size_t)(bsz - ne * ts));
      } else {
        memcpy(dst + b * bs, tmp, (size_t)bsz);
      }
    }
  }
done:
  free(tmp);
  return result;
}

/* ---- _uncompress (storUtil.py:182-235) ------------------------------------
 * compressor: 0 = none / scaleoffset, 1 = gzip/deflate/zlib, 2 = another Blosc
 * codec name (decodable only as a Blosc frame).  shuffle: 0, 1 (byte), 2 (bit).
 * expected: the chunk byte size (prod(chunk_shape)*itemsize); output must match. */
int64_t orc_uncompress(const uint8_t *src, int64_t srclen, int compressor, int shuffle,
                       int itemsize, uint8_t *dst, int64_t expected) {
  int64_t n;
  uint8_t *stage = dst;
  int need_unshuffle = 0;
  if (compressor) {
    if (shuffle == 1 && itemsize > 1) {
      stage = (uint8_t *)malloc((size_t)(expected > 0 ? expected : 1));
    }
    if (orc_is_blosc(src, srclen)) {
      n = orc_blosc_decode(src, srclen, stage, expected);
      if (shuffle == 1) shuffle = 0; /* blosc unshuffles in-frame (storUtil.py:203-204) */
    } else if (compressor == 1) {
      n = orc_zlib_decode(src, srclen, stage, expected);
    } else {
      n = ORC_ERR_UNSUPPORTED;
    }
    if (n >= 0 && n != expected) n = ORC_ERR_SIZE;
    if (n < 0) { if (stage != dst) free(stage); return n; }
    need_unshuffle = shuffle;
  } else {
    if (srclen != expected) return ORC_ERR_SIZE;
    if (shuffle == 1 && itemsize > 1) {
      stage = (uint8_t *)malloc((size_t)(expected > 0 ? expected : 1));
    }
    memcpy(stage, src, (size_t)srclen);
    n = srclen;
    need_unshuffle = shuffle;
  }
  if (need_unshuffle == 2) { if (stage != dst) free(stage); return ORC_ERR_UNSUPPORTED; }
  if (need_unshuffle == 1 && itemsize > 1) {
    if (n % itemsize) { if (stage != dst) free(stage); return ORC_ERR_ARG; }
    orc_unshuffle(stage, n, itemsize, dst);
  } else if (stage != dst) {
    memcpy(dst, stage, (size_t)n);
  }
  if (stage != dst) free(stage);
  return n;
}

/* ---- Blosc1 zlib encode (c-blosc 1.21 blosc_compress_ctx semantics) --------
 * Restates compute_blocksize / split_block(FORWARD_COMPAT) / blosc_c /
 * serial_blosc / memcpyed fallback for the zlib codec, with libz compress2 per
 * split exactly as c-blosc's zlib_wrap_compress.  dst must hold nbytes + 16. */
static int split_ok(int ts, int64_t bs) { return ts <= 16 && bs / ts >= 128; }

/* c-blosc 1.21 compute_blocksize.  hcr: the high-compression-ratio codecs (zlib,
 * lz4hc, zstd) start from L1 x 2 and double again at level 9; lz4 / blosclz start
 * from L1 (32 KiB).  Pinned against libblosc 1.21.0 by the codec2 golden table. */
int64_t orc_blosc_blocksize_codec(int clevel, int ts, int64_t nbytes, int hcr) {
  if (nbytes < ts) return 1;
  int64_t bs = nbytes;
  if (nbytes >= 32 * 1024) {
    bs = hcr ? 32 * 1024 * 2 : 32 * 1024;
    switch (clevel) {
      case 0: bs /= 4; break;
      case 1: bs /= 2; break;
      case 2: break;
      case 3: bs *= 2; break;
      case 4: case 5: bs *= 4; break;
      case 6: case 7: case 8: bs *= 8; break;
      default: bs *= hcr ? 16 : 8; break; /* 9: x8, x2 for HCR codecs */
    }
  }
  if (clevel > 0 && split_ok(ts, bs)) {
    if (bs > (1 << 18)) bs = 1 << 18;
    bs *= ts;
    if (bs < (1 << 16)) bs = 1 << 16;
    if (bs > 1024 * 1024) bs = 1024 * 1024;
  }
  if (bs > nbytes) bs = nbytes;
  if (bs > ts) bs = bs / ts * ts;
  return bs;
}

int64_t orc_blosc_blocksize(int clevel, int ts, int64_t nbytes) { return orc_blosc_blocksize_codec(clevel, ts, nbytes, 1); }

/* Greedy LZ4 block writer (4-byte hash, distance <= 65535) obeying the block end
 * rules LZ4_decompress_safe checks: the last match starts at least MFLIMIT (12) bytes
 * before the end and ends at least LASTLITERALS (5) bytes before it.  Corpus writer
 * only: parity is judged on decoding, and any valid block decodes identically.
 * Returns the block size, or ORC_ERR_SIZE when it would exceed cap. */
int64_t orc_lz4_encode(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
  enum { HB = 14 };
  int32_t *ht = (int32_t *)calloc((size_t)1 << HB, sizeof(int32_t));
  int64_t ip = 0, anchor = 0, op = 0;
#define PUT(b) do { if (op >= cap) { free(ht); return ORC_ERR_SIZE; } dst[op++] = (uint8_t)(b); } while (0)
#define PUTLEN(v) do { int64_t _v = (v); while (_v >= 255) { PUT(255); _v -= 255; } PUT(_v); } while (0)
  while (n >= 13 && ip < n - 12) {
    uint32_t seq = rd32(src + ip);
    uint32_t h = (seq * 2654435761u) >> (32 - HB);
    int64_t ref = (int64_t)ht[h] - 1;
    ht[h] = (int32_t)(ip + 1);
    if (ref < 0 || ip - ref > 65535 || rd32(src + ref) != seq) { ip++; continue; }
    int64_t ml = 4;
    while (ip + ml < n - 5 && src[ref + ml] == src[ip + ml]) ml++;
    int64_t lit = ip - anchor;
    PUT(((lit < 15 ? lit : 15) << 4) | (ml - 4 < 15 ? ml - 4 : 15));
    if (lit >= 15) PUTLEN(lit - 15);
    if (op + lit > cap) { free(ht); return ORC_ERR_SIZE; }
    memcpy(dst + op, src + anchor, (size_t)lit);
    op += lit;
    PUT((ip - ref) & 0xff);
    PUT((ip - ref) >> 8);
    if (ml - 4 >= 15) PUTLEN(ml - 4 - 15);
    ip += ml;
    anchor = ip;
  }
  int64_t lit = n - anchor;
  PUT((lit < 15 ? lit : 15) << 4);
  if (lit >= 15) PUTLEN(lit - 15);
  if (op + lit > cap) { free(ht); return ORC_ERR_SIZE; }
  memcpy(dst + op, src + anchor, (size_t)lit);
  op += lit;
#undef PUT
#undef PUTLEN
  free(ht);
  return op;
}

static int64_t blosc_encode(int codec, const uint8_t *src, int64_t nbytes, int ts, int clevel, int64_t bs,
                            int doshuffle_flag, uint8_t *dst, int64_t dstcap) {
  if (ts < 1) ts = 1;
  if (ts > 255) ts = 1; /* c-blosc: typesize > BLOSC_MAX_TYPESIZE -> 1 */
  if (dstcap < nbytes + 16) return ORC_ERR_ARG;
  int64_t maxbytes = nbytes + 16;
  int flags = codec << 5;
  if (doshuffle_flag) flags |= 0x01;
  if (!split_ok(ts, bs)) flags |= 0x10;
  int memcpyed = (nbytes < 128) || clevel == 0;
  int64_t nblocks = bs > 0 ? (nbytes + bs - 1) / bs : 0;
  int64_t leftover = bs > 0 ? nbytes % bs : 0;
  dst[0] = 2; dst[1] = 1; dst[3] = (uint8_t)ts;
  wr32(dst + 4, (uint32_t)nbytes);
  wr32(dst + 8, (uint32_t)bs);
  int64_t ntbytes = 0;
  if (!memcpyed) {
    ntbytes = 16 + 4 * nblocks;
    if (ntbytes > maxbytes) ntbytes = 0;
    uint8_t *tmp = (uint8_t *)malloc((size_t)(bs > 0 ? bs : 1));
    for (int64_t b = 0; b < nblocks && ntbytes > 0; b++) {
      int isleft = (b == nblocks - 1) && leftover;
      int64_t bsz = isleft ? leftover : bs;
      wr32(dst + 16 + 4 * b, (uint32_t)ntbytes);
      const uint8_t *blk = src + b * bs;
      if ((flags & 0x01) && ts > 1) { orc_shuffle(blk, bsz, ts, tmp); blk = tmp; }
      int nspl = (!(flags & 0x10) && !isleft) ? ts : 1;
      int64_t neblock = bsz / nspl;
      for (int j = 0; j < nspl; j++) {
        ntbytes += 4;
        int64_t maxout = neblock;
        if (ntbytes + maxout > maxbytes) {
          maxout = maxbytes - ntbytes;
          if (maxout <= 0) { ntbytes = 0; break; }
        }
        int64_t cb = 0;
        if (codec == 3) {
          uLongf cl = (uLongf)maxout;
          if (compress2(dst + ntbytes, &cl, blk + j * neblock, (uLong)neblock, clevel) == Z_OK) cb = (int64_t)cl;
        } else {
          cb = orc_lz4_encode(blk + j * neblock, neblock, dst + ntbytes, maxout);
          if (cb < 0 || cb >= neblock) cb = 0;
        }
        if (cb == 0 || cb == neblock) {
          if (ntbytes + neblock > maxbytes) { ntbytes = 0; break; }
          memcpy(dst + ntbytes, blk + j * neblock, (size_t)neblock);
          cb = neblock;
        }
        wr32(dst + ntbytes - 4, (uint32_t)cb);
        ntbytes += cb;
      }
    }
    free(tmp);
    if (ntbytes == 0) memcpyed = 1;
  }
  if (memcpyed) {
    flags |= 0x02;
    memcpy(dst + 16, src, (size_t)nbytes);
    ntbytes = nbytes + 16;
  }
  dst[2] = (uint8_t)flags;
  wr32(dst + 12, (uint32_t)ntbytes);
  return ntbytes;
}


int64_t orc_blosc_encode_zlib(const uint8_t *src, int64_t nbytes, int ts, int clevel,
                              int doshuffle_flag, uint8_t *dst, int64_t dstcap) {
  if (ts < 1 || ts > 255) ts = 1;
  return blosc_encode(3, src, nbytes, ts, clevel, orc_blosc_blocksize(clevel, ts, nbytes), doshuffle_flag,
                      dst, dstcap);
}

/* Blosc1 frame with LZ4 splits (codec 1) at an explicit blocksize: the corpus writer for
 * lz4 tests and the bench (its payload bytes differ from lz4's own compressor; every
 * valid LZ4 block decodes the same way, and the frame layout follows c-blosc 1.21). */
int64_t orc_blosc_encode_lz4(const uint8_t *src, int64_t nbytes, int ts, int64_t bs, int doshuffle_flag,
                             uint8_t *dst, int64_t dstcap) {
  if (ts < 1 || ts > 255) ts = 1;
  if (bs <= 0 || bs > nbytes) bs = nbytes;
  return blosc_encode(1, src, nbytes, ts, 5, bs, doshuffle_flag, dst, dstcap);
}

/* zlib.compress(data, level) equivalent (the F2 stream producer for fixtures) */
int64_t orc_zlib_encode(const uint8_t *src, int64_t n, int level, uint8_t *dst, int64_t cap) {
  uLongf cl = (uLongf)cap;
  if (compress2(dst, &cl, src, (uLong)n, level) != Z_OK) return ORC_ERR_SIZE;
  return (int64_t)cl;
}

uint32_t orc_adler32(const uint8_t *p, int64_t n) {
  return (uint32_t)adler32(adler32(0L, Z_NULL, 0), p, (uInt)n);
}

/* ---- threaded batch helpers (bench cpu_baseline / corpus generation) ------- */

typedef struct {
  int op; /* 0 uncompress, 1 blosc encode, 2 zlib encode */
  const uint8_t *const *src;
  const int64_t *srclen;
  uint8_t *const *dst;
  const int64_t *dstlen;
  int64_t *status;
  int64_t n;
  int compressor, shuffle, itemsize, clevel;
  volatile int64_t next;
} orc_batch_t;

static void *batch_worker(void *arg) {
  orc_batch_t *b = (orc_batch_t *)arg;
  for (;;) {
    int64_t i = __sync_fetch_and_add(&b->next, 1);
    if (i >= b->n) break;
    if (b->op == 0)
      b->status[i] = orc_uncompress(b->src[i], b->srclen[i], b->compressor, b->shuffle,
                                    b->itemsize, b->dst[i], b->dstlen[i]);
    else if (b->op == 1)
      b->status[i] = orc_blosc_encode_zlib(b->src[i], b->srclen[i], b->itemsize, b->clevel,
                                           b->shuffle, b->dst[i], b->dstlen[i]);
    else
      b->status[i] = orc_zlib_encode(b->src[i], b->srclen[i], b->clevel, b->dst[i], b->dstlen[i]);
  }
  return NULL;
}

static void run_batch(orc_batch_t *b, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, b);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orc_uncompress_batch(const uint8_t *const *src, const int64_t *srclen, uint8_t *const *dst,
                          const int64_t *expected, int64_t n, int compressor, int shuffle,
                          int itemsize, int nthreads, int64_t *status) {
  orc_batch_t b = {0, src, srclen, dst, expected, status, n, compressor, shuffle, itemsize, 0, 0};
  run_batch(&b, nthreads);
}

void orc_encode_batch(int op, const uint8_t *const *src, const int64_t *srclen, uint8_t *const *dst,
                      const int64_t *dstcap, int64_t n, int typesize, int clevel, int doshuffle,
                      int nthreads, int64_t *status) {
  orc_batch_t b = {op, src, srclen, dst, dstcap, status, n, 0, doshuffle, typesize, clevel, 0};
  run_batch(&b, nthreads);
}


/* ---- bitshuffle + LZ4 (shuffle = 2) ------------------------------------------------
 * HSDS frame (storUtil._shuffle, storUtil.py:103-131): u64 BE chunk bytes, u32 BE
 * block_size * itemsize, then bitshuffle.compress_lz4: per block of block_size
 * elements a u32 BE LZ4 block size and the LZ4 block of the block's bit transposition
 * (bshuf_trans_bit_elem); a last block of the remaining elements rounded down to a
 * multiple of 8; the n % 8 leftover elements raw.  Bit transposition of n elements
 * (n % 8 == 0) of es bytes: row r = 8 j + k holds bit k of byte j of every element,
 * element i at bit i % 8 of row byte i / 8.
 */
#define BSHUF_ERR ORC_ERR_DATA

static int64_t bshuf_default_block(int64_t es) {     /* bshuf_default_block_size */
  int64_t bs = (8192 / es) / 8 * 8;
  return bs < 128 ? 128 : bs;
}

static void bshuf_trans(const uint8_t *in, uint8_t *out, int64_t n, int64_t es) {
  const int64_t row = n / 8;
  memset(out, 0, (size_t)(n * es));
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = 0; j < es; j++) {
      const uint8_t b = in[i * es + j];
      for (int k = 0; k < 8; k++)
        out[(j * 8 + k) * row + i / 8] |= (uint8_t)(((b >> k) & 1) << (i % 8));
    }
}

static void bshuf_untrans(const uint8_t *in, uint8_t *out, int64_t n, int64_t es) {
  const int64_t row = n / 8;
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = 0; j < es; j++) {
      uint8_t b = 0;
      for (int k = 0; k < 8; k++) b |= (uint8_t)(((in[(j * 8 + k) * row + i / 8] >> (i % 8)) & 1) << k);
      out[i * es + j] = b;
    }
}

static uint32_t rd32be(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

/* storUtil._unshuffle(codec=2) (storUtil.py:144-174) + bitshuffle.decompress_lz4:
 * returns chunk_bytes or an error (each error is HTTPInternalServerError there). */
int64_t orc_bitshuffle_decode(const uint8_t *src, int64_t srclen, uint8_t *dst, int64_t chunk_bytes, int64_t es) {
  if (srclen < 12 || es < 1 || chunk_bytes < 0 || chunk_bytes % es) return ORC_ERR_FRAME;    /* :148-152 */
  uint64_t total = 0;
  for (int i = 0; i < 8; i++) total = total << 8 | src[i];
  if (total != (uint64_t)chunk_bytes) return ORC_ERR_SIZE;                                 /* :160-164 */
  int64_t bs = (int64_t)rd32be(src + 8) / es;                                              /* :167 */
  if (bs == 0) bs = bshuf_default_block(es);
  if (bs % 8) return ORC_ERR_FRAME;                           /* bshuf: block size not a multiple of 8 */
  const int64_t n = chunk_bytes / es;
  uint8_t *tmp = (uint8_t *)malloc((size_t)(bs * es) + 1);
  int64_t p = 12, e = 0;
  int64_t rc = chunk_bytes;
  while (e + 8 <= n && rc >= 0) {
    int64_t cnt = n - e >= bs ? bs : (n - e) / 8 * 8;
    if (p + 4 > srclen) { rc = ORC_ERR_TRUNC; break; }
    const int64_t nb = (int64_t)rd32be(src + p);
    p += 4;
    if (nb > srclen - p) { rc = ORC_ERR_TRUNC; break; }
    const int64_t r = orc_lz4_decode(src + p, nb, tmp, cnt * es);
    if (r != cnt * es) { rc = r < 0 ? r : ORC_ERR_SIZE; break; }
    bshuf_untrans(tmp, dst + e * es, cnt, es);
    p += nb;
    e += cnt;
  }
  free(tmp);
  if (rc < 0) return rc;
  const int64_t left = (n - e) * es;                          /* n % 8 elements, raw */
  if (p + left > srclen) return ORC_ERR_TRUNC;
  memcpy(dst + e * es, src + p, (size_t)left);
  p += left;
  if (p != srclen) return ORC_ERR_SIZE;                       /* decompress_lz4: consumed != input */
  return chunk_bytes;
}

/* storUtil._shuffle(codec=2) with the oracle's greedy LZ4 writer (the LZ4 bytes differ
 * from liblz4's; any LZ4 decoder reads both).  Returns the frame size or an error. */
int64_t orc_bitshuffle_encode(const uint8_t *src, int64_t nbytes, int64_t es, int64_t block, uint8_t *dst,
                              int64_t cap) {
  if (es < 1 || nbytes % es || block < 0 || block % 8 || cap < 12) return ORC_ERR_FRAME;
  const int64_t bs = block ? block : bshuf_default_block(es), n = nbytes / es;
  for (int i = 0; i < 8; i++) dst[i] = (uint8_t)((uint64_t)nbytes >> (56 - 8 * i));
  const uint32_t bn = (uint32_t)(block * es);
  dst[8] = (uint8_t)(bn >> 24); dst[9] = (uint8_t)(bn >> 16); dst[10] = (uint8_t)(bn >> 8); dst[11] = (uint8_t)bn;
  uint8_t *tmp = (uint8_t *)malloc((size_t)(bs * es) + 1);
  int64_t p = 12, e = 0, rc = 0;
  while (e + 8 <= n) {
    const int64_t cnt = n - e >= bs ? bs : (n - e) / 8 * 8;
    bshuf_trans(src + e * es, tmp, cnt, es);
    if (p + 4 > cap) { rc = ORC_ERR_SIZE; break; }
    const int64_t c = orc_lz4_encode(tmp, cnt * es, dst + p + 4, cap - p - 4);
    if (c < 0) { rc = c; break; }
    dst[p] = (uint8_t)(c >> 24); dst[p + 1] = (uint8_t)(c >> 16); dst[p + 2] = (uint8_t)(c >> 8); dst[p + 3] = (uint8_t)c;
    p += 4 + c;
    e += cnt;
  }
  free(tmp);
  if (rc < 0) return rc;
  const int64_t left = (n - e) * es;
  if (p + left > cap) return ORC_ERR_SIZE;
  memcpy(dst + p, src + e * es, (size_t)left);
  return p + left;
}

/* the bare transposition (tests) */
void orc_bshuf_trans(const uint8_t *in, uint8_t *out, int64_t n, int64_t es) { bshuf_trans(in, out, n, es); }
void orc_bshuf_untrans(const uint8_t *in, uint8_t *out, int64_t n, int64_t es) { bshuf_untrans(in, out, n, es); }
