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
 *     orc_blosclz_decode).  zstd and snappy stay unsupported.
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
  int codec = (flags >> 5) & 7;   /* 0 blosclz, 1 lz4/lz4hc, 3 zlib; 2 snappy, 4 zstd unsupported */
  if (codec != 3 && codec != 1 && codec != 0) return ORC_ERR_UNSUPPORTED;
  if (verlz != 1) return ORC_ERR_FRAME;
  if (flags & 0x04) return ORC_ERR_UNSUPPORTED; /* bitshuffle inside Blosc */
  if (nbytes == 0) return 0;
  if (bs <= 0 || ts <= 0 || bs > nbytes) return ORC_ERR_FRAME;
  int64_t nblocks = (nbytes + bs - 1) / bs;
  int64_t leftover = nbytes % bs;
  int64_t hdr = 16 + 4 * nblocks;
  if (hdr > cbytes) return ORC_ERR_FRAME;
  int doshuffle = (flags & 0x01) && ts > 1;
  uint8_t *tmp = doshuffle ? (uint8_t *)malloc((size_t)bs) : NULL;
  int64_t result = nbytes;
  for (int64_t b = 0; b < nblocks; b++) {
    int isleft = (b == nblocks - 1) && leftover;
    int64_t bsz = isleft ? leftover : bs;
    int nspl = blosc_nsplits(flags, ts, bs, isleft);
    int64_t neblock = bsz / nspl;
    int64_t p = (int32_t)rd32(src + 16 + 4 * b);
    if (p < hdr || p >= cbytes) { result = ORC_ERR_FRAME; break; }
    uint8_t *out = doshuffle ? tmp : dst + b * bs;
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
                               : orc_blosclz_decode(src + p, cs, out + j * neblock, neblock);
        if (r < 0) { result = r == ORC_ERR_SIZE ? ORC_ERR_SIZE : r; goto done; }
        if (r != neblock) { result = ORC_ERR_SIZE; goto done; }
      }
      p += cs;
    }
    if (doshuffle) orc_unshuffle(tmp, bsz, ts, dst + b * bs);
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
