// bshuf.h -- bitshuffle+LZ4 chunk decode (shuffle = 2), one wavefront per chunk.
//
// HSDS writes a bitshuffle chunk as storUtil._shuffle(codec=2) (storUtil.py:103-131):
// u64 BE chunk bytes, u32 BE block_size * itemsize, then bitshuffle.compress_lz4:
// per block of block_size elements a u32 BE size and the LZ4 block of the block's bit
// transposition; a last block of the remaining elements rounded down to a multiple of
// 8; the n % 8 leftover elements raw.  storUtil._unshuffle(codec=2)
// (storUtil.py:144-174) checks the header and calls bitshuffle.decompress_lz4, which
// also rejects a frame whose bytes are not all consumed.
//
// The wave walks the block sizes (lane 0, GROUP blocks ahead), LZ4-decodes GROUP
// blocks at a time with lz_wave.h's group decoder into a staging copy of the chunk,
// and then inverts the bit transposition of those blocks into the destination with
// all 64 lanes.  Transposed layout of n elements (n % 8 == 0) of es bytes: row
// r = 8 j + k holds bit k of byte j of every element, element i at bit i % 8 of row
// byte i / 8.
//
// Single source: tests/emu/bshuf_emu.cpp runs the same code on CPU.
#pragma once
#include "lz_wave.h"

#ifndef BS_PRIO_KB
#define BS_PRIO_KB 64                 // wave priority: one level per 64 KiB of the chunk's input left (0: off)
#endif
namespace bs {

// bshuf_default_block_size: an 8 KiB target, a multiple of 8, at least 128 elements
HZ_HD uint32_t default_block(uint32_t es) {
  uint32_t b = (8192u / es) / 8u * 8u;
  return b < 128u ? 128u : b;
}

// 8x8 bit matrix transpose: bit 8 r + c <-> bit 8 c + r
HZ_HD uint64_t t8x8(uint64_t x) {
  uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

// inverse bit transposition of row byte q of a block of cnt elements (cnt % 8 == 0, row =
// cnt / 8) of es bytes: elements 8 q .. 8 q + 7, all es bytes, from in (transposed) to out
HZ_HD void untrans_row(hz_gcu8* in, hz_gu8* out, uint32_t q, uint32_t row, uint32_t es) {
  hz_gu8* o = out + (uint64_t)q * 8u * es;
  if (es <= 8u) {
    uint64_t el[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // element 8q + m, bytes packed little-endian
    for (uint32_t j = 0; j < es; j++) {
      uint64_t x = 0;
      for (uint32_t k = 0; k < 8u; k++) x |= (uint64_t)in[(uint64_t)(j * 8u + k) * row + q] << (8u * k);
      const uint64_t y = t8x8(x);                  // byte m: byte j of element 8q + m
      for (uint32_t m = 0; m < 8u; m++) el[m] |= ((y >> (8u * m)) & 0xffull) << (8u * j);
    }
    if (es == 4u && !(((uintptr_t)o) & 3u)) {
      for (uint32_t m = 0; m < 8u; m++) *(hz_gu32*)(o + 4u * m) = (uint32_t)el[m];
    } else if (es == 8u && !(((uintptr_t)o) & 3u)) {
      for (uint32_t m = 0; m < 8u; m++) {
        *(hz_gu32*)(o + 8u * m) = (uint32_t)el[m];
        *(hz_gu32*)(o + 8u * m + 4u) = (uint32_t)(el[m] >> 32);
      }
    } else {
      for (uint32_t m = 0; m < 8u; m++)
        for (uint32_t j = 0; j < es; j++) o[m * es + j] = (uint8_t)(el[m] >> (8u * j));
    }
  } else {
    for (uint32_t j = 0; j < es; j++) {
      uint64_t x = 0;
      for (uint32_t k = 0; k < 8u; k++) x |= (uint64_t)in[(uint64_t)(j * 8u + k) * row + q] << (8u * k);
      const uint64_t y = t8x8(x);
      for (uint32_t m = 0; m < 8u; m++) o[m * es + j] = (uint8_t)(y >> (8u * m));
    }
  }
}

// inverse bit transposition of one block: cnt elements (cnt % 8 == 0) of es bytes from
// in (transposed) to out.  Work item = 8 elements (one row byte q) x all es bytes.
#if HZ_GPU
__device__
#else
static
#endif
inline void untrans_block(hz_gcu8* in, hz_gu8* out, uint32_t cnt, uint32_t es) {
  const uint32_t row = cnt / 8u;
  LANE_LOOP {
    for (uint32_t q = (uint32_t)lane; q < row; q += 64u) untrans_row(in, out, q, row, es);
  }
}

// Forward bit transposition (the write path, storUtil._shuffle codec 2 ->
// bshuf_trans_bit_elem) of elements 8 q .. 8 q + 7 of a block of cnt elements
// (cnt % 8 == 0, row = cnt / 8): blk points at the block's first element, out at its
// transposed copy.  Row byte q of rows 8 j .. 8 j + 7 comes from byte j of the 8
// elements, through the same 8x8 bit transpose the decoder inverts with.
HZ_HD void trans_group(hz_gcu8* blk, hz_gu8* out, uint32_t q, uint32_t row, uint32_t es) {
  hz_gcu8* e = blk + (uint64_t)q * 8u * es;
  if (es == 4u && !(((uintptr_t)e) & 3u)) {
    uint32_t w[8];
    for (uint32_t m = 0; m < 8u; m++) w[m] = *(const hz_gu32*)(e + 4u * m);
    for (uint32_t j = 0; j < 4u; j++) {
      uint64_t x = 0;
      for (uint32_t m = 0; m < 8u; m++) x |= (uint64_t)((w[m] >> (8u * j)) & 0xffu) << (8u * m);
      const uint64_t y = t8x8(x);                        // byte k: bit k of byte j of each element
      for (uint32_t k = 0; k < 8u; k++) out[(uint64_t)(j * 8u + k) * row + q] = (uint8_t)(y >> (8u * k));
    }
    return;
  }
  for (uint32_t j = 0; j < es; j++) {
    uint64_t x = 0;
    for (uint32_t m = 0; m < 8u; m++) x |= (uint64_t)e[m * es + j] << (8u * m);
    const uint64_t y = t8x8(x);
    for (uint32_t k = 0; k < 8u; k++) out[(uint64_t)(j * 8u + k) * row + q] = (uint8_t)(y >> (8u * k));
  }
}

HZ_HD uint32_t be32(hz_gcu8* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

#ifndef BS_GK
#define BS_GK 16
#endif
struct Shared {
  lz::SharedT<BS_GK> lz;      // 8 KiB LZ4 blocks: 16 sequences per round (A/B: 272 vs 255 GB/s at 32)
  uint32_t blk_e[lz::GROUP];      // first element of each block of the group
  uint32_t blk_n[lz::GROUP];      // elements
  uint32_t next_p, next_e;        // walk position after the group
  int32_t walk_st;
};

// Decode one chunk: src (n bytes) -> dst (chunk_bytes), staging copy stg (chunk_bytes).
// Returns ST_OK or a negative status (uniform).
#if HZ_GPU
__device__
#else
static
#endif
inline int chunk(Shared& sh, const uint8_t* srcp, uint32_t n, uint8_t* dstp, uint8_t* stgp, uint32_t chunk_bytes,
                 uint32_t es) {
  hz_gcu8* src = HZ_GLOBAL(hz_gcu8*, srcp);
  hz_gu8* dst = HZ_GLOBAL(hz_gu8*, dstp);
  hz_gu8* stg = HZ_GLOBAL(hz_gu8*, stgp);
  if (n < 12u || es < 1u || chunk_bytes % es) return hz::ST_TRUNC;               // storUtil.py:148-152
  uint64_t total = 0;
  for (uint32_t i = 0; i < 8u; i++) total = total << 8 | src[i];
  if (total != (uint64_t)chunk_bytes) return hz::ST_SIZE;                         // storUtil.py:160-164
  uint32_t bsz = be32(src + 8) / es;                                              // storUtil.py:167
  if (bsz == 0) bsz = default_block(es);
  if (bsz % 8u) return hz::ST_DATA;
  const uint32_t nel = chunk_bytes / es;
  uint32_t p = 12, e = 0;
  while (e + 8u <= nel) {
#if HZ_GPU && BS_PRIO_KB
    {
      // wave priority by the chunk's remaining input (inflate2.h HZ2_PRIO_ABS; A/B round 5,
      // bench bshuf leg: off 274.6, 64 KiB 285.2, 128 KiB 282.9, 192 KiB 280.0 GB/s)
      const uint32_t lv = ((n - p) >> 10) / (uint32_t)BS_PRIO_KB;
      if (lv >= 3u) __builtin_amdgcn_s_setprio(3);
      else if (lv == 2u) __builtin_amdgcn_s_setprio(2);
      else if (lv == 1u) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    // ---- lane 0 walks the next GROUP block headers ----
    WAVE_SYNC();
    LANE_LOOP {
      if (lane == 0) {
        uint32_t pp = p, ee = e;
        int32_t wst = hz::ST_OK;
        for (int g = 0; g < lz::GROUP; g++) {
          lz::LaneJob j = {nullptr, nullptr, 0u, 0u, lz::FMT_LZ4, 0u};
          if (wst == hz::ST_OK && ee + 8u <= nel) {
            const uint32_t cnt = nel - ee >= bsz ? bsz : (nel - ee) / 8u * 8u;
            if (pp + 4u > n) wst = hz::ST_TRUNC;
            else {
              const uint32_t nb = be32(src + pp);
              if (nb > n - pp - 4u) wst = hz::ST_TRUNC;
              else {
                j = {srcp + pp + 4u, stgp + (uint64_t)ee * es, nb, cnt * es, lz::FMT_LZ4, 1u};
                sh.blk_e[g] = ee;
                sh.blk_n[g] = cnt;
                pp += 4u + nb;
                ee += cnt;
              }
            }
          }
          if (!j.valid) sh.blk_n[g] = 0;
          sh.lz.job[g] = j;
        }
        sh.next_p = pp;
        sh.next_e = ee;
        sh.walk_st = wst;
      }
    }
    WAVE_SYNC();
    lz::lz_group<false>(sh.lz, nullptr);
    WAVE_SYNC_GLOBAL();        // the group's staged blocks visible to every lane
    for (int g = 0; g < lz::GROUP; g++)
      if (sh.blk_n[g] && sh.lz.m_st[g] != hz::ST_OK) return sh.lz.m_st[g];
    if (sh.walk_st != hz::ST_OK) return sh.walk_st;
    for (int g = 0; g < lz::GROUP; g++)
      if (sh.blk_n[g]) untrans_block(stg + (uint64_t)sh.blk_e[g] * es, dst + (uint64_t)sh.blk_e[g] * es, sh.blk_n[g], es);
    p = sh.next_p;
    e = sh.next_e;
  }
  const uint32_t left = (nel - e) * es;                   // n % 8 elements, raw
  if (left > n - p) return hz::ST_TRUNC;
  LANE_LOOP { for (uint32_t i = (uint32_t)lane; i < left; i += 64u) dst[(uint64_t)e * es + i] = src[p + i]; }
  if (p + left != n) return hz::ST_SIZE;                   // decompress_lz4: bytes left over
  return hz::ST_OK;
}

}  // namespace bs
