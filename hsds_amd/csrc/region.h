// region.h -- strided N-d region copy / compare (numpy basic slicing) for the hyperslab
// copies of the HSDS data path: chunkReadSelection's chunk_arr[slices] gather and
// chunkWriteSelection's compare + scatter (hsds/util/chunkUtil.py:882-995), the SN slab
// placement np_arr[data_sel] = chunk_arr and the write-side arr[data_sel] gather
// (hsds/chunk_crawl.py:118-150,395-418).  One record = hsds_copy_desc (include/hsds_amd.h).
//
// A record is first normalised (nreg_make): dims of count 1 dropped, an innermost dim
// that is contiguous on both sides folded into bytes, and outer dims that continue their
// inner neighbour on both sides merged into it -- a 512 x 2048-byte chunk piece of a slab
// becomes 512 rows of one 2048-byte run, a whole contiguous chunk one run.  The work unit
// is a ROW (all dims but the innermost); a wave takes a group of rows, its lanes split
// evenly between them (lanes per row = the power of two covering the row's units), and a
// row's offsets come from one 32-bit mixed-radix unravel per row, not per element.
//  - contiguous runs: 16-byte slots of the DESTINATION, every full slot one 16-byte store;
//    its source by one 16-byte load (same alignment), four dword loads (alignment equal
//    mod 4) or five dword loads and byte funnel shifts; only a run's first and last slot
//    move bytes singly.  Four slots per lane are in flight before the first store.
//  - strided elements with a contiguous destination (the chunk -> packed piece gathers of
//    a stepped selection): a lane gathers the 16 / itemsize elements of one destination
//    slot and stores them as one 16-byte store.
//  - anything else: one element per lane, typed loads / stores when aligned.
//
// SINGLE SOURCE for the HIP kernels (engine.hip copy_kernel / compare_kernel) and the CPU
// emulation (tests/emu/region_emu.cpp), which runs every lane of every wave in turn.
#pragma once
#include <stdint.h>
#include <string.h>
#include "../../include/hsds_amd.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RG_HD __device__ __forceinline__
#define RG_GPU 1
typedef uint32_t rg_v4 __attribute__((ext_vector_type(4)));
#define RG_V4(a, b, c, d) ((rg_v4){(a), (b), (c), (d)})
RG_HD uint32_t rg_alignbit(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbit(hi, lo, sh); }
#else
#define RG_HD static inline
#define RG_GPU 0
struct rg_v4 { uint32_t x, y, z, w; };
static inline rg_v4 rg_make4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { rg_v4 v = {a, b, c, d}; return v; }
#define RG_V4(a, b, c, d) rg_make4((a), (b), (c), (d))
RG_HD uint32_t rg_alignbit(uint32_t hi, uint32_t lo, uint32_t sh) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31u));
}
#endif

namespace rg {

struct NReg {
  int64_t so, doff;
  int64_t ss[HSDS_MAX_RANK], ds[HSDS_MAX_RANK];
  uint32_t cnt[HSDS_MAX_RANK];
  int32_t r, isz;
  uint64_t nrows;      // product of cnt[0 .. r-2]
};

// 0: the region is empty.  d and n live in memory (global / LDS on the GPU): their dims
// are indexed at run time
RG_HD int nreg_make(const hsds_copy_desc& d, int fold, NReg& n) {
  n.so = (int64_t)d.src_off;
  n.doff = (int64_t)d.dst_off;
  n.isz = d.itemsize;
  int r = 0;
  for (int k = 0; k < d.rank && k < HSDS_MAX_RANK; k++) {
    const int64_t c = d.count[k];
    if (c <= 0) return 0;
    if (c >= (1ll << 31)) return 0;     // outside the ABI's range (hsds_copy_desc): the host splits such dims
    if (c == 1) continue;
    n.cnt[r] = (uint32_t)c;
    n.ss[r] = d.src_stride[k];
    n.ds[r] = d.dst_stride[k];
    r++;
  }
  if (r == 0) { n.cnt[0] = 1; n.ss[0] = n.isz; n.ds[0] = n.isz; r = 1; }
  if (fold && n.ss[r - 1] == n.isz && n.ds[r - 1] == n.isz && (uint64_t)n.cnt[r - 1] * (uint64_t)n.isz < (1ull << 31)) {
    n.cnt[r - 1] *= (uint32_t)n.isz;
    n.ss[r - 1] = 1;
    n.ds[r - 1] = 1;
    n.isz = 1;
  }
  while (r > 1 && n.ss[r - 2] == (int64_t)n.cnt[r - 1] * n.ss[r - 1] && n.ds[r - 2] == (int64_t)n.cnt[r - 1] * n.ds[r - 1] &&
         (uint64_t)n.cnt[r - 2] * n.cnt[r - 1] < (1ull << 31)) {
    n.cnt[r - 2] *= n.cnt[r - 1];
    n.ss[r - 2] = n.ss[r - 1];
    n.ds[r - 2] = n.ds[r - 1];
    r--;
  }
  n.r = r;
  uint64_t rows = 1;
  for (int k = 0; k < r - 1; k++) rows *= n.cnt[k];
  n.nrows = rows;
  return 1;
}

// source / destination byte offsets of row q (mixed radix over dims r-2 .. 0)
RG_HD void nreg_row(const NReg& n, uint64_t q, int64_t& so, int64_t& doff) {
  so = n.so;
  doff = n.doff;
  if (q < (1ull << 32)) {
    uint32_t t = (uint32_t)q;
    for (int k = n.r - 2; k >= 0; k--) {
      const uint32_t c = n.cnt[k];
      const uint32_t i = t % c;
      t /= c;
      so += (int64_t)i * n.ss[k];
      doff += (int64_t)i * n.ds[k];
    }
  } else {
    for (int k = n.r - 2; k >= 0; k--) {
      const uint64_t c = n.cnt[k];
      const uint64_t i = q % c;
      q /= c;
      so += (int64_t)i * n.ss[k];
      doff += (int64_t)i * n.ds[k];
    }
  }
}

RG_HD uint32_t pow2_at_least(uint32_t v) { return v <= 1u ? 1u : 1u << (32 - __builtin_clz(v - 1u)); }

// how a region's rows are cut: units per row (destination slots or elements), lanes per
// row (a power of two), rows per wave group
// (a row longer than UPIECE units is cut into pieces, one wave group each, so one long
// contiguous run still spreads over the whole grid)
constexpr uint32_t UPIECE = 4096;
struct Plan {
  uint32_t C, lpr, rpw;
  int64_t iss, ids;
  int isz;
  int run, gather;
  uint32_t pieces;     // wave groups per row (1 unless the row is longer than UPIECE units)
  uint64_t ngroups;
};

RG_HD void plan_groups(const NReg& n, uint32_t units, Plan& p) {
  p.lpr = units >= 64u ? 64u : pow2_at_least(units);
  p.rpw = 64u / p.lpr;
  p.pieces = units > UPIECE ? (units + UPIECE - 1u) / UPIECE : 1u;
  p.ngroups = p.pieces > 1u ? n.nrows * p.pieces : (n.nrows + p.rpw - 1u) / p.rpw;
}

// row q and the unit range [u0, u1) of group g for this lane's row slot
RG_HD bool group_row(const NReg& n, const Plan& p, uint64_t g, uint32_t rsub, uint64_t& q, uint32_t& u0, uint32_t& u1) {
  if (p.pieces > 1u) {
    q = g / p.pieces;
    const uint32_t k = (uint32_t)(g - q * p.pieces);
    u0 = k * UPIECE;
    u1 = u0 + UPIECE;
  } else {
    q = g * p.rpw + rsub;
    u0 = 0u;
    u1 = 0xffffffffu;
  }
  return q < n.nrows;
}

RG_HD Plan plan_copy(const NReg& n) {
  Plan p;
  p.C = n.cnt[n.r - 1];
  p.iss = n.ss[n.r - 1];
  p.ids = n.ds[n.r - 1];
  p.isz = n.isz;
  p.run = p.isz == 1 && p.iss == 1 && p.ids == 1;
  // (the 16-byte slot paths count a row's bytes in 32 bits)
  p.gather = !p.run && p.ids == p.isz && (p.isz == 1 || p.isz == 2 || p.isz == 4 || p.isz == 8) &&
             (uint64_t)p.C * (uint64_t)p.isz < (1ull << 31);
  const uint32_t units = p.run ? (p.C + 30u) / 16u : p.gather ? (p.C * (uint32_t)p.isz + 30u) / 16u : p.C;
  plan_groups(n, units, p);
  return p;
}

// the 16 source bytes at sp (any alignment): the aligned dwords that hold them each hold
// at least one source byte, so no load leaves the source's pages
RG_HD rg_v4 load16_any(const uint8_t* sp) {
  const uintptr_t a = (uintptr_t)sp;
  if (!(a & 15u)) return *(const rg_v4*)sp;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  if (!(a & 3u)) return RG_V4(w[0], w[1], w[2], w[3]);
  const uint32_t sh = (uint32_t)(a & 3u) * 8u;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return RG_V4(rg_alignbit(w1, w0, sh), rg_alignbit(w2, w1, sh), rg_alignbit(w3, w2, sh), rg_alignbit(w4, w3, sh));
}

RG_HD void copy_elem(const uint8_t* s, uint8_t* d, int itemsize) {
  const uintptr_t a = (uintptr_t)s | (uintptr_t)d;
  if (itemsize == 16 && !(a & 15u)) { *(rg_v4*)d = *(const rg_v4*)s; return; }
  if (itemsize == 4 && !(a & 3u)) { *(uint32_t*)d = *(const uint32_t*)s; return; }
  if (itemsize == 8 && !(a & 7u)) { *(uint64_t*)d = *(const uint64_t*)s; return; }
  if (itemsize == 2 && !(a & 1u)) { *(uint16_t*)d = *(const uint16_t*)s; return; }
  for (int b = 0; b < itemsize; b++) d[b] = s[b];
}

// one element of 1, 2, 4 or 8 bytes as the low bits of a u64
RG_HD uint64_t load_elem(const uint8_t* p, int isz) {
  const uintptr_t a = (uintptr_t)p;
  if (isz == 4 && !(a & 3u)) return *(const uint32_t*)p;
  if (isz == 2 && !(a & 1u)) return *(const uint16_t*)p;
  if (isz == 8 && !(a & 7u)) return *(const uint64_t*)p;
  uint64_t v = 0;
  for (int b = 0; b < isz; b++) v |= (uint64_t)p[b] << (8 * b);
  return v;
}

// lane `lane` of the wave that copies row group g of region n
RG_HD void copy_group(const uint8_t* src, uint8_t* dst, const NReg& n, const Plan& p, uint64_t g, uint32_t lane) {
  const uint32_t sub = lane & (p.lpr - 1u), rsub = lane / p.lpr;
  uint64_t q;
  uint32_t u0, u1;
  if (!group_row(n, p, g, rsub, q, u0, u1)) return;
  int64_t so, doff;
  nreg_row(n, q, so, doff);
  const uint8_t* s = src + so;
  uint8_t* d = dst + doff;
  const int isz = p.isz;
  if (p.run || p.gather) {
    const uint32_t bytes = p.run ? p.C : p.C * (uint32_t)isz;
    const uintptr_t d0 = (uintptr_t)d, dend = d0 + bytes;
    const uintptr_t x00 = d0 & ~(uintptr_t)15;
    const uint32_t nall = (uint32_t)((dend - x00 + 15u) >> 4);
    const uint32_t nslots = nall < u1 ? nall : u1;
    const bool ealign = p.run || !(d0 & (uintptr_t)(isz - 1));
    for (uint32_t j0 = u0 + sub; j0 < nslots; j0 += 4u * p.lpr) {
      rg_v4 v[4];
      uint32_t full = 0;
      for (uint32_t u = 0; u < 4u; u++) {
        const uint32_t j = j0 + u * p.lpr;
        const uintptr_t x0 = x00 + 16u * (uintptr_t)j;
        v[u] = RG_V4(0u, 0u, 0u, 0u);
        if (j < nslots && x0 >= d0 && x0 + 16u <= dend && ealign) {
          full |= 1u << u;
          if (p.run) {
            v[u] = load16_any(s + (x0 - d0));
          } else {
            const uint32_t e0 = (uint32_t)((x0 - d0) / (uintptr_t)isz);
            const uint32_t G = 16u / (uint32_t)isz;
            uint64_t lo = 0, hi = 0;
            for (uint32_t k = 0; k < G; k++) {
              const uint64_t x = load_elem(s + (int64_t)(e0 + k) * p.iss, isz);
              const uint32_t bit = k * (uint32_t)isz * 8u;
              if (bit < 64u) lo |= x << bit; else hi |= x << (bit - 64u);
            }
            v[u] = RG_V4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
          }
        }
      }
      for (uint32_t u = 0; u < 4u; u++) {
        const uint32_t j = j0 + u * p.lpr;
        if (j >= nslots) continue;
        const uintptr_t x0 = x00 + 16u * (uintptr_t)j;
        if ((full >> u) & 1u) {
          *(rg_v4*)x0 = v[u];
        } else {
          // a run's partial first / last slot (or an element-misaligned gather row)
          const uintptr_t lo = x0 > d0 ? x0 : d0, hi = x0 + 16u < dend ? x0 + 16u : dend;
          if (p.run) {
            for (uintptr_t x = lo; x < hi; x++) *(uint8_t*)x = s[x - d0];
          } else {
            for (uintptr_t x = lo; x < hi; x++) {
              const uint32_t off = (uint32_t)(x - d0);
              *(uint8_t*)x = s[(int64_t)(off / (uint32_t)isz) * p.iss + off % (uint32_t)isz];
            }
          }
        }
      }
    }
  } else {
    const uint32_t e1 = p.C < u1 ? p.C : u1;
    for (uint32_t e = u0 + sub; e < e1; e += p.lpr) copy_elem(s + (int64_t)e * p.iss, d + (int64_t)e * p.ids, isz);
  }
}

RG_HD int elem_differs(const uint8_t* a, const uint8_t* b, int itemsize, int kind) {
  switch (kind) {
    case HSDS_KIND_F32: { float x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return !(x == y); }
    case HSDS_KIND_F64: { double x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return !(x == y); }
#if RG_GPU
    case HSDS_KIND_F16: { _Float16 x, y; memcpy(&x, a, 2); memcpy(&y, b, 2); return !(x == y); }
#else
    case HSDS_KIND_F16: {   // IEEE half compare without a half type: NaN never equal, +-0 equal
      uint16_t x, y; memcpy(&x, a, 2); memcpy(&y, b, 2);
      const int xn = (x & 0x7c00u) == 0x7c00u && (x & 0x3ffu), yn = (y & 0x7c00u) == 0x7c00u && (y & 0x3ffu);
      if (xn || yn) return 1;
      if (!((x | y) & 0x7fffu)) return 0;
      return x != y;
    }
#endif
    case HSDS_KIND_C64: { float x[2], y[2]; memcpy(x, a, 8); memcpy(y, b, 8); return !(x[0] == y[0] && x[1] == y[1]); }
    case HSDS_KIND_C128: { double x[2], y[2]; memcpy(x, a, 16); memcpy(y, b, 16); return !(x[0] == y[0] && x[1] == y[1]); }
    default: {
      const uintptr_t al = (uintptr_t)a | (uintptr_t)b;
      if (itemsize == 4 && !(al & 3u)) return *(const uint32_t*)a != *(const uint32_t*)b;
      if (itemsize == 2 && !(al & 1u)) return *(const uint16_t*)a != *(const uint16_t*)b;
      if (itemsize == 8 && !(al & 7u)) return *(const uint64_t*)a != *(const uint64_t*)b;
      for (int k = 0; k < itemsize; k++) if (a[k] != b[k]) return 1;
      return 0;
    }
  }
}

// compare: units are 16-byte pieces of a run (bytewise kinds fold runs) or elements
RG_HD Plan plan_compare(const NReg& n) {
  Plan p;
  p.C = n.cnt[n.r - 1];
  p.iss = n.ss[n.r - 1];
  p.ids = n.ds[n.r - 1];
  p.isz = n.isz;
  p.run = p.isz == 1 && p.iss == 1 && p.ids == 1;
  p.gather = 0;
  const uint32_t units = p.run ? (p.C + 15u) / 16u : p.C;
  plan_groups(n, units, p);
  return p;
}

// lane `lane` of the wave comparing row group g: does chunk a (dst side) differ from data
// b (src side)?  numpy array_equal: NaN never equal, -0.0 == 0.0 for float kinds
RG_HD int compare_group(const uint8_t* b, const uint8_t* a, const NReg& n, const Plan& p, uint64_t g, uint32_t lane,
                        int kind) {
  const uint32_t sub = lane & (p.lpr - 1u), rsub = lane / p.lpr;
  uint64_t q;
  uint32_t u0, u1;
  if (!group_row(n, p, g, rsub, q, u0, u1)) return 0;
  int64_t so, doff;
  nreg_row(n, q, so, doff);
  const uint8_t* pb = b + so;
  const uint8_t* pa = a + doff;
  int found = 0;
  if (p.run) {
    const uint32_t nall = (p.C + 15u) / 16u, units = nall < u1 ? nall : u1;
    for (uint32_t j = u0 + sub; j < units && !found; j += p.lpr) {
      const uint32_t o = 16u * j, m = p.C - o < 16u ? p.C - o : 16u;
      if (m == 16u && !((((uintptr_t)(pa + o)) | (uintptr_t)(pb + o)) & 15u)) {
        const rg_v4 x = *(const rg_v4*)(pa + o), y = *(const rg_v4*)(pb + o);
        found = (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
      } else {
        for (uint32_t k = 0; k < m; k++) found |= pa[o + k] != pb[o + k];
      }
    }
  } else {
    const uint32_t e1 = p.C < u1 ? p.C : u1;
    for (uint32_t e = u0 + sub; e < e1 && !found; e += p.lpr)
      found = elem_differs(pa + (int64_t)e * p.ids, pb + (int64_t)e * p.iss, p.isz, kind);
  }
  return found;
}

}  // namespace rg
