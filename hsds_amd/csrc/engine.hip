// engine.hip -- MI355X (gfx950) chunk codec + hyperslab engine behind include/hsds_amd.h.
//
// Kernels (all batched over many chunks, one launch per stage):
//  decode (storUtil._uncompress, storUtil.py:182-235)
//   frame_walk_kernel   one thread per chunk: Blosc1 / zlib / raw detection and emission
//                       of one work item per deflate stream / LZ / zstd / raw split into
//                       a compact item pool (no per-chunk split cap)
//   inflate2_kernel     persistent waves pull zlib / raw items from a device counter; one
//                       wavefront decodes one zlib stream (inflate2.h) in stream order
//   lz_kernel           LZ4 / BloscLZ Blosc splits, 8 per wavefront (lz_wave.h)
//   zstd_kernel         zstd Blosc splits, one wavefront per split (zstd_wave.h)
//   bshuf_kernel        bitshuffle+LZ4 chunks (shuffle = 2), one wavefront per chunk (bshuf.h)
//   unshuffle_kernel    byte / bit unshuffle of staged chunks: shuffled Blosc blocks (any
//                       codec), HDF5-shuffled F2 streams
//  hyperslab copies (chunkUtil.py:882-995, chunk_crawl.py:118-150,395-418)
//   copy_kernel / compare_kernel   strided N-d region copies / numpy-equal compares
//   plan_descs_kernel   one thread per piece: copy records of a hyperslab plan
//  encode (storUtil._compress, storUtil.py:238-281)
//   enc_plan_kernel     one thread per chunk: c-blosc 1.21 frame geometry, one item per split
//   parse_kernel        persistent waves, one zlib / LZ stream each: hash chains + parse
//   huff_kernel, emit_kernel     one wave per 8 KiB segment: Huffman code, bit emission
//   lz4_block_kernel    LZ4 / BloscLZ blocks from the parse tokens (lz4_enc.h)
//   layout_kernel, raw_copy_kernel   frame layout, raw splits and memcpyed payloads
//   bs_*_kernel         bitshuffle+LZ4 writer (plan, fill, transposition, layout)
// Every launch is asynchronous on the caller's stream; no host synchronisation
// inside the batched entry points.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/hsds_amd.h"
#include "inflate_wave.h"
#include "inflate2.h"
#include "deflate_wave.h"
#include "lz_wave.h"
#include "lz4_enc.h"
#include "zstd_wave.h"
#include "bshuf.h"
#include "zstd_enc.h"
#include "region.h"

#ifndef HZ_ZSTD_WPE
#define HZ_ZSTD_WPE 4      // zstd_kernel waves per SIMD the compiler must allow (VGPR budget)
#endif
#ifndef HZ2_WPE
#define HZ2_WPE 4          // inflate2_kernel waves per SIMD the compiler must allow (VGPR budget)
#endif
#ifndef HZ2_PIPE_DEFAULT
#define HZ2_PIPE_DEFAULT 0   // wavefronts per zlib stream: 0 by batch size (4 or 2 when a batch cannot fill the GPU), or 1, 2, 4
#endif
#define HSDS_VERSION "hsds_amd 0.1.0 (gfx950)"

namespace {


// ITEM_LZ4 / ITEM_BLOSCLZ: Blosc splits of the byte-LZ77 codecs (lz_wave.h)
enum : uint32_t { ITEM_ZLIB = 0, ITEM_RAW = 1, ITEM_LZ4 = 2, ITEM_BLOSCLZ = 3, ITEM_ZSTD = 4, ITEM_INEXACT = 0x100 };

// decode work item (32 bytes): one zlib stream / raw span / LZ split.  kind word: bits 0-7
// decoder, bit 8 inexact size, bits 16-23 byte-unshuffle element size n of a raw span (<= 1:
// none; compressed items always write plain bytes)
struct Item {
  uint64_t src;
  uint64_t dst;
  uint32_t src_len;
  uint32_t dst_len;
  uint32_t chunk;
  uint32_t kind;
};

struct ChunkMeta {     // post-decode unshuffle of LZ / zstd Blosc blocks staged in tmp
  uint64_t tmp;        // staged (shuffled) bytes
  uint64_t dst;
  uint32_t mode;       // 0 none, 1 byte unshuffle of Blosc blocks (ts, bs), 2 bit unshuffle of Blosc blocks
  uint32_t ts;
  uint32_t bs;
  uint32_t nbytes;
};

__device__ __forceinline__ uint32_t rd8(const uint8_t* p) { return p[0]; }
__device__ __forceinline__ uint32_t rd32le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// output map of an item (hz2::Perm): a shuffled raw span (shuffle-only objects) lands unshuffled
__device__ __forceinline__ hz2::Perm item_perm(const Item& it) {
  const uint32_t n = (it.kind >> 16) & 0xffu;
  if (n <= 1u) return hz2::perm_make(1u, 1u, 0u);
  return hz2::perm_make(n, it.dst_len / n, 0u);
}

// -------------------------------------------------------------------------
// frame walk: one thread per chunk.  Restates c-blosc 1.21 blosc_decompress frame rules
// (oracle/oracle.c orc_blosc_decode) and storUtil._uncompress's dispatch
// (storUtil.py:182-235).  The walk runs twice: once to count the chunk's items, then -- after
// one atomic allocation from the batch's item pool -- to write them, so a chunk may have any
// number of Blosc splits (pool capacity: 8 per chunk + 1 per 2 KiB of destination).
// A batch whose items exceed the pool fails only the chunks that do not fit (pool_reserve).
// Every decoder writes plain bytes: the splits of a shuffled (byte or bit) Blosc frame and a
// shuffled F2 stream are staged in tmp and unshuffled by unshuffle_kernel; only a shuffled
// raw object carries an unshuffle map (item_perm).
// -------------------------------------------------------------------------
// reserve n consecutive pool slots without ever moving the fill count past cap
__device__ __forceinline__ int pool_reserve(uint32_t* ctr, uint32_t n, uint32_t cap, uint32_t* base) {
  uint32_t cur = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (n > cap || cur > cap - n) return 0;
    const uint32_t prev = atomicCAS(ctr, cur, cur + n);
    if (prev == cur) { *base = cur; return 1; }
    cur = prev;
  }
}

__global__ void frame_walk_kernel(const uint8_t* __restrict__ src_base, const hsds_chunk_desc* __restrict__ chunks,
                                  int64_t nchunks, uint8_t* dst_base, uint8_t* tmp_base, Item* __restrict__ pool,
                                  uint32_t pool_cap, uint32_t* __restrict__ pool_ctr, ChunkMeta* __restrict__ meta,
                                  uint32_t* __restrict__ meta_list, uint32_t* __restrict__ meta_count,
                                  uint32_t* __restrict__ kind_counts, int32_t* __restrict__ status,
                                  int compressor, int shuffle, int itemsize, int inexact) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = ci < nchunks;      // every lane stays for the wave-wide pool reservation
  const hsds_chunk_desc c = chunks[valid ? ci : 0];
  const uint8_t* s = src_base + c.src_off;
  const uint64_t L = c.src_len, n = c.dst_len;
  uint8_t* out = dst_base + c.dst_off;
  uint8_t* tmp = tmp_base ? tmp_base + c.dst_off : nullptr;
  int st = HSDS_OK;
  uint32_t cnt = 0, base = 0, nlz = 0, nzs = 0;
  Item* slot = nullptr;
  ChunkMeta m = {0, (uint64_t)out, 0, 0, 0, (uint32_t)n};
  auto walk = [&](int pass) {
    cnt = 0; nlz = 0; nzs = 0;
    m.mode = 0;
    auto emit = [&](uint32_t kind, const uint8_t* sp, uint64_t sl, uint8_t* dp, uint64_t dl) {
      if (pass == 1) {
        Item it;
        it.src = (uint64_t)sp; it.dst = (uint64_t)dp; it.src_len = (uint32_t)sl; it.dst_len = (uint32_t)dl;
        it.chunk = (uint32_t)ci; it.kind = kind;
        slot[cnt] = it;
      }
      cnt++;
      nlz += (kind & 0xff) == ITEM_LZ4 || (kind & 0xff) == ITEM_BLOSCLZ;
      nzs += (kind & 0xff) == ITEM_ZSTD;
    };
    const uint32_t shuf_n = (shuffle == HSDS_SHUFFLE_BYTE && itemsize > 1) ? ((uint32_t)itemsize << 16) : 0u;
    if (L >= (1ull << 28) || n >= (1ull << 31)) {
      st = HSDS_ERR_UNSUPPORTED;
    } else if (compressor == HSDS_COMP_NONE) {
      if (L != n) st = HSDS_ERR_SIZE;
      else if (shuffle == HSDS_SHUFFLE_BIT) st = HSDS_ERR_UNSUPPORTED;
      else if (shuf_n && (n % (uint64_t)itemsize)) st = HSDS_ERR_ARG;
      else if (shuf_n && itemsize > 255) st = HSDS_ERR_UNSUPPORTED;
      else emit(ITEM_RAW | shuf_n, s, L, out, n);
    } else if (L >= 4 && rd8(s) <= 2 && rd8(s + 3) > 0) {
      // ---- Blosc1 frame (shuffle filter handled in-frame: storUtil.py:203-204) ----
      if (L < 16) st = HSDS_ERR_FRAME;
      else {
        const uint32_t ver = rd8(s), verlz = rd8(s + 1), flags = rd8(s + 2), ts = rd8(s + 3);
        const uint32_t codec = (flags >> 5) & 7;   // 0 blosclz, 1 lz4/lz4hc, 2 snappy, 3 zlib, 4 zstd
        const uint32_t kind = codec == 3 ? ITEM_ZLIB : codec == 1 ? ITEM_LZ4 : codec == 4 ? ITEM_ZSTD : ITEM_BLOSCLZ;
        const uint64_t nbytes = rd32le(s + 4), bs = rd32le(s + 8), cbytes = rd32le(s + 12);
        if (ver != 2 || cbytes > L || cbytes < 16) st = HSDS_ERR_FRAME;
        else if (nbytes != n) st = HSDS_ERR_SIZE;
        else if (flags & 0x02) {
          if (nbytes + 16 > cbytes) st = HSDS_ERR_FRAME;
          else emit(ITEM_RAW, s + 16, nbytes, out, nbytes);
        } else if (codec != 3 && codec != 1 && codec != 0 && codec != 4) st = HSDS_ERR_UNSUPPORTED;   // snappy
        else if (verlz != 1) st = HSDS_ERR_FRAME;
        else if (nbytes > 0) {
          if (bs == 0 || bs > nbytes) st = HSDS_ERR_FRAME;
          else {
            const uint64_t nblocks = (nbytes + bs - 1) / bs, leftover = nbytes % bs;
            const uint64_t hdr = 16 + 4 * nblocks;
            // c-blosc 1.21 blosc_d: byte unshuffle when 0x01 and typesize > 1, else bit
            // unshuffle when 0x04 (any typesize; oracle orc_blosc_decode)
            const int doshuffle = (flags & 0x01) && ts > 1;
            const int dobit = !doshuffle && (flags & 0x04);
            // every decoder writes plain bytes: shuffled frames go through tmp and are
            // unshuffled (byte or bit) by unshuffle_kernel
            const int staged = doshuffle || dobit;
            if (staged && !tmp) st = HSDS_ERR_UNSUPPORTED;
            uint8_t* target = staged ? tmp : out;
            if (hdr > cbytes) st = HSDS_ERR_FRAME;
            for (uint64_t b = 0; b < nblocks && st == HSDS_OK; b++) {
              const int isleft = (b == nblocks - 1) && leftover;
              const uint64_t bsz = isleft ? leftover : bs;
              const uint32_t nspl = (!(flags & 0x10) && ts <= 16 && bs / ts >= 128 && !isleft) ? ts : 1;
              const uint64_t neblock = bsz / nspl;
              int64_t p = (int32_t)rd32le(s + 16 + 4 * b);
              if (p < (int64_t)hdr || p >= (int64_t)cbytes) { st = HSDS_ERR_FRAME; break; }
              for (uint32_t j = 0; j < nspl; j++) {
                if (p + 4 > (int64_t)cbytes) { st = HSDS_ERR_FRAME; break; }
                const int64_t cs = (int32_t)rd32le(s + p);
                p += 4;
                if (cs < 0 || p + cs > (int64_t)cbytes) { st = HSDS_ERR_FRAME; break; }
                const uint32_t k = (uint64_t)cs == neblock ? ITEM_RAW : kind;
                emit(k, s + p, (uint64_t)cs, target + b * bs + j * neblock, neblock);
                p += cs;
              }
            }
            if (staged) { m.mode = dobit ? 2u : 1u; m.tmp = (uint64_t)tmp; m.ts = ts; m.bs = (uint32_t)bs; }
          }
        }
      }
    } else if (compressor == HSDS_COMP_ZLIB) {
      if (shuffle == HSDS_SHUFFLE_BIT) st = HSDS_ERR_UNSUPPORTED;
      else if (shuf_n && (n % (uint64_t)itemsize)) st = HSDS_ERR_ARG;
      else if (shuf_n && itemsize > 255) st = HSDS_ERR_UNSUPPORTED;
      else if (shuf_n && tmp) {
        // F2 chunk: inflated in stream order into tmp (the plain output path: literal windows
        // and whole-dword match resolve), then unshuffled by unshuffle_kernel -- cheaper than
        // byte stores through the output map (measured: DESIGN.md section 5)
        emit(ITEM_ZLIB, s, L, tmp, n);
        m.mode = 1; m.tmp = (uint64_t)tmp; m.ts = (uint32_t)itemsize; m.bs = (uint32_t)n;
      }
      else if (shuf_n) st = HSDS_ERR_UNSUPPORTED;       // (compressed batches always have tmp)
      else emit(inexact ? (ITEM_ZLIB | ITEM_INEXACT) : ITEM_ZLIB, s, L, out, n);
    } else {
      st = HSDS_ERR_UNSUPPORTED;
    }
    if (st != HSDS_OK) { cnt = 0; m.mode = 0; }
  };
  if (valid) walk(0);
  // pool reservation, wave-wide: one compare-and-swap for the wave's items, so the fill
  // count never passes pool_cap.  If they do not fit, the wave's chunks reserve one at a
  // time: an oversized chunk fails alone (HSDS_ERR_UNSUPPORTED) and its neighbours keep
  // their slots; no consumer ever sees a slot that was not written.
  {
    const int lane = (int)(threadIdx.x & 63u);
    const uint32_t want = (valid && st == HSDS_OK) ? cnt : 0u;
    const uint32_t off = hz::wave_excl_scan(want, lane);
    const uint32_t tot = hz::wave_sum(want);
    if (tot) {
      uint32_t wb = 0;
      int ok = 0;
      if (lane == 0) ok = pool_reserve(pool_ctr, tot, pool_cap, &wb);
      ok = __shfl(ok, 0, 64);
      wb = (uint32_t)__shfl((int)wb, 0, 64);
      if (ok) {
        base = wb + off;
      } else {
        for (int l = 0; l < 64; l++) {
          if (lane == l && want) {
            if (!pool_reserve(pool_ctr, want, pool_cap, &base)) { st = HSDS_ERR_UNSUPPORTED; cnt = 0; m.mode = 0; }
          }
        }
      }
    }
  }
  if (!valid) return;
  if (st == HSDS_OK && cnt) {
    slot = pool + base;
    walk(1);
  }
  // items per decoder (kind_counts[0]: LZ splits for lz_kernel, [1]: zlib + raw for
  // inflate2_kernel, [2]: zstd), so that a kernel with nothing to do exits at once
  if (nlz && cnt) atomicAdd(&kind_counts[0], nlz);
  if (cnt - nlz - nzs && cnt) atomicAdd(&kind_counts[1], cnt - nlz - nzs);
  if (nzs && cnt) atomicAdd(&kind_counts[2], nzs);
  status[ci] = st;
  meta[ci] = m;
  if (m.mode) {
    const uint32_t k = atomicAdd(meta_count, 1u);
    meta_list[k] = (uint32_t)ci;
  }
}

// item index -> (chunk, slot) by binary search over the exclusive item offsets (encode side)
__device__ __forceinline__ int64_t item_chunk(const uint32_t* offs, int64_t nchunks, uint32_t item) {
  int64_t lo = 0, hi = nchunks - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (offs[mid] <= item) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// exclusive scan of counts[0..n) into offs[0..n], single workgroup of 1024 threads
__global__ void scan_kernel(const uint32_t* __restrict__ counts, uint32_t* __restrict__ offs, int64_t n) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const uint32_t v = i < n ? counts[i] : 0u;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const uint32_t y = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
      __syncthreads();
      part[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < n) offs[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) offs[n] = carry;
}

// -------------------------------------------------------------------------
// inflate: persistent 64-thread workgroups; each pulls items from the pool until the
// pool's fill count is reached.  zlib streams go to hz2::inflate_stream (inflate2.h) with
// the wave's own scratch (rings + blockIdx.x * SCRATCH_BYTES: match ring + literal stream);
// raw spans are copied.
// -------------------------------------------------------------------------
__device__ __forceinline__ void raw_copy(const Item& it, int lane) {
  const uint8_t* sp = (const uint8_t*)it.src;
  uint8_t* dp = (uint8_t*)it.dst;
  const uint32_t len = it.dst_len;
  const hz2::Perm P = item_perm(it);
  if (P.n == 1u && !(((uintptr_t)sp | (uintptr_t)dp) & 15u)) {
    const uint32_t n16 = len >> 4;
    for (uint32_t i = lane; i < n16; i += 64) ((uint4*)dp)[i] = ((const uint4*)sp)[i];
    for (uint32_t i = (n16 << 4) + lane; i < len; i += 64) dp[i] = sp[i];
  } else {
    for (uint32_t i = lane; i < len; i += 64) dp[hz2::perm_at(P, i)] = sp[i];
  }
}

// Longest streams first (HZ2_LPT): the batch kernel's waves claim items in the order
// ord[0..total), the pool's items sorted by compressed length, longest first (a counting
// sort over 1024 log-linear length classes: 5 bits of exponent, 5 of mantissa), so the
// last claims are the shortest streams and the waves end closer together.  One workgroup;
// ties keep no particular order (scheduling only: every item decodes the same either way).
#ifndef HZ2_LPT
#define HZ2_LPT 1
#endif
__device__ __forceinline__ uint32_t lpt_key(uint32_t len) {
  const uint32_t ex = 31u - (uint32_t)__builtin_clz(len | 1u);
  const uint32_t mt = ex >= 5u ? (len >> (ex - 5u)) & 31u : (len << (5u - ex)) & 31u;
  return 1023u - (ex * 32u + mt);                     // descending length -> ascending key
}
__global__ void __launch_bounds__(1024) order_kernel(const Item* __restrict__ pool, const uint32_t* __restrict__ pool_ctr,
                                                     uint32_t* __restrict__ ord) {
  __shared__ uint32_t cnt[1024];
  __shared__ uint32_t sum[1024];
  const uint32_t total = *pool_ctr, t = threadIdx.x;
  cnt[t] = 0;
  __syncthreads();
  for (uint32_t i = t; i < total; i += 1024u) atomicAdd(&cnt[lpt_key(pool[i].src_len)], 1u);
  __syncthreads();
  // inclusive scan of the counts (Hillis-Steele, double-buffered), then each class's start
  uint32_t v = cnt[t];
  sum[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 1024u; o <<= 1) {
    const uint32_t a = t >= o ? sum[t - o] : 0u;
    __syncthreads();
    v += a;
    sum[t] = v;
    __syncthreads();
  }
  cnt[t] = v - cnt[t];                                // exclusive start of class t
  __syncthreads();
  for (uint32_t i = t; i < total; i += 1024u) {
    const uint32_t k = atomicAdd(&cnt[lpt_key(pool[i].src_len)], 1u);
    ord[k] = i;
  }
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HZ2_WPE))) inflate2_kernel(const Item* __restrict__ pool, const uint32_t* __restrict__ pool_ctr,
                                                      uint32_t* __restrict__ counter, int32_t* __restrict__ status,
                                                      uint32_t* __restrict__ sizes,
                                                      const uint32_t* __restrict__ kind_counts, hz2::Tune tune,
                                                      uint8_t* __restrict__ rings, const uint32_t* __restrict__ ord) {
  __shared__ hz2::Shared sh;
  if (kind_counts[1] == 0) return;   // only LZ / zstd splits in this batch
  const uint32_t total = *pool_ctr;
  const int lane = threadIdx.x;
  uint8_t* ring = rings + (size_t)blockIdx.x * hz2::SCRATCH_BYTES;
#ifdef HZ_PROFILE
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  uint64_t t_busy = 0;
  HzProf prof_;
  for (int i = 0; i < 16; i++) prof_.acc[i] = 0;
  prof_.last = __builtin_amdgcn_s_memtime();
  prof_.cur = 0;
  HzProf* prof = &prof_;
#else
  HzProf* prof = nullptr;
#endif
  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(counter, 1u);
    item = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(item, 0, 64));
    if (item >= total) break;
    if (ord) item = (uint32_t)__builtin_amdgcn_readfirstlane((int)ord[item]);
    const Item it = pool[item];
    const uint32_t kind = it.kind & 0xff;
    int st;
    if (kind == ITEM_RAW) {
      raw_copy(it, lane);
      st = HSDS_OK;
    } else if (kind == ITEM_ZLIB) {
      hz2::Job job = {(const uint8_t*)it.src, it.src_len, (uint8_t*)it.dst, it.dst_len,
                      (it.kind & ITEM_INEXACT) ? 0u : 1u, (it.kind & ITEM_INEXACT) ? &sizes[it.chunk] : nullptr,
                      item_perm(it)};
#ifdef HZ_PROFILE
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
      st = hz2::inflate_stream<hz2::Stats, 1>(sh, job, tune, ring, (hz2::Stats*)nullptr, prof);
#ifdef HZ_PROFILE
      t_busy += __builtin_amdgcn_s_memrealtime() - t0;
      if (lane == 0) atomicMax(&hz_tail[5], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
#endif
    } else {
      continue;                        // lz_kernel's / zstd_kernel's item
    }
    if (lane == 0 && st != HSDS_OK) atomicMin(&status[it.chunk], st);
    __syncthreads();
  }
#ifdef HZ_PROFILE
  {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    prof_.acc[prof_.cur] += now - prof_.last;
    if (lane == 0) for (int i = 0; i < 16; i++) atomicAdd(&hz_prof[i], (unsigned long long)prof_.acc[i]);
    // tail: wave start / end in the 100 MHz real-time clock, streams' decode time
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      atomicMin(&hz_tail[0], (unsigned long long)t_start);
      atomicMax(&hz_tail[1], (unsigned long long)t_end);
      atomicAdd(&hz_tail[2], (unsigned long long)t_end);
      atomicAdd(&hz_tail[3], 1ull);
      atomicAdd(&hz_tail[4], (unsigned long long)t_busy);
      atomicMin(&hz_tail[6], (unsigned long long)t_end);
    }
  }
#endif
  (void)prof;
}

// -------------------------------------------------------------------------
// inflate, two wavefronts per stream (small batches: fewer zlib streams than resident
// wavefronts).  Persistent 128-thread workgroups; both wavefronts decode the same item,
// alternating its windows (inflate2.h, inflate_stream<NW = 2>): one window's header, sync
// phases and emit run beside the other's resolve, about halving a stream's latency.
// -------------------------------------------------------------------------
template <int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(HZ2_WPE))) inflate2w_kernel(const Item* __restrict__ pool, const uint32_t* __restrict__ pool_ctr,
                                                      uint32_t* __restrict__ counter, int32_t* __restrict__ status,
                                                      uint32_t* __restrict__ sizes,
                                                      const uint32_t* __restrict__ kind_counts, hz2::Tune tune,
                                                      uint8_t* __restrict__ rings) {
  __shared__ hz2::Shared sh[NW];
  __shared__ hz2::Ctl ctl;
  if (kind_counts[1] == 0) return;
  const uint32_t total = *pool_ctr;
  const uint32_t w = threadIdx.x >> 6;
  const int lane = (int)(threadIdx.x & 63u);
  uint8_t* ring = rings + ((size_t)blockIdx.x * NW + w) * hz2::SCRATCH_BYTES;
  HzProf* prof = nullptr;
  for (;;) {
    if (threadIdx.x == 0) {
      hz2::ctl_reset(&ctl, atomicAdd(counter, 1u));
      ctl.bar = 0;
    }
    __syncthreads();
    const uint32_t item = (uint32_t)__builtin_amdgcn_readfirstlane((int)ctl.item);
    if (item >= total) break;
    const Item it = pool[item];
    const uint32_t kind = it.kind & 0xff;
    int st = HSDS_OK;
    if (kind == ITEM_RAW) {
      if (w == 0) raw_copy(it, lane);
    } else if (kind == ITEM_ZLIB) {
      hz2::Job job = {(const uint8_t*)it.src, it.src_len, (uint8_t*)it.dst, it.dst_len,
                      (it.kind & ITEM_INEXACT) ? 0u : 1u, (it.kind & ITEM_INEXACT) ? &sizes[it.chunk] : nullptr,
                      item_perm(it)};
      // (only wavefront 0 reports the decoded length of an inexact item)
      if (w != 0) job.out_len = nullptr;
      st = hz2::inflate_stream_pipe<hz2::Stats, NW>(sh[w], job, tune, ring, (hz2::Stats*)nullptr, prof,
                                                    hz2::Pipe{&ctl, &sh[(w + NW - 1u) % NW], w});
    }
    if (w == 0 && lane == 0 && st != HSDS_OK) atomicMin(&status[it.chunk], st);
    __syncthreads();
  }
}

// -------------------------------------------------------------------------
// LZ4 / BloscLZ splits (lz_wave.h): persistent 64-thread workgroups over the same
// item table as inflate_kernel; a wave takes lz::GROUP consecutive items at a time
// and decodes the LZ ones among them together (one split per header-walking lane).
// -------------------------------------------------------------------------
__global__ void __launch_bounds__(64) lz_kernel(const Item* __restrict__ pool, const uint32_t* __restrict__ pool_ctr,
                                                uint32_t* __restrict__ counter,
                                                int32_t* __restrict__ status,
                                                const uint32_t* __restrict__ kind_counts) {
  __shared__ lz::Shared ls;
  __shared__ lz::Stage stg;
  if (kind_counts[0] == 0) return;
  const uint32_t total = *pool_ctr;
  const int lane = threadIdx.x;
#ifdef HZ_PROFILE
  HzProf prof_;
  for (int i = 0; i < 16; i++) prof_.acc[i] = 0;
  prof_.last = __builtin_amdgcn_s_memtime();
  prof_.cur = 0;
  HzProf* prof = &prof_;
#else
  HzProf* prof = nullptr;
#endif
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(counter, (uint32_t)lz::GROUP);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(base, 0, 64));
    if (base >= total) break;
    const uint32_t item = base + (uint32_t)lane;
    lz::LaneJob j = {nullptr, nullptr, 0u, 0u, 0u, 0u};
    uint32_t chunk = 0;
    if (lane < lz::GROUP && item < total) {
      const Item it = pool[item];
      const uint32_t kind = it.kind & 0xff;
      if (kind == ITEM_LZ4 || kind == ITEM_BLOSCLZ) {
        j = {(const uint8_t*)it.src, (uint8_t*)it.dst, it.src_len, it.dst_len,
             kind == ITEM_LZ4 ? lz::FMT_LZ4 : lz::FMT_BLOSCLZ, 1u};
        chunk = it.chunk;
      }
    }
    if (lane < lz::GROUP) ls.job[lane] = j;
    __syncthreads();
    lz::lz_group<true>(ls, &stg, prof);
    if (j.valid && ls.m_st[lane] != HSDS_OK) atomicMin(&status[chunk], ls.m_st[lane]);
    __syncthreads();
  }
#ifdef HZ_PROFILE
  {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    prof_.acc[prof_.cur] += now - prof_.last;
    if (lane == 0) for (int i = 0; i < 16; i++) atomicAdd(&hz_prof[i], (unsigned long long)prof_.acc[i]);
  }
#endif
  (void)prof;
}

// -------------------------------------------------------------------------
// zstd splits (zstd_wave.h): persistent 64-thread workgroups, one split per wave
// (tables and the sequence window in LDS, all lanes resolving the output)
// -------------------------------------------------------------------------
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HZ_ZSTD_WPE))) zstd_kernel(const Item* __restrict__ pool, const uint32_t* __restrict__ pool_ctr,
                                                  uint32_t* __restrict__ counter,
                                                  int32_t* __restrict__ status,
                                                  const uint32_t* __restrict__ kind_counts) {
  __shared__ zw::Shared ls;
  if (kind_counts[2] == 0) return;
  const uint32_t total = *pool_ctr;
  const int lane = threadIdx.x;
#ifdef HZ_PROFILE
  HzProf prof_;
  for (int i = 0; i < 16; i++) prof_.acc[i] = 0;
  prof_.last = __builtin_amdgcn_s_memtime();
  prof_.cur = 0;
  HzProf* prof = &prof_;
#else
  HzProf* prof = nullptr;
#endif
  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(counter, 1u);
    item = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(item, 0, 64));
    if (item >= total) break;
    const Item it = pool[item];
    if ((zw::uni(it.kind) & 0xff) != ITEM_ZSTD) continue;
    // the frame walk is uniform: keep its operands in scalar registers
    const uint64_t src = ((uint64_t)zw::uni((uint32_t)(it.src >> 32)) << 32) | zw::uni((uint32_t)it.src);
    const uint64_t dst = ((uint64_t)zw::uni((uint32_t)(it.dst >> 32)) << 32) | zw::uni((uint32_t)it.dst);
    const int st = zw::frame(ls, (const uint8_t*)src, zw::uni(it.src_len), (uint8_t*)dst, zw::uni(it.dst_len), prof);
    if (lane == 0 && st != HSDS_OK) atomicMin(&status[it.chunk], st);
    __syncthreads();
  }
#ifdef HZ_PROFILE
  {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    prof_.acc[prof_.cur] += now - prof_.last;
    if (lane == 0) for (int i = 0; i < 16; i++) atomicAdd(&hz_prof[i], (unsigned long long)prof_.acc[i]);
  }
#endif
  (void)prof;
}

// -------------------------------------------------------------------------
// bitshuffle+LZ4 chunks (storUtil._unshuffle codec 2, storUtil.py:144-174): persistent
// 64-thread workgroups take one chunk at a time (bshuf.h); the LZ4 blocks are staged in
// `stg` at the chunk's destination offsets, then un-transposed into dst.
// -------------------------------------------------------------------------
__global__ void __launch_bounds__(64) bshuf_kernel(const uint8_t* __restrict__ src,
                                                   const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks,
                                                   uint8_t* __restrict__ dst, uint8_t* __restrict__ stg,
                                                   int32_t* __restrict__ status, uint32_t* __restrict__ counter,
                                                   int itemsize) {
  __shared__ bs::Shared sh;
  const int lane = threadIdx.x;
  for (;;) {
    uint32_t ci = 0;
    if (lane == 0) ci = atomicAdd(counter, 1u);
    ci = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(ci, 0, 64));
    if ((int64_t)ci >= nchunks) break;
    const hsds_chunk_desc d = chunks[ci];
    int st;
    if (d.src_len > 0xffffffffull || d.dst_len > 0xffffffffull) st = HSDS_ERR_SIZE;
    else
      st = bs::chunk(sh, src + d.src_off, (uint32_t)d.src_len, dst + d.dst_off, stg + d.dst_off, (uint32_t)d.dst_len,
                     (uint32_t)itemsize);
    if (lane == 0) status[ci] = st;
    __syncthreads();
  }
}

// -------------------------------------------------------------------------
// unshuffle of staged chunks: work items = (listed chunk, 4 KiB output tile)
// -------------------------------------------------------------------------
// Byte (un)shuffle of one span (numcodecs.Shuffle / HDF5 shuffle filter): element-
// major `elem` (count = len / n elements of n bytes, then len % n tail bytes) <->
// plane-major `plane` (byte k of every element in plane k).  Word path: a thread
// owns 4 consecutive elements, reads one dword per plane (coalesced across the
// group) and writes the 4 elements as n whole dwords (16 B per lane for n = 4), a
// register byte transpose instead of per-byte gathers.  `tid`/`nthr` stride the
// groups over whatever set of threads shares the span.
template <bool UNSHUFFLE, int NT>
__device__ __forceinline__ void shuffle_span_n(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t len,
                                               uint32_t n_rt, uint64_t tid, uint64_t nthr) {
  const uint32_t n = NT ? (uint32_t)NT : n_rt;   // compile-time plane count for the common dtypes
  const uint64_t count = len / n, body = count * n;
  const bool words = n >= 2 && n <= 16 && (count & 3) == 0 && (((uintptr_t)in | (uintptr_t)out) & 3) == 0;
  uint64_t done = 0;
  if (words) {
    const uint64_t groups = count / 4;
    for (uint64_t g = tid; g < groups; g += nthr) {
      uint32_t p[16], w[16];
      if (UNSHUFFLE) {
        for (uint32_t k = 0; k < n; k++) p[k] = ((const uint32_t*)(in + k * count))[g];
        for (uint32_t i = 0; i < n; i++) w[i] = 0;
        for (uint32_t e = 0; e < 4; e++)
          for (uint32_t k = 0; k < n; k++) {
            const uint32_t ob = e * n + k;                       // output byte within the 4 elements
            w[ob >> 2] |= ((p[k] >> (8 * e)) & 0xffu) << (8 * (ob & 3));
          }
        uint32_t* o = (uint32_t*)out + g * n;
        for (uint32_t i = 0; i < n; i++) o[i] = w[i];
      } else {
        const uint32_t* ip = (const uint32_t*)in + g * n;
        for (uint32_t i = 0; i < n; i++) w[i] = ip[i];
        for (uint32_t k = 0; k < n; k++) p[k] = 0;
        for (uint32_t e = 0; e < 4; e++)
          for (uint32_t k = 0; k < n; k++) {
            const uint32_t ib = e * n + k;
            p[k] |= ((w[ib >> 2] >> (8 * (ib & 3))) & 0xffu) << (8 * e);
          }
        for (uint32_t k = 0; k < n; k++) ((uint32_t*)(out + k * count))[g] = p[k];
      }
    }
    done = body;
  }
  for (uint64_t q = done + tid; q < len; q += nthr) {
    if (q >= body) { out[q] = in[q]; continue; }
    if (UNSHUFFLE) out[q] = in[(q % n) * count + q / n];
    else out[(q % n) * count + q / n] = in[q];
  }
}

template <bool UNSHUFFLE>
__device__ __forceinline__ void shuffle_span(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t len,
                                             uint32_t n, uint64_t tid, uint64_t nthr) {
  switch (n) {
    case 2: shuffle_span_n<UNSHUFFLE, 2>(in, out, len, n, tid, nthr); break;
    case 4: shuffle_span_n<UNSHUFFLE, 4>(in, out, len, n, tid, nthr); break;
    case 8: shuffle_span_n<UNSHUFFLE, 8>(in, out, len, n, tid, nthr); break;
    default: shuffle_span_n<UNSHUFFLE, 0>(in, out, len, n, tid, nthr); break;
  }
}

__global__ void __launch_bounds__(256) unshuffle_kernel(const ChunkMeta* __restrict__ meta,
                                                        const uint32_t* __restrict__ meta_list,
                                                        const uint32_t* __restrict__ meta_count,
                                                        const int32_t* __restrict__ status) {
  const uint32_t nlist = *meta_count;
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
    const uint32_t ci = meta_list[li];
    if (status[ci] != HSDS_OK) continue;
    const ChunkMeta m = meta[ci];
    const uint8_t* in = (const uint8_t*)m.tmp;
    uint8_t* out = (uint8_t*)m.dst;
    for (uint64_t b0 = 0; b0 < m.nbytes; b0 += m.bs) {
      const uint64_t bsz = m.nbytes - b0 < m.bs ? m.nbytes - b0 : m.bs;
      if (m.mode == 1u) {
        shuffle_span<true>(in + b0, out + b0, bsz, m.ts, threadIdx.x, blockDim.x);
        continue;
      }
      // bitunshuffle (c-blosc 1.21, format version 2): the block's bsz / ts elements are
      // untransposed when their count is a multiple of 8, else the block stays as decoded;
      // bytes past the last whole element stay as decoded
      const uint32_t ne = (uint32_t)(bsz / m.ts);
      const uint32_t body = (ne & 7u) ? 0u : ne * m.ts;
      for (uint32_t q = threadIdx.x; q < ne / 8u && body; q += blockDim.x)
        bs::untrans_row(HZ_GLOBAL(hz_gcu8*, in + b0), HZ_GLOBAL(hz_gu8*, out + b0), q, ne / 8u, m.ts);
      for (uint64_t i = body + threadIdx.x; i < bsz; i += blockDim.x) out[b0 + i] = in[b0 + i];
    }
  }
}

// plain device shuffle / unshuffle of one buffer (numcodecs.Shuffle semantics)
__global__ void shuffle_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t len,
                               uint32_t n, int inverse) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nthr = (uint64_t)gridDim.x * blockDim.x;
  if (inverse) shuffle_span<true>(in, out, len, n, tid, nthr);
  else shuffle_span<false>(in, out, len, n, tid, nthr);
}

// -------------------------------------------------------------------------
// strided region copy / compare (numpy basic slicing: chunkUtil.py:882-995,
// chunk_crawl.py:118-150,395-418), as streaming kernels
//
// A record is first normalised (nreg_make): dims of count 1 dropped, an innermost dim
// that is contiguous on both sides folded into bytes, and outer dims that continue their
// inner neighbour on both sides merged into it -- a 512 x 2048-byte chunk piece of a slab
// row becomes 512 rows of one 2048-byte run, a whole contiguous chunk one run.  The work
// unit is a ROW (all dims but the innermost); a wave takes a group of rows, its lanes split
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
// -------------------------------------------------------------------------
// grid: x splits a record's row groups, y walks the records; 4 waves per block.  The
// normalised record lives in LDS (its dims are indexed at run time).
__global__ void __launch_bounds__(256) copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const hsds_copy_desc* __restrict__ descs, int64_t n,
                                                   const int32_t* __restrict__ flags) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * 4u;
  __shared__ rg::NReg sr;
  __shared__ int sok;
  for (int64_t di = blockIdx.y; di < n; di += gridDim.y) {
    if (flags && !flags[di]) continue;
    if (threadIdx.x == 0) sok = rg::nreg_make(descs[di], 1, sr);
    __syncthreads();
    if (sok) {
      const rg::Plan p = rg::plan_copy(sr);
      for (uint64_t g = wave; g < p.ngroups; g += nwaves) rg::copy_group(src, dst, sr, p, g, lane);
    }
    __syncthreads();
  }
}

// d_b: new data (desc.src_*), d_a: chunk (desc.dst_*).  Bytewise kinds compare 16-byte
// pieces of contiguous runs, float kinds element by element; a wave stops at the first
// difference it sees, every wave once its record is marked.
__global__ void __launch_bounds__(256) compare_kernel(const uint8_t* __restrict__ b, const uint8_t* __restrict__ a,
                                                      const hsds_copy_desc* __restrict__ descs, int64_t n, int kind,
                                                      int32_t* __restrict__ differs) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * 4u;
  __shared__ rg::NReg sr;
  __shared__ int sok;
  for (int64_t di = blockIdx.y; di < n; di += gridDim.y) {
    if (threadIdx.x == 0) sok = rg::nreg_make(descs[di], kind == HSDS_KIND_BYTES, sr);
    __syncthreads();
    if (sok) {
      const rg::Plan p = rg::plan_compare(sr);
      for (uint64_t g = wave; g < p.ngroups; g += nwaves) {
        if (__hip_atomic_load(&differs[di], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        const int found = rg::compare_group(b, a, sr, p, g, lane, kind);
        if (__any(found)) {
          if (lane == 0) atomicOr(&differs[di], 1);
          break;
        }
      }
    }
    __syncthreads();
  }
}

__global__ void zero_i32_kernel(int32_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}


// =========================================================================
// encode (storUtil._compress -> c-blosc 1.21 blosc_compress_ctx, zlib codec)
// =========================================================================
struct EncItem {       // 40 bytes: one zlib stream (Blosc split)
  uint64_t src;        // block base (stream input when ts == 1)
  uint32_t len;        // stream input bytes (neblock)
  uint32_t off;        // stream offset inside the (shuffled) block
  uint32_t ts;         // > 1: gather from the byte-shuffled block
  uint32_t neb;        // elements per block plane
  uint32_t chunk;
  uint32_t seg0;       // first segment, relative to the chunk's first segment
  uint32_t pad[2];
};

struct EncGeom {       // per-chunk frame geometry (plan -> layout -> raw copies)
  uint64_t nbytes;
  uint64_t bs;
  uint32_t nblocks;
  uint32_t flags;
  uint32_t ts;
  uint32_t memcpyed;
};

struct ItemOut {       // layout -> raw copies
  uint32_t pos;        // payload offset of the split in the frame
  uint32_t raw;        // 1: stored raw (c-blosc csize == neblock)
};

struct SegMeta {       // parse -> huffman
  uint32_t item;       // EncItem slot
  uint32_t seglen;
};

// c-blosc 1.21 compute_blocksize (oracle.c orc_blosc_blocksize_codec): the HCR codecs
// (zlib, lz4hc) start from 2 x L1 and double again at level 9, lz4 from L1
// (zstd: HCR sizes, but c-blosc never splits zstd blocks, so no split enlargement;
// pinned against libblosc 1.21 zstd headers, tests/test_oracle_golden.py)
__device__ __forceinline__ uint64_t enc_blocksize(int clevel, uint32_t ts, uint64_t nbytes, int hcr, int splittable = 1) {
  if (nbytes < ts) return 1;
  uint64_t bs = nbytes;
  if (nbytes >= 32 * 1024) {
    bs = hcr ? 32 * 1024 * 2 : 32 * 1024;
    switch (clevel) {
      case 0: bs /= 4; break;
      case 1: bs /= 2; break;
      case 2: break;
      case 3: bs *= 2; break;
      case 4: case 5: bs *= 4; break;
      case 6: case 7: case 8: bs *= 8; break;
      default: bs *= hcr ? 16 : 8; break;
    }
  }
  if (splittable && clevel > 0 && ts <= 16 && bs / ts >= 128) {
    if (bs > (1u << 18)) bs = 1u << 18;
    bs *= ts;
    if (bs < (1u << 16)) bs = 1u << 16;
    if (bs > 1024u * 1024u) bs = 1024u * 1024u;
  }
  if (bs > nbytes) bs = nbytes;
  if (bs > ts) bs = bs / ts * ts;
  return bs;
}

// two passes over the same split walk: fill = 0 counts every chunk's splits (and zlib
// segments) and its geometry; after the prefix sums, fill = 1 writes the splits compactly
// at offs[ci] (no per-chunk split cap: a chunk whose splits pass item_cap fails alone)
__global__ void enc_plan_kernel(const uint8_t* __restrict__ src_base, const hsds_chunk_desc* __restrict__ chunks,
                                int64_t nchunks, EncItem* __restrict__ slots, uint32_t* __restrict__ counts,
                                uint32_t* __restrict__ segcnt, EncGeom* __restrict__ geom,
                                int32_t* __restrict__ status, int clevel, int shuffle, int typesize, int cname,
                                const uint32_t* __restrict__ offs, uint32_t item_cap, int fill) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  if (fill && status[ci] != HSDS_OK) return;
  const uint64_t base_slot = fill ? offs[ci] : 0;
  const hsds_chunk_desc c = chunks[ci];
  const uint32_t ts = typesize < 1 || typesize > 255 ? 1u : (uint32_t)typesize;
  const uint64_t nbytes = c.src_len;
  int st = HSDS_OK;
  uint32_t cnt = 0, nseg = 0;
  // Blosc1 codec: zlib 3, zstd 4, lz4 / lz4hc 1, blosclz 0
  const uint32_t fmt = cname == HSDS_CNAME_ZLIB ? 3u : cname == HSDS_CNAME_ZSTD ? 4u : cname == HSDS_CNAME_BLOSCLZ ? 0u : 1u;
  const int zstd = cname == HSDS_CNAME_ZSTD;
  EncGeom g = {nbytes, 0, 0, (fmt << 5) | (shuffle ? 1u : 0u), ts, 0};
  if (c.dst_len < nbytes + 16 || nbytes >= (1ull << 31) - 16 || (c.dst_off & 3)) {
    st = HSDS_ERR_ARG;
  } else {
    const uint64_t bs = enc_blocksize(clevel, ts, nbytes, cname == HSDS_CNAME_ZLIB || cname == HSDS_CNAME_LZ4HC || zstd,
                                      !zstd);
    g.bs = bs;
    if (zstd || !(ts <= 16 && bs / ts >= 128)) g.flags |= 0x10;
    g.memcpyed = (nbytes < 128 || clevel <= 0) ? 1u : 0u;
    const uint64_t nblocks = bs ? (nbytes + bs - 1) / bs : 0;
    const uint64_t leftover = bs ? nbytes % bs : 0;
    g.nblocks = (uint32_t)nblocks;
    if (!g.memcpyed) {
      const uint8_t* csrc = src_base + c.src_off;
      const int doshuffle = (g.flags & 0x01) && ts > 1;
      for (uint64_t b = 0; b < nblocks && st == HSDS_OK; b++) {
        const int isleft = (b == nblocks - 1) && leftover;
        const uint64_t bsz = isleft ? leftover : bs;
        const uint32_t nspl = (!(g.flags & 0x10) && !isleft) ? ts : 1u;
        const uint64_t neblock = bsz / nspl;
        for (uint32_t j = 0; j < nspl; j++) {
          if (cnt == 0xffffffffu) { st = HSDS_ERR_UNSUPPORTED; break; }
          if (!fill) { cnt++; nseg += hd::nsegments((uint32_t)neblock); continue; }
          EncItem it;
          it.src = (uint64_t)(csrc + b * bs + (doshuffle ? 0 : j * neblock));
          it.len = (uint32_t)neblock;
          it.off = doshuffle ? (uint32_t)(j * neblock) : 0u;
          it.ts = doshuffle ? ts : 1u;
          it.neb = doshuffle ? (uint32_t)(bsz / ts) : 0u;
          it.chunk = (uint32_t)ci;
          it.seg0 = nseg;
          it.pad[0] = it.pad[1] = 0;
          if (base_slot + cnt < item_cap) slots[base_slot + cnt] = it;
          cnt++;
          nseg += hd::nsegments((uint32_t)neblock);
        }
      }
    }
  }
  if (fill) {
    // splits past the slot capacity: the chunk fails (its in-capacity splits stay valid
    // work items; layout and the raw copies skip a failed chunk)
    if (base_slot + cnt > item_cap) status[ci] = HSDS_ERR_UNSUPPORTED;
    return;
  }
  if (st != HSDS_OK) { cnt = 0; nseg = 0; }
  counts[ci] = cnt;
  segcnt[ci] = nseg;
  status[ci] = st;
  geom[ci] = g;
}


// P: persistent waves, one zlib stream each
__global__ void __launch_bounds__(64) parse_kernel(const EncItem* __restrict__ slots,
                                                   const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                   uint32_t* __restrict__ counter, hd::SegParse* __restrict__ sp,
                                                   SegMeta* __restrict__ meta, uint16_t* __restrict__ tok,
                                                   uint32_t* __restrict__ adler, uint32_t seg_cap, int level,
                                                   uint32_t ks, uint32_t item_cap, uint16_t* __restrict__ far,
                                                   uint32_t chain_ovr) {
  __shared__ hd::ParseShared sh;
  // far: one FARW-entry chain ring per workgroup (zlib streams: 32 KiB window), or null
  uint16_t* const my_far = far ? far + (size_t)blockIdx.x * hd::FARW : nullptr;
  const uint32_t total = offs[nchunks] < item_cap ? offs[nchunks] : item_cap;
  const int lane = threadIdx.x;
  hd::Tune tune = hd::tune_for_level(level);
  // development overrides (HSDS_DEFLATE_CHAIN, HSDS_DEFLATE_FAR): chain depth, far ring
  if (chain_ovr & 0xffffu) tune.chain = chain_ovr & 0xffffu;
  if (chain_ovr >> 16) tune.far = 1u;
#ifdef HZ_PROFILE
  HzProf prof_;
  for (int i = 0; i < 16; i++) prof_.acc[i] = 0;
  prof_.last = __builtin_amdgcn_s_memtime();
  prof_.cur = 0;
  HzProf* prof = &prof_;
#else
  HzProf* prof = nullptr;
#endif
  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(counter, 1u);
    item = __shfl(item, 0, 64);
    if (item >= total) break;
    const int64_t ci = item_chunk(offs, nchunks, item);
    // ks: slots per chunk (Blosc splits), or 0 for the compact layout (slot = item)
    const uint32_t slot = ks ? (uint32_t)(ci * ks + (item - offs[ci])) : item;
    const EncItem it = slots[slot];
    const uint32_t g0 = segoffs[ci] + it.seg0;
    const uint32_t nseg = hd::nsegments(it.len);
    if (g0 + nseg > seg_cap) continue;          // the layout phase fails the chunk
    hd::EncJob job = {(const uint8_t*)it.src, it.len, level, it.ts, it.neb, it.off};
    const uint32_t a = hd::parse_stream(sh, job, tune, sp + g0, tok + (size_t)g0 * hd::SEG_TOK, prof, my_far);
    for (uint32_t s = (uint32_t)lane; s < nseg; s += 64) {
      const uint32_t s0 = s * (uint32_t)hd::SEG;
      meta[g0 + s] = SegMeta{slot, it.len - s0 < (uint32_t)hd::SEG ? it.len - s0 : (uint32_t)hd::SEG};
    }
    if (lane == 0) adler[slot] = a;
    __syncthreads();
  }
#ifdef HZ_PROFILE
  {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    prof_.acc[prof_.cur] += now - prof_.last;
    if (lane == 0) for (int i = 0; i < 16; i++) atomicAdd(&hz_prof[i], (unsigned long long)prof_.acc[i]);
  }
#endif
  (void)prof;
}

// H: one wave per segment
#ifndef HZ_HUFF_WPE
#define HZ_HUFF_WPE 6    // 80 VGPRs: 6 waves per SIMD (4: 113 VGPRs); cfg5 deflate 236.6 -> 225.4 ms
#endif
#ifndef HZ_EMIT_WPE
#define HZ_EMIT_WPE 4
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HZ_HUFF_WPE))) huff_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                  uint32_t* __restrict__ counter,
                                                  const hd::SegParse* __restrict__ sp,
                                                  const SegMeta* __restrict__ meta, hd::SegCode* __restrict__ sc,
                                                  uint32_t seg_cap, int level) {
  __shared__ hd::HuffShared sh;
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  const int lane = threadIdx.x;
  for (;;) {
    uint32_t s = 0;
    if (lane == 0) s = atomicAdd(counter, 1u);
    s = __shfl(s, 0, 64);
    if (s >= total) break;
    hd::huff_segment(sh, sp + s, sc + s, meta[s].seglen, level <= 0);
    __syncthreads();
  }
}

// L: one thread per chunk: stream sizes -> c-blosc frame layout (serial_blosc /
// blosc_c with the raw split and memcpyed fallbacks, oracle.c orc_blosc_encode_zlib)
// -> block bit positions, frame header, bstarts, split length prefixes, zlib headers
__global__ void layout_kernel(const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks, uint8_t* dst_base,
                              const EncItem* __restrict__ slots, const uint32_t* __restrict__ counts,
                              const uint32_t* __restrict__ offs,
                              const uint32_t* __restrict__ segoffs, EncGeom* __restrict__ geom,
                              const hd::SegCode* __restrict__ sc, const uint32_t* __restrict__ adler,
                              ItemOut* __restrict__ iout, hd::SegOut* __restrict__ so, int64_t* __restrict__ sizes,
                              int32_t* __restrict__ status, uint32_t seg_cap, int level,
                              const uint32_t* __restrict__ lzsize) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  const uint32_t cnt = counts[ci];
  const uint32_t g0 = segoffs[ci], g1 = segoffs[ci + 1];
  // every segment of the chunk gets a record (E skips the ones not emitted)
  for (uint32_t s = g0; s < g1 && s < seg_cap; s++) so[s].flags = 0;
  if (status[ci] != HSDS_OK) { sizes[ci] = status[ci]; return; }
  if (g1 > seg_cap) { status[ci] = HSDS_ERR_UNSUPPORTED; sizes[ci] = HSDS_ERR_UNSUPPORTED; return; }
  const hsds_chunk_desc c = chunks[ci];
  EncGeom g = geom[ci];
  const uint32_t i0 = offs[ci];
  const EncItem* it = slots + i0;
  ItemOut* io = iout + i0;
  uint8_t* out = dst_base + c.dst_off;
  const uint64_t maxbytes = g.nbytes + 16;
  uint32_t memcpyed = g.memcpyed;
  uint64_t nt = 16 + 4ull * g.nblocks;
  if (!memcpyed && nt > maxbytes) memcpyed = 1;
  const uint64_t leftover = g.bs ? g.nbytes % g.bs : 0;
  uint32_t k = 0;
  for (uint32_t b = 0; b < g.nblocks && !memcpyed; b++) {
    const int isleft = (b == g.nblocks - 1) && leftover;
    const uint32_t nspl = (!(g.flags & 0x10) && !isleft) ? g.ts : 1u;
    for (uint32_t j = 0; j < nspl && !memcpyed; j++, k++) {
      const uint64_t neblock = it[k].len;
      nt += 4;
      int64_t maxout = (int64_t)neblock;
      if (nt + neblock > maxbytes) {
        maxout = (int64_t)maxbytes - (int64_t)nt;
        if (maxout <= 0) { memcpyed = 1; break; }
      }
      int64_t cb = lzsize ? (int64_t)lzsize[i0 + k]
                          : (int64_t)hd::stream_layout(sc + g0 + it[k].seg0, it[k].len, nullptr);
      if (cb > maxout) cb = 0;                     // compress2 / LZ4_compress would not fit
      uint32_t israw = 0;
      if (cb == 0 || (uint64_t)cb >= neblock) {    // c-blosc: csize == neblock is raw
        if (nt + neblock > maxbytes) { memcpyed = 1; break; }
        cb = (int64_t)neblock;
        israw = 1;
      }
      io[k].pos = (uint32_t)nt;
      io[k].raw = israw;
      nt += (uint64_t)cb;
    }
  }
  if (memcpyed) nt = g.nbytes + 16;
  g.memcpyed = memcpyed;
  geom[ci] = g;
  uint32_t* dw = (uint32_t*)dst_base;
  if (!memcpyed && !lzsize) {
    // block bit positions; zero the two edge words of every emitted block
    for (uint32_t kk = 0; kk < cnt; kk++) {
      if (io[kk].raw) continue;
      const hd::SegCode* scs = sc + g0 + it[kk].seg0;
      const uint32_t len = it[kk].len;
      const uint32_t nseg = hd::nsegments(len);
      const uint64_t base = (c.dst_off + io[kk].pos) * 8ull;
      uint64_t bpos = 16;
      for (uint32_t s = 0; s < nseg; s++) {
        const uint32_t s0 = s * (uint32_t)hd::SEG;
        const uint32_t seglen = len - s0 < (uint32_t)hd::SEG ? len - s0 : (uint32_t)hd::SEG;
        const uint64_t start = bpos;
        if (scs[s].btype == 0) bpos = ((bpos + 3u + 7u) & ~7ull) + 32u + 8ull * seglen;
        else bpos += scs[s].bits;
        const bool last = s + 1 == nseg;
        uint64_t end = bpos;
        if (last) end = ((bpos + 7u) & ~7ull) + 32u;
        hd::SegOut& o = so[g0 + it[kk].seg0 + s];
        o.bitpos = base + start;
        o.item = i0 + kk;
        o.seg = s;
        o.flags = 1u | (last ? 2u : 0u);
        o.adler = adler[i0 + kk];
        dw[(base + start) >> 5] = 0;
        dw[(base + end - 1) >> 5] = 0;
      }
    }
  }
  // frame header (blosc write header: version 2, versionlz 1, flags, typesize, sizes)
  const uint32_t flags = g.flags | (memcpyed ? 0x02u : 0u);
  uint8_t hdr[16] = {2, 1, (uint8_t)flags, (uint8_t)g.ts};
  for (int i = 0; i < 4; i++) {
    hdr[4 + i] = (uint8_t)(g.nbytes >> (8 * i));
    hdr[8 + i] = (uint8_t)(g.bs >> (8 * i));
    hdr[12 + i] = (uint8_t)(nt >> (8 * i));
  }
  for (int i = 0; i < 16; i++) out[i] = hdr[i];
  if (!memcpyed) {
    uint32_t kk = 0;
    for (uint32_t b = 0; b < g.nblocks; b++) {
      const int isleft = (b == g.nblocks - 1) && leftover;
      const uint32_t nspl = (!(g.flags & 0x10) && !isleft) ? g.ts : 1u;
      const uint32_t bstart = io[kk].pos - 4u;
      for (int i = 0; i < 4; i++) out[16 + 4 * b + i] = (uint8_t)(bstart >> (8 * i));
      for (uint32_t j = 0; j < nspl; j++, kk++) {
        const uint32_t p = io[kk].pos;
        const uint32_t cs = io[kk].raw ? it[kk].len
                            : lzsize ? lzsize[i0 + kk]
                                     : (uint32_t)hd::stream_layout(sc + g0 + it[kk].seg0, it[kk].len, nullptr);
        for (int i = 0; i < 4; i++) out[p - 4 + i] = (uint8_t)(cs >> (8 * i));
        if (!io[kk].raw && !lzsize) {
          out[p] = 0x78;
          out[p + 1] = (uint8_t)hd::zlib_flg(level);
        }
      }
    }
  }
  sizes[ci] = (int64_t)nt;
}

// E: one wave per segment
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HZ_EMIT_WPE))) emit_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                  uint32_t* __restrict__ counter,
                                                  const hd::SegOut* __restrict__ so,
                                                  const hd::SegCode* __restrict__ sc,
                                                  const hd::SegParse* __restrict__ sp,
                                                  const uint16_t* __restrict__ tok,
                                                  const EncItem* __restrict__ slots, uint32_t* dst_words,
                                                  uint32_t seg_cap, int level) {
  __shared__ hd::EmitShared sh;
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  const int lane = threadIdx.x;
  for (;;) {
    uint32_t s = 0;
    if (lane == 0) s = atomicAdd(counter, 1u);
    s = __shfl(s, 0, 64);
    if (s >= total) break;
    const hd::SegOut o = so[s];
    if (!(o.flags & 1u)) continue;
    const EncItem it = slots[o.item];
    hd::EncJob job = {(const uint8_t*)it.src, it.len, level, it.ts, it.neb, it.off};
    hd::emit_segment(sh, o, sc + s, sp + s, tok + (size_t)s * hd::SEG_TOK, job, dst_words);
    __syncthreads();
  }
}

// LZ4 write path (lz4_enc.h): one wavefront per split walks its parse tokens (each
// lane its own token range), first for the block size (-> layout_kernel), then to
// write the block into the frame
__global__ void __launch_bounds__(64) lz4_block_kernel(const EncItem* __restrict__ slots,
                                                       const uint32_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                       const hd::SegParse* __restrict__ sp,
                                                       const uint16_t* __restrict__ tok,
                                                       uint32_t* __restrict__ lzsize, uint32_t seg_cap, int level,
                                                       const hsds_chunk_desc* __restrict__ chunks, uint8_t* dst_base,
                                                       const EncGeom* __restrict__ geom,
                                                       const ItemOut* __restrict__ iout,
                                                       const int32_t* __restrict__ status, int write, int blosclz,
                                                       uint32_t ks, uint32_t item_cap) {
  __shared__ lze::CopyList cl;
  if (threadIdx.x == 0) cl.n = 0;
  __syncthreads();
  const uint32_t total = offs[nchunks] < item_cap ? offs[nchunks] : item_cap;
  for (uint32_t item = blockIdx.x; item < total; item += gridDim.x) {
    const int64_t ci = item_chunk(offs, nchunks, item);
    const uint32_t slot = ks ? (uint32_t)(ci * ks + (item - offs[ci])) : item;
    const EncItem it = slots[slot];
    const uint32_t g0 = segoffs[ci] + it.seg0;
    if (g0 + hd::nsegments(it.len) > seg_cap) continue;   // the layout phase fails the chunk
    hd::EncJob job = {(const uint8_t*)it.src, it.len, level, it.ts, it.neb, it.off};
    if (!write) {
      const uint32_t sz = blosclz ? lze::blosclz_block_wave(sp + g0, tok + (size_t)g0 * hd::SEG_TOK, job, nullptr, 0)
                                  : lze::lz4_block_wave(sp + g0, tok + (size_t)g0 * hd::SEG_TOK, job, nullptr, 0);
      if (threadIdx.x == 0) lzsize[slot] = sz;
    } else {
      if (status[ci] != HSDS_OK || geom[ci].memcpyed || iout[slot].raw) continue;
      uint8_t* o = dst_base + chunks[ci].dst_off + iout[slot].pos;
      if (blosclz) lze::blosclz_block_wave(sp + g0, tok + (size_t)g0 * hd::SEG_TOK, job, o, 1);
      else lze::lz4_block_wave(sp + g0, tok + (size_t)g0 * hd::SEG_TOK, job, o, 1, &cl);
    }
  }
}

// zstd write path (zstd_enc.h): one lane per 8 KiB segment writes that segment as one zstd
// block into its scratch slot; zstd_size_kernel sums a stream's blocks for the layout;
// zstd_write_kernel (one wave per stream) writes the frame header and moves the blocks
__global__ void __launch_bounds__(64) zstd_lit_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                      const hd::SegParse* __restrict__ sp,
                                                      const uint16_t* __restrict__ tok, uint8_t* __restrict__ lsec,
                                                      uint32_t* __restrict__ lsz, uint32_t seg_cap) {
  __shared__ hze::LitShared sh;
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  for (uint32_t s = blockIdx.x; s < total; s += gridDim.x) {
    const uint32_t n = hze::lit_section(sh, tok + (size_t)s * hd::SEG_TOK, sp + s, lsec + (size_t)s * hze::LCAP);
    if (threadIdx.x == 0) lsz[s] = n;
    __syncthreads();
  }
}

// zstd sequence tables, one FSE_Compressed_Mode set per frame (zstd_enc.h frame_tables):
// zstd_count_kernel adds every segment's sequence codes to its frame's counts (lane per
// segment; the counts of the first ZT_SLOTS frames of the wave's segments gather in LDS),
// zstd_table_kernel builds each frame's tables and descriptions (thread per frame), and
// zstd_seg_kernel encodes every block of a frame with them, ZT_SLOTS frames' tables in LDS
// at a time (round 4's predefined tables made the objects 1.24x libblosc-zstd's)
constexpr uint32_t ZT_SLOTS = 4;
constexpr uint32_t ZT_NCODE = sizeof(hze::SeqCounts) / 4u;
static_assert(ZT_NCODE == 36u + 32u + 53u, "SeqCounts: ll, of, ml codes");
// zstd_count_kernel: one workgroup per ZC_SEGS consecutive segments, one lane per parse
// lane of a segment: lane l walks its own token slots forward (the slots are interleaved by
// parse lane, so the 64 lanes' loads are one coalesced 256-byte row), counting the codes of
// its matches; the literal run of a lane's first match continues from earlier lanes (its
// literal ordinal minus the ordinal after the nearest earlier match: an add scan and a max
// scan over the lanes).  Each lane keeps its own counters in LDS (two 16-bit counts per
// dword, code-major: no atomic contention, distinct banks); they go to the frame's counts in
// HBM whenever the frame changes.  (A lane per segment walking all 64 columns serially
// took 34 ms on the cfg5 slab: every load touched 64 lines.)
constexpr uint32_t ZT_NW = (ZT_NCODE + 1u) / 2u;
constexpr uint32_t ZC_SEGS = 8;
__global__ void __launch_bounds__(64) zstd_count_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                        const SegMeta* __restrict__ meta,
                                                        const hd::SegParse* __restrict__ sp,
                                                        const uint16_t* __restrict__ tok,
                                                        hze::SeqCounts* __restrict__ counts, uint32_t seg_cap) {
  __shared__ uint32_t c[ZT_NW][64];
  __shared__ hze::CodeTabs ct;
  const uint32_t l = threadIdx.x;
  for (uint32_t k = l; k < ZT_NW * 64u; k += 64u) (&c[0][0])[k] = 0;
  hze::code_tabs_fill(ct, l, 64u);
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  const uint32_t sa = blockIdx.x * ZC_SEGS;
  if (sa >= total) return;
  const uint32_t sb = sa + ZC_SEGS < total ? sa + ZC_SEGS : total;
  __syncthreads();
  auto add = [&](uint32_t code) { atomicAdd(&c[code >> 1][l], (code & 1u) ? 0x10000u : 1u); };
  auto flush = [&](uint32_t item) {
    __syncthreads();
    if (l < ZT_NW) {
      uint32_t a = 0, b = 0;
      for (uint32_t k = 0; k < 64u; k++) {
        const uint32_t v = c[l][k];
        a += v & 0xffffu;
        b += v >> 16;
        c[l][k] = 0;
      }
      uint32_t* const dst = (uint32_t*)&counts[item];
      if (a) atomicAdd(dst + 2u * l, a);
      if (b && 2u * l + 1u < ZT_NCODE) atomicAdd(dst + 2u * l + 1u, b);
    }
    __syncthreads();
  };
  uint32_t cur = meta[sa].item;
  for (uint32_t s = sa; s < sb; s++) {
    const uint32_t item = meta[s].item;
    if (item != cur) { flush(cur); cur = item; }
    hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, tok + (size_t)s * hd::SEG_TOK);
    const hze::LaneCount r = hze::lane_count(ct, gw, sp[s].nslot[l], l, add);
    // literal ordinals: L = before this lane, q = after its last match (0: none before)
    const uint32_t L = hz::wave_incl_scan_dpp(r.lits) - r.lits;
    const uint32_t qprev = hz::wave_excl_max(hze::lane_q(L, r), (int)l);
    if (r.hm) add(hze::make_seq_t(ct, hze::first_run(L, r, qprev), 3u, 1u).llc);
  }
  flush(cur);
}

// zstd_seq_kernel: the compact sequence array of every segment, one wave per segment, each
// lane on its own parse lane (zstd_enc.h "the compact sequences"); the raw literals section
// straight into the segment's block scratch (levels below 6).  Runs after zstd_count_kernel and
// zstd_lit_kernel: the sequences overwrite the token slots they read.
__global__ void __launch_bounds__(64) zstd_seq_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                      const hd::SegParse* __restrict__ sp, uint16_t* __restrict__ tok,
                                                      uint8_t* __restrict__ zscr, const uint32_t* __restrict__ lsz,
                                                      uint32_t seg_cap) {
  __shared__ uint32_t sa[hze::SEQ_MAX];
  __shared__ uint16_t sb[hze::SEQ_MAX];
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  const uint32_t l = threadIdx.x;
  for (uint32_t s = blockIdx.x; s < total; s += gridDim.x) {
    uint16_t* const ts = tok + (size_t)s * hd::SEG_TOK;
    hz_gcu32* const gw = HZ_GLOBAL(hz_gcu32*, ts);
    const uint32_t ns = sp[s].nslot[l];
    const hze::LaneSeq r = hze::lane_seq_count<16>(gw, ns, l);
    const uint32_t Li = hz::wave_incl_scan_dpp(r.lits), Si = hz::wave_incl_scan_dpp(r.nm);
    const uint32_t L = Li - r.lits, S = Si - r.nm;
    const uint32_t qprev = hz::wave_excl_max(r.hm ? Li - r.run : 0u, (int)l);
    const uint32_t nlit = (uint32_t)__builtin_amdgcn_readlane((int)Li, 63);
    const uint32_t nseq = (uint32_t)__builtin_amdgcn_readlane((int)Si, 63);
    // the raw literals section (levels below 6): its header after the block header's 3 bytes
    // (encode_segment writes those last), then every lane's literal bytes at their offsets
    const bool raw = lsz[s] == 0u;
    uint8_t h[3] = {0, 0, 0};
    const uint32_t p0 = 3u + hze::lit_header(nlit, h);
    uint8_t* const blk = zscr + (size_t)s * hze::ZCAP;
    if (raw && l < p0 - 3u) blk[3u + l] = l == 0u ? h[0] : l == 1u ? h[1] : h[2];
    hze::lane_seq_emit<16>(gw, ns, l, L + r.lead - qprev,
                           [&](uint32_t k, uint32_t v) { if (raw) blk[p0 + L + k] = (uint8_t)v; },
                           [&](uint32_t j, uint32_t run, uint32_t ml, uint32_t off) {
                             sa[S + j] = run | (ml << 16);
                             sb[S + j] = (uint16_t)(off - 1u);
                           });
    __syncthreads();            // every lane's slot reads are done: the sequences may overwrite them
    uint32_t* const ga = hze::seq_a(ts);
    uint16_t* const gb = hze::seq_b(ts);
    for (uint32_t i = l; i < nseq; i += 64u) { ga[i] = sa[i]; gb[i] = sb[i]; }
    __syncthreads();            // (the LDS of the next segment)
  }
}

__global__ void zstd_table_kernel(const uint32_t* __restrict__ offs, int64_t nchunks,
                                  const hze::SeqCounts* __restrict__ counts, hze::Tabs* __restrict__ tabs,
                                  uint32_t item_cap) {
  const uint32_t total = offs[nchunks] < item_cap ? offs[nchunks] : item_cap;
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= total) return;
  hze::build_all(tabs[item]);      // (the predefined tables of a code type with < 2 distinct codes)
  hze::frame_tables(tabs[item], counts[item]);
}

__global__ void __launch_bounds__(64) zstd_seg_kernel(const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                      const SegMeta* __restrict__ meta,
                                                      const EncItem* __restrict__ slots,
                                                      const hd::SegParse* __restrict__ sp,
                                                      const uint16_t* __restrict__ tok, uint8_t* __restrict__ zscr,
                                                      uint32_t* __restrict__ zsz, const uint8_t* __restrict__ lsec,
                                                      const uint32_t* __restrict__ lsz, uint32_t seg_cap, int level,
                                                      const hze::Tabs* __restrict__ tabs) {
  __shared__ hze::Tabs T[ZT_SLOTS];
  __shared__ hze::CodeTabs ct;
  hze::code_tabs_fill(ct, threadIdx.x, 64u);
  uint32_t total = segoffs[nchunks];
  if (total > seg_cap) total = seg_cap;
  const uint32_t s0 = blockIdx.x * 64u;
  if (s0 >= total) return;
  const uint32_t s = s0 + threadIdx.x;
  const uint32_t base = meta[s0].item;
  const uint32_t nframes = meta[(s0 + 64u < total ? s0 + 64u : total) - 1u].item - base + 1u;
  // the wave's segments span nframes frames: their tables go to LDS ZT_SLOTS at a time
  for (uint32_t f0 = 0; f0 < nframes; f0 += ZT_SLOTS) {
    __syncthreads();
    const uint32_t nf = nframes - f0 < ZT_SLOTS ? nframes - f0 : ZT_SLOTS;
    constexpr uint32_t TW = sizeof(hze::Tabs) / 4u;
    static_assert(sizeof(hze::Tabs) % 4u == 0u, "Tabs: whole dwords");
    for (uint32_t k = threadIdx.x; k < nf * TW; k += 64u)
      ((uint32_t*)&T[0])[k] = ((const uint32_t*)&tabs[base + f0])[k];
    __syncthreads();
    if (s >= total) continue;
    const SegMeta m = meta[s];
    if (m.item < base + f0 || m.item >= base + f0 + nf) continue;
    const EncItem it = slots[m.item];
    const uint32_t g0 = segoffs[it.chunk] + it.seg0;
    const uint32_t seg = s - g0;
    hd::EncJob job = {(const uint8_t*)it.src, it.len, level, it.ts, it.neb, it.off};
    const uint32_t last = seg + 1 == hd::nsegments(it.len) ? 1u : 0u;
    zsz[s] = hze::encode_segment(T[m.item - base - f0], ct, tok + (size_t)s * hd::SEG_TOK, sp + s, job,
                                 seg * (uint32_t)hd::SEG, m.seglen, last, zscr + (size_t)s * hze::ZCAP, hze::ZCAP,
                                 lsec + (size_t)s * hze::LCAP, lsz[s], 1);
  }
}

__global__ void zstd_size_kernel(const uint32_t* __restrict__ offs, const uint32_t* __restrict__ segoffs,
                                 int64_t nchunks, const EncItem* __restrict__ slots, const uint32_t* __restrict__ zsz,
                                 uint32_t* __restrict__ lzsize, uint32_t seg_cap, uint32_t item_cap) {
  const uint32_t total = offs[nchunks] < item_cap ? offs[nchunks] : item_cap;
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= total) return;
  const EncItem it = slots[item];
  const uint32_t g0 = segoffs[it.chunk] + it.seg0, ns = hd::nsegments(it.len);
  if (g0 + ns > seg_cap) { lzsize[item] = 0xffffffffu; return; }
  uint64_t sz = hze::frame_header_size(it.len);
  for (uint32_t k = 0; k < ns; k++) sz += zsz[g0 + k];
  lzsize[item] = sz < 0xffffffffull ? (uint32_t)sz : 0xffffffffu;
}

__global__ void __launch_bounds__(64) zstd_write_kernel(const uint32_t* __restrict__ offs,
                                                        const uint32_t* __restrict__ segoffs, int64_t nchunks,
                                                        const EncItem* __restrict__ slots,
                                                        const uint8_t* __restrict__ zscr,
                                                        const uint32_t* __restrict__ zsz,
                                                        const hsds_chunk_desc* __restrict__ chunks, uint8_t* dst_base,
                                                        const EncGeom* __restrict__ geom,
                                                        const ItemOut* __restrict__ iout,
                                                        const int32_t* __restrict__ status, uint32_t seg_cap,
                                                        uint32_t item_cap) {
  const uint32_t total = offs[nchunks] < item_cap ? offs[nchunks] : item_cap;
  for (uint32_t item = blockIdx.x; item < total; item += gridDim.x) {
    const EncItem it = slots[item];
    const int64_t ci = it.chunk;
    if (status[ci] != HSDS_OK || geom[ci].memcpyed || iout[item].raw) continue;
    const uint32_t g0 = segoffs[ci] + it.seg0, ns = hd::nsegments(it.len);
    if (g0 + ns > seg_cap) continue;
    uint8_t* o = dst_base + chunks[ci].dst_off + iout[item].pos;
    uint8_t hdr[16];
    const uint32_t h = hze::frame_header(hdr, it.len);
    if (threadIdx.x < h) o[threadIdx.x] = hdr[threadIdx.x];
    uint64_t p = h;
    for (uint32_t k = 0; k < ns; k++) {
      const uint32_t n = zsz[g0 + k];
      const uint8_t* src = zscr + (size_t)(g0 + k) * hze::ZCAP;
      for (uint32_t i = threadIdx.x; i < n; i += 64u) o[p + i] = src[i];
      p += n;
    }
  }
}

// bounded unaligned 32-bit load: bytes [p, p+4) of a buffer whose valid bytes are [b, e)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p, const uint8_t* b, const uint8_t* e) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
  const uint32_t s = (uint32_t)((uintptr_t)p & 3u) * 8u;
  const uint8_t* ab = (const uint8_t*)((uintptr_t)b & ~(uintptr_t)3);
  const uint32_t lo = (uint32_t)((uintptr_t)b - (uintptr_t)ab), hi = (uint32_t)((uintptr_t)e - (uintptr_t)ab);
  hz_gcu8* g = HZ_GLOBAL(hz_gcu8*, ab);
  const uint32_t k = (uint32_t)((a - (uintptr_t)ab) >> 2);
  const uint32_t w0 = hz::load_word(g, k, lo, hi);
  if (!s) return w0;
  const uint32_t w1 = hz::load_word(g, k + 1u, lo, hi);
  return (w0 >> s) | (w1 << (32u - s));
}

// workgroup copy of n bytes, any alignment of either side; ts > 1 gathers the bytes
// [off, off + n) of the byte-shuffled block at src (c-blosc raw split of a shuffled block)
__device__ void wg_copy(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t ts, uint32_t neb, uint32_t off) {
  if (ts > 1) {
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x)
      dst[i] = src[hd::shuffled_src_index(off + (uint32_t)i, ts, neb)];
    return;
  }
  uint64_t head = (4u - ((uintptr_t)dst & 3u)) & 3u;
  if (head > n) head = n;
  if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
  const uint64_t nw = (n - head) >> 2;
  uint32_t* d4 = (uint32_t*)(dst + head);
  const uint8_t* s = src + head;
  const uint8_t* e = src + n;
  if (((uintptr_t)s & 3u) == 0) {
    const uint32_t* s4 = (const uint32_t*)s;
    for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x) d4[w] = s4[w];
  } else {
    for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x) d4[w] = ld32u(s + 4 * w, src, e);
  }
  const uint64_t t0 = head + 4 * nw;
  if (t0 + threadIdx.x < n) dst[t0 + threadIdx.x] = src[t0 + threadIdx.x];
}

// R: one workgroup per chunk: raw splits and memcpyed frames
__global__ void __launch_bounds__(256) raw_copy_kernel(const uint8_t* __restrict__ src_base,
                                                       const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks,
                                                       uint8_t* dst_base, const EncItem* __restrict__ slots,
                                                       const uint32_t* __restrict__ counts,
                                                       const uint32_t* __restrict__ offs,
                                                       const EncGeom* __restrict__ geom,
                                                       const ItemOut* __restrict__ iout,
                                                       const int32_t* __restrict__ status) {
  const int64_t ci = blockIdx.x;
  if (ci >= nchunks || status[ci] != HSDS_OK) return;
  const hsds_chunk_desc c = chunks[ci];
  const EncGeom g = geom[ci];
  uint8_t* out = dst_base + c.dst_off;
  if (g.memcpyed) {
    wg_copy(out + 16, src_base + c.src_off, g.nbytes, 1, 0, 0);
    return;
  }
  const uint32_t cnt = counts[ci];
  const EncItem* it = slots + offs[ci];
  const ItemOut* io = iout + offs[ci];
  for (uint32_t k = 0; k < cnt; k++)
    if (io[k].raw) wg_copy(out + io[k].pos, (const uint8_t*)it[k].src, it[k].len, it[k].ts, it[k].neb, it[k].off);
}

// -------------------------------------------------------------------------
// bitshuffle+LZ4 write path (storUtil._shuffle codec 2, storUtil.py:103-131 ->
// bitshuffle.compress_lz4): plan -> scan -> fill (one LZ4 item per block, compact slot
// layout) -> forward bit transposition into a staging copy -> parse -> LZ4 size pass ->
// layout (12-byte header, u32 BE block sizes, raw n % 8 leftover) -> LZ4 write pass.
// EncGeom reuse: nbytes = chunk bytes, bs = block elements, nblocks = full blocks,
// ts = itemsize, flags = elements of the last (partial) block.
// -------------------------------------------------------------------------
constexpr int BSHUF_PARSE_LEVEL = 1;   // one hash candidate per position, as LZ4_compress_default

// compact staging: exclusive prefix of the chunks' 16-byte aligned source lengths (one
// workgroup of 1024), soffs[n] = total
__global__ void stage_scan_kernel(const hsds_chunk_desc* __restrict__ chunks, int64_t n, uint64_t* __restrict__ soffs) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const uint64_t v = i < n ? ((chunks[i].src_len + 15) & ~15ull) : 0ull;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const uint64_t y = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0ull;
      __syncthreads();
      part[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < n) soffs[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) soffs[n] = carry;
}

__global__ void bs_plan_kernel(const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks,
                               uint32_t* __restrict__ counts, uint32_t* __restrict__ segcnt,
                               EncGeom* __restrict__ geom, int32_t* __restrict__ status, uint32_t es,
                               uint32_t block, uint64_t src_extent) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  const hsds_chunk_desc c = chunks[ci];
  const uint64_t n = c.src_len;
  const uint32_t bsz = block ? block : bs::default_block(es);
  EncGeom g = {n, bsz, 0, 0, es, 0};
  int st = HSDS_OK;
  uint32_t cnt = 0, nseg = 0;
  if (n % es || c.src_off > src_extent || n > src_extent - c.src_off || n >= (1ull << 31) - 64 || c.dst_len < 12) {
    st = HSDS_ERR_ARG;
  } else {
    const uint32_t nel = (uint32_t)(n / es);
    const uint32_t nfull = nel / bsz;
    const uint32_t last = (nel - nfull * bsz) / 8u * 8u;
    g.nblocks = nfull;
    g.flags = last;
    cnt = nfull + (last ? 1u : 0u);
    nseg = nfull * hd::nsegments(bsz * es) + (last ? hd::nsegments(last * es) : 0u);
  }
  counts[ci] = cnt;
  segcnt[ci] = nseg;
  status[ci] = st;
  geom[ci] = g;
}

// one thread per chunk: the chunk's LZ4 items at slots[offs[ci] ..] (those below
// slot_cap; a chunk that crosses it fails)
__global__ void bs_fill_kernel(const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks,
                               const uint32_t* __restrict__ offs, const EncGeom* __restrict__ geom,
                               EncItem* __restrict__ slots, int32_t* __restrict__ status, const uint8_t* stg,
                               uint32_t slot_cap, const uint64_t* __restrict__ soffs, uint64_t stg_bytes) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  const EncGeom g = geom[ci];
  const uint32_t o0 = offs[ci], o1 = offs[ci + 1];
  if (o1 > slot_cap && status[ci] == HSDS_OK) status[ci] = HSDS_ERR_UNSUPPORTED;
  if (soffs[ci] + chunks[ci].src_len > stg_bytes && status[ci] == HSDS_OK) status[ci] = HSDS_ERR_ARG;
  const uint64_t bbytes = g.bs * g.ts;
  const uint32_t segs_full = hd::nsegments((uint32_t)bbytes);
  for (uint32_t k = 0; k < o1 - o0 && o0 + k < slot_cap; k++) {
    EncItem it;
    it.src = (uint64_t)(stg + soffs[ci] + k * bbytes);
    it.len = k < g.nblocks ? (uint32_t)bbytes : g.flags * g.ts;
    it.off = 0;
    it.ts = 1;
    it.neb = 0;
    it.chunk = (uint32_t)ci;
    it.seg0 = k * segs_full;
    it.pad[0] = it.pad[1] = 0;
    slots[o0 + k] = it;
  }
}

// forward bit transposition of every block: work item = 8 elements (one row byte q)
__global__ void __launch_bounds__(256) bs_trans_kernel(const uint8_t* __restrict__ src,
                                                       const hsds_chunk_desc* __restrict__ chunks, int64_t nchunks,
                                                       const EncGeom* __restrict__ geom,
                                                       const int32_t* __restrict__ status, uint8_t* __restrict__ stg,
                                                       const uint64_t* __restrict__ soffs) {
  for (int64_t ci = blockIdx.y; ci < nchunks; ci += gridDim.y) {
    if (status[ci] != HSDS_OK) continue;
    const EncGeom g = geom[ci];
    const uint32_t bsz = (uint32_t)g.bs, es = g.ts;
    const uint32_t nq = (g.nblocks * bsz + g.flags) / 8u;
    const uint64_t base = chunks[ci].src_off, sbase = soffs[ci];
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
      const uint32_t e0 = q * 8u, b = e0 / bsz;
      const uint32_t cnt = b < g.nblocks ? bsz : g.flags;
      const uint64_t boff = (uint64_t)b * bsz * es;
      bs::trans_group(HZ_GLOBAL(hz_gcu8*, src + base + boff), HZ_GLOBAL(hz_gu8*, stg + sbase + boff),
                      (e0 - b * bsz) / 8u, cnt / 8u, es);
    }
  }
}

// one thread per chunk: LZ4 block sizes -> frame positions, header, u32 BE sizes, raw
// leftover elements, frame size (or HSDS_ERR_SIZE when it exceeds dst_len)
__global__ void bs_layout_kernel(const uint8_t* __restrict__ src, const hsds_chunk_desc* __restrict__ chunks,
                                 int64_t nchunks, uint8_t* __restrict__ dst_base, const uint32_t* __restrict__ offs,
                                 const uint32_t* __restrict__ segoffs, const EncGeom* __restrict__ geom,
                                 const uint32_t* __restrict__ lzsize, ItemOut* __restrict__ iout,
                                 int64_t* __restrict__ sizes, int32_t* __restrict__ status, uint32_t hdr_block,
                                 uint32_t seg_cap) {
  const int64_t ci = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  sizes[ci] = 0;
  if (status[ci] != HSDS_OK) return;
  if (segoffs[ci + 1] > seg_cap) { status[ci] = HSDS_ERR_UNSUPPORTED; return; }
  const hsds_chunk_desc c = chunks[ci];
  const EncGeom g = geom[ci];
  const uint32_t o0 = offs[ci], o1 = offs[ci + 1];
  uint64_t pos = 12;
  for (uint32_t k = o0; k < o1; k++) {
    iout[k] = ItemOut{(uint32_t)(pos + 4), 0u};
    pos += 4 + (uint64_t)lzsize[k];
  }
  const uint64_t done = ((uint64_t)g.nblocks * g.bs + g.flags) * g.ts;
  const uint64_t left = g.nbytes - done;
  const uint64_t total = pos + left;
  if (total > c.dst_len || total > 0xffffffffull) { status[ci] = HSDS_ERR_SIZE; return; }
  uint8_t* out = dst_base + c.dst_off;
  for (int i = 0; i < 8; i++) out[i] = (uint8_t)(g.nbytes >> (56 - 8 * i));        // storUtil.py:127
  for (int i = 0; i < 4; i++) out[8 + i] = (uint8_t)(hdr_block >> (24 - 8 * i));    // storUtil.py:128
  for (uint32_t k = o0; k < o1; k++) {
    const uint32_t p = iout[k].pos - 4, v = lzsize[k];
    out[p] = (uint8_t)(v >> 24); out[p + 1] = (uint8_t)(v >> 16); out[p + 2] = (uint8_t)(v >> 8); out[p + 3] = (uint8_t)v;
  }
  for (uint64_t i = 0; i < left; i++) out[pos + i] = src[c.src_off + done + i];
  sizes[ci] = (int64_t)total;
}

}  // namespace

// =========================================================================
// engine
// =========================================================================
struct hsds_engine {
  int device;
  int num_cus;
  int inflate_blocks_per_cu;   // occupancy of inflate2_kernel
  int inflate2w_blocks_per_cu; // occupancy of inflate2w_kernel<2> (two wavefronts per workgroup)
  int inflate4w_blocks_per_cu; // occupancy of inflate2w_kernel<4>
  int inflate8w_blocks_per_cu; // occupancy of inflate2w_kernel<8>
  int inflate_pipe;            // wavefronts per stream: 0 by batch size, else 1, 2 or 4
  int lz_blocks_per_cu;        // occupancy of lz_kernel
  int bshuf_blocks_per_cu;     // occupancy of bshuf_kernel
  int zstd_blocks_per_cu;      // occupancy of zstd_kernel
  int lz4w_blocks_per_cu = 16; // occupancy of lz4_block_kernel (LZ4 / BloscLZ writer)
  hz2::Tune tune;
  // workspace (grown on demand)
  uint8_t* ws = nullptr;
  size_t ws_bytes = 0;
  uint8_t* rings = nullptr;    // inflate2 match rings, one per resident wave
  size_t rings_bytes = 0;
  uint8_t* tmp = nullptr;
  size_t tmp_bytes = 0;
  // host staging for the single-chunk host API
  uint8_t* h_dev_src = nullptr;
  size_t h_dev_src_bytes = 0;
  uint8_t* h_dev_dst = nullptr;
  size_t h_dev_dst_bytes = 0;
  hipEvent_t ev0, ev1;
  int ev_valid = 0;
  // encode workspace (items, sizes, geometry) and per-split output scratch
  int parse_blocks_per_cu = 1;
  int zlit_blocks_per_cu = 1;
  int huff_blocks_per_cu = 1;
  int emit_blocks_per_cu = 1;
  uint8_t* ews = nullptr;
  size_t ews_bytes = 0;
  uint8_t* ecw = nullptr;      // encode: per-chunk plan arrays
  size_t ecw_bytes = 0;
  uint8_t* escr = nullptr;
  size_t escr_bytes = 0;
  uint8_t* efar = nullptr;     // encode: zlib parse far-chain rings, one per parse workgroup
  size_t efar_bytes = 0;
  uint8_t* ezs = nullptr;      // encode: zstd block scratch (one ZCAP slot + size per segment)
  size_t ezs_bytes = 0;
  uint32_t enc_chain = 0;      // development overrides: parse chain depth (bits 0-15, 0: the level's),
                               // far ring at any level (bit 16)
  hipEvent_t ev2, ev3;
  int ev_enc_valid = 0;
  // re-entrancy (SURVEY 8b "Threading"): every entry point that uses the workspace holds mu
  // while it enqueues, and a call on another stream first waits for the workspace's last
  // use (ws_ev) -- so a DN running calls from a thread pool, on any streams, never races
  std::recursive_mutex mu;
  hipEvent_t ws_ev;
  hipStream_t ws_st = nullptr;
  int ws_ev_valid = 0;
};

// holds the engine for one workspace use on `stream` (see hsds_engine::mu)
struct WsGuard {
  hsds_engine* e;
  hipStream_t st;
  WsGuard(hsds_engine* e_, void* stream) : e(e_), st((hipStream_t)stream) {
    e->mu.lock();
    if (e->ws_ev_valid && e->ws_st != st) hipStreamWaitEvent(st, e->ws_ev, 0);
  }
  ~WsGuard() {
    hipEventRecord(e->ws_ev, st);
    e->ws_st = st;
    e->ws_ev_valid = 1;
    e->mu.unlock();
  }
  WsGuard(const WsGuard&) = delete;
  WsGuard& operator=(const WsGuard&) = delete;
};

static int grow(void** p, size_t* have, size_t need) {
  if (*have >= need) return 0;
  if (*p) hipFree(*p);
  *p = nullptr;
  *have = 0;
  size_t sz = need + need / 4 + 4096;
  if (hipMalloc(p, sz) != hipSuccess) return HSDS_ERR_DEVICE;
  *have = sz;
  return 0;
}

// ---- host: MD5 (RFC 1321) for the chunk -> GPU partition rule (idUtil.getIdHash) ----
namespace {
struct Md5 {
  uint32_t a, b, c, d;
};
inline uint32_t rotl32(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
void md5_block(Md5& h, const uint8_t* p) {
  static const uint32_t K[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
      0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
      0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
      0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
      0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
      0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
      0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
  static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                            5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                            4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                            6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
  uint32_t m[16];
  for (int i = 0; i < 16; i++) m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) |
                                      ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
  uint32_t a = h.a, b = h.b, c = h.c, d = h.d;
  for (int i = 0; i < 64; i++) {
    uint32_t f;
    int g;
    if (i < 16) { f = (b & c) | (~b & d); g = i; }
    else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
    else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
    else { f = c ^ (b | ~d); g = (7 * i) & 15; }
    const uint32_t t = d;
    d = c; c = b;
    b = b + rotl32(a + f + K[i] + m[g], R[i]);
    a = t;
  }
  h.a += a; h.b += b; h.c += c; h.d += d;
}
// first 20 bits of md5(msg) (the 5 hex digits of getIdHash)
uint32_t md5_prefix20(const uint8_t* msg, size_t n) {
  Md5 h = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
  size_t i = 0;
  for (; i + 64 <= n; i += 64) md5_block(h, msg + i);
  uint8_t tail[128] = {0};
  const size_t r = n - i;
  memcpy(tail, msg + i, r);
  tail[r] = 0x80;
  const size_t tl = r + 9 <= 64 ? 64 : 128;
  const uint64_t bits = (uint64_t)n * 8u;
  for (int k = 0; k < 8; k++) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
  md5_block(h, tail);
  if (tl == 128) md5_block(h, tail + 64);
  const uint32_t b0 = h.a & 0xff, b1 = (h.a >> 8) & 0xff, b2 = (h.a >> 16) & 0xff;
  return (b0 << 12) | (b1 << 4) | (b2 >> 4);
}
}  // namespace

extern "C" {

const char* hsds_version(void) { return HSDS_VERSION; }

const char* hsds_strerror(int s) {
  switch (s) {
    case HSDS_OK: return "ok";
    case HSDS_ERR_FRAME: return "malformed Blosc frame";
    case HSDS_ERR_DATA: return "corrupt deflate stream";
    case HSDS_ERR_TRUNC: return "truncated stream";
    case HSDS_ERR_SIZE: return "decoded size mismatch";
    case HSDS_ERR_UNSUPPORTED: return "unsupported codec or layout";
    case HSDS_ERR_ARG: return "invalid argument";
    case HSDS_ERR_DEVICE: return "HIP runtime error";
    default: return "unknown status";
  }
}

int hsds_engine_create(int device, hsds_engine** out) {
  if (!out) return HSDS_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return HSDS_ERR_DEVICE;
  hsds_engine* e = new (std::nothrow) hsds_engine();
  if (!e) return HSDS_ERR_DEVICE;
  e->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete e; return HSDS_ERR_DEVICE; }
  e->num_cus = prop.multiProcessorCount;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, inflate2_kernel, 64, 0) != hipSuccess || occ < 1)
    occ = 8;
  // development override (A/B experiments): fewer resident inflate wavefronts per CU
  if (const char* ev = getenv("HSDS_INFLATE_WAVES")) {
    const int v = atoi(ev);
    if (v >= 1 && v < occ) occ = v;
  }
  e->inflate_blocks_per_cu = occ;
  int occ2 = 0, occ4 = 0, occ8 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, inflate2w_kernel<2>, 128, 0) != hipSuccess || occ2 < 1)
    occ2 = occ / 2 > 0 ? occ / 2 : 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ4, inflate2w_kernel<4>, 256, 0) != hipSuccess || occ4 < 1)
    occ4 = occ / 4 > 0 ? occ / 4 : 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ8, inflate2w_kernel<8>, 512, 0) != hipSuccess || occ8 < 1)
    occ8 = occ / 8 > 0 ? occ / 8 : 1;
  e->inflate2w_blocks_per_cu = occ2;
  e->inflate4w_blocks_per_cu = occ4;
  e->inflate8w_blocks_per_cu = occ8;
  e->inflate_pipe = HZ2_PIPE_DEFAULT;
  if (const char* ev = getenv("HSDS_INFLATE_PIPE")) {       // 0 (or < 0): by batch size; 1, 2, 4, 8 wavefronts
    const int v = atoi(ev);
    e->inflate_pipe = v == 1 || v == 2 || v == 4 || v == 8 ? v : 0;
  }
  int olz = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&olz, lz_kernel, 64, 0) != hipSuccess || olz < 1) olz = 8;
  e->lz_blocks_per_cu = olz;
  int obs = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&obs, bshuf_kernel, 64, 0) != hipSuccess || obs < 1) obs = 8;
  e->bshuf_blocks_per_cu = obs;
  int ozs = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&ozs, zstd_kernel, 64, 0) != hipSuccess || ozs < 1) ozs = 8;
  e->zstd_blocks_per_cu = ozs;
  int olw = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&olw, lz4_block_kernel, 64, 0) != hipSuccess || olw < 1) olw = 16;
  e->lz4w_blocks_per_cu = olw;
  int o1 = 0, o2 = 0, o3 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, parse_kernel, 64, 0) != hipSuccess || o1 < 1) o1 = 2;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, huff_kernel, 64, 0) != hipSuccess || o2 < 1) o2 = 4;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o3, emit_kernel, 64, 0) != hipSuccess || o3 < 1) o3 = 4;
  e->parse_blocks_per_cu = o1;
  {
    int oz = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&oz, zstd_lit_kernel, 64, 0) != hipSuccess || oz < 1) oz = 4;
    e->zlit_blocks_per_cu = oz;
  }
  if (const char* ev = getenv("HSDS_DEFLATE_CHAIN")) {   // development override (A/B experiments)
    const int v = atoi(ev);
    if (v >= 1 && v <= 4096) e->enc_chain = (uint32_t)v;
  }
  if (const char* ev = getenv("HSDS_DEFLATE_FAR")) {     // development override: far ring at any level
    if (atoi(ev) == 1) e->enc_chain |= 1u << 16;
  }
  e->huff_blocks_per_cu = o2;
  e->emit_blocks_per_cu = o3;
  // warm-up 1024 bits, segments sized to 1 + 1/16 of the previous block, 4 repair rounds
  e->tune.W = 1024;         // GPU sweep (tools/ab_tune.sh) with the warm-up in a loop of its own (round 6,
                            // profiles/r6_ab_warmup.txt): 640 / 768 / 1024 / 1280 bits -> F1 188.3 / 190.8 /
                            // 190.7 / 189.2 GB/s, F2 141.9 / 145.8 / 146.7 / 148.4 (round 5: 768 best)
  e->tune.max_rounds = 4;
  e->tune.over16 = 1;
  e->tune.spin_max = 0;     // window pipeline waits: hz2::SPIN_MAX polls (~1 s), then one-wavefront re-decode
  // development override (A/B experiments): "W,rounds,over16"
  if (const char* ev = getenv("HSDS_INFLATE_TUNE")) {
    unsigned w, ov; int rd;
    if (sscanf(ev, "%u,%d,%u", &w, &rd, &ov) == 3 && w <= 4096u && rd >= 0 && rd <= 64 && ov <= 16u) {
      e->tune.W = w; e->tune.max_rounds = rd; e->tune.over16 = ov;
      fprintf(stderr, "hsds_amd: inflate tune override %s\n", ev);
    }
  }
  if (hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess ||
      hipEventCreate(&e->ev2) != hipSuccess || hipEventCreate(&e->ev3) != hipSuccess ||
      hipEventCreateWithFlags(&e->ws_ev, hipEventDisableTiming) != hipSuccess) { delete e; return HSDS_ERR_DEVICE; }
  *out = e;
  return HSDS_OK;
}

void hsds_engine_destroy(hsds_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  if (e->ws) hipFree(e->ws);
  if (e->rings) hipFree(e->rings);
  if (e->tmp) hipFree(e->tmp);
  if (e->h_dev_src) hipFree(e->h_dev_src);
  if (e->h_dev_dst) hipFree(e->h_dev_dst);
  if (e->ews) hipFree(e->ews);
  if (e->ecw) hipFree(e->ecw);
  if (e->escr) hipFree(e->escr);
  if (e->efar) hipFree(e->efar);
  if (e->ezs) hipFree(e->ezs);
  hipEventDestroy(e->ev0);
  hipEventDestroy(e->ev1);
  hipEventDestroy(e->ev2);
  hipEventDestroy(e->ev3);
  hipEventDestroy(e->ws_ev);
  delete e;
}

int hsds_set_tuning(hsds_engine* e, uint32_t seg_over16, uint32_t warmup_bits, uint32_t waves_per_stream,
                    int32_t rounds) {
  if (!e) return HSDS_ERR_ARG;
  // HSDS_TUNE_KEEP (0xffffffff; -1 for rounds) leaves a setting as it is
  if ((seg_over16 > 16u && seg_over16 != HSDS_TUNE_KEEP) || (warmup_bits > 4096u && warmup_bits != HSDS_TUNE_KEEP) ||
      (waves_per_stream != HSDS_TUNE_KEEP && waves_per_stream > 2u && waves_per_stream != 4u && waves_per_stream != 8u) ||
      rounds < -1 ||
      rounds > 64)
    return HSDS_ERR_ARG;
  if (waves_per_stream != HSDS_TUNE_KEEP) e->inflate_pipe = (int)waves_per_stream;
  if (seg_over16 != HSDS_TUNE_KEEP) e->tune.over16 = seg_over16;
  if (warmup_bits != HSDS_TUNE_KEEP) e->tune.W = warmup_bits;
  if (rounds >= 0) e->tune.max_rounds = rounds;
  return HSDS_OK;
}

static int decode_batch_impl(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                             void* d_dst, uint64_t dst_extent, int32_t* d_status, int compressor, int shuffle,
                             int itemsize, void* stream, int inexact, uint32_t** inexact_size) {
  if (!e || nchunks < 0 || (nchunks && (!d_src || !d_chunks || !d_dst || !d_status))) return HSDS_ERR_ARG;
  if (itemsize < 1) itemsize = 1;
  if (nchunks == 0) return HSDS_OK;
  if (nchunks > (int64_t)(1u << 24)) return HSDS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  WsGuard guard(e, stream);
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  if (shuffle == HSDS_SHUFFLE_BIT && compressor == HSDS_COMP_NONE) {
    // bitshuffle+LZ4 objects as stored (no outer compressor): bshuf_kernel alone
    if (inexact) return HSDS_ERR_UNSUPPORTED;       // _unshuffle needs the chunk shape
    if (grow((void**)&e->ws, &e->ws_bytes, 256)) return HSDS_ERR_DEVICE;
    if (grow((void**)&e->tmp, &e->tmp_bytes, dst_extent ? dst_extent : 1)) return HSDS_ERR_DEVICE;
    uint32_t* ctr = (uint32_t*)e->ws;
    if (hipMemsetAsync(ctr, 0, 4, st) != hipSuccess) return HSDS_ERR_DEVICE;
    int64_t grid = (int64_t)e->num_cus * e->bshuf_blocks_per_cu;
    if (grid > nchunks) grid = nchunks;
    hipEventRecord(e->ev0, st);
    hipLaunchKernelGGL(bshuf_kernel, dim3((unsigned)grid), dim3(64), 0, st, (const uint8_t*)d_src, d_chunks, nchunks,
                       (uint8_t*)d_dst, e->tmp, d_status, ctr, itemsize);
    hipEventRecord(e->ev1, st);
    e->ev_valid = 1;
    return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
  }
  // workspace: the item pool (8 per chunk + 1 per 2 KiB of destination: HSDS's frames fit
  // many times over; a frame with more splits -- tiny blocks of a wide type -- fails alone,
  // frame_walk_kernel's pool_reserve), chunk meta and the unshuffle list
  const uint64_t cap64 = (uint64_t)nchunks * 8u + dst_extent / 2048u + 64u;
  const uint32_t pool_cap = cap64 > 0xffffffffull ? 0xffffffffu : (uint32_t)cap64;
  const size_t sz_pool = ((size_t)pool_cap * sizeof(Item) + 255) & ~(size_t)255;
  const size_t sz_meta = ((size_t)nchunks * sizeof(ChunkMeta) + 255) & ~(size_t)255;
  const size_t sz_list = ((size_t)nchunks * 4 + 255) & ~(size_t)255;
  const size_t sz_ord = ((size_t)pool_cap * 4 + 255) & ~(size_t)255;
  const size_t need = sz_pool + sz_meta + sz_list + sz_ord + 256;
  if (grow((void**)&e->ws, &e->ws_bytes, need)) return HSDS_ERR_DEVICE;
  uint8_t* w = e->ws;
  Item* pool = (Item*)w; w += sz_pool;
  ChunkMeta* meta = (ChunkMeta*)w; w += sz_meta;
  uint32_t* list = (uint32_t*)w; w += sz_list;
  uint32_t* ord = (uint32_t*)w; w += sz_ord;          // the batch kernel's claim order (HZ2_LPT)
  // [0] inflate item counter, [1] meta list count, [2] inexact size, [3] LZ item counter,
  // [4] LZ items, [5] zlib + raw items, [6] zstd items, [7] zstd item counter, [8] pool fill
  uint32_t* ctr = (uint32_t*)w;
  // staging for LZ / zstd Blosc frames with typesize > 1, bitshuffled Blosc frames and
  // shuffled F2 chunks (unshuffled by unshuffle_kernel afterwards; zlib Blosc splits and
  // raw items land unshuffled through their output map)
  uint8_t* tmp = nullptr;
  // (Blosc frames with the bitshuffle flag can come with any codec: every compressed batch
  // has the staging; it is grown once and only touched by frames that need it)
  if (compressor != HSDS_COMP_NONE) {
    if (grow((void**)&e->tmp, &e->tmp_bytes, dst_extent ? dst_extent : 1)) return HSDS_ERR_DEVICE;
    tmp = e->tmp;
  }
  // one match ring per resident inflate wave.  A batch whose zlib streams (at most 4 per
  // chunk in HSDS's F1 frames, 1 per F2 chunk) cannot fill the resident wavefronts decodes
  // every stream with two or four wavefronts (inflate2w_kernel)
  const int64_t waves1 = (int64_t)e->num_cus * e->inflate_blocks_per_cu;
  // wavefronts per stream: by batch size, the most whose streams (at most 4 per chunk) all
  // fit in the resident wavefronts (256 F1 chunks, DN micro-batcher: 4 wavefronts decode
  // in 3.9 ms, 2 in 5.1, 1 in 5.6; tools/batcher_prof.py)
  int nw = e->inflate_pipe;
  if (nw == 0) nw = nchunks * 4 * 4 <= waves1 ? 4 : nchunks * 4 * 2 <= waves1 ? 2 : 1;
  const bool pipe = nw > 1;
  int64_t grid = nw == 8 ? (int64_t)e->num_cus * e->inflate8w_blocks_per_cu
                 : nw == 4 ? (int64_t)e->num_cus * e->inflate4w_blocks_per_cu
                 : nw == 2 ? (int64_t)e->num_cus * e->inflate2w_blocks_per_cu : waves1;
  if (grid > nchunks * 64) grid = nchunks * 64;
  if (grid < 1) grid = 1;
  if (grow((void**)&e->rings, &e->rings_bytes, (size_t)grid * (size_t)nw * hz2::SCRATCH_BYTES))
    return HSDS_ERR_DEVICE;
  if (hipMemsetAsync(ctr, 0, 64, st) != hipSuccess) return HSDS_ERR_DEVICE;
  const int tpb = 256;
  const int nb = (int)((nchunks + tpb - 1) / tpb);
  hipLaunchKernelGGL(frame_walk_kernel, dim3(nb), dim3(tpb), 0, st, (const uint8_t*)d_src, d_chunks, nchunks,
                     (uint8_t*)d_dst, tmp, pool, pool_cap, ctr + 8, meta, list, ctr + 1, ctr + 4, d_status,
                     compressor, shuffle, itemsize, inexact);
  if (!pipe && HZ2_LPT) hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, st, pool, ctr + 8, ord);
  hipEventRecord(e->ev0, st);
  if (nw == 8)
    hipLaunchKernelGGL(inflate2w_kernel<8>, dim3((unsigned)grid), dim3(512), 0, st, pool, ctr + 8, ctr, d_status,
                       ctr + 2, ctr + 4, e->tune, e->rings);
  else if (nw == 4)
    hipLaunchKernelGGL(inflate2w_kernel<4>, dim3((unsigned)grid), dim3(256), 0, st, pool, ctr + 8, ctr, d_status,
                       ctr + 2, ctr + 4, e->tune, e->rings);
  else if (pipe)
    hipLaunchKernelGGL(inflate2w_kernel<2>, dim3((unsigned)grid), dim3(128), 0, st, pool, ctr + 8, ctr, d_status,
                       ctr + 2, ctr + 4, e->tune, e->rings);
  else
    hipLaunchKernelGGL(inflate2_kernel, dim3((unsigned)grid), dim3(64), 0, st, pool, ctr + 8, ctr, d_status, ctr + 2,
                       ctr + 4, e->tune, e->rings, HZ2_LPT ? (const uint32_t*)ord : (const uint32_t*)nullptr);
  int64_t lgrid = (int64_t)e->num_cus * e->lz_blocks_per_cu;
  if (lgrid > (nchunks * 64 + lz::GROUP - 1) / lz::GROUP) lgrid = (nchunks * 64 + lz::GROUP - 1) / lz::GROUP;
  if (lgrid < 1) lgrid = 1;
  hipLaunchKernelGGL(lz_kernel, dim3((unsigned)lgrid), dim3(64), 0, st, pool, ctr + 8, ctr + 3, d_status, ctr + 4);
  int64_t zgrid = (int64_t)e->num_cus * e->zstd_blocks_per_cu;
  if (zgrid > nchunks * 16) zgrid = nchunks * 16;
  if (zgrid < 1) zgrid = 1;
  hipLaunchKernelGGL(zstd_kernel, dim3((unsigned)zgrid), dim3(64), 0, st, pool, ctr + 8, ctr + 7, d_status, ctr + 4);
  hipEventRecord(e->ev1, st);
  e->ev_valid = 1;
  if (tmp) hipLaunchKernelGGL(unshuffle_kernel, dim3(2048), dim3(256), 0, st, meta, list, ctr + 1, d_status);
  if (hipGetLastError() != hipSuccess) return HSDS_ERR_DEVICE;
  if (inexact_size) *inexact_size = ctr + 2;
  return HSDS_OK;
}

int hsds_decode_batch(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                      void* d_dst, uint64_t dst_extent, int32_t* d_status, int compressor, int shuffle,
                      int itemsize, void* stream) {
  return decode_batch_impl(e, d_src, d_chunks, nchunks, d_dst, dst_extent, d_status, compressor, shuffle, itemsize,
                           stream, 0, nullptr);
}

// inflate2_kernel wave timing of the HZ_PROFILE build (100 MHz ticks): min start, max end,
// sum of ends, waves, sum of stream decode time, longest stream, min end
int hsds_debug_tail(unsigned long long* out8, int reset) {
#ifdef HZ_PROFILE
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(hz_tail), 8 * sizeof(unsigned long long)) != hipSuccess) return HSDS_ERR_DEVICE;
  if (reset) {
    unsigned long long z[8] = {~0ull, 0, 0, 0, 0, 0, ~0ull, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hz_tail), z, sizeof(z)) != hipSuccess) return HSDS_ERR_DEVICE;
  }
  return HSDS_OK;
#else
  (void)out8; (void)reset;
  return HSDS_ERR_UNSUPPORTED;
#endif
}

int hsds_debug_profile(unsigned long long* out16, int reset) {
#ifdef HZ_PROFILE
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(hz_prof), 16 * sizeof(unsigned long long)) != hipSuccess) return HSDS_ERR_DEVICE;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hz_prof), z, sizeof(z)) != hipSuccess) return HSDS_ERR_DEVICE;
  }
  return HSDS_OK;
#else
  (void)out16; (void)reset;
  return HSDS_ERR_UNSUPPORTED;
#endif
}

int hsds_partition_ids(const char* prefix, int rank, const int64_t* idx, int64_t n, int world, int32_t* owner) {
  if (!prefix || rank < 1 || rank > 32 || n < 0 || world < 1 || (n && (!idx || !owner))) return HSDS_ERR_ARG;
  const size_t pl = strlen(prefix);
  if (pl > 256) return HSDS_ERR_ARG;
  for (int64_t i = 0; i < n * rank; i++)
    if (idx[i] < 0) return HSDS_ERR_ARG;
  auto work = [=](int64_t i0, int64_t i1) {
    char buf[256 + 32 * 21];
    memcpy(buf, prefix, pl);
    for (int64_t i = i0; i < i1; i++) {
      size_t len = pl;
      for (int d = 0; d < rank; d++) {
        int64_t v = idx[i * rank + d];
        if (d) buf[len++] = '_';
        char tmp[21];
        int k = 0;
        do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (k) buf[len++] = tmp[--k];
      }
      owner[i] = (int32_t)(md5_prefix20((const uint8_t*)buf, len) % (uint32_t)world);
    }
  };
  // one host thread per 4096 ids, at most 8
  int nt = (int)((n + 4095) / 4096);
  if (nt > 8) nt = 8;
  if (nt <= 1) { work(0, n); return HSDS_OK; }
  // (nothing may throw across the C ABI: a range whose thread cannot be created -- thread
  // limit, std::system_error -- or a failed allocation is done by the calling thread)
  std::vector<std::thread> th;
  int t = 0;
  try {
    th.reserve(nt);
    for (; t < nt; t++) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
  } catch (...) {
  }
  for (; t < nt; t++) work(n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
  return HSDS_OK;
}

int hsds_last_inflate_ms(hsds_engine* e, float* ms) {
  if (!e || !ms || !e->ev_valid) return HSDS_ERR_ARG;
  if (hipEventElapsedTime(ms, e->ev0, e->ev1) != hipSuccess) return HSDS_ERR_DEVICE;
  return HSDS_OK;
}

int64_t hsds_uncompress(hsds_engine* e, const void* src, int64_t srclen, int compressor, int shuffle, int itemsize,
                        void* dst, int64_t expected) {
  if (!e || srclen < 0 || (srclen && !src) || (expected && !dst)) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  WsGuard guard(e, nullptr);
  const int inexact = expected < 0;
  if (inexact) expected = -expected;
  // device staging: [src bytes | chunk descriptor] and [dst bytes | status]
  const size_t desc_off = ((size_t)srclen + 255) & ~(size_t)255;
  const size_t stat_off = ((size_t)expected + 255) & ~(size_t)255;
  if (grow((void**)&e->h_dev_src, &e->h_dev_src_bytes, desc_off + sizeof(hsds_chunk_desc))) return HSDS_ERR_DEVICE;
  if (grow((void**)&e->h_dev_dst, &e->h_dev_dst_bytes, stat_off + 64)) return HSDS_ERR_DEVICE;
  hsds_chunk_desc c = {0, (uint64_t)srclen, 0, (uint64_t)expected};
  hsds_chunk_desc* dd = (hsds_chunk_desc*)(e->h_dev_src + desc_off);
  int32_t* dstat = (int32_t*)(e->h_dev_dst + stat_off);
  if (srclen && hipMemcpy(e->h_dev_src, src, (size_t)srclen, hipMemcpyHostToDevice) != hipSuccess)
    return HSDS_ERR_DEVICE;
  if (hipMemcpy(dd, &c, sizeof(c), hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  uint32_t* dsize = nullptr;
  int r = decode_batch_impl(e, e->h_dev_src, dd, 1, e->h_dev_dst, (uint64_t)expected, dstat, compressor, shuffle,
                            itemsize, nullptr, inexact, &dsize);
  if (r) return r;
  int32_t status = 0;
  if (hipMemcpy(&status, dstat, 4, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  if (status) return status;
  if (inexact) {
    uint32_t got = 0;
    if (hipMemcpy(&got, dsize, 4, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
    expected = got;
  }
  if (expected && hipMemcpy(dst, e->h_dev_dst, (size_t)expected, hipMemcpyDeviceToHost) != hipSuccess)
    return HSDS_ERR_DEVICE;
  return expected;
}

static int launch_shuffle(const void* d_src, int64_t n, int itemsize, void* d_dst, void* stream, int inverse) {
  if (n < 0 || itemsize < 1 || (n && (!d_src || !d_dst))) return HSDS_ERR_ARG;
  if (n == 0) return HSDS_OK;
  if (itemsize == 1) {
    return hipMemcpyAsync(d_dst, d_src, (size_t)n, hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess
               ? HSDS_OK : HSDS_ERR_DEVICE;
  }
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(shuffle_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)d_src, (uint8_t*)d_dst, (uint64_t)n, (uint32_t)itemsize, inverse);
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

int hsds_shuffle_device(hsds_engine* e, const void* d_src, int64_t n, int itemsize, void* d_dst, void* stream) {
  if (!e) return HSDS_ERR_ARG;
  return launch_shuffle(d_src, n, itemsize, d_dst, stream, 0);
}
int hsds_unshuffle_device(hsds_engine* e, const void* d_src, int64_t n, int itemsize, void* d_dst, void* stream) {
  if (!e) return HSDS_ERR_ARG;
  return launch_shuffle(d_src, n, itemsize, d_dst, stream, 1);
}

static int host_shuffle(hsds_engine* e, const void* src, int64_t n, int itemsize, void* dst, int inverse) {
  if (!e || n < 0 || itemsize < 1 || (n && (!src || !dst))) return HSDS_ERR_ARG;
  if (n == 0) return HSDS_OK;
  hipSetDevice(e->device);
  WsGuard guard(e, nullptr);
  if (grow((void**)&e->h_dev_src, &e->h_dev_src_bytes, (size_t)n)) return HSDS_ERR_DEVICE;
  if (grow((void**)&e->h_dev_dst, &e->h_dev_dst_bytes, (size_t)n)) return HSDS_ERR_DEVICE;
  if (hipMemcpy(e->h_dev_src, src, (size_t)n, hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  int r = launch_shuffle(e->h_dev_src, n, itemsize, e->h_dev_dst, nullptr, inverse);
  if (r) return r;
  if (hipMemcpy(dst, e->h_dev_dst, (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  return HSDS_OK;
}

int hsds_shuffle(hsds_engine* e, const void* src, int64_t n, int itemsize, void* dst) {
  return host_shuffle(e, src, n, itemsize, dst, 0);
}
int hsds_unshuffle(hsds_engine* e, const void* src, int64_t n, int itemsize, void* dst) {
  return host_shuffle(e, src, n, itemsize, dst, 1);
}

// blocks per record: enough blocks in all (~4096: 16 per CU) whatever the record count
static unsigned copy_gx(int64_t n) {
  const int64_t y = n < 65535 ? n : 65535;
  int64_t x = 4096 / (y > 0 ? y : 1);
  return (unsigned)(x < 1 ? 1 : x > 2048 ? 2048 : x);
}

static int launch_copy(const void* d_src, void* d_dst, const hsds_copy_desc* d_desc, int64_t n, const int32_t* flags,
                       void* stream) {
  if (n < 0 || (n && (!d_src || !d_dst || !d_desc))) return HSDS_ERR_ARG;
  if (n == 0) return HSDS_OK;
  const unsigned gy = (unsigned)(n < 65535 ? n : 65535);
  hipLaunchKernelGGL(copy_kernel, dim3(copy_gx(n), gy), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d_src,
                     (uint8_t*)d_dst, d_desc, n, flags);
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

int hsds_copy_batch(hsds_engine* e, const void* d_src, void* d_dst, const hsds_copy_desc* d_desc, int64_t n,
                    void* stream) {
  if (!e) return HSDS_ERR_ARG;
  return launch_copy(d_src, d_dst, d_desc, n, nullptr, stream);
}

int hsds_copy_batch_if(hsds_engine* e, const void* d_src, void* d_dst, const hsds_copy_desc* d_desc, int64_t n,
                       const int32_t* d_flags, void* stream) {
  if (!e || (n && !d_flags)) return HSDS_ERR_ARG;
  return launch_copy(d_src, d_dst, d_desc, n, d_flags, stream);
}

int hsds_compare_batch(hsds_engine* e, const void* d_b, const void* d_a, const hsds_copy_desc* d_desc, int64_t n,
                       int kind, int32_t* d_differs, void* stream) {
  if (!e || n < 0 || (n && (!d_a || !d_b || !d_desc || !d_differs))) return HSDS_ERR_ARG;
  if (n == 0) return HSDS_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(zero_i32_kernel, dim3(64), dim3(256), 0, st, d_differs, n);
  const unsigned gy = (unsigned)(n < 65535 ? n : 65535);
  hipLaunchKernelGGL(compare_kernel, dim3(copy_gx(n), gy), dim3(256), 0, st, (const uint8_t*)d_b, (const uint8_t*)d_a,
                     d_desc, n, kind, d_differs);
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

// ---- hyperslab plan records -------------------------------------------------
// one thread per piece: unravel the product-grid index over the per-dimension tables,
// then the record of the requested direction (crawl.SelectionPlan._descs on the device)
__global__ void plan_descs_kernel(hsds_plan_geom g, const int64_t* __restrict__ tabs,
                                  const int64_t* __restrict__ piece, const int64_t* __restrict__ poff,
                                  const int64_t* __restrict__ coff, int64_t n, hsds_copy_desc* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int R = g.rank;
  int64_t tab0[HSDS_MAX_RANK];
  int64_t t = 0;
#pragma unroll
  for (int d = 0; d < HSDS_MAX_RANK; d++) {
    if (d < R) { tab0[d] = t; t += 3 * g.nk[d]; }
  }
  int64_t gi = piece[k];
  int64_t cst[HSDS_MAX_RANK], cnt[HSDS_MAX_RANK], dst[HSDS_MAX_RANK];
#pragma unroll
  for (int d = HSDS_MAX_RANK - 1; d >= 0; d--) {
    if (d < R) {
      const int64_t nk = g.nk[d];
      const int64_t j = gi % nk;
      gi /= nk;
      cst[d] = tabs[tab0[d] + j];
      cnt[d] = tabs[tab0[d] + nk + j];
      dst[d] = tabs[tab0[d] + 2 * nk + j];
    } else {
      cst[d] = 0; cnt[d] = 0; dst[d] = 0;
    }
  }
  hsds_copy_desc r;
  int64_t pst[HSDS_MAX_RANK];
  int64_t acc = g.itemsize;
#pragma unroll
  for (int d = HSDS_MAX_RANK - 1; d >= 0; d--) {
    if (d < R) { pst[d] = acc; acc *= cnt[d]; } else pst[d] = 0;
  }
  if (g.mode == HSDS_PLAN_DIRECT) {
    // chunk [chunk_sel] -> slab [data_sel]: no packed buffer in between
    int64_t so = coff[k], dof = g.slab_base;
#pragma unroll
    for (int d = 0; d < HSDS_MAX_RANK; d++) {
      if (d < R) {
        so += cst[d] * g.chunk_stride[d];
        dof += dst[d] * g.slab_stride[d];
      }
      r.src_stride[d] = d < R ? g.chunk_stride[d] * g.step[d] : 0;
      r.dst_stride[d] = d < R ? g.slab_stride[d] : 0;
      r.count[d] = cnt[d];
    }
    r.src_off = (uint64_t)so;
    r.dst_off = (uint64_t)dof;
    r.rank = R;
    r.itemsize = g.itemsize;
    out[k] = r;
    return;
  }
  const bool chunk_side = g.mode == HSDS_PLAN_PACK || g.mode == HSDS_PLAN_APPLY || g.mode == HSDS_PLAN_APPLY_BCAST;
  const bool to_region = g.mode == HSDS_PLAN_PLACE || g.mode == HSDS_PLAN_APPLY || g.mode == HSDS_PLAN_APPLY_BCAST;
  int64_t roff = chunk_side ? coff[k] : g.slab_base;
  int64_t rst[HSDS_MAX_RANK];
#pragma unroll
  for (int d = 0; d < HSDS_MAX_RANK; d++) {
    if (d < R) {
      roff += chunk_side ? cst[d] * g.chunk_stride[d] : dst[d] * g.slab_stride[d];
      rst[d] = chunk_side ? g.chunk_stride[d] * g.step[d] : g.slab_stride[d];
    } else {
      rst[d] = 0;
    }
  }
  const bool bcast = g.mode == HSDS_PLAN_APPLY_BCAST;
  r.src_off = (uint64_t)(to_region ? poff[k] : roff);
  r.dst_off = (uint64_t)(to_region ? roff : poff[k]);
#pragma unroll
  for (int d = 0; d < HSDS_MAX_RANK; d++) {
    r.src_stride[d] = to_region ? (bcast ? 0 : pst[d]) : rst[d];
    r.dst_stride[d] = to_region ? rst[d] : pst[d];
    r.count[d] = cnt[d];
  }
  r.rank = R;
  r.itemsize = g.itemsize;
  out[k] = r;
}

int hsds_host_map(hsds_engine* e, void* p, uint64_t n, void** d_ptr) {
  if (!e || !p || !n || !d_ptr) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  if (hipHostRegister(p, (size_t)n, hipHostRegisterMapped) != hipSuccess) return HSDS_ERR_DEVICE;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    hipHostUnregister(p);
    return HSDS_ERR_DEVICE;
  }
  *d_ptr = d;
  return HSDS_OK;
}

int hsds_host_unmap(hsds_engine* e, void* p) {
  if (!e || !p) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  return hipHostUnregister(p) == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

// Staging of a read batch's stored objects: `threads` host threads (the calling one among
// them) take pieces of whole objects in ascending order, copy them into the page-locked
// buffer and queue each piece's host-to-device copy as soon as it is staged, so the link
// starts after the first pieces instead of after the last.  At most 16 pieces of at least
// 2 MiB: 150 MiB goes up at 57 GB/s in one copy, 54 in 16, 46 in 64 and 29 in 256
// (tools/pcie_bw.py).
int hsds_stage_upload(hsds_engine* e, const void* const* srcs, const uint64_t* lens, const uint64_t* offs,
                      int64_t n, void* h_stage, void* d_dst, uint64_t total, int threads, void* stream) {
  if (!e || n < 0 || (n && (!srcs || !lens || !offs || !h_stage || !d_dst))) return HSDS_ERR_ARG;
  if (n == 0 || total == 0) return HSDS_OK;
  for (int64_t k = 0; k < n; k++)
    if ((lens[k] && !srcs[k]) || offs[k] > total || lens[k] > total - offs[k] || (k && offs[k] < offs[k - 1]))
      return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  uint8_t* const host = (uint8_t*)h_stage;
  // piece p = objects [cut[p], cut[p + 1]); the last piece's upload runs to `total`
  int64_t parts = (int64_t)(total >> 21);
  parts = parts < 1 ? 1 : parts > 16 ? 16 : parts;
  if (parts > n) parts = n;
  // (nothing may throw across the C ABI: an allocation failure is HSDS_ERR_DEVICE, and a
  // helper thread that cannot be created -- thread limit, std::system_error -- only leaves
  // its pieces to the threads that run, the calling one always among them)
  std::vector<int64_t> cut;
  try {
    cut.resize(parts + 1);
  } catch (...) {
    return HSDS_ERR_DEVICE;
  }
  for (int64_t p = 0; p <= parts; p++) cut[p] = n * p / parts;
  std::atomic<int64_t> next{0};
  std::atomic<int> rc{HSDS_OK};
  const int dev = e->device;
  auto worker = [&]() {
    if (hipSetDevice(dev) != hipSuccess) { rc.store(HSDS_ERR_DEVICE); return; }
    for (int64_t p; (p = next.fetch_add(1, std::memory_order_relaxed)) < parts;) {
      for (int64_t k = cut[p]; k < cut[p + 1]; k++)
        if (lens[k]) memcpy(host + offs[k], srcs[k], (size_t)lens[k]);
      const uint64_t lo = offs[cut[p]];
      const uint64_t hi = p + 1 < parts ? offs[cut[p + 1]] : total;
      if (hi > lo && hipMemcpyAsync((uint8_t*)d_dst + lo, host + lo, (size_t)(hi - lo), hipMemcpyHostToDevice,
                                    (hipStream_t)stream) != hipSuccess)
        rc.store(HSDS_ERR_DEVICE);
    }
  };
  const int nt = threads < 1 ? 0 : (threads > 64 ? 63 : threads - 1);
  std::vector<std::thread> pool;
  try {
    pool.reserve(nt);
    for (int t = 0; t < nt && t + 1 < parts; t++) pool.emplace_back(worker);
  } catch (...) {
  }
  worker();
  for (auto& t : pool) t.join();
  return rc.load();
}

int hsds_plan_descs(hsds_engine* e, const hsds_plan_geom* geom, const int64_t* d_tabs, const int64_t* d_piece,
                    const int64_t* d_poff, const int64_t* d_coff, int64_t n, hsds_copy_desc* d_out,
                    void* stream) {
  if (!e || !geom || n < 0) return HSDS_ERR_ARG;
  if (n == 0) return HSDS_OK;
  const hsds_plan_geom g = *geom;
  if (g.rank < 1 || g.rank > HSDS_MAX_RANK || g.itemsize < 1 || g.mode < HSDS_PLAN_PACK ||
      g.mode > HSDS_PLAN_DIRECT || !d_tabs || !d_piece || (!d_poff && g.mode != HSDS_PLAN_DIRECT) || !d_out)
    return HSDS_ERR_ARG;
  const bool chunk_side = g.mode == HSDS_PLAN_PACK || g.mode == HSDS_PLAN_APPLY || g.mode == HSDS_PLAN_APPLY_BCAST ||
                          g.mode == HSDS_PLAN_DIRECT;
  if (chunk_side && !d_coff) return HSDS_ERR_ARG;
  for (int d = 0; d < g.rank; d++)
    if (g.nk[d] < 1) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  const int tpb = 256;
  hipLaunchKernelGGL(plan_descs_kernel, dim3((unsigned)((n + tpb - 1) / tpb)), dim3(tpb), 0, (hipStream_t)stream, g,
                     d_tabs, d_piece, d_poff, d_coff, n, d_out);
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

// ---- encode -----------------------------------------------------------------
int hsds_encode_batch_codec(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                            void* d_dst, uint64_t dst_extent, int64_t* d_sizes, int32_t* d_status, int clevel,
                            int shuffle, int typesize, int cname, void* stream) {
  if (!e || nchunks < 0 || (nchunks && (!d_src || !d_chunks || !d_dst || !d_sizes || !d_status))) return HSDS_ERR_ARG;
  if (cname != HSDS_CNAME_ZLIB && cname != HSDS_CNAME_LZ4 && cname != HSDS_CNAME_LZ4HC && cname != HSDS_CNAME_BLOSCLZ &&
      cname != HSDS_CNAME_ZSTD)
    return HSDS_ERR_ARG;
  if (clevel < 0 || clevel > 9 || (shuffle != HSDS_SHUFFLE_NONE && shuffle != HSDS_SHUFFLE_BYTE)) return HSDS_ERR_ARG;
  if (((uintptr_t)d_dst & 3u) != 0) return HSDS_ERR_ARG;
  if (nchunks == 0) return HSDS_OK;
  if (nchunks > (int64_t)(1u << 22)) return HSDS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  WsGuard guard(e, stream);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  // per-chunk plan arrays (own buffer: they survive the resize of the split / segment area)
  const size_t sz_counts = al((size_t)nchunks * 4);
  const size_t sz_offs = al((size_t)(nchunks + 1) * 4);
  const size_t sz_geom = al((size_t)nchunks * sizeof(EncGeom));
  if (grow((void**)&e->ecw, &e->ecw_bytes, 2 * sz_counts + 2 * sz_offs + sz_geom + 256)) return HSDS_ERR_DEVICE;
  uint8_t* w = e->ecw;
  uint32_t* counts = (uint32_t*)w; w += sz_counts;
  uint32_t* segcnt = (uint32_t*)w; w += sz_counts;
  uint32_t* offs = (uint32_t*)w; w += sz_offs;
  uint32_t* segoffs = (uint32_t*)w; w += sz_offs;
  EncGeom* geom = (EncGeom*)w; w += sz_geom;
  uint32_t* ctr = (uint32_t*)w;    // [0] parse items, [1] huffman segments, [2] emit segments
  if (hipMemsetAsync(ctr, 0, 32, st) != hipSuccess) return HSDS_ERR_DEVICE;
  const int tpb = 256;
  const int nb = (int)((nchunks + tpb - 1) / tpb);
  // pass 1: every chunk's split and segment counts (no per-chunk split cap), prefix sums,
  // then the exact totals to the host: the split / segment work areas (about 24 KB of
  // parse state + tokens per 8 KiB segment) are sized by the batch, not by a worst case
  hipLaunchKernelGGL(enc_plan_kernel, dim3(nb), dim3(tpb), 0, st, (const uint8_t*)d_src, d_chunks, nchunks,
                     (EncItem*)nullptr, counts, segcnt, geom, d_status, clevel, shuffle, typesize, cname,
                     (const uint32_t*)nullptr, 0u, 0);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, counts, offs, nchunks);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, segcnt, segoffs, nchunks);
  uint32_t tot[2] = {0, 0};
  if (hipMemcpyAsync(&tot[0], offs + nchunks, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&tot[1], segoffs + nchunks, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return HSDS_ERR_DEVICE;
  const uint32_t item_cap = tot[0] + 1, seg_cap = tot[1] + 1;
  const size_t ns = (size_t)item_cap;
  const size_t sz_slots = al(ns * sizeof(EncItem));
  const size_t sz_adler = al(ns * 4);
  const size_t sz_iout = al(ns * sizeof(ItemOut));
  const size_t sz_sp = al((size_t)seg_cap * sizeof(hd::SegParse));
  const size_t sz_sc = al((size_t)seg_cap * sizeof(hd::SegCode));
  const size_t sz_so = al((size_t)seg_cap * sizeof(hd::SegOut));
  const size_t sz_meta = al((size_t)seg_cap * sizeof(SegMeta));
  const size_t sz_lzsize = al(ns * 4);
  const size_t need = sz_slots + sz_adler + sz_iout + sz_sp + sz_sc + sz_so + sz_meta + sz_lzsize + 256;
  if (grow((void**)&e->ews, &e->ews_bytes, need)) return HSDS_ERR_DEVICE;
  w = e->ews;
  EncItem* slots = (EncItem*)w; w += sz_slots;
  uint32_t* adler = (uint32_t*)w; w += sz_adler;
  ItemOut* iout = (ItemOut*)w; w += sz_iout;
  hd::SegParse* sp = (hd::SegParse*)w; w += sz_sp;
  hd::SegCode* sc = (hd::SegCode*)w; w += sz_sc;
  hd::SegOut* so = (hd::SegOut*)w; w += sz_so;
  SegMeta* meta = (SegMeta*)w; w += sz_meta;
  uint32_t* lzsize = (uint32_t*)w; w += sz_lzsize;
  // token slots: SEG_TOK per segment
  if (grow((void**)&e->escr, &e->escr_bytes, (size_t)seg_cap * hd::SEG_TOK * 2 + 256)) return HSDS_ERR_DEVICE;
  uint16_t* tok = (uint16_t*)e->escr;
  // pass 2: the splits, compact at offs[ci]
  hipLaunchKernelGGL(enc_plan_kernel, dim3(nb), dim3(tpb), 0, st, (const uint8_t*)d_src, d_chunks, nchunks, slots,
                     counts, segcnt, geom, d_status, clevel, shuffle, typesize, cname, (const uint32_t*)offs,
                     item_cap, 1);
  auto grid_for = [&](int per_cu, int64_t cap) {
    int64_t g = (int64_t)e->num_cus * per_cu;
    if (g > cap) g = cap;
    return (unsigned)(g < 1 ? 1 : g);
  };
  const unsigned pgrid = grid_for(e->parse_blocks_per_cu, item_cap);
  uint16_t* far = nullptr;
  if ((cname == HSDS_CNAME_ZLIB || cname == HSDS_CNAME_ZSTD) && (hd::far_level(clevel) || (e->enc_chain >> 16))) {
    // levels >= 6: matches reach 32 KiB back, the chains beyond the LDS ring live in HBM
    if (grow((void**)&e->efar, &e->efar_bytes, (size_t)pgrid * hd::FARW * 2)) return HSDS_ERR_DEVICE;
    far = (uint16_t*)e->efar;
  }
  hipEventRecord(e->ev2, st);
  hipLaunchKernelGGL(parse_kernel, dim3(pgrid), dim3(64), 0, st, slots,
                     offs, segoffs, nchunks, ctr, sp, meta, tok, adler, seg_cap,
                     clevel, 0u, item_cap, far,
                     e->enc_chain);
  if (cname == HSDS_CNAME_ZSTD) {
    const size_t sz_zseg = al((size_t)seg_cap * (hze::ZCAP + hze::LCAP + 8));
    const size_t sz_cnt = al((size_t)item_cap * sizeof(hze::SeqCounts));
    if (grow((void**)&e->ezs, &e->ezs_bytes, sz_zseg + sz_cnt + (size_t)item_cap * sizeof(hze::Tabs) + 256))
      return HSDS_ERR_DEVICE;
    uint8_t* zscr = e->ezs;
    uint8_t* lsec = zscr + (size_t)seg_cap * hze::ZCAP;
    uint32_t* zsz = (uint32_t*)(lsec + (size_t)seg_cap * hze::LCAP);
    uint32_t* lsz = zsz + seg_cap;
    hze::SeqCounts* zcnt = (hze::SeqCounts*)(e->ezs + sz_zseg);
    hze::Tabs* ztab = (hze::Tabs*)(e->ezs + sz_zseg + sz_cnt);
    // the frames' sequence tables (FSE_Compressed_Mode, one set per frame)
    if (hipMemsetAsync(zcnt, 0, sz_cnt, st) != hipSuccess) return HSDS_ERR_DEVICE;
    hipLaunchKernelGGL(zstd_count_kernel, dim3((seg_cap + ZC_SEGS - 1) / ZC_SEGS), dim3(64), 0, st, segoffs, nchunks,
                       meta, sp, tok,
                       zcnt, seg_cap);
    hipLaunchKernelGGL(zstd_table_kernel, dim3((item_cap + 63) / 64), dim3(64), 0, st, offs, nchunks,
                       (const hze::SeqCounts*)zcnt, ztab, item_cap);
    if (hze::huff_lit_level(clevel))
      hipLaunchKernelGGL(zstd_lit_kernel, dim3(grid_for(e->zlit_blocks_per_cu, seg_cap)), dim3(64), 0, st, segoffs,
                         nchunks, sp, tok, lsec, lsz, seg_cap);
    else if (hipMemsetAsync(lsz, 0, (size_t)seg_cap * 4, st) != hipSuccess)
      return HSDS_ERR_DEVICE;
    hipLaunchKernelGGL(zstd_seq_kernel, dim3(grid_for(6, seg_cap)), dim3(64), 0, st, segoffs, nchunks, sp, tok, zscr,
                       (const uint32_t*)lsz, seg_cap);
    hipLaunchKernelGGL(zstd_seg_kernel, dim3((seg_cap + 63) / 64), dim3(64), 0, st, segoffs, nchunks, meta, slots, sp,
                       tok, zscr, zsz, lsec, lsz, seg_cap, clevel, (const hze::Tabs*)ztab);
    hipLaunchKernelGGL(zstd_size_kernel, dim3((item_cap + 255) / 256), dim3(256), 0, st, offs, segoffs, nchunks, slots,
                       zsz, lzsize, seg_cap, item_cap);
    hipLaunchKernelGGL(layout_kernel, dim3(nb), dim3(tpb), 0, st, d_chunks, nchunks, (uint8_t*)d_dst, slots, counts,
                       offs, segoffs, geom, sc, adler, iout, so, d_sizes, d_status, seg_cap, clevel, (const uint32_t*)lzsize);
    hipLaunchKernelGGL(zstd_write_kernel, dim3(grid_for(16, item_cap)), dim3(64), 0, st, offs, segoffs, nchunks, slots,
                       zscr, zsz, d_chunks, (uint8_t*)d_dst, geom, iout, d_status, seg_cap, item_cap);
  } else if (cname == HSDS_CNAME_ZLIB) {
    hipLaunchKernelGGL(huff_kernel, dim3(grid_for(e->huff_blocks_per_cu, seg_cap)), dim3(64), 0, st, segoffs,
                       nchunks, ctr + 1, sp, meta, sc, seg_cap, clevel);
    hipLaunchKernelGGL(layout_kernel, dim3(nb), dim3(tpb), 0, st, d_chunks, nchunks, (uint8_t*)d_dst, slots, counts,
                       offs, segoffs, geom, sc, adler, iout, so, d_sizes, d_status, seg_cap, clevel, (const uint32_t*)nullptr);
    hipLaunchKernelGGL(emit_kernel, dim3(grid_for(e->emit_blocks_per_cu, seg_cap)), dim3(64), 0, st, segoffs,
                       nchunks, ctr + 2, so, sc, sp, tok, slots, (uint32_t*)d_dst, seg_cap, clevel);
  } else {
    const unsigned lgrid = grid_for(e->lz4w_blocks_per_cu, item_cap);
    hipLaunchKernelGGL(lz4_block_kernel, dim3(lgrid), dim3(64), 0, st, slots, offs, segoffs, nchunks, sp, tok, lzsize,
                       seg_cap, clevel, d_chunks, (uint8_t*)d_dst, geom, iout, d_status, 0,
                       (int)(cname == HSDS_CNAME_BLOSCLZ), 0u, item_cap);
    hipLaunchKernelGGL(layout_kernel, dim3(nb), dim3(tpb), 0, st, d_chunks, nchunks, (uint8_t*)d_dst, slots, counts,
                       offs, segoffs, geom, sc, adler, iout, so, d_sizes, d_status, seg_cap, clevel, (const uint32_t*)lzsize);
    hipLaunchKernelGGL(lz4_block_kernel, dim3(lgrid), dim3(64), 0, st, slots, offs, segoffs, nchunks, sp, tok, lzsize,
                       seg_cap, clevel, d_chunks, (uint8_t*)d_dst, geom, iout, d_status, 1,
                       (int)(cname == HSDS_CNAME_BLOSCLZ), 0u, item_cap);
  }
  hipLaunchKernelGGL(raw_copy_kernel, dim3((unsigned)nchunks), dim3(256), 0, st, (const uint8_t*)d_src, d_chunks,
                     nchunks, (uint8_t*)d_dst, slots, counts, offs, geom, iout, d_status);
  hipEventRecord(e->ev3, st);
  e->ev_enc_valid = 1;
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

int hsds_encode_batch(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                      void* d_dst, uint64_t dst_extent, int64_t* d_sizes, int32_t* d_status, int clevel,
                      int shuffle, int typesize, void* stream) {
  return hsds_encode_batch_codec(e, d_src, d_chunks, nchunks, d_dst, dst_extent, d_sizes, d_status, clevel, shuffle,
                                 typesize, HSDS_CNAME_ZLIB, stream);
}

int hsds_last_deflate_ms(hsds_engine* e, float* ms) {
  if (!e || !ms || !e->ev_enc_valid) return HSDS_ERR_ARG;
  if (hipEventElapsedTime(ms, e->ev2, e->ev3) != hipSuccess) return HSDS_ERR_DEVICE;
  return HSDS_OK;
}

int64_t hsds_compress_codec(hsds_engine* e, const void* src, int64_t n, int clevel, int shuffle, int typesize,
                            int cname, void* dst, int64_t cap) {
  if (!e || n < 0 || (n && !src) || !dst || cap < n + 16) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  WsGuard guard(e, nullptr);
  const size_t desc_off = ((size_t)n + 255) & ~(size_t)255;
  const size_t frame_cap = (size_t)n + 16;
  const size_t stat_off = (frame_cap + 255) & ~(size_t)255;
  if (grow((void**)&e->h_dev_src, &e->h_dev_src_bytes, desc_off + sizeof(hsds_chunk_desc))) return HSDS_ERR_DEVICE;
  if (grow((void**)&e->h_dev_dst, &e->h_dev_dst_bytes, stat_off + 64)) return HSDS_ERR_DEVICE;
  hsds_chunk_desc c = {0, (uint64_t)n, 0, (uint64_t)frame_cap};
  hsds_chunk_desc* dd = (hsds_chunk_desc*)(e->h_dev_src + desc_off);
  int64_t* dsize = (int64_t*)(e->h_dev_dst + stat_off);
  int32_t* dstat = (int32_t*)(e->h_dev_dst + stat_off + 16);
  if (n && hipMemcpy(e->h_dev_src, src, (size_t)n, hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  if (hipMemcpy(dd, &c, sizeof(c), hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  int r = hsds_encode_batch_codec(e, e->h_dev_src, dd, 1, e->h_dev_dst, frame_cap, dsize, dstat, clevel, shuffle,
                                  typesize, cname, nullptr);
  if (r) return r;
  int32_t status = 0;
  int64_t size = 0;
  if (hipMemcpy(&status, dstat, 4, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  if (status) return status;
  if (hipMemcpy(&size, dsize, 8, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  if (size < 16 || size > cap) return HSDS_ERR_SIZE;
  if (hipMemcpy(dst, e->h_dev_dst, (size_t)size, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  return size;
}

// ---- bitshuffle+LZ4 encode (storUtil._shuffle codec 2) ---------------------------
static uint32_t host_bshuf_default_block(uint32_t es) {   // bs::default_block on the host
  const uint32_t b = (8192u / es) / 8u * 8u;
  return b < 128u ? 128u : b;
}

int hsds_encode_bitshuffle_batch(hsds_engine* e, const void* d_src, uint64_t src_extent, uint64_t src_bytes,
                                 const hsds_chunk_desc* d_chunks, int64_t nchunks, void* d_dst, uint64_t dst_extent,
                                 int64_t* d_sizes, int32_t* d_status, int itemsize, int block, void* stream) {
  if (!e || nchunks < 0 || (nchunks && (!d_src || !d_chunks || !d_dst || !d_sizes || !d_status))) return HSDS_ERR_ARG;
  if (itemsize < 1 || itemsize > 4096 || block < 0 || block % 8) return HSDS_ERR_ARG;
  if (nchunks == 0) return HSDS_OK;
  if (nchunks > (int64_t)(1u << 22)) return HSDS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  WsGuard guard(e, stream);
  const uint32_t es = (uint32_t)itemsize;
  const uint64_t bsz = block ? (uint64_t)block : host_bshuf_default_block(es);
  // work areas and the transposition staging are sized by the batch's own bytes (sum of
  // src_len, 16-byte aligned per chunk: the staging holds the chunks back to back), not by
  // the extent of the buffer they sit in (a flush from a large cache arena)
  const uint64_t sb = src_bytes ? src_bytes + 16u * (uint64_t)nchunks : src_extent + 16u * (uint64_t)nchunks;
  // every block but a chunk's last is bsz elements: slots and segments bounded by sb
  const uint64_t slot_cap64 = sb / (bsz * es) + (uint64_t)nchunks + 64;
  const uint64_t seg_cap64 = sb / hd::SEG + slot_cap64 + 64;
  if (seg_cap64 > 0xffffffffull || (uint64_t)block * es > 0xffffffffull) return HSDS_ERR_ARG;
  const uint32_t slot_cap = (uint32_t)slot_cap64, seg_cap = (uint32_t)seg_cap64;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t sz_slots = al((size_t)slot_cap * sizeof(EncItem));
  const size_t sz_iout = al((size_t)slot_cap * sizeof(ItemOut));
  const size_t sz_lzsize = al((size_t)slot_cap * 4);
  const size_t sz_counts = al((size_t)nchunks * 4);
  const size_t sz_offs = al((size_t)(nchunks + 1) * 4);
  const size_t sz_geom = al((size_t)nchunks * sizeof(EncGeom));
  const size_t sz_sp = al((size_t)seg_cap * sizeof(hd::SegParse));
  const size_t sz_meta = al((size_t)seg_cap * sizeof(SegMeta));
  const size_t sz_adler = al((size_t)slot_cap * 4);
  const size_t sz_soffs = al((size_t)(nchunks + 1) * 8);
  const size_t need = sz_slots + sz_iout + sz_lzsize + 2 * sz_counts + 2 * sz_offs + sz_geom + sz_sp + sz_meta +
                      sz_adler + sz_soffs + 256;
  if (grow((void**)&e->ews, &e->ews_bytes, need)) return HSDS_ERR_DEVICE;
  uint8_t* w = e->ews;
  EncItem* slots = (EncItem*)w; w += sz_slots;
  ItemOut* iout = (ItemOut*)w; w += sz_iout;
  uint32_t* lzsize = (uint32_t*)w; w += sz_lzsize;
  uint32_t* counts = (uint32_t*)w; w += sz_counts;
  uint32_t* segcnt = (uint32_t*)w; w += sz_counts;
  uint32_t* offs = (uint32_t*)w; w += sz_offs;
  uint32_t* segoffs = (uint32_t*)w; w += sz_offs;
  EncGeom* geom = (EncGeom*)w; w += sz_geom;
  hd::SegParse* sp = (hd::SegParse*)w; w += sz_sp;
  SegMeta* meta = (SegMeta*)w; w += sz_meta;
  uint32_t* adler = (uint32_t*)w; w += sz_adler;
  uint64_t* soffs = (uint64_t*)w; w += sz_soffs;
  uint32_t* ctr = (uint32_t*)w;
  if (grow((void**)&e->escr, &e->escr_bytes, (size_t)seg_cap * hd::SEG_TOK * 2 + 256)) return HSDS_ERR_DEVICE;
  uint16_t* tok = (uint16_t*)e->escr;
  if (grow((void**)&e->tmp, &e->tmp_bytes, sb ? sb : 1)) return HSDS_ERR_DEVICE;
  uint8_t* stg = e->tmp;
  if (hipMemsetAsync(ctr, 0, 32, st) != hipSuccess) return HSDS_ERR_DEVICE;
  const int tpb = 256;
  const int nb = (int)((nchunks + tpb - 1) / tpb);
  hipEventRecord(e->ev2, st);
  hipLaunchKernelGGL(bs_plan_kernel, dim3(nb), dim3(tpb), 0, st, d_chunks, nchunks, counts, segcnt, geom, d_status,
                     es, (uint32_t)block, src_extent);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, counts, offs, nchunks);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, segcnt, segoffs, nchunks);
  hipLaunchKernelGGL(stage_scan_kernel, dim3(1), dim3(1024), 0, st, d_chunks, nchunks, soffs);
  hipLaunchKernelGGL(bs_fill_kernel, dim3(nb), dim3(tpb), 0, st, d_chunks, nchunks, offs, geom, slots, d_status, stg,
                     slot_cap, soffs, sb);
  const unsigned gy = (unsigned)(nchunks < 65535 ? nchunks : 65535);
  hipLaunchKernelGGL(bs_trans_kernel, dim3(16, gy), dim3(256), 0, st, (const uint8_t*)d_src, d_chunks, nchunks, geom,
                     d_status, stg, soffs);
  auto grid_for = [&](int per_cu, int64_t cap) {
    int64_t g = (int64_t)e->num_cus * per_cu;
    if (g > cap) g = cap;
    return (unsigned)(g < 1 ? 1 : g);
  };
  hipLaunchKernelGGL(parse_kernel, dim3(grid_for(e->parse_blocks_per_cu, slot_cap)), dim3(64), 0, st, slots, offs,
                     segoffs, nchunks, ctr, sp, meta, tok, adler, seg_cap, BSHUF_PARSE_LEVEL, 0u,
                     slot_cap, (uint16_t*)nullptr, 0u);
  const unsigned lgrid = grid_for(e->lz4w_blocks_per_cu, slot_cap);
  hipLaunchKernelGGL(lz4_block_kernel, dim3(lgrid), dim3(64), 0, st, slots, offs, segoffs, nchunks, sp, tok, lzsize,
                     seg_cap, BSHUF_PARSE_LEVEL, d_chunks, (uint8_t*)d_dst, geom, iout, d_status, 0, 0, 0u, slot_cap);
  hipLaunchKernelGGL(bs_layout_kernel, dim3(nb), dim3(tpb), 0, st, (const uint8_t*)d_src, d_chunks, nchunks,
                     (uint8_t*)d_dst, offs, segoffs, geom, lzsize, iout, d_sizes, d_status,
                     (uint32_t)((uint64_t)block * es), seg_cap);
  hipLaunchKernelGGL(lz4_block_kernel, dim3(lgrid), dim3(64), 0, st, slots, offs, segoffs, nchunks, sp, tok, lzsize,
                     seg_cap, BSHUF_PARSE_LEVEL, d_chunks, (uint8_t*)d_dst, geom, iout, d_status, 1, 0, 0u, slot_cap);
  hipEventRecord(e->ev3, st);
  e->ev_enc_valid = 1;
  return hipGetLastError() == hipSuccess ? HSDS_OK : HSDS_ERR_DEVICE;
}

// frame bound: header, a u32 size and an LZ4 worst case (n + n / 255 + 16) per block, leftover
int64_t hsds_bitshuffle_bound(int64_t n, int itemsize, int block) {
  if (n < 0 || itemsize < 1 || block < 0 || block % 8) return HSDS_ERR_ARG;
  const int64_t bb = (block ? (int64_t)block : (int64_t)host_bshuf_default_block((uint32_t)itemsize)) * itemsize;
  const int64_t nblk = n / bb + 1;
  return 12 + n + nblk * (4 + 16) + n / 255 + 16;
}

int64_t hsds_bitshuffle_compress(hsds_engine* e, const void* src, int64_t n, int itemsize, int block, void* dst,
                                 int64_t cap) {
  const int64_t bound = hsds_bitshuffle_bound(n, itemsize, block);
  if (!e || bound < 0 || (n && !src) || !dst || cap < 12) return HSDS_ERR_ARG;
  if (n % itemsize) return HSDS_ERR_ARG;
  if (hipSetDevice(e->device) != hipSuccess) return HSDS_ERR_DEVICE;
  WsGuard guard(e, nullptr);
  const size_t desc_off = ((size_t)n + 255) & ~(size_t)255;
  const size_t stat_off = ((size_t)bound + 255) & ~(size_t)255;
  if (grow((void**)&e->h_dev_src, &e->h_dev_src_bytes, desc_off + sizeof(hsds_chunk_desc))) return HSDS_ERR_DEVICE;
  if (grow((void**)&e->h_dev_dst, &e->h_dev_dst_bytes, stat_off + 64)) return HSDS_ERR_DEVICE;
  hsds_chunk_desc c = {0, (uint64_t)n, 0, (uint64_t)bound};
  hsds_chunk_desc* dd = (hsds_chunk_desc*)(e->h_dev_src + desc_off);
  int64_t* dsize = (int64_t*)(e->h_dev_dst + stat_off);
  int32_t* dstat = (int32_t*)(e->h_dev_dst + stat_off + 16);
  if (n && hipMemcpy(e->h_dev_src, src, (size_t)n, hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  if (hipMemcpy(dd, &c, sizeof(c), hipMemcpyHostToDevice) != hipSuccess) return HSDS_ERR_DEVICE;
  int r = hsds_encode_bitshuffle_batch(e, e->h_dev_src, (uint64_t)n, (uint64_t)n, dd, 1, e->h_dev_dst, (uint64_t)bound, dsize,
                                       dstat, itemsize, block, nullptr);
  if (r) return r;
  int32_t status = 0;
  int64_t size = 0;
  if (hipMemcpy(&status, dstat, 4, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  if (status) return status;
  if (hipMemcpy(&size, dsize, 8, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  if (size < 12) return HSDS_ERR_SIZE;
  if (size > cap) return HSDS_ERR_SIZE;
  if (hipMemcpy(dst, e->h_dev_dst, (size_t)size, hipMemcpyDeviceToHost) != hipSuccess) return HSDS_ERR_DEVICE;
  return size;
}

int64_t hsds_compress(hsds_engine* e, const void* src, int64_t n, int clevel, int shuffle, int typesize, void* dst,
                      int64_t cap) {
  return hsds_compress_codec(e, src, n, clevel, shuffle, typesize, HSDS_CNAME_ZLIB, dst, cap);
}

}  // extern "C"
