/*
 * hsds_amd.h -- C ABI of the MI355X chunk codec / hyperslab engine for the HSDS
 * data-node hot path.  Plain pointers and sizes only; every entry point returns
 * 0 (or a byte count) on success and a negative HSDS_ERR_* code on failure.
 *
 * Reference interfaces replaced (paths relative to the HSDS 0.9.4 source tree):
 *   hsds_uncompress      <- hsds/util/storUtil.py:182  _uncompress(data, compressor, shuffle, level, dtype, chunk_shape)
 *   hsds_decode_batch    <- the per-chunk _uncompress loop of getStorBytes (storUtil.py:486-519),
 *                           getHyperChunks (storUtil.py:557-580) and get_chunk_bytes
 *                           (hsds/datanode_lib.py:796-945), batched over many chunks
 *   hsds_shuffle         <- storUtil.py:94   _shuffle(codec=1, ...)   (numcodecs.Shuffle.encode)
 *   hsds_unshuffle       <- storUtil.py:136  _unshuffle(codec=1, ...) (numcodecs.Shuffle.decode)
 *   hsds_copy_batch      <- hsds/util/chunkUtil.py:882 chunkReadSelection (chunk_arr[slices]) and
 *                           hsds/chunk_crawl.py:418 np_arr[data_sel] = chunk_arr (SN slab scatter),
 *                           chunk_crawl.py:135 arr[data_sel] (SN write gather)
 *   hsds_compare_batch + hsds_copy_batch_if
 *                        <- chunkUtil.py:932 chunkWriteSelection (ndarray_compare, then chunk_arr[slices] = data)
 *   hsds_compress        <- storUtil.py:238  _compress(data, compressor, level, shuffle, dtype, chunk_shape)
 *   hsds_encode_batch    <- the per-chunk _compress of putStorBytes (storUtil.py:584-600) reached from
 *                           write_s3_obj (hsds/datanode_lib.py:126-311), batched over many dirty chunks
 *   hsds_encode_batch_codec / hsds_compress_codec
 *                        <- the same with Blosc(cname = "lz4" / "lz4hc" / "blosclz") (storUtil.py:255-262)
 *   hsds_encode_bitshuffle_batch / hsds_bitshuffle_compress / hsds_bitshuffle_bound
 *                        <- storUtil.py:94-131 _shuffle(codec=2, ...) (bitshuffle.compress_lz4 behind
 *                           the 12-byte header), reached from _compress(shuffle=2) (storUtil.py:243-251)
 *
 * Threading: an engine is bound to one device and is re-entrant: its calls may come from
 * any host threads (a DN running them off the event loop in a thread pool).  Calls that
 * use the engine's workspace (decode, encode, the host-buffer codec calls) hold an
 * engine mutex while they enqueue, and a call on a different stream than the previous
 * workspace user first waits (hipStreamWaitEvent) for that use to finish on the device.
 * All *_batch calls are asynchronous on the given hipStream_t (pass NULL for the
 * default stream); host-buffer calls are synchronous.
 */
#ifndef HSDS_AMD_H
#define HSDS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (per call and per chunk) ------------------------------- */
#define HSDS_OK 0
#define HSDS_ERR_FRAME -1       /* malformed Blosc frame                          */
#define HSDS_ERR_DATA -2        /* corrupt deflate data, bad adler32, bad header  */
#define HSDS_ERR_TRUNC -3       /* stream ends before its end-of-stream marker    */
#define HSDS_ERR_SIZE -4        /* decoded size differs from the expected size    */
#define HSDS_ERR_UNSUPPORTED -5 /* snappy Blosc codec, bitshuffle, rank > 8 ...  */
#define HSDS_ERR_ARG -6         /* invalid argument                               */
#define HSDS_ERR_DEVICE -7      /* HIP runtime failure                            */

/* compressor codes (storUtil._uncompress compressor argument) */
#define HSDS_COMP_NONE 0        /* None / "scaleoffset"                           */
#define HSDS_COMP_ZLIB 1        /* "gzip" / "deflate" / "zlib"                    */
#define HSDS_COMP_OTHER 2       /* lz4 / lz4hc / blosclz / zstd: Blosc frames only */

/* Blosc inner codec of the write path (storUtil._compress cname) */
#define HSDS_CNAME_ZLIB 0       /* "gzip" / "deflate" / "zlib": Blosc codec 3      */
#define HSDS_CNAME_LZ4 1        /* "lz4": Blosc codec 1, c-blosc's lz4 blocksize   */
#define HSDS_CNAME_LZ4HC 2      /* "lz4hc": Blosc codec 1, HCR blocksize           */
#define HSDS_CNAME_BLOSCLZ 3    /* "blosclz": Blosc codec 0, c-blosc's L1 blocksize */
#define HSDS_CNAME_ZSTD 4       /* "zstd": Blosc codec 4, HCR blocksize, never split */

/* shuffle codes (storUtil.BYTE_SHUFFLE / BIT_SHUFFLE) */
#define HSDS_SHUFFLE_NONE 0
#define HSDS_SHUFFLE_BYTE 1
#define HSDS_SHUFFLE_BIT 2      /* bitshuffle+LZ4 objects (decode, no outer codec) */

#define HSDS_MAX_RANK 8

typedef struct hsds_engine hsds_engine;

/* One stored chunk in a batch: byte ranges in the batch source / destination. */
typedef struct {
  uint64_t src_off;  /* offset of the stored (compressed) bytes in the source buffer   */
  uint64_t src_len;  /* stored length                                                  */
  uint64_t dst_off;  /* offset of the decoded chunk in the destination buffer          */
  uint64_t dst_len;  /* expected decoded size = prod(chunk_shape) * itemsize           */
} hsds_chunk_desc;

/* One strided N-d region copy (numpy basic-slicing semantics):
 *   for every index tuple i (0 <= i[k] < count[k]):
 *     dst[dst_off + sum i[k]*dst_stride[k]] <- src[src_off + sum i[k]*src_stride[k]]
 * moving `itemsize` bytes per element.  Strides are in bytes and already include
 * the slice step.  Every count must be below 2^31 (hsds_amd.engine splits larger
 * dimensions into several records); a record with a larger count copies nothing. */
typedef struct {
  uint64_t src_off;
  uint64_t dst_off;
  int64_t src_stride[HSDS_MAX_RANK];
  int64_t dst_stride[HSDS_MAX_RANK];
  int64_t count[HSDS_MAX_RANK];
  int32_t rank;
  int32_t itemsize;
} hsds_copy_desc;

/* element kinds for hsds_compare_batch (numpy array_equal semantics) */
#define HSDS_KIND_BYTES 0       /* integers, bool, fixed strings: bytewise         */
#define HSDS_KIND_F16 1
#define HSDS_KIND_F32 2
#define HSDS_KIND_F64 3
#define HSDS_KIND_C64 4
#define HSDS_KIND_C128 5

/* ---- engine lifecycle ------------------------------------------------------ */
int hsds_engine_create(int device, hsds_engine** out);
void hsds_engine_destroy(hsds_engine* e);
const char* hsds_version(void);
const char* hsds_strerror(int status);

/* Tuning of the inflate kernel: segment over-provisioning against the previous
 * deflate block in 16ths (0..16), warm-up bits before a segment (0..4096), wavefronts
 * per zlib stream (0: by batch size -- four or two when the batch's streams times that
 * fit in the resident wavefronts --, 1, 2, 4 or 8), repair rounds per window (0..64).  Any setting
 * decodes the same bytes; it only moves work between the phases and wavefronts.
 * Defaults are set by hsds_engine_create; HSDS_TUNE_KEEP (rounds: -1) leaves a setting
 * unchanged. */
#define HSDS_TUNE_KEEP 0xffffffffu
int hsds_set_tuning(hsds_engine* e, uint32_t seg_over16, uint32_t warmup_bits, uint32_t waves_per_stream,
                    int32_t repair_rounds);

/* ---- partition ------------------------------------------------------------- */
/* getObjPartition (hsds/util/idUtil.py:61-66, 481-486) for a batch of chunk ids of one
 * dataset: owner[i] = int(md5(prefix + "i0_i1_..")[:5], 16) % world, where row i of the
 * n x rank index array idx holds the chunk index (chunkUtil.getChunkId,
 * chunkUtil.py:353-371: prefix = "c-<dset uuid>_").  Host-only; no engine needed. */
int hsds_partition_ids(const char* prefix, int rank, const int64_t* idx, int64_t n, int world, int32_t* owner);

/* ---- decode -------------------------------------------------------------- */
/* Batched, device-resident decode.  d_src, d_chunks, d_dst, d_status are device
 * pointers; decoded chunk k is written to d_dst + d_chunks[k].dst_off and its
 * status (HSDS_OK or HSDS_ERR_*) to d_status[k].  compressor / shuffle / itemsize
 * follow storUtil._uncompress: Blosc frames are detected per chunk
 * (cbuffer_metainfo typesize > 0) and unshuffle themselves; otherwise a zlib
 * stream is inflated (compressor == HSDS_COMP_ZLIB) and then byte-unshuffled
 * with `itemsize` when shuffle == HSDS_SHUFFLE_BYTE.  dst_extent = bytes spanned by
 * d_dst (max dst_off + dst_len); the engine keeps a staging buffer of that size
 * for chunks that must be unshuffled after inflate.
 * shuffle == HSDS_SHUFFLE_BIT with compressor == HSDS_COMP_NONE decodes the
 * bitshuffle+LZ4 objects of storUtil._shuffle(codec=2) (12-byte header, replaces
 * storUtil._unshuffle codec 2, storUtil.py:144-174; dst_len = the chunk bytes the
 * header must state).  With an outer compressor, decode with HSDS_SHUFFLE_NONE first
 * and then run this on its outputs (per-chunk status HSDS_ERR_UNSUPPORTED otherwise). */
int hsds_decode_batch(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks,
                      int64_t nchunks, void* d_dst, uint64_t dst_extent, int32_t* d_status,
                      int compressor, int shuffle, int itemsize, void* stream);

/* Host-buffer single chunk: mirrors storUtil._uncompress.  Returns the decoded
 * length (== expected) or a negative HSDS_ERR_* code.  expected < 0 means the
 * size is unknown (zlib.decompress without a chunk shape): capacity is -expected
 * and the actual decoded length is returned. */
int64_t hsds_uncompress(hsds_engine* e, const void* src, int64_t srclen, int compressor, int shuffle,
                        int itemsize, void* dst, int64_t expected);

/* Device time (ms) of the inflate kernel of the most recent hsds_decode_batch,
 * measured with HIP events on that call's stream (valid after the stream syncs). */
int hsds_last_inflate_ms(hsds_engine* e, float* ms);

/* ---- shuffle ------------------------------------------------------------- */
int hsds_shuffle_device(hsds_engine* e, const void* d_src, int64_t n, int itemsize, void* d_dst,
                        void* stream);
int hsds_unshuffle_device(hsds_engine* e, const void* d_src, int64_t n, int itemsize, void* d_dst,
                          void* stream);
int hsds_shuffle(hsds_engine* e, const void* src, int64_t n, int itemsize, void* dst);
int hsds_unshuffle(hsds_engine* e, const void* src, int64_t n, int itemsize, void* dst);

/* ---- hyperslab selection ---------------------------------------------------- */
int hsds_copy_batch(hsds_engine* e, const void* d_src, void* d_dst, const hsds_copy_desc* d_desc,
                    int64_t n, void* stream);
/* d_differs[k] = 1 if region k of d_a (chunk) differs from region k of d_b (data)
 * under numpy array_equal semantics for `kind`, else 0.  The region geometry is
 * desc.src_* for d_b and desc.dst_* for d_a (the write direction). */
int hsds_compare_batch(hsds_engine* e, const void* d_b, const void* d_a, const hsds_copy_desc* d_desc,
                       int64_t n, int kind, int32_t* d_differs, void* stream);
/* copy only the descriptors whose d_flags[k] != 0 */
int hsds_copy_batch_if(hsds_engine* e, const void* d_src, void* d_dst, const hsds_copy_desc* d_desc,
                       int64_t n, const int32_t* d_flags, void* stream);

/* Hyperslab plan geometry for hsds_plan_descs: the pieces of a selection are the
 * Cartesian product (C order) of per-dimension tables, one entry per chunk the slice
 * touches in that dimension (chunkUtil.getChunkIds / getChunkCoverage / getDataCoverage,
 * chunkUtil.py:459-790): chunk-relative start, count and slab start. */
typedef struct {
  int32_t rank;
  int32_t itemsize;
  int32_t mode;                          /* HSDS_PLAN_* */
  int32_t reserved;
  int64_t nk[HSDS_MAX_RANK];             /* table length per dimension                 */
  int64_t chunk_stride[HSDS_MAX_RANK];   /* C strides of a chunk (layout), bytes       */
  int64_t slab_stride[HSDS_MAX_RANK];    /* C strides of the slab (selection shape)    */
  int64_t step[HSDS_MAX_RANK];           /* selection step per dimension               */
  int64_t slab_base;                     /* slab byte offset (PLACE / GATHER)          */
} hsds_plan_geom;
#define HSDS_PLAN_PACK 0        /* decoded chunk [chunk_sel] -> packed piece (SN read)   */
#define HSDS_PLAN_PLACE 1       /* packed piece -> slab [data_sel]                       */
#define HSDS_PLAN_GATHER 2      /* slab [data_sel] -> packed piece (SN write gather)     */
#define HSDS_PLAN_APPLY 3       /* packed piece -> chunk [chunk_sel] (PUT_Chunk)         */
#define HSDS_PLAN_APPLY_BCAST 4 /* the one element at d_poff[k] -> chunk [chunk_sel]     */
#define HSDS_PLAN_DIRECT 5      /* decoded chunk [chunk_sel] -> slab [data_sel] (PACK and
                                   PLACE in one record: the root's own pieces; d_poff unused) */
/* One copy record per piece, built on the device (chunk_crawl.py:118-150,395-418):
 * d_tabs holds, per dimension d in order, nk[d] chunk-relative starts, nk[d] counts and
 * nk[d] slab starts (int64); d_piece[k] is piece k's index in the product grid,
 * d_poff[k] its byte offset in the packed buffer and d_coff[k] (PACK / APPLY) the byte
 * offset of its chunk array (PACK / APPLY / DIRECT).  Records go to d_out[0..n). */
int hsds_plan_descs(hsds_engine* e, const hsds_plan_geom* geom, const int64_t* d_tabs, const int64_t* d_piece,
                    const int64_t* d_poff, const int64_t* d_coff, int64_t n, hsds_copy_desc* d_out,
                    void* stream);

/* ---- host response buffers (the "no gather" sharded read) ---------
 * The SN streams each page of a GET_Value to the client (chunk_sn.py:1085-1135): the
 * bytes end in host memory.  hsds_host_map page-locks n bytes of host memory at p
 * (private, or a shared-memory mapping every rank of the node maps) and returns the
 * address kernels on the engine's device write through (zero-copy over PCIe), so each GPU
 * places its own pieces straight into the response: no gather over xGMI. */
int hsds_host_map(hsds_engine* e, void* p, uint64_t n, void** d_ptr);
int hsds_host_unmap(hsds_engine* e, void* p);

/* ---- read-batch staging (the DN's get_chunk batch, datanode_lib.py:948-1142) -----
 * The stored objects a batch fetched (storUtil.getStorBytes' bytes, storUtil.py:450-522)
 * are host buffers srcs[k] of lens[k] bytes.  hsds_stage_upload copies object k to
 * h_stage + offs[k] (page-locked, offs ascending, every object inside [0, total)) with
 * `threads` host threads, and queues the host-to-device copy of h_stage[0, total) to
 * d_dst on `stream` in pieces of whole objects, each as soon as it is staged.
 * Returns once every copy is queued; h_stage must stay allocated until the stream has
 * run them. */
int hsds_stage_upload(hsds_engine* e, const void* const* srcs, const uint64_t* lens, const uint64_t* offs,
                      int64_t n, void* h_stage, void* d_dst, uint64_t total, int threads, void* stream);

/* ---- encode (write path) ---------------------------------------------------- */
/* Batched, device-resident encode into HSDS F1 objects: chunk k (d_chunks[k].src_off /
 * src_len in d_src) becomes a Blosc1 frame with the zlib codec at level `clevel`
 * (0-9), the byte-shuffle flag `shuffle` (0 / 1) and `typesize` (the reference's
 * _compress always uses typesize 1) at d_dst + dst_off; dst_len is the frame
 * capacity and must be >= src_len + 16 (c-blosc MAX_OVERHEAD).  Frame geometry,
 * raw splits and the memcpyed fallback follow c-blosc 1.21 blosc_compress; the
 * deflate streams are produced by the GPU encoder (any valid deflate: they inflate
 * through libz, c-blosc and storUtil._uncompress).  The frame size goes to
 * d_sizes[k] (int64), the status to d_status[k].  dst_extent = bytes spanned by d_dst. */
int hsds_encode_batch(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                      void* d_dst, uint64_t dst_extent, int64_t* d_sizes, int32_t* d_status, int clevel,
                      int shuffle, int typesize, void* stream);

/* The same with the Blosc inner codec `cname` (HSDS_CNAME_*): lz4 / lz4hc frames
 * carry LZ4 blocks, blosclz frames BloscLZ blocks (any valid block; the frame layout
 * follows c-blosc 1.21 for that codec).  hsds_encode_batch == cname HSDS_CNAME_ZLIB. */
int hsds_encode_batch_codec(hsds_engine* e, const void* d_src, const hsds_chunk_desc* d_chunks, int64_t nchunks,
                            void* d_dst, uint64_t dst_extent, int64_t* d_sizes, int32_t* d_status, int clevel,
                            int shuffle, int typesize, int cname, void* stream);

/* Host-buffer single object: mirrors storUtil._compress for the zlib compressor.
 * Returns the frame size (<= cap; cap must be >= n + 16) or a negative HSDS_ERR_*. */
int64_t hsds_compress(hsds_engine* e, const void* src, int64_t n, int clevel, int shuffle, int typesize,
                      void* dst, int64_t cap);
/* ... and for any HSDS_CNAME_* */
int64_t hsds_compress_codec(hsds_engine* e, const void* src, int64_t n, int clevel, int shuffle, int typesize,
                            int cname, void* dst, int64_t cap);

/* Batched bitshuffle+LZ4 objects (storUtil._shuffle codec 2, storUtil.py:103-131):
 * chunk k (src_len bytes of itemsize-byte elements) becomes u64 BE src_len, u32 BE
 * block * itemsize (0 when block == 0: the bitshuffle default block), then per block
 * of `block` elements (0: bshuf_default_block_size) a u32 BE size and the LZ4 block of
 * the block's bit transposition, a last block of the remaining elements rounded down
 * to a multiple of 8, and the n % 8 leftover elements raw.  LZ4 bytes come from the
 * GPU writer (any valid block; they decode through bitshuffle.decompress_lz4).
 * src_extent = bytes spanned by d_src (descriptor bounds check); src_bytes = sum of
 * the batch's src_len (0: use src_extent): the engine's scratch (block work items,
 * LZ4 token segments, the transposition staging, which holds the chunks back to
 * back) is sized by it, so a flush of a few chunks from a large arena stays small;
 * a batch whose src_len sum exceeds src_bytes fails with HSDS_ERR_ARG.  dst_len
 * should be >= hsds_bitshuffle_bound(src_len, ...), else the chunk may fail with
 * HSDS_ERR_SIZE.  Frame sizes to d_sizes[k], statuses to d_status[k]. */
int hsds_encode_bitshuffle_batch(hsds_engine* e, const void* d_src, uint64_t src_extent, uint64_t src_bytes,
                                 const hsds_chunk_desc* d_chunks, int64_t nchunks, void* d_dst, uint64_t dst_extent,
                                 int64_t* d_sizes, int32_t* d_status, int itemsize, int block, void* stream);
/* Worst-case object size for n bytes (LZ4 bound per block + headers). */
int64_t hsds_bitshuffle_bound(int64_t n, int itemsize, int block);
/* Host-buffer single object (storUtil._shuffle(2, data, chunk_shape, dtype)).
 * Returns the object size (<= cap) or a negative HSDS_ERR_*. */
int64_t hsds_bitshuffle_compress(hsds_engine* e, const void* src, int64_t n, int itemsize, int block, void* dst,
                                 int64_t cap);

/* Device time (ms) of the deflate kernel of the most recent hsds_encode_batch. */
int hsds_last_deflate_ms(hsds_engine* e, float* ms);

#ifdef __cplusplus
}
#endif

#endif /* HSDS_AMD_H */
