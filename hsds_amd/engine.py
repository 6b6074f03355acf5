"""Batched, device-resident chunk decode and hyperslab copies (torch tensors in HBM).

This is the batched form of the DN hot loop: the reference decodes one chunk per
request (datanode_lib.get_chunk -> get_chunk_bytes -> storUtil._uncompress,
hsds/datanode_lib.py:796-945, 948-1142) and copies one selection per chunk
(chunkUtil.chunkReadSelection, chunkUtil.py:882; chunk_crawl.py:418).  Here a whole
request's chunks go to the GPU in one call.  torch is used only for device memory
and streams; all byte work happens in the C-ABI kernels.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat

CHUNK_DESC_DTYPE = np.dtype([("src_off", "<u8"), ("src_len", "<u8"), ("dst_off", "<u8"), ("dst_len", "<u8")])
COPY_DESC_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("src_stride", "<i8", (nat.MAX_RANK,)),
                            ("dst_stride", "<i8", (nat.MAX_RANK,)), ("count", "<i8", (nat.MAX_RANK,)),
                            ("rank", "<i4"), ("itemsize", "<i4")])
assert CHUNK_DESC_DTYPE.itemsize == 32 and COPY_DESC_DTYPE.itemsize == 216


def _stream_handle(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def _ptr(t):
    if t is None:
        return None
    if isinstance(t, HostBuffer):
        return t.d_ptr
    if not t.is_cuda:
        raise ValueError("device tensor expected")
    return t.data_ptr()


class HostBuffer:
    """Page-locked host memory that kernels of `device` write directly (hsds_host_map):
    the response buffer of the "no gather" sharded read.  `path`: a shared-memory file
    (/dev/shm) that every rank of the node maps, so all GPUs place their pieces into the
    same buffer; otherwise private memory.  `.array` is the host uint8 view."""

    def __init__(self, nbytes, device, path=None, create=True):
        import mmap
        import os as _os
        self.nbytes = int(nbytes)
        self.device = torch.device(device)
        self.path = path
        if path is None:
            self._mm = mmap.mmap(-1, self.nbytes)
        else:
            if create:
                fd = _os.open(path, _os.O_RDWR | _os.O_CREAT, 0o600)
                _os.ftruncate(fd, self.nbytes)
            else:
                fd = _os.open(path, _os.O_RDWR)
            try:
                self._mm = mmap.mmap(fd, self.nbytes)
            finally:
                _os.close(fd)
        self.array = np.frombuffer(self._mm, np.uint8, self.nbytes)
        self.array[::4096] = self.array[::4096]          # fault the pages in before locking them
        self._eng = nat.engine(self.device.index)
        self._hptr = self.array.ctypes.data
        d = ctypes.c_void_p()
        rc = nat.lib().hsds_host_map(self._eng.h, self._hptr, self.nbytes, ctypes.byref(d))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_host_map")
        self.d_ptr = int(d.value)

    def close(self):
        if self._hptr:
            nat.lib().hsds_host_unmap(self._eng.h, self._hptr)
            self._hptr = 0
            # the mapping closes with its last numpy view (pages handed to a sink may
            # still be referenced)
            self.array = None
            self._mm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def to_device_bytes(arr, device, stream=None):
    """numpy structured / uint8 array -> uint8 tensor on `device`, queued on `stream` (the
    current stream by default), the stream the kernel that reads it is launched on: the
    bytes go through page-locked staging with an asynchronous copy (a pageable copy makes
    torch synchronise the stream, i.e. wait for every kernel queued before it).  The
    staging block stays reserved by torch's pinned-memory cache until the copy ran, and
    the device tensor is recorded on `stream`, so its memory is not reused while a kernel
    on that stream may still read it."""
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    h = torch.empty(max(raw.size, 1), dtype=torch.uint8, pin_memory=True)
    h.numpy()[:raw.size] = raw
    if stream is None:
        return h[:raw.size].to(device, non_blocking=True)
    with torch.cuda.stream(stream):
        t = h[:raw.size].to(device, non_blocking=True)
    t.record_stream(stream)
    return t


class ChunkEngine:
    """Batched decode of HSDS chunk objects (F1 Blosc-zlib frames, F2 zlib+shuffle
    streams, raw chunks) resident in device memory."""

    def __init__(self, device=None):
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.eng = nat.engine(self.device.index)

    def set_tuning(self, **kw):
        self.eng.set_tuning(**kw)

    def decode(self, src, chunk_descs, dst, status, compressor="zlib", shuffle=1, itemsize=1, stream=None):
        """Asynchronously decode `chunk_descs` (uint8 device tensor holding
        CHUNK_DESC_DTYPE records, or a numpy array of them) from `src` into `dst`;
        per-chunk HSDS_* status codes land in `status` (int32 device tensor)."""
        if isinstance(chunk_descs, np.ndarray):
            n = chunk_descs.size
            chunk_descs = to_device_bytes(chunk_descs, self.device, stream)
        else:
            n = chunk_descs.numel() // CHUNK_DESC_DTYPE.itemsize
        comp = {None: 0, "": 0, "scaleoffset": 0, "gzip": 1, "deflate": 1, "zlib": 1}.get(compressor, 2)
        rc = nat.lib().hsds_decode_batch(self.eng.h, _ptr(src), _ptr(chunk_descs), n, _ptr(dst),
                                         dst.numel() * dst.element_size(), _ptr(status), comp, int(shuffle),
                                         int(itemsize), _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_decode_batch")
        return chunk_descs

    def last_inflate_ms(self):
        return self.eng.last_inflate_ms()

    def encode(self, src, chunk_descs, dst, sizes, status, clevel=5, shuffle=1, typesize=1, stream=None,
               compressor="zlib"):
        """Asynchronously encode the chunks `chunk_descs` (src_off/src_len in `src`)
        into HSDS objects -- Blosc1 frames with the zlib (default), lz4 or lz4hc codec,
        what storUtil._compress stores (storUtil.py:238-281) -- at dst_off in `dst`
        (dst_len = capacity >= src_len + 16).  Frame sizes land in `sizes` (int64
        device tensor), HSDS_* status codes in `status` (int32)."""
        cname = nat.cname_code(compressor)
        if cname is None:
            raise NotImplementedError(f"Blosc codec {compressor!r} has no encoder in the hsds_amd engine")
        if isinstance(chunk_descs, np.ndarray):
            n = chunk_descs.size
            chunk_descs = to_device_bytes(chunk_descs, self.device, stream)
        else:
            n = chunk_descs.numel() // CHUNK_DESC_DTYPE.itemsize
        rc = nat.lib().hsds_encode_batch_codec(self.eng.h, _ptr(src), _ptr(chunk_descs), n, _ptr(dst),
                                               dst.numel() * dst.element_size(), _ptr(sizes), _ptr(status),
                                               int(clevel), int(shuffle), int(typesize), cname,
                                               _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_encode_batch_codec")
        return chunk_descs

    def encode_bitshuffle(self, src, chunk_descs, dst, sizes, status, itemsize, block=2048, stream=None,
                          src_bytes=None):
        """Asynchronously write bitshuffle+LZ4 objects (storUtil._shuffle codec 2,
        storUtil.py:103-131) for the chunks `chunk_descs` at dst_off in `dst` (dst_len =
        capacity, >= nat.lib().hsds_bitshuffle_bound(src_len, itemsize, block)).  `block`
        is the bitshuffle block in elements (HSDS config bit_shuffle_default_blocksize,
        2048).  The engine's scratch is sized by `src_bytes` (the batch's total src_len,
        taken from host descriptors when not given), not by the extent of `src`."""
        if isinstance(chunk_descs, np.ndarray):
            n = chunk_descs.size
            if src_bytes is None:
                src_bytes = int(chunk_descs["src_len"].sum()) if n else 0
            chunk_descs = to_device_bytes(chunk_descs, self.device, stream)
        else:
            n = chunk_descs.numel() // CHUNK_DESC_DTYPE.itemsize
        rc = nat.lib().hsds_encode_bitshuffle_batch(self.eng.h, _ptr(src), src.numel() * src.element_size(),
                                                    int(src_bytes or 0), _ptr(chunk_descs), n, _ptr(dst),
                                                    dst.numel() * dst.element_size(), _ptr(sizes), _ptr(status),
                                                    int(itemsize), int(block), _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_encode_bitshuffle_batch")
        return chunk_descs

    def last_deflate_ms(self):
        return self.eng.last_deflate_ms()

    def copy(self, src, dst, copy_descs, stream=None, flags=None):
        """Asynchronous strided region copies (COPY_DESC_DTYPE records).  Dimensions of
        2^31 elements or more (outside the ABI's range) are split into several records."""
        if isinstance(copy_descs, np.ndarray):
            if flags is None:
                copy_descs = split_large_copy_descs(copy_descs)
            n = copy_descs.size
            copy_descs = to_device_bytes(copy_descs, self.device, stream)
        else:
            n = copy_descs.numel() // COPY_DESC_DTYPE.itemsize
        if flags is None:
            rc = nat.lib().hsds_copy_batch(self.eng.h, _ptr(src), _ptr(dst), _ptr(copy_descs), n,
                                           _stream_handle(stream))
        else:
            rc = nat.lib().hsds_copy_batch_if(self.eng.h, _ptr(src), _ptr(dst), _ptr(copy_descs), n,
                                              _ptr(flags), _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_copy_batch")
        return copy_descs

    def compare(self, data, chunk, copy_descs, kind, differs, stream=None):
        if isinstance(copy_descs, np.ndarray):
            n = copy_descs.size
            copy_descs = to_device_bytes(copy_descs, self.device, stream)
        else:
            n = copy_descs.numel() // COPY_DESC_DTYPE.itemsize
        rc = nat.lib().hsds_compare_batch(self.eng.h, _ptr(data), _ptr(chunk), _ptr(copy_descs), n, int(kind),
                                          _ptr(differs), _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_compare_batch")
        return copy_descs

    def unshuffle(self, src, dst, itemsize, stream=None):
        rc = nat.lib().hsds_unshuffle_device(self.eng.h, _ptr(src), src.numel(), int(itemsize), _ptr(dst),
                                             _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_unshuffle_device")

    def shuffle(self, src, dst, itemsize, stream=None):
        rc = nat.lib().hsds_shuffle_device(self.eng.h, _ptr(src), src.numel(), int(itemsize), _ptr(dst),
                                           _stream_handle(stream))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_shuffle_device")


COUNT_LIMIT = 1 << 31       # hsds_copy_desc: every count below 2^31


def split_large_copy_descs(recs, limit=COUNT_LIMIT):
    """Records whose counts reach `limit` split along those dimensions into pieces of
    limit // 2 elements (offsets advanced by the piece's stride); other records pass
    through unchanged and in order."""
    recs = np.ascontiguousarray(recs)
    if recs.size == 0 or not (recs["count"] >= limit).any():
        return recs
    out = []
    for r in recs:
        todo = [r.copy()]
        while todo:
            x = todo.pop()
            big = [k for k in range(int(x["rank"])) if x["count"][k] >= limit]
            if not big:
                out.append(x)
                continue
            k = big[0]
            c, piece = int(x["count"][k]), limit // 2
            for start in range(0, c, piece):
                y = x.copy()
                y["count"][k] = min(piece, c - start)
                y["src_off"] = int(x["src_off"]) + start * int(x["src_stride"][k])
                y["dst_off"] = int(x["dst_off"]) + start * int(x["dst_stride"][k])
                todo.append(y)
    return np.array(out, dtype=recs.dtype)


def encode_descs(src_lens, align=256, overhead=16):
    """Descriptors for an encode batch of chunks stored back to back (src) with one
    frame slot of src_len + 16 bytes (c-blosc MAX_OVERHEAD) each in dst.
    Returns (descs CHUNK_DESC_DTYPE ndarray, src_extent, dst_extent)."""
    n = len(src_lens)
    descs = np.zeros(n, CHUNK_DESC_DTYPE)
    if n == 0:
        return descs, 0, 0
    L = np.asarray(src_lens, np.int64)
    sa = (L + align - 1) // align * align
    da = (L + overhead + align - 1) // align * align
    so, do = np.cumsum(sa), np.cumsum(da)
    descs["src_off"] = so - sa
    descs["src_len"] = L
    descs["dst_off"] = do - da
    descs["dst_len"] = L + overhead
    return descs, int(so[-1]), int(do[-1])


def pack_chunks(blobs, dst_lens, align=256):
    """Concatenate stored chunk blobs into one uint8 array and build descriptors.
    Returns (src uint8 ndarray, descs CHUNK_DESC_DTYPE ndarray, dst_extent)."""
    n = len(blobs)
    descs = np.zeros(n, CHUNK_DESC_DTYPE)
    off = 0
    for i, b in enumerate(blobs):
        descs[i]["src_off"] = off
        descs[i]["src_len"] = len(b)
        off += (len(b) + align - 1) // align * align
    src = np.zeros(max(off, 1), np.uint8)
    for i, b in enumerate(blobs):
        o = int(descs[i]["src_off"])
        src[o:o + len(b)] = np.frombuffer(b, np.uint8) if not isinstance(b, np.ndarray) else b
    doff = 0
    for i, L in enumerate(dst_lens):
        descs[i]["dst_off"] = doff
        descs[i]["dst_len"] = L
        doff += (L + align - 1) // align * align
    return src, descs, doff
