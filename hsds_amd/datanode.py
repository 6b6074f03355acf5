"""Data-node read side of the hot path, batched on the GPU (SURVEY.md section 8a rows
a8-a12 and section 8f items 1-2).

Reference flow, one chunk per request:
  get_chunk (hsds/datanode_lib.py:948-1142): chunk cache lookup, in-flight read dedupe,
  get_chunk_bytes (datanode_lib.py:796-945):
    * plain objects: getStorBytes -> _uncompress (storUtil.py:450-522), bytesToArray,
      H5D_CONTIGUOUS_REF reads zero-extended to the chunk size (:833-844);
    * H5D_CHUNKED_REF_INDIRECT "hyper chunks": a chunk made of k HDF5 chunks at byte
      offsets of an HDF5 file; the array is prefilled (fill value or zeros), empty
      ranges are skipped, the locations are coalesced by chunkMunge
      (rangegetUtil.py:111-159) into range reads, and getHyperChunks
      (storUtil.py:525-580) decodes every HDF5 chunk and places it at
      hyper_index * hyper_dims;
  then the array goes into the chunk LruCache (lruCache.py:37-410) if there is room.

Here a whole request's chunks are one batch: every stored object and every HDF5 chunk
of the batch is decoded by ONE hsds_decode_batch call into a contiguous device buffer,
and ONE hsds_copy_batch launch per destination places plain chunks and hyper chunks
into their slots of an HBM-resident cache arena (DeviceChunkCache).  The
storage read itself (POSIX / S3 / Azure drivers) stays outside this engine: callers
pass `fetch(key, offset, length) -> bytes | None` (None = object not found).
"""
import ctypes
import os
import time
from collections import OrderedDict, namedtuple
from operator import attrgetter

import numpy as np

from . import _native as nat
from .codec import BIT_SHUFFLE_BLOCK, HTTPInternalServerError

# HDF5 file chunk location (rangegetUtil.py:9): index = hyper-chunk index tuple,
# offset / length = byte range in the HDF5 file
ChunkLocation = namedtuple("ChunkLocation", ["index", "offset", "length"])

H5D_CONTIGUOUS_REF = "H5D_CONTIGUOUS_REF"


class HTTPNotFound(Exception):
    """Stored object missing (the reference raises aiohttp's HTTPNotFound -> 404)."""


# ---------------------------------------------------------------------------
# rangegetUtil restatement (pure logic, pinned by tests/golden/rangeget_cases.json)
# ---------------------------------------------------------------------------
def getHyperChunkFactors(chunk_dims, hyper_dims):
    """Per-dimension ratio chunk extent / hyper-chunk extent (rangegetUtil.py:24-38);
    ValueError when the ranks differ or an extent does not divide."""
    if len(hyper_dims) != len(chunk_dims):
        raise ValueError("unexpected length for hyper_dims")
    factors = []
    for c, h in zip(chunk_dims, hyper_dims):
        if c % h:
            raise ValueError("unexpected value for hyper_dims")
        factors.append(c // h)
    return factors


def getHyperChunkIndex(i, factors):
    """Index tuple of the i-th hyper chunk, C order over `factors` (rangegetUtil.py:41-52)."""
    idx = []
    for d in range(len(factors)):
        stride = int(np.prod(factors[d + 1:], dtype=np.int64))
        idx.append((i // stride) % factors[d])
    return tuple(idx)


def _span(c):
    if isinstance(c, list):
        return min(e.offset for e in c), max(e.offset + e.length for e in c)
    return c.offset, c.offset + c.length


def chunkMunge(h5chunks, max_gap=1024):
    """Coalesce ChunkLocations into range-read groups (rangegetUtil.py:111-159).

    Sorted by offset; repeatedly the closest adjacent pair (gap = start of the right
    item minus end of the left item, first pair on ties, a zero gap wins at once) whose
    gap is <= max_gap is merged into one list, until no pair qualifies.  Items that
    never merge stay bare ChunkLocations, merged ones become lists in offset order."""
    items = sorted(h5chunks, key=attrgetter("offset"))
    while len(items) > 1:
        best, best_d = None, None
        for i in range(1, len(items)):
            ls, le = _span(items[i - 1])
            rs, re = _span(items[i])
            d = rs - le if ls < rs else ls - re
            if d < 0:
                raise ValueError("unexpected chunk position")
            if d == 0:
                best = i
                break
            if d <= max_gap and (best_d is None or d < best_d):
                best, best_d = i, d
        if best is None:
            break
        left, right = items[best - 1], items[best]
        merged = (list(left) if isinstance(left, list) else [left])
        merged += right if isinstance(right, list) else [right]
        items = items[:best - 1] + [merged] + items[best + 1:]
    return items


# ---------------------------------------------------------------------------
# HBM arena + chunk cache (lruCache.LruCache semantics, device-resident)
# ---------------------------------------------------------------------------
class DeviceArena:
    """One preallocated uint8 HBM tensor carved into 256-byte aligned slots.  Freed
    slots go to an exact-size free list (HSDS datasets have a handful of chunk sizes)
    and are reused first; the bump pointer serves the rest."""

    ALIGN = 256

    def __init__(self, nbytes, device):
        import torch
        self.capacity = int(nbytes)
        self.buf = torch.empty(self.capacity, dtype=torch.uint8, device=device)
        self.top = 0
        self.free_lists = {}
        self.used = 0

    def _round(self, n):
        return max(self.ALIGN, (int(n) + self.ALIGN - 1) // self.ALIGN * self.ALIGN)

    def alloc(self, nbytes):
        n = self._round(nbytes)
        fl = self.free_lists.get(n)
        if fl:
            off = fl.pop()
        elif self.top + n <= self.capacity:
            off = self.top
            self.top += n
        else:
            return None
        self.used += n
        return off

    def free(self, off, nbytes):
        n = self._round(nbytes)
        self.free_lists.setdefault(n, []).append(off)
        self.used -= n

    def view(self, off, nbytes):
        return self.buf[off:off + int(nbytes)]


class _Node:
    __slots__ = ("off", "nbytes", "shape", "dtype", "dirty", "pinned", "last_access")

    def __init__(self, off, nbytes, shape, dtype):
        self.off, self.nbytes, self.shape, self.dtype = off, int(nbytes), tuple(shape), np.dtype(dtype)
        self.dirty = False
        self.pinned = 0          # pin count (read batches / writes in flight): not evictable while > 0
        self.last_access = time.time()


_TORCH_DT = {}


def _torch_dtype(dtype):
    """torch dtype of a numpy dtype (None: no equivalent, e.g. compound types); cached, as
    a read batch asks once per chunk"""
    dt = np.dtype(dtype)
    if dt not in _TORCH_DT:
        import torch
        m = {np.dtype(k): v for k, v in ((np.float32, torch.float32), (np.float64, torch.float64),
                                         (np.float16, torch.float16), (np.int8, torch.int8), (np.uint8, torch.uint8),
                                         (np.int16, torch.int16), (np.int32, torch.int32), (np.int64, torch.int64),
                                         (np.uint16, torch.uint16), (np.uint32, torch.uint32),
                                         (np.uint64, torch.uint64), (np.bool_, torch.bool))}
        _TORCH_DT[dt] = m.get(dt.newbyteorder("=")) if dt.isnative or dt.itemsize == 1 else None
    return _TORCH_DT[dt]


# get_chunks_deferred(views=False): the value of a chunk that is resident in the cache
RESIDENT = object()


def device_view(u8, shape, dtype):
    """Typed torch view of a uint8 device slice (falls back to the uint8 bytes for
    numpy dtypes torch has no equivalent of, e.g. compound types)."""
    td = _torch_dtype(dtype)
    if td is None:
        return u8
    return u8.view(td).reshape(shape)


class DeviceChunkCache:
    """HBM-resident replacement of the DN chunk LruCache (lruCache.py:37-410): the same
    operations and accounting (mem_target, dirty set, memFree = target - dirty bytes,
    cacheUtilizationPercent, dirty nodes never evicted, clearCache refuses dirty
    nodes), but entries are slots of one DeviceArena, so decodes land in place.  The
    reference's default 128 MiB target (config.yml:58) becomes an HBM-sized one.

    Deviation (documented): the reference's __setitem__ on an existing key computes
    its size delta from the already-updated node (always 0, lruCache.py:181-183);
    here the delta is applied."""

    def __init__(self, mem_target, device, name="ChunkCache", expire_time=None, arena_bytes=None):
        self._target = int(mem_target)
        self._name = name
        self._expire = expire_time
        self._lru = OrderedDict()        # key -> _Node, most recent last
        self._mem = 0
        self._dirty = set()
        self._dirty_size = 0
        self.arena = DeviceArena(arena_bytes or int(mem_target * 1.25) + (1 << 20), device)

    # -- LruCache surface --
    def __len__(self):
        return len(self._lru)

    def __iter__(self):
        return iter(reversed(list(self._lru.keys())))    # most recent first, like the LRU list

    def _has(self, key):
        n = self._lru.get(key)
        if n is None:
            return False
        if self._expire and not n.dirty and time.time() - n.last_access > self._expire:
            return False
        return True

    def __contains__(self, key):
        return self._has(key)

    def __getitem__(self, key):
        if not self._has(key):
            raise KeyError(key)
        self._lru.move_to_end(key)
        n = self._lru[key]
        return device_view(self.arena.view(n.off, n.nbytes), n.shape, n.dtype)

    def node_bytes(self, key):
        n = self._lru[key]
        return self.arena.view(n.off, n.nbytes)

    def __delitem__(self, key):
        n = self._lru.pop(key)
        self._mem -= n.nbytes
        if key in self._dirty:
            self._dirty.discard(key)
            self._dirty_size = max(0, self._dirty_size - n.nbytes)
        self.arena.free(n.off, n.nbytes)

    def reserve(self, key, shape, dtype, pin=False):
        """Slot for `key` (existing or new, moved to the front), evicting clean LRU
        nodes until the arena has room; None when nothing more can be evicted.  A
        pinned slot (a read batch in flight) is not evicted until unpin()."""
        nbytes = int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize
        if key in self._lru:
            n = self._lru[key]
            if n.nbytes == nbytes:
                self._lru.move_to_end(key)
                n.shape, n.dtype, n.last_access = tuple(shape), np.dtype(dtype), time.time()
                n.pinned += 1 if pin else 0
                return self.arena.view(n.off, n.nbytes)
            dirty = n.dirty
            del self[key]
        else:
            dirty = False
        off = self.arena.alloc(nbytes)
        while off is None and self._evict_one(exclude=key):
            off = self.arena.alloc(nbytes)
        if off is None:
            return None
        node = _Node(off, nbytes, shape, dtype)
        node.pinned = 1 if pin else 0
        self._lru[key] = node
        self._mem += nbytes
        if dirty:
            self.setDirty(key)
        if self._mem > self._target:
            keep = node.dirty
            node.dirty = True        # never evict the node just added (lruCache.py:215-222)
            self._reduce()
            node.dirty = keep
        return self.arena.view(off, nbytes)

    def __setitem__(self, key, arr):
        """Store a host ndarray or a device tensor (copied into the arena)."""
        import torch
        if isinstance(arr, np.ndarray):
            shape, dtype = arr.shape, arr.dtype
            src = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1))
        else:
            raise TypeError("DeviceChunkCache stores numpy arrays or uses reserve() for device data")
        slot = self.reserve(key, shape, dtype)
        if slot is None:
            raise MemoryError("chunk cache full of dirty chunks")
        slot.copy_(src, non_blocking=False)

    def pin(self, key):
        """Hold `key`'s slot (a counted pin: every pin() / reserve(pin=True) needs its unpin())."""
        self._lru[key].pinned += 1

    def unpin(self, key):
        n = self._lru.get(key)
        if n is not None and n.pinned > 0:
            n.pinned -= 1

    def _evict_one(self, exclude=None):
        for k, n in self._lru.items():          # least recent first
            if not n.dirty and not n.pinned and k != exclude:
                del self[k]
                return True
        return False

    def _reduce(self):
        for k in [k for k, n in self._lru.items() if not n.dirty and not n.pinned]:
            if self._mem <= self._target:
                break
            del self[k]

    def clearCache(self):
        if any(n.dirty for n in self._lru.values()):
            raise ValueError("Unable to clear cache")
        for k in list(self._lru):
            del self[k]

    def setDirty(self, key):
        self._lru.move_to_end(key)
        n = self._lru[key]
        if not n.dirty:
            self._dirty_size += n.nbytes
        n.dirty = True
        self._dirty.add(key)

    def clearDirty(self, key):
        self._lru.move_to_end(key)
        n = self._lru[key]
        if n.dirty:
            self._dirty_size -= n.nbytes
        n.dirty = False
        if key in self._dirty:
            self._dirty.discard(key)
            if self._mem > self._target:
                self._reduce()

    def isDirty(self, key):
        return key in self._dirty

    @property
    def cacheUtilizationPercent(self):
        return int(self._mem / self._target * 100.0)

    @property
    def dirtyCount(self):
        return len(self._dirty)

    @property
    def memUsed(self):
        return self._mem

    @property
    def memFree(self):
        return max(0, self._target - self._dirty_size)

    @property
    def memTarget(self):
        return self._target

    @property
    def memDirty(self):
        return self._dirty_size


# ---------------------------------------------------------------------------
# batched get_chunk_bytes / get_chunk
# ---------------------------------------------------------------------------
class ChunkRead:
    """One chunk of a read batch.  Plain object: offset / length ints (0, 0 = whole
    object).  Hyper chunk (H5D_CHUNKED_REF_INDIRECT): offset and length are lists, one
    entry per hyper chunk in C order (datanode_lib.py:857-906)."""

    def __init__(self, chunk_id, key, offset=0, length=0):
        self.chunk_id, self.key, self.offset, self.length = chunk_id, key, offset, length


def _decode_batch(eng, d_src, descs, dbuf, status, comp, shuffle, isz, blobs):
    """hsds_decode_batch for one batch.  Bitshuffle objects under an outer compressor
    (what _compress(shuffle=2) stores when the dataset also has one, storUtil.py:243-262)
    take two launches on the same stream, as _uncompress does (storUtil.py:189-227):
    the outer Blosc frames into a staging buffer sized by their headers' nbytes, then
    the bitshuffle objects from there into `dbuf`.  A status from the first stage wins.

    Each object is judged alone, as the reference's per-chunk _uncompress is: a blob that
    is not a Blosc frame goes through zlib.decompress semantics when the compressor is
    zlib (codec._uncompress on the engine, storUtil.py:206-217) and otherwise fails that
    chunk only (storUtil.py:218-221); a header whose nbytes exceeds the largest
    bitshuffle object the chunk can have (hsds_bitshuffle_bound at the smallest block)
    fails that chunk instead of sizing the staging buffer."""
    import torch
    if not (shuffle == 2 and comp != nat.COMP_NONE):
        eng.decode(d_src, descs, dbuf, status, compressor=_comp_name(comp), shuffle=shuffle, itemsize=isz)
        return
    from .codec import HTTPInternalServerError as _Err500, _as_bytes, _blosc_nbytes, _uncompress
    from .engine import CHUNK_DESC_DTYPE
    n = len(blobs)
    pre = np.zeros(n, np.int32)                # per-chunk failures found on the host
    inner, host_inner = [0] * n, {}
    for k, b in enumerate(blobs):
        cap = int(nat.lib().hsds_bitshuffle_bound(int(descs[k]["dst_len"]), isz, 8))
        nb = _blosc_nbytes(_as_bytes(b)) if len(b) else None
        if nb is None:
            if comp != nat.COMP_ZLIB:
                pre[k] = nat.ERR_FRAME
                continue
            try:
                raw = _uncompress(bytes(b), "zlib", 0)
            except _Err500:
                pre[k] = nat.ERR_DATA
                continue
            if len(raw) > cap:
                pre[k] = nat.ERR_DATA
                continue
            host_inner[k] = raw
            inner[k] = len(raw)
        elif nb > cap:
            pre[k] = nat.ERR_DATA
        else:
            inner[k] = nb
    ok = np.flatnonzero(pre == 0)
    blosc = np.array([k for k in ok if k not in host_inner], np.int64)
    off, ioff = 0, np.zeros(n, np.int64)
    for k in ok:
        ioff[k] = off
        off += (inner[k] + 255) // 256 * 256
    ibuf = torch.empty(max(off, 1), dtype=torch.uint8, device=dbuf.device)
    st1 = torch.zeros_like(status)
    if blosc.size:
        d1 = np.zeros(blosc.size, CHUNK_DESC_DTYPE)
        for j, k in enumerate(blosc):
            d1[j] = (descs[k]["src_off"], descs[k]["src_len"], ioff[k], inner[k])
        s1 = torch.full((blosc.size,), 99, dtype=status.dtype, device=status.device)
        eng.decode(d_src, d1, ibuf, s1, compressor=_comp_name(comp), shuffle=0, itemsize=1)
        st1[torch.from_numpy(blosc).to(status.device)] = s1
    for k, raw in host_inner.items():
        if raw:
            ibuf[int(ioff[k]):int(ioff[k]) + len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8) \
                .to(ibuf.device, non_blocking=False)
    if ok.size:
        d2 = np.zeros(ok.size, CHUNK_DESC_DTYPE)
        for j, k in enumerate(ok):
            d2[j] = (ioff[k], inner[k], descs[k]["dst_off"], descs[k]["dst_len"])
        s2 = torch.full((ok.size,), 99, dtype=status.dtype, device=status.device)
        eng.decode(ibuf, d2, dbuf, s2, compressor=None, shuffle=2, itemsize=isz)
        status[torch.from_numpy(ok).to(status.device)] = s2
    torch.where(st1 != nat.OK, st1, status, out=status)
    if (pre != 0).any():
        bad = np.flatnonzero(pre != 0)
        status[torch.from_numpy(bad).to(status.device)] = torch.from_numpy(pre[bad]).to(status.device)


def _filter_args(filter_ops, dtype):
    """(compressor code, shuffle, itemsize) for hsds_decode_batch from getFilterOps."""
    if not filter_ops:
        return nat.COMP_NONE, 0, np.dtype(dtype).itemsize
    comp = filter_ops.get("compressor")
    code = nat.COMP_NONE if not comp or comp == "scaleoffset" else \
        nat.COMP_ZLIB if comp in ("gzip", "deflate", "zlib") else nat.COMP_OTHER
    shuffle = int(filter_ops.get("shuffle") or 0)
    dt = filter_ops.get("dtype", dtype)
    return code, shuffle, np.dtype(dt if dt is not None else dtype).itemsize


class ChunkReader:
    """Batched get_chunk / get_chunk_bytes for one dataset (datanode_lib.py:796-1142).

    `fetch(key, offset, length)` is the storage read (storUtil.getStorBytes without
    the codec): bytes, or None when the object does not exist."""

    def __init__(self, fetch, cache=None, device=None, max_gap=1024):
        import torch
        from .engine import ChunkEngine
        self.fetch = fetch
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.eng = ChunkEngine(self.device.index)
        self.cache = cache
        self.max_gap = int(max_gap)
        self.stats = {"decode_calls": 0, "objects": 0, "h5_chunks": 0, "range_reads": 0, "cache_hits": 0}

    # -- host side: gather every stored byte range of the batch --
    def _plan(self, reads, dtype, chunk_dims, hyper_dims):
        itemsize = np.dtype(dtype).itemsize
        chunk_size = int(np.prod(chunk_dims, dtype=np.int64)) * itemsize
        blobs, jobs = [], []          # jobs: (read index, kind, blob index, hyper index or None)
        errors = {}
        for ri, r in enumerate(reads):
            if not isinstance(r.offset, list):
                data = self.fetch(r.key, r.offset, r.length)
                self.stats["range_reads"] += 1
                if data is None:
                    errors[ri] = HTTPNotFound(r.chunk_id)
                    continue
                # the staging copy is the only copy of the object (a view is copied now); an
                # ndarray is taken as its bytes, a flat uint8 view, so len() is its byte count
                data = _as_blob(data)
                if r.length and r.length > 0 and len(data) != r.length:
                    data = bytes(r.length)      # storUtil.py:480-485 (bytearray(length), data not copied)
                blobs.append(data)
                jobs.append((ri, "plain", len(blobs) - 1, None))
                continue
            # hyper chunk (datanode_lib.py:851-906)
            if hyper_dims is None or len(hyper_dims) != len(chunk_dims):
                errors[ri] = ValueError(f"invalid hyper_dims: {hyper_dims}")
                continue
            factors = getHyperChunkFactors(chunk_dims, hyper_dims)
            n = len(r.offset)
            h5_size = int(np.prod(hyper_dims, dtype=np.int64)) * itemsize
            if int(np.prod(factors)) != n or not isinstance(r.length, list) or len(r.length) != n \
                    or n > chunk_size // h5_size:
                errors[ri] = ValueError(f"unexpected number of hyperchunks: {n}")
                continue
            locs = [ChunkLocation(getHyperChunkIndex(i, factors), r.offset[i], r.length[i])
                    for i in range(n) if r.length[i] != 0]
            jobs.append((ri, "hyper_init", None, None))
            for group in chunkMunge(locs, max_gap=self.max_gap):
                group = group if isinstance(group, list) else [group]
                lo = min(c.offset for c in group)
                hi = max(c.offset + c.length for c in group)
                data = self.fetch(r.key, lo, hi - lo)
                self.stats["range_reads"] += 1
                if not data:
                    continue                     # storUtil.py:544-546: no data, leave the prefill
                for c in group:
                    o = c.offset - lo
                    if o + c.length > len(data):     # edge chunk: zero-padded to h5_size (:559-563)
                        piece = bytearray(h5_size)
                        k = len(data) - o
                        piece[:k] = data[o:o + k]
                        piece = bytes(piece)
                    else:
                        piece = bytes(data[o:o + c.length])
                    blobs.append(piece)
                    jobs.append((ri, "h5", len(blobs) - 1, c.index))
        return blobs, jobs, errors, chunk_size

    def get_stor_bytes(self, key, chunk_locations, h5_size, filter_ops=None, offset=None, length=None):
        """getStorBytes with chunk_locations (storUtil.py:450-522): one range read
        [offset, offset + length) (default: the span of the locations), every location
        decoded by one batch call; locations before `offset` and decodes whose size is
        not h5_size are skipped, a codec failure raises HTTPInternalServerError."""
        import torch
        from .engine import pack_chunks
        locs = [c if isinstance(c, ChunkLocation) else ChunkLocation(*c) for c in chunk_locations]
        if offset is None:
            offset = min(c.offset for c in locs)
            length = max(c.offset + c.length for c in locs) - offset
        data = self.fetch(key, offset, length)
        self.stats["range_reads"] += 1
        if data is None or len(data) == 0:
            return data
        if length and length > 0 and len(data) != length:
            data = bytes(length)
        pieces = [data[c.offset - offset:c.offset - offset + c.length] for c in locs if c.offset >= offset]
        if not pieces:
            return []
        comp, shuffle, isz = _filter_args(filter_ops, (filter_ops or {}).get("dtype", np.uint8))
        src, descs, ext = pack_chunks(pieces, [int(h5_size)] * len(pieces))
        dbuf = torch.empty(max(ext, 1), dtype=torch.uint8, device=self.device)
        status = torch.full((len(pieces),), 99, dtype=torch.int32, device=self.device)
        _decode_batch(self.eng, torch.from_numpy(src).to(self.device), descs, dbuf, status, comp, shuffle, isz,
                      pieces)
        self.stats["decode_calls"] += 1
        st = status.cpu().numpy()
        host = dbuf.cpu().numpy()
        out = []
        for k in range(len(pieces)):
            if st[k] == nat.ERR_SIZE:
                continue                       # "expected chunk ... to have size", skipped
            if st[k] != nat.OK:
                raise HTTPInternalServerError()
            o = int(descs[k]["dst_off"])
            out.append(host[o:o + int(h5_size)].tobytes())
        return out

    def read(self, reads, dtype, chunk_dims, filter_ops=None, fill_value=None, layout_class=None,
             hyper_dims=None, defer=False):
        """Decode a batch of chunks.  Returns a list (one entry per read) of device
        arrays (typed torch views of chunk_dims), or an exception instance:
        HTTPNotFound (object missing), HTTPInternalServerError (codec failure or a
        decoded size that is not the chunk size -- get_chunk's 500), ValueError (a
        malformed hyper-chunk request).

        defer=True returns (results, finish) without waiting for the device: the views
        are valid once the current stream has drained, and finish() -- called after
        that -- turns failed decodes into HTTPInternalServerError and returns the final
        list (the batcher gathers the selections before its single synchronisation)."""
        import torch
        from .engine import COPY_DESC_DTYPE, pack_chunks
        dtype = np.dtype(dtype)
        chunk_dims = tuple(int(c) for c in chunk_dims)
        comp, shuffle, isz = _filter_args(filter_ops, dtype)
        blobs, jobs, errors, chunk_size = self._plan(reads, dtype, chunk_dims, hyper_dims)
        h5_size = int(np.prod(hyper_dims, dtype=np.int64)) * dtype.itemsize if hyper_dims is not None else 0
        if layout_class == H5D_CONTIGUOUS_REF and not filter_ops:
            # short contiguous reads near the end of the file are zero-extended (:833-844)
            for ri, kind, bi, _ in jobs:
                if kind == "plain" and len(blobs[bi]) < chunk_size:
                    pad = bytes(chunk_size - len(blobs[bi]))
                    b = blobs[bi]
                    blobs[bi] = np.concatenate([b, np.frombuffer(pad, np.uint8)]) if isinstance(b, np.ndarray) \
                        else b + pad
        results = [None] * len(reads)
        for ri, e in errors.items():
            results[ri] = e
        need = [ri for ri in range(len(reads)) if ri not in errors]
        slots = {}
        pinned = []
        released = [False]

        def unpin_all(drop=False):
            # the batch's slot pins, released exactly once: by finish(), or by abort() when
            # the caller gives up on the batch, or here when the batch fails before returning.
            # A batch given up also drops its reserved slots: their bytes were never decoded
            if not released[0]:
                released[0] = True
                for cid in pinned:
                    self.cache.unpin(cid)
                    if drop and cid in self.cache and not self.cache.isDirty(cid):
                        del self.cache[cid]

        def abort():
            unpin_all(drop=True)

        def reserve_slots():
            # destination slots (base tensor, byte offset): cache arena, else a batch tensor
            if self.cache is not None:
                abase = self.cache.arena.buf
                for ri in need:
                    cid = reads[ri].chunk_id
                    # get_chunk caches when `chunk_id in cache or memFree >= size` (:1094-1103)
                    if cid not in self.cache and self.cache.memFree < chunk_size:
                        continue
                    v = self.cache.reserve(cid, chunk_dims, dtype, pin=True)
                    if v is not None:
                        slots[ri] = (abase, v.data_ptr() - abase.data_ptr())
                        pinned.append(cid)
            rest = [ri for ri in need if ri not in slots]
            if rest:
                tmp = torch.empty(len(rest) * chunk_size, dtype=torch.uint8, device=self.device)
                for k, ri in enumerate(rest):
                    slots[ri] = (tmp, k * chunk_size)
            # prefill hyper chunks with the fill value or zeros (datanode_lib.py:884-888)
            fill_chunk = None
            for ri, kind, _, _ in jobs:
                if kind != "hyper_init":
                    continue
                base, off = slots[ri]
                view = base[off:off + chunk_size]
                if fill_value is None or not np.array(fill_value, dtype=dtype).reshape(1).view(np.uint8).any():
                    view.zero_()
                else:
                    if fill_chunk is None:
                        fill_chunk = torch.from_numpy(np.full(chunk_dims, fill_value, dtype=dtype).view(np.uint8)
                                                      .reshape(-1).copy()).to(self.device)
                    view.copy_(fill_chunk)

        # ONE decode batch into a contiguous buffer (plain objects and HDF5 chunks): the
        # stored objects are packed straight into page-locked staging and go up with one
        # asynchronous copy; statuses come back with one asynchronous copy as well, and
        # every chunk is placed whatever its status (a failed chunk's slot is dropped in
        # finish(), after the one stream synchronisation)
        dec = [j for j in jobs if j[1] in ("plain", "h5")]
        st_host = None
        try:
            st_host = self._launch(reads, dtype, chunk_dims, hyper_dims, comp, shuffle, isz, blobs, jobs, dec,
                                   chunk_size, h5_size, slots, reserve_slots)
        except BaseException:
            abort()
            raise
        for ri in need:
            base, off = slots[ri]
            if results[ri] is None:
                results[ri] = device_view(base[off:off + chunk_size], chunk_dims, dtype)

        def finish():
            """after the stream has drained: decode failures become 500s (and leave the
            cache), the batch's slots are unpinned"""
            try:
                if st_host is not None:
                    st = st_host.numpy()
                    for k, (ri, _, _, _) in enumerate(dec):
                        if st[k] != nat.OK:
                            results[ri] = HTTPInternalServerError()
            finally:
                unpin_all()           # (pinned slots are never evicted: release them whatever happens)
            for ri in need:
                if isinstance(results[ri], HTTPInternalServerError) and self.cache is not None \
                        and reads[ri].chunk_id in self.cache:
                    del self.cache[reads[ri].chunk_id]     # failed reads are not cached
            if self.cache is not None and self.cache.memUsed > self.cache.memTarget:
                self.cache._reduce()
            return results

        finish.abort = abort
        if defer:
            return results, finish
        try:
            torch.cuda.current_stream(self.device).synchronize()
        except BaseException:
            abort()
            raise
        return finish()

    def _launch(self, reads, dtype, chunk_dims, hyper_dims, comp, shuffle, isz, blobs, jobs, dec, chunk_size,
                h5_size, slots, reserve_slots):
        """read()'s device half: the decode batch, the slot reservation and the placement
        copies, queued on the current stream.  Returns the page-locked status buffer (None
        when nothing is decoded)."""
        import torch
        from .engine import COPY_DESC_DTYPE
        st_host = None
        if dec:
            sizes = [chunk_size if kind == "plain" else h5_size for _, kind, _, _ in dec]
            dblobs = [blobs[bi] for _, _, bi, _ in dec]
            d_src, descs, ext = _stage_blobs(dblobs, sizes, self.device)
            dbuf = torch.empty(max(ext, 1), dtype=torch.uint8, device=self.device)
            status = torch.full((len(dec),), 99, dtype=torch.int32, device=self.device)
            _decode_batch(self.eng, d_src, descs, dbuf, status, comp, shuffle, isz, dblobs)
            self.stats["decode_calls"] += 1
            self.stats["objects"] += sum(1 for _, k, _, _ in dec if k == "plain")
            self.stats["h5_chunks"] += sum(1 for _, k, _, _ in dec if k == "h5")
            st_host = torch.empty(len(dec), dtype=torch.int32, pin_memory=True)
            st_host.copy_(status, non_blocking=True)
            reserve_slots()      # while the device copies and decodes
            # placement: ONE copy batch per destination tensor (whole objects: flat records
            # built at once; HDF5 chunks: one strided record each)
            recs = np.zeros(len(dec), COPY_DESC_DTYPE)
            groups = {}
            flat = np.zeros(len(dec), bool)
            for k, (ri, kind, bi, hidx) in enumerate(dec):
                base, off = slots[ri]
                if kind == "plain":
                    flat[k] = True
                    recs["dst_off"][k] = off
                else:
                    recs[k] = _place_desc(int(descs[k]["dst_off"]), off, chunk_dims, hyper_dims, hidx, dtype.itemsize)
                groups.setdefault(id(base), (base, []))[1].append(k)
            if flat.any():
                so = descs["dst_off"][flat].astype(np.uint64)
                do = recs["dst_off"][flat]
                a = so | do | np.uint64(chunk_size)
                w = np.where(a % 8 == 0, 8, np.where(a % 4 == 0, 4, 1)).astype(np.int64)
                recs["src_off"][flat] = so
                recs["src_stride"][flat, 0] = w
                recs["dst_stride"][flat, 0] = w
                recs["count"][flat, 0] = chunk_size // w
                recs["rank"][flat] = 1
                recs["itemsize"][flat] = w
            for base, rows in groups.values():
                self.eng.copy(dbuf, base, recs[np.asarray(rows)])
        else:
            reserve_slots()
        return st_host


def _as_blob(data):
    """a fetched object as bytes, or an ndarray as a flat uint8 view of its bytes"""
    if isinstance(data, bytes):
        return data
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).reshape(-1).view(np.uint8)
    return bytes(data)


# host threads copying a large batch into page-locked staging (the GPU box's CPU share is
# 16 cores; the DN's event loop and the batch worker keep theirs)
_STAGE_THREADS = int(os.environ.get("HSDS_STAGE_THREADS", "8"))


def _stage_blobs(blobs, dst_lens, device, align=256):
    """pack_chunks into page-locked memory and one asynchronous host-to-device copy:
    (device uint8 tensor, CHUNK_DESC_DTYPE descriptors, decoded extent).  The staging
    block returns to torch's pinned-memory cache once the copy has run."""
    import torch
    from .engine import CHUNK_DESC_DTYPE
    n = len(blobs)
    lens = np.fromiter((len(b) for b in blobs), np.int64, n)
    descs = np.zeros(n, CHUNK_DESC_DTYPE)
    pad = (lens + align - 1) // align * align
    src_off = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(pad[:-1], out=src_off[1:])
    descs["src_off"] = src_off
    descs["src_len"] = lens
    dl = np.asarray(dst_lens, np.int64)
    dpad = (dl + align - 1) // align * align
    dst_off = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(dpad[:-1], out=dst_off[1:])
    descs["dst_off"] = dst_off
    descs["dst_len"] = dl
    total = int(pad.sum()) if n else 0
    host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
    d_src = torch.empty(max(total, 1), dtype=torch.uint8, device=device)
    if total:
        # hsds_stage_upload: the copies into staging run on native threads (no GIL), in
        # pieces that go up as soon as they are staged, so the link works while the later
        # pieces are still being copied
        keep, ptrs = [], np.empty(n, np.uint64)
        for k, b in enumerate(blobs):
            if isinstance(b, np.ndarray):
                b = np.ascontiguousarray(b).reshape(-1).view(np.uint8)
                keep.append(b)
                ptrs[k] = b.__array_interface__["data"][0]
            else:
                ptrs[k] = ctypes.cast(b, ctypes.c_void_p).value or 0
        lens_u = lens.astype(np.uint64)
        offs_u = src_off.astype(np.uint64)
        threads = _STAGE_THREADS if total >= (8 << 20) else 1
        rc = nat.lib().hsds_stage_upload(nat.engine(d_src.device.index).h, ptrs.ctypes.data, lens_u.ctypes.data,
                                         offs_u.ctypes.data, n, host.data_ptr(), d_src.data_ptr(), total, threads,
                                         torch.cuda.current_stream(d_src.device).cuda_stream)
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_stage_upload")
        # one byte through torch's copy on the same stream, after the staged copies: the
        # pinned-memory cache records its event and keeps `host` reserved until they ran
        d_src[:1].copy_(host[:1], non_blocking=True)
    return d_src, descs, int(dpad.sum()) if n else 0


def _comp_name(code):
    return {nat.COMP_NONE: None, nat.COMP_ZLIB: "zlib"}.get(code, "other")


def _copy_rec():
    return np.zeros((), dtype=[("src_off", "<u8"), ("dst_off", "<u8"), ("src_stride", "<i8", (8,)),
                               ("dst_stride", "<i8", (8,)), ("count", "<i8", (8,)), ("rank", "<i4"),
                               ("itemsize", "<i4")])


def _flat_desc(src_off, dst_off, nbytes):
    """1-d copy of nbytes (8-byte elements when the sizes and offsets allow)."""
    d = _copy_rec()
    w = 8 if not (nbytes | src_off | dst_off) & 7 else 4 if not (nbytes | src_off | dst_off) & 3 else 1
    d["src_off"], d["dst_off"] = src_off, dst_off
    d["src_stride"][0] = d["dst_stride"][0] = w
    d["count"][0] = nbytes // w
    d["rank"], d["itemsize"] = 1, w
    return d


def _place_desc(src_off, dst_off, chunk_dims, hyper_dims, hidx, itemsize):
    """copy for `chunk_arr[hidx*hyper : (hidx+1)*hyper] = hyper_chunk` (storUtil.py:568-580)."""
    rank = len(chunk_dims)
    d = _copy_rec()
    cstr = [itemsize] * rank
    hstr = [itemsize] * rank
    for k in range(rank - 2, -1, -1):
        cstr[k] = cstr[k + 1] * chunk_dims[k + 1]
        hstr[k] = hstr[k + 1] * hyper_dims[k + 1]
    d["src_off"] = src_off
    d["dst_off"] = dst_off + sum(int(hidx[k]) * hyper_dims[k] * cstr[k] for k in range(rank))
    d["src_stride"][:rank] = hstr
    d["dst_stride"][:rank] = cstr
    d["count"][:rank] = hyper_dims
    d["rank"] = rank
    d["itemsize"] = itemsize
    return d


def _locked(fn):
    """run a ChunkStore method under the store's lock"""
    import functools

    @functools.wraps(fn)
    def wrap(self, *a, **kw):
        with self.lock:
            return fn(self, *a, **kw)
    return wrap


class ChunkStore:
    """get_chunk for many chunks at once (datanode_lib.py:948-1142).  The returned
    device arrays are views of HBM cache slots: valid until the next call that may
    evict them (the DN uses a chunk right after get_chunk).  Cache hits are
    served from HBM, the misses are read as one batch by ChunkReader and cached when
    there is room (`chunk_id in cache or memFree >= nbytes`), duplicates in a batch
    are read once (the reference's pending_s3_read dedupe), and a missing object
    with chunk_init yields a fill-value (or zero) chunk of the full layout dims."""

    def __init__(self, fetch, mem_target=1 << 30, device=None, max_gap=1024):
        import threading
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.cache = DeviceChunkCache(mem_target, dev)
        self.reader = ChunkReader(fetch, cache=self.cache, device=dev, max_gap=max_gap)
        # every public call holds this lock: the DN event loop and the batcher's worker
        # thread share one store (the cache's LRU, arena and pins are not thread-safe)
        self.lock = threading.RLock()

    def get_chunks(self, reads, dtype, chunk_dims, filter_ops=None, fill_value=None, layout_class=None,
                   hyper_dims=None, chunk_init=False):
        with self.lock:
            vals, finish = self.get_chunks_deferred(reads, dtype, chunk_dims, filter_ops=filter_ops,
                                                    fill_value=fill_value, layout_class=layout_class,
                                                    hyper_dims=hyper_dims, chunk_init=chunk_init)
            import torch
            try:
                torch.cuda.current_stream(self.cache.arena.buf.device).synchronize()
            except BaseException:
                finish.abort()
                raise
            return finish()

    def get_chunks_deferred(self, reads, dtype, chunk_dims, filter_ops=None, fill_value=None, layout_class=None,
                            hyper_dims=None, chunk_init=False, views=True):
        """get_chunks without waiting for the device: (values, finish).  The values are
        device views (None for a 404, an exception for a malformed request) whose bytes
        are ready once the current stream has drained; finish(), called after that,
        returns the final list with decode failures as HTTPInternalServerError.  Call it
        under self.lock and keep the lock until the views are consumed (the batcher
        gathers its selections in between).  Cache hits stay pinned until finish(), so
        the misses' slot reservations cannot evict them.  views=False: a cache hit's value
        is RESIDENT instead of a device view (a caller that addresses the slots itself, as
        the write paths do, skips building thousands of tensor views on the host)."""
        out = {}
        todo, seen, hits = [], set(), []
        for r in reads:
            if r.chunk_id in self.cache:
                if r.chunk_id not in out:
                    out[r.chunk_id] = self.cache[r.chunk_id] if views else RESIDENT
                    self.cache.pin(r.chunk_id)
                    hits.append(r.chunk_id)
                self.reader.stats["cache_hits"] += 1
            elif r.chunk_id not in seen:
                seen.add(r.chunk_id)
                todo.append(r)
        rfin, init, init_pinned = None, [], False
        try:
            if todo:
                res, rfin = self.reader.read(todo, dtype, chunk_dims, filter_ops=filter_ops, fill_value=fill_value,
                                             layout_class=layout_class, hyper_dims=hyper_dims, defer=True)
                init = [r.chunk_id for r, v in zip(todo, res) if isinstance(v, HTTPNotFound) and chunk_init]
                if init:
                    self._fill_new(init, dtype, chunk_dims, fill_value)   # (unpins its own keys when it fails)
                    init_pinned = True
                for r, v in zip(todo, res):
                    if isinstance(v, HTTPNotFound) and chunk_init:
                        v = self.cache[r.chunk_id]
                    elif isinstance(v, HTTPNotFound):
                        v = None                               # 404: no chunk
                    out[r.chunk_id] = v
        except BaseException:
            if rfin is not None:
                rfin.abort()
            for key in (init if init_pinned else []) + hits:
                self.cache.unpin(key)
            raise
        released = [False]

        def release():
            # every pin of this call, released exactly once (finish() or abort())
            if not released[0]:
                released[0] = True
                for key in init:
                    self.cache.unpin(key)
                for key in hits:
                    self.cache.unpin(key)

        def finish():
            try:
                if rfin is not None:
                    res = rfin()
                    for r, v in zip(todo, res):
                        if isinstance(v, HTTPInternalServerError):
                            out[r.chunk_id] = v
            finally:
                release()
            return [out[r.chunk_id] for r in reads]

        def abort():
            """give up on the batch (the caller failed before finish()): drop its pins"""
            if rfin is not None:
                rfin.abort()
            release()

        finish.abort = abort
        finish.reads_pending = rfin is not None      # stored objects being decoded (statuses to check)
        return [out[r.chunk_id] for r in reads], finish

    def _resident(self, reads, dtype, chunk_dims, filter_ops, fill_value):
        """PUT_Chunk's read (get_chunk with chunk_init, chunk_dn.py:174-190): every target
        chunk resident in the cache -- a stored object decoded, else the fill value.  A read's
        own error (get_chunk's 500) is raised.  The write paths address the slots by their
        offsets, so cache hits build no device views (views=False)."""
        import torch
        vals, finish = self.get_chunks_deferred(reads, dtype, chunk_dims, filter_ops=filter_ops,
                                                fill_value=fill_value, chunk_init=True, views=False)
        # only decoded objects have statuses to wait for: cache hits and fill-value slots are
        # stream-ordered before the write's copies, so the host goes on without waiting for
        # the kernels queued before (the previous request's encode)
        try:
            if finish.reads_pending:
                torch.cuda.current_stream(self.cache.arena.buf.device).synchronize()
        except BaseException:
            finish.abort()
            raise
        for v in finish():
            if isinstance(v, Exception):
                raise v

    def _fill_new(self, keys, dtype, chunk_dims, fill_value):
        """get_chunk's chunk_init for missing objects (datanode_lib.py:1132-1138): a cache
        slot per key holding the fill value (or zeros) over the full layout dims -- ONE
        broadcast copy launch from a one-element device buffer, not one upload per chunk."""
        import torch
        from .engine import COPY_DESC_DTYPE
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(chunk_dims, dtype=np.int64)) * dtype.itemsize
        one = np.zeros(1, dtype)
        if fill_value is not None:
            one[...] = fill_value
        pat = one.view(np.uint8)
        # widest pattern that tiles the chunk: 16 bytes when the element size divides it
        unit = 16 if (16 % dtype.itemsize == 0 and nbytes % 16 == 0) else dtype.itemsize
        pat = np.tile(pat, unit // dtype.itemsize) if unit != dtype.itemsize else pat
        abase = self.cache.arena.buf
        d_pat = torch.from_numpy(np.ascontiguousarray(pat).copy()).to(abase.device)
        recs = np.zeros(len(keys), COPY_DESC_DTYPE)
        for k, key in enumerate(keys):
            # pinned: a later reserve of this batch must not evict an earlier fill slot
            # (get_chunks unpins them once it has read them back)
            slot = self.cache.reserve(key, chunk_dims, dtype, pin=True)
            if slot is None:
                for kk in keys[:k]:
                    self.cache.unpin(kk)
                raise MemoryError("chunk cache full of dirty chunks")
            recs[k]["dst_off"] = slot.data_ptr() - abase.data_ptr()
        recs["src_off"] = 0
        recs["dst_stride"][:, 0] = unit
        recs["count"][:, 0] = nbytes // unit
        recs["rank"] = 1
        recs["itemsize"] = unit
        self.reader.eng.copy(d_pat, abase, recs)

    # ---- write side (PUT_Chunk -> save_chunk -> s3sync / write_s3_obj) ------------
    @_locked
    def put_selections(self, writes, dtype, chunk_dims, filter_ops=None, fill_value=None, write_zero_chunks=False):
        """PUT_Chunk for many chunks at once (chunk_dn.py:55-314).  `writes` is a list
        of (ChunkRead, slices, data) with data a host ndarray of the selection shape
        (a compound field subset, PUT_Chunk's `fields`, updates those fields only).
        Every target chunk is fetched (get_chunk with chunk_init: missing chunks start
        from the fill value), then ONE compare launch (chunkWriteSelection's
        ndarray_compare, chunkUtil.py:983) and ONE conditional copy launch update the
        chunks in HBM; changed chunks (or all with write_zero_chunks,
        chunk_dn.py:306) are marked dirty for the next flush (save_chunk,
        datanode_lib.py:1145-1183).  Returns one is_dirty flag per write."""
        import torch
        from .selection import _write_data, apply_writes, write_selection_descs
        dtype = np.dtype(dtype)
        chunk_dims = tuple(int(c) for c in chunk_dims)
        # requests are applied in order: writes to the same chunk go to later rounds
        seen, first, later = set(), [], []
        for i, w in enumerate(writes):
            (later if w[0].chunk_id in seen else first).append(i)
            seen.add(w[0].chunk_id)
        if later:
            res = dict(zip(first, self.put_selections([writes[i] for i in first], dtype, chunk_dims, filter_ops,
                                                      fill_value, write_zero_chunks)))
            res.update(zip(later, self.put_selections([writes[i] for i in later], dtype, chunk_dims, filter_ops,
                                                      fill_value, write_zero_chunks)))
            return [res[i] for i in range(len(writes))]
        reads = [w[0] for w in writes]
        self._resident(reads, dtype, chunk_dims, filter_ops, fill_value)
        # pin the target slots while the update runs
        for r in reads:
            n = self.cache._lru.get(r.chunk_id)
            if n is None:
                raise MemoryError("chunk cache cannot hold the write batch")
            n.pinned += 1
        try:
            abase = self.cache.arena.buf
            data_parts, items, offs = [], [], 0
            for wi, (r, slices, data) in enumerate(writes):
                data = _write_data(dtype, data)      # a field subset: PUT_Chunk `fields` (chunk_dn.py:112-140)
                slot = self.cache.node_bytes(r.chunk_id)
                slot_off = slot.data_ptr() - abase.data_ptr()
                items.append((wi, write_selection_descs(chunk_dims, dtype, tuple(slices), data.shape, data.dtype,
                                                        data_base=offs, chunk_base=slot_off)))
                data_parts.append(data.view(np.uint8).reshape(-1))
                offs += (data.nbytes + 255) // 256 * 256
            host = np.zeros(max(offs, 1), np.uint8)
            o = 0
            for part in data_parts:
                host[o:o + part.size] = part
                o += (part.size + 255) // 256 * 256
            d_data = torch.from_numpy(host).to(abase.device)
            differs = apply_writes(self.reader.eng, d_data, abase, items, len(writes))
            dirty = differs[:len(writes)].cpu().numpy().astype(bool)
        finally:
            for r in reads:
                self.cache.unpin(r.chunk_id)
        out = []
        for (r, _, _), d in zip(writes, dirty):
            if d or write_zero_chunks:
                self.cache.setDirty(r.chunk_id)
            out.append(bool(d))
        return out

    @_locked
    def put_pieces(self, reads, d_data, make_descs, dtype, chunk_dims, filter_ops=None, fill_value=None,
                   write_zero_chunks=False):
        """PUT_Chunk for many chunks with the request data already in HBM (the sharded
        write path, crawl.ShardedWriter).  `reads` are the target chunks (distinct ids),
        `make_descs(slot_offsets)` returns the copy records d_data -> cache arena for
        those slots (SelectionPlan.apply_descs).  The chunks are read with chunk_init
        (RMW of an existing object, else the fill value: chunk_dn.py:174-190), then ONE
        compare launch (chunkWriteSelection's no-change test, chunkUtil.py:983) and ONE
        conditional copy launch update them; changed chunks (all with write_zero_chunks,
        chunk_dn.py:306) are marked dirty (save_chunk).  Returns the dirty flag per read."""
        import torch
        from .selection import _kind
        dtype = np.dtype(dtype)
        if dtype.names or dtype.subdtype is not None:
            # the whole-element compare below has one kind per dtype; compound / subarray
            # elements compare leaf by leaf (NaN fields, -0.0) in put_selections
            # (write_selection_descs), which the sharded path does not build
            raise NotImplementedError("put_pieces (the sharded write path) takes scalar dtypes; "
                                      "compound datasets go through put_selections")
        chunk_dims = tuple(int(c) for c in chunk_dims)
        if len({r.chunk_id for r in reads}) != len(reads):
            raise ValueError("put_pieces takes each chunk once")
        # chunk_init reads without a wait: the stored objects' decodes, the compare and the
        # copy are stream-ordered, and the one wait of the batch (the dirty flags below)
        # covers the decode statuses too -- the host builds the write while the device still
        # runs what was queued before (the previous request's encode)
        _, rfin = self.get_chunks_deferred(reads, dtype, chunk_dims, filter_ops=filter_ops, fill_value=fill_value,
                                           chunk_init=True, views=False)
        pinned = []
        try:
            for r in reads:
                n = self.cache._lru.get(r.chunk_id)
                if n is None:
                    raise MemoryError("chunk cache cannot hold the write batch")
                n.pinned += 1
                pinned.append(r.chunk_id)
            abase = self.cache.arena.buf
            offs = [self.cache._lru[r.chunk_id].off for r in reads]
            dd = make_descs(offs)
            differs = torch.zeros(max(len(reads), 1), dtype=torch.int32, device=abase.device)
            if len(dd):
                d_desc = self.reader.eng.compare(d_data, abase, dd, _kind(dtype), differs)
                self.reader.eng.copy(d_data, abase, d_desc, flags=differs)
            dirty = differs[:len(reads)].cpu().numpy().astype(bool)
        except BaseException:
            for key in pinned:
                self.cache.unpin(key)
            rfin.abort()
            raise
        for key in pinned:
            self.cache.unpin(key)
        # each chunk's PUT stands alone (one PUT_Chunk per chunk in the reference): a chunk
        # whose stored object failed to decode leaves the cache (finish) and its 500 is
        # raised after the other chunks' updates are marked
        vals = rfin()
        err = None
        out = []
        for r, d, v in zip(reads, dirty, vals):
            if isinstance(v, Exception):
                err = err or v
                out.append(False)
                continue
            if d or write_zero_chunks:
                self.cache.setDirty(r.chunk_id)
            out.append(bool(d))
        if err is not None:
            raise err
        return out

    @_locked
    def encode_dirty(self, filter_ops, stream=None):
        """The device half of flush for a dataset with a Blosc compressor (no bitshuffle):
        ONE asynchronous hsds_encode_batch_codec of every dirty chunk straight from its cache
        slot.  Returns (ids, frames, descs, sizes, status) -- device tensors, nothing copied
        to the host, chunks still dirty (flush() finishes the s3sync)."""
        import torch
        from .engine import encode_descs
        comp = (filter_ops or {}).get("compressor")
        if not comp or comp == "scaleoffset" or (filter_ops or {}).get("shuffle") == 2:
            raise ValueError("encode_dirty covers Blosc-compressed datasets without bitshuffle")
        if nat.cname_code(comp) is None:
            raise NotImplementedError(f"Blosc codec {comp!r} has no encoder in the hsds_amd engine")
        ids = [k for k in list(self.cache._lru) if self.cache.isDirty(k)]
        abase = self.cache.arena.buf
        nodes = [self.cache._lru[k] for k in ids]
        descs, _, dext = encode_descs([n.nbytes for n in nodes])
        if len(ids):
            descs["src_off"] = [n.off for n in nodes]
        level = filter_ops.get("level", 5)
        level = 5 if level is None else int(level)
        frames = torch.empty(max(dext, 1), dtype=torch.uint8, device=abase.device)
        sizes = torch.zeros(max(len(ids), 1), dtype=torch.int64, device=abase.device)
        status = torch.full((max(len(ids), 1),), 99, dtype=torch.int32, device=abase.device)
        if ids:
            self.reader.eng.encode(abase, descs, frames, sizes, status, clevel=level,
                                   shuffle=int(filter_ops.get("shuffle") or 0), typesize=1, compressor=comp,
                                   stream=stream)
        return ids, frames, descs, sizes, status

    @_locked
    def flush(self, put, filter_ops=None, keys=None):
        """s3sync for every dirty chunk (datanode_lib.py:1186-1318, 126-311): ONE
        hsds_encode_batch_codec straight from the HBM cache slots (storUtil._compress's
        Blosc frames with the dataset's codec (zlib, lz4, lz4hc), level and shuffle flag; no compressor
        -> the raw bytes, putStorBytes semantics; a bitshuffle dataset first goes through ONE
        hsds_encode_bitshuffle_batch, storUtil.py:243-251), one device-to-host copy of the
        frames, `put(key, bytes)` per chunk, then clearDirty.  `keys` maps chunk id ->
        storage key (default: hsds_amd.partition.getS3Key).  Returns the flushed ids."""
        import torch
        from .engine import encode_descs
        from .partition import getS3Key
        ids = [k for k in list(self.cache._lru) if self.cache.isDirty(k)]
        if not ids:
            return []
        abase = self.cache.arena.buf
        nodes = [self.cache._lru[k] for k in ids]
        comp = (filter_ops or {}).get("compressor")
        if comp == "scaleoffset":
            comp = None
        if comp and nat.cname_code(comp) is None:
            raise NotImplementedError(f"Blosc codec {comp!r} has no encoder in the hsds_amd engine")
        bitshuffle = (filter_ops or {}).get("shuffle") == 2
        src, src_nodes_off = abase, [n.off for n in nodes]
        src_lens = [n.nbytes for n in nodes]
        if bitshuffle:
            # _compress(shuffle=2): bitshuffle+LZ4 objects first (storUtil.py:243-251), in
            # ONE hsds_encode_bitshuffle_batch from the cache slots; Blosc (shuffle off)
            # wraps them when the dataset also has a compressor
            dt = np.dtype(filter_ops.get("dtype") or np.uint8)
            bounds = [int(nat.lib().hsds_bitshuffle_bound(L, dt.itemsize, BIT_SHUFFLE_BLOCK)) for L in src_lens]
            bdescs, _, bext = encode_descs(src_lens, overhead=0)
            for d, n, b in zip(bdescs, nodes, bounds):
                d["src_off"] = n.off
                d["dst_len"] = b
            bdescs["dst_off"] = np.concatenate([[0], np.cumsum([(b + 255) // 256 * 256 for b in bounds])[:-1]])
            bext = int(sum((b + 255) // 256 * 256 for b in bounds))
            bframes = torch.empty(max(bext, 1), dtype=torch.uint8, device=abase.device)
            bsizes = torch.zeros(len(ids), dtype=torch.int64, device=abase.device)
            bstatus = torch.full((len(ids),), 99, dtype=torch.int32, device=abase.device)
            self.reader.eng.encode_bitshuffle(abase, bdescs, bframes, bsizes, bstatus, itemsize=dt.itemsize,
                                              block=BIT_SHUFFLE_BLOCK)
            if (bstatus.cpu().numpy() != 0).any():
                raise HTTPInternalServerError()
            src, src_nodes_off = bframes, [int(d["dst_off"]) for d in bdescs]
            src_lens = [int(x) for x in bsizes.cpu().numpy()]
            if not comp:
                host = bframes.cpu().numpy()
                blobs = [host[o:o + L].tobytes() for o, L in zip(src_nodes_off, src_lens)]
        if comp:
            level = filter_ops.get("level", 5)
            level = 5 if level is None else int(level)
            descs, _, dext = encode_descs(src_lens)
            for d, o in zip(descs, src_nodes_off):
                d["src_off"] = o
            frames = torch.empty(max(dext, 1), dtype=torch.uint8, device=abase.device)
            sizes = torch.zeros(len(ids), dtype=torch.int64, device=abase.device)
            status = torch.full((len(ids),), 99, dtype=torch.int32, device=abase.device)
            self.reader.eng.encode(src, descs, frames, sizes, status, clevel=level,
                                   shuffle=0 if bitshuffle else int(filter_ops.get("shuffle") or 0), typesize=1,
                                   compressor=comp)
            st = status.cpu().numpy()
            if (st != 0).any():
                raise HTTPInternalServerError()
            host = frames.cpu().numpy()
            sz = sizes.cpu().numpy()
            blobs = [host[int(d["dst_off"]):int(d["dst_off"]) + int(s)].tobytes() for d, s in zip(descs, sz)]
        elif not bitshuffle:
            blobs = [self.cache.node_bytes(k).cpu().numpy().tobytes() for k in ids]
        for k, b in zip(ids, blobs):
            put(keys[k] if keys else getS3Key(k), b)
            self.cache.clearDirty(k)
        return ids
