"""Chunk-sharded hyperslab read and write across the GPUs of one node (SURVEY.md section 8e,
cfg3 / cfg4 reads, cfg5 writes).

Reference flow (one HTTP request per chunk): the SN crawler fans a selection out to the
data nodes by `getObjPartition(chunk_id, dn_count)` (hsds/chunk_crawl.py:362-418,
hsds/util/idUtil.py:481-486); each DN decodes the chunk (datanode_lib.get_chunk ->
storUtil._uncompress) and returns `chunkReadSelection(chunk_arr, chunk_sel)`
(chunkUtil.py:882, chunk_dn.py:552); the SN places it with
`np_arr[data_sel] = chunk_arr` (chunk_crawl.py:418) into a slab prefilled with the
fill value (dset_lib.py:590-597).

Here one process per GPU plays the DN role for the chunks the same md5 rule assigns to
it.  Every rank computes the identical `SelectionPlan` from (dataset, layout,
selection, world), so no metadata is exchanged: each rank
  1. decodes its chunks in one batch (ChunkEngine.decode),
  2. gathers each chunk's selected sub-block into a packed per-rank buffer
     (one hsds_copy_batch launch; pieces in getChunkIds order),
  3. sends the packed buffer to the root (one point-to-point message per rank: RCCL
     over xGMI on GPUs, gloo on CPU -- the only data-path collective),
and the root scatters every piece into the slab with one more hsds_copy_batch launch.
Missing chunks (no stored object) are decoded as fill-value chunks, which leaves the
slab exactly as the reference leaves it (prefilled, chunk_crawl.py:362-366).

The write is the mirror (PUT_Value -> _doHyperslabWrite -> write_chunk_hyperslab ->
PUT_Chunk -> save_chunk -> s3sync, chunk_sn.py:555-646, chunk_crawl.py:75-150,
chunk_dn.py:41-314, datanode_lib.py:1186-1318): the root gathers every chunk's piece of
the request array, arr[data_sel], into per-owner packed buffers (one copy launch), sends
each owner its buffer (one point-to-point message per rank), and every rank applies its
pieces to its chunks through its HBM chunk store (read-modify-write with chunk_init,
compare, conditional copy, dirty marking) and encodes its dirty chunks locally on flush.
"""
from dataclasses import dataclass

import ctypes

import numpy as np

from . import _native as nat
from . import selection as sel
from .partition import getObjPartition


@dataclass
class Piece:
    chunk_id: str
    owner: int
    chunk_slices: tuple       # chunk-relative selection (getChunkCoverage)
    data_slices: tuple        # slab-relative placement (getDataCoverage)
    shape: tuple              # getSelectionShape(chunk selection)
    nbytes: int
    off: int = 0              # byte offset inside the owner's packed buffer


def _align(n, a):
    return (n + a - 1) // a * a


def _dim_pieces(s, c):
    """One dimension of a hyperslab over chunks of extent c, vectorized: arrays of chunk
    index, chunk-relative start, count and slab start for every chunk the slice touches, in
    getChunkIds order (chunkUtil.py:459-582), with getChunkSelection's start snapped onto
    the step lattice and getChunkCoverage / getDataCoverage's slices (chunkUtil.py:608-790)."""
    start, stop, step = int(s.start), int(s.stop), int(s.step or 1)
    if stop <= start:
        z = np.zeros(0, np.int64)
        return z, z, z, z
    if step > c:
        pts = np.arange(start, stop, step, dtype=np.int64)
        idx = pts // c
        return idx, pts - idx * c, np.ones_like(idx), (pts - start) // step
    last = sel.slice_stop(slice(start, stop, step))
    idx = np.arange(start // c, -(-last // c), dtype=np.int64)
    lo = idx * c
    first = np.where(start >= lo, start, start + (-(-(lo - start) // step)) * step)
    end = np.minimum(stop, lo + c)
    count = np.where(end > first, -(-(end - first) // step), 0)
    return idx, first - lo, count, (first - start) // step


def _c_strides(shape, itemsize):
    st = [itemsize] * len(shape)
    for d in range(len(shape) - 2, -1, -1):
        st[d] = st[d + 1] * int(shape[d + 1])
    return np.array(st, np.int64)


class SelectionPlan:
    """Per-chunk plan of a hyperslab selection sharded over `world` ranks, computed with
    numpy over the per-dimension chunk grids (O(#chunks) array work, no Python loop per
    chunk) and the batched md5 partition of the C ABI (hsds_partition_ids).

    Read side (SN read, chunk_crawl.py:395-418): decoded chunk -> packed piece
    (pack_descs) -> slab (place_descs).  Write side (SN write, chunk_crawl.py:118-135, and
    PUT_Chunk, chunk_dn.py:284-302): slab -> packed piece (gather_descs) -> chunk
    (apply_descs).  `selection` is a tuple of slices (getSelectionList output).  Point
    (coordinate) selections are not hyperslabs and are outside the distributed path."""

    ALIGN = 16

    def __init__(self, dset_id, dims, layout, selection, dtype, world, partition=None):
        self.dims = tuple(int(d) for d in dims)
        self.layout = tuple(int(c) for c in layout)
        self.selection = tuple(selection)
        if any(not isinstance(s, slice) for s in self.selection):
            raise NotImplementedError("coordinate selections are outside the distributed hyperslab path")
        if len(self.selection) != len(self.dims) or len(self.layout) != len(self.dims):
            raise ValueError("selection / layout rank does not match dataset rank")
        self.dset_id = dset_id
        self.dtype = np.dtype(dtype)
        self.itemsize = self.dtype.itemsize
        self.world = int(world)
        self.rank = len(self.dims)
        self.slab_shape = tuple(sel.getSelectionShape(self.selection))
        self.slab_nbytes = int(np.prod(self.slab_shape, dtype=np.int64)) * self.itemsize
        self.chunk_nbytes = int(np.prod(self.layout, dtype=np.int64)) * self.itemsize
        self.steps = np.array([int(s.step or 1) for s in self.selection], np.int64)
        if not dset_id.startswith("d-"):
            raise ValueError(f"Bad Request: invalid dset id: {dset_id}")
        self.prefix = "c-" + dset_id[2:] + "_"
        # per-dimension tables; a chunk that a slice touches without selecting anything
        # (count 0) is dropped per dimension, so the pieces are exactly the C-order product
        # of the tables (the device record builder, hsds_plan_descs, unravels that grid)
        per_dim = []
        for s_, c in zip(self.selection, self.layout):
            t = _dim_pieces(s_, c)
            k = t[2] > 0
            per_dim.append(t if k.all() else tuple(a[k] for a in t))
        self._tabs = per_dim
        R = self.rank
        n = int(np.prod([len(t[0]) for t in per_dim], dtype=np.int64)) if R else 0
        cols = [np.empty((n, R), np.int64) for _ in range(4)]
        rep = n
        for d, t in enumerate(per_dim):
            nk = len(t[0])
            rep //= max(nk, 1)
            tile = n // max(nk * rep, 1)
            for k in range(4):
                cols[k][:, d] = np.tile(np.repeat(t[k], rep), tile) if n else 0
        self.idx, self.cstart, self.count, self.dstart = cols
        self.nbytes = np.prod(self.count, axis=1) * self.itemsize if n else np.zeros(0, np.int64)
        if partition is not None:
            self.owner = np.array([partition(self._cid(i)) for i in range(n)], np.int32)
        elif self.world == 1:
            self.owner = np.zeros(n, np.int32)
        else:
            self.owner = partition_ids(self.prefix, self.idx, self.world)
        self.by_rank = [np.nonzero(self.owner == r)[0] for r in range(self.world)]
        sizes = (self.nbytes + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.off = np.zeros(n, np.int64)
        self.rank_bytes = []
        for r in range(self.world):
            ir = self.by_rank[r]
            if len(ir):
                cs = np.cumsum(sizes[ir])
                self.off[ir] = cs - sizes[ir]
                self.rank_bytes.append(int(cs[-1]))
            else:
                self.rank_bytes.append(0)
        self.rank_base = np.concatenate([[0], np.cumsum(self.rank_bytes)]).astype(np.int64)
        self.gathered_nbytes = int(self.rank_base[-1])
        self._pieces = None

    def _cid(self, i):
        return self.prefix + "_".join(str(int(v)) for v in self.idx[i])

    @property
    def pieces(self):
        """Piece records (built on first use; the plan itself is arrays)."""
        if self._pieces is None:
            out = []
            for i in range(len(self.idx)):
                cs = tuple(slice(int(a), int(a) + (int(c) - 1) * int(t) + 1, int(t))
                           for a, c, t in zip(self.cstart[i], self.count[i], self.steps))
                ds = tuple(slice(int(a), int(a) + int(c), 1) for a, c in zip(self.dstart[i], self.count[i]))
                out.append(Piece(self._cid(i), int(self.owner[i]), cs, ds, tuple(int(c) for c in self.count[i]),
                                 int(self.nbytes[i]), int(self.off[i])))
            self._pieces = out
        return self._pieces

    def chunk_ids(self, rank):
        """Chunk ids this rank decodes (or writes), in packing order."""
        return [self._cid(i) for i in self.by_rank[rank]]

    def selected_bytes(self, rank=None):
        return int(self.nbytes.sum() if rank is None else self.nbytes[self.by_rank[rank]].sum())

    # -- copy descriptors (COPY_DESC_DTYPE records, one per piece) --
    def _descs(self, ii, chunk_side, chunk_base, packed_base, to_chunk):
        """Descriptors between each piece's chunk-side region (chunk arrays at
        chunk_base[k], or the slab when chunk_side is False) and its packed bytes."""
        from .engine import COPY_DESC_DTYPE
        n, R = len(ii), self.rank
        if n == 0:
            return np.zeros((0, 27), np.int64)
        # the 216-byte record as 27 int64 words: src_off, dst_off, src_stride[8],
        # dst_stride[8], count[8], rank | itemsize << 32
        m = np.zeros((n, 27), np.int64)
        cnt = self.count[ii]
        # packed piece: C-contiguous array of its selection shape
        pst = np.empty((n, R), np.int64)
        pst[:, R - 1] = self.itemsize
        for d in range(R - 2, -1, -1):
            pst[:, d] = pst[:, d + 1] * cnt[:, d + 1]
        if chunk_side:
            cs = _c_strides(self.layout, self.itemsize)
            off = np.asarray(chunk_base, np.int64) + self.cstart[ii] @ cs
            st = cs * self.steps
        else:
            ss = _c_strides(self.slab_shape, self.itemsize)
            off = int(chunk_base) + self.dstart[ii] @ ss
            st = ss
        poff = np.asarray(packed_base, np.int64) + self.off[ii]
        if to_chunk:
            m[:, 0], m[:, 1] = poff, off
            m[:, 2:2 + R], m[:, 10:10 + R] = pst, st
        else:
            m[:, 0], m[:, 1] = off, poff
            m[:, 2:2 + R], m[:, 10:10 + R] = st, pst
        m[:, 18:18 + R] = cnt
        m[:, 26] = R | (self.itemsize << 32)
        return m

    # -- the same records built on the device (hsds_plan_descs): only the per-dimension
    # tables and per-piece grid index / packed offset / chunk offset travel over PCIe --
    def device_descs(self, mode, device, ranks=None, chunk_offsets=None, packed_base=0, slab_base=0):
        """COPY_DESC records as a uint8 device tensor for `mode` (nat.PLAN_*):
        PACK / APPLY / APPLY_BCAST / DIRECT for ranks=[r] with chunk_offsets (one per owned
        piece), PLACE / GATHER for `ranks` (default all) at their rank_base offsets.
        DIRECT is direct_descs built on the device (chunk -> slab at slab_base)."""
        import torch
        from . import _native as nat
        from .engine import COPY_DESC_DTYPE, _ptr, _stream_handle, to_device_bytes
        rs = list(range(self.world)) if ranks is None else list(ranks)
        ii = np.concatenate([self.by_rank[r] for r in rs]) if rs else np.zeros(0, np.int64)
        n = len(ii)
        out = torch.empty(max(n, 1) * COPY_DESC_DTYPE.itemsize, dtype=torch.uint8, device=device)
        if n == 0:
            return out[:0]
        chunk_side = mode in (nat.PLAN_PACK, nat.PLAN_APPLY, nat.PLAN_APPLY_BCAST, nat.PLAN_DIRECT)
        if mode == nat.PLAN_APPLY_BCAST:
            poff = np.full(n, int(packed_base), np.int64)
        elif chunk_side:
            poff = int(packed_base) + self.off[ii]
        else:
            poff = np.concatenate([self.rank_base[r] + self.off[self.by_rank[r]] for r in rs])
        tabs = np.concatenate([np.concatenate(t[1:4]) for t in self._tabs])
        parts = [tabs, ii.astype(np.int64), poff]
        if chunk_side:
            co = np.asarray(chunk_offsets, np.int64)
            if len(co) != n:
                raise ValueError("one chunk offset per owned piece expected")
            parts.append(co)
        # (page-locked staging, asynchronous: the host does not wait here for the kernels
        # queued before -- the previous request's decode or encode)
        buf = to_device_bytes(np.concatenate(parts), device)
        g = nat.PlanGeom()
        g.rank, g.itemsize, g.mode = self.rank, self.itemsize, int(mode)
        cs = _c_strides(self.layout, self.itemsize)
        ss = _c_strides(self.slab_shape, self.itemsize)
        for d, t in enumerate(self._tabs):
            g.nk[d], g.chunk_stride[d], g.slab_stride[d], g.step[d] = len(t[0]), cs[d], ss[d], self.steps[d]
        g.slab_base = int(slab_base)
        base = _ptr(buf)
        t0, t1 = tabs.size, tabs.size + n
        rc = nat.lib().hsds_plan_descs(nat.engine(device.index).h, ctypes.byref(g), base, base + 8 * t0,
                                       base + 8 * t1, base + 8 * (t1 + n) if chunk_side else None, n, _ptr(out),
                                       _stream_handle(None))
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_plan_descs")
        return out

    def pack_descs(self, rank, chunk_offsets, packed_base=0):
        """Read: decoded chunk k (C-order `layout` array at byte offset chunk_offsets[k]
        of the decode buffer) -> its piece in the rank's packed buffer."""
        ii = self.by_rank[rank]
        if len(chunk_offsets) != len(ii):
            raise ValueError("one decoded chunk offset per owned piece expected")
        return _recs(self._descs(ii, True, chunk_offsets, packed_base, False))

    def direct_descs(self, rank, chunk_offsets, slab_base=0):
        """Read without a gather: decoded chunk k (at chunk_offsets[k]) [chunk_sel] ->
        slab[data_sel] at slab_base, for this rank's pieces (pack and place fused: each GPU
        writes its pieces straight into the response buffer)."""
        ii = self.by_rank[rank]
        if len(chunk_offsets) != len(ii):
            raise ValueError("one decoded chunk offset per owned piece expected")
        m = self._descs(ii, True, chunk_offsets, 0, False)          # chunk side -> (packed)
        p = self._descs(ii, False, slab_base, 0, True)              # (packed) -> slab side
        m[:, 1] = p[:, 1]
        m[:, 10:18] = p[:, 10:18]
        return _recs(m)

    def place_descs(self, ranks=None):
        """Read: gathered buffer (rank r's packed bytes at rank_base[r]) -> slab[data_slices]."""
        rs = range(self.world) if ranks is None else ranks
        return _cat([self._descs(self.by_rank[r], False, 0, self.rank_base[r], True) for r in rs])

    def gather_descs(self, ranks=None, slab_base=0):
        """Write: slab[data_slices] (the request's array, C order, at slab_base) -> each
        piece in the scattered buffer (rank r's pieces at rank_base[r]): arr[data_sel] of
        write_chunk_hyperslab (chunk_crawl.py:135)."""
        rs = range(self.world) if ranks is None else ranks
        return _cat([self._descs(self.by_rank[r], False, slab_base, self.rank_base[r], False) for r in rs])

    def apply_descs(self, rank, chunk_offsets, packed_base=0, broadcast=False):
        """Write: the rank's packed piece k -> chunk k (at chunk_offsets[k]) [chunk_sel]:
        chunkWriteSelection's copy (chunkUtil.py:983-986).  broadcast: every element of
        every piece reads the one value at packed_base (element_count == 1,
        chunk_crawl.py:118-133, chunk_dn.py:292-297)."""
        ii = self.by_rank[rank]
        if len(chunk_offsets) != len(ii):
            raise ValueError("one chunk offset per owned piece expected")
        m = self._descs(ii, True, chunk_offsets, packed_base, True)
        if broadcast:
            m[:, 0] = packed_base
            m[:, 2:10] = 0
        return _recs(m)


def partition_ids(prefix, idx, world):
    """getObjPartition of every chunk id prefix + '_'.join(idx[i]) (C ABI, batched md5)."""
    import ctypes
    from . import _native as nat
    idx = np.ascontiguousarray(idx, np.int64)
    n = len(idx)
    owner = np.zeros(n, np.int32)
    if n:
        rc = nat.lib().hsds_partition_ids(prefix.encode(), idx.shape[1], idx.ctypes.data, n, int(world),
                                          owner.ctypes.data)
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_partition_ids")
    return owner


def _recs(m):
    """int64 (n, 27) matrix -> COPY_DESC_DTYPE records (a view, no copy)."""
    from .engine import COPY_DESC_DTYPE
    return np.ascontiguousarray(m).view(COPY_DESC_DTYPE).reshape(len(m))


def _cat(mats):
    mats = [m for m in mats if len(m)]
    return _recs(np.concatenate(mats) if mats else np.zeros((0, 27), np.int64))


def exchange(packed, plan, rank, root=0, group=None, gathered=None):
    """Point-to-point gather of every rank's packed pieces to `root`.

    `packed`: 1-D uint8 tensor of plan.rank_bytes[rank] bytes (on the root it may be
    the view of `gathered` it was packed into).  Returns the gathered uint8 tensor on
    the root (rank r's bytes at plan.rank_base[r]), None elsewhere.  Works with any
    torch.distributed backend that has send/recv (RCCL on GPUs, gloo on CPU)."""
    import torch
    import torch.distributed as dist
    if rank != root:
        if plan.rank_bytes[rank]:
            if dist.get_backend(group) == "nccl":
                for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed[:plan.rank_bytes[rank]], root,
                                                            group=group)]):
                    q.wait()
            else:
                dist.send(packed[:plan.rank_bytes[rank]], root, group=group)
        return None
    if gathered is None:
        gathered = torch.empty(plan.gathered_nbytes, dtype=torch.uint8, device=packed.device)
    b0 = int(plan.rank_base[root])
    own = gathered[b0:b0 + plan.rank_bytes[root]]
    if plan.rank_bytes[root] and packed.data_ptr() != own.data_ptr():
        own.copy_(packed[:plan.rank_bytes[root]])
    peers = [r for r in range(plan.world) if r != root and plan.rank_bytes[r]]
    if dist.get_backend(group) == "nccl" and peers:
        # one RCCL group call: the receives from every peer run concurrently (one
        # xGMI link per peer) instead of one after another
        ops = [dist.P2POp(dist.irecv, gathered[int(plan.rank_base[r]):int(plan.rank_base[r]) + plan.rank_bytes[r]],
                          r, group=group) for r in peers]
        for q in dist.batch_isend_irecv(ops):
            q.wait()
        return gathered
    reqs = [dist.irecv(gathered[int(plan.rank_base[r]):int(plan.rank_base[r]) + plan.rank_bytes[r]], r, group=group)
            for r in peers]
    for q in reqs:
        q.wait()
    return gathered


def stage_objects(blobs, ids, device, eng=None, replicate=True):
    """Stored objects of chunk ids `ids` (dict chunk_id -> bytes / uint8 array; absent ids
    are missing chunks) staged in HBM.  An object shared by several ids (bench corpora)
    crosses PCIe once; with `replicate` every id still gets its own copy at a distinct HBM
    address (one copy launch), so no decode reads another chunk's bytes from cache.
    Returns (d_src, {chunk_id: (src_off, src_len)})."""
    import torch
    from .engine import COPY_DESC_DTYPE, ChunkEngine, pack_chunks
    present = [c for c in ids if c in blobs]
    uniq, objs, which = {}, [], []
    for c in present:
        b = blobs[c]
        k = uniq.setdefault(id(b), len(objs))
        if k == len(objs):
            objs.append(b)
        which.append(k)
    if not present:
        return torch.empty(1, dtype=torch.uint8, device=device), {}
    usrc, udescs, _ = pack_chunks(objs, [0] * len(objs))
    d_usrc = torch.from_numpy(np.concatenate([usrc, np.zeros(16, np.uint8)])).to(device)
    lens = np.array([len(objs[k]) for k in which], np.int64)
    if not replicate:
        offs = udescs["src_off"][which].astype(np.int64)
        return d_usrc, {c: (int(o), int(n)) for c, o, n in zip(present, offs, lens)}
    alen = (lens + 255) // 256 * 256
    soff = np.concatenate([[0], np.cumsum(alen)[:-1]]).astype(np.int64)
    d_src = torch.empty(max(int(alen.sum()), 1), dtype=torch.uint8, device=device)
    rec = np.zeros(len(present), COPY_DESC_DTYPE)
    rec["src_off"] = udescs["src_off"][which]
    rec["dst_off"] = soff
    rec["rank"], rec["itemsize"] = 2, 16
    rec["count"][:, 0] = (lens + 15) // 16
    rec["count"][:, 1] = 1
    rec["src_stride"][:, 0] = rec["dst_stride"][:, 0] = 16
    (eng or ChunkEngine(device.index)).copy(d_usrc, d_src, rec)
    return d_src, {c: (int(o), int(n)) for c, o, n in zip(present, soff, lens)}


class ShardedReader:
    """GPU read of a hyperslab: decode owned chunks -> pack -> exchange -> place."""

    def __init__(self, plan, rank, device, compressor="zlib", shuffle=1, root=0, group=None):
        import torch
        from .engine import ChunkEngine
        self.plan, self.rank, self.root, self.group = plan, rank, root, group
        self.device = device
        self.compressor, self.shuffle = compressor, shuffle
        self.eng = ChunkEngine(device.index)
        self.torch = torch

    def upload(self, blobs, fill_value=None):
        """Stage the stored objects of this rank's chunks (dict chunk_id -> bytes,
        absent ids are missing chunks) in HBM.  Returns the staged batch."""
        from .engine import CHUNK_DESC_DTYPE, to_device_bytes
        torch = self.torch
        ids = self.plan.chunk_ids(self.rank)
        present = [cid for cid in ids if cid in blobs]
        # an object shared by many chunk ids (bench corpora) crosses PCIe once and is
        # replicated into the batch layout on the device (stage_objects)
        d_src, table = stage_objects(blobs, ids, self.device, self.eng)
        descs = np.zeros(len(present), CHUNK_DESC_DTYPE)
        descs["src_off"] = [table[c][0] for c in present]
        descs["src_len"] = [table[c][1] for c in present]
        descs["dst_len"] = self.plan.chunk_nbytes
        descs["dst_off"] = np.arange(len(present), dtype=np.int64) * _align(self.plan.chunk_nbytes, 256)
        ext = len(present) * _align(self.plan.chunk_nbytes, 256)
        # missing chunks get their own fill-value slot after the decoded ones
        slot = {c: int(descs[k]["dst_off"]) for k, c in enumerate(present)}
        for c in ids:
            if c not in slot:
                slot[c] = ext
                ext += _align(self.plan.chunk_nbytes, 256)
        d_dst = torch.empty(max(ext, 1), dtype=torch.uint8, device=self.device)
        if len(slot) > len(present):
            fill = np.zeros(self.plan.layout, self.plan.dtype)
            if fill_value is not None:
                fill[...] = fill_value
            d_fill = torch.from_numpy(fill.view(np.uint8).reshape(-1).copy()).to(self.device)
            for c in ids:
                if c not in blobs:
                    o = slot[c]
                    d_dst[o:o + self.plan.chunk_nbytes].copy_(d_fill)
        offs = np.array([slot[c] for c in ids], np.int64)
        return {
            "n": len(present),
            "d_src": d_src,
            "d_desc": to_device_bytes(descs, self.device) if len(present) else None,
            "d_dst": d_dst,
            "d_status": torch.zeros(max(len(present), 1), dtype=torch.int32, device=self.device),
            "offs": offs,
            "npack": len(ids),
            "itemsize": self.plan.itemsize,
            **self._records(self.plan, offs),
        }

    def _records(self, plan, offs):
        """Copy records of a staged batch.  The root places its own pieces straight from its
        decoded chunks into the slab (one copy, no packed buffer: DIRECT) and the peers'
        packed pieces from the gathered buffer (PLACE); every other rank packs (PACK)."""
        if self.rank != self.root:
            return {"d_pack": plan.device_descs(nat.PLAN_PACK, self.device, ranks=[self.rank], chunk_offsets=offs),
                    "d_direct": None, "d_place": None}
        peers = [r for r in range(plan.world) if r != self.root and len(plan.by_rank[r])]
        return {"d_pack": None,
                "d_direct": plan.device_descs(nat.PLAN_DIRECT, self.device, ranks=[self.rank], chunk_offsets=offs),
                "d_place": plan.device_descs(nat.PLAN_PLACE, self.device, ranks=peers) if peers else None}

    def replan(self, st, plan):
        """Take a freshly built plan of the same request (same chunks per rank) for a
        staged batch: its copy records are rebuilt on the device (the per-request planning
        cost the bench times inside each step)."""
        if [len(b) for b in plan.by_rank] != [len(b) for b in self.plan.by_rank]:
            raise ValueError("replan needs the same request")
        self.plan = plan
        st.update(self._records(plan, st["offs"]))
        return st

    def _decode(self, st, stream=None):
        if st["n"]:
            self.eng.decode(st["d_src"], st["d_desc"], st["d_dst"], st["d_status"], compressor=self.compressor,
                            shuffle=self.shuffle, itemsize=st["itemsize"], stream=stream)

    def decode_and_pack(self, st, packed, stream=None):
        """A non-root rank: decode, then pack its pieces for the gather."""
        self._decode(st, stream)
        if st["npack"]:
            self.eng.copy(st["d_dst"], packed, st["d_pack"], stream=stream)

    def decode_and_place(self, st, slab, stream=None):
        """The root: decode, then copy its own pieces straight into the slab."""
        self._decode(st, stream)
        if st["npack"]:
            self.eng.copy(st["d_dst"], slab, st["d_direct"], stream=stream)

    def read(self, st, slab=None, gathered=None, fill_value=None, check=True):
        """Whole read; returns the slab (uint8 tensor, C order) on the root."""
        torch = self.torch
        plan = self.plan
        if self.rank == self.root:
            if slab is None:
                slab = torch.empty(max(plan.slab_nbytes, 1), dtype=torch.uint8, device=self.device)
                fill = np.zeros(1, plan.dtype)
                if fill_value is not None:
                    fill[...] = fill_value
                if fill.view(np.uint8).any():
                    pat = torch.from_numpy(np.full(plan.slab_nbytes // plan.itemsize, fill[0], plan.dtype)
                                           .view(np.uint8).copy()).to(self.device)
                    slab[:plan.slab_nbytes].copy_(pat)
                else:
                    slab.zero_()
            if plan.world > 1 and gathered is None:
                gathered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=self.device)
            # the root's own section of the gathered buffer stays unused: its pieces go
            # straight from its decoded chunks into the slab
            b = int(plan.rank_base[self.root])
            packed = None if plan.world == 1 else gathered[b:b + max(plan.rank_bytes[self.root], 1)]
            self.decode_and_place(st, slab)
        else:
            packed = torch.empty(max(plan.rank_bytes[self.rank], 1), dtype=torch.uint8, device=self.device)
            self.decode_and_pack(st, packed)
        if check and st["n"]:
            bad = st["d_status"][:st["n"]].ne(0).any()
            if bool(bad):
                raise RuntimeError("chunk decode failed: " + str(torch.unique(st["d_status"][:st["n"]]).tolist()))
        if plan.world > 1:
            exchange(packed, plan, self.rank, self.root, self.group, gathered)
        if self.rank != self.root:
            return None
        if st["d_place"] is not None:
            self.eng.copy(gathered, slab, st["d_place"])
        return slab


def broadcast_write(arr, selection):
    """write_chunk_hyperslab's broadcast test (chunk_crawl.py:118-135): a one-element
    request array and no step > 1 in the selection -> the value is sent to every chunk
    with element_count = 1.  A one-element array with a stepped selection that has more
    than one element cannot be indexed by data_sel there either (the reference fails)."""
    n = int(np.prod(np.shape(arr)))
    if n != 1:
        return False
    if any((s.step or 1) > 1 for s in selection):
        if int(np.prod(sel.getSelectionShape(selection))) != 1:
            raise ValueError("one-element write with a stepped selection: no broadcast")
        return False
    return True


class ShardedWriter:
    """GPU write of a hyperslab: gather per-owner pieces on the root -> scatter -> apply
    (RMW in each rank's HBM chunk store) -> flush (local encode).

    `store` is this rank's hsds_amd.datanode.ChunkStore (its chunks are the ones the md5
    rule assigns to it, like a DN's)."""

    def __init__(self, plan, rank, store, root=0, group=None):
        import torch
        from .engine import ChunkEngine
        dt = np.dtype(plan.dtype)
        if dt.names or dt.subdtype is not None:
            raise NotImplementedError("ShardedWriter takes scalar dtypes (ChunkStore.put_pieces); "
                                      "write compound datasets with ChunkStore.put_selections")
        self.plan, self.rank, self.store, self.root, self.group = plan, rank, store, root, group
        self.device = store.cache.arena.buf.device
        self.eng = ChunkEngine(self.device.index)
        self.torch = torch

    def scatter(self, arr=None, broadcast=False):
        """Root: `arr` is the request array (numpy or a uint8 / typed device tensor, C order,
        selection shape; one element when broadcasting).  Returns this rank's packed pieces
        (uint8 device tensor; the single value when broadcasting)."""
        torch = self.torch
        plan = self.plan
        if broadcast:
            val = np.zeros(1, plan.dtype)
            if self.rank == self.root:
                val[...] = np.asarray(arr).reshape(-1)[0] if not isinstance(arr, torch.Tensor) else \
                    arr.reshape(-1).view(torch.uint8)[:plan.itemsize].cpu().numpy().view(plan.dtype)[0]
            t = torch.from_numpy(val.view(np.uint8).copy()).to(self.device)
            if plan.world > 1:
                import torch.distributed as dist
                dist.broadcast(t, self.root, group=self.group)
            return t
        if self.rank == self.root:
            if isinstance(arr, torch.Tensor):
                d_arr = arr.reshape(-1).view(torch.uint8) if arr.dtype != torch.uint8 else arr.reshape(-1)
                if d_arr.device != self.device:
                    d_arr = d_arr.to(self.device)
            else:
                a = np.ascontiguousarray(arr, dtype=plan.dtype)
                if tuple(a.shape) != tuple(plan.slab_shape):
                    raise ValueError(f"request array shape {a.shape} != selection shape {plan.slab_shape}")
                d_arr = torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(self.device)
            if d_arr.numel() != plan.slab_nbytes:
                raise ValueError("request array size does not match the selection")
            scattered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=self.device)
            if len(plan.idx):
                self.eng.copy(d_arr, scattered, plan.device_descs(nat.PLAN_GATHER, self.device))
        else:
            scattered = None
        if plan.world == 1:
            return scattered
        return scatter_exchange(scattered, plan, self.rank, self.root, self.group, self.device)

    def apply(self, packed, filter_ops=None, fill_value=None, write_zero_chunks=False, broadcast=False):
        """PUT_Chunk for every piece this rank owns; returns {chunk_id: dirty}."""
        from .datanode import ChunkRead
        from .partition import getS3Key
        plan = self.plan
        ids = plan.chunk_ids(self.rank)
        if not ids:
            return {}
        reads = [ChunkRead(c, getS3Key(c)) for c in ids]

        def make(offs):
            # `packed` starts at this rank's first piece (the root's is a view at its rank_base)
            return plan.device_descs(nat.PLAN_APPLY_BCAST if broadcast else nat.PLAN_APPLY, self.device,
                                     ranks=[self.rank], chunk_offsets=offs, packed_base=0)
        dirty = self.store.put_pieces(reads, packed, make, plan.dtype, plan.layout, filter_ops=filter_ops,
                                      fill_value=fill_value, write_zero_chunks=write_zero_chunks)
        return dict(zip(ids, dirty))

    def write(self, arr=None, filter_ops=None, fill_value=None, write_zero_chunks=False):
        """scatter + apply; `arr` matters on the root only."""
        bc = False
        if self.rank == self.root:
            bc = broadcast_write(arr, self.plan.selection) if arr is not None and not \
                isinstance(arr, self.torch.Tensor) else False
        if self.plan.world > 1:
            import torch.distributed as dist
            flag = self.torch.tensor([1 if bc else 0], dtype=self.torch.int32, device=self.device)
            dist.broadcast(flag, self.root, group=self.group)
            bc = bool(flag.item())
        packed = self.scatter(arr, broadcast=bc)
        return self.apply(packed, filter_ops=filter_ops, fill_value=fill_value, write_zero_chunks=write_zero_chunks,
                          broadcast=bc)

    def flush(self, put, filter_ops=None):
        """s3sync of this rank's dirty chunks (local encode, ChunkStore.flush)."""
        return self.store.flush(put, filter_ops=filter_ops)


def scatter_exchange(scattered, plan, rank, root=0, group=None, device=None):
    """Root -> every rank: rank r receives plan.rank_bytes[r] bytes (its pieces, the root's
    scattered[rank_base[r]:...]).  One point-to-point message per rank (RCCL over xGMI on
    GPUs, gloo on CPU).  Returns this rank's packed tensor."""
    import torch
    import torch.distributed as dist
    nb = plan.rank_bytes[rank]
    if rank == root:
        peers = [r for r in range(plan.world) if r != root and plan.rank_bytes[r]]
        parts = {r: scattered[int(plan.rank_base[r]):int(plan.rank_base[r]) + plan.rank_bytes[r]] for r in peers}
        if dist.get_backend(group) == "nccl" and peers:
            for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, parts[r], r, group=group) for r in peers]):
                q.wait()
        else:
            reqs = [dist.isend(parts[r], r, group=group) for r in peers]
            for q in reqs:
                q.wait()
        b = int(plan.rank_base[root])
        return scattered[b:b + max(nb, 1)]
    dev = device if device is not None else torch.device("cpu")
    out = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    if nb:
        if dist.get_backend(group) == "nccl":
            for q in dist.batch_isend_irecv([dist.P2POp(dist.irecv, out[:nb], root, group=group)]):
                q.wait()
        else:
            dist.recv(out[:nb], root, group=group)
    return out


class PagedReader:
    """GET_Value with stream pagination (chunk_sn.py:1085-1135) on the sharded GPU path.

    getSelectionPagination (dsetUtil.py:689-800) cuts the selection along its first
    dimension of extent > 1 into pages of at most max_request_size bytes; pages are read
    in order and each page's bytes are handed to `sink(page_no, page_selection, host_u8)`
    -- the reference's resp.write(arrayToBytes(arr)) -- so the response is the pages
    concatenated.  Per page every rank decodes only the chunks it does not already hold:
    its decoded chunks live in a slot pool and a chunk shared by consecutive pages (pages
    cut through chunk rows) is decoded once, as the DN's chunk cache would serve it.

    mode "gather": pack -> RCCL gather to the root -> place into a device page slab ->
    one D2H into the host page buffer.  mode "direct" (no gather): every rank places its
    pieces straight into the host page buffer (hsds_host_map'ed; with world > 1 a
    /dev/shm file every rank of the node maps, `shm_path`), then a barrier.

    `source` is get_blobs(chunk_ids) -> {chunk_id: stored object bytes / uint8 array}
    (host objects, staged per decode batch), or a (d_src, {chunk_id: (src_off, src_len)})
    pair of objects already in HBM (stage_objects); an id without an object reads as the
    fill value."""

    def __init__(self, dset_id, dims, layout, selection, dtype, world, rank, device, max_request_size=100 << 20,
                 compressor="zlib", shuffle=1, mode="gather", root=0, group=None, shm_path=None, batch_chunks=2048):
        import torch
        from .engine import ChunkEngine, HostBuffer
        if mode not in ("gather", "direct"):
            raise ValueError("mode: gather or direct")
        self.dset_id, self.dims, self.layout = dset_id, tuple(dims), tuple(layout)
        self.dtype = np.dtype(dtype)
        self.world, self.rank, self.root, self.group = int(world), int(rank), root, group
        self.device = torch.device(device)
        self.compressor, self.shuffle, self.mode = compressor, shuffle, mode
        self.pages = sel.getSelectionPagination(tuple(selection), self.dims, self.dtype.itemsize, max_request_size)
        self.page_bytes = [int(np.prod(sel.getSelectionShape(p), dtype=np.int64)) * self.dtype.itemsize
                           for p in self.pages]
        self.eng = ChunkEngine(self.device.index)
        self.torch = torch
        cap = max(self.page_bytes) if self.page_bytes else 1
        if mode == "direct":
            shared = self.world > 1
            if shared and shm_path is None:
                raise ValueError("direct mode with world > 1 needs a shm_path every rank maps")
            if shared and self.rank != self.root:
                import torch.distributed as dist
                dist.barrier(group=group)                       # the root has created the file
                self.host = HostBuffer(cap, self.device, path=shm_path, create=False)
            else:
                self.host = HostBuffer(cap, self.device, path=shm_path if shared else None)
                if shared:
                    import torch.distributed as dist
                    dist.barrier(group=group)
        else:
            self.host = torch.empty(cap, dtype=torch.uint8).pin_memory() if self.rank == root else None
        # decode look-ahead: a page whose chunks are not all resident decodes them together
        # with the next pages' missing chunks, up to batch_chunks per rank (one page's chunk
        # row alone is a quarter of a decode round)
        self.batch_chunks = max(1, int(batch_chunks))
        self.csize = int(np.prod(self.layout, dtype=np.int64)) * self.dtype.itemsize
        self.cstride = _align(self.csize, 256)
        self.pool = None
        self.slot_of = {}                      # chunk id -> pool slot
        self.stats = {"pages": 0, "decoded": 0, "reused": 0, "decode_batches": 0}

    def _slots(self, ids):
        """Pool slots for the chunk ids `ids` (a page and its look-ahead): keep the ones
        already decoded, free the rest, hand free slots to new ids.  Returns (offsets,
        new ids, their slots)."""
        torch = self.torch
        keep = {c: self.slot_of[c] for c in ids if c in self.slot_of}
        need = len(ids)
        if self.pool is None or self.pool.numel() < need * self.cstride:
            # a bigger pool: the decoded chunks keep their slot offsets
            big = torch.empty(max(2 * need, 1) * self.cstride, dtype=torch.uint8, device=self.device)
            if self.pool is not None:
                big[:self.pool.numel()].copy_(self.pool)
            self.pool = big
        nslots = self.pool.numel() // self.cstride
        used = set(keep.values())
        free = (k for k in range(nslots) if k not in used)
        new, new_slots = [], []
        for c in ids:
            if c not in keep:
                k = next(free)
                keep[c] = k
                new.append(c)
                new_slots.append(k)
        self.slot_of = keep
        offs = np.array([keep[c] * self.cstride for c in ids], np.int64)
        return offs, new, new_slots

    def _decode(self, new, new_slots, source, fill_value):
        from .engine import CHUNK_DESC_DTYPE, pack_chunks
        torch = self.torch
        staged = isinstance(source, tuple)
        table = source[1] if staged else (source(new) if new else {})
        present = [(c, k) for c, k in zip(new, new_slots) if c in table]
        missing = [k for c, k in zip(new, new_slots) if c not in table]
        if present:
            if staged:
                d_src = source[0]
                descs = np.zeros(len(present), CHUNK_DESC_DTYPE)
                descs["src_off"] = [table[c][0] for c, _ in present]
                descs["src_len"] = [table[c][1] for c, _ in present]
                descs["dst_len"] = self.csize
            else:
                src, descs, _ = pack_chunks([table[c] for c, _ in present], [self.csize] * len(present))
                d_src = torch.from_numpy(src).to(self.device)
            descs["dst_off"] = np.array([k * self.cstride for _, k in present], np.uint64)
            st = torch.full((len(present),), 99, dtype=torch.int32, device=self.device)
            self.eng.decode(d_src, descs, self.pool, st, compressor=self.compressor, shuffle=self.shuffle,
                            itemsize=self.dtype.itemsize)
            bad = st.ne(0)
            if bool(bad.any()):
                raise RuntimeError("chunk decode failed: " + str(torch.unique(st).tolist()))
        if missing:
            fill = np.zeros(self.layout, self.dtype)
            if fill_value is not None:
                fill[...] = fill_value
            d_fill = torch.from_numpy(fill.view(np.uint8).reshape(-1).copy()).to(self.device)
            for k in missing:
                self.pool[k * self.cstride:k * self.cstride + self.csize].copy_(d_fill)
        self.stats["decoded"] += len(new)

    def read(self, source, sink, fill_value=None):
        """Read every page in order; returns the total bytes handed to `sink` (root)."""
        torch = self.torch
        total = 0
        plans = {}

        def plan_of(q):
            if q not in plans:
                plans[q] = SelectionPlan(self.dset_id, self.dims, self.layout, self.pages[q], self.dtype, self.world)
            return plans[q]
        for pno, page in enumerate(self.pages):
            plan = plan_of(pno)
            plans.pop(pno - 1, None)
            ids = plan.chunk_ids(self.rank)
            if any(c not in self.slot_of for c in ids):
                want, seen = list(ids), set(ids)
                nnew = sum(1 for c in ids if c not in self.slot_of)
                q = pno + 1
                while q < len(self.pages) and nnew < self.batch_chunks:
                    for c in plan_of(q).chunk_ids(self.rank):
                        if c not in seen:
                            seen.add(c)
                            want.append(c)
                            nnew += c not in self.slot_of
                    q += 1
                _, new, new_slots = self._slots(want)
                self._decode(new, new_slots, source, fill_value)
                self.stats["decode_batches"] += 1
            else:
                new = []
            offs = np.array([self.slot_of[c] * self.cstride for c in ids], np.int64)
            fresh = set(new)
            self.stats["reused"] += sum(1 for c in ids if c not in fresh)
            nb = self.page_bytes[pno]
            if self.mode == "direct":
                if len(ids):
                    self.eng.copy(self.pool, self.host, plan.direct_descs(self.rank, offs))
                torch.cuda.synchronize(self.device)
                if self.world > 1:
                    import torch.distributed as dist
                    dist.barrier(group=self.group)
                if self.rank == self.root:
                    sink(pno, page, self.host.array[:nb])
                if self.world > 1:
                    dist.barrier(group=self.group)           # the page buffer is free again
            else:
                if self.rank == self.root:
                    gathered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=self.device)
                    b = int(plan.rank_base[self.root])
                    packed = gathered[b:b + max(plan.rank_bytes[self.root], 1)]
                else:
                    gathered = None
                    packed = torch.empty(max(plan.rank_bytes[self.rank], 1), dtype=torch.uint8, device=self.device)
                if len(ids):
                    self.eng.copy(self.pool, packed, plan.device_descs(nat.PLAN_PACK, self.device, ranks=[self.rank],
                                                                       chunk_offsets=offs))
                got = exchange(packed, plan, self.rank, self.root, self.group, gathered) if self.world > 1 \
                    else gathered
                if self.rank == self.root:
                    slab = torch.empty(max(nb, 1), dtype=torch.uint8, device=self.device)
                    if len(plan.idx):
                        self.eng.copy(got, slab, plan.device_descs(nat.PLAN_PLACE, self.device))
                    self.host[:nb].copy_(slab[:nb])
                    sink(pno, page, self.host[:nb].numpy())
            total += nb
            self.stats["pages"] += 1
        return total

    def close(self):
        if self.mode == "direct":
            self.host.close()
