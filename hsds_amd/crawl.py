"""Chunk-sharded hyperslab read across the GPUs of one node.

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
"""
from dataclasses import dataclass

import numpy as np

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


class SelectionPlan:
    """Per-chunk read plan of a hyperslab selection sharded over `world` ranks.

    `selection` is a tuple of slices (getSelectionList output).  Point (coordinate)
    selections are not hyperslabs and are outside the distributed path."""

    ALIGN = 16

    def __init__(self, dset_id, dims, layout, selection, dtype, world, partition=None):
        self.dims = tuple(int(d) for d in dims)
        self.layout = tuple(int(c) for c in layout)
        self.selection = tuple(selection)
        if any(not isinstance(s, slice) for s in self.selection):
            raise NotImplementedError("coordinate selections are outside the distributed hyperslab path")
        if len(self.selection) != len(self.dims) or len(self.layout) != len(self.dims):
            raise ValueError("selection / layout rank does not match dataset rank")
        self.dtype = np.dtype(dtype)
        self.itemsize = self.dtype.itemsize
        self.world = int(world)
        self.slab_shape = tuple(sel.getSelectionShape(self.selection))
        self.slab_nbytes = int(np.prod(self.slab_shape, dtype=np.int64)) * self.itemsize
        self.chunk_nbytes = int(np.prod(self.layout, dtype=np.int64)) * self.itemsize
        part = partition or (lambda cid: getObjPartition(cid, self.world))
        self.pieces = []
        for cid in sel.getChunkIds(dset_id, self.selection, self.layout):
            csel = sel.getChunkSelection(cid, self.selection, self.layout)
            if csel is None:
                continue
            shape = tuple(sel.getSelectionShape(csel))
            n = int(np.prod(shape, dtype=np.int64)) * self.itemsize
            if n == 0:
                continue
            self.pieces.append(Piece(cid, part(cid), tuple(sel.getChunkCoverage(cid, self.selection, self.layout)),
                                     tuple(sel.getDataCoverage(cid, self.selection, self.layout)), shape, n))
        self.by_rank = [[] for _ in range(self.world)]
        for i, p in enumerate(self.pieces):
            self.by_rank[p.owner].append(i)
        self.rank_bytes = []
        for r in range(self.world):
            off = 0
            for i in self.by_rank[r]:
                self.pieces[i].off = off
                off += _align(self.pieces[i].nbytes, self.ALIGN)
            self.rank_bytes.append(off)
        self.rank_base = np.concatenate([[0], np.cumsum(self.rank_bytes)]).astype(np.int64)
        self.gathered_nbytes = int(self.rank_base[-1])

    def chunk_ids(self, rank):
        """Chunk ids this rank decodes, in packing order."""
        return [self.pieces[i].chunk_id for i in self.by_rank[rank]]

    def selected_bytes(self, rank=None):
        idx = range(len(self.pieces)) if rank is None else self.by_rank[rank]
        return sum(self.pieces[i].nbytes for i in idx)

    def pack_descs(self, rank, chunk_offsets, packed_base=0):
        """Copy descriptors: decoded chunk k (C-order `layout` array at byte offset
        chunk_offsets[k] of the decode buffer) -> its piece in the packed buffer."""
        idx = self.by_rank[rank]
        if len(chunk_offsets) != len(idx):
            raise ValueError("one decoded chunk offset per owned piece expected")
        recs = [sel.copy_desc(self.layout, p.chunk_slices, p.shape, sel._contig_slices(p.shape), self.itemsize,
                              src_base=int(o), dst_base=packed_base + p.off)
                for p, o in ((self.pieces[i], o) for i, o in zip(idx, chunk_offsets))]
        return _cat(recs)

    def place_descs(self, ranks=None):
        """Copy descriptors: gathered buffer (rank r's packed bytes at rank_base[r]) ->
        slab[data_slices]."""
        recs = []
        for r in (range(self.world) if ranks is None else ranks):
            for i in self.by_rank[r]:
                p = self.pieces[i]
                recs.append(sel.copy_desc(p.shape, sel._contig_slices(p.shape), self.slab_shape, p.data_slices,
                                          self.itemsize, src_base=int(self.rank_base[r]) + p.off))
        return _cat(recs)


def _cat(recs):
    from .engine import COPY_DESC_DTYPE
    if not recs:
        return np.zeros(0, COPY_DESC_DTYPE)
    return np.concatenate(recs)


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
        from .engine import pack_chunks, to_device_bytes
        torch = self.torch
        ids = self.plan.chunk_ids(self.rank)
        present = [cid for cid in ids if cid in blobs]
        src, descs, ext = pack_chunks([blobs[c] for c in present], [self.plan.chunk_nbytes] * len(present))
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
            "d_src": torch.from_numpy(src).to(self.device),
            "d_desc": to_device_bytes(descs, self.device) if len(present) else None,
            "d_dst": d_dst,
            "d_status": torch.zeros(max(len(present), 1), dtype=torch.int32, device=self.device),
            "d_pack": to_device_bytes(self.plan.pack_descs(self.rank, offs), self.device),
            "npack": len(ids),
            "d_place": (to_device_bytes(self.plan.place_descs(), self.device) if self.rank == self.root
                        else None),
            "itemsize": self.plan.itemsize,
        }

    def decode_and_pack(self, st, packed, stream=None):
        if st["n"]:
            self.eng.decode(st["d_src"], st["d_desc"], st["d_dst"], st["d_status"], compressor=self.compressor,
                            shuffle=self.shuffle, itemsize=st["itemsize"], stream=stream)
        if st["npack"]:
            self.eng.copy(st["d_dst"], packed, st["d_pack"], stream=stream)

    def read(self, st, slab=None, gathered=None, fill_value=None, check=True):
        """Whole read; returns the slab (uint8 tensor, C order) on the root."""
        torch = self.torch
        plan = self.plan
        if self.rank == self.root:
            if gathered is None:
                gathered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=self.device)
            b = int(plan.rank_base[self.root])
            packed = gathered[b:b + max(plan.rank_bytes[self.root], 1)]
        else:
            packed = torch.empty(max(plan.rank_bytes[self.rank], 1), dtype=torch.uint8, device=self.device)
        self.decode_and_pack(st, packed)
        if check and st["n"]:
            bad = st["d_status"][:st["n"]].ne(0).any()
            if bool(bad):
                raise RuntimeError("chunk decode failed: " + str(torch.unique(st["d_status"][:st["n"]]).tolist()))
        if plan.world > 1:
            got = exchange(packed, plan, self.rank, self.root, self.group, gathered)
        else:
            got = gathered
        if self.rank != self.root:
            return None
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
        if len(plan.pieces):
            self.eng.copy(got, slab, st["d_place"])
        return slab
