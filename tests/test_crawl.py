"""Distributed hyperslab read plan (hsds_amd/crawl.py): md5 sharding, pack/place copy
descriptors and the point-to-point exchange, checked on CPU against numpy slicing
(`full[selection]`, the reference's chunk_crawl.py:418 semantics).  The exchange runs
over gloo with world_size 2 (and 3); the GPU path uses the same plan with RCCL."""
import os
import socket

import numpy as np
import pytest

from hsds_amd import crawl, selection as sel
from hsds_amd.partition import getObjPartition

DSET = "d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d"


def apply_descs(src, dst, descs):
    """numpy interpreter of hsds_copy_desc records (the hsds_copy_batch contract):
    for every multi-index i: dst[dst_off + i.dst_stride] = src[src_off + i.src_stride]."""
    from numpy.lib.stride_tricks import as_strided
    for d in descs:
        r, isz = int(d["rank"]), int(d["itemsize"])
        cnt = tuple(int(x) for x in d["count"][:r]) + (isz,)
        s = as_strided(src[int(d["src_off"]):], cnt, tuple(int(x) for x in d["src_stride"][:r]) + (1,))
        t = as_strided(dst[int(d["dst_off"]):], cnt, tuple(int(x) for x in d["dst_stride"][:r]) + (1,))
        t[...] = s


def chunk_array(full, layout, cid):
    """Decoded chunk (full layout dims, zero-padded at the dataset edge)."""
    idx = sel.getChunkIndex(cid)
    out = np.zeros(layout, full.dtype)
    region = tuple(slice(i * c, min((i + 1) * c, n)) for i, c, n in zip(idx, layout, full.shape))
    out[tuple(slice(0, r.stop - r.start) for r in region)] = full[region]
    return out


def pack_rank(plan, full, rank):
    ids = plan.chunk_ids(rank)
    cbytes = plan.chunk_nbytes
    dec = np.concatenate([chunk_array(full, plan.layout, c).view(np.uint8).reshape(-1) for c in ids]) \
        if ids else np.zeros(1, np.uint8)
    packed = np.zeros(max(plan.rank_bytes[rank], 1), np.uint8)
    apply_descs(dec, packed, plan.pack_descs(rank, [k * cbytes for k in range(len(ids))]))
    return packed


CASES = [
    ((100, 90), (16, 32), np.float32, (slice(3, 97, 1), slice(5, 90, 1))),
    ((100, 90), (16, 32), np.float32, (slice(0, 100, 3), slice(1, 88, 7))),
    ((40, 70, 33), (8, 16, 16), np.int16, (slice(0, 40, 2), slice(3, 70, 5), slice(1, 33, 3))),
    ((64, 64), (16, 16), np.float64, (slice(10, 11, 1), slice(0, 64, 40))),
    ((33, 50), (8, 8), np.uint8, (slice(0, 33, 1), slice(0, 50, 1))),
    ((20, 30, 10, 6), (4, 8, 5, 3), np.int32, (slice(1, 20, 4), slice(2, 30, 1), slice(0, 10, 9), slice(0, 6, 2))),
]


def _full(dims, dtype, seed=3):
    return (np.random.default_rng(seed).integers(0, 120, size=dims)).astype(dtype)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plan_pack_place_matches_numpy(case, world):
    dims, layout, dt, selection = CASES[case]
    full = _full(dims, dt)
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
    # every intersecting chunk appears once, owned by the md5 rule
    ids = [p.chunk_id for p in plan.pieces]
    assert len(set(ids)) == len(ids)
    for p in plan.pieces:
        assert p.owner == getObjPartition(p.chunk_id, world)
    assert plan.selected_bytes() == plan.slab_nbytes
    gathered = np.zeros(max(plan.gathered_nbytes, 1), np.uint8)
    for r in range(world):
        b = int(plan.rank_base[r])
        gathered[b:b + plan.rank_bytes[r]] = pack_rank(plan, full, r)[:plan.rank_bytes[r]]
    slab = np.zeros(plan.slab_nbytes, np.uint8)
    apply_descs(gathered, slab, plan.place_descs())
    assert np.array_equal(slab.view(dt).reshape(plan.slab_shape), full[selection])


def test_coordinate_selection_is_rejected():
    with pytest.raises(NotImplementedError):
        crawl.SelectionPlan(DSET, (10, 10), (5, 5), ([1, 2], slice(0, 10, 1)), np.float32, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dims, layout, dt, selection = CASES[case]
        full = _full(dims, dt)
        plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
        packed = torch.from_numpy(pack_rank(plan, full, rank))
        got = crawl.exchange(packed, plan, rank, root=0)
        if rank == 0:
            slab = np.zeros(plan.slab_nbytes, np.uint8)
            apply_descs(got.numpy(), slab, plan.place_descs())
            ok = np.array_equal(slab.view(dt).reshape(plan.slab_shape), full[selection])
            q.put(("ok" if ok else "mismatch", plan.rank_bytes))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, 0), (2, 2), (3, 5)])
def test_gloo_exchange(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, rank_bytes = q.get(timeout=5)
    assert status == "ok"
    assert sum(1 for b in rank_bytes if b) >= 2       # data really crossed ranks


# ---------------------------------------------------------------------------
# write side: slab -> per-owner pieces -> chunks (write_chunk_hyperslab + PUT_Chunk)
# ---------------------------------------------------------------------------
def _chunks_of(full, layout, plan, rank):
    ids = plan.chunk_ids(rank)
    cb = plan.chunk_nbytes
    buf = np.concatenate([chunk_array(full, layout, c).view(np.uint8).reshape(-1) for c in ids]) \
        if ids else np.zeros(1, np.uint8)
    return ids, buf, [k * cb for k in range(len(ids))]


def _assemble(full, layout, chunks):
    """dataset from chunk arrays {chunk_id: ndarray(layout)} (edges cropped)."""
    out = full.copy()
    for cid, arr in chunks.items():
        idx = sel.getChunkIndex(cid)
        region = tuple(slice(i * c, min((i + 1) * c, n)) for i, c, n in zip(idx, layout, full.shape))
        out[region] = arr[tuple(slice(0, r.stop - r.start) for r in region)]
    return out


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_write_plan_gather_apply_matches_numpy(case, world):
    """root: arr[data_sel] for every chunk packed per owner (gather_descs); each owner:
    packed piece -> its chunk[chunk_sel] (apply_descs); result == numpy full[sel] = arr"""
    dims, layout, dt, selection = CASES[case]
    before = _full(dims, dt, seed=11)
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
    arr = (np.arange(int(np.prod(plan.slab_shape))) % 97 + 1).astype(dt).reshape(plan.slab_shape)
    scattered = np.zeros(max(plan.gathered_nbytes, 1), np.uint8)
    apply_descs(np.ascontiguousarray(arr).view(np.uint8).reshape(-1), scattered, plan.gather_descs())
    chunks = {}
    for r in range(world):
        ids, buf, offs = _chunks_of(before, layout, plan, r)
        if not ids:
            continue
        b = int(plan.rank_base[r])
        apply_descs(scattered[b:b + plan.rank_bytes[r]], buf, plan.apply_descs(r, offs))
        cb = plan.chunk_nbytes
        for k, c in enumerate(ids):
            chunks[c] = buf[k * cb:(k + 1) * cb].view(dt).reshape(layout)
    want = before.copy()
    want[selection] = arr
    assert np.array_equal(_assemble(before, layout, chunks), want)


def test_write_broadcast_rule_and_apply():
    """element_count == 1 (chunk_crawl.py:118-135): one value, no step > 1 -> broadcast to
    every piece (source stride 0)"""
    dims, layout, dt = (100, 90), (16, 32), np.float32
    selection = (slice(3, 97, 1), slice(5, 90, 1))
    assert crawl.broadcast_write(np.float32(7.5), selection)
    assert crawl.broadcast_write(np.array([[7.5]], np.float32), selection)
    assert not crawl.broadcast_write(np.ones((2, 2), np.float32), selection)
    assert not crawl.broadcast_write(np.float32(1), (slice(3, 4, 1), slice(5, 6, 2)))
    with pytest.raises(ValueError):
        crawl.broadcast_write(np.float32(1), (slice(0, 10, 2), slice(5, 90, 1)))
    before = _full(dims, dt, seed=5)
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, 3)
    val = np.array([7.5], dt).view(np.uint8)
    chunks = {}
    for r in range(3):
        ids, buf, offs = _chunks_of(before, layout, plan, r)
        if ids:
            apply_descs(val, buf, plan.apply_descs(r, offs, broadcast=True))
            for k, c in enumerate(ids):
                chunks[c] = buf[k * plan.chunk_nbytes:(k + 1) * plan.chunk_nbytes].view(dt).reshape(layout)
    want = before.copy()
    want[selection] = 7.5
    assert np.array_equal(_assemble(before, layout, chunks), want)


def test_planning_scales_to_cfg4():
    """vectorized plan: configs[3] (65 536 chunks, 8 ranks) and configs[2] (16 384 chunks)
    plans plus descriptors in well under a second on one CPU core"""
    import time
    t = time.perf_counter()
    p = crawl.SelectionPlan(DSET, (131072, 131072), (512, 512), (slice(0, 131072, 4), slice(0, 131072, 4)),
                            np.float32, 8)
    p.place_descs()
    p.pack_descs(0, [0] * len(p.by_rank[0]))
    assert len(p.idx) == 65536 and p.slab_nbytes == 32768 * 32768 * 4
    p3 = crawl.SelectionPlan(DSET, (512, 2048, 2048), (16, 64, 128),
                             (slice(0, 512, 2), slice(3, 2048, 5), slice(1, 2048, 3)), np.int16, 1)
    p3.pack_descs(0, [0] * len(p3.by_rank[0]))
    p3.place_descs()
    assert len(p3.idx) == 16384
    assert time.perf_counter() - t < 2.0
    # the batched md5 partition is the reference rule
    ids = [p._cid(i) for i in range(0, 65536, 511)]
    assert [getObjPartition(c, 8) for c in ids] == [int(p.owner[i]) for i in range(0, 65536, 511)]


def _wworker(rank, world, port, case, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dims, layout, dt, selection = CASES[case]
        before = _full(dims, dt, seed=11)
        plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
        scattered = None
        if rank == 0:
            arr = (np.arange(int(np.prod(plan.slab_shape))) % 89 + 3).astype(dt).reshape(plan.slab_shape)
            s = np.zeros(max(plan.gathered_nbytes, 1), np.uint8)
            apply_descs(np.ascontiguousarray(arr).view(np.uint8).reshape(-1), s, plan.gather_descs())
            scattered = torch.from_numpy(s)
        packed = crawl.scatter_exchange(scattered, plan, rank, root=0).numpy()
        ids, buf, offs = _chunks_of(before, layout, plan, rank)
        if ids:
            apply_descs(packed, buf, plan.apply_descs(rank, offs))
        # ship the updated chunks to rank 0 for the check
        t = torch.from_numpy(buf.copy())
        n = torch.tensor([t.numel()], dtype=torch.int64)
        if rank == 0:
            chunks = {c: buf[k * plan.chunk_nbytes:(k + 1) * plan.chunk_nbytes].view(dt).reshape(layout)
                      for k, c in enumerate(ids)}
            for r in range(1, world):
                m = torch.zeros(1, dtype=torch.int64)
                dist.recv(m, r)
                b = torch.zeros(int(m.item()), dtype=torch.uint8)
                dist.recv(b, r)
                for k, c in enumerate(plan.chunk_ids(r)):
                    chunks[c] = b.numpy()[k * plan.chunk_nbytes:(k + 1) * plan.chunk_nbytes].view(dt).reshape(layout)
            want = before.copy()
            want[selection] = arr
            ok = np.array_equal(_assemble(before, layout, chunks), want)
            q.put(("ok" if ok else "mismatch", plan.rank_bytes))
        else:
            dist.send(n, 0)
            dist.send(t, 0)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, 1), (2, 2)])
def test_gloo_write_scatter(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wworker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, rank_bytes = q.get(timeout=5)
    assert status == "ok"
    assert sum(1 for b in rank_bytes if b) >= 2


def test_plan_grid_equals_meshgrid_product():
    """the plan's piece arrays are the C-order product of the per-dimension tables with
    untouched (count 0) entries dropped per dimension, as the meshgrid + mask form"""
    from hsds_amd import crawl
    cases = [((300, 200, 64), (64, 64, 32), (slice(3, 300, 7), slice(1, 200, 3), slice(0, 64, 5))),
             ((1000, 4000), (10, 100), (slice(5, 1000, 37), slice(0, 4000, 250))),
             ((50,), (7,), (slice(3, 49, 1),)),
             ((40, 40), (8, 8), (slice(9, 10, 1), slice(0, 40, 9)))]
    for dims, layout, sl in cases:
        plan = crawl.SelectionPlan("d-1a2b3c4d-5e6f7a8b-9c0d-1e2f3a-4b5c6d", dims, layout, sl, np.int16, 3)
        per = [crawl._dim_pieces(s, c) for s, c in zip(sl, layout)]
        grids = [np.meshgrid(*[p[k] for p in per], indexing="ij") for k in range(4)]
        cols = [np.stack([g.reshape(-1) for g in gk], axis=1) for gk in grids]
        keep = (cols[2] > 0).all(axis=1)
        for got, want in zip((plan.idx, plan.cstart, plan.count, plan.dstart), cols):
            assert np.array_equal(got, want[keep])


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [1, 3])
def test_direct_descs_place_every_rank_into_one_slab(case, world):
    """No-gather read: each rank writes its own pieces chunk -> slab (pack and place
    fused); all ranks together fill the whole selection."""
    dims, layout, dt, selection = CASES[case]
    full = _full(dims, dt)
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
    slab = np.zeros(plan.slab_nbytes + 64, np.uint8)
    cbytes = plan.chunk_nbytes
    for r in range(world):
        ids = plan.chunk_ids(r)
        if not ids:
            continue
        dec = np.concatenate([chunk_array(full, plan.layout, c).view(np.uint8).reshape(-1) for c in ids])
        apply_descs(dec, slab, plan.direct_descs(r, [k * cbytes for k in range(len(ids))], slab_base=32))
    assert np.array_equal(slab[32:32 + plan.slab_nbytes].view(dt).reshape(plan.slab_shape), full[selection])


@pytest.mark.parametrize("case", [0, 1, 2, 5])
def test_pages_concatenate_to_the_selection(case):
    """GET_Value streams getSelectionPagination's pages in order (chunk_sn.py:1085-1135):
    the pages' slabs concatenated are the whole selection's bytes."""
    dims, layout, dt, selection = CASES[case]
    full = _full(dims, dt)
    isz = np.dtype(dt).itemsize
    size = int(np.prod(sel.getSelectionShape(selection))) * isz
    pages = sel.getSelectionPagination(selection, dims, isz, max(size // 5, 1))
    assert len(pages) > 1
    out = []
    for page in pages:
        plan = crawl.SelectionPlan(DSET, dims, layout, page, dt, 2)
        slab = np.zeros(plan.slab_nbytes, np.uint8)
        for r in range(2):
            ids = plan.chunk_ids(r)
            if ids:
                dec = np.concatenate([chunk_array(full, layout, c).view(np.uint8).reshape(-1) for c in ids])
                apply_descs(dec, slab, plan.direct_descs(r, [k * plan.chunk_nbytes for k in range(len(ids))]))
        out.append(slab)
    # the reference streams full[page] for each page; those are the selection's rows in
    # order except where a stepped first slice starts off its step lattice (case 5: the
    # reference rounds page ends to multiples of the step, dsetUtil.py:759-770)
    want = np.concatenate([full[p].reshape(-1) for p in pages])
    assert np.array_equal(np.concatenate(out).view(dt), want)
    if case != 5:
        assert np.array_equal(want, full[selection].reshape(-1))
