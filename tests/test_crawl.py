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
