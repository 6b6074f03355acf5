"""Paginated sharded reads on the GPU (GET_Value stream pagination, chunk_sn.py:1085-1135,
over getSelectionPagination, dsetUtil.py:689-800): gather mode (pack -> exchange ->
place -> D2H) and the no-gather mode (every rank places its pieces straight into a
host response buffer it maps), checked against numpy."""
import os
import socket

import numpy as np
import pytest

from hsds_amd import crawl, selection as sel

pytestmark = pytest.mark.gpu

DSET = "d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d"
DIMS, LAYOUT = (600, 500), (64, 128)
SELECT = (slice(5, 590, 1), slice(3, 500, 2))


def _data():
    rng = np.random.default_rng(9)
    return np.round(np.cumsum(rng.normal(size=DIMS), axis=1), 2).astype(np.float32)


def _blobs(full, missing=()):
    from oracle import oracle as orc
    out = {}
    nr, nc = (-(-d // c) for d, c in zip(DIMS, LAYOUT))
    for i in range(nr):
        for j in range(nc):
            cid = "c-" + DSET[2:] + f"_{i}_{j}"
            if (i, j) in missing:
                continue
            c = np.zeros(LAYOUT, np.float32)
            blk = full[i * 64:(i + 1) * 64, j * 128:(j + 1) * 128]
            c[:blk.shape[0], :blk.shape[1]] = blk
            out[cid] = orc.blosc_encode(c.tobytes(), typesize=1, clevel=4, shuffle=1)
    return out


@pytest.mark.parametrize("mode", ["gather", "direct"])
@pytest.mark.parametrize("staged", [False, True])
def test_paged_read_matches_numpy(mode, staged):
    import torch
    full = _data()
    blobs = _blobs(full, missing={(3, 1)})
    size = int(np.prod(sel.getSelectionShape(SELECT))) * 4
    dev = torch.device("cuda", 0)
    rd = crawl.PagedReader(DSET, DIMS, LAYOUT, SELECT, np.float32, 1, 0, dev, max_request_size=size // 6, mode=mode,
                           batch_chunks=6)
    assert len(rd.pages) >= 6
    got = []
    if staged:     # objects already in HBM (one copy per chunk id)
        source = crawl.stage_objects(blobs, sorted(blobs), dev)
    else:          # host objects fetched per decode batch
        source = lambda ids: {c: blobs[c] for c in ids if c in blobs}   # noqa: E731
    n = rd.read(source, lambda pno, page, b: got.append(np.array(b, copy=True)), fill_value=-1.5)
    rd.close()
    assert n == size
    want = full.copy()
    want[3 * 64:4 * 64, 1 * 128:2 * 128] = -1.5          # the missing chunk reads as the fill value
    assert np.array_equal(np.concatenate(got).view(np.float32).reshape(want[SELECT].shape), want[SELECT])
    # chunk rows shared by consecutive pages were decoded once
    assert rd.stats["reused"] > 0
    assert rd.stats["decoded"] == len(blobs) + 1          # every chunk once (+ the fill-value one)
    assert 1 < rd.stats["decode_batches"] < len(rd.pages)  # look-ahead: several pages per decode batch


def test_direct_placement_from_two_ranks_into_one_shared_buffer(tmp_path):
    """Two ranks' pieces (world 2 plan) written by the copy kernel into two mappings of one
    shared-memory file (as two processes of a node map it): together the whole slab."""
    import torch
    from hsds_amd.engine import ChunkEngine, HostBuffer, pack_chunks
    full = _data()
    blobs = _blobs(full)
    dev = torch.device("cuda", 0)
    plan = crawl.SelectionPlan(DSET, DIMS, LAYOUT, SELECT, np.float32, 2)
    path = "/dev/shm/hsds_amd_test_direct_%d" % os.getpid()
    hb = [HostBuffer(plan.slab_nbytes, dev, path=path, create=True)]
    hb.append(HostBuffer(plan.slab_nbytes, dev, path=path, create=False))
    try:
        eng = ChunkEngine(0)
        for r in (0, 1):
            ids = plan.chunk_ids(r)
            src, descs, ext = pack_chunks([blobs[c] for c in ids], [plan.chunk_nbytes] * len(ids))
            d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
            st = torch.full((len(ids),), 99, dtype=torch.int32, device=dev)
            eng.decode(torch.from_numpy(src).to(dev), descs, d_dst, st, compressor="zlib", shuffle=1, itemsize=4)
            eng.copy(d_dst, hb[r], plan.direct_descs(r, descs["dst_off"].astype(np.int64)))
            torch.cuda.synchronize()
            assert int(st.abs().sum()) == 0
        got = hb[0].array[:plan.slab_nbytes].view(np.float32).reshape(plan.slab_shape)
        assert np.array_equal(got, full[SELECT])
    finally:
        for h in hb:
            h.close()
        os.unlink(path)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, path, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        full = _data()
        blobs = _blobs(full)
        size = int(np.prod(sel.getSelectionShape(SELECT))) * 4
        rd = crawl.PagedReader(DSET, DIMS, LAYOUT, SELECT, np.float32, 2, rank, torch.device("cuda", 0),
                               max_request_size=size // 4, mode="direct", shm_path=path)
        got = []
        rd.read(lambda ids: {c: blobs[c] for c in ids}, lambda pno, page, b: got.append(np.array(b, copy=True)))
        rd.close()
        if rank == 0:
            ok = np.array_equal(np.concatenate(got).view(np.float32).reshape(full[SELECT].shape), full[SELECT])
            q.put(("ok" if ok else "mismatch", len(rd.pages)))
    except Exception as e:   # surfaced to the parent
        q.put((f"{type(e).__name__}: {e}", 0))
    finally:
        dist.destroy_process_group()


def test_paged_direct_two_processes():
    """The no-gather read across two processes (gloo barriers, one /dev/shm page buffer
    both map; both ranks use the one GPU of the test box)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = "/dev/shm/hsds_amd_test_paged_%d" % os.getpid()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, path, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = q.get(timeout=100)
    finally:
        for p in ps:
            p.join(timeout=60)
        if os.path.exists(path):
            os.unlink(path)
    assert res[0] == "ok", res
    assert res[1] >= 4
