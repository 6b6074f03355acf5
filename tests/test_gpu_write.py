"""GPU parity of the sharded hyperslab write (hsds_amd.crawl.ShardedWriter, configs[4] path):
SN write gather by the plan (write_chunk_hyperslab's arr[data_sel], chunk_crawl.py:75-150),
per-owner pieces, DN PUT_Chunk on every owner (RMW through the HBM chunk store with
chunk_init, chunkWriteSelection compare + copy, chunk_dn.py:174-310) and the local encode of
s3sync (datanode_lib.py:1186-1318).  Eight ranks are simulated in one process (one chunk store
per rank on cuda:0, the root's scattered buffer handed to each rank as a view); the stored
objects are decoded by the oracle (c-blosc frame walk + libz) and compared with numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
DSET = "d-9e8d7c6b-5a4f3e2d-1c0b-9a8f7e-6d5c4b"


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


def _ops(dt, layout):
    from hsds_amd.filters import getFilterOps
    return getFilterOps({"filter_map": {}}, DSET, [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                                                   {"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": 4}],
                        dtype=dt, chunk_shape=layout)


def _simulate(dev, orc, dims, layout, dt, selection, arr, world, stored, fill_value=None, broadcast=False):
    """One write request through `world` simulated ranks.  `stored`: storage key -> object
    bytes (existing chunks: read-modify-write).  Returns the stored objects after the
    flush and the dirty flags."""
    import torch
    from hsds_amd import crawl
    from hsds_amd.datanode import ChunkStore
    from hsds_amd.engine import ChunkEngine
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, world)
    ops = _ops(dt, layout)
    eng = ChunkEngine(dev.index)
    if broadcast:
        value = torch.from_numpy(np.asarray(arr, dt).reshape(1).view(np.uint8).copy()).to(dev)
    else:
        d_arr = torch.from_numpy(np.ascontiguousarray(arr, dt).view(np.uint8).reshape(-1).copy()).to(dev)
        scattered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=dev)
        eng.copy(d_arr, scattered, plan.gather_descs())          # root: every piece, per owner
    out, dirty = dict(stored), {}
    for r in range(world):
        if not plan.by_rank[r].size:
            continue
        store = ChunkStore(lambda k, o, n: stored.get(k), mem_target=64 << 20, device=dev)
        w = crawl.ShardedWriter(plan, r, store)
        packed = value if broadcast else \
            scattered[int(plan.rank_base[r]):int(plan.rank_base[r]) + max(plan.rank_bytes[r], 1)]
        dirty.update(w.apply(packed, filter_ops=ops, fill_value=fill_value, broadcast=broadcast))
        w.flush(lambda k, b: out.__setitem__(k, b), filter_ops=ops)
    return plan, out, dirty


def _dataset(orc, objs, dims, layout, dt, fill):
    """decode every stored chunk object (oracle) into the full dataset"""
    from hsds_amd import selection as sel
    from hsds_amd.partition import getS3Key
    full = np.full(dims, fill, dt)
    cb = int(np.prod(layout)) * dt.itemsize
    grid = [range(-(-d // c)) for d, c in zip(dims, layout)]
    for idx in np.ndindex(*[len(g) for g in grid]):
        cid = "c-" + DSET[2:] + "_" + "_".join(str(i) for i in idx)
        key = getS3Key(cid)
        if key not in objs:
            continue
        raw = orc.uncompress(objs[key], "zlib", 1, dt.itemsize, cb)
        assert not isinstance(raw, int), (cid, raw)
        a = np.frombuffer(raw, dt).reshape(layout)
        region = tuple(slice(i * c, min((i + 1) * c, n)) for i, c, n in zip(idx, layout, dims))
        full[region] = a[tuple(slice(0, s.stop - s.start) for s in region)]
    assert sel is not None
    return full


def _existing(orc, dims, layout, dt, before, which):
    """stored objects for the chunks `which` (oracle F1 encoder = the reference's _compress)"""
    from hsds_amd.partition import getS3Key
    objs = {}
    for idx in which:
        cid = "c-" + DSET[2:] + "_" + "_".join(str(i) for i in idx)
        region = tuple(slice(i * c, min((i + 1) * c, n)) for i, c, n in zip(idx, layout, dims))
        a = np.zeros(layout, dt)
        a[tuple(slice(0, s.stop - s.start) for s in region)] = before[region]
        objs[getS3Key(cid)] = orc.blosc_encode(a.tobytes(), typesize=1, clevel=4, shuffle=1)
    return objs


@pytest.mark.parametrize("offset", [(0, 0), (100, 100)])
def test_sharded_write_8_ranks_512x512(dev, oracle_lib, offset):
    """configs[4] layout (512x512 f32 chunks) over 8 ranks: full-chunk writes, and the
    (100,100)-offset variant whose edge chunks are read-modify-written from stored objects"""
    orc = oracle_lib
    dt = np.dtype("<f4")
    dims, layout = (2048, 2560), (512, 512)
    rng = np.random.default_rng(21)
    before = np.round(np.cumsum(rng.normal(size=dims), axis=1), 2).astype(dt)
    grid = [(i, j) for i in range(4) for j in range(5)]
    stored = _existing(orc, dims, layout, dt, before, grid)
    y0, x0 = offset
    selection = (slice(y0, 2048, 1), slice(x0, 2560, 1))
    arr = np.round(np.cumsum(rng.normal(size=(2048 - y0, 2560 - x0)), axis=0), 2).astype(dt)
    plan, objs, dirty = _simulate(dev, orc, dims, layout, dt, selection, arr, 8, stored)
    assert sum(1 for b in plan.rank_bytes if b) >= 4          # the pieces really spread over owners
    assert all(dirty.values()) and len(dirty) == len(plan.idx)
    want = before.copy()
    want[selection] = arr
    assert np.array_equal(_dataset(orc, objs, dims, layout, dt, 0), want)


def test_sharded_write_strided_missing_chunks_fill_value(dev, oracle_lib):
    """a stepped selection over chunks with no stored object: chunk_init starts them from the
    fill value (datanode_lib.py:1132-1138); unchanged-data rewrites are not dirty"""
    orc = oracle_lib
    dt = np.dtype("<i2")
    dims, layout = (300, 200, 64), (64, 64, 32)
    selection = (slice(3, 300, 7), slice(1, 200, 3), slice(0, 64, 5))
    from hsds_amd import selection as sel
    shape = tuple(sel.getSelectionShape(selection))
    arr = (np.arange(int(np.prod(shape))) % 3001 - 1500).astype(dt).reshape(shape)
    plan, objs, dirty = _simulate(dev, orc, dims, layout, dt, selection, arr, 8, {}, fill_value=-7)
    want = np.full(dims, -7, dt)
    want[selection] = arr
    assert np.array_equal(_dataset(orc, objs, dims, layout, dt, -7), want)
    # writing the same values again over the stored objects changes nothing
    plan, objs2, dirty2 = _simulate(dev, orc, dims, layout, dt, selection, arr, 8, objs, fill_value=-7)
    assert not any(dirty2.values())


def test_sharded_write_broadcast(dev, oracle_lib):
    """element_count == 1 (chunk_crawl.py:118-135): one value broadcast to every piece"""
    orc = oracle_lib
    dt = np.dtype("<f8")
    dims, layout = (1000, 700), (256, 128)
    rng = np.random.default_rng(2)
    before = rng.normal(size=dims).astype(dt)
    grid = [(i, j) for i in range(4) for j in range(6)]
    stored = _existing(orc, dims, layout, dt, before, grid)
    selection = (slice(10, 990, 1), slice(50, 650, 1))
    from hsds_amd import crawl
    assert crawl.broadcast_write(np.float64(3.25), selection)
    plan, objs, dirty = _simulate(dev, orc, dims, layout, dt, selection, np.float64(3.25), 8, stored,
                                  broadcast=True)
    want = before.copy()
    want[selection] = 3.25
    assert np.array_equal(_dataset(orc, objs, dims, layout, dt, 0), want)


def test_sharded_write_corrupt_stored_object(dev, oracle_lib):
    """A chunk whose stored object fails to decode (get_chunk's 500 in its PUT_Chunk): the
    write raises it, that chunk leaves the cache, and every other chunk's update stands
    (one PUT_Chunk per chunk in the reference: the others are not undone)."""
    import torch
    from hsds_amd import crawl
    from hsds_amd.codec import HTTPInternalServerError
    from hsds_amd.datanode import ChunkStore
    from hsds_amd.partition import getS3Key
    orc = oracle_lib
    dt = np.dtype("<f4")
    dims, layout = (192, 256), (64, 64)
    rng = np.random.default_rng(5)
    before = np.round(np.cumsum(rng.normal(size=dims), axis=1), 2).astype(dt)
    grid = [(i, j) for i in range(3) for j in range(4)]
    stored = _existing(orc, dims, layout, dt, before, grid)
    bad = "c-" + DSET[2:] + "_1_2"
    blob = bytearray(stored[getS3Key(bad)])
    blob[16:] = bytes(len(blob) - 16)                 # header intact, stream zeroed: decode fails
    stored[getS3Key(bad)] = bytes(blob)
    selection = (slice(10, 192, 1), slice(20, 256, 1))  # every chunk partly covered: all are read
    arr = np.full((182, 236), 7.5, dt)
    plan = crawl.SelectionPlan(DSET, dims, layout, selection, dt, 1)
    store = ChunkStore(lambda k, o, n: stored.get(k), mem_target=64 << 20, device=dev)
    w = crawl.ShardedWriter(plan, 0, store)
    with pytest.raises(HTTPInternalServerError):
        w.write(arr, filter_ops=_ops(dt, layout))
    torch.cuda.synchronize()
    assert bad not in store.cache
    out = {}
    store.flush(lambda k, b: out.__setitem__(k, b), filter_ops=_ops(dt, layout))
    assert getS3Key(bad) not in out and len(out) == len(grid) - 1
    expect = before.copy()
    expect[selection] = 7.5
    cb = int(np.prod(layout)) * dt.itemsize
    for i, j in grid:
        cid = "c-" + DSET[2:] + f"_{i}_{j}"
        if cid == bad:
            continue
        got = np.frombuffer(orc.uncompress(out[getS3Key(cid)], "zlib", 1, 4, cb), dt).reshape(layout)
        assert np.array_equal(got, expect[i * 64:(i + 1) * 64, j * 64:(j + 1) * 64]), cid
