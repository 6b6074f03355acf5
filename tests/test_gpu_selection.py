"""GPU parity of the hyperslab copies: chunkReadSelection / chunkWriteSelection
(chunkUtil.py:882-995) against the reference goldens and numpy slicing, and the
sharded read path (decode -> pack -> place, hsds_amd/crawl.py) against numpy
`full[selection]` with the oracle encoder producing the stored chunks."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def _dec(enc):
    return tuple(slice(*e["slice"]) if "slice" in e else list(e["coords"]) for e in enc)


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


def test_read_write_selection_goldens(selection_golden, dev):
    from hsds_amd.selection import chunkReadSelection, chunkWriteSelection
    rng = np.random.default_rng(99)       # same draw order as tests/golden/make_golden.py
    for rc, wc in zip(selection_golden["readSelection"], selection_golden["writeSelection"]):
        arr = rng.integers(-1000, 1000, size=tuple(rc["shape"])).astype(rc["dtype"])
        sl = _dec(rc["slices"])
        out = chunkReadSelection(arr, slices=sl)
        assert list(out.shape) == rc["out_shape"] and _sha(out.tobytes()) == rc["out_sha256"]
        data = rng.integers(-1000, 1000, size=out.shape).astype(rc["dtype"])
        a2 = arr.copy()
        assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) == wc["updated"]
        assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) == wc["updated_again"]
        assert _sha(a2.tobytes()) == wc["out_sha256"]


@pytest.mark.parametrize("seed", range(6))
def test_random_strided_read_write(seed, dev):
    from hsds_amd.selection import chunkReadSelection, chunkWriteSelection
    rng = np.random.default_rng(seed)
    rank = int(rng.integers(1, 6))
    shape = tuple(int(x) for x in rng.integers(1, 24 if rank > 2 else 300, rank))
    dt = [np.uint8, np.int16, np.float32, np.float64, np.complex64, np.int64][seed % 6]
    arr = (rng.normal(size=shape) * 100).astype(dt)
    sl = []
    for n in shape:
        a = int(rng.integers(0, n))
        b = int(rng.integers(a + 1, n + 1))
        sl.append(slice(a, b, int(rng.integers(1, 5))))
    sl = tuple(sl)
    assert np.array_equal(chunkReadSelection(arr, slices=sl), arr[sl])
    data = (rng.normal(size=arr[sl].shape) * 100).astype(dt)
    a2 = arr.copy()
    ref = arr.copy()
    ref[sl] = data
    assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) == (not np.array_equal(arr[sl], data))
    assert np.array_equal(a2, ref)
    assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) is False


def test_write_selection_nan_is_always_an_update(dev):
    # numpy array_equal: NaN != NaN, so the reference rewrites (and dirties) the chunk
    from hsds_amd.selection import chunkWriteSelection
    arr = np.full((8, 8), np.nan, np.float32)
    data = np.full((2, 2), np.nan, np.float32)
    assert chunkWriteSelection(chunk_arr=arr, slices=(slice(0, 2, 1), slice(0, 2, 1)), data=data) is True


CASES = [
    # (dims, layout, dtype, selection, world)  -- cfg3/cfg4 shapes at test scale
    ((96, 80, 70), (16, 32, 32), np.int16, (slice(0, 96, 2), slice(3, 80, 5), slice(1, 70, 3)), 1),
    ((96, 80, 70), (16, 32, 32), np.int16, (slice(0, 96, 2), slice(3, 80, 5), slice(1, 70, 3)), 4),
    ((300, 260), (128, 128), np.float32, (slice(0, 300, 1), slice(0, 260, 1)), 2),
    ((300, 260), (128, 128), np.float32, (slice(0, 300, 4), slice(0, 260, 4)), 8),
    # the configs' own chunk layouts: cfg3 (16x64x128 int16, its strided selection), cfg4
    # (512x512 f32, [::4, ::4] and a full extent) over 8 ranks, and cfg1's uncompressed 64x64
    ((48, 192, 256), (16, 64, 128), np.int16, (slice(0, 48, 2), slice(3, 192, 5), slice(1, 256, 3)), 8),
    ((1536, 1280), (512, 512), np.float32, (slice(0, 1536, 4), slice(0, 1280, 4)), 8),
    ((1100, 700), (512, 512), np.float32, (slice(0, 1100, 1), slice(0, 700, 1)), 8),
    ((300, 260), (64, 64), np.float32, (slice(10, 290, 1), slice(5, 250, 1)), 3, None),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sharded_read_matches_numpy(case, dev, oracle_lib):
    """Every rank of the plan runs in this process (on cuda:0); the non-root ranks pack
    into their slices of the gathered buffer, the root copies its own pieces straight
    into the slab and then places the peers' -- the same kernels and descriptors the
    multi-GPU run uses around the RCCL exchange."""
    import torch
    from hsds_amd import crawl, selection as sel
    dims, layout, dt, selection, world = CASES[case][:5]
    comp = CASES[case][5] if len(CASES[case]) > 5 else "zlib"
    rng = np.random.default_rng(case)
    full = (np.cumsum(rng.normal(size=dims), axis=-1) * 100).astype(dt)
    plan = crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", dims, layout, selection, dt, world)
    gathered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=dev)
    missing = plan.pieces[0].chunk_id if plan.pieces else None     # one absent object -> fill value
    fill = 7
    sts = []
    for r in range(world):
        blobs = {}
        for cid in plan.chunk_ids(r):
            if cid == missing:
                continue
            idx = sel.getChunkIndex(cid)
            c = np.zeros(layout, dt)
            reg = tuple(slice(i * L, min((i + 1) * L, n)) for i, L, n in zip(idx, layout, dims))
            c[tuple(slice(0, s.stop - s.start) for s in reg)] = full[reg]
            blobs[cid] = oracle_lib.blosc_encode(c.tobytes(), typesize=1, clevel=4, shuffle=1) if comp else c.tobytes()
        rd = crawl.ShardedReader(plan, r, dev, root=0, compressor=comp, shuffle=1 if comp else 0)
        st = rd.upload(blobs, fill_value=fill)
        b = int(plan.rank_base[r])
        if r:
            rd.decode_and_pack(st, gathered[b:b + max(plan.rank_bytes[r], 1)])
            assert st["d_direct"] is None and st["d_place"] is None
        sts.append((rd, st))
    # the root: its own pieces straight into the slab, then the peers' packed pieces
    rd0, st0 = sts[0]
    slab = torch.full((plan.slab_nbytes,), 0, dtype=torch.uint8, device=dev)
    slab.copy_(torch.from_numpy(np.full(plan.slab_shape, fill, dt).view(np.uint8).reshape(-1).copy()).to(dev))
    rd0.decode_and_place(st0, slab)
    assert st0["d_pack"] is None and (world > 1 or st0["d_place"] is None)
    if st0["d_place"] is not None:
        rd0.eng.copy(gathered, slab, st0["d_place"])
    for _, st in sts:
        if st["n"]:
            assert int(st["d_status"][:st["n"]].abs().sum()) == 0
    got = slab.cpu().numpy().view(dt).reshape(plan.slab_shape)
    expect = full[selection].copy()
    if missing is not None:
        # the missing chunk's piece reads as the fill value
        p = plan.pieces[0]
        expect[p.data_slices] = fill
    assert np.array_equal(got, expect)


@pytest.mark.parametrize("case", [0, 2, 7])
def test_single_rank_read(case, dev, oracle_lib):
    """ShardedReader.read at world size 1: decode + one direct copy per piece into a
    fill-valued slab (a missing chunk reads as the fill value)."""
    from hsds_amd import crawl, selection as sel
    dims, layout, dt, selection = CASES[case][:4]
    comp = CASES[case][5] if len(CASES[case]) > 5 else "zlib"
    rng = np.random.default_rng(100 + case)
    full = (np.cumsum(rng.normal(size=dims), axis=-1) * 100).astype(dt)
    plan = crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", dims, layout, selection, dt, 1)
    missing = plan.pieces[-1].chunk_id
    blobs = {}
    for cid in plan.chunk_ids(0):
        if cid == missing:
            continue
        idx = sel.getChunkIndex(cid)
        c = np.zeros(layout, dt)
        reg = tuple(slice(i * L, min((i + 1) * L, n)) for i, L, n in zip(idx, layout, dims))
        c[tuple(slice(0, s.stop - s.start) for s in reg)] = full[reg]
        blobs[cid] = oracle_lib.blosc_encode(c.tobytes(), typesize=1, clevel=4, shuffle=1) if comp else c.tobytes()
    rd = crawl.ShardedReader(plan, 0, dev, compressor=comp, shuffle=1 if comp else 0)
    st = rd.upload(blobs, fill_value=3)
    got = rd.read(st, fill_value=3).cpu().numpy()[:plan.slab_nbytes].view(dt).reshape(plan.slab_shape)
    expect = full[selection].copy()
    expect[plan.pieces[-1].data_slices] = 3
    assert np.array_equal(got, expect)
