"""GPU parity of the batched DN read path (hsds_amd.datanode) against the reference's
own getHyperChunks / getStorBytes outputs (tests/golden/rangeget_cases.*) and the
CPU oracle: hyper-chunk assembly (H5D_CHUNKED_REF_INDIRECT), plain F1/F2 objects,
CONTIGUOUS_REF zero extension, the HBM chunk cache, missing objects and chunk_init.
Bit-exact."""
import json
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def rg():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "rangeget_cases.json")))
    a = np.load(os.path.join(ROOT, "tests", "golden", "rangeget_cases.npz"))
    return d, a


def _ops(fo):
    if fo is None:
        return None
    return {k: (np.dtype(v) if k == "dtype" else v) for k, v in fo.items()}


def test_hyper_chunks_match_reference_getHyperChunks(dev, rg):
    from hsds_amd.datanode import ChunkRead, ChunkReader, getHyperChunkFactors, getHyperChunkIndex
    meta, arrs = rg
    for case in meta["hyper"]:
        file_np = arrs[case["name"] + "__file"]
        want = arrs[case["name"] + "__chunk"]
        reads = []

        def fetch(key, offset, length, f=file_np):
            return f[offset:offset + length].tobytes()

        f = getHyperChunkFactors(case["chunk_dims"], case["hyper_dims"])
        by_idx = {tuple(x[0]): (x[1], x[2]) for x in case["locs"]}
        offs, lens = [], []
        for i in range(int(np.prod(f))):
            o, n = by_idx.get(getHyperChunkIndex(i, f), (0, 0))
            offs.append(o)
            lens.append(n)
        reads.append(ChunkRead("c-x_0", "file.h5", offs, lens))
        r = ChunkReader(fetch, device=dev)
        out = r.read(reads, case["dtype"], case["chunk_dims"], filter_ops=_ops(case["filter_ops"]),
                     hyper_dims=case["hyper_dims"])
        got = out[0]
        assert not isinstance(got, Exception), (case["name"], got)
        assert got.cpu().numpy().tobytes() == want.tobytes(), case["name"]
        assert r.stats["decode_calls"] == 1                    # one batch for all hyper chunks


def test_hyper_chunk_fill_value_and_corruption(dev, rg):
    from hsds_amd.codec import HTTPInternalServerError
    from hsds_amd.datanode import ChunkRead, ChunkReader, getHyperChunkFactors, getHyperChunkIndex
    meta, arrs = rg
    case = [c for c in meta["hyper"] if c["name"] == "h_i16_deflate_missing"][0]
    file_np = arrs[case["name"] + "__file"].copy()
    want = arrs[case["name"] + "__chunk"].copy()
    f = getHyperChunkFactors(case["chunk_dims"], case["hyper_dims"])
    by_idx = {tuple(x[0]): (x[1], x[2]) for x in case["locs"]}
    offs, lens = [], []
    for i in range(int(np.prod(f))):
        o, n = by_idx.get(getHyperChunkIndex(i, f), (0, 0))
        offs.append(o)
        lens.append(n)
    # missing hyper chunks keep the fill value instead of zeros
    hd = case["hyper_dims"]
    for i in range(int(np.prod(f))):
        idx = getHyperChunkIndex(i, f)
        if idx not in by_idx:
            sl = tuple(slice(idx[k] * hd[k], (idx[k] + 1) * hd[k]) for k in range(len(hd)))
            want[sl] = -7
    r = ChunkReader(lambda k, o, n: file_np[o:o + n].tobytes(), device=dev)
    out = r.read([ChunkRead("c", "f", offs, lens)], case["dtype"], case["chunk_dims"],
                 filter_ops=_ops(case["filter_ops"]), fill_value=-7, hyper_dims=hd)
    assert out[0].cpu().numpy().tobytes() == want.tobytes()
    # a corrupt HDF5 chunk fails the whole HSDS chunk (500), like getHyperChunks' _uncompress
    bad = file_np.copy()
    o0 = next(o for o, n in zip(offs, lens) if n)
    bad[o0 + 2:o0 + 40] ^= 0x5A
    r2 = ChunkReader(lambda k, o, n: bad[o:o + n].tobytes(), device=dev)
    out2 = r2.read([ChunkRead("c", "f", offs, lens)], case["dtype"], case["chunk_dims"],
                   filter_ops=_ops(case["filter_ops"]), hyper_dims=hd)
    assert isinstance(out2[0], HTTPInternalServerError)
    # malformed requests are ValueErrors (HTTPBadRequest in the reference)
    out3 = r.read([ChunkRead("c", "f", offs[:-1], lens[:-1])], case["dtype"], case["chunk_dims"],
                  filter_ops=_ops(case["filter_ops"]), hyper_dims=hd)
    assert isinstance(out3[0], ValueError)


def test_plain_objects_cache_and_missing(dev, oracle_lib):
    import torch
    from hsds_amd.datanode import ChunkRead, ChunkStore, H5D_CONTIGUOUS_REF
    orc = oracle_lib
    rng = np.random.default_rng(3)
    dims = (128, 256)
    store = {}
    want = {}
    for i in range(24):
        a = np.round(np.cumsum(rng.normal(size=dims[0] * dims[1])), 2).astype(np.float32).reshape(dims)
        cid = f"c-d_{i}_0"
        if i % 3 == 0:
            store[cid] = orc.blosc_encode(a.tobytes(), typesize=1, clevel=4, shuffle=1)    # F1
        elif i % 3 == 1:
            store[cid] = zlib.compress(orc.shuffle(a.tobytes(), 4), 5)                    # F2
        else:
            store[cid] = orc.blosc_encode(a.tobytes(), typesize=4, clevel=5, shuffle=1)    # ts=4 frame
        want[cid] = a
    fetched = []

    def fetch(key, offset, length):
        fetched.append(key)
        return store.get(key)

    ops = {"compressor": "zlib", "shuffle": 1, "level": 5, "dtype": np.dtype("<f4")}
    cs = ChunkStore(fetch, mem_target=12 * dims[0] * dims[1] * 4, device=dev)
    ids = list(store)[:16]
    reads = [ChunkRead(c, c) for c in ids] + [ChunkRead(ids[0], ids[0])]    # duplicate read once
    res = cs.get_chunks(reads, "<f4", dims, filter_ops=ops)
    for c, r in zip([r.chunk_id for r in reads], res):
        assert np.array_equal(r.cpu().numpy(), want[c]), c
    assert len(fetched) == 16
    assert cs.cache.memUsed <= cs.cache.memTarget
    # hits are served from HBM without a storage read
    n0 = len(fetched)
    last = ids[-4:]
    res2 = cs.get_chunks([ChunkRead(c, c) for c in last], "<f4", dims, filter_ops=ops)
    assert len(fetched) == n0 and cs.reader.stats["cache_hits"] >= 4
    assert all(np.array_equal(r.cpu().numpy(), want[c]) for c, r in zip(last, res2))
    # missing object: None (404), or a fill-value chunk with chunk_init
    res3 = cs.get_chunks([ChunkRead("c-d_99_0", "nope")], "<f4", dims, filter_ops=ops)
    assert res3[0] is None
    res4 = cs.get_chunks([ChunkRead("c-d_98_0", "nope")], "<f4", dims, filter_ops=ops, fill_value=2.5,
                         chunk_init=True)
    assert torch.all(res4[0] == 2.5)
    # H5D_CONTIGUOUS_REF: a short read near the end of the file is zero-extended
    raw = want[ids[1]].tobytes()
    short = raw[:len(raw) - 1000]
    cs2 = ChunkStore(lambda k, o, n: short, mem_target=1 << 24, device=dev)
    r = cs2.get_chunks([ChunkRead("c-ref", "file")], "<f4", dims, layout_class=H5D_CONTIGUOUS_REF)
    exp = np.frombuffer(short + bytes(1000), np.float32).reshape(dims)
    assert np.array_equal(r[0].cpu().numpy(), exp)


def test_getstorbytes_chunk_locations_skip_mismatch(dev, rg):
    # getStorBytes with chunk_locations decodes every location and skips those whose
    # size is not h5_size (storUtil.py:486-516): the same decode batch, kept statuses
    from hsds_amd.datanode import ChunkRead, ChunkReader
    meta, arrs = rg
    sb = meta["storbytes"]
    body = arrs["sb__file"]
    base = sb["base"]
    locs = sb["locs"]
    want = [arrs[f"sb__out{k}"].tobytes() for k in range(sb["n_out"])]
    r = ChunkReader(lambda k, o, n: body[o - base:o - base + n].tobytes(), device=dev)
    got = r.get_stor_bytes("f", [(tuple(x[0]), x[1], x[2]) for x in locs], sb["h5_size"], _ops(sb["filter_ops"]))
    assert got == want


def test_put_selections_and_flush(dev, oracle_lib):
    """PUT_Chunk + s3sync, batched: chunkWriteSelection semantics (no change -> not
    dirty, NaN always an update), missing chunks start from the fill value, the
    flush encodes every dirty chunk in one batch from HBM, and the stored objects
    decode (oracle: c-blosc frame walk + libz) to numpy's result of the same writes."""
    from hsds_amd.datanode import ChunkRead, ChunkStore
    from hsds_amd.filters import getFilterOps
    orc = oracle_lib
    dims = (64, 96)
    dt = np.dtype("<f4")
    rng = np.random.default_rng(11)
    ops = getFilterOps({"filter_map": {}}, "d-w", [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                                                   {"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": 4}],
                       dtype=dt, chunk_shape=dims)
    truth, store = {}, {}
    for i in range(3):
        a = np.round(np.cumsum(rng.normal(size=dims[0] * dims[1])), 2).astype(dt).reshape(dims)
        truth[f"c-w_{i}_0"] = a
        store[f"k{i}"] = orc.blosc_encode(a.tobytes(), typesize=1, clevel=4, shuffle=1)
    keys = {f"c-w_{i}_0": f"k{i}" for i in range(5)}
    cs = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    s1 = (slice(3, 40, 2), slice(10, 90, 7))
    d1 = rng.normal(size=(len(range(3, 40, 2)), len(range(10, 90, 7)))).astype(dt)
    s2 = (slice(0, 64, 1), slice(0, 96, 1))
    s3 = (slice(5, 9, 1), slice(0, 4, 1))
    d3 = np.full((4, 4), np.nan, dt)
    writes = [(ChunkRead("c-w_0_0", "k0"), s1, d1),                          # changes
              (ChunkRead("c-w_1_0", "k1"), s2, truth["c-w_1_0"].copy()),     # identical: not dirty
              (ChunkRead("c-w_3_0", "k3"), s1, d1),                          # missing -> fill, changes
              (ChunkRead("c-w_2_0", "k2"), s3, d3),                          # NaN: always an update
              (ChunkRead("c-w_2_0", "k2"), s3, d3)]                          # again (next round)
    dirty = cs.put_selections(writes, dt, dims, filter_ops=ops, fill_value=1.5)
    assert dirty == [True, False, True, True, True]
    want = {k: v.copy() for k, v in truth.items()}
    want["c-w_0_0"][s1] = d1
    want["c-w_3_0"] = np.full(dims, 1.5, dt)
    want["c-w_3_0"][s1] = d1
    want["c-w_2_0"][s3] = d3
    flushed = {}
    ids = cs.flush(lambda k, b: flushed.__setitem__(k, b), filter_ops=ops, keys=keys)
    assert sorted(ids) == ["c-w_0_0", "c-w_2_0", "c-w_3_0"]
    assert cs.cache.dirtyCount == 0
    for cid in ids:
        got = orc.uncompress(flushed[keys[cid]], "zlib", 1, 4, dims[0] * dims[1] * 4)
        assert np.frombuffer(got, dt).reshape(dims).tobytes() == want[cid].tobytes(), cid
    # the flushed objects read back through the GPU path
    store.update(flushed)
    cs2 = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    res = cs2.get_chunks([ChunkRead(c, keys[c]) for c in ids], dt, dims, filter_ops=ops)
    for cid, r in zip(ids, res):
        assert r.cpu().numpy().tobytes() == want[cid].tobytes()


def test_put_and_flush_lz4_dataset(dev, oracle_lib):
    """An lz4-filtered dataset (getFilterOps -> compressor "lz4"): PUT_Chunk on stored
    Blosc-lz4 objects, flush through the GPU lz4 encoder, objects decode through the
    oracle (frame walk + LZ4) and read back through the GPU LZ4 decoder."""
    from hsds_amd.datanode import ChunkRead, ChunkStore
    from hsds_amd.filters import getFilterOps
    orc = oracle_lib
    dims = (128, 256)
    dt = np.dtype("<i4")
    rng = np.random.default_rng(12)
    ops = getFilterOps({"filter_map": {}}, "d-l", [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                                                   {"class": "H5Z_FILTER_LZ4", "id": 32004, "name": "lz4"}],
                       dtype=dt, chunk_shape=dims)
    assert ops["compressor"] == "lz4" and ops["level"] == 5
    truth, store = {}, {}
    for i in range(4):
        a = (np.cumsum(rng.normal(size=dims[0] * dims[1])) * 10).astype(dt).reshape(dims)
        truth[f"c-l_{i}_0"] = a
        store[f"k{i}"] = orc.blosc_encode_lz4(a.tobytes(), typesize=1, blocksize=131072, shuffle=1)
    keys = {f"c-l_{i}_0": f"k{i}" for i in range(4)}
    cs = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    sel = (slice(7, 120, 3), slice(0, 256, 5))
    d = rng.integers(-1000, 1000, size=(len(range(7, 120, 3)), len(range(0, 256, 5)))).astype(dt)
    writes = [(ChunkRead(f"c-l_{i}_0", f"k{i}"), sel, d) for i in (0, 2, 3)]
    assert cs.put_selections(writes, dt, dims, filter_ops=ops) == [True, True, True]
    flushed = {}
    ids = cs.flush(lambda k, b: flushed.__setitem__(k, b), filter_ops=ops, keys=keys)
    assert sorted(ids) == ["c-l_0_0", "c-l_2_0", "c-l_3_0"]
    for cid in ids:
        f = flushed[keys[cid]]
        assert f[2] >> 5 == 1                      # Blosc codec 1: lz4
        want = truth[cid].copy()
        want[sel] = d
        got = orc.uncompress(f, "lz4", 1, 4, want.nbytes)
        assert got == want.tobytes(), cid
    store.update(flushed)
    cs2 = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    res = cs2.get_chunks([ChunkRead(c, keys[c]) for c in sorted(keys)], dt, dims, filter_ops=ops)
    for cid, r in zip(sorted(keys), res):
        want = truth[cid].copy()
        if cid in ids:
            want[sel] = d
        assert r.cpu().numpy().tobytes() == want.tobytes(), cid


@pytest.mark.parametrize("with_deflate", [False, True])
def test_put_and_flush_bitshuffle_dataset(dev, oracle_lib, with_deflate):
    """A bitshuffle dataset (getFilterOps -> shuffle 2): PUT_Chunk into fill-initialised
    chunks, flush through ONE bitshuffle encode batch (and the Blosc zlib wrap when the
    dataset also has deflate, storUtil.py:243-262); the objects decode through the
    oracle, bare objects read back through the batched GPU reader, wrapped ones
    through codec._uncompress."""
    from hsds_amd import codec
    from hsds_amd.datanode import ChunkRead, ChunkStore
    from hsds_amd.filters import getFilterOps
    orc = oracle_lib
    dims = (64, 200)
    dt = np.dtype("<f4")
    filters = [{"class": "H5Z_FILTER_BITSHUFFLE", "id": 32008, "name": "bitshuffle"}]
    if with_deflate:
        filters.append({"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": 4})
    ops = getFilterOps({"filter_map": {}}, "d-b", filters, dtype=dt, chunk_shape=dims)
    assert ops["shuffle"] == 2
    rng = np.random.default_rng(21)
    cs = ChunkStore(lambda k, o, n: None, mem_target=1 << 24, device=dev)
    sel = (slice(0, 64), slice(3, 200, 2))
    writes, truth = [], {}
    for i in range(3):
        d = np.round(np.cumsum(rng.normal(size=(64, len(range(3, 200, 2)))), axis=1), 2).astype(dt)
        writes.append((ChunkRead(f"c-b_{i}_0", f"k{i}"), sel, d))
        w = np.zeros(dims, dt)
        w[sel] = d
        truth[f"c-b_{i}_0"] = w
    cs.put_selections(writes, dt, dims, filter_ops=ops)
    flushed = {}
    keys = {f"c-b_{i}_0": f"k{i}" for i in range(3)}
    ids = cs.flush(lambda k, b: flushed.__setitem__(k, b), filter_ops=ops, keys=keys)
    assert sorted(ids) == sorted(keys)
    for cid in ids:
        f = flushed[keys[cid]]
        want = truth[cid].tobytes()
        obj = orc.blosc_decode(f, len(f) * 64) if with_deflate else f
        if with_deflate:
            assert f[2] >> 5 == 3 and not (f[2] & 1)        # Blosc zlib, shuffle off
        assert bytes(orc.bitshuffle_decode(obj, len(want), 4)) == want, cid
        assert codec._uncompress(f, compressor=ops.get("compressor"), shuffle=2, dtype=dt,
                                 chunk_shape=dims) == want
    # batched read-back: one bitshuffle decode launch, or two (outer Blosc, then
    # bitshuffle) when the dataset also has deflate; a corrupted object fails alone
    store = dict(flushed)
    bad = bytearray(store["k1"])
    if with_deflate:
        bad[4:8] = (0x7FFFFFF0).to_bytes(4, "little")   # Blosc nbytes past any chunk's object
    else:
        bad[12:16] = (0x7FFFFF00).to_bytes(4, "big")    # first LZ4 block size past the object
    store["k1"] = bytes(bad)
    cs2 = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    res = cs2.get_chunks([ChunkRead(c, keys[c]) for c in sorted(keys)], dt, dims, filter_ops=ops)
    for cid, r in zip(sorted(keys), res):
        if keys[cid] == "k1":
            assert isinstance(r, codec.HTTPInternalServerError), r
            continue
        assert r.cpu().numpy().tobytes() == truth[cid].tobytes(), cid


def test_bitshuffle_deflate_batch_fails_per_chunk(dev, oracle_lib):
    """bitshuffle + deflate dataset read in one batch with objects the reference judges one
    by one (storUtil._uncompress, storUtil.py:189-227): Blosc-wrapped (decoded), a bare
    zlib stream around the bitshuffle object (zlib.decompress path, decoded), a zero-filled
    short read (storUtil.py:480-485), a truncated frame and a frame with an oversized
    nbytes (500 for that chunk only)."""
    import torch
    from hsds_amd import codec
    from hsds_amd.datanode import ChunkRead, ChunkStore
    from hsds_amd.filters import getFilterOps
    orc = oracle_lib
    dims, dt = (32, 100), np.dtype("<i4")
    filters = [{"class": "H5Z_FILTER_BITSHUFFLE", "id": 32008, "name": "bitshuffle"},
               {"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": 4}]
    ops = getFilterOps({"filter_map": {}}, "d-c", filters, dtype=dt, chunk_shape=dims)
    rng = np.random.default_rng(4)
    truth, store = {}, {}
    for i in range(6):
        a = (np.cumsum(rng.integers(-50, 50, size=dims), axis=1)).astype(dt)
        truth[f"k{i}"] = a.tobytes()
        obj = codec._compress(a.tobytes(), compressor=None, shuffle=2, dtype=dt, chunk_shape=dims)
        store[f"k{i}"] = codec._compress(obj, compressor="deflate", level=4) if i != 1 else zlib.compress(obj, 6)
        assert bytes(orc.bitshuffle_decode(obj, a.nbytes, 4)) == a.tobytes()
    store["k2"] = store["k2"][:len(store["k2"]) // 2]                # truncated Blosc frame
    big = bytearray(store["k3"])
    big[4:8] = (0xFFFFFF00).to_bytes(4, "little")                     # nbytes ~4 GiB
    store["k3"] = bytes(big)
    reads = [ChunkRead(f"c-c_{i}", f"k{i}") for i in range(6)]
    reads[4] = ChunkRead("c-c_4", "k4", offset=0, length=len(store["k4"]) + 10)   # short read: zeros
    fetch = lambda k, o, n: store.get(k) if not n else store[k][o:o + n]
    cs = ChunkStore(fetch, mem_target=1 << 24, device=dev)
    res = cs.get_chunks(reads, dt, dims, filter_ops=ops)
    torch.cuda.synchronize()
    for i, r in enumerate(res):
        if i in (2, 3, 4):
            assert isinstance(r, codec.HTTPInternalServerError), (i, r)
        else:
            assert r.cpu().numpy().tobytes() == truth[f"k{i}"], i


def test_put_and_flush_zstd_dataset(dev, oracle_lib):
    """A zstd-filtered dataset (H5Z_FILTER_ZSTD 32015): PUT_Chunk on stored Blosc-zstd
    objects (written by libblosc, as the reference would), flush through the GPU zstd
    writer; the objects decode through the oracle and read back through the GPU."""
    import ctypes
    import os
    from hsds_amd.datanode import ChunkRead, ChunkStore
    from hsds_amd.filters import getFilterOps
    p = "/opt/conda/lib/libblosc.so.1"
    if not os.path.exists(p):
        pytest.skip("libblosc absent")
    lb = ctypes.CDLL(p)
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    orc = oracle_lib
    dims = (128, 256)
    dt = np.dtype("<f4")
    rng = np.random.default_rng(13)
    ops = getFilterOps({"filter_map": {}}, "d-z", [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                                                   {"class": "H5Z_FILTER_ZSTD", "id": 32015, "name": "zstd"}],
                       dtype=dt, chunk_shape=dims)
    assert ops["compressor"] == "zstd"
    truth, store = {}, {}
    for i in range(4):
        a = np.round(np.cumsum(rng.normal(size=dims[0] * dims[1])), 2).astype(dt).reshape(dims)
        truth[f"c-z_{i}_0"] = a
        out = np.empty(a.nbytes + 64, np.uint8)
        k = lb.blosc_compress_ctx(ops["level"], 1, 1, a.nbytes, a.ctypes.data, out.ctypes.data, out.size, b"zstd", 0, 1)
        store[f"k{i}"] = out[:k].tobytes()
    keys = {f"c-z_{i}_0": f"k{i}" for i in range(4)}
    cs = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    sel = (slice(3, 128, 2), slice(10, 250, 7))
    d = np.round(rng.normal(size=(len(range(3, 128, 2)), len(range(10, 250, 7)))), 3).astype(dt)
    writes = [(ChunkRead(f"c-z_{i}_0", f"k{i}"), sel, d) for i in (1, 3)]
    assert cs.put_selections(writes, dt, dims, filter_ops=ops) == [True, True]
    flushed = {}
    ids = cs.flush(lambda k, b: flushed.__setitem__(k, b), filter_ops=ops, keys=keys)
    assert sorted(ids) == ["c-z_1_0", "c-z_3_0"]
    for cid in ids:
        f = flushed[keys[cid]]
        assert f[2] >> 5 == 4                      # Blosc codec 4: zstd
        want = truth[cid].copy()
        want[sel] = d
        assert orc.uncompress(f, "zstd", 1, 4, want.nbytes) == want.tobytes(), cid
    store.update(flushed)
    cs2 = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
    res = cs2.get_chunks([ChunkRead(c, keys[c]) for c in sorted(keys)], dt, dims, filter_ops=ops)
    for cid, r in zip(sorted(keys), res):
        want = truth[cid].copy()
        if cid in ids:
            want[sel] = d
        assert r.cpu().numpy().tobytes() == want.tobytes(), cid


@pytest.mark.parametrize("n,size", [(1, 100), (7, 3000), (300, 70_000)])
def test_stage_upload_objects(dev, n, size):
    """hsds_stage_upload (native threads copy a batch's objects into page-locked staging,
    pieces go up as they are staged): bytes, numpy and empty objects land at their 256-byte
    aligned offsets of the device buffer, bit-exact; a 300-object batch of ~21 MB takes the
    threaded path"""
    import torch
    from hsds_amd.datanode import _stage_blobs
    rng = np.random.default_rng(n)
    blobs = []
    for k in range(n):
        m = int(rng.integers(0, size))
        b = rng.integers(0, 256, m, dtype=np.uint8)
        blobs.append(b.tobytes() if k % 3 else (b if k % 2 else b.tobytes()))
    if n > 1:
        blobs[1] = b""
    d_src, descs, _ = _stage_blobs(blobs, [size] * n, dev)
    host = d_src.cpu().numpy()
    torch.cuda.synchronize()
    for k, b in enumerate(blobs):
        o, ln = int(descs[k]["src_off"]), int(descs[k]["src_len"])
        assert ln == len(b) and o % 256 == 0
        assert host[o:o + ln].tobytes() == (b.tobytes() if isinstance(b, np.ndarray) else b)
