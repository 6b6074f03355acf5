"""DN micro-batcher on the GPU (hsds_amd.batcher over a real ChunkStore): 64 concurrent
GET_Chunk-style requests with strided selections become one decode batch (one decode
launch) and one selection gather; every response equals numpy's chunk_arr[slices] of the
oracle-encoded chunk (HSDS F1 objects, storUtil._compress layout), bit for bit."""
import asyncio

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batched_get_selection_matches_numpy(oracle_lib):
    import torch
    from hsds_amd.batcher import ChunkBatcher
    from hsds_amd.datanode import ChunkRead, ChunkStore
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    orc = oracle_lib
    dims = (64, 96)
    rng = np.random.default_rng(5)
    truth, objs = {}, {}
    for i in range(40):
        a = np.round(np.cumsum(rng.normal(size=dims[0] * dims[1])), 2).astype("<f4").reshape(dims)
        truth[f"c-b_{i}_0"] = a
        objs[f"k{i}"] = orc.blosc_encode(a.tobytes(), typesize=1, clevel=4, shuffle=1)
    fetched = []

    def fetch(key, offset, length):
        fetched.append(key)
        return objs.get(key)

    cs = ChunkStore(fetch, mem_target=1 << 26, device=dev)
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    b = ChunkBatcher(cs, window_ms=50)
    sels = [(slice(0, 64, 1), slice(0, 96, 1)), (slice(3, 61, 4), slice(1, 96, 5)), (slice(10, 11, 1), slice(0, 96, 2))]

    async def main():
        reqs = []
        for j in range(64):
            i = j % 40 if j < 60 else 45                   # 4 requests for an object that does not exist
            reqs.append(b.get_selection(ChunkRead(f"c-b_{i}_0", f"k{i}"), "<f4", dims, sels[j % 3], filter_ops=ops))
        return await asyncio.gather(*reqs)

    res = asyncio.run(main())
    assert b.stats["batches"] == 1 and b.stats["requests"] == 64 and b.stats["reads"] == 41
    assert len(fetched) == 41
    for j, r in enumerate(res):
        i = j % 40 if j < 60 else 45
        if i == 45:
            assert r is None
        else:
            np.testing.assert_array_equal(r, truth[f"c-b_{i}_0"][sels[j % 3]])


def _objs(orc, n, dims, seed):
    rng = np.random.default_rng(seed)
    truth, objs = {}, {}
    for i in range(n):
        a = np.round(np.cumsum(rng.normal(size=dims[0] * dims[1])), 2).astype("<f4").reshape(dims)
        truth[f"c-b_{i}_0"] = a
        objs[f"k{i}"] = orc.blosc_encode(a.tobytes(), typesize=1, clevel=4, shuffle=1)
    return truth, objs


def test_batch_larger_than_cache(oracle_lib):
    """misses the cache has no room for land in a per-batch buffer, not in the
    arena; the gather must read them from that buffer (one copy launch per source)"""
    import torch
    from hsds_amd.batcher import ChunkBatcher
    from hsds_amd.datanode import ChunkRead, ChunkStore
    dev = torch.device("cuda", 0)
    dims = (64, 96)
    truth, objs = _objs(oracle_lib, 48, dims, 11)
    chunk_bytes = dims[0] * dims[1] * 4
    cs = ChunkStore(lambda key, off, ln: objs.get(key), mem_target=5 * chunk_bytes, device=dev)
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    b = ChunkBatcher(cs, window_ms=50)
    sels = [None, (slice(3, 61, 4), slice(1, 96, 5))]

    async def main():
        return await asyncio.gather(*[b.get_selection(ChunkRead(f"c-b_{j % 48}_0", f"k{j % 48}"), "<f4", dims,
                                                      sels[j % 2], filter_ops=ops) for j in range(96)])

    res = asyncio.run(main())
    assert b.stats["batches"] == 1 and b.stats["reads"] == 48
    assert len(cs.cache) <= 6
    for j, r in enumerate(res):
        t = truth[f"c-b_{j % 48}_0"]
        np.testing.assert_array_equal(r, t if sels[j % 2] is None else t[sels[j % 2]])


def test_hits_stay_pinned_while_misses_reserve(oracle_lib):
    """cache hits of a batch are pinned until it completes, so the misses' slot
    reservations (which evict clean LRU nodes) cannot reuse a hit's slot mid-batch"""
    import torch
    from hsds_amd.batcher import ChunkBatcher
    from hsds_amd.datanode import ChunkRead, ChunkStore
    dev = torch.device("cuda", 0)
    dims = (64, 96)
    truth, objs = _objs(oracle_lib, 30, dims, 12)
    chunk_bytes = dims[0] * dims[1] * 4
    cs = ChunkStore(lambda key, off, ln: objs.get(key), mem_target=12 * chunk_bytes, device=dev)
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    warm = cs.get_chunks([ChunkRead(f"c-b_{i}_0", f"k{i}") for i in range(10)], "<f4", dims, filter_ops=ops)
    assert all(v is not None for v in warm) and len(cs.cache) == 10
    b = ChunkBatcher(cs, window_ms=50)

    async def main():
        return await asyncio.gather(*[b.get_chunk(ChunkRead(f"c-b_{i}_0", f"k{i}"), "<f4", dims, filter_ops=ops)
                                      for i in range(30)])

    res = asyncio.run(main())
    for i, r in enumerate(res):
        np.testing.assert_array_equal(r, truth[f"c-b_{i}_0"])
    assert all(n.pinned == 0 for n in cs.cache._lru.values())



def test_failed_batch_releases_every_pin(oracle_lib, monkeypatch):
    """a batch that fails between get_chunks_deferred and finish() (here: the
    selection gather launch, then the reader's placement copy) must not leave slots pinned
    -- pinned slots are never evicted.  The requests get the exception; afterwards every
    node has pinned == 0 and the store still serves reads."""
    import torch
    import hsds_amd.batcher as hb
    from hsds_amd.batcher import ChunkBatcher
    from hsds_amd.datanode import ChunkRead, ChunkStore
    dev = torch.device("cuda", 0)
    dims = (64, 96)
    truth, objs = _objs(oracle_lib, 24, dims, 13)
    chunk_bytes = dims[0] * dims[1] * 4
    cs = ChunkStore(lambda key, off, ln: objs.get(key), mem_target=32 * chunk_bytes, device=dev)
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    cs.get_chunks([ChunkRead(f"c-b_{i}_0", f"k{i}") for i in range(8)], "<f4", dims, filter_ops=ops)   # hits
    b = ChunkBatcher(cs, window_ms=50)

    def boom(*a, **k):
        raise RuntimeError("injected gather failure")

    async def main():
        return await asyncio.gather(*[b.get_chunk(ChunkRead(f"c-b_{i}_0", f"k{i}"), "<f4", dims, filter_ops=ops)
                                      for i in range(16)], return_exceptions=True)

    monkeypatch.setattr(hb, "_gather_launch", boom)
    res = asyncio.run(main())
    assert all(isinstance(r, RuntimeError) for r in res)
    assert all(n.pinned == 0 for n in cs.cache._lru.values())
    monkeypatch.undo()
    # the reader's own device half failing after its slots are reserved
    real_copy = cs.reader.eng.copy

    def copy_boom(*a, **k):
        raise RuntimeError("injected placement failure")

    cs.reader.eng.copy = copy_boom
    with pytest.raises(RuntimeError):
        cs.get_chunks([ChunkRead(f"c-b_{i}_0", f"k{i}") for i in range(4, 20)], "<f4", dims, filter_ops=ops)
    assert all(n.pinned == 0 for n in cs.cache._lru.values())
    cs.reader.eng.copy = real_copy
    vals = cs.get_chunks([ChunkRead(f"c-b_{i}_0", f"k{i}") for i in range(24)], "<f4", dims, filter_ops=ops)
    for i, v in enumerate(vals):
        np.testing.assert_array_equal(v.cpu().numpy(), truth[f"c-b_{i}_0"])
    assert all(n.pinned == 0 for n in cs.cache._lru.values())


def test_small_responses_do_not_pin_the_batch_buffer(oracle_lib):
    """responses are views of one page-locked buffer per batch; a small one (at
    most COPY_OUT_MAX bytes, under 1/COPY_OUT_FRACTION of it) is copied out, so keeping it
    does not keep the whole buffer.  A full-chunk response among 64 is a view (zero copy);
    the small selections own their bytes."""
    import torch
    from hsds_amd.batcher import ChunkBatcher, COPY_OUT_FRACTION
    from hsds_amd.datanode import ChunkRead, ChunkStore
    dev = torch.device("cuda", 0)
    dims = (64, 96)
    truth, objs = _objs(oracle_lib, 8, dims, 14)
    cs = ChunkStore(lambda key, off, ln: objs.get(key), mem_target=1 << 26, device=dev)
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    b = ChunkBatcher(cs, window_ms=50)
    sels = [None] + [(slice(j, j + 1, 1), slice(0, 96, 1)) for j in range(63)]

    async def main():
        return await asyncio.gather(*[b.get_selection(ChunkRead(f"c-b_{j % 8}_0", f"k{j % 8}"), "<f4", dims,
                                                      sels[j], filter_ops=ops) for j in range(64)])

    res = asyncio.run(main())
    assert b.stats["batches"] == 1 and b.stats["host_bytes"] > 0
    full = res[0]
    assert full.base is not None                              # the whole chunk: a view
    for j in range(1, 64):
        np.testing.assert_array_equal(res[j], truth[f"c-b_{j % 8}_0"][sels[j]])
        assert res[j].nbytes * COPY_OUT_FRACTION < b.stats["host_bytes"]
        assert res[j].base is None or res[j].base.nbytes == res[j].nbytes     # owns its bytes
    assert b.stats["copied_out"] == 63
