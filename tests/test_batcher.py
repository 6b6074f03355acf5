"""DN micro-batcher (hsds_amd.batcher) on CPU with a fake store: 64
concurrent GET_Chunk-style coroutines become ONE get_chunks batch, duplicate chunk ids are
read once (datanode_lib.py:1041-1065 pending_s3_read), parameter groups stay apart, 404s
and per-chunk errors reach only their own requests, and selections equal numpy's
chunk_arr[slices] (chunkUtil.py:882-929)."""
import asyncio

import numpy as np
import pytest

from hsds_amd.batcher import ChunkBatcher
from hsds_amd.datanode import ChunkRead


class FakeStore:
    def __init__(self, chunks, errors=()):
        self.chunks, self.errors, self.calls = chunks, set(errors), []

    def get_chunks(self, reads, dtype, chunk_dims, filter_ops=None, fill_value=None, layout_class=None,
                   hyper_dims=None, chunk_init=False):
        self.calls.append([r.chunk_id for r in reads])
        out = []
        for r in reads:
            if r.chunk_id in self.errors:
                out.append(RuntimeError(f"500 {r.chunk_id}"))
            elif r.chunk_id in self.chunks:
                out.append(self.chunks[r.chunk_id])
            elif chunk_init:
                out.append(np.full(chunk_dims, fill_value or 0, dtype))
            else:
                out.append(None)
        return out


def _chunks(n, dims=(8, 16)):
    rng = np.random.default_rng(0)
    return {f"c-{i}": rng.normal(size=dims).astype(np.float32) for i in range(n)}


def test_64_concurrent_requests_one_batch():
    chunks = _chunks(48)
    store = FakeStore(chunks)
    b = ChunkBatcher(store, window_ms=20)
    sel = (slice(1, 7, 2), slice(0, 16, 3))

    async def main():
        reqs = [ChunkRead(f"c-{i % 48}", f"k{i % 48}") for i in range(64)]      # 16 duplicates
        return await asyncio.gather(*[b.get_selection(r, np.float32, (8, 16), sel) for r in reqs])

    res = asyncio.run(main())
    assert len(store.calls) == 1                           # one decode launch for all 64
    assert len(store.calls[0]) == 48                       # each chunk id read once
    assert {k: b.stats[k] for k in ("batches", "requests", "reads")} == {"batches": 1, "requests": 64, "reads": 48}
    for i, r in enumerate(res):
        np.testing.assert_array_equal(r, chunks[f"c-{i % 48}"][sel])


def test_groups_missing_and_errors():
    chunks = _chunks(4)
    store = FakeStore(chunks, errors={"c-3"})
    b = ChunkBatcher(store, window_ms=20)

    async def main():
        f32 = [b.get_chunk(ChunkRead(f"c-{i}", "k"), np.float32, (8, 16)) for i in range(4)]
        missing = b.get_chunk(ChunkRead("c-9", "k"), np.float32, (8, 16))
        init = b.get_chunk(ChunkRead("c-9", "k"), np.float32, (8, 16), chunk_init=True, fill_value=7)
        return await asyncio.gather(*f32, missing, init, return_exceptions=True)

    res = asyncio.run(main())
    assert len(store.calls) == 2                           # chunk_init is a group of its own
    for i in range(3):
        np.testing.assert_array_equal(res[i], chunks[f"c-{i}"])
    assert isinstance(res[3], RuntimeError)                # only that request fails
    assert res[4] is None                                  # 404
    assert (res[5] == 7).all() and res[5].shape == (8, 16)


def test_max_batch_dispatches_early():
    chunks = _chunks(10)
    store = FakeStore(chunks)
    b = ChunkBatcher(store, window_ms=10_000, max_batch=5)     # the window never expires

    async def main():
        return await asyncio.wait_for(asyncio.gather(*[b.get_chunk(ChunkRead(f"c-{i}", "k"), np.float32, (8, 16))
                                                       for i in range(10)]), 5)

    res = asyncio.run(main())
    assert [len(c) for c in store.calls] == [5, 5]
    for i in range(10):
        np.testing.assert_array_equal(res[i], chunks[f"c-{i}"])


def test_group_keys():
    """equal parameters share a group whatever the dict object or key order; different
    values, unhashable values (JSON fallback) and NaN fill values behave as values"""
    from hsds_amd.batcher import _freeze
    a = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    b = {"dtype": np.dtype("<f4"), "level": 4, "shuffle": 1, "compressor": "zlib"}
    assert _freeze(a) == _freeze(b) and hash(_freeze(a)) == hash(_freeze(b))
    assert _freeze(a) != _freeze(dict(a, level=5))
    assert _freeze({"x": [1, 2]}) == _freeze({"x": [1, 2]}) != _freeze({"x": [1, 3]})
    assert _freeze(float("nan")) == _freeze(np.nan) and _freeze(None) is None
    assert _freeze([1.5, 2]) == _freeze([1.5, 2])
    chunks = _chunks(2)
    store = FakeStore(chunks)
    bt = ChunkBatcher(store, window_ms=20)

    async def main():
        return await asyncio.gather(*[bt.get_chunk(ChunkRead(f"c-{i}", "k"), np.float32, (8, 16),
                                                   filter_ops=dict(a) if i else dict(b)) for i in range(2)])
    asyncio.run(main())
    assert len(store.calls) == 1
