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
