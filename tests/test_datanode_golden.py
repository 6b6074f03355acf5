"""DN read-side helpers against goldens produced by the reference itself
(tests/golden/make_rangeget_golden.py: rangegetUtil.chunkMunge /
getHyperChunkFactors / getHyperChunkIndex), and the device chunk cache's LruCache
semantics (hsds/util/lruCache.py:37-410) on CPU tensors."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rg_golden():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "rangeget_cases.json")))


def _loc(x):
    from hsds_amd.datanode import ChunkLocation
    return ChunkLocation(tuple(x[0]), x[1], x[2])


def _enc(c):
    if isinstance(c, list):
        return [_enc(e) for e in c]
    return [list(c.index), int(c.offset), int(c.length)]


def test_chunk_munge_matches_reference(rg_golden):
    from hsds_amd.datanode import chunkMunge
    assert len(rg_golden["munge"]) >= 60
    for case in rg_golden["munge"]:
        got = chunkMunge([_loc(x) for x in case["locs"]], max_gap=case["max_gap"])
        assert _enc(got) == case["out"], case


def test_hyper_chunk_factors_and_index(rg_golden):
    from hsds_amd.datanode import getHyperChunkFactors, getHyperChunkIndex
    for case in rg_golden["factors"]:
        if "error" in case:
            with pytest.raises(ValueError):
                getHyperChunkFactors(case["chunk_dims"], case["hyper_dims"])
            continue
        f = getHyperChunkFactors(case["chunk_dims"], case["hyper_dims"])
        assert f == case["factors"]
        assert [list(getHyperChunkIndex(i, f)) for i in range(int(np.prod(f)))] == case["indices"]


def test_device_cache_lru_semantics_on_cpu():
    # the cache logic is device-agnostic: exercise it on CPU tensors
    from hsds_amd.datanode import DeviceChunkCache
    kb = 1024
    c = DeviceChunkCache(mem_target=10 * kb, device="cpu", arena_bytes=64 * kb)
    for i in range(8):
        c[f"c{i}"] = np.full((256,), i, np.float32)        # 1 KiB each
    assert len(c) == 8 and c.memUsed == 8 * kb and c.cacheUtilizationPercent == 80
    _ = c["c0"]                                              # c0 becomes most recent
    c.setDirty("c1")
    assert c.dirtyCount == 1 and c.memDirty == kb and c.memFree == 9 * kb
    for i in range(8, 12):                                   # 12 KiB > target: evict clean LRU
        c[f"c{i}"] = np.full((256,), i, np.float32)
    assert c.memUsed <= 10 * kb
    assert "c1" in c                                         # dirty: never evicted
    assert "c0" in c                                         # recently used survives
    assert "c2" not in c and "c3" not in c                   # least recent clean ones went first
    assert float(c["c11"][0]) == 11.0 and c["c11"].shape == (256,)
    with pytest.raises(ValueError):
        c.clearCache()                                       # dirty node present
    c.clearDirty("c1")
    assert c.dirtyCount == 0 and c.memDirty == 0
    c.clearCache()
    assert len(c) == 0 and c.memUsed == 0
    # arena slots are reused after eviction
    c[f"x"] = np.zeros((1024,), np.float64)
    assert c.arena.used == 8 * kb


def test_filter_ops_match_reference(rg_golden):
    from hsds_amd.filters import getFilterOps
    vlen = np.dtype("O", metadata={"vlen": str})
    dts = {"<f4": np.dtype("<f4"), "vlen": vlen, "cmpd_vlen": np.dtype([("a", "<i4"), ("s", vlen)]), "none": None}
    fdefs = rg_golden["filter_defs"]
    assert len(rg_golden["filter_ops"]) >= 40
    for case in rg_golden["filter_ops"]:
        app = {"filter_map": {}}
        dt = dts[case["dtype"]]
        if "error" in case:
            with pytest.raises(Exception) as ei:
                getFilterOps(app, "d-x", [fdefs[k] for k in case["filters"]], dtype=dt, chunk_shape=(4, 5))
            assert type(ei.value).__name__ == case["error"]
            continue
        ops = getFilterOps(app, "d-x", [fdefs[k] for k in case["filters"]], dtype=dt, chunk_shape=(4, 5))
        again = getFilterOps(app, "d-x", [], dtype=dt, chunk_shape=(4, 5))
        enc = {k: (list(v) if k == "chunk_shape" else (None if v is None else str(v)) if k == "dtype" else v)
               for k, v in ops.items()}
        assert enc == case["ops"], case
        assert (again is ops) == case["cached"]
