"""Device-built hyperslab copy records (hsds_plan_descs) equal the host plan's records
(crawl.SelectionPlan._descs, the restatement of chunk_crawl.py:118-150,395-418 pinned
by the selection goldens) for every direction: read pack / place / direct, write gather /
apply / broadcast apply, over strided, offset and sparse (step > chunk) selections."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
DSET = "d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d"


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


CASES = [((2048, 2560), (512, 512), (slice(100, 2048, 1), slice(100, 2560, 1)), "<f4", 8),
         ((512, 2048, 2048), (16, 64, 128), (slice(0, 512, 2), slice(3, 2048, 5), slice(1, 2048, 3)), "<i2", 1),
         ((300, 200, 64), (64, 64, 32), (slice(3, 300, 7), slice(1, 200, 3), slice(0, 64, 5)), "<i2", 3),
         ((1000, 4000), (10, 100), (slice(5, 1000, 37), slice(0, 4000, 250)), "<f8", 2),
         ((50,), (7,), (slice(3, 49, 1),), "|u1", 4),
         ((6, 7, 8, 9, 10), (2, 3, 4, 5, 6), (slice(1, 6, 2), slice(0, 7, 1), slice(2, 8, 3), slice(0, 9, 4),
                                              slice(1, 10, 1)), "<c8", 2)]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_device_records_equal_host(dev, case):
    from hsds_amd import _native as nat
    from hsds_amd import crawl
    from hsds_amd.engine import COPY_DESC_DTYPE
    dims, layout, sel, dt, world = CASES[case]
    plan = crawl.SelectionPlan(DSET, dims, layout, sel, np.dtype(dt), world)

    def host(recs):
        return np.ascontiguousarray(recs).view(np.uint8)

    def device(t):
        return t.cpu().numpy()

    assert np.array_equal(device(plan.device_descs(nat.PLAN_PLACE, dev)), host(plan.place_descs()))
    assert np.array_equal(device(plan.device_descs(nat.PLAN_GATHER, dev, slab_base=4096)),
                          host(plan.gather_descs(slab_base=4096)))
    for r in range(world):
        n = len(plan.by_rank[r])
        co = np.arange(n, dtype=np.int64) * (plan.chunk_nbytes + 256) + 512
        assert np.array_equal(device(plan.device_descs(nat.PLAN_PACK, dev, ranks=[r], chunk_offsets=co,
                                                       packed_base=64)),
                              host(plan.pack_descs(r, co, packed_base=64))), r
        assert np.array_equal(device(plan.device_descs(nat.PLAN_APPLY, dev, ranks=[r], chunk_offsets=co,
                                                       packed_base=32)),
                              host(plan.apply_descs(r, co, packed_base=32))), r
        assert np.array_equal(device(plan.device_descs(nat.PLAN_APPLY_BCAST, dev, ranks=[r], chunk_offsets=co,
                                                       packed_base=8)),
                              host(plan.apply_descs(r, co, packed_base=8, broadcast=True))), r
        assert np.array_equal(device(plan.device_descs(nat.PLAN_DIRECT, dev, ranks=[r], chunk_offsets=co,
                                                       slab_base=1024)),
                              host(plan.direct_descs(r, co, slab_base=1024))), r
    assert COPY_DESC_DTYPE.itemsize == 216
