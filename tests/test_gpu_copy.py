"""Streaming copy / compare kernels against a numpy model of
the hsds_copy_desc contract (numpy basic-slicing copies, chunkUtil.py:882-995 and
chunk_crawl.py:118-150,395-418): every byte each record names is moved, and no other byte
of the destination changes.  Random records cover contiguous runs at every relative
alignment (16-byte, dword and byte-funnel source paths, partial first / last slots),
stepped gathers into packed pieces (itemsize 1/2/4/8), broadcast sources (stride 0),
wide and odd itemsizes, many short rows per wave and rank up to 5."""
import numpy as np
import pytest

from copy_cases import _model, _offsets, _record, batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("seed", range(6))
def test_random_records_match_model(dev, seed):
    import torch
    from hsds_amd.engine import ChunkEngine
    src, dst0, recs = batch(seed)
    want = _model(src, dst0, recs)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.from_numpy(dst0).to(dev)
    eng.copy(d_src, d_dst, recs)
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    # copy_if: only flagged records move
    flags = torch.tensor([i % 3 == 0 for i in range(len(recs))], dtype=torch.int32, device=dev)
    d_dst = torch.from_numpy(dst0).to(dev)
    eng.copy(d_src, d_dst, recs, flags=flags)
    torch.cuda.synchronize()
    want_if = _model(src, dst0, recs[::3])
    assert (d_dst.cpu().numpy() == want_if).all()


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 4, 7, 8, 12, 15])
def test_slab_rows_every_relative_alignment(dev, shift):
    """the cfg5 slab -> chunk scatter shape (rows of 2 KiB) with the source shifted by
    every offset mod 16: 16-byte, dword and funnel paths, partial slots at both ends"""
    import torch
    from hsds_amd.engine import ChunkEngine, COPY_DESC_DTYPE
    rng = np.random.default_rng(shift)
    rows, row_bytes, slab_row = 64, 2048 + shift, 8192
    src = rng.integers(0, 256, rows * slab_row + 64, dtype=np.uint8)
    rec = np.zeros(2, COPY_DESC_DTYPE)
    for i, (so, do) in enumerate([(shift, 0), (3, rows * row_bytes + 64 + shift)]):
        rec[i]["src_off"], rec[i]["dst_off"] = so, do
        rec[i]["rank"], rec[i]["itemsize"] = 2, 1
        rec[i]["count"][:2] = [rows, row_bytes]
        rec[i]["src_stride"][:2] = [slab_row, 1]
        rec[i]["dst_stride"][:2] = [row_bytes, 1]
    dst0 = rng.integers(0, 256, 2 * rows * row_bytes + 256, dtype=np.uint8)
    want = _model(src, dst0, rec)
    eng = ChunkEngine(0)
    d_dst = torch.from_numpy(dst0).to(dev)
    eng.copy(torch.from_numpy(src).to(dev), d_dst, rec)
    torch.cuda.synchronize()
    assert (d_dst.cpu().numpy() == want).all()


@pytest.mark.parametrize("isz,kind_name", [(1, "KIND_BYTES"), (2, "KIND_BYTES"), (4, "KIND_F32"), (8, "KIND_F64"),
                                           (4, "KIND_BYTES"), (2, "KIND_F16"), (8, "KIND_C64")])
def test_compare_finds_single_difference(dev, isz, kind_name):
    """compare: equal regions report 0; one changed element anywhere (first, middle, last
    row) reports 1; float kinds follow numpy array_equal (NaN != NaN, -0.0 == 0.0)"""
    import torch
    from hsds_amd import _native as nat
    from hsds_amd.engine import ChunkEngine
    kind = getattr(nat, kind_name)
    rng = np.random.default_rng(isz * 7 + kind)
    recs, base = [], 0
    for i in range(8):
        r, ext = _record(rng, 1 << 20, base, isz)
        if kind != nat.KIND_BYTES:       # float elements on the float grid of `a`
            r["dst_off"] -= int(r["dst_off"][0]) % isz
        r["src_off"] = r["dst_off"]      # the data buffer mirrors the chunk layout: same offsets
        r["src_stride"] = r["dst_stride"]
        recs.append(r)
        base += ext
    recs = np.concatenate(recs)
    a = rng.integers(0, 256, base + 64, dtype=np.uint8)
    if kind != nat.KIND_BYTES:
        a = np.zeros(base + 64, np.uint8)          # finite floats: no NaN from random bytes
        fl = {nat.KIND_F32: np.float32, nat.KIND_F64: np.float64, nat.KIND_F16: np.float16,
              nat.KIND_C64: np.float32}[kind]
        n = a.size // np.dtype(fl).itemsize
        a[:n * np.dtype(fl).itemsize] = rng.normal(size=n).astype(fl).view(np.uint8)
    b = a.copy()
    eng = ChunkEngine(0)

    def run(bb):
        differs = torch.zeros(len(recs), dtype=torch.int32, device=dev)
        eng.compare(torch.from_numpy(bb).to(dev), torch.from_numpy(a).to(dev), recs, kind, differs)
        torch.cuda.synchronize()
        return differs.cpu().numpy()

    assert (run(b) == 0).all()
    for which in range(len(recs)):
        r = recs[which]
        k = int(r["rank"])
        offs = _offsets([int(c) for c in r["count"][:k]], r["dst_stride"][:k], int(r["dst_off"]))
        for pos in (offs[0], offs[len(offs) // 2], offs[-1]):
            bb = b.copy()
            bb[pos] ^= 0x10 if kind == nat.KIND_BYTES else 0x40     # the element's value changes
            got = run(bb)
            assert got[which] == 1 and got.sum() == 1, (which, pos, got)
    if kind == nat.KIND_F32:
        r = recs[0]
        pos = int(r["dst_off"])
        an, bn = a.copy(), b.copy()
        an[pos:pos + 4] = np.array([np.nan], np.float32).view(np.uint8)
        bn[pos:pos + 4] = an[pos:pos + 4]
        differs = torch.zeros(len(recs), dtype=torch.int32, device=dev)
        eng.compare(torch.from_numpy(bn).to(dev), torch.from_numpy(an).to(dev), recs, kind, differs)
        assert differs.cpu().numpy()[0] == 1                       # NaN is never equal
        an[pos:pos + 4] = np.array([-0.0], np.float32).view(np.uint8)
        bn[pos:pos + 4] = np.array([0.0], np.float32).view(np.uint8)
        differs.zero_()
        eng.compare(torch.from_numpy(bn).to(dev), torch.from_numpy(an).to(dev), recs, kind, differs)
        assert differs.cpu().numpy()[0] == 0                       # -0.0 == 0.0
