"""CPU emulation of the streaming copy / compare kernels (hsds_amd/csrc/region.h, run lane
by lane by tests/emu/region_emu.cpp) against the numpy model of the hsds_copy_desc
contract -- the same random records as tests/test_gpu_copy.py, plus every relative
alignment of a 2 KiB slab row and the compare semantics.  Test infrastructure only."""
import ctypes
import os

import numpy as np
import pytest

from copy_cases import _model, _offsets, batch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libregion_emu.so")


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("build() the emulators first")
    L = ctypes.CDLL(EMU)
    P = ctypes.c_void_p
    L.emu_copy.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_uint32]
    L.emu_compare.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, P]
    return L


def _copy(emu, src, dst, recs, flags=None, nwaves=3):
    out = dst.copy()
    f = None if flags is None else np.ascontiguousarray(flags, np.int32)
    emu.emu_copy(src.ctypes.data, out.ctypes.data, recs.ctypes.data, len(recs),
                 None if f is None else f.ctypes.data, nwaves)
    return out


@pytest.mark.parametrize("seed", range(12))
def test_random_records(emu, seed):
    src, dst0, recs = batch(seed)
    got = _copy(emu, src, dst0, recs, nwaves=1 + seed % 5)
    want = _model(src, dst0, recs)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    flags = np.array([i % 3 == 0 for i in range(len(recs))], np.int32)
    assert (_copy(emu, src, dst0, recs, flags) == _model(src, dst0, recs[::3])).all()


@pytest.mark.parametrize("shift", range(16))
def test_slab_rows_every_relative_alignment(emu, shift):
    from hsds_amd.engine import COPY_DESC_DTYPE
    rng = np.random.default_rng(shift)
    rows, row_bytes, slab_row = 16, 2048 + shift, 8192
    src = rng.integers(0, 256, rows * slab_row + 64, dtype=np.uint8)
    rec = np.zeros(2, COPY_DESC_DTYPE)
    for i, (so, do) in enumerate([(shift, 0), (3, rows * row_bytes + 64 + shift)]):
        rec[i]["src_off"], rec[i]["dst_off"] = so, do
        rec[i]["rank"], rec[i]["itemsize"] = 2, 1
        rec[i]["count"][:2] = [rows, row_bytes]
        rec[i]["src_stride"][:2] = [slab_row, 1]
        rec[i]["dst_stride"][:2] = [row_bytes, 1]
    dst0 = rng.integers(0, 256, 2 * rows * row_bytes + 256, dtype=np.uint8)
    assert (_copy(emu, src, dst0, rec) == _model(src, dst0, rec)).all()


@pytest.mark.parametrize("isz,kind", [(1, 0), (2, 0), (4, 2), (8, 3), (4, 0), (2, 1), (8, 4)])
def test_compare_single_difference(emu, isz, kind):
    _, _, recs = batch(isz * 7 + kind, n=8, kinds=(isz,))
    recs = recs[0::2].copy()                    # records of this itemsize
    if kind != 0:                                  # float elements on the float grid of `a`
        recs["dst_off"] -= recs["dst_off"] % isz
    recs["src_off"] = recs["dst_off"]
    recs["src_stride"] = recs["dst_stride"]
    size = int(max(int(r["dst_off"]) + 1 + sum((int(c) - 1) * int(s) for c, s in
                                               zip(r["count"][:r["rank"]], r["dst_stride"][:r["rank"]]))
                   + int(r["itemsize"]) for r in recs)) + 64
    rng = np.random.default_rng(kind)
    if kind == 0:
        a = rng.integers(0, 256, size, dtype=np.uint8)
    else:
        fl = {1: np.float16, 2: np.float32, 3: np.float64, 4: np.float32}[kind]
        n = size // np.dtype(fl).itemsize + 1
        a = rng.normal(size=n).astype(fl).view(np.uint8)[:size].copy()
    differs = np.zeros(len(recs), np.int32)

    def run(b, aa=a):
        emu.emu_compare(b.ctypes.data, aa.ctypes.data, recs.ctypes.data, len(recs), kind, differs.ctypes.data)
        return differs.copy()

    assert (run(a.copy()) == 0).all()
    for which in range(len(recs)):
        r = recs[which]
        k = int(r["rank"])
        offs = _offsets([int(c) for c in r["count"][:k]], r["dst_stride"][:k], int(r["dst_off"]))
        for pos in (offs[0], offs[len(offs) // 2], offs[-1]):
            b = a.copy()
            b[pos] ^= 0x10 if kind == 0 else 0x40
            got = run(b)
            assert got[which] == 1 and got.sum() == 1, (which, pos, got)
    if kind == 2:                                  # numpy array_equal float semantics
        pos = int(recs[0]["dst_off"])
        an = a.copy()
        an[pos:pos + 4] = np.array([np.nan], np.float32).view(np.uint8)
        assert run(an.copy(), an)[0] == 1            # NaN is never equal
        b = an.copy()
        an[pos:pos + 4] = np.array([-0.0], np.float32).view(np.uint8)
        b[pos:pos + 4] = np.array([0.0], np.float32).view(np.uint8)
        assert run(b, an)[0] == 0                    # -0.0 == 0.0


@pytest.mark.parametrize("n,so,do,isz", [(3 << 20, 0, 0, 1), ((3 << 20) + 5, 3, 17, 1), (1 << 20, 8, 4, 4),
                                          (200000, 2, 6, 2)])
def test_long_rows_are_split(emu, n, so, do, isz):
    """one long row (a whole contiguous chunk, a 3 MiB run) is cut into pieces; strided
    long rows too"""
    from hsds_amd.engine import COPY_DESC_DTYPE
    rng = np.random.default_rng(n)
    step = 1 if isz == 1 else 3
    src = rng.integers(0, 256, so + n * isz * step + 64, dtype=np.uint8)
    rec = np.zeros(1, COPY_DESC_DTYPE)
    rec["src_off"], rec["dst_off"], rec["rank"], rec["itemsize"] = so, do, 1, isz
    rec["count"][0, 0] = n
    rec["src_stride"][0, 0] = isz * step
    rec["dst_stride"][0, 0] = isz
    dst0 = rng.integers(0, 256, do + n * isz + 64, dtype=np.uint8)
    assert (_copy(emu, src, dst0, rec, nwaves=7) == _model(src, dst0, rec)).all()
    # compare over the same long row: equal, then one byte changed near the end
    rec2 = rec.copy()
    rec2["src_stride"][0, 0] = isz
    rec2["src_off"] = do
    a = dst0.copy()
    differs = np.zeros(1, np.int32)
    emu.emu_compare(a.ctypes.data, a.ctypes.data, rec2.ctypes.data, 1, 0, differs.ctypes.data)
    assert differs[0] == 0
    b = a.copy()
    b[do + n * isz - 2] ^= 1
    emu.emu_compare(b.ctypes.data, a.ctypes.data, rec2.ctypes.data, 1, 0, differs.ctypes.data)
    assert differs[0] == 1


@pytest.mark.parametrize("seed", range(4))
def test_split_of_large_counts(emu, seed):
    """counts of 2^31 or more are split on the host (ChunkEngine.copy); the
    split is checked here at a small limit against the unsplit records"""
    from hsds_amd.engine import split_large_copy_descs
    src, dst0, recs = batch(100 + seed)
    lim = 8
    parts = split_large_copy_descs(recs, limit=lim)
    assert (parts["count"] < lim).all() and len(parts) > len(recs)
    assert (_copy(emu, src, dst0, parts) == _model(src, dst0, recs)).all()


def test_count_beyond_abi_range_copies_nothing(emu):
    """a record with a count of 2^31 or more (outside hsds_copy_desc's range) is skipped by
    the kernel, not narrowed to 32 bits"""
    from hsds_amd.engine import COPY_DESC_DTYPE
    src = np.arange(64, dtype=np.uint8)
    dst0 = np.zeros(64, np.uint8)
    rec = np.zeros(1, COPY_DESC_DTYPE)
    rec["rank"], rec["itemsize"] = 1, 1
    rec["count"][0, 0] = (1 << 32) + 4                  # narrowed to 32 bits this would be 4
    rec["src_stride"][0, 0] = rec["dst_stride"][0, 0] = 1
    assert (_copy(emu, src, dst0, rec) == dst0).all()
