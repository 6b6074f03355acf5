"""Compound field subsets in chunkReadSelection / chunkWriteSelection (chunkUtil.py:882-995)
against goldens from the reference itself (tests/golden/make_field_golden.py: the
reference's chunkUtil with getSubType select types, hdf5dtype.py:857-876).

CPU tests: the descriptor records hsds_amd.selection builds (one copy record per field,
one compare record per scalar leaf, per-field update units) are interpreted by a small
numpy model of the copy / compare kernels (copy_kernel / compare_kernel in engine.hip)
and must reproduce the goldens byte for byte.  `-m gpu` tests run the same records on
the MI355X through the C ABI (chunkReadSelection / chunkWriteSelection / ChunkStore
put_selections)."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

DTYPES = {
    "mixed": np.dtype([("a", "<i4"), ("b", "<f8"), ("c", "S3"), ("d", "<f4", (2,)), ("e", "<f2")]),
    "nested": np.dtype([("p", [("x", "<f4"), ("y", "<i2")]), ("q", "u1"), ("r", "<c8")]),
    "aligned": np.dtype({"names": ["u", "v", "w"], "formats": ["u1", "<f8", "<i2"], "offsets": [0, 8, 16],
                         "itemsize": 24}),
}


def _jdescr(dt):
    return json.loads(json.dumps(np.lib.format.dtype_to_descr(dt)))


def sub_type(dt, fields):
    """hdf5dtype.getSubType (hdf5dtype.py:857-876): packed compound of the fields in order"""
    return np.dtype([(f, dt[f]) for f in fields])


@pytest.fixture(scope="module")
def gold():
    meta = json.load(open(os.path.join(GOLD, "field_cases.json")))
    arrs = np.load(os.path.join(GOLD, "field_cases.npz"))
    for k, dt in DTYPES.items():
        assert _jdescr(dt) == meta["dtypes"][k], k
    return meta, arrs


def _fieldbytes(a):
    """the field bytes of a compound array (numpy leaves padding bytes undefined when it
    copies a structured array, so the reference's padding is not part of the golden)"""
    from numpy.lib import recfunctions
    return recfunctions.repack_fields(a).tobytes() if a.dtype.names else a.tobytes()


def _sl(c):
    return tuple(slice(*s) for s in c["slices"])


def _chunk(c, arrs, key="__chunk"):
    return arrs[c["name"] + key].copy().view(DTYPES[c["dtype"]]).reshape(c["shape"])


# -- numpy model of copy_kernel / compare_kernel over COPY_DESC records --
def _elem_offsets(rec):
    rank = int(rec["rank"])
    cnt = [int(x) for x in rec["count"][:rank]]
    so = np.full(1, int(rec["src_off"]), np.int64)
    do = np.full(1, int(rec["dst_off"]), np.int64)
    for d in range(rank):
        k = np.arange(cnt[d], dtype=np.int64)
        so = (so[:, None] + k[None, :] * int(rec["src_stride"][d])).reshape(-1)
        do = (do[:, None] + k[None, :] * int(rec["dst_stride"][d])).reshape(-1)
    return so, do


def model_copy(src, dst, recs, flags=None):
    for i, r in enumerate(recs):
        if flags is not None and not flags[i]:
            continue
        so, do = _elem_offsets(r)
        n = int(r["itemsize"])
        for b in range(n):
            dst[do + b] = src[so + b]


def model_compare(new, chunk, recs, kind):
    from hsds_amd import _native as nat
    out = np.zeros(len(recs), np.int32)
    for i, r in enumerate(recs):
        so, do = _elem_offsets(r)
        n = int(r["itemsize"])
        a = np.stack([chunk[do + b] for b in range(n)], 1).copy()
        b_ = np.stack([new[so + b] for b in range(n)], 1).copy()
        fdt = {nat.KIND_F16: "<f2", nat.KIND_F32: "<f4", nat.KIND_F64: "<f8", nat.KIND_C64: "<c8",
               nat.KIND_C128: "<c16"}.get(kind)
        if fdt is None:
            out[i] = int((a != b_).any())
        else:
            out[i] = int(not np.array_equal(a.view(fdt), b_.view(fdt)))
    return out


def model_read(arr, sl, select_dt):
    from hsds_amd.selection import _contig_slices, copy_desc
    dt = arr.dtype
    out_shape = arr[sl].shape
    out = np.zeros(out_shape, select_dt)
    recs = np.concatenate([copy_desc(arr.shape, sl, out_shape, _contig_slices(out_shape), dt.fields[f][0].itemsize,
                                     src_base=dt.fields[f][1], dst_base=select_dt.fields[f][1],
                                     src_itemsize=dt.itemsize, dst_itemsize=select_dt.itemsize)
                           for f in select_dt.names])
    o = out.view(np.uint8).reshape(-1)
    model_copy(arr.view(np.uint8).reshape(-1), o, recs)
    return out


def model_write(arr, sl, data):
    """the records of write_selection_descs run through the model: (updated, arr)"""
    from hsds_amd.selection import _write_data, write_selection_descs
    data = _write_data(arr.dtype, data)
    units = write_selection_descs(arr.shape, arr.dtype, sl, data.shape, data.dtype)
    new = data.view(np.uint8).reshape(-1)
    ch = arr.view(np.uint8).reshape(-1)
    updated = False
    flags = []
    for copies, leaves in units:
        d = any(model_compare(new, ch, [rec[0]], kind)[0] for kind, rec in leaves)
        flags.append(d)
    for (copies, _), d in zip(units, flags):
        if d:
            model_copy(new, ch, np.concatenate(copies))
            updated = True
    return updated


def test_read_goldens_descriptor_model(gold):
    meta, arrs = gold
    for c in meta["read"]:
        if "error" in c:
            continue
        arr = _chunk(c, arrs)
        sdt = sub_type(arr.dtype, c["fields"])
        assert _jdescr(sdt) == c["out_descr"], c["name"]
        if len(sdt) == len(arr.dtype):
            continue                                     # no field selection: the plain gather
        out = model_read(arr, _sl(c), sdt)
        assert list(out.shape) == c["out_shape"]
        assert out.tobytes() == arrs[c["name"] + "__out"].tobytes(), c["name"]


def test_write_goldens_descriptor_model(gold):
    meta, arrs = gold
    for c in meta["write"]:
        arr = _chunk(c, arrs)
        dt = arr.dtype
        sdt = sub_type(dt, c["fields"]) if c["fields"] else dt
        sl = _sl(c)
        data = arrs[c["name"] + "__data"].copy().view(sdt).reshape(arr[sl].shape)
        a2 = arr.copy()
        assert model_write(a2, sl, data) == c["updated"], c["name"]
        assert model_write(a2, sl, data) == c["updated_again"], c["name"]
        assert _fieldbytes(a2) == _fieldbytes(_chunk(c, arrs, "__out")), c["name"]


def test_write_units_and_leaves():
    """a field subset gives one unit per field; the whole compound one unit whose copy
    records skip padding and whose leaves carry each scalar's compare kind"""
    from hsds_amd import _native as nat
    from hsds_amd.selection import write_selection_descs
    dt = DTYPES["mixed"]
    sl = (slice(0, 4, 1), slice(0, 6, 2))
    units = write_selection_descs((4, 6), dt, sl, (4, 3), sub_type(dt, ["d", "a"]))
    assert len(units) == 2
    (cd, ld), (ca, la) = units
    assert [int(r["itemsize"]) for r in cd] == [8] and [k for k, _ in ld] == [nat.KIND_F32]
    assert int(ld[0][1]["rank"][0]) == 3 and int(ld[0][1]["count"][0][2]) == 2   # array field: inner dim
    assert [k for k, _ in la] == [nat.KIND_BYTES]
    whole = write_selection_descs((40,), DTYPES["aligned"], (slice(0, 40, 1),), (40,), DTYPES["aligned"])
    assert len(whole) == 1
    assert [int(r["itemsize"]) for r in whole[0][0]] == [1, 8, 2]      # padding bytes are not copied


# -- GPU: the same records through the C ABI --
@pytest.mark.gpu
def test_read_goldens_gpu(gold):
    import torch
    from hsds_amd.selection import chunkReadSelection
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    meta, arrs = gold
    for c in meta["read"]:
        arr = _chunk(c, arrs)
        sdt = sub_type(arr.dtype, c["fields"])
        if "error" in c:
            with pytest.raises({"ValueError": ValueError, "TypeError": TypeError}[c["error"]]):
                chunkReadSelection(arr, slices=_sl(c), select_dt=sdt)
            continue
        out = chunkReadSelection(arr, slices=_sl(c), select_dt=sdt)
        assert list(out.shape) == c["out_shape"] and _jdescr(out.dtype) == c["out_descr"]
        assert out.tobytes() == arrs[c["name"] + "__out"].tobytes(), c["name"]


@pytest.mark.gpu
def test_write_goldens_gpu(gold):
    import torch
    from hsds_amd.selection import chunkWriteSelection
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    meta, arrs = gold
    for c in meta["write"]:
        arr = _chunk(c, arrs)
        dt = arr.dtype
        sdt = sub_type(dt, c["fields"]) if c["fields"] else dt
        sl = _sl(c)
        data = arrs[c["name"] + "__data"].copy().view(sdt).reshape(arr[sl].shape)
        a2 = arr.copy()
        assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) == c["updated"], c["name"]
        assert chunkWriteSelection(chunk_arr=a2, slices=sl, data=data) == c["updated_again"], c["name"]
        assert _fieldbytes(a2) == _fieldbytes(_chunk(c, arrs, "__out")), c["name"]


@pytest.mark.gpu
def test_put_selections_field_subsets_gpu(gold):
    """PUT_Chunk with `fields` through the batched DN path: the golden writes as one
    put_selections batch per dtype over chunks that start from stored objects"""
    import torch
    from hsds_amd import codec
    from hsds_amd.datanode import ChunkRead, ChunkStore
    meta, arrs = gold
    dev = torch.device("cuda", 0)
    for dn in DTYPES:
        cases = [c for c in meta["write"] if c["dtype"] == dn]
        dt = DTYPES[dn]
        shape = tuple(cases[0]["shape"])
        store = {f"k{c['name']}": _chunk(c, arrs).tobytes() for c in cases}
        cs = ChunkStore(lambda k, o, n: store.get(k), mem_target=1 << 24, device=dev)
        writes = []
        for c in cases:
            sdt = sub_type(dt, c["fields"]) if c["fields"] else dt
            sl = _sl(c)
            data = arrs[c["name"] + "__data"].copy().view(sdt).reshape(_chunk(c, arrs)[sl].shape)
            writes.append((ChunkRead(f"c-{c['name']}", f"k{c['name']}"), sl, data))
        dirty = cs.put_selections(writes, dt, shape)
        assert dirty == [c["updated"] for c in cases], dn
        got = cs.get_chunks([w[0] for w in writes], dt, shape)
        for c, g in zip(cases, got):
            assert not isinstance(g, Exception)
            assert _fieldbytes(g.cpu().numpy().view(dt).reshape(shape)) == _fieldbytes(_chunk(c, arrs, "__out")), \
                c["name"]
        assert codec is not None
