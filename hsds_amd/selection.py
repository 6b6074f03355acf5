"""Hyperslab selection math and GPU selection copies for the HSDS DN/SN hot path.

Host-side index math restated from the reference (results must be identical; pinned
by tests/golden/selection_cases.json generated from the reference itself):
  getSelectionList / getSelectionShape / getSelectionPagination / getSliceQueryParam
      hsds/util/dsetUtil.py:333, 560-660, 689-800, 803-843
  getNumChunks / getChunkIds / getChunkSelection / getChunkCoverage / getDataCoverage
      hsds/util/chunkUtil.py:268-350, 459-582, 608-790
The byte movement (chunkReadSelection, chunkWriteSelection, the SN slab scatter
np_arr[data_sel] = chunk_arr) runs as batched strided-copy kernels on the GPU
(include/hsds_amd.h hsds_copy_batch / hsds_compare_batch).
"""
import numpy as np

from . import _native as nat


def frac(x, d):
    """ceil(x / d) for integers (chunkUtil.frac)."""
    return -((-x) // d)


def _step(s):
    return 1 if s.step is None else s.step


def slice_stop(s):
    """Last selected index + 1 of a slice whose step may not divide its width."""
    step = _step(s)
    if step > 1:
        npts = frac(s.stop - s.start, step)
        return s.start + npts * step - (step - 1)
    return s.stop


def _span(s):
    """Width from the first to just past the last selected point."""
    return slice_stop(s) - s.start


# ---------------------------------------------------------------------------
# selection strings  (dsetUtil.getSelectionList and helpers)
# ---------------------------------------------------------------------------
def _split_dims(select):
    """'[a:b, [1,2], 3]' -> ['a:b', '[1,2]', '3'] ; raises ValueError on bad syntax."""
    body = select[1:-1]
    parts, cur, in_list = [], [], False
    for ch in body:
        if ch.isspace():
            continue
        if ch == "," and not in_list:
            if not cur:
                raise ValueError("invalid query")
            parts.append("".join(cur))
            cur = []
            continue
        if ch == "[":
            if in_list:
                raise ValueError("invalid query")
            in_list = True
        elif ch == "]":
            if not in_list:
                raise ValueError("invalid query")
            in_list = False
        elif ch == ":" and in_list:
            raise ValueError("invalid query")
        cur.append(ch)
    if not cur:
        raise ValueError("invalid query")
    parts.append("".join(cur))
    return parts


def _body_to_select(body):
    start = body["start"]
    start = list(start) if isinstance(start, (list, tuple)) else [start]
    stop = body["stop"]
    stop = list(stop) if isinstance(stop, (list, tuple)) else [stop]
    if len(stop) != len(start):
        raise ValueError("start and stop values have different ranks")
    step = body.get("step")
    if step is not None:
        step = list(step) if isinstance(step, (list, tuple)) else [step]
        if len(step) != len(start):
            raise ValueError("step values have different rank from start and stop selections")
    dims = [f"{a}:{b}" + (f":{step[i]}" if step else "") for i, (a, b) in enumerate(zip(start, stop))]
    return "[" + ",".join(dims) + "]"


def _parse_int(text, what, dim):
    try:
        return int(text)
    except ValueError:
        raise ValueError(f"Invalid selection - {what} value for dim {dim}")


def getSelectionList(select, dims):
    """Tuple of slices / coordinate lists for a select string (or request-body dict)."""
    if isinstance(select, dict):
        select = _body_to_select(select)
    if select is None or len(select) == 0:
        return tuple(slice(0, extent, 1) for extent in dims)
    elements = select if isinstance(select, (list, tuple)) else _split_dims(select)
    if len(dims) != len(elements):
        raise ValueError("invalid rank for selection")
    out = []
    for dim, (extent, el) in enumerate(zip(dims, elements)):
        if isinstance(el, list) or (isinstance(el, str) and el.startswith("[")):
            fields = el if isinstance(el, list) else el[1:-1].split(",")
            coords = []
            for f in fields:
                try:
                    v = int(f)
                except ValueError:
                    raise ValueError(f"Invalid coordinate for dim {dim}")
                if v < 0 or v >= extent:
                    raise ValueError(f"out of range coordinate for dim {dim}")
                coords.append(v)
            out.append(coords)
        elif el == ":":
            out.append(slice(0, extent, 1))
        elif isinstance(el, str) and ":" in el:
            fields = el.split(":")
            if len(fields) not in (2, 3):
                raise ValueError(f"Invalid selection format for dim {dim}")
            start = 0 if fields[0] == "" else _parse_int(fields[0], "start", dim)
            if fields[0] != "" and (start < 0 or start >= extent):
                raise ValueError(f"Invalid selection - start value out of range for dim {dim}")
            stop = extent if fields[1] == "" else _parse_int(fields[1], "stop", dim)
            if fields[1] != "" and (stop < 0 or stop > extent or stop <= start):
                raise ValueError(f"Invalid selection - stop value out of range for dim {dim}")
            step = 1
            if len(fields) == 3 and fields[2] != "":
                step = _parse_int(fields[2], "step", dim)
                if step <= 0:
                    raise ValueError(f"Invalid selection - step value out of range for dim {dim}")
            out.append(slice(start, stop, step))
        else:
            idx = _parse_int(el, "index", dim)
            if idx < 0 or idx >= extent:
                raise ValueError(f"Invalid selection - index value out of range for dim {dim}")
            out.append(slice(idx, idx + 1, 1))
    return tuple(out)


def getSelectionShape(selection):
    """Result shape of a selection (dsetUtil.getSelectionShape semantics)."""
    shape, ncoords = [], None
    for s in selection:
        if isinstance(s, slice):
            step = s.step if (s.step and s.step > 1) else 1
            width = s.stop - s.start if s.stop > s.start else 0
            extent = width // step if (step > 1 and width > 0) else width
            if (s.stop - s.start) % step != 0:
                extent += 1
            shape.append(extent)
        else:
            if ncoords is None:
                ncoords = len(s)
                shape.append(ncoords)
            elif ncoords != len(s):
                raise ValueError("shape mismatch: indexing arrays could not be broadcast together")
    return shape


def getSliceQueryParam(sel):
    """Select string for a chunk-relative selection ('[a:b:s,[i,j],...]')."""
    if len(sel) == 0:
        return None
    items = []
    for s in sel:
        if isinstance(s, slice):
            items.append(f"{s.start}:{s.stop}" + (f":{s.step}" if s.step > 1 else ""))
        else:
            items.append("[" + ",".join(str(x) for x in s) + "]")
    return "[" + ",".join(items) + "]"


def getSelectionPagination(select, dims, itemsize, max_request_size):
    """Split a selection along its first dimension of extent > 1 into pages of at
    most max_request_size bytes (dsetUtil.getSelectionPagination)."""
    size = int(np.prod(getSelectionShape(select))) * itemsize
    if size <= max_request_size:
        return (select,)
    pdim, pext = None, None
    for i, s in enumerate(select):
        if isinstance(s, slice):
            pext = s.stop - s.start if s.stop > s.start else 0
        else:
            pext = len(s)
        if pext > 1:
            pdim = i
            break
    if pdim is None:
        raise ValueError("unable to determine pagination dimension")
    npages = size // max_request_size + 1
    if pext < npages:
        raise ValueError(f"select pagination unable to paginate select dim: {pdim} into {npages} pages")
    per_page = max(pext // npages, 1)
    s = select[pdim]
    pieces = []
    if isinstance(s, slice):
        step = s.step if (s.step and s.stop > 1) else 1   # reference tests s.stop, not s.step
        lo = s.start
        while lo < s.stop:
            hi = lo + per_page
            if hi % step:
                hi += step - hi % step
            hi = min(hi, s.stop)
            pieces.append(slice(lo, hi, step))
            lo = hi
    else:
        for lo in range(0, len(s), per_page):
            pieces.append(tuple(s[lo:lo + per_page]))
    return tuple(tuple(p if i == pdim else select[i] for i in range(len(select))) for p in pieces)


# ---------------------------------------------------------------------------
# chunk iteration  (chunkUtil)
# ---------------------------------------------------------------------------
def getNumChunks(selection, layout):
    """Number of chunks a selection may touch (chunkUtil.getNumChunks, including its
    estimate for steps larger than the chunk extent)."""
    if len(selection) != len(layout):
        raise ValueError(f"selection list has {len(selection)} items, but rank is {len(layout)}")
    for s in selection:
        if (isinstance(s, slice) and s.stop <= s.start) or (not isinstance(s, slice) and len(s) == 0):
            return 0
    keys = None
    for s, c in zip(selection, layout):
        if isinstance(s, slice):
            continue
        if keys is None:
            keys = [""] * len(s)
        elif len(s) != len(keys):
            raise ValueError("shape mismatch: indexing arrays could not be broadcast together")
        keys = [(k + "_" if k else "") + str(v // c) for k, v in zip(keys, s)]
    total = len(set(keys)) if keys else 1
    for s, c in zip(selection, layout):
        if not isinstance(s, slice):
            continue
        step = _step(s)
        w = _span(slice(s.start, s.stop, step))
        left = frac(s.start, c) * c
        if s.start + w <= left:
            continue
        right = ((s.start + w) // c) * c
        inner = right - left
        n = inner // c if c > step else inner // step
        n += (s.start < left) + (s.start + w > right)
        total *= n
    return total


def getChunkIndex(chunk_id):
    n = chunk_id.find("_")
    if n < 0:
        raise ValueError(f"Invalid chunk_id: {chunk_id}")
    return [int(p) for p in chunk_id[n + 1:].split("_")]


def getChunkSuffix(chunk_id):
    n = chunk_id.find("_")
    if n < 0:
        raise ValueError(f"Invalid chunk_id: {chunk_id}")
    return chunk_id[n + 1:]


def getChunkCoordinate(chunk_id, layout):
    return [i * c for i, c in zip(getChunkIndex(chunk_id), layout)]


def getChunkId(dset_id, point, layout):
    pt = [point] if len(layout) == 1 and not isinstance(point, (list, tuple, np.ndarray)) else point
    return "c-" + dset_id[2:] + "_" + "_".join(str(int(pt[d]) // layout[d]) for d in range(len(layout)))


def _dim_chunk_indices(s, c):
    step = _step(s)
    if step > c:
        return [i // c for i in range(s.start, s.stop, step)]
    w = _span(slice(s.start, s.stop, step))
    return list(range(s.start // c, frac(s.start + w, c)))


def getChunkIds(dset_id, selection, layout, prefix=None):
    """Chunk ids intersecting a selection, last dimension fastest (chunkUtil.getChunkIds)."""
    if getNumChunks(selection, layout) == 0:
        return []
    if prefix is None:
        if not dset_id.startswith("d-"):
            raise ValueError(f"Bad Request: invalid dset id: {dset_id}")
        prefix = "c-" + dset_id[2:] + "_"
    rank = len(selection)
    ncoord = None
    for s in selection:
        if not isinstance(s, slice):
            if ncoord is None:
                ncoord = len(s)
            elif len(s) != ncoord:
                raise ValueError("coordinate length mismatch")
    # distinct partial indices from coordinate dimensions (None = slice dimension)
    seen = {}
    for i in range(ncoord if ncoord is not None else 1):
        key = tuple(None if isinstance(s, slice) else s[i] // c for s, c in zip(selection, layout))
        seen.setdefault("_".join("*" if k is None else str(k) for k in key), list(key))
    items = [list(v) for v in seen.values()]
    for d in range(rank):
        s = selection[d]
        if not isinstance(s, slice):
            continue
        idx = _dim_chunk_indices(s, layout[d])
        items = [it[:d] + [j] + it[d + 1:] for it in items for j in idx]
    return [prefix + "_".join(str(x) for x in it) for it in items]


def getChunkSelection(chunk_id, slices, layout):
    """Dataset-space intersection of a chunk with a selection, start snapped onto the
    selection's step lattice (chunkUtil.getChunkSelection); None when disjoint."""
    index = getChunkIndex(chunk_id)
    rank = len(layout)
    mask = None
    for d in range(rank):
        s = slices[d]
        if isinstance(s, slice):
            continue
        lo, c = index[d] * layout[d], layout[d]
        if mask is None:
            mask = [True] * len(s)
        if len(s) != len(mask):
            raise ValueError("mismatched number of coordinates for fancy selection")
        mask = [m and lo <= v < lo + c for m, v in zip(mask, s)]
    out = []
    for d in range(rank):
        s, c = slices[d], layout[d]
        lo = index[d] * c
        if not isinstance(s, slice):
            out.append([v for v, m in zip(s, mask) if m])
            continue
        step = _step(s)
        if s.start >= lo + c or s.stop < lo:
            return None
        stop = min(s.stop, lo + c)
        start = s.start if s.start >= lo else s.start + frac(lo - s.start, step) * step
        out.append(slice(start, slice_stop(slice(start, stop, step)), step))
    return out


def getChunkCoverage(chunk_id, slices, layout):
    """Chunk-relative selection (chunkUtil.getChunkCoverage)."""
    index = getChunkIndex(chunk_id)
    sel = getChunkSelection(chunk_id, slices, layout)
    if not sel:
        return None
    if len(slices) != len(layout):
        raise ValueError(f"invalid slices value for dataset of rank: {len(layout)}")
    out = []
    for d, s in enumerate(sel):
        off = index[d] * layout[d]
        if isinstance(s, slice):
            start, stop = s.start - off, s.stop - off
            if start < 0 or stop > layout[d]:
                raise ValueError("Unexpected chunk selection")
            out.append(slice(start, stop, s.step))
        else:
            out.append(tuple(v - off for v in s))
    return out


def getDataCoverage(chunk_id, slices, layout):
    """Position of a chunk's selected points inside the result slab
    (chunkUtil.getDataCoverage): slices with step 1, or point indices."""
    csel = getChunkSelection(chunk_id, slices, layout)
    rank = len(layout)
    ncoord = None
    for d in range(rank):
        s, cs = slices[d], csel[d]
        if isinstance(s, slice):
            continue
        if isinstance(cs, slice):
            raise ValueError("expecting coordinate chunk selection for data coord selection")
        if len(cs) < 1:
            raise ValueError("expected at least one chunk coordinate")
        if ncoord is None:
            ncoord = len(s)
        elif ncoord != len(s):
            raise ValueError("shape mismatch: indexing arrays could not be broadcast together")
    out, pts_dim = [], None
    for d in range(rank):
        s, cs = slices[d], csel[d]
        if isinstance(s, slice):
            step = _step(s)
            if cs.step != step:
                raise ValueError("expecting step for chunk selection to be the same as data selection")
            out.append(slice((cs.start - s.start) // step, frac(cs.stop - s.start, step), 1))
        elif pts_dim is None:
            pts_dim = len(out)
            out.append([])
    if pts_dim is not None:
        corner = getChunkCoordinate(chunk_id, layout)
        for i in range(ncoord):
            inside = True
            for d in range(rank):
                s = slices[d]
                if isinstance(s, slice):
                    continue
                if not (corner[d] <= s[i] < corner[d] + layout[d]):
                    inside = False
                    break
            if inside:
                out[pts_dim].append(i)
    return tuple(out)


# ---------------------------------------------------------------------------
# strided copy descriptors + GPU selection copies
# ---------------------------------------------------------------------------
def _region(shape, itemsize, slices):
    """(byte offset of the first element, byte strides per dim, counts) of
    arr[slices] for a C-contiguous array of `shape`."""
    rank = len(shape)
    strides = [itemsize] * rank
    for d in range(rank - 2, -1, -1):
        strides[d] = strides[d + 1] * shape[d + 1]
    off, st, cnt = 0, [], []
    for d in range(rank):
        s = slices[d]
        if not isinstance(s, slice):
            raise NotImplementedError("point selections are outside the hyperslab engine")
        start, stop, step = s.indices(shape[d])
        n = len(range(start, stop, step))
        off += start * strides[d]
        st.append(step * strides[d])
        cnt.append(n)
    return off, st, cnt


def copy_desc(src_shape, src_slices, dst_shape, dst_slices, itemsize, src_base=0, dst_base=0,
              src_itemsize=None, dst_itemsize=None, inner=None):
    """One hsds_copy_desc record: dst[dst_slices] = src[src_slices] (shapes must agree).
    `itemsize` bytes are copied per element; the element strides of the two arrays are
    src_itemsize / dst_itemsize (default itemsize), so a record can move one field of a
    compound element (src_base / dst_base = the field offsets).  inner = (count, stride)
    adds a trailing dimension (the scalars of an array field)."""
    from .engine import COPY_DESC_DTYPE
    so, sst, scnt = _region(src_shape, src_itemsize or itemsize, src_slices)
    do, dstr, dcnt = _region(dst_shape, dst_itemsize or itemsize, dst_slices)
    if scnt != dcnt:
        raise ValueError(f"selection shapes differ: {scnt} vs {dcnt}")
    if inner is not None:
        scnt, dcnt = scnt + [int(inner[0])], dcnt + [int(inner[0])]
        sst, dstr = sst + [int(inner[1])], dstr + [int(inner[1])]
    if len(scnt) > nat.MAX_RANK:
        raise NotImplementedError(f"rank > {nat.MAX_RANK}")
    rec = np.zeros(1, COPY_DESC_DTYPE)
    rank = len(scnt)
    rec["src_off"] = src_base + so
    rec["dst_off"] = dst_base + do
    rec["rank"] = rank
    rec["itemsize"] = itemsize
    rec["src_stride"][0, :rank] = sst
    rec["dst_stride"][0, :rank] = dstr
    rec["count"][0, :rank] = scnt
    return rec


def _leaves(dt, off=0):
    """(byte offset, scalar dtype, count) of every scalar leaf of `dt`: the units numpy's
    array_equal compares with the leaf's own semantics (float NaN / -0.0)"""
    if dt.subdtype is not None:
        base, shape = dt.subdtype
        n = int(np.prod(shape))
        if base.names:
            return [x for i in range(n) for x in _leaves(base, off + i * base.itemsize)]
        return [(off, base, n)]
    if dt.names:
        return [x for name in dt.names for x in _leaves(dt.fields[name][0], off + dt.fields[name][1])]
    return [(off, dt, 1)]


def _fields(dt):
    """(name, dtype, offset) of the top-level fields; a plain dtype is one unnamed field"""
    if not dt.names:
        return [(None, dt, 0)]
    return [(n, dt.fields[n][0], dt.fields[n][1]) for n in dt.names]


def _contig_slices(shape):
    return tuple(slice(0, n, 1) for n in shape)


def _kind(dtype):
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return {2: nat.KIND_F16, 4: nat.KIND_F32, 8: nat.KIND_F64}.get(dt.itemsize, nat.KIND_BYTES)
    if dt.kind == "c":
        return {8: nat.KIND_C64, 16: nat.KIND_C128}.get(dt.itemsize, nat.KIND_BYTES)
    return nat.KIND_BYTES


def _to_dev(arr, dev):
    import torch
    if isinstance(arr, torch.Tensor):
        return arr
    a = np.ascontiguousarray(arr)
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(dev)


def chunkReadSelection(chunk_arr, slices=None, select_dt=None):
    """chunkUtil.chunkReadSelection (chunkUtil.py:882-929): chunk_arr[slices] as a new
    C-contiguous array, the strided gather running on the GPU.  A field subset of a
    compound type (select_dt with fewer fields, getSubType at chunk_dn.py:488-497) is
    gathered field by field into a zero-filled select_dt array: one copy record per field
    (chunk field offset -> select_dt field offset), all in one launch.  A single field
    that is an array or a compound raises as the reference's `arr[...] = out[field]`
    does (ValueError / TypeError)."""
    import torch
    from .engine import ChunkEngine
    arr = np.asarray(chunk_arr)
    rank = arr.ndim
    if rank == 0:
        raise ValueError("No dimension passed to chunkReadSelection")
    slices = tuple(slices)
    if len(slices) != rank:
        raise ValueError("Selection rank does not match shape rank")
    dt = arr.dtype
    out_shape = tuple(len(range(*s.indices(n))) for s, n in zip(slices, arr.shape))
    fields = None
    if select_dt is not None and len(select_dt) < len(dt):
        select_dt = np.dtype(select_dt)
        fields = list(select_dt.names)
        for f in fields:
            if f not in (dt.names or ()):
                raise ValueError(f"no field of name {f}")
            if select_dt.fields[f][0] != dt.fields[f][0]:
                raise NotImplementedError("field selection with a converted field type")
        if len(fields) == 1:
            fdt = dt.fields[fields[0]][0]
            if fdt.subdtype is not None:
                raise ValueError(f"could not broadcast the array field {fields[0]} into shape {out_shape}")
            if fdt.names:
                raise TypeError(f"cannot assign the compound field {fields[0]} to a one-field structure")
    out_dt = select_dt if fields else dt
    out = np.zeros(out_shape, out_dt)
    if out.size == 0:
        return out
    dev = torch.device("cuda", torch.cuda.current_device())
    d_src = _to_dev(arr, dev)
    if fields:
        d_dst = torch.zeros(out.nbytes, dtype=torch.uint8, device=dev)
        desc = np.concatenate([copy_desc(arr.shape, slices, out_shape, _contig_slices(out_shape),
                                         dt.fields[f][0].itemsize, src_base=dt.fields[f][1],
                                         dst_base=out_dt.fields[f][1], src_itemsize=dt.itemsize,
                                         dst_itemsize=out_dt.itemsize) for f in fields])
    else:
        d_dst = torch.empty(out.nbytes, dtype=torch.uint8, device=dev)
        desc = copy_desc(arr.shape, slices, out_shape, _contig_slices(out_shape), dt.itemsize)
    ChunkEngine().copy(d_src, d_dst, desc)
    out.view(np.uint8).reshape(-1)[:] = d_dst.cpu().numpy()
    return out


def write_selection_descs(chunk_shape, chunk_dt, slices, data_shape, data_dt, data_base=0, chunk_base=0):
    """Device records for chunkWriteSelection (chunkUtil.py:932-995) of `data` (dtype
    data_dt, C-contiguous data_shape at data_base) into chunk[slices] (chunk_base).

    Units are what the reference updates as a whole: every field of data_dt when it is a
    field subset of chunk_dt (field-wise update, one ndarray_compare per field), else the
    whole element (one compare; numpy assigns structured elements field by field, so
    padding bytes are left alone).  Returns a list of units, each
    (copy records, [(kind, compare record)] over its scalar leaves): a unit differs when
    any of its leaves differs under the leaf's own semantics (float NaN != NaN,
    -0.0 == 0.0), and its copy records are applied only then."""
    chunk_dt, data_dt = np.dtype(chunk_dt), np.dtype(data_dt)
    field_update = len(data_dt) > 0 and len(data_dt) < len(chunk_dt)
    if field_update:
        units = [[(chunk_dt.fields[f][1], data_dt.fields[f][1], chunk_dt.fields[f][0])] for f in data_dt.names]
    else:
        units = [[(off, off, fdt) for _, fdt, off in _fields(chunk_dt)]]
    full = _contig_slices(data_shape)
    out = []
    for parts in units:
        copies, leaves = [], []
        for coff, doff, fdt in parts:
            copies.append(copy_desc(data_shape, full, chunk_shape, slices, fdt.itemsize, src_base=data_base + doff,
                                    dst_base=chunk_base + coff, src_itemsize=data_dt.itemsize,
                                    dst_itemsize=chunk_dt.itemsize))
            for loff, base, n in _leaves(fdt):
                leaves.append((_kind(base), copy_desc(data_shape, full, chunk_shape, slices, base.itemsize,
                                                      src_base=data_base + doff + loff,
                                                      dst_base=chunk_base + coff + loff,
                                                      src_itemsize=data_dt.itemsize, dst_itemsize=chunk_dt.itemsize,
                                                      inner=(n, base.itemsize) if n > 1 else None)))
        out.append((copies, leaves))
    return out


def apply_writes(eng, d_data, d_chunk, items, nwrites, stream=None):
    """Compare + conditional copy for a batch of writes: `items` = [(write index, units
    from write_selection_descs)].  One compare launch per leaf kind (one for plain
    dtypes) and ONE copy launch; returns the per-write changed flags (int32 device
    tensor, no host sync)."""
    import torch
    from .engine import COPY_DESC_DTYPE
    dev = d_data.device
    by_kind, copies, copy_unit, unit_write = {}, [], [], []
    for w, units in items:
        for copy_recs, leaves in units:
            u = len(unit_write)
            unit_write.append(w)
            copies += copy_recs
            copy_unit += [u] * len(copy_recs)
            for kind, rec in leaves:
                by_kind.setdefault(kind, ([], []))
                by_kind[kind][0].append(rec)
                by_kind[kind][1].append(u)
    nunits = len(unit_write)
    flags_w = torch.zeros(max(nwrites, 1), dtype=torch.int32, device=dev)
    if not nunits:
        return flags_w
    nleaf = sum(len(v[0]) for v in by_kind.values())
    differs = torch.zeros(nleaf, dtype=torch.int32, device=dev)
    leaf_unit, lo = [], 0
    for kind, (recs, us) in by_kind.items():
        eng.compare(d_data, d_chunk, np.concatenate(recs), kind, differs[lo:lo + len(recs)], stream=stream)
        leaf_unit += us
        lo += len(recs)
    if nleaf == nunits and leaf_unit == list(range(nunits)) and len(copies) == nunits:
        unit = differs                       # one leaf and one record per unit: flags as they are
    else:
        unit = torch.zeros(nunits, dtype=torch.int32, device=dev)
        unit.index_add_(0, torch.tensor(leaf_unit, dtype=torch.int64, device=dev), differs)
    cflags = unit if len(copies) == nunits and copy_unit == list(range(nunits)) else \
        unit[torch.tensor(copy_unit, dtype=torch.int64, device=dev)]
    eng.copy(d_data, d_chunk, np.concatenate(copies) if copies else np.zeros(0, COPY_DESC_DTYPE),
             flags=cflags, stream=stream)
    flags_w.index_add_(0, torch.tensor(unit_write, dtype=torch.int64, device=dev), unit)
    return flags_w


def _write_data(arr_dt, data):
    """the write's data as a C-contiguous array: a field subset keeps its fields (in the
    chunk's field types, getSubType order), anything else takes the chunk dtype"""
    if len(data.dtype) > 0 and len(data.dtype) < len(arr_dt):
        for f in data.dtype.names:
            if f not in arr_dt.names:
                raise ValueError(f"no field of name {f}")
        sub = np.dtype([(f, arr_dt.fields[f][0]) for f in data.dtype.names])
        return np.ascontiguousarray(data if data.dtype == sub else data.astype(sub))
    return np.ascontiguousarray(data, dtype=arr_dt)


def chunkWriteSelection(chunk_arr=None, slices=None, data=None):
    """chunkUtil.chunkWriteSelection (chunkUtil.py:932-995): if data differs from
    chunk_arr[slices] (ndarray_compare = numpy array_equal semantics) write it and return
    True.  A compound `data` with fewer fields than the chunk is a field-wise update
    (chunkUtil.py:956-979): each field is compared and written on its own."""
    import torch
    from .engine import ChunkEngine
    arr = chunk_arr
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("chunk arrays are C-contiguous")
    rank = arr.ndim
    if rank == 0:
        raise ValueError("No dimension passed to chunkWriteSelection")
    if len(slices) != rank:
        raise ValueError("Selection rank does not match dataset rank")
    if len(data.shape) != rank:
        raise ValueError("Input arr does not match dataset rank")
    sel_shape = tuple(len(range(*s.indices(n))) for s, n in zip(slices, arr.shape))
    if tuple(data.shape) != sel_shape:
        raise ValueError(f"could not broadcast input array from shape {data.shape} into shape {sel_shape}")
    data = _write_data(arr.dtype, data)
    if data.size == 0:
        return False
    dev = torch.device("cuda", torch.cuda.current_device())
    d_chunk = _to_dev(arr, dev)
    d_data = _to_dev(data, dev)
    units = write_selection_descs(arr.shape, arr.dtype, tuple(slices), data.shape, data.dtype)
    flags = apply_writes(ChunkEngine(), d_data, d_chunk, [(0, units)], 1)
    updated = bool(flags[0].item())
    if updated:
        np.copyto(arr, d_chunk.cpu().numpy().view(arr.dtype).reshape(arr.shape))
    return updated
