"""Random hsds_copy_desc records and a numpy model of their contract (shared by the CPU
emulation test tests/test_copy_emu.py and the GPU test tests/test_gpu_copy.py): every byte
each record names is moved, and no other byte of the destination changes."""
import numpy as np

def _offsets(counts, strides, base):
    idx = np.indices(counts, dtype=np.int64).reshape(len(counts), -1)
    return base + (idx * np.asarray(strides, np.int64)[:, None]).sum(axis=0)


def _model(src, dst, recs):
    out = dst.copy()
    for r in recs:
        k = int(r["rank"])
        cnt = [int(c) for c in r["count"][:k]]
        isz = int(r["itemsize"])
        so = _offsets(cnt, r["src_stride"][:k], int(r["src_off"]))
        do = _offsets(cnt, r["dst_stride"][:k], int(r["dst_off"]))
        for b in range(isz):
            out[do + b] = src[so + b]
    return out


def _record(rng, src_size, dst_base, kind):
    """one random record whose destination elements are distinct and lie in
    [dst_base, dst_base + returned extent)"""
    from hsds_amd.engine import COPY_DESC_DTYPE
    while True:
        rec, ext, sext = _record_try(rng, dst_base, kind)
        if sext < src_size // 2 and ext < (1 << 19):
            rec["src_off"] = int(rng.integers(0, src_size - sext))
            return rec, ext


def _record_try(rng, dst_base, kind):
    from hsds_amd.engine import COPY_DESC_DTYPE
    rank = int(rng.integers(1, 6))
    isz = int(rng.choice([1, 2, 3, 4, 8, 12, 16])) if kind is None else kind
    counts = [int(rng.integers(1, 9)) for _ in range(rank)]
    counts[-1] = int(rng.choice([1, 3, 17, 64, 100, 257, 1000]))
    # destination: C-contiguous, or a stepped view of a larger C array
    dstep = [int(rng.choice([1, 1, 2, 3])) for _ in range(rank)]
    dshape = [c * s for c, s in zip(counts, dstep)]
    dstr = [isz] * rank
    for k in range(rank - 2, -1, -1):
        dstr[k] = dstr[k + 1] * dshape[k + 1]
    dstr = [a * s for a, s in zip(dstr, dstep)]
    dext = int(np.prod(dshape)) * isz
    # source: contiguous, stepped, or broadcast along some dims
    sstep = [int(rng.choice([0, 1, 1, 1, 2, 5])) for _ in range(rank)]
    sshape = [max(c * s, 1) for c, s in zip(counts, sstep)]
    sstr = [isz] * rank
    for k in range(rank - 2, -1, -1):
        sstr[k] = sstr[k + 1] * sshape[k + 1]
    sstr = [a * s for a, s in zip(sstr, sstep)]
    sext = int(np.prod(sshape)) * isz
    rec = np.zeros(1, COPY_DESC_DTYPE)
    rec["dst_off"] = dst_base + int(rng.integers(0, 40))
    rec["rank"] = rank
    rec["itemsize"] = isz
    rec["count"][0, :rank] = counts
    rec["src_stride"][0, :rank] = sstr
    rec["dst_stride"][0, :rank] = dstr
    return rec, dext + 40, sext


def batch(seed, n=40, kinds=(1, 2, 4, 8)):
    """(src, dst0, records) of one random batch with disjoint destination extents"""
    rng = np.random.default_rng(1000 + seed)
    src = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    recs, base = [], 0
    for i in range(n):
        r, ext = _record(rng, src.size, base, None if i % 2 else int(rng.choice(kinds)))
        recs.append(r)
        base += ext + int(rng.integers(0, 48))
    recs = np.concatenate(recs)
    dst0 = rng.integers(0, 256, base + 64, dtype=np.uint8)
    return src, dst0, recs
