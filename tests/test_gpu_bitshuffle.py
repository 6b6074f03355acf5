"""GPU parity for bitshuffle+LZ4 objects (shuffle = 2; storUtil._unshuffle codec 2,
storUtil.py:144-174): bshuf_kernel through the C ABI against the golden frames of
tests/golden/make_bitshuffle_golden.py (expected results from liblz4 1.9.3 and
imagecodecs' bitshuffle 0.3.5 core) and against the oracle (oracle.c
orc_bitshuffle_decode / _encode).  Bit-exact."""
import hashlib
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


def _dtype(c):
    return np.dtype("S%d" % c["itemsize"]) if c["itemsize"] not in (1, 2, 4, 8, 16) else \
        np.dtype({1: "u1", 2: "<u2", 4: "<u4", 8: "<u8", 16: "<c16"}[c["itemsize"]])


def test_unshuffle_goldens(bshuf_golden, torch_dev):
    from hsds_amd import codec
    meta, arrs = bshuf_golden
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        dt = _dtype(c)
        shape = (c["nbytes"] // c["itemsize"],)
        if c["status"] == "error":
            with pytest.raises(codec.HTTPInternalServerError):
                codec._unshuffle(2, blob, dtype=dt, chunk_shape=shape)
            continue
        out = codec._unshuffle(2, blob, dtype=dt, chunk_shape=shape)
        assert _sha(out) == c["out_sha256"], c["name"]
        # the same through _uncompress(compressor=None, shuffle=2)
        assert codec._uncompress(blob, None, 2, None, dt, shape) == out


def test_batch_mixed_goldens_and_oracle_frames(bshuf_golden, oracle_lib, torch_dev):
    """one hsds_decode_batch over golden frames of every itemsize is not possible (one
    itemsize per call, as per dataset); per itemsize, a batch of goldens + oracle frames
    at unaligned destination offsets"""
    import torch
    from hsds_amd.engine import ChunkEngine, CHUNK_DESC_DTYPE
    meta, arrs = bshuf_golden
    eng = ChunkEngine(0)
    rng = np.random.default_rng(9)
    by_es = {}
    for c in meta["cases"]:
        by_es.setdefault(c["itemsize"], []).append((arrs[c["name"] + "__in"].tobytes(), c["nbytes"],
                                                   c["out_sha256"] if c["status"] == "ok" else None))
    for es, items in by_es.items():
        for k in range(6):
            n = int(rng.integers(1, 40000))
            raw = (np.cumsum(rng.integers(-2, 3, n * es)) % 256).astype(np.uint8).tobytes()
            block = [2048, 256, 0, 8, 64, 1024][k]
            items.append((oracle_lib.bitshuffle_encode(raw, es, block), len(raw), _sha(raw)))
        src_off, dst_off, blob = 0, 0, bytearray()
        descs = np.zeros(len(items), CHUNK_DESC_DTYPE)
        for i, (b, nb, _) in enumerate(items):
            descs[i] = (src_off, len(b), dst_off, nb)
            blob += b + b"\0" * 3
            src_off += len(b) + 3
            dst_off += nb + 5                      # unaligned destinations
        src = torch.from_numpy(np.frombuffer(bytes(blob), np.uint8).copy()).to(torch_dev)
        dst = torch.zeros(dst_off + 8, dtype=torch.uint8, device=torch_dev)
        st = torch.full((len(items),), 99, dtype=torch.int32, device=torch_dev)
        eng.decode(src, descs, dst, st, compressor=None, shuffle=2, itemsize=es)
        torch.cuda.synchronize()
        st_h, dst_h = st.cpu().numpy(), dst.cpu().numpy()
        for i, (b, nb, want) in enumerate(items):
            if want is None:
                assert st_h[i] < 0, (es, i)
                continue
            assert st_h[i] == 0, (es, i, st_h[i])
            o = int(descs[i]["dst_off"])
            assert _sha(dst_h[o:o + nb].tobytes()) == want, (es, i)


def test_outer_codec_then_bitshuffle(oracle_lib, torch_dev):
    """_uncompress(compressor, shuffle=2): the outer codec's output is the bitshuffle
    object (storUtil.py:189-227)"""
    from hsds_amd import codec
    raw = (np.arange(300000, dtype="<f4") * 0.25).tobytes()
    frame = oracle_lib.bitshuffle_encode(raw, 4, 2048)
    shape, dt = (300000,), np.dtype("<f4")
    assert codec._uncompress(zlib.compress(frame), "deflate", 2, None, dt, shape) == raw
    blosc = oracle_lib.blosc_encode(frame, typesize=1, clevel=5, shuffle=0)
    assert codec._uncompress(blosc, "gzip", 2, None, dt, shape) == raw
    with pytest.raises(codec.HTTPInternalServerError):
        codec._uncompress(zlib.compress(frame[:-4]), "deflate", 2, None, dt, shape)


def test_full_size_chunks(oracle_lib, torch_dev):
    """64 x 1 MiB f32 chunks at the HSDS default block (2048 elements): bit-exact"""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    rng = np.random.default_rng(21)
    raws, blobs = [], []
    for i in range(64):
        a = (np.cumsum(rng.standard_normal(262144)) * 0.01).astype("<f4") if i % 2 else \
            rng.integers(0, 1000, 262144).astype("<f4")
        raws.append(a.tobytes())
        blobs.append(oracle_lib.bitshuffle_encode(a.tobytes(), 4, 2048))
    src, descs, ext = pack_chunks(blobs, [1 << 20] * 64)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    st = torch.full((64,), 99, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, st, compressor=None, shuffle=2, itemsize=4)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    h = d_dst.cpu().numpy()
    for i in range(64):
        o = int(descs[i]["dst_off"])
        assert h[o:o + (1 << 20)].tobytes() == raws[i], i


# ---- write path: storUtil._shuffle codec 2 (storUtil.py:103-131) -----------------------

def _walk(frame, nbytes, es):
    """(header, [decoded LZ4 blocks], leftover bytes) of a bitshuffle+LZ4 object, the
    blocks decoded by the oracle's LZ4 decoder."""
    from oracle import oracle as orc
    b = bytes(frame)
    hdr = b[:12]
    bs = int.from_bytes(b[8:12], "big") // es
    if bs == 0:
        bs = max(128, (8192 // es) // 8 * 8)
    n, e, p, blocks = nbytes // es, 0, 12, []
    while e + 8 <= n:
        cnt = bs if n - e >= bs else (n - e) // 8 * 8
        nb = int.from_bytes(b[p:p + 4], "big")
        blk = orc.lz4_decode(b[p + 4:p + 4 + nb], cnt * es)
        assert not isinstance(blk, int), blk
        blocks.append(bytes(blk))
        p += 4 + nb
        e += cnt
    left = b[p:]
    assert len(left) == (n - e) * es
    return hdr, blocks, left


def test_shuffle_codec2_matches_reference_goldens(bshuf_golden, torch_dev):
    """codec._shuffle(2, raw) against the frames the reference's libraries wrote for the
    same raw bytes: identical header, block count, decoded (bit-transposed) block bytes
    and raw leftover; the LZ4 bytes themselves may differ (any valid block)."""
    from hsds_amd import codec
    meta, arrs = bshuf_golden
    n_checked = 0
    for c in meta["cases"]:
        if c["status"] != "ok" or c["block"] != 2048:
            continue
        raw = arrs[c["name"] + "__raw"].tobytes()
        gold = arrs[c["name"] + "__in"].tobytes()
        dt = _dtype(c)
        shape = (c["nbytes"] // c["itemsize"],)
        got = codec._shuffle(2, raw, chunk_shape=shape, dtype=dt)
        assert _walk(got, c["nbytes"], c["itemsize"]) == _walk(gold, c["nbytes"], c["itemsize"]), c["name"]
        assert codec._unshuffle(2, got, dtype=dt, chunk_shape=shape) == raw
        n_checked += 1
    assert n_checked >= 5


def _bshuf_batch(eng, torch, dev, chunks, es, block, src_pad=0, caps=None):
    from hsds_amd import _native as nat
    from hsds_amd.engine import CHUNK_DESC_DTYPE
    descs = np.zeros(len(chunks), CHUNK_DESC_DTYPE)
    srcb, off = [], 0
    for i, c in enumerate(chunks):
        off += src_pad
        srcb.append((off, c))
        off += len(c)
    src = np.zeros(max(off, 1), np.uint8)
    doff = 0
    for i, (o, c) in enumerate(srcb):
        src[o:o + len(c)] = np.frombuffer(c, np.uint8)
        cap = int(nat.lib().hsds_bitshuffle_bound(max(len(c) // es * es, 0), es, block)) if caps is None else caps[i]
        descs[i] = (o, len(c), doff, cap)
        doff += (cap + 3) // 4 * 4
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(max(doff, 1), dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(chunks), dtype=torch.int64, device=dev)
    status = torch.full((len(chunks),), 99, dtype=torch.int32, device=dev)
    eng.encode_bitshuffle(d_src, descs, d_dst, sizes, status, itemsize=es, block=block)
    torch.cuda.synchronize()
    host = d_dst.cpu().numpy()
    st = status.cpu().numpy()
    sz = sizes.cpu().numpy()
    return [host[int(d["dst_off"]):int(d["dst_off"]) + int(s)].tobytes() for d, s in zip(descs, sz)], st, descs


@pytest.mark.parametrize("es,block", [(4, 2048), (1, 2048), (2, 256), (8, 64), (3, 128), (4, 0), (16, 16)])
def test_encode_batch_roundtrip_oracle(torch_dev, es, block):
    """Mixed batch at unaligned source offsets: every object decodes through the oracle
    (orc_bitshuffle_decode, pinned by the reference goldens) and bshuf_kernel to the
    input; headers carry the chunk bytes and block * itemsize as storUtil.py:127-128."""
    import torch
    from hsds_amd.engine import ChunkEngine as Engine
    from oracle import oracle as orc
    eng = Engine(0)
    rng = np.random.default_rng(es * 7 + block)
    chunks = []
    for nel in (0, 5, 8, 1003, 4096, 65536 + 13, 262144):
        kind = len(chunks) % 3
        if kind == 0:
            sm = (np.cumsum(rng.normal(size=max(nel, 1))) * 100).astype("<i8").view(np.uint8)
            x = np.resize(sm, nel * es).astype(np.uint8)
        elif kind == 1:
            x = rng.integers(0, 256, nel * es, dtype=np.uint8)
        else:
            x = np.zeros(nel * es, np.uint8)
        chunks.append(x.tobytes())
    frames, st, _ = _bshuf_batch(eng, torch, torch_dev, chunks, es, block, src_pad=3)
    assert (st == 0).all(), st
    for raw, fr in zip(chunks, frames):
        assert int.from_bytes(fr[:8], "big") == len(raw)
        assert int.from_bytes(fr[8:12], "big") == block * es
        back = orc.bitshuffle_decode(fr, len(raw), es)
        assert not isinstance(back, int), back
        assert bytes(back) == raw
        bs = block or max(128, (8192 // es) // 8 * 8)
        if len(raw) >= bs * es:
            hdr, blocks, left = _walk(fr, len(raw), es)
            assert blocks[0] == orc.bshuf_trans(raw[:bs * es], es)
    # and through the GPU decoder
    from hsds_amd import codec
    for raw, fr in zip(chunks, frames):
        dt = np.dtype("V%d" % es)
        assert codec._unshuffle(2, fr, dtype=dt, chunk_shape=(len(raw) // es,)) == raw


def test_encode_batch_statuses(torch_dev):
    """A capacity below the object size fails that chunk alone (HSDS_ERR_SIZE); a length
    that is not a whole number of elements is an argument error."""
    import torch
    from hsds_amd import _native as nat
    from hsds_amd.engine import ChunkEngine as Engine
    from oracle import oracle as orc
    eng = Engine(0)
    rng = np.random.default_rng(5)
    good = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    frames, st, descs = _bshuf_batch(eng, torch, torch_dev, [good, good[:4003], good], 4, 2048,
                                     caps=[30000, 8000, 40011])
    assert st[0] == nat.ERR_SIZE and st[2] == nat.ERR_SIZE
    assert st[1] == nat.ERR_ARG
    frames, st, _ = _bshuf_batch(eng, torch, torch_dev, [good, good[:4000]], 4, 2048)
    assert (st == 0).all()
    assert bytes(orc.bitshuffle_decode(frames[1], 4000, 4)) == good[:4000]


def test_compress_shuffle2(torch_dev):
    """_compress(shuffle=2) (storUtil.py:238-281): the bitshuffle object alone without a
    compressor, wrapped in a Blosc frame (shuffle off) with one; _uncompress reads both
    back.  A shape that does not match the bytes leaves them unshuffled, as there."""
    from hsds_amd import codec
    from oracle import oracle as orc
    rng = np.random.default_rng(11)
    arr = np.round(np.cumsum(rng.normal(size=(64, 1024)), axis=1), 2).astype("<f4")
    raw = arr.tobytes()
    dt = arr.dtype
    obj = codec._compress(raw, compressor=None, shuffle=2, dtype=dt, chunk_shape=arr.shape)
    assert len(obj) < len(raw)
    assert bytes(orc.bitshuffle_decode(obj, len(raw), 4)) == raw
    assert codec._uncompress(obj, compressor=None, shuffle=2, dtype=dt, chunk_shape=arr.shape) == raw
    for comp in ("gzip", "lz4"):
        fr = codec._compress(raw, compressor=comp, level=5, shuffle=2, dtype=dt, chunk_shape=arr.shape)
        assert fr[3] == 1 and not (fr[2] & 0x01)          # Blosc typesize 1, no byte shuffle
        assert bytes(orc.bitshuffle_decode(orc.blosc_decode(fr, len(obj) + 64), len(raw), 4)) == raw
        assert codec._uncompress(fr, compressor=comp, shuffle=2, dtype=dt, chunk_shape=arr.shape) == raw
    assert codec._compress(raw, compressor=None, shuffle=2, dtype=dt, chunk_shape=(3, 3)) == raw


def test_encode_scratch_sized_by_batch_not_arena(torch_dev):
    """A flush of two dirty chunks out of a 1 GiB cache arena: the engine's scratch (block
    work items, LZ4 token segments, transposition staging) follows the batch's bytes, so
    the device memory it takes stays a few MiB; objects still decode through the oracle."""
    import torch
    from hsds_amd import _native as nat
    from hsds_amd.engine import CHUNK_DESC_DTYPE, ChunkEngine as Engine
    from oracle import oracle as orc
    arena = torch.zeros(1 << 30, dtype=torch.uint8, device=torch_dev)
    rng = np.random.default_rng(11)
    raws = [(np.cumsum(rng.normal(size=65536)) * 10).astype("<f4").tobytes(), rng.bytes(4 * 3001)]
    offs = [(1 << 30) - (3 << 20), (1 << 29) + 4096]
    for o, r in zip(offs, raws):
        arena[o:o + len(r)] = torch.from_numpy(np.frombuffer(r, np.uint8).copy()).to(torch_dev)
    descs = np.zeros(2, CHUNK_DESC_DTYPE)
    doff = 0
    for i, (o, r) in enumerate(zip(offs, raws)):
        cap = int(nat.lib().hsds_bitshuffle_bound(len(r), 4, 2048))
        descs[i] = (o, len(r), doff, cap)
        doff += (cap + 255) // 256 * 256
    dst = torch.zeros(doff, dtype=torch.uint8, device=torch_dev)
    sizes = torch.zeros(2, dtype=torch.int64, device=torch_dev)
    status = torch.full((2,), 99, dtype=torch.int32, device=torch_dev)
    torch.cuda.synchronize()
    eng = Engine(0)
    free0 = torch.cuda.mem_get_info()[0]
    eng.encode_bitshuffle(arena, descs, dst, sizes, status, itemsize=4, block=2048)
    torch.cuda.synchronize()
    used = free0 - torch.cuda.mem_get_info()[0]
    assert used < (96 << 20), used
    assert (status.cpu().numpy() == 0).all()
    host, sz = dst.cpu().numpy(), sizes.cpu().numpy()
    for d, s, r in zip(descs, sz, raws):
        fr = host[int(d["dst_off"]):int(d["dst_off"]) + int(s)].tobytes()
        assert bytes(orc.bitshuffle_decode(fr, len(r), 4)) == r
    # descriptors whose src_len sum exceeds the declared src_bytes fail as an argument error
    status.fill_(99)
    eng.encode_bitshuffle(arena, descs, dst, sizes, status, itemsize=4, block=2048, src_bytes=1024)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() != 0).any()
