"""GPU parity: hsds_amd decode (C ABI -> HIP kernels) vs the reference goldens and the
CPU oracle.  Bit-exact (lossless codecs)."""
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


def test_native_library_is_loaded(torch_dev):
    from hsds_amd import _native
    assert _native.lib().hsds_version().startswith(b"hsds_amd")
    _native.engine(0)


def test_uncompress_matches_reference_goldens(golden, torch_dev):
    from hsds_amd import codec
    meta, arrs = golden
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        dtype = np.dtype(c["dtype"]) if c["dtype"] else None
        shape = tuple(c["chunk_shape"]) if c["chunk_shape"] else None
        kw = dict(compressor=c["compressor"], shuffle=c["shuffle"], level=c["level"], dtype=dtype, chunk_shape=shape)
        if c["status"] == "error":
            with pytest.raises(codec.HTTPInternalServerError):
                codec._uncompress(blob, **kw)
            continue
        out = codec._uncompress(blob, **kw)
        assert len(out) == c["out_len"], c["name"]
        assert _sha(out) == c["out_sha256"], c["name"]


def test_zlib_without_chunk_shape(torch_dev):
    # compression_test.testZLibCompression: dtype only, size unknown
    from hsds_amd import codec
    arr = np.random.default_rng(1).integers(0, 200, 1_000_000, dtype="<i4")
    out = codec._uncompress(zlib.compress(arr.tobytes()), compressor="zlib", dtype=arr.dtype)
    assert out == arr.tobytes()


def test_shuffle_kat(golden, torch_dev):
    from hsds_amd import codec
    meta, _ = golden
    kat = meta["shuffle_kat"]
    data = bytes.fromhex(kat["in"])
    sh = codec._shuffle(1, data, chunk_shape=(3,), dtype=np.dtype("<u2"))
    assert sh.hex() == kat["shuffled"]
    assert codec._unshuffle(1, sh, dtype=np.dtype("<u2"), chunk_shape=(3,)).hex() == kat["unshuffled"]
    for c in meta["shuffle_cases"]:
        data = bytes.fromhex(c["in"])
        dt = np.dtype(c["dtype"])
        assert codec._shuffle(1, data, chunk_shape=(c["n"],), dtype=dt).hex() == c["shuffled"]
        assert codec._unshuffle(1, bytes.fromhex(c["shuffled"]), dtype=dt, chunk_shape=(c["n"],)) == data


def _corpus(rng, n, size, kind):
    out = []
    for i in range(n):
        if kind == "smooth":
            a = np.round(np.cumsum(rng.normal(size=size // 4)), 2).astype(np.float32).tobytes()
        elif kind == "int16":
            a = (np.cumsum(rng.normal(size=size // 2)) * 100).astype("<i2").tobytes()
        elif kind == "zeros":
            a = bytes(size)
        elif kind == "random":
            a = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        else:  # mixed
            a = (np.round(np.cumsum(rng.normal(size=size // 8)), 1).astype(np.float32).tobytes()
                 + rng.integers(0, 4, size // 2, dtype=np.uint8).tobytes())
        out.append(a[:size])
    return out


@pytest.mark.parametrize("fmt,kind,size,level", [
    ("F1", "smooth", 1 << 20, 4), ("F1", "smooth", 262144, 1), ("F1", "int16", 262144, 4),
    ("F1", "zeros", 1 << 20, 4), ("F1", "random", 65536, 4), ("F1", "mixed", 300000, 9),
    ("F2", "smooth", 1 << 20, 4), ("F2", "int16", 262144, 4), ("F2", "mixed", 500000, 1),
    ("F2", "zeros", 262144, 6), ("F2", "random", 100000, 4), ("F2", "smooth", 65536, 0),
    ("F1ts4", "smooth", 1 << 20, 4), ("F1ts8", "smooth", 262144 + 1000 * 8, 5),
])
def test_batch_decode_matches_oracle(fmt, kind, size, level, oracle_lib, torch_dev):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    rng = np.random.default_rng(abs(hash((fmt, kind, size, level))) % (1 << 32))
    chunks = _corpus(rng, 12, size, kind)
    itemsize = 4 if kind in ("smooth", "mixed", "zeros", "random") else 2
    if fmt == "F1":
        blobs = [orc.blosc_encode(c, typesize=1, clevel=level, shuffle=1) for c in chunks]
    elif fmt.startswith("F1ts"):
        ts = int(fmt[4:])
        blobs = [orc.blosc_encode(c, typesize=ts, clevel=level, shuffle=1) for c in chunks]
    else:
        blobs = [zlib.compress(orc.shuffle(c, itemsize), level) for c in chunks]
    src, descs, ext = pack_chunks(blobs, [len(c) for c in chunks])
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=itemsize)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    for k, c in enumerate(chunks):
        ref = orc.uncompress(blobs[k], "zlib", 1, itemsize, len(c))
        assert not isinstance(ref, int)
        assert st[k] == 0, (k, st[k])
        o = int(descs[k]["dst_off"])
        assert out[o:o + len(c)].tobytes() == ref, k


def test_error_statuses(oracle_lib, torch_dev):
    """Corrupt / truncated / mis-sized streams fail exactly when the oracle fails."""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    rng = np.random.default_rng(5)
    base = np.round(np.cumsum(rng.normal(size=65536)), 2).astype(np.float32).tobytes()
    good = zlib.compress(base, 4)
    blobs, sizes = [], []
    for t in range(60):
        b = bytearray(good)
        kind = t % 4
        if kind == 0:
            b = b[:rng.integers(2, len(b) - 1)]
        elif kind == 1:
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            b[-1 - int(rng.integers(0, 4))] ^= 0x10
        blobs.append(bytes(b))
        sizes.append(len(base) if kind != 3 else len(base) - 4)
    src, descs, ext = pack_chunks(blobs, sizes)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=0, itemsize=1)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    for k, b in enumerate(blobs):
        ref = orc.uncompress(b, "zlib", 0, 1, sizes[k])
        if isinstance(ref, int):
            assert st[k] < 0, (k, ref, st[k])
        else:
            assert st[k] == 0, (k, st[k])
            o = int(descs[k]["dst_off"])
            assert out[o:o + sizes[k]].tobytes() == ref


def test_other_blosc_codecs_match_reference_goldens(golden2, torch_dev):
    """lz4 / lz4hc / blosclz / zstd objects of the reference (codec2 goldens) through
    _uncompress on the GPU: every byte and every error; a truncated object is rejected
    (the reference reads past its end)."""
    from hsds_amd import codec
    meta, arrs = golden2
    checked = 0
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        kw = dict(compressor=c["compressor"], shuffle=c["shuffle"], level=c["level"],
                  dtype=np.dtype(c["dtype"]), chunk_shape=tuple(c["chunk_shape"]))
        if c["status"] == "error" or c["name"].endswith("_trunc"):
            with pytest.raises(codec.HTTPInternalServerError):
                codec._uncompress(blob, **kw)
            continue
        out = codec._uncompress(blob, **kw)
        assert len(out) == c["out_len"] and _sha(out) == c["out_sha256"], c["name"]
        checked += 1
    assert checked >= 90


@pytest.mark.parametrize("kind,size,ts,bs", [
    ("smooth", 1 << 20, 1, 131072), ("smooth", 1 << 20, 4, 262144), ("int16", 262144, 2, 65536),
    ("zeros", 1 << 20, 1, 131072), ("random", 65536, 1, 32768), ("mixed", 300000 + 5, 1, 65536),
    ("mixed", 500000, 8, 524288),
])
def test_batch_decode_lz4_matches_oracle(kind, size, ts, bs, oracle_lib, torch_dev):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    rng = np.random.default_rng(abs(hash(("lz4", kind, size, ts))) % (1 << 32))
    chunks = _corpus(rng, 16, size, kind)
    blobs = [orc.blosc_encode_lz4(c, typesize=ts, blocksize=bs, shuffle=1) for c in chunks]
    src, descs, ext = pack_chunks(blobs, [len(c) for c in chunks])
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="lz4", shuffle=1, itemsize=ts)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    for k, c in enumerate(chunks):
        assert orc.uncompress(blobs[k], "lz4", 1, ts, len(c)) == c
        assert st[k] == 0, (k, st[k])
        o = int(descs[k]["dst_off"])
        assert out[o:o + len(c)].tobytes() == c, k


def test_lz4_blosclz_error_statuses(golden2, oracle_lib, torch_dev):
    """corrupted lz4 / blosclz frames in one batch: status < 0 exactly where the oracle
    fails, identical bytes where it decodes."""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    meta, arrs = golden2
    rng = np.random.default_rng(11)
    blobs, sizes = [], []
    for c in meta["cases"]:
        if c["codec"] not in (0, 1) or c["memcpyed"] or c["in_len"] > 300000:
            continue
        good = arrs[c["name"] + "__in"].tobytes()
        n = int(np.prod(c["chunk_shape"])) * np.dtype(c["dtype"]).itemsize
        for t in range(3):
            b = bytearray(good)
            i = int(rng.integers(16, len(b)))
            b[i] ^= int(rng.integers(1, 256))
            blobs.append(bytes(b))
            sizes.append(n)
    src, descs, ext = pack_chunks(blobs, sizes)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="lz4", shuffle=1, itemsize=1)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    assert len(blobs) >= 60
    for k, b in enumerate(blobs):
        ref = orc.uncompress(b, "lz4", 1, 1, sizes[k])
        if isinstance(ref, int):
            assert st[k] < 0, (k, ref, st[k])
        else:
            assert st[k] == 0, (k, st[k])
            o = int(descs[k]["dst_off"])
            assert out[o:o + sizes[k]].tobytes() == ref, k


def test_batch_decode_zstd_goldens_with_oracle(golden2, oracle_lib, torch_dev):
    """every zstd golden object (and mixed lz4 / zlib neighbours) in ONE batch: status
    and bytes against the oracle's zstd restatement"""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    meta, arrs = golden2
    blobs, sizes, names = [], [], []
    for c in meta["cases"]:
        if c["codec"] not in (1, 4) or c["name"].endswith("_trunc"):
            continue
        blobs.append(arrs[c["name"] + "__in"].tobytes())
        sizes.append(int(np.prod(c["chunk_shape"])) * np.dtype(c["dtype"]).itemsize)
        names.append(c["name"])
    src, descs, ext = pack_chunks(blobs, sizes)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="zstd", shuffle=1, itemsize=1)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    nz = 0
    for k, b in enumerate(blobs):
        ref = orc.uncompress(b, "zstd", 1, 1, sizes[k])
        if isinstance(ref, int):
            assert st[k] < 0, names[k]
        else:
            assert st[k] == 0, (names[k], st[k])
            o = int(descs[k]["dst_off"])
            assert out[o:o + sizes[k]].tobytes() == ref, names[k]
            nz += "zstd" in names[k]
    assert nz >= 40


def test_batch_decode_zstd_literal_heavy(torch_dev):
    """Blosc-zstd frames (the image's libblosc 1.21) of literal-heavy data in ONE batch: the
    Huffman literal streams decoded on every lane (zstd_wave.h huf_streams_wave) -- skewed
    and near-uniform bytes, text with noise, one- and four-stream literal sections, levels
    1 / 5 / 9 -- decode to their input"""
    import ctypes
    import os
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    if not os.path.exists("/opt/conda/lib/libblosc.so.1"):
        pytest.skip("the image's libblosc is absent")
    lb = ctypes.CDLL("/opt/conda/lib/libblosc.so.1")
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    rng = np.random.default_rng(62)
    raws, blobs = [], []
    for n in (40, 300, 1500, 5000, 40000, 131072, 300000, 1 << 20):
        for kind in range(3):
            if kind == 0:
                a = np.minimum(rng.geometric(0.08, n), 255).astype(np.uint8)
            elif kind == 1:
                a = (rng.integers(0, 200, n) + (np.arange(n) % 7)).astype(np.uint8)
            else:
                a = np.frombuffer((b"the quick brown fox %d jumps " * (n // 20 + 1))[:n], np.uint8).copy()
                a[rng.integers(0, n, n // 5)] = rng.integers(0, 256, n // 5).astype(np.uint8)
            for level in (1, 5, 9):
                out = np.zeros(a.size + 64, np.uint8)
                k = lb.blosc_compress_ctx(level, 0, 1, a.size, a.ctypes.data, out.ctypes.data, out.size, b"zstd", 0, 1)
                assert k > 0
                raws.append(a)
                blobs.append(out[:k].tobytes())
    src, descs, ext = pack_chunks(blobs, [a.size for a in raws])
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="zstd", shuffle=0, itemsize=1)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    for k, a in enumerate(raws):
        assert st[k] == 0, (k, a.size, st[k])
        o = int(descs[k]["dst_off"])
        assert out[o:o + a.size].tobytes() == a.tobytes(), (k, a.size)
