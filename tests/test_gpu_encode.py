"""GPU parity of the write path: hsds_amd encode (C ABI -> HIP kernels) against the CPU
oracle's restatement of storUtil._compress (c-blosc 1.21 frame rules + libz,
pinned byte-for-byte to the reference's own _compress output by
tests/test_oracle_golden.py).

Parity contract: every object the GPU writes must decode to
the original bytes through the oracle's independent frame walker + libz AND
through the GPU decoder; the Blosc header (version, versionlz, flags, typesize,
nbytes, blocksize) must equal the reference's for the same input; the compressed
payload may differ (any valid deflate) and its size is checked against libz's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


def smooth(seed, n):
    rng = np.random.default_rng(seed)
    return np.round(np.cumsum(rng.normal(size=n // 4)), 2).astype(np.float32).tobytes()


def header(frame):
    b = np.frombuffer(frame[:16], np.uint8)
    return dict(version=int(b[0]), versionlz=int(b[1]), flags=int(b[2]), typesize=int(b[3]),
                nbytes=int(b[4:8].view("<u4")[0]), blocksize=int(b[8:12].view("<u4")[0]),
                cbytes=int(b[12:16].view("<u4")[0]))


INPUTS = {
    "smooth_1MiB": lambda: smooth(1, 1 << 20),
    "smooth_256KiB": lambda: smooth(2, 1 << 18),
    "smooth_odd": lambda: smooth(3, 300000) + b"\x01\x02\x03",
    "zeros_1MiB": lambda: bytes(1 << 20),
    "int16": lambda: (np.cumsum(np.random.default_rng(4).normal(size=131072)) * 100).astype("<i2").tobytes(),
    "random_100k": lambda: np.random.default_rng(5).integers(0, 256, 100000, dtype=np.uint8).tobytes(),
    "small_100": lambda: bytes(range(100)),
    "small_200": lambda: bytes(range(200)),
    "empty": lambda: b"",
    "text_40k": lambda: (b"HSDS chunk " * 4000)[:40001],
}


@pytest.mark.parametrize("name", sorted(INPUTS))
@pytest.mark.parametrize("level", [4, 5])
def test_compress_decodes_through_oracle_and_gpu(dev, oracle_lib, name, level):
    from hsds_amd import codec
    orc = oracle_lib
    data = INPUTS[name]()
    frame = codec._compress(data, compressor="zlib", level=level, shuffle=1)
    assert isinstance(frame, bytes)
    ref = orc.blosc_encode(data, typesize=1, clevel=level, shuffle=1)
    h, hr = header(frame), header(ref)
    for k in ("version", "versionlz", "typesize", "nbytes", "blocksize"):
        assert h[k] == hr[k], (k, h, hr)
    if name not in ("random_100k",):   # compressible or tiny: same memcpyed decision as c-blosc
        assert h["flags"] == hr["flags"], (h, hr)
    assert h["cbytes"] == len(frame)
    if data:
        assert orc.uncompress(frame, "zlib", 1, 1, len(data)) == data
        assert codec._uncompress(frame, compressor="zlib", shuffle=1, dtype=np.dtype("u1"),
                                 chunk_shape=(len(data),)) == data


@pytest.mark.parametrize("level", [0, 1, 2, 3, 6, 7, 8, 9])
def test_all_levels(dev, oracle_lib, level):
    from hsds_amd import codec
    data = smooth(10 + level, 1 << 19)
    frame = codec._compress(data, compressor="gzip", level=level, shuffle=1)
    hr = header(oracle_lib.blosc_encode(data, typesize=1, clevel=level, shuffle=1))
    h = header(frame)
    assert (h["flags"], h["blocksize"]) == (hr["flags"], hr["blocksize"])
    assert oracle_lib.uncompress(frame, "zlib", 1, 1, len(data)) == data


def test_size_close_to_libz(dev, oracle_lib):
    from hsds_amd import codec
    ours = ref = 0
    for s in range(6):
        data = smooth(100 + s, 1 << 20)
        ours += len(codec._compress(data, compressor="zlib", level=4, shuffle=1))
        ref += len(oracle_lib.blosc_encode(data, typesize=1, clevel=4, shuffle=1))
    assert ours / ref < 1.06, ours / ref


def test_compress_passthrough_and_errors(dev):
    from hsds_amd import codec
    data = b"abc" * 100
    assert codec._compress(data) is data                 # no compressor: unchanged (storUtil.py:239-241)
    assert codec._compress(data, compressor=None, shuffle=1) is data
    # shuffle=2 without a dtype: _shuffle fails, the reference logs it and Blosc-encodes
    # the bytes unshuffled (storUtil.py:243-251)
    fr = codec._compress(data, compressor="zlib", shuffle=2)
    assert fr[2] >> 5 == 3 and not (fr[2] & 1)
    assert codec._uncompress(fr, compressor="zlib") == data
    with pytest.raises(NotImplementedError):     # snappy: no Blosc build of the reference has it
        codec._compress(data, compressor="snappy")
    assert codec._compress(data, compressor="zstd")[2] >> 5 == 4



@pytest.mark.parametrize("ts", [2, 4, 8, 32])
def test_batch_typesize_shuffle(dev, oracle_lib, ts):
    # Blosc frames with typesize > 1 (in-frame byte shuffle, one split per byte plane
    # when ts <= 16); the reference's _compress never writes them but the ABI does
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs
    data = [smooth(200 + ts, 1 << 18), smooth(300 + ts, 65536 * 3 + 4 * ts), bytes(70000 // ts * ts)]
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(max(sext, 1), np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(d_src, descs, d_dst, sizes, st, clevel=5, shuffle=1, typesize=ts)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    out = d_dst.cpu().numpy()
    for d, r, n in zip(data, descs, sizes.cpu().numpy()):
        frame = out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes()
        hr = header(oracle_lib.blosc_encode(d, typesize=ts, clevel=5, shuffle=1))
        h = header(frame)
        assert (h["typesize"], h["blocksize"], h["flags"]) == (hr["typesize"], hr["blocksize"], hr["flags"])
        assert oracle_lib.uncompress(frame, "zlib", 1, ts, len(d)) == d


def test_batch_mixed_matches_oracle_and_gpu_decode(dev, oracle_lib):
    # one batch of mixed chunks, then the GPU decoder reads the objects back
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs, pack_chunks
    rng = np.random.default_rng(9)
    data = []
    for i in range(48):
        k = i % 4
        if k == 0:
            data.append(smooth(400 + i, 1 << 20))
        elif k == 1:
            data.append((np.cumsum(rng.normal(size=131072)) * 100).astype("<i2").tobytes())
        elif k == 2:
            data.append(rng.integers(0, 256, 1 << 18, dtype=np.uint8).tobytes())
        else:
            data.append(bytes(1 << 20))
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(sext, np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(d_src, descs, d_dst, sizes, st, clevel=4, shuffle=1, typesize=1)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    out = d_dst.cpu().numpy()
    frames = [out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes() for r, n in zip(descs, sizes.cpu().numpy())]
    for d, f in zip(data, frames):
        assert oracle_lib.uncompress(f, "zlib", 1, 1, len(d)) == d
    # GPU decode of the GPU-written objects
    psrc, pdescs, ext = pack_chunks(frames, [len(d) for d in data])
    g_src = torch.from_numpy(psrc).to(dev)
    g_dst = torch.zeros(ext, dtype=torch.uint8, device=dev)
    g_st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng.decode(g_src, pdescs, g_dst, g_st, compressor="zlib", shuffle=1, itemsize=1)
    torch.cuda.synchronize()
    assert (g_st.cpu().numpy() == 0).all()
    dec = g_dst.cpu().numpy()
    for d, r in zip(data, pdescs):
        assert dec[int(r["dst_off"]):int(r["dst_off"]) + len(d)].tobytes() == d
    assert eng.last_deflate_ms() > 0


def test_encode_rejects_small_capacity(dev):
    import torch
    from hsds_amd import _native as nat
    from hsds_amd.engine import ChunkEngine, encode_descs
    descs, sext, dext = encode_descs([4096])
    descs[0]["dst_len"] = 4096          # < src_len + 16
    d_src = torch.zeros(sext, dtype=torch.uint8, device=dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    ChunkEngine(0).encode(d_src, descs, d_dst, sizes, st, clevel=4)
    torch.cuda.synchronize()
    assert int(st[0]) == nat.ERR_ARG


def test_streams_equal_cpu_emulation(dev):
    """The GPU kernels and the CPU emulation run the same single-source encoder
    (deflate_wave.h), so every zlib stream of a GPU frame must equal the emulator's
    bytes for the same split: this pins the wave-level orchestration (chain sort,
    lane ranges, Huffman build, bit placement) beyond "it inflates"."""
    import ctypes
    import os
    from hsds_amd import codec
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "libdeflate_emu.so")
    L = ctypes.CDLL(lib)
    L.emu_deflate.restype = ctypes.c_int64
    L.emu_deflate.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                              ctypes.c_int]
    for seed, level, n in ((1, 4, 1 << 20), (2, 1, 1 << 19), (3, 9, 300000), (4, 5, 70001), (5, 6, 262144)):
        data = smooth(seed, n - n % 4) + bytes(n % 4)
        if seed == 5:   # repeats 20 000 bytes back: the far chain ring in HBM (levels >= 6)
            blk = np.random.default_rng(seed).integers(0, 256, 20000, dtype=np.uint8).tobytes()
            data = (blk * 14)[:n]
        frame = codec._compress(data, compressor="zlib", level=level, shuffle=1)
        h = header(frame)
        assert not (h["flags"] & 0x02)
        bs, nblocks = h["blocksize"], (h["nbytes"] + h["blocksize"] - 1) // h["blocksize"]
        fb = np.frombuffer(frame, np.uint8)
        for b in range(nblocks):
            start = int(fb[16 + 4 * b:20 + 4 * b].view("<i4")[0])
            cs = int(fb[start:start + 4].view("<i4")[0])
            blk = np.frombuffer(data[b * bs:(b + 1) * bs], np.uint8)
            out = np.zeros((len(blk) + 4096) // 4 + 8, np.uint32)
            r = L.emu_deflate(blk.ctypes.data, len(blk), out.ctypes.data, len(blk) + 4096, level, 0)
            assert r == cs, (seed, b, r, cs)
            assert out.view(np.uint8)[:r].tobytes() == fb[start + 4:start + 4 + cs].tobytes(), (seed, b)


def test_lz4_streams_equal_cpu_emulation(dev):
    """Blosc-lz4 objects are parsed with the approximate chains (level + 100): the hash head
    of a step is its highest lane with that hash, on the GPU as in the emulator, so every
    LZ4 block the GPU writes equals the emulator's block byte for byte."""
    import ctypes
    import os
    from hsds_amd import codec
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "libdeflate_emu.so")
    L = ctypes.CDLL(lib)
    L.emu_lz4_block.restype = ctypes.c_int64
    L.emu_lz4_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    rng = np.random.default_rng(9)
    inputs = [smooth(5, 1 << 20), rng.integers(0, 4, 400000, dtype=np.uint8).tobytes(),
              (np.arange(300000) % 97).astype(np.uint8).tobytes()]
    for k, data in enumerate(inputs):
        for level in (1, 5, 9):
            frame = codec._compress(data, compressor="lz4", level=level, shuffle=1)
            h = header(frame)
            if h["flags"] & 0x02:
                continue                        # memcpyed: no LZ4 block
            bs, nblocks = h["blocksize"], (h["nbytes"] + h["blocksize"] - 1) // h["blocksize"]
            fb = np.frombuffer(frame, np.uint8)
            for b in range(nblocks):
                start = int(fb[16 + 4 * b:20 + 4 * b].view("<i4")[0])
                cs = int(fb[start:start + 4].view("<i4")[0])
                blk = np.frombuffer(data[b * bs:(b + 1) * bs], np.uint8)
                if cs == len(blk):
                    continue                    # raw split
                out = np.zeros(len(blk) + 4096, np.uint8)
                r = L.emu_lz4_block(blk.ctypes.data, len(blk), out.ctypes.data, out.size, level)
                assert r == cs, (k, level, b, r, cs)
                assert out[:r].tobytes() == fb[start + 4:start + 4 + cs].tobytes(), (k, level, b)


# ---- the lz4 / lz4hc write path (Blosc codec 1, LZ4 blocks from the parse tokens) ----

@pytest.mark.parametrize("name", sorted(INPUTS))
@pytest.mark.parametrize("cname,level", [("lz4", 5), ("lz4hc", 5), ("lz4", 1), ("lz4", 9), ("blosclz", 5),
                                         ("blosclz", 9)])
def test_lz4_compress_decodes_through_oracle_and_gpu(dev, oracle_lib, name, cname, level):
    """storUtil._compress(compressor="lz4"/"lz4hc"): header fields as c-blosc 1.21
    writes them for that codec (blocksize rule pinned by the codec2 golden table),
    and the object decodes to the input through the oracle and the GPU decoder."""
    from hsds_amd import codec
    data = INPUTS[name]()
    frame = codec._compress(data, compressor=cname, level=level, shuffle=1)
    h = header(frame)
    n = len(data)
    bs = oracle_lib.blosc_blocksize_codec(level, 1, n, cname)
    assert (h["version"], h["versionlz"], h["typesize"], h["nbytes"], h["blocksize"]) == (2, 1, 1, n, bs)
    assert h["cbytes"] == len(frame) <= n + 16
    assert h["flags"] & 0xE1 == (0x01 if cname == "blosclz" else 0x21)    # codec 0 / 1, shuffle flag
    assert bool(h["flags"] & 0x02) == (n < 128 or h["flags"] & 0x02 != 0)
    assert oracle_lib.uncompress(frame, cname, 1, 1, n) == data
    if n:
        assert codec._uncompress(frame, compressor=cname, shuffle=1, dtype=np.dtype("u1"), chunk_shape=(n,)) == data


@pytest.mark.parametrize("ts", [2, 4, 8, 32])
@pytest.mark.parametrize("cname", ["lz4", "blosclz"])
def test_lz4_batch_typesize_shuffle(dev, oracle_lib, ts, cname):
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs
    data = [smooth(500 + ts, 1 << 18), smooth(600 + ts, 65536 * 3 + 4 * ts), bytes(70000 // ts * ts)]
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(max(sext, 1), np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(d_src, descs, d_dst, sizes, st, clevel=5, shuffle=1, typesize=ts, compressor=cname)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    out = d_dst.cpu().numpy()
    for d, r, n in zip(data, descs, sizes.cpu().numpy()):
        frame = out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes()
        h = header(frame)
        assert h["typesize"] == ts and h["blocksize"] == oracle_lib.blosc_blocksize_codec(5, ts, len(d), cname)
        assert bool(h["flags"] & 0x10) == (not (ts <= 16 and h["blocksize"] // ts >= 128))
        assert oracle_lib.uncompress(frame, cname, 1, ts, len(d)) == d


def test_lz4_batch_mixed_gpu_roundtrip(dev, oracle_lib):
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs, pack_chunks
    rng = np.random.default_rng(19)
    data = []
    for i in range(40):
        k = i % 4
        data.append(smooth(700 + i, 1 << 20) if k == 0 else
                    (np.cumsum(rng.normal(size=131072)) * 100).astype("<i2").tobytes() if k == 1 else
                    rng.integers(0, 256, 1 << 18, dtype=np.uint8).tobytes() if k == 2 else
                    np.repeat(rng.integers(0, 9, 4000), 97).astype("<i4").tobytes())
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(sext, np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(d_src, descs, d_dst, sizes, st, clevel=5, shuffle=1, typesize=1, compressor="lz4")
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    out = d_dst.cpu().numpy()
    frames = [out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes() for r, n in zip(descs, sizes.cpu().numpy())]
    for d, f in zip(data, frames):
        assert oracle_lib.uncompress(f, "lz4", 1, 1, len(d)) == d
    psrc, pdescs, ext = pack_chunks(frames, [len(d) for d in data])
    g_src = torch.from_numpy(psrc).to(dev)
    g_dst = torch.zeros(ext, dtype=torch.uint8, device=dev)
    g_st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng.decode(g_src, pdescs, g_dst, g_st, compressor="lz4", shuffle=1, itemsize=1)
    torch.cuda.synchronize()
    assert (g_st.cpu().numpy() == 0).all()
    dec = g_dst.cpu().numpy()
    for d, r in zip(data, pdescs):
        assert dec[int(r["dst_off"]):int(r["dst_off"]) + len(d)].tobytes() == d


# ---- the zstd write path (Blosc codec 4, zstd_enc.h blocks from the parse tokens) ----

def _libblosc():
    import ctypes
    import os
    p = "/opt/conda/lib/libblosc.so.1"
    if not os.path.exists(p):
        pytest.skip("libblosc absent")
    lb = ctypes.CDLL(p)
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    lb.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return lb


@pytest.mark.parametrize("name", sorted(INPUTS))
@pytest.mark.parametrize("level", [1, 5, 9])
def test_zstd_compress_matches_libblosc_geometry_and_decodes(dev, oracle_lib, name, level):
    """storUtil._compress(compressor="zstd"): the Blosc header (flags, typesize, nbytes,
    blocksize) equals libblosc 1.21's for the same input and level, and the object decodes
    to the input through libblosc's own blosc_decompress (the reference's c-blosc), the
    oracle and the GPU decoder."""
    from hsds_amd import codec
    lb = _libblosc()
    data = INPUTS[name]()
    n = len(data)
    frame = codec._compress(data, compressor="zstd", level=level, shuffle=1)
    h = header(frame)
    a = np.frombuffer(data, np.uint8) if n else np.zeros(1, np.uint8)
    ref = np.empty(n + 64, np.uint8)
    k = lb.blosc_compress_ctx(level, 1, 1, n, a.ctypes.data, ref.ctypes.data, ref.size, b"zstd", 0, 1)
    assert k > 0
    r = header(ref[:k].tobytes())
    assert (h["version"], h["typesize"], h["nbytes"], h["blocksize"]) == (r["version"], r["typesize"], r["nbytes"],
                                                                          r["blocksize"])
    if not (h["flags"] & 0x02) and not (r["flags"] & 0x02):
        assert h["flags"] == r["flags"]
    assert h["cbytes"] == len(frame) <= n + 16
    if n:
        back = np.zeros(n, np.uint8)
        f = np.frombuffer(frame, np.uint8)
        assert lb.blosc_decompress_ctx(f.ctypes.data, back.ctypes.data, n, 1) == n
        assert back.tobytes() == data
        assert oracle_lib.uncompress(frame, "zstd", 1, 1, n) == data
        assert codec._uncompress(frame, compressor="zstd", shuffle=1, dtype=np.dtype("u1"), chunk_shape=(n,)) == data


@pytest.mark.parametrize("ts", [2, 4, 8, 32])
def test_zstd_batch_typesize_shuffle(dev, oracle_lib, ts):
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs, pack_chunks
    data = [smooth(800 + ts, 1 << 18), smooth(900 + ts, 65536 * 3 + 4 * ts), bytes(70000 // ts * ts),
            smooth(950 + ts, 1 << 20)]
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(max(sext, 1), np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(d_src, descs, d_dst, sizes, st, clevel=5, shuffle=1, typesize=ts, compressor="zstd")
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    out = d_dst.cpu().numpy()
    frames = [out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes() for r, n in zip(descs, sizes.cpu().numpy())]
    for d, f in zip(data, frames):
        h = header(f)
        assert h["typesize"] == ts and h["flags"] & 0x10 and h["flags"] >> 5 == 4
        assert oracle_lib.uncompress(f, "zstd", 1, ts, len(d)) == d
    # and back through the GPU decoder (zstd_kernel + unshuffle)
    psrc, pdescs, ext = pack_chunks(frames, [len(d) for d in data])
    g_dst = torch.zeros(ext, dtype=torch.uint8, device=dev)
    g_st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng.decode(torch.from_numpy(psrc).to(dev), pdescs, g_dst, g_st, compressor="zstd", shuffle=1, itemsize=ts)
    torch.cuda.synchronize()
    assert (g_st.cpu().numpy() == 0).all()
    got = g_dst.cpu().numpy()
    for d, r in zip(data, pdescs):
        assert got[int(r["dst_off"]):int(r["dst_off"]) + len(d)].tobytes() == d


def test_zstd_streams_equal_cpu_emulation(dev):
    """The GPU zstd writer and the CPU emulation run the same source (zstd_enc.h over the
    deflate parse): every split's zstd frame equals the emulator's bytes."""
    import ctypes
    import os
    from hsds_amd import codec
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "libdeflate_emu.so")
    L = ctypes.CDLL(lib)
    L.emu_zstd_frame.restype = ctypes.c_int64
    L.emu_zstd_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    for seed, level, n in ((1, 5, 1 << 20), (2, 1, 1 << 19), (3, 9, 300000), (4, 6, 70001)):
        data = smooth(seed, n - n % 4) + bytes(n % 4)
        frame = codec._compress(data, compressor="zstd", level=level, shuffle=1)
        h = header(frame)
        assert not (h["flags"] & 0x02)
        bs, nblocks = h["blocksize"], (h["nbytes"] + h["blocksize"] - 1) // h["blocksize"]
        fb = np.frombuffer(frame, np.uint8)
        for b in range(nblocks):
            start = int(fb[16 + 4 * b:20 + 4 * b].view("<i4")[0])
            cs = int(fb[start:start + 4].view("<i4")[0])
            blk = np.frombuffer(data[b * bs:(b + 1) * bs], np.uint8)
            if cs == len(blk):
                continue                    # raw split
            out = np.zeros(len(blk) + 4096, np.uint8)
            r = L.emu_zstd_frame(blk.ctypes.data, len(blk), out.ctypes.data, out.size, level)
            assert r == cs, (seed, b, r, cs)
            assert out[:r].tobytes() == fb[start + 4:start + 4 + cs].tobytes(), (seed, b)


@pytest.mark.parametrize("cname", ["zlib", "lz4", "zstd"])
def test_full_size_roundtrip_configs1(dev, oracle_lib, cname):
    """BASELINE.json configs[1] at full size (4096 x 1 MiB f32 chunks, 4 GiB): GPU encode ->
    GPU decode is the identity on every byte (compared on the device), and sampled frames
    decode through the oracle to the same chunks (size-independent round-trip property)."""
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs, to_device_bytes
    n, cb = 4096, 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    chunks = torch.empty(n * cb, dtype=torch.uint8, device=dev)
    view = chunks.view(torch.float32).view(n, cb // 4)
    for k in range(0, n, 512):
        z = torch.randn((512, cb // 4), generator=g, device=dev, dtype=torch.float32)
        view[k:k + 512] = torch.round(torch.cumsum(z, dim=1) * 100) / 100
        del z
    descs, _, dext = encode_descs([cb] * n)
    frames = torch.empty(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(n, dtype=torch.int64, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(chunks, to_device_bytes(descs, dev), frames, sizes, st, clevel=4, shuffle=1, typesize=1,
               compressor=cname)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    # decode straight from the frame slots (dst_off of the encode descriptors)
    ddescs = descs.copy()
    ddescs["src_off"], ddescs["src_len"] = descs["dst_off"], sizes.cpu().numpy()
    ddescs["dst_off"], ddescs["dst_len"] = descs["src_off"], cb
    back = torch.empty_like(chunks)
    dst = torch.full((n,), 99, dtype=torch.int32, device=dev)
    eng.decode(frames, to_device_bytes(ddescs, dev), back, dst, compressor="zlib" if cname == "zlib" else cname,
               shuffle=1, itemsize=1)
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert torch.equal(back, chunks)
    hs = sizes.cpu().numpy()
    for k in (0, 1234, n - 1):
        o = int(descs[k]["dst_off"])
        fr = frames[o:o + int(hs[k])].cpu().numpy().tobytes()
        assert oracle_lib.uncompress(fr, cname, 1, 1, cb) == chunks[k * cb:(k + 1) * cb].cpu().numpy().tobytes()
