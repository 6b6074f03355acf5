"""Blosc frames with many splits per chunk (no per-chunk split cap).

c-blosc 1.21 splits every block of a typesize <= 16 chunk into typesize streams when
blocksize / typesize >= 128 (blosc.c split_block).  At HSDS's max_chunk_size 4m
(admin/config/config.yml:49) lz4 / blosclz level 1 with typesize 4 give exactly 256 splits
(64 KiB blocks x 4); an 8 MiB chunk, which a raised MAX_CHUNK_SIZE allows, gives 512.  The
GPU decoder (frame walk into a pooled item list) and the GPU writer (two-pass compact split
plan) take both, bit-exact against the oracle's c-blosc restatement."""
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


def nsplits(frame):
    h = np.frombuffer(frame[:16], np.uint8)
    flags, ts = int(h[2]), int(h[3])
    nbytes, bs = int(h[4:8].view("<u4")[0]), int(h[8:12].view("<u4")[0])
    nblocks = -(-nbytes // bs)
    full = nbytes // bs
    return full * ts + (nblocks - full) if not flags & 0x10 else nblocks


def _gpu_decode(dev, frames, sizes, compressor, ts):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    src, descs, ext = pack_chunks(frames, sizes)
    dbuf = torch.empty(ext, dtype=torch.uint8, device=dev)
    st = torch.full((len(frames),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.decode(torch.from_numpy(src).to(dev), descs, dbuf, st, compressor=compressor, shuffle=1, itemsize=ts)
    torch.cuda.synchronize()
    out = dbuf.cpu().numpy()
    return st.cpu().numpy(), [out[int(d["dst_off"]):int(d["dst_off"]) + n].tobytes() for d, n in zip(descs, sizes)]


def test_decode_256_and_512_split_frames(dev, oracle_lib):
    orc = oracle_lib
    data = [smooth(1, 4 << 20), smooth(2, 8 << 20), smooth(3, 8 << 20)[:(8 << 20) - 4 * 77], smooth(4, 1 << 20)]
    frames = [orc.blosc_encode_lz4(d, typesize=4, blocksize=65536, shuffle=1) for d in data]
    assert [nsplits(f) for f in frames[:2]] == [256, 512]
    assert nsplits(frames[2]) > 256
    st, outs = _gpu_decode(dev, frames, [len(d) for d in data], "lz4", 4)
    assert (st == 0).all(), st
    for d, o in zip(data, outs):
        assert o == d
    # zlib frames past 256 splits (c-blosc zlib level 1, typesize 4: 128 KiB blocks)
    zdata = [smooth(5, 16 << 20), smooth(6, 4 << 20)]
    zframes = [orc.blosc_encode(d, typesize=4, clevel=1, shuffle=1) for d in zdata]
    assert nsplits(zframes[0]) == 512
    st, outs = _gpu_decode(dev, zframes, [len(d) for d in zdata], "zlib", 4)
    assert (st == 0).all(), st
    for d, o in zip(zdata, outs):
        assert o == d


@pytest.mark.parametrize("cname", ["lz4", "blosclz", "zlib"])
def test_encode_many_split_chunks(dev, oracle_lib, cname):
    """the GPU writer at 256 / 512 / 1024 splits per chunk in one batch with small chunks;
    headers equal c-blosc's geometry, objects decode through the oracle and the GPU"""
    import torch
    from hsds_amd.engine import ChunkEngine, encode_descs
    orc = oracle_lib
    big = {"lz4": 8 << 20, "blosclz": 8 << 20, "zlib": 16 << 20}[cname]
    data = [smooth(10, 4 << 20), smooth(11, big), bytes(1000), smooth(12, big * 2 if cname != "zlib" else 4 << 20)]
    descs, sext, dext = encode_descs([len(d) for d in data])
    src = np.zeros(sext, np.uint8)
    for d, r in zip(data, descs):
        src[int(r["src_off"]):int(r["src_off"]) + len(d)] = np.frombuffer(d, np.uint8)
    d_dst = torch.zeros(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(len(data), dtype=torch.int64, device=dev)
    st = torch.full((len(data),), 99, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(torch.from_numpy(src).to(dev), descs, d_dst, sizes, st, clevel=1, shuffle=1, typesize=4,
               compressor=cname)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all(), st
    out = d_dst.cpu().numpy()
    frames = [out[int(r["dst_off"]):int(r["dst_off"]) + int(n)].tobytes() for r, n in zip(descs, sizes.cpu().numpy())]
    got = [nsplits(f) for f in frames]
    want = [128, 512, 4, 128] if cname == "zlib" else [256, 512, 4, 1024]    # zlib: 128 KiB blocks at L1
    assert got == want, got
    for d, f in zip(data, frames):
        h = np.frombuffer(f[:16], np.uint8)
        assert int(h[8:12].view("<u4")[0]) == orc.blosc_blocksize_codec(1, 4, len(d), cname) or len(d) < 128
        assert orc.uncompress(f, cname, 1, 4, len(d)) == d
    st2, outs = _gpu_decode(dev, frames, [len(d) for d in data], cname, 4)
    assert (st2 == 0).all(), st2
    assert all(o == d for o, d in zip(outs, data))


def test_pool_overflow_fails_only_that_chunk(dev, oracle_lib):
    """a legal frame with more splits than the batch's item pool holds (typesize 16, 2 KiB
    blocks: 16 splits per block, 8192 items for 1 MiB) fails alone with HSDS_ERR_UNSUPPORTED;
    the chunks before and after it in the same batch decode byte-exact (the pool
    fill count never passes its capacity, no consumer reads an unwritten slot)"""
    orc = oracle_lib
    good = [smooth(20 + i, 1 << 20) for i in range(5)]
    bad = smooth(30, 1 << 20)
    bad_frame = orc.blosc_encode_lz4(bad, typesize=16, blocksize=2048, shuffle=1)
    assert nsplits(bad_frame) == 8192
    assert orc.blosc_decode(bad_frame, len(bad)) == bad          # a valid c-blosc frame
    frames = [orc.blosc_encode_lz4(d, typesize=4, blocksize=65536, shuffle=1) for d in good]
    order = [frames[0], frames[1], bad_frame, frames[2], frames[3], frames[4]]
    data = [good[0], good[1], bad, good[2], good[3], good[4]]
    st, outs = _gpu_decode(dev, order, [len(d) for d in data], "lz4", 4)
    assert st[2] == -5, st          # HSDS_ERR_UNSUPPORTED
    for i in (0, 1, 3, 4, 5):
        assert st[i] == 0, st
        assert outs[i] == data[i]
    # the same engine decodes a normal batch afterwards (no stale items left behind)
    st, outs = _gpu_decode(dev, frames, [len(d) for d in good], "lz4", 4)
    assert (st == 0).all(), st
    assert outs == good
