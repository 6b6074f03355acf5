"""Every inflate mode on the GPU, bit-exact against the CPU oracle: one wavefront per zlib
stream (inflate2_kernel, large batches) and two, four or eight wavefronts per stream
(inflate2w_kernel<2|4|8>, the window pipeline used when a batch cannot fill the GPU: lone
GET_Chunk requests, small batches).  Every batch here is decoded in each mode explicitly (hsds_set_tuning's
waves_per_stream), with multi-block streams, stored blocks, F2 1 MiB streams and
corruptions."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _decode(blobs, sizes, mode, shuffle, itemsize):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    dev = torch.device("cuda", 0)
    src, descs, ext = pack_chunks(blobs, sizes)
    eng = ChunkEngine(0)
    eng.set_tuning(waves_per_stream=mode)
    try:
        d_src = torch.from_numpy(src).to(dev)
        d_dst = torch.zeros(ext, dtype=torch.uint8, device=dev)
        d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=dev)
        eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=shuffle, itemsize=itemsize)
        torch.cuda.synchronize()
    finally:
        eng.set_tuning(waves_per_stream=0)
    return d_st.cpu().numpy(), d_dst.cpu().numpy(), descs


def _streams(rng):
    """F2-style zlib streams: smooth shuffled f32 (1 MiB: 30+ blocks), mixed, random
    (stored blocks), zeros, and full-flush pieces (many small blocks of every type)"""
    sm = np.round(np.cumsum(rng.normal(size=1 << 18)), 2).astype(np.float32)
    shuf = sm.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
    out = [shuf, sm.tobytes()[:300001], rng.integers(0, 256, 200000, dtype=np.uint8).tobytes(), bytes(400000)]
    co = zlib.compressobj(6)
    data, c = b"", b""
    for i in range(40):
        piece = rng.integers(0, 256 if i % 3 == 0 else 4, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes()
        data += piece
        c += co.compress(piece) + co.flush(zlib.Z_FULL_FLUSH)
    c += co.flush()
    return out, [zlib.compress(x, lv) for x, lv in zip(out, (4, 1, 6, 9))] + [c], out + [data]


@pytest.mark.parametrize("mode", [1, 2, 4, 8])
def test_zlib_streams_both_modes(mode, oracle_lib):
    rng = np.random.default_rng(31)
    _, blobs, raws = _streams(rng)
    st, out, descs = _decode(blobs, [len(r) for r in raws], mode, 0, 1)
    for k, r in enumerate(raws):
        assert st[k] == 0, (mode, k, st[k])
        o = int(descs[k]["dst_off"])
        assert out[o:o + len(r)].tobytes() == r, (mode, k)


@pytest.mark.parametrize("mode", [1, 2, 4, 8])
def test_f1_frames_both_modes(mode, oracle_lib):
    orc = oracle_lib
    rng = np.random.default_rng(32)
    chunks = [np.round(np.cumsum(rng.normal(size=1 << 18)), 2).astype(np.float32).tobytes() for _ in range(6)]
    blobs = [orc.blosc_encode(c, typesize=1, clevel=4, shuffle=1) for c in chunks]
    st, out, descs = _decode(blobs, [len(c) for c in chunks], mode, 1, 4)
    for k, c in enumerate(chunks):
        assert st[k] == 0
        o = int(descs[k]["dst_off"])
        assert out[o:o + len(c)].tobytes() == c, (mode, k)


@pytest.mark.parametrize("mode", [1, 2, 4, 8])
def test_corruptions_both_modes(mode, oracle_lib):
    orc = oracle_lib
    rng = np.random.default_rng(33)
    base = np.round(np.cumsum(rng.normal(size=200000)), 2).astype(np.float32).tobytes()
    good = zlib.compress(base, 4)                  # several blocks: errors in later windows too
    blobs, sizes = [], []
    for t in range(48):
        b = bytearray(good)
        kind = t % 4
        if kind == 0:
            b = b[:int(rng.integers(2, len(b) - 1))]
        elif kind == 1:
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            b[-1 - int(rng.integers(0, 4))] ^= 0x10
        blobs.append(bytes(b))
        sizes.append(len(base) if kind != 3 else len(base) - 4)
    st, out, descs = _decode(blobs, sizes, mode, 0, 1)
    for k, b in enumerate(blobs):
        ref = orc.uncompress(b, "zlib", 0, 1, sizes[k])
        if isinstance(ref, int):
            assert st[k] < 0, (mode, k, ref, st[k])
        else:
            assert st[k] == 0, (mode, k, st[k])
            o = int(descs[k]["dst_off"])
            assert out[o:o + sizes[k]].tobytes() == ref
