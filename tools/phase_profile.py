"""Diagnostic: per-phase cycle breakdown of the inflate kernel (HZ_PROFILE build).
Stamps are s_memtime deltas summed over all waves; only shares are meaningful."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from hsds_amd import _native  # noqa: E402

_native.LIB_PATH = os.environ.get("HZ_PROF_LIB") or os.path.join(ROOT, "tools", "libhsds_prof.so")
L = _native.lib()
L.hsds_debug_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
import torch  # noqa: E402
from bench import make_corpus, CHUNK_BYTES  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402

NAMES = ["other", "blk-hdr", "tables", "A", "A'", "repair", "valid+scan", "E", "M-fill", "trailer", "win-end",
         "M-jump", "M-gather", "M-store", "M-setup", "M-prefetch"]


LZ_NAMES = ["other", "parse", "resolve"]
ZSTD_NAMES = ["other", "lit-stream", "seq-walk", "res-store", "huf-tree", "seq-tables", "res-load", "res-rounds", "seq-lanes", "res-walk"]


def run(fmt, n, unique, tune=None):
    raw, blobs = make_corpus(fmt, unique, 20261015, 16)
    order = [i % unique for i in range(n)]
    src, descs, ext = pack_chunks([blobs[i] for i in order], [CHUNK_BYTES] * n)
    dev = torch.device("cuda", 0)
    eng = ChunkEngine(0)
    if tune:
        eng.set_tuning(**tune)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    comp = {"LZ4": "lz4", "ZSTD": "zstd"}.get(fmt, "zlib")
    eng.decode(d_src, descs, d_dst, d_st, compressor=comp, shuffle=1, itemsize=4)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    L.hsds_debug_profile(buf, 1)
    t = time.perf_counter()
    eng.decode(d_src, descs, d_dst, d_st, compressor=comp, shuffle=1, itemsize=4)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    L.hsds_debug_profile(buf, 1)
    assert (d_st.cpu().numpy() == 0).all()
    tot = sum(buf)
    print(f"{fmt} n={n} tune={tune} wall={el*1e3:.1f} ms  {n*CHUNK_BYTES/el/1e9:.2f} GB/s  kernel={eng.last_inflate_ms():.1f} ms")
    streams = n * 4
    for i in range(16):
        if buf[i]:
            print(f"   {(LZ_NAMES if fmt == 'LZ4' else ZSTD_NAMES if fmt == 'ZSTD' else NAMES)[i]:10s} {100.0*buf[i]/tot:6.2f}%   {buf[i]/streams/1e3:9.1f} kcyc/stream")


if __name__ == "__main__":
    if os.environ.get("HZ_PROF_LONE", "0") == "1":
        # one chunk alone on the GPU (latency): F1 and F2 with one and four wavefronts per stream
        for fmt in ("F1", "F2"):
            for w in (1, 4):
                run(fmt, 1, 1, tune={"waves_per_stream": w})
        sys.exit(0)
    n1 = int(os.environ.get("HZ_PROF_N1", "1024"))
    run("F1", n1, 256)
    if os.environ.get("HZ_PROF_F2W1", "0") == "1":
        # one wavefront per stream (the batch path's one-pass decoder), so the phases are stamped
        run("F2", int(os.environ.get("HZ_PROF_N2", "1024")), 128, tune={"waves_per_stream": 1})
    else:
        run("F2", int(os.environ.get("HZ_PROF_N2", "256")), 128)
    if os.environ.get("HZ_PROF_ZSTD", "0") == "1":
        run("ZSTD", int(os.environ.get("HZ_PROF_NZS", "512")), 128)
    if os.environ.get("HZ_PROF_LZ", "1") == "1":
        run("LZ4", int(os.environ.get("HZ_PROF_NLZ", "1024")), 256)
