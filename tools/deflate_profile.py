"""Diagnostic: per-phase cycle breakdown of the deflate kernel (HZ_PROFILE build,
tools/libhsds_prof.so).  s_memtime deltas summed over all waves; shares only."""
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
from hsds_amd.engine import ChunkEngine, encode_descs  # noqa: E402

NAMES = ["other", "stage", "chains", "parse", "", "", "", "", "", "adler", "", "", "", "", "", ""]


def main():
    n = int(os.environ.get("HZ_PROF_N", "512"))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    z = torch.randn((n, 262144), generator=g, device=dev, dtype=torch.float64)
    data = torch.round(torch.cumsum(z, dim=1), decimals=2).to(torch.float32).view(torch.uint8).reshape(-1)
    del z
    descs, _, dext = encode_descs([1 << 20] * n)
    frames = torch.empty(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(n, dtype=torch.int64, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    if os.environ.get("HZ_PROF_BSHUF", "0") == "1":
        # bitshuffle+LZ4 objects: parse level 1 over 8 KiB transposed blocks
        bound = int(L.hsds_bitshuffle_bound(1 << 20, 4, 2048))
        descs, _, dext = encode_descs([1 << 20] * n, overhead=bound - (1 << 20))
        frames = torch.empty(dext, dtype=torch.uint8, device=dev)

        def enc():
            eng.encode_bitshuffle(data, descs, frames, sizes, st, itemsize=4, block=2048)
    else:
        def enc():
            eng.encode(data, descs, frames, sizes, st, clevel=4)
    enc()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    L.hsds_debug_profile(buf, 1)
    t = time.perf_counter()
    enc()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    L.hsds_debug_profile(buf, 1)
    assert (st.cpu().numpy() == 0).all()
    tot = sum(buf)
    comp = int(sizes.sum())
    print(f"encode n={n} wall={el*1e3:.1f} ms  {n*(1<<20)/el/1e9:.2f} GB/s  kernel={eng.last_deflate_ms():.1f} ms "
          f"ratio={comp/(n<<20):.4f}")
    segs = n * 128   # parse phases only (rocprof has the per-kernel split)
    for i in range(16):
        if buf[i]:
            print(f"   {NAMES[i]:16s} {100.0*buf[i]/tot:6.2f}%   {buf[i]/segs/1e3:9.1f} kcyc/segment")


if __name__ == "__main__":
    main()
