"""Diagnostic: per-phase cycle shares of the deflate encoder's kernels (HZ_PROFILE build,
tools/libhsds_prof.so): the parse's staging, hash chains and greedy parse (parse_stream
HZ_T marks), over 512 chunks of the cfg5 data (smooth f32 rows, 512x512 chunks, zlib L4).
Stamps are s_memtime deltas summed over all waves; only shares are meaningful."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from hsds_amd import _native  # noqa: E402

_native.LIB_PATH = os.environ.get("HZ_PROF_LIB") or os.path.join(ROOT, "tools", "libhsds_prof.so")
L = _native.lib()
L.hsds_debug_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
from hsds_amd.engine import ChunkEngine, encode_descs  # noqa: E402

NAMES = {0: "other", 1: "stage", 2: "chains", 3: "parse", 9: "end"}


def main():
    n = int(os.environ.get("HZ_ENC_N", "512"))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    rows = torch.round(torch.cumsum(torch.randn((n * 512, 512), generator=g, device=dev), dim=1), decimals=2)
    src = rows.to(torch.float32).reshape(-1).view(torch.uint8)
    cb = 512 * 512 * 4
    descs, _, dext = encode_descs([cb] * n)
    dst = torch.empty(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(n, dtype=torch.int64, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    eng = ChunkEngine(0)
    eng.encode(src, descs, dst, sizes, st, clevel=4, shuffle=1, typesize=4)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    L.hsds_debug_profile(buf, 1)
    eng.encode(src, descs, dst, sizes, st, clevel=4, shuffle=1, typesize=4)
    torch.cuda.synchronize()
    L.hsds_debug_profile(buf, 1)
    assert (st.cpu().numpy() == 0).all()
    tot = sum(buf)
    print(f"deflate encode n={n} chunks, ratio {n * cb / float(sizes.sum()):.3f}")
    for i in range(16):
        if buf[i]:
            print(f"   {NAMES.get(i, str(i)):8s} {100.0 * buf[i] / tot:6.2f}%")


if __name__ == "__main__":
    main()
