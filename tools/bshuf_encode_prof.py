"""Bitshuffle+LZ4 encode alone (for rocprofv3 --kernel-trace --stats): 4096 x 1 MiB
smooth f32 chunks generated on the device, 3 encode batches."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hsds_amd import _native as nat  # noqa: E402
from hsds_amd.engine import ChunkEngine, encode_descs  # noqa: E402


dev = torch.device("cuda", 0)
n, cb = 4096, 1 << 20
g = torch.Generator(device=dev)
g.manual_seed(7)
z = torch.randn((n, cb // 4), generator=g, device=dev, dtype=torch.float64)
src = torch.round(torch.cumsum(z, dim=1), decimals=2).to(torch.float32).view(torch.uint8).reshape(-1)
del z
bound = int(nat.lib().hsds_bitshuffle_bound(cb, 4, 2048))
descs, _, ext = encode_descs([cb] * n, overhead=bound - cb)
dst = torch.empty(ext, dtype=torch.uint8, device=dev)
sizes = torch.zeros(n, dtype=torch.int64, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)
eng = ChunkEngine(0)
d = None
for i in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = eng.encode_bitshuffle(src, descs if d is None else d, dst, sizes, st, itemsize=4, block=2048)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert int(st.abs().sum()) == 0
    print(f"iter {i}: {el * 1e3:.1f} ms, {n * cb / el / 1e9:.2f} GB/s, ratio {int(sizes.sum()) / (n * cb):.3f}",
          flush=True)
