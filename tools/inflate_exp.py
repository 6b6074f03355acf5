"""Diagnostic timing of experimental inflate builds (HZ_EXP_LIB=<.so>): F1 / F2 decode kernel
time over n chunks, statuses ignored (experimental builds may skip work)."""
import os
import sys
import torch  # noqa: F401
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hsds_amd import _native  # noqa: E402
_native.LIB_PATH = os.environ["HZ_EXP_LIB"]
from bench import make_corpus, CHUNK_BYTES  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402

for fmt in ("F1", "F2"):
    n = 4096
    raw, blobs = make_corpus(fmt, 512, 20261015, 16)
    order = [i % 512 for i in range(n)]
    src, descs, ext = pack_chunks([blobs[i] for i in order], [CHUNK_BYTES] * n)
    dev = torch.device("cuda", 0)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ms = []
    for _ in range(4):
        eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4)
        torch.cuda.synchronize()
        ms.append(eng.last_inflate_ms())
    print(os.path.basename(_native.LIB_PATH), fmt, "kernel ms", [round(m, 2) for m in ms], flush=True)
