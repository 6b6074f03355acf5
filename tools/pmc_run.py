"""Fixed workload for rocprofv3 counter collection: F1 decode of 512 chunks (2 launches)."""
import os
import sys
import torch  # noqa: F401  (HIP runtime first)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import make_corpus, CHUNK_BYTES  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "F1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
raw, blobs = make_corpus(fmt, min(n, 256), 20261015, 16)
order = [i % len(blobs) for i in range(n)]
src, descs, ext = pack_chunks([blobs[i] for i in order], [CHUNK_BYTES] * n)
dev = torch.device("cuda", 0)
eng = ChunkEngine(0)
d_src = torch.from_numpy(src).to(dev)
d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
d_st = torch.zeros(n, dtype=torch.int32, device=dev)
for _ in range(2):
    eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4)
torch.cuda.synchronize()
if not os.environ.get("HZ_NOCHECK"):
    assert (d_st.cpu().numpy() == 0).all()
print("pmc_run done", fmt, n, eng.last_inflate_ms(), "ms")
