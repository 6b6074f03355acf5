"""Lone-chunk device latency of one library build (HSDS_AMD_LIB, HSDS_AMD_DEV=1): one 1 MiB
F1 and one F2 chunk of the bench data decoded alone, 1 / 2 / 4 / 8 wavefronts per stream, median of
15 HIP-event kernel times.  Prints one JSON line.  (tools/latency.py has the full set.)"""
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import smooth_chunk, CHUNK_BYTES  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    raw = smooth_chunk(20261015).view(np.uint8).tobytes()
    objs = {"F1": orc.blosc_encode(raw, typesize=1, clevel=4, shuffle=1),
            "F2": orc.zlib_encode(orc.shuffle(raw, 4), 4)}
    eng = ChunkEngine(0)
    out = {"lib": os.path.basename(os.environ.get("HSDS_AMD_LIB", "in-tree"))}
    for fmt, blob in objs.items():
        src, descs, ext = pack_chunks([np.frombuffer(blob, np.uint8)], [CHUNK_BYTES])
        d_src = torch.from_numpy(src).to(dev)
        d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(1, dtype=torch.int32, device=dev)
        for w in (1, 2, 4, 8):
            eng.set_tuning(waves_per_stream=w)
            ks = []
            for _ in range(15):
                eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4)
                torch.cuda.synchronize()
                ks.append(eng.last_inflate_ms())
            assert int(d_st.cpu()[0]) == 0 and d_dst[:CHUNK_BYTES].cpu().numpy().tobytes() == raw
            out[f"{fmt}_w{w}_ms"] = round(statistics.median(ks), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
