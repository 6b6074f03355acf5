"""Per-request latency of the DN seam: one 1 MiB chunk through
codec._uncompress (storUtil._uncompress's signature: host bytes in, host bytes out, H2D +
decode + D2H) for an F1 (HSDS Blosc-zlib L4) and an F2 (HDF5 zlib of shuffled f32) object,
the same chunk device-resident (hsds_decode_batch of one chunk, HIP-event kernel time), the
oracle on one host thread (the reference's c-blosc + libz path), and the DN micro-batcher
(hsds_amd.batcher) serving N concurrent GET_Chunk-style requests (whole-chunk selections)
as one batch.  Prints one JSON object.  Run on the GPU box:  python tools/latency.py"""
import asyncio
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import smooth_chunk, CHUNK_BYTES  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from hsds_amd import codec  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402


def med(f, n=15):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e3


def main():
    dev = torch.device("cuda", 0)
    raw = smooth_chunk(20261015).view(np.uint8).tobytes()
    objs = {"F1": orc.blosc_encode(raw, typesize=1, clevel=4, shuffle=1),
            "F2": orc.zlib_encode(orc.shuffle(raw, 4), 4)}
    kw = {"F1": dict(compressor="zlib", shuffle=1, dtype=np.dtype("<f4"), chunk_shape=(CHUNK_BYTES // 4,)),
          "F2": dict(compressor="zlib", shuffle=1, dtype=np.dtype("<f4"), chunk_shape=(CHUNK_BYTES // 4,))}
    out = {"chunk_bytes": CHUNK_BYTES}
    eng = ChunkEngine(0)
    for fmt, blob in objs.items():
        assert codec._uncompress(blob, **kw[fmt]) == raw
        r = {"uncompress_ms": round(med(lambda: codec._uncompress(blob, **kw[fmt])), 3),
             "oracle_1thread_ms": round(med(lambda: orc.uncompress(blob, "zlib", 1, 4, CHUNK_BYTES), 7), 3)}
        src, descs, ext = pack_chunks([np.frombuffer(blob, np.uint8)], [CHUNK_BYTES])
        d_src = torch.from_numpy(src).to(dev)
        d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(1, dtype=torch.int32, device=dev)
        for mode, key in ((0, "device_one_chunk_kernel_ms"), (1, "device_one_chunk_kernel_ms_1wave"),
                          (2, "device_one_chunk_kernel_ms_2wave"), (4, "device_one_chunk_kernel_ms_4wave")):
            eng.set_tuning(waves_per_stream=mode)
            ks = []
            for _ in range(10):
                d_dst.zero_()
                eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4)
                torch.cuda.synchronize()
                ks.append(eng.last_inflate_ms())
            assert int(d_st[0]) == 0 and d_dst[:CHUNK_BYTES].cpu().numpy().tobytes() == raw
            r[key] = round(statistics.median(ks), 3)
        eng.set_tuning(waves_per_stream=0)
        out[fmt] = r
    # micro-batcher: N concurrent whole-chunk requests of distinct F1 chunks
    from hsds_amd.batcher import ChunkBatcher
    from hsds_amd.datanode import ChunkRead, ChunkStore
    chunks = [smooth_chunk(777 + i).view(np.uint8).tobytes() for i in range(64)]
    store_objs = {f"k{i}": orc.blosc_encode(c, typesize=1, clevel=4, shuffle=1) for i, c in enumerate(chunks)}
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    dims = (CHUNK_BYTES // 4,)
    res = {}
    cs = ChunkStore(lambda key, off, ln: store_objs.get(key), mem_target=1 << 31, device=dev)
    for n in (1, 16, 64, 256):
        ts = []
        for rep in range(11):
            # an emptied cache per trial: every request decodes (no cache hits)
            cs.cache.clearCache()
            b = ChunkBatcher(cs, window_ms=0.5)

            async def run():
                reqs = [b.get_chunk(ChunkRead(f"c-x_{j}", f"k{j % 64}"), "<f4", dims, filter_ops=ops) for j in range(n)]
                return await asyncio.gather(*reqs)
            t = time.perf_counter()
            got = asyncio.run(run())
            ts.append(time.perf_counter() - t)
            assert b.stats["batches"] == 1
            assert got[0].tobytes() == chunks[0] and got[-1].tobytes() == chunks[(n - 1) % 64]
            del got              # responses sent: their page-locked buffer returns to the cache
        el = statistics.median(ts[2:])      # two warm-up trials (page-locked buffers of this size)
        res[str(n)] = {"ms": round(el * 1e3, 2), "GBps": round(n * CHUNK_BYTES / el / 1e9, 2),
                       "trials_ms": [round(x * 1e3, 2) for x in ts]}
    out["batcher_F1_concurrent_requests"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
