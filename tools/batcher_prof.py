"""Diagnostic: where the DN micro-batcher's time goes for N concurrent whole-chunk F1
requests (stage timers around the batch's steps + cProfile's top entries).  GPU box:
python tools/batcher_prof.py [N]"""
import asyncio
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import smooth_chunk, CHUNK_BYTES  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from hsds_amd import batcher as bt, datanode as dn  # noqa: E402

T = {}
E = {}          # per batch: end time of each timed step, relative to the batch's start
T0 = [0.0]


def timed(mod, name):
    f = getattr(mod, name)

    def w(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            t1 = time.perf_counter()
            T[name] = T.get(name, 0.0) + t1 - t
            E[name] = t1 - T0[0]
    setattr(mod, name, w)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    EV = []
    dev = torch.device("cuda", 0)
    chunks = [smooth_chunk(777 + i).view(np.uint8).tobytes() for i in range(64)]
    objs = {f"k{i}": orc.blosc_encode(c, typesize=1, clevel=4, shuffle=1) for i, c in enumerate(chunks)}
    ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype("<f4")}
    dims = (CHUNK_BYTES // 4,)
    cs = dn.ChunkStore(lambda key, off, ln: objs.get(key), mem_target=1 << 31, device=dev)
    for name in ("_stage_blobs", "_decode_batch", "device_view", "_flat_desc"):
        timed(dn, name)
    for cls, names in ((dn.ChunkReader, ("_plan", "read")), (dn.DeviceChunkCache, ("reserve", "unpin")),
                       (dn.ChunkStore, ("get_chunks_deferred",)),
                       (bt.ChunkBatcher, ("_run_batch", "_dispatch", "_finish"))):
        for name in names:
            timed(cls, name)
    from hsds_amd import engine as en
    for name in ("decode", "copy"):
        timed(en.ChunkEngine, name)
    # device timeline: HIP events before / after the decode and copy launches (on the
    # current stream, where the batch queues them)
    def evwrap(name):
        f = getattr(en.ChunkEngine, name)

        def w(*a, **k):
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = f(*a, **k)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            EV.append((name, e0, e1))
            return r
        setattr(en.ChunkEngine, name, w)
    evwrap("decode")
    evwrap("copy")
    fst = dn._stage_blobs

    def stage_ev(*a, **k):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fst(*a, **k)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        EV.append(("stage+upload", e0, e1))
        return r
    dn._stage_blobs = stage_ev
    for name in ("_gather_launch", "_gather_finish"):
        timed(bt, name)
    sync = torch.cuda.Stream.synchronize

    def tsync(self):
        t = time.perf_counter()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(self)
        EV.append(("stream_end", ev, ev))
        sync(self)
        t1 = time.perf_counter()
        T["stream_sync"] = T.get("stream_sync", 0.0) + t1 - t
        E["stream_sync"] = t1 - T0[0]
    torch.cuda.Stream.synchronize = tsync

    def one():
        cs.cache.clearCache()
        b = bt.ChunkBatcher(cs, window_ms=0.5)

        async def run():
            return await asyncio.gather(*[b.get_chunk(dn.ChunkRead(f"c-x_{j}", f"k{j % 64}"), "<f4", dims,
                                                      filter_ops=ops) for j in range(n)])
        t = time.perf_counter()
        T0[0] = t
        got = asyncio.run(run())
        el = time.perf_counter() - t
        assert got[-1].tobytes() == chunks[(n - 1) % 64]
        return el
    for _ in range(3):
        one()
    T.clear()
    els, ends, DEV = [], [], []
    for _ in range(9):
        E.clear()
        EV.clear()
        els.append(one())
        ends.append(dict(E))
        base = EV[0][1]
        DEV.append([(nm, base.elapsed_time(a), base.elapsed_time(b)) for nm, a, b in EV])
    print(f"n={n} median {np.median(els)*1e3:.2f} ms  {n * CHUNK_BYTES / np.median(els) / 1e9:.2f} GB/s  "
          f"(batches: {' '.join(f'{e * 1e3:.1f}' for e in els)})")
    for k, v in T.items():
        print(f"  {k:16s} {v / len(els) * 1e3:8.2f} ms per batch (mean)")
    print("  device timeline of the last batch (ms after the staging call): " +
          ", ".join(f"{nm} {a:.2f}-{b:.2f}" for nm, a, b in DEV[-1]))
    print("  step ends after the batch's start (median ms):")
    for k in sorted(ends[0], key=lambda k: np.median([e[k] for e in ends])):
        print(f"    {k:22s} {np.median([e[k] for e in ends]) * 1e3:8.2f}")
    # the batch runs on the batcher's worker thread: profile inside _run_batch
    pr = cProfile.Profile()
    orig = bt.ChunkBatcher._run_batch

    def prof_run(self, *a, **k):
        pr.enable()
        try:
            return orig(self, *a, **k)
        finally:
            pr.disable()
    bt.ChunkBatcher._run_batch = prof_run
    one()
    bt.ChunkBatcher._run_batch = orig
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
