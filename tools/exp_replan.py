"""timing experiment: selection read with and without the per-step plan rebuild"""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from hsds_amd import crawl

dev = torch.device("cuda", 0)
if len(sys.argv) > 1:
    import argparse
    a = argparse.Namespace(steps=3, warmup=1, chunks=1024, unique=256, cpu_seconds=0, kernel_timing=0)
    bench.run_format("F1", a, dev, 0, 1)
    print("ran F1 leg", flush=True)
plan = crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", bench.CFG1_DIMS, bench.CFG1_LAYOUT, bench.CFG1_SEL,
                           np.float32, 1)
ids = plan.chunk_ids(0)
csz = int(np.prod(bench.CFG1_LAYOUT)) * 4
raw = {cid: np.random.default_rng(k).integers(0, 255, csz, dtype=np.uint8) for k, cid in enumerate(ids)}
rd = crawl.ShardedReader(plan, 0, dev, compressor=None, shuffle=0)
st = rd.upload(raw)
gathered = torch.empty(plan.gathered_nbytes, dtype=torch.uint8, device=dev)
slab = torch.zeros(plan.slab_nbytes, dtype=torch.uint8, device=dev)


def timeit(name, fn, n=20):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(name, "%.3f ms" % ((time.perf_counter() - t) / n * 1e3), flush=True)


timeit("read", lambda: rd.read(st, slab=slab, gathered=gathered, check=False))
mk = lambda: crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", bench.CFG1_DIMS, bench.CFG1_LAYOUT,
                                 bench.CFG1_SEL, np.float32, 1)
timeit("plan", mk)
p2 = mk()
timeit("replan", lambda: rd.replan(st, p2))
timeit("replan+read", lambda: (rd.replan(st, p2), rd.read(st, slab=slab, gathered=gathered, check=False)))
timeit("read again", lambda: rd.read(st, slab=slab, gathered=gathered, check=False))
from hsds_amd.engine import to_device_bytes
timeit("host descs", lambda: to_device_bytes(p2.place_descs(), dev))
timeit("dev descs", lambda: p2.device_descs(1, dev))
