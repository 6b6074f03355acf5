"""Headline benchmark: GB/s of device-resident chunk decode (shuffle+deflate L4, 1 MiB
float32 chunks) -- BASELINE.json `metric`, configs[1] (4096-chunk batch per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

`--gpus N` with no WORLD_SIZE in the environment starts the N rank processes itself
(before anything touches the GPU: children, not exec) on 127.0.0.1 and exits with the
worst rank's status; N larger than the visible devices is an error, never a silent
one-GPU run.  Under an outside launcher (torchrun) WORLD_SIZE must equal N.

A step = one hsds_decode_batch over the rank's 4096 stored chunks (inputs already in
HBM).  Chunks are HSDS-native F1 objects (Blosc1 frame, zlib inner codec, typesize 1,
4 x 256 KiB zlib streams per chunk) produced by the oracle's c-blosc 1.21
restatement, which is byte-identical to the reference's storUtil._compress output
(tests/test_oracle_golden.py).  Data: smooth float32 `round(cumsum(N(0,1)), 2)`,
seed 20261015 + global chunk index; `--unique` distinct chunks
per rank are stored several times at distinct HBM addresses.

Prints ONE JSON line on rank 0.  roofline.achieved = (compressed + decoded bytes per
launch) / inflate-kernel time (HIP events on the launch stream); cpu_baseline = the
oracle (same c-blosc frame walk + libz inflate) on a bounded sample with 16 threads.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CHUNK_BYTES = 1 << 20
HBM_PEAK_GBPS = 8000.0


def smooth_chunk(seed):
    rng = np.random.default_rng(seed)
    return np.round(np.cumsum(rng.normal(size=CHUNK_BYTES // 4)), 2).astype(np.float32)


def make_corpus(fmt, n_unique, base_seed, threads):
    """n_unique distinct chunks -> list of stored blobs (uint8 arrays) + raw chunks."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as orc
    with ThreadPoolExecutor(threads) as ex:
        raw = list(ex.map(lambda i: smooth_chunk(base_seed + i).view(np.uint8), range(n_unique)))
    if fmt == "F1":
        blobs = orc.encode_batch(raw, op="blosc", typesize=1, clevel=4, shuffle=1, nthreads=threads)
    elif fmt == "ZSTD":
        # Blosc-zstd frames as _compress(compressor="zstd", level=5) writes them: the
        # image's libblosc 1.21 (the c-blosc the reference's numcodecs vendors), 16 threads
        import ctypes
        lb = ctypes.CDLL("/opt/conda/lib/libblosc.so.1")
        lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                          ctypes.c_size_t, ctypes.c_int]

        def enc(r):
            out = np.empty(r.size + 16, np.uint8)
            k = lb.blosc_compress_ctx(5, 1, 1, r.size, r.ctypes.data, out.ctypes.data, out.size, b"zstd", 0, 1)
            assert k > 0
            return out[:k].copy()
        with ThreadPoolExecutor(threads) as ex:
            blobs = list(ex.map(enc, raw))
    elif fmt == "BSHUF":
        # bitshuffle+LZ4 objects as _shuffle(codec=2) writes them for an f32 chunk
        # (HSDS default block 2048 elements, 12-byte header); oracle LZ4 writer
        with ThreadPoolExecutor(threads) as ex:
            blobs = [np.frombuffer(b, np.uint8) for b in ex.map(lambda r: orc.bitshuffle_encode(r, 4, 2048), raw)]
    elif fmt == "LZ4":
        # Blosc-lz4 frames as _compress(compressor="lz4", level=5) lays them out
        # (typesize 1, 128 KiB blocks); the payload is the oracle's greedy LZ4 writer
        with ThreadPoolExecutor(threads) as ex:
            blobs = [np.frombuffer(b, np.uint8) for b in
                     ex.map(lambda r: orc.blosc_encode_lz4(r, typesize=1, blocksize=131072, shuffle=1), raw)]
    else:
        shuf = [np.frombuffer(orc.shuffle(r, 4), np.uint8) for r in raw]
        blobs = orc.encode_batch(shuf, op="zlib", clevel=4, nthreads=threads)
    return raw, blobs


def run_format(fmt, args, dev, rank, world):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    threads = box_threads()
    base_seed = 20261015 + rank * args.chunks
    raw, blobs = make_corpus(fmt, args.unique, base_seed, threads)
    order = [i % args.unique for i in range(args.chunks)]
    src, descs, ext = pack_chunks([blobs[i] for i in order], [CHUNK_BYTES] * args.chunks)
    comp_bytes = int(sum(len(blobs[i]) for i in order))
    dec_bytes = CHUNK_BYTES * args.chunks
    eng = ChunkEngine(dev.index)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
    d_st = torch.full((args.chunks,), 99, dtype=torch.int32, device=dev)
    from hsds_amd.engine import to_device_bytes
    d_desc = to_device_bytes(descs, dev)
    stream = torch.cuda.current_stream()

    comp = {"LZ4": "lz4", "ZSTD": "zstd", "BSHUF": None}.get(fmt, "zlib")
    shuffle = 2 if fmt == "BSHUF" else 1

    def step():
        eng.decode(d_src, d_desc, d_dst, d_st, compressor=comp, shuffle=shuffle, itemsize=4, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness of what is timed: statuses + sampled chunks vs the raw data
    st = d_st.cpu().numpy()
    assert (st == 0).all(), f"decode status errors: {np.unique(st)}"
    for k in list(range(0, args.chunks, max(1, args.chunks // 8))):
        o = int(descs[k]["dst_off"])
        got = d_dst[o:o + CHUNK_BYTES].cpu().numpy()
        assert np.array_equal(got, raw[order[k]]), f"chunk {k} mismatch"
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    kern_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if args.kernel_timing:
            torch.cuda.synchronize()
            kern_ms.append(eng.last_inflate_ms())
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if not kern_ms:   # one extra timed launch for the kernel-event duration
        step()
        torch.cuda.synchronize()
        kern_ms.append(eng.last_inflate_ms())
    res = {"fmt": fmt, "elapsed_s": elapsed, "comp_bytes": comp_bytes, "dec_bytes": dec_bytes,
           "kernel_ms": float(np.mean(kern_ms)), "blobs": blobs, "raw": raw, "order": order}
    del d_src, d_dst
    torch.cuda.empty_cache()
    return res


def run_e2e(r, args, dev, nsub=8):
    """PCIe-inclusive rate: stored objects in pinned host memory
    -> hipMemcpyAsync H2D -> decode -> D2H into a pinned host buffer, pipelined over
    `nsub` sub-batches on three streams (copy-in / decode / copy-out)."""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks, to_device_bytes, CHUNK_DESC_DTYPE
    blobs, order = r["blobs"], r["order"]
    n = len(order)
    src, descs, ext = pack_chunks([blobs[i] for i in order], [CHUNK_BYTES] * n)
    h_src = torch.from_numpy(src).pin_memory()
    h_out = torch.empty(ext, dtype=torch.uint8).pin_memory()
    d_src = torch.empty(src.size, dtype=torch.uint8, device=dev)
    d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    d_desc = to_device_bytes(descs, dev)
    eng = ChunkEngine(dev.index)
    s_in, s_dec, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    bounds = [n * k // nsub for k in range(nsub + 1)]
    D = CHUNK_DESC_DTYPE.itemsize

    def rng_src(a, b):
        return int(descs[a]["src_off"]), int(descs[b - 1]["src_off"] + descs[b - 1]["src_len"])

    def rng_dst(a, b):
        return int(descs[a]["dst_off"]), int(descs[b - 1]["dst_off"] + descs[b - 1]["dst_len"])

    def step():
        for k in range(nsub):
            a, b = bounds[k], bounds[k + 1]
            s0, s1 = rng_src(a, b)
            o0, o1 = rng_dst(a, b)
            with torch.cuda.stream(s_in):
                d_src[s0:s1].copy_(h_src[s0:s1], non_blocking=True)
                e_in = torch.cuda.Event()
                e_in.record(s_in)
            s_dec.wait_event(e_in)
            eng.decode(d_src, d_desc[a * D:b * D], d_dst, d_st[a:b], compressor="zlib", shuffle=1,
                       itemsize=4 if r["fmt"] == "F2" else 1, stream=s_dec)
            e_dec = torch.cuda.Event()
            e_dec.record(s_dec)
            s_out.wait_event(e_dec)
            with torch.cuda.stream(s_out):
                h_out[o0:o1].copy_(d_dst[o0:o1], non_blocking=True)

    step()
    torch.cuda.synchronize()
    assert int(d_st.abs().sum()) == 0
    o = int(descs[n - 1]["dst_off"])
    assert np.array_equal(h_out[o:o + CHUNK_BYTES].numpy(), r["raw"][order[n - 1]])
    steps = max(1, min(args.steps, 3))
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # raw link rates for context (one direction at a time)
    t1 = time.perf_counter()
    d_src.copy_(h_src, non_blocking=True)
    torch.cuda.synchronize()
    h2d = src.size / (time.perf_counter() - t1) / 1e9
    t1 = time.perf_counter()
    h_out.copy_(d_dst, non_blocking=True)
    torch.cuda.synchronize()
    d2h = ext / (time.perf_counter() - t1) / 1e9
    out = {"value": round(n * CHUNK_BYTES * steps / el / 1e9, 2), "unit": "GB/s",
           "what": f"pinned host stored objects -> H2D -> decode -> D2H pinned, {nsub} pipelined sub-batches",
           "h2d_GBps": round(h2d, 1), "d2h_GBps": round(d2h, 1), "steps": steps}
    del d_src, d_dst, h_src, h_out
    torch.cuda.empty_cache()
    return out


CFG3_DIMS, CFG3_LAYOUT = (512, 2048, 2048), (16, 64, 128)
CFG3_SEL = (slice(0, 512, 2), slice(3, 2048, 5), slice(1, 2048, 3))


def run_cfg3(args, dev):
    """configs[2]: 3D int16 dataset, shuffle+deflate 256 KiB chunks, strided selection
    [0:512:2, 3:2048:5, 1:2048:3] across all 16 384 chunks; one step = batch decode +
    fused strided gather of every chunk's selection + placement into the result slab."""
    import torch
    from hsds_amd import crawl
    from oracle import oracle as orc
    from concurrent.futures import ThreadPoolExecutor
    threads = box_threads()
    plan = crawl.SelectionPlan("d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", CFG3_DIMS, CFG3_LAYOUT, CFG3_SEL,
                               np.int16, 1)
    ids = plan.chunk_ids(0)
    nuniq = min(args.unique, len(ids))
    csz = int(np.prod(CFG3_LAYOUT))

    def mk(i):
        g = np.random.default_rng(20261015 + i)
        return (np.cumsum(g.normal(size=csz)) * 100).astype("<i2").view(np.uint8)
    with ThreadPoolExecutor(threads) as ex:
        raw = list(ex.map(mk, range(nuniq)))
    enc = orc.encode_batch(raw, op="blosc", typesize=1, clevel=4, shuffle=1, nthreads=threads)
    blobs = {cid: enc[k % nuniq] for k, cid in enumerate(ids)}
    rd = crawl.ShardedReader(plan, 0, dev)
    st = rd.upload(blobs)
    gathered = torch.empty(plan.gathered_nbytes, dtype=torch.uint8, device=dev)
    slab = torch.zeros(plan.slab_nbytes, dtype=torch.uint8, device=dev)
    for _ in range(max(1, args.warmup)):
        rd.read(st, slab=slab, gathered=gathered, check=False)
    torch.cuda.synchronize()
    assert int(st["d_status"].abs().sum()) == 0
    host = slab.cpu().numpy().view(np.int16).reshape(plan.slab_shape)
    for k in (0, len(ids) // 3, len(ids) - 1):
        p = plan.pieces[plan.by_rank[0][k]]
        c = raw[k % nuniq].view(np.int16).reshape(CFG3_LAYOUT)
        assert np.array_equal(host[p.data_slices], c[p.chunk_slices]), f"cfg3 piece {k}"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan_s = 0.0
    for _ in range(args.steps):
        # the request's plan (chunk ids, md5 owners, pieces) and its device copy records
        # are rebuilt every step: per-request host cost inside the timed region
        tp = time.perf_counter()
        p_ = crawl.SelectionPlan("d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", CFG3_DIMS, CFG3_LAYOUT, CFG3_SEL,
                                 np.int16, 1)
        plan_s += time.perf_counter() - tp
        rd.replan(st, p_)
        rd.read(st, slab=slab, gathered=gathered, check=False)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    comp = sum(len(blobs[c]) for c in ids)
    out = {"value": round(plan.slab_nbytes / el / 1e9, 3), "unit": "GB/s selected",
           "decoded_GBps": round(len(ids) * csz * 2 / el / 1e9, 2), "ms_per_step": round(el * 1e3, 3),
           "plan_ms": round(plan_s / args.steps * 1e3, 2), "plan_note": "host SelectionPlan per step; the device "
                                                                          "record build is inside ms_per_step",
           "chunks": len(ids), "selected_bytes": plan.slab_nbytes, "compressed_bytes": comp,
           "algorithmic_GBps": round((comp + plan.slab_nbytes) / el / 1e9, 2),
           "workload": "configs[2]: int16 512x2048x2048, 16x64x128 chunks (F1 L4), "
                       "select [0:512:2,3:2048:5,1:2048:3], decode+gather+place"}
    tr = load_traffic(args, 1, "_cfg3")
    if tr is not None:
        # HBM bytes of every kernel of one step (PMC passes) against the algorithmic bytes
        out["traffic"] = tr["bytes_per_step"]
        out["traffic_undoubled"] = tr["bytes_per_step_undoubled"]
        out["traffic_ratio"] = round(tr["bytes_per_step"] / (comp + plan.slab_nbytes), 3)
        out["traffic_source"] = tr["source"]
    if args.cpu_seconds > 0:
        # the reference's per-chunk path on the box's cores: _uncompress -- c-blosc's
        # blosc_decompress, here the image's libblosc 1.21.0 (storUtil.py:195-208), one chunk
        # per thread -- + chunkReadSelection / slab assignment (numpy, chunkUtil.py:882-929,
        # chunk_crawl.py:395-418); the oracle port of the same decode is kept beside it
        import ctypes
        from concurrent.futures import ThreadPoolExecutor
        ns = min(512, len(ids))
        samp = [np.ascontiguousarray(enc[k % nuniq]) for k in range(ns)]
        pieces = [plan.pieces[plan.by_rank[0][k]] for k in range(ns)]
        outb = [np.empty(csz * 2, np.uint8) for _ in range(ns)]
        cpu_slab = np.zeros(plan.slab_shape, np.int16)
        lb = ctypes.CDLL(LIBBLOSC)
        lb.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        lb.blosc_decompress_ctx.restype = ctypes.c_int
        lb.blosc_get_version_string.restype = ctypes.c_char_p

        def one(k):
            r = lb.blosc_decompress_ctx(samp[k].ctypes.data, outb[k].ctypes.data, csz * 2, 1)
            assert r == csz * 2, r
            p = pieces[k]
            cpu_slab[p.data_slices] = outb[k].view(np.int16).reshape(CFG3_LAYOUT)[p.chunk_slices]
        done, t1 = 0, time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            while time.perf_counter() - t1 < min(args.cpu_seconds, 4.0):
                list(ex.map(one, range(ns)))
                done += 1
        cel = (time.perf_counter() - t1) / done
        sel_bytes = int(sum(p.nbytes for p in pieces))
        assert np.array_equal(cpu_slab[pieces[1].data_slices], host[pieces[1].data_slices])
        pdone, t2 = 0, time.perf_counter()
        while time.perf_counter() - t2 < min(args.cpu_seconds / 2, 2.0):
            _, stt = orc.uncompress_batch(samp, [csz * 2] * ns, "zlib", 1, 2, nthreads=threads, out=outb)
            assert (stt == csz * 2).all()
            for b, p in zip(outb, pieces):
                cpu_slab[p.data_slices] = b.view(np.int16).reshape(CFG3_LAYOUT)[p.chunk_slices]
            pdone += 1
        pel = (time.perf_counter() - t2) / pdone
        out["cpu_baseline"] = {"value": round(sel_bytes / cel / 1e9, 4), "unit": "GB/s selected", "cores": threads,
                               "kind": "reference", "cpu_model": cpu_model(),
                               "sample": f"{done} x {ns} of the {len(ids)} chunks: libblosc "
                                         f"{lb.blosc_get_version_string().decode()} blosc_decompress_ctx "
                                         f"({threads} threads, one chunk each) + numpy selection into the slab",
                               "port_value": round(sel_bytes / pel / 1e9, 4),
                               "port_sample": f"{pdone} x {ns} chunks: oracle decode + numpy selection"}
    del gathered, slab, st
    torch.cuda.empty_cache()
    return out


CFG1_DIMS, CFG1_LAYOUT = (4096, 4096), (64, 64)
CFG1_SEL = (slice(1000, 3000, 1), slice(500, 3500, 1))


def run_cfg1(args, dev):
    """configs[0], the reference's CPU-runnable case: f32 4096x4096 in 64x64 chunks
    (16 KiB, stored uncompressed), selection [1000:3000,500:3500] (32 x 48 = 1536
    chunks, 24 MB out).  One step = the chunks' read selections + placement into the
    slab (no codec).  The reference's rate here is bounded by HTTP per chunk."""
    import torch
    from hsds_amd import crawl
    plan = crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", CFG1_DIMS, CFG1_LAYOUT, CFG1_SEL,
                               np.float32, 1)
    ids = plan.chunk_ids(0)
    csz = int(np.prod(CFG1_LAYOUT)) * 4
    raw = {}
    for k, cid in enumerate(ids):
        g = np.random.default_rng(20261015 + k)
        raw[cid] = np.round(np.cumsum(g.normal(size=csz // 4)), 2).astype(np.float32).view(np.uint8)
    rd = crawl.ShardedReader(plan, 0, dev, compressor=None, shuffle=0)
    st = rd.upload(raw)
    gathered = torch.empty(plan.gathered_nbytes, dtype=torch.uint8, device=dev)
    slab = torch.zeros(plan.slab_nbytes, dtype=torch.uint8, device=dev)
    for _ in range(max(1, args.warmup)):
        rd.read(st, slab=slab, gathered=gathered, check=False)
    torch.cuda.synchronize()
    assert int(st["d_status"].abs().sum()) == 0
    host = slab.cpu().numpy().view(np.float32).reshape(plan.slab_shape)
    for k in (0, len(ids) // 2, len(ids) - 1):
        p = plan.pieces[plan.by_rank[0][k]]
        c = raw[ids[k]].view(np.float32).reshape(CFG1_LAYOUT)
        assert np.array_equal(host[p.data_slices], c[p.chunk_slices]), f"cfg1 piece {k}"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan_s = 0.0
    for _ in range(args.steps):
        tp = time.perf_counter()
        p_ = crawl.SelectionPlan("d-0a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", CFG1_DIMS, CFG1_LAYOUT, CFG1_SEL,
                                 np.float32, 1)
        plan_s += time.perf_counter() - tp
        rd.replan(st, p_)
        rd.read(st, slab=slab, gathered=gathered, check=False)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    out = {"value": round(plan.slab_nbytes / el / 1e9, 3), "unit": "GB/s selected", "ms_per_step": round(el * 1e3, 3),
           "plan_ms": round(plan_s / args.steps * 1e3, 2), "plan_note": "host SelectionPlan per step; the device "
                                                                          "record build is inside ms_per_step",
           "chunks": len(ids), "selected_bytes": plan.slab_nbytes,
           "workload": "configs[0]: f32 4096x4096, 64x64 chunks stored uncompressed, select [1000:3000,500:3500], "
                       "gather+place"}
    if args.cpu_seconds > 0:
        # the reference's per-chunk path on one core: bytesToArray + chunkReadSelection
        # (numpy slicing, chunkUtil.py:882-929) + the SN slab assignment (chunk_crawl.py:418)
        arrs = [raw[c].view(np.float32).reshape(CFG1_LAYOUT) for c in ids]
        pieces = [plan.pieces[plan.by_rank[0][k]] for k in range(len(ids))]
        cpu_slab = np.zeros(plan.slab_shape, np.float32)
        t1 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t1 < min(args.cpu_seconds, 2.0):
            for a, p in zip(arrs, pieces):
                cpu_slab[p.data_slices] = a[p.chunk_slices]
            reps += 1
        cel = (time.perf_counter() - t1) / reps
        assert np.array_equal(cpu_slab, host)
        out["cpu_baseline"] = {"value": round(plan.slab_nbytes / cel / 1e9, 3), "unit": "GB/s selected", "cores": 1,
                               "kind": "port", "sample": f"{reps} x the full 1536-chunk selection, numpy slicing "
                                                         "(chunkReadSelection + slab assignment), 1 thread"}
    del gathered, slab, st
    torch.cuda.empty_cache()
    return out


CFG5_CHUNK = (512, 512)
CFG5_DIMS = (65536, 131072)
CFG5_DSET = "d-7f6e5d4c-3b2a1908-f7e6-d5c4b3-a29180"


def _partial(cid, sel):
    """the selection covers chunk `cid` (a 512 x 512 chunk of CFG5_DIMS) only in part"""
    from hsds_amd import selection as hsel
    idx = hsel.getChunkIndex(cid)
    for k, s in enumerate(sel):
        lo, hi = idx[k] * CFG5_CHUNK[k], min((idx[k] + 1) * CFG5_CHUNK[k], CFG5_DIMS[k])
        if s.start > lo or s.stop < hi:
            return True
    return False


def run_cfg5_sharded(args, dev, rank, world):
    """configs[4] through the write path itself (crawl.ShardedWriter): f32 dataset
    65536 x 131072 in 512x512 chunks; the request covers 8192 x world rows (all 32 768 chunks
    at N = 8, one GPU's 4096 at N = 1: weak scaling).  One step = the root gathers every
    chunk's piece of the request array by the plan (arr[data_sel], chunk_crawl.py:135) and
    sends each owner its pieces (RCCL P2P), every rank runs PUT_Chunk on its chunks (RMW
    through its HBM chunk store: chunk_init, compare, conditional copy, chunk_dn.py:174-310;
    write_zero_chunks so that every step re-dirties them) and encodes its dirty chunks into
    F1 objects (the device half of s3sync).  Plan, descriptors and host bookkeeping are
    inside the step.  A second request offset by (100, 100) exercises partial edge chunks."""
    import torch
    import torch.distributed as dist
    from hsds_amd import crawl
    from hsds_amd.datanode import ChunkStore
    from hsds_amd.filters import getFilterOps
    rows = min(8192 * world, CFG5_DIMS[0])
    cols = CFG5_DIMS[1]
    ops = getFilterOps({"filter_map": {}}, CFG5_DSET,
                       [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                        {"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": 4}],
                       dtype=np.dtype("<f4"), chunk_shape=CFG5_CHUNK)
    slab = None
    if rank == 0:
        g = torch.Generator(device=dev)
        g.manual_seed(20261015)
        slab = torch.empty((rows, cols), dtype=torch.float32, device=dev)
        for r0 in range(0, rows, 512):
            z = torch.randn((512, cols), generator=g, device=dev, dtype=torch.float64)
            slab[r0:r0 + 512] = torch.round(torch.cumsum(z, dim=1), decimals=2).to(torch.float32)
            del z
    per_rank = 4096 * 1024 * 1024 * 5 // 4 + (1 << 30)
    # the DN's object storage: S3 key -> stored F1 object (filled from the first variant's
    # encode); a chunk the cache does not hold is read from here (get_chunk's fetch)
    objects = {}
    store = ChunkStore(lambda k, o, n: (objects[k][o:o + n] if n else objects[k][o:]) if k in objects else None,
                       mem_target=per_rank, device=dev)
    out = {}
    variants = [v for v in (("full", (0, 0)), ("offset_100_100", (100, 100)))
                if v[0] in args.cfg5w_variants.split(",")]
    for name, (y0, x0) in variants:
        sel = (slice(y0, rows, 1), slice(x0, cols, 1))
        req = slab[y0:, x0:].contiguous() if rank == 0 else None
        stats = {}
        # the chunks this request covers only in part: PUT_Chunk reads them (RMW).  Before every
        # step they leave the cache, so each step decodes their stored objects as a DN does
        # for a chunk it does not hold (chunk_dn.py:174-190, datanode_lib.get_chunk)
        plan0 = crawl.SelectionPlan(CFG5_DSET, CFG5_DIMS, CFG5_CHUNK, sel, np.float32, world)
        edge = [c for c in plan0.chunk_ids(rank) if _partial(c, sel)] if objects else []

        def step():
            t0 = time.perf_counter()
            for cid in edge:
                if cid in store.cache:
                    store.cache.clearDirty(cid)
                    del store.cache[cid]
            plan = crawl.SelectionPlan(CFG5_DSET, CFG5_DIMS, CFG5_CHUNK, sel, np.float32, world)
            t1 = time.perf_counter()
            w = crawl.ShardedWriter(plan, rank, store)
            w.write(req, filter_ops=ops, write_zero_chunks=True)
            ids, frames, descs, sizes, status = store.encode_dirty(ops)
            stats.update(plan_ms=(t1 - t0) * 1e3, ids=ids, frames=frames, descs=descs, sizes=sizes,
                         status=status, plan=plan)
        for _ in range(max(1, args.warmup)):
            step()
        torch.cuda.synchronize()
        assert int((stats["status"][:len(stats["ids"])] != 0).sum()) == 0, "encode status errors"
        if not objects and stats["ids"]:
            # the stored objects of this rank's chunks (the s3sync of the first variant)
            from hsds_amd.partition import getS3Key
            hs = stats["sizes"].cpu().numpy()
            hf = stats["frames"].cpu().numpy()
            for k, cid in enumerate(stats["ids"]):
                o = int(stats["descs"][k]["dst_off"])
                objects[getS3Key(cid)] = hf[o:o + int(hs[k])].tobytes()
            del hf
        ok = 1
        if rank == 0 and stats["ids"]:
            # sampled objects (a fully covered chunk, and a partly covered one at the offset,
            # whose uncovered part came from its stored object) decode (oracle) to the chunk
            # the request and the previous contents make: here the slab's block
            from oracle import oracle as orc
            from hsds_amd import selection as hsel
            hs = stats["sizes"].cpu().numpy()
            for k in (0, len(stats["ids"]) // 2):
                cid = stats["ids"][k]
                i, j = hsel.getChunkIndex(cid)
                o = int(stats["descs"][k]["dst_off"])
                fr = stats["frames"][o:o + int(hs[k])].cpu().numpy().tobytes()
                got = np.frombuffer(orc.uncompress(fr, "zlib", 1, 1, 1 << 20), np.float32).reshape(CFG5_CHUNK)
                want = slab[i * 512:(i + 1) * 512, j * 512:(j + 1) * 512].cpu().numpy()
                ok &= int(np.array_equal(got, want))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pms = []
        for _ in range(args.cfg5_steps):
            step()
            pms.append(stats["plan_ms"])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if os.environ.get("HSDS_PROFILE_CFG5W") and rank == 0:
            # host hot spots of the write path (tools/gpu_r6p.sh): two more steps under cProfile
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            pr.disable()
            print(f"--- cfg5w {name} host profile (2 steps)", file=sys.stderr)
            pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        el /= args.cfg5_steps
        nbytes = (rows - y0) * (cols - x0) * 4
        comp = int(stats["sizes"][:len(stats["ids"])].sum()) if stats["ids"] else 0
        out[name] = {"value": round(nbytes / el / 1e9, 2), "unit": "GB/s of request array (all ranks)",
                     "ms_per_step": round(el * 1e3, 3), "request_bytes": nbytes,
                     "chunks": int(len(stats["plan"].idx)), "chunks_this_rank": len(stats["ids"]),
                     "rmw_chunks_from_storage_rank0": len(edge),
                     "plan_ms": round(float(np.mean(pms)), 2), "compressed_bytes_rank0": comp,
                     "sample_check": bool(ok)}
        del req
    out["workload"] = (f"configs[4]: f32 {CFG5_DIMS[0]}x{CFG5_DIMS[1]}, 512x512 chunks, request rows [0:{rows}] "
                       f"(and offset by (100,100)), md5-sharded over {world} rank(s): plan + root gather + RCCL "
                       "scatter + PUT_Chunk RMW (compare + copy) + F1 zlib L4 encode; the offset request's "
                       "partly covered chunks are read back from their stored F1 objects every step")
    del slab, store
    torch.cuda.empty_cache()
    return out


def isolated_kernel_ms(step, eng, reps=3):
    """The encode's device time: the engine's HIP event pair (recorded on the launch stream
    around the encode's kernels, hsds_last_deflate_ms) of `reps` steps run one at a time
    with the device idle before and after each, median.  (Read after a pipelined loop, the
    last step's pair can also span a host-side gap, so it could exceed the step time.)"""
    import torch
    v = []
    for _ in range(reps):
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        v.append(eng.last_deflate_ms())
    return float(np.median(v))


def run_cfg5(args, dev, rank=0):
    """configs[4] write path, one GPU's share (32k chunks / 8 GPUs = 4096): a
    float32 slab of 16 x 256 chunks of 512x512 (4 GiB, smooth rows generated on the
    device) is scattered into 1 MiB chunk arrays (chunk_crawl.py:118-140 write
    gather + chunkWriteSelection's copy) and every chunk is encoded into an HSDS F1
    object (storUtil._compress: Blosc1 frame, zlib L4, shuffle flag, typesize 1).
    One step = scatter + encode.  Algorithmic bytes:
    slab bytes in + compressed bytes out."""
    import torch
    from hsds_amd.engine import ChunkEngine, COPY_DESC_DTYPE, encode_descs, to_device_bytes
    from oracle import oracle as orc
    R, C = 16, args.chunks // 16
    cr, cc = CFG5_CHUNK
    rows, cols = R * cr, C * cc
    g = torch.Generator(device=dev)
    g.manual_seed(20261015 + rank)
    slab = torch.empty((rows, cols), dtype=torch.float32, device=dev)
    for r0 in range(0, rows, 512):   # round(cumsum(N(0,1)), 2) along rows, float64 then float32
        z = torch.randn((512, cols), generator=g, device=dev, dtype=torch.float64)
        slab[r0:r0 + 512] = torch.round(torch.cumsum(z, dim=1), decimals=2).to(torch.float32)
        del z
    n = R * C
    cbytes = cr * cc * 4
    cd = np.zeros(n, COPY_DESC_DTYPE)
    for k in range(n):
        i, j = divmod(k, C)
        cd[k]["src_off"] = (i * cr * cols + j * cc) * 4
        cd[k]["dst_off"] = k * cbytes
        cd[k]["src_stride"][:2] = (cols * 4, 4)
        cd[k]["dst_stride"][:2] = (cc * 4, 4)
        cd[k]["count"][:2] = (cr, cc)
        cd[k]["rank"] = 2
        cd[k]["itemsize"] = 4
    d_cd = to_device_bytes(cd, dev)
    descs, _, dext = encode_descs([cbytes] * n)
    # chunk arrays back to back (src of the encode), frames in 1 MiB + 16 slots
    chunks = torch.empty(n * cbytes, dtype=torch.uint8, device=dev)
    frames = torch.empty(dext, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(n, dtype=torch.int64, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    d_desc = to_device_bytes(descs, dev)
    eng = ChunkEngine(dev.index)
    slab_u8 = slab.view(torch.uint8).reshape(-1)
    stream = torch.cuda.current_stream()

    def step():
        eng.copy(slab_u8, chunks, d_cd, stream=stream)
        eng.encode(chunks, d_desc, frames, sizes, st, clevel=4, shuffle=1, typesize=1, stream=stream)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0, "encode status errors"
    hs = sizes.cpu().numpy()
    host_slab = None
    for k in (0, n // 2, n - 1):    # sampled frames decode (oracle) to the slab's chunk
        i, j = divmod(k, C)
        o = int(descs[k]["dst_off"])
        fr = frames[o:o + int(hs[k])].cpu().numpy().tobytes()
        want = slab[i * cr:(i + 1) * cr, j * cc:(j + 1) * cc].contiguous().cpu().numpy().tobytes()
        assert orc.uncompress(fr, "zlib", 1, 1, cbytes) == want, f"cfg5 chunk {k}"
    del host_slab
    kern = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    kern.append(isolated_kernel_ms(step, eng))
    comp = int(sizes.sum())
    slab_bytes = n * cbytes
    # libz reference size (oracle = reference _compress bytes) on 16 chunks spread over the
    # slab's rows and columns, and on 16 chunks of its first column (the worst case: walks
    # that start at 0 repeat values most, so window and chain depth matter most there)
    ks = [(i * (n // 16) + i * (C // 16 + 1)) % n for i in range(16)]
    k0 = [(i * C) % n for i in range(16)]
    samp = [chunks[k * cbytes:(k + 1) * cbytes].cpu().numpy() for k in ks]
    ref = sum(len(orc.blosc_encode(x, typesize=1, clevel=4, shuffle=1)) for x in samp)
    ours = sum(int(hs[k]) for k in ks)
    ref0 = sum(len(orc.blosc_encode(chunks[k * cbytes:(k + 1) * cbytes].cpu().numpy(), typesize=1, clevel=4,
                                    shuffle=1)) for k in k0)
    ours0 = sum(int(hs[k]) for k in k0)
    # the slab -> chunk scatter alone (copy_kernel), HIP events on the launch stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(5):
        eng.copy(slab_u8, chunks, d_cd, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    scat_ms = e0.elapsed_time(e1) / 5
    out = {"value": round(slab_bytes / el / 1e9, 2), "unit": "GB/s slab (scatter + encode)",
           "scatter_ms": round(scat_ms, 3), "scatter_GBps": round(2 * slab_bytes / (scat_ms / 1e3) / 1e9, 1),
           "ms_per_step": round(el * 1e3, 3), "chunks": n, "slab_bytes": slab_bytes, "compressed_bytes": comp,
           "algorithmic_GBps": round((slab_bytes + comp) / el / 1e9, 2),
           "deflate_kernel_ms": round(kern[-1], 3),
           "deflate_kernel_GBps": round((slab_bytes + comp) / (kern[-1] / 1e3) / 1e9, 2),
           "size_vs_libz": round(ours / ref, 4), "size_vs_libz_first_column": round(ours0 / ref0, 4),
           "workload": "configs[4] per-GPU share: f32 slab 8192x131072 -> 4096 chunks 512x512 -> F1 zlib L4 frames"}
    # the same scatter + encode for an lz4 dataset (Blosc-lz4 frames, level 5)
    def step_lz4():
        eng.copy(slab_u8, chunks, d_cd, stream=stream)
        eng.encode(chunks, d_desc, frames, sizes, st, clevel=5, shuffle=1, typesize=1, stream=stream,
                   compressor="lz4")

    step_lz4()
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0, "lz4 encode status errors"
    o = int(descs[n // 3]["dst_off"])
    fr = frames[o:o + int(sizes[n // 3])].cpu().numpy().tobytes()
    assert orc.uncompress(fr, "lz4", 1, 1, cbytes) == chunks[(n // 3) * cbytes:(n // 3 + 1) * cbytes].cpu().numpy().tobytes()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_lz4()
    torch.cuda.synchronize()
    el4 = (time.perf_counter() - t0) / args.steps
    comp4 = int(sizes.sum())
    k4 = isolated_kernel_ms(step_lz4, eng)
    out["lz4_encode"] = {"value": round(slab_bytes / el4 / 1e9, 2), "unit": "GB/s slab (scatter + encode)",
                         "ms_per_step": round(el4 * 1e3, 3), "compressed_bytes": comp4,
                         "encode_ms": round(k4, 3),
                         "format": "Blosc-lz4 frames (typesize 1, c-blosc lz4 blocksize), parse tokens -> LZ4 blocks"}
    # the same scatter + encode for a zstd dataset (Blosc-zstd frames, level 5)
    def step_zstd():
        eng.copy(slab_u8, chunks, d_cd, stream=stream)
        eng.encode(chunks, d_desc, frames, sizes, st, clevel=5, shuffle=1, typesize=1, stream=stream,
                   compressor="zstd")

    step_zstd()
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0, "zstd encode status errors"
    o = int(descs[n // 5]["dst_off"])
    fr = frames[o:o + int(sizes[n // 5])].cpu().numpy().tobytes()
    assert orc.uncompress(fr, "zstd", 1, 1, cbytes) == chunks[(n // 5) * cbytes:(n // 5 + 1) * cbytes].cpu().numpy().tobytes()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_zstd()
    torch.cuda.synchronize()
    elz = (time.perf_counter() - t0) / args.steps
    compz = int(sizes.sum())
    kz = isolated_kernel_ms(step_zstd, eng)
    zr = None
    try:   # libblosc's own zstd objects for the same sampled chunks (the reference's c-blosc)
        import ctypes
        lb = ctypes.CDLL("/opt/conda/lib/libblosc.so.1")
        lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                          ctypes.c_size_t, ctypes.c_int]
        refz = 0
        for x in samp:
            ob = np.empty(x.size + 64, np.uint8)
            refz += lb.blosc_compress_ctx(5, 1, 1, x.size, x.ctypes.data, ob.ctypes.data, ob.size, b"zstd", 0, 1)
        zr = round(sum(int(sizes[k]) for k in ks) / refz, 4)
    except OSError:
        pass
    out["zstd_encode"] = {"value": round(slab_bytes / elz / 1e9, 2), "unit": "GB/s slab (scatter + encode)",
                          "ms_per_step": round(elz * 1e3, 3), "compressed_bytes": compz,
                          "encode_ms": round(kz, 3), "size_vs_libblosc_zstd": zr,
                          "format": "Blosc-zstd frames (HCR blocksize, never split): raw literals + each frame's "
                                    "own FSE_Compressed_Mode sequence tables, one zstd block per 8 KiB"}
    # the same scatter + encode for a bitshuffle dataset (storUtil._shuffle codec 2:
    # bitshuffle+LZ4 objects, f32, 2048-element blocks, no outer compressor)
    from hsds_amd import _native as nat
    bound = int(nat.lib().hsds_bitshuffle_bound(cbytes, 4, 2048))
    bdescs, _, bext = encode_descs([cbytes] * n, overhead=bound - cbytes)
    d_bdesc = to_device_bytes(bdescs, dev)
    del frames
    frames = torch.empty(bext, dtype=torch.uint8, device=dev)

    def step_bshuf():
        eng.copy(slab_u8, chunks, d_cd, stream=stream)
        eng.encode_bitshuffle(chunks, d_bdesc, frames, sizes, st, itemsize=4, block=2048, stream=stream)

    step_bshuf()
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0, "bitshuffle encode status errors"
    for k in (0, n // 3, n - 1):
        o = int(bdescs[k]["dst_off"])
        fr = frames[o:o + int(sizes[k])].cpu().numpy().tobytes()
        back = orc.bitshuffle_decode(fr, cbytes, 4)
        assert not isinstance(back, int) and bytes(back) == chunks[k * cbytes:(k + 1) * cbytes].cpu().numpy().tobytes(), \
            f"bitshuffle chunk {k}"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_bshuf()
    torch.cuda.synchronize()
    elb = (time.perf_counter() - t0) / args.steps
    compb = int(sizes.sum())
    kb = isolated_kernel_ms(step_bshuf, eng)
    out["bshuf_encode"] = {"value": round(slab_bytes / elb / 1e9, 2), "unit": "GB/s slab (scatter + encode)",
                           "ms_per_step": round(elb * 1e3, 3), "compressed_bytes": compb,
                           "encode_ms": round(kb, 3),
                           "algorithmic_GBps": round((slab_bytes + compb) / (kb / 1e3) / 1e9, 2),
                           "format": "bitshuffle+LZ4 objects (f32, 2048-element blocks, 12-byte header)"}
    if args.cpu_seconds > 0 and rank == 0:
        from concurrent.futures import ThreadPoolExecutor
        threads = box_threads()
        t1 = time.perf_counter()
        done = 0
        with ThreadPoolExecutor(threads) as ex:
            while time.perf_counter() - t1 < min(args.cpu_seconds / 4, 3.0):
                for r in ex.map(lambda x: orc.bitshuffle_encode(x, 4, 2048), samp):
                    assert len(r) > 12
                done += len(samp)
        cel = time.perf_counter() - t1
        out["bshuf_encode"]["cpu_baseline"] = {
            "value": round(done * cbytes / cel / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{done} x 1 MiB bitshuffle+LZ4 encodes (oracle transposition + greedy LZ4)"}
    if args.cpu_seconds > 0 and rank == 0:
        threads = box_threads()
        # the reference's encoder: libblosc's blosc_compress_ctx(4, shuffle, typesize 1, zlib)
        v, n_enc, _, ver = cpu_encode_libblosc(samp, args.cpu_seconds / 3, threads, clevel=4, cname=b"zlib")
        t1 = time.perf_counter()
        done = 0
        while time.perf_counter() - t1 < args.cpu_seconds / 6:
            orc.encode_batch(samp, op="blosc", typesize=1, clevel=4, shuffle=1, nthreads=threads)
            done += len(samp)
        cel = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
                               "sample": f"{n_enc} x 1 MiB F1 encodes by libblosc {ver} blosc_compress_ctx "
                                         f"(clevel 4, shuffle, typesize 1, zlib: the reference's _compress), "
                                         f"{threads} threads",
                               "port_value": round(done * cbytes / cel / 1e9, 3),
                               "port_sample": f"{done} x 1 MiB F1 encodes (oracle c-blosc + libz L4)"}
    del slab, chunks, frames
    torch.cuda.empty_cache()
    return out


CFG4_DIMS, CFG4_LAYOUT = (131072, 131072), (512, 512)
CFG4_SEL = (slice(0, 131072, 4), slice(0, 131072, 4))


def run_cfg4(args, dev, rank, world):
    """configs[3]: f32 dataset 131072 x 131072 in 1 MiB chunks (65 536 chunks), strided
    selection [::4, ::4] (4 GiB slab), chunks sharded by getObjPartition(chunk_id,
    world) -- HSDS's own DN rule -- over the ranks.  One step = every rank decodes its
    chunks (one batch), packs their selected sub-blocks (one copy launch) and sends
    them to rank 0 over RCCL (one grouped P2P call), rank 0 places every piece into the
    slab (one copy launch).  value = decoded bytes of all ranks / max-over-ranks time."""
    import torch
    import torch.distributed as dist
    from hsds_amd import crawl
    threads = max(1, min(16, (os.cpu_count() or 1) // max(1, world)))
    sc = max(1, args.cfg4_scale)
    dims = tuple(d // sc for d in CFG4_DIMS)
    sel = tuple(slice(0, d, 4) for d in dims)
    plan = crawl.SelectionPlan("d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", dims, CFG4_LAYOUT, sel,
                               np.float32, world)
    ids = plan.chunk_ids(rank)
    nuniq = min(args.cfg4_unique, len(ids))
    raw, enc = make_corpus("F1", nuniq, 20261015 + 7919 * rank, threads)
    blobs = {cid: enc[k % nuniq] for k, cid in enumerate(ids)}
    rd = crawl.ShardedReader(plan, rank, dev)
    st = rd.upload(blobs)
    gathered = torch.empty(max(plan.gathered_nbytes, 1), dtype=torch.uint8, device=dev) if rank == 0 else None
    slab = torch.zeros(max(plan.slab_nbytes, 1), dtype=torch.uint8, device=dev) if rank == 0 else None
    rd.read(st, slab=slab, gathered=gathered, check=True)          # warm-up (+ statuses checked)
    torch.cuda.synchronize()
    ok = 1
    if rank == 0:
        host = slab[:plan.slab_nbytes].view(torch.float32).reshape(plan.slab_shape)
        for r in range(world):                                      # one piece per rank vs its raw chunk
            if not len(plan.by_rank[r]):
                continue
            p = plan.pieces[plan.by_rank[r][0]]
            if r == 0:
                c = raw[0].view(np.float32).reshape(CFG4_LAYOUT)
                ok &= int(np.array_equal(host[p.data_slices].cpu().numpy(), c[p.chunk_slices]))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan_s = 0.0
    for _ in range(args.cfg4_steps):
        tp = time.perf_counter()
        p_ = crawl.SelectionPlan("d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d", dims, CFG4_LAYOUT, sel, np.float32,
                                 world)
        plan_s += time.perf_counter() - tp
        rd.replan(st, p_)
        rd.read(st, slab=slab, gathered=gathered, check=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    el /= args.cfg4_steps
    n_all = len(plan.pieces)
    out = {"value": round(n_all * (1 << 20) / el / 1e9, 2), "unit": "GB/s decoded (all ranks)",
           "selected_GBps": round(plan.slab_nbytes / el / 1e9, 2), "ms_per_step": round(el * 1e3, 3),
           "plan_ms": round(plan_s / args.cfg4_steps * 1e3, 2),
           "chunks": n_all, "chunks_per_rank": [len(b) for b in plan.by_rank],
           "gathered_bytes_from_peers": int(sum(plan.rank_bytes[r] for r in range(1, world))),
           "root_piece_check": bool(ok), "steps": args.cfg4_steps,
           "workload": f"configs[3]: f32 {dims[0]}x{dims[1]}, 512x512 chunks (F1 L4), select [::4, ::4], "
                       "md5-sharded decode + pack + RCCL P2P gather + place on rank 0"}
    del st, gathered, slab
    torch.cuda.empty_cache()
    return out


TRAFFIC_ROUND = "r6"


def run_cfg4_full(args, dev, rank, world):
    """configs[3], full-extent variant: f32 131072 x 131072 in 512x512 chunks, selection
    [:, :] (64 GiB), read as GET_Value streams it -- getSelectionPagination pages of at
    most max_request_size (100 MiB: 659 pages of 199 rows) -- by crawl.PagedReader over the
    md5-sharded chunks, in both modes: "gather" (pack, RCCL gather to rank 0, place, D2H
    of each page) and "direct" (no gather: every GPU writes its pieces of the page straight
    into the pinned host page buffer, shared by the node's ranks through /dev/shm).  The
    stored objects are staged in HBM first (each chunk id its own copy); each page's
    bytes go to a sink that stands in for resp.write."""
    import torch
    import torch.distributed as dist
    from hsds_amd import crawl
    threads = max(1, min(16, (os.cpu_count() or 1) // max(1, world)))
    sc = max(1, args.cfg4_scale)
    dims = tuple(d // sc for d in CFG4_DIMS)
    full_sel = tuple(slice(0, d, 1) for d in dims)
    dset = "d-5a1b2c3d-4e5f6a7b-8c9d-0e1f2a-3b4c5d"
    plan = crawl.SelectionPlan(dset, dims, CFG4_LAYOUT, full_sel, np.float32, world)
    ids = plan.chunk_ids(rank)
    nuniq = min(args.cfg4_unique, len(ids))
    raw, enc = make_corpus("F1", nuniq, 20261015 + 7919 * rank, threads)
    blobs = {cid: enc[k % nuniq] for k, cid in enumerate(ids)}
    first = {cid: k % nuniq for k, cid in enumerate(ids)}
    eng_src = crawl.stage_objects(blobs, ids, dev)
    del blobs
    out = {}
    port = os.environ.get("MASTER_PORT", "0")
    for mode in ("direct", "gather"):
        shm = f"/dev/shm/hsds_amd_bench_{port}_{os.getuid()}" if (mode == "direct" and world > 1) else None
        rd = crawl.PagedReader(dset, dims, CFG4_LAYOUT, full_sel, np.float32, world, rank, dev,
                               max_request_size=args.max_request_size, mode=mode, shm_path=shm)
        checked = {"ok": 1, "bytes": 0}
        c00 = plan.prefix + "0_0"

        def sink(pno, page, b):
            checked["bytes"] += len(b)
            if pno == 0 and c00 in first:
                # row 0, columns 0..511 of the page = row 0 of chunk (0, 0)
                want = raw[first[c00]].view(np.float32)[:CFG4_LAYOUT[1]]
                checked["ok"] &= int(np.array_equal(np.asarray(b[:CFG4_LAYOUT[1] * 4]).view(np.float32), want))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        total = rd.read(eng_src, sink)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        rd.close()
        if shm and rank == 0 and os.path.exists(shm):
            os.unlink(shm)
        out[mode] = {"value": round(total / el / 1e9, 2), "unit": "GB/s selected (response bytes, all ranks)",
                     "seconds": round(el, 3), "pages": len(rd.pages), "response_bytes": total,
                     "chunk_decodes_rank0": rd.stats["decoded"], "chunk_reuses_rank0": rd.stats["reused"],
                     "decode_batches_rank0": rd.stats["decode_batches"],
                     "decoded_GBps": round(len(plan.idx) * plan.chunk_nbytes / el / 1e9, 2),
                     "page0_check": bool(checked["ok"]) if rank == 0 else None}
        del rd
        torch.cuda.empty_cache()
    out["workload"] = (f"configs[3] full extent: f32 {dims[0]}x{dims[1]}, 512x512 chunks (F1 L4), [:, :], "
                       f"GET_Value pagination at max_request_size {args.max_request_size} B, "
                       f"md5-sharded over {world} rank(s)")
    del eng_src
    torch.cuda.empty_cache()
    return out


def load_traffic(args, world, leg=""):
    """HBM bytes per inflate launch (or per cfg3 step, leg="_cfg3") from the committed PMC
    passes (tools/pmc_traffic.sh): 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md
    HBM section) + WRITE_SIZE."""
    p = os.path.join(ROOT, "profiles", f"{TRAFFIC_ROUND}_traffic{leg}.json")
    if not os.path.exists(p):
        return None
    t = json.load(open(p))
    if not leg and (t.get("chunks") != args.chunks or t.get("unique") != args.unique):
        return None
    return t


def box_threads():
    """the host CPUs this run may use: the affinity mask, capped by the CPU share the
    box grants (OMP_NUM_THREADS is set to it on the GPU box; nproc there shows the whole
    machine)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def copy_ceiling(dev, nbytes=2 << 30, reps=5):
    """Measured HIP streaming-copy ceilings (BASELINE 4): a device-to-device
    hipMemcpyAsync (torch copy_) and the engine's copy_kernel over the same bytes as
    1-byte-element records of 256 MiB each (the contiguous byte runs the kernel's 16-byte
    slot path streams: a record's bytes must stay below 2^31); GB/s of read + write
    bytes, HIP events on the launch stream."""
    import torch
    from hsds_amd.engine import ChunkEngine, COPY_DESC_DTYPE, to_device_bytes
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(7)
    piece = 256 << 20
    nrec = nbytes // piece
    rec = np.zeros(nrec, COPY_DESC_DTYPE)
    rec["rank"], rec["itemsize"] = 1, 1
    rec["src_off"] = rec["dst_off"] = np.arange(nrec, dtype=np.uint64) * piece
    rec["count"][:, 0] = piece
    rec["src_stride"][:, 0] = rec["dst_stride"][:, 0] = 1
    d_rec = to_device_bytes(rec, dev)
    eng = ChunkEngine(dev.index)
    stream = torch.cuda.current_stream()
    out = {}
    for name, fn in (("hipMemcpy_d2d", lambda: b.copy_(a)),
                     ("copy_kernel", lambda: eng.copy(a, b, d_rec, stream=stream))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = round(2 * nbytes / (ms / 1e3) / 1e9, 1)
    assert bool((b[:4096] == 7).all()) and bool((b[-4096:] == 7).all())
    del a, b
    torch.cuda.empty_cache()
    return out


def calibration():
    p = os.path.join(ROOT, "profiles", "r2_cpu_calibration.json")
    return json.load(open(p)) if os.path.exists(p) else None


def cpu_baseline(blobs, seconds, threads, compressor="zlib"):
    """Oracle decode (c-blosc frame walk + libz / LZ4, same as the reference path) on
    the box's host cores, bounded to about `seconds` of wall time."""
    from oracle import oracle as orc
    exp = [CHUNK_BYTES] * len(blobs)
    out = [np.empty(CHUNK_BYTES, np.uint8) for _ in blobs]
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, status = orc.uncompress_batch(blobs, exp, compressor, 1, 4, nthreads=threads, out=out)
        assert (status == CHUNK_BYTES).all()
        done += len(blobs)
    el = time.perf_counter() - t0
    return done * CHUNK_BYTES / el / 1e9, done


LIBBLOSC = "/opt/conda/lib/libblosc.so.1"


def cpu_baseline_libblosc(blobs, seconds, threads):
    """The reference's own codec on the box's host cores: numcodecs' Blosc().decode is
    c-blosc's blosc_decompress (storUtil.py:195-208), here the image's libblosc 1.21.0
    (the c-blosc numcodecs 0.12/0.13 vendor), one blosc_decompress_ctx per chunk with one
    internal thread, `threads` chunks at a time, bounded to about `seconds` of wall time.
    Returns (GB/s decoded, chunks decoded, library version string)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    lb = ctypes.CDLL(LIBBLOSC)
    lb.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lb.blosc_decompress_ctx.restype = ctypes.c_int
    lb.blosc_get_version_string.restype = ctypes.c_char_p
    srcs = [np.ascontiguousarray(np.frombuffer(b, np.uint8) if not isinstance(b, np.ndarray) else b) for b in blobs]
    outs = [np.empty(CHUNK_BYTES, np.uint8) for _ in srcs]

    def one(k):
        return lb.blosc_decompress_ctx(srcs[k].ctypes.data, outs[k].ctypes.data, CHUNK_BYTES, 1)
    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            for r in ex.map(one, range(len(srcs))):
                assert r == CHUNK_BYTES, r
            done += len(srcs)
    el = time.perf_counter() - t0
    return done * CHUNK_BYTES / el / 1e9, done, lb.blosc_get_version_string().decode()


def cpu_encode_libblosc(raws, seconds, threads, clevel=4, cname=b"zlib"):
    """The reference's own writer on the box's host cores: storUtil._compress
    (storUtil.py:238-281) is numcodecs' Blosc(cname, clevel, shuffle).encode(bytes), i.e.
    c-blosc's blosc_compress with typesize 1 and the automatic block size -- here the
    image's libblosc 1.21.0 blosc_compress_ctx, one internal thread per call, `threads`
    chunks at a time, bounded to about `seconds` of wall time.  Returns (GB/s of input,
    chunks encoded, compressed bytes of one pass, library version string)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    lb = ctypes.CDLL(LIBBLOSC)
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                      ctypes.c_size_t, ctypes.c_int]
    lb.blosc_compress_ctx.restype = ctypes.c_int
    lb.blosc_get_version_string.restype = ctypes.c_char_p
    srcs = [np.ascontiguousarray(r).reshape(-1).view(np.uint8) for r in raws]
    outs = [np.empty(x.size + 16, np.uint8) for x in srcs]

    def one(k):
        return lb.blosc_compress_ctx(clevel, 1, 1, srcs[k].size, srcs[k].ctypes.data, outs[k].ctypes.data,
                                     outs[k].size, cname, 0, 1)
    done, csum = 0, 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            rs = list(ex.map(one, range(len(srcs))))
            assert min(rs) > 0, rs
            csum = sum(rs)
            done += len(srcs)
    el = time.perf_counter() - t0
    nbytes = sum(x.size for x in srcs) * done // max(1, len(srcs))
    return nbytes / el / 1e9, done, csum, lb.blosc_get_version_string().decode()


def cpu_baseline_bshuf(blobs, seconds, threads):
    """Oracle bitshuffle+LZ4 decode (storUtil._unshuffle codec 2 restated) on the box's
    host cores, one chunk per task, bounded to about `seconds` of wall time."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as orc
    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            for r in ex.map(lambda b: orc.bitshuffle_decode(b, CHUNK_BYTES, 4), blobs):
                assert not isinstance(r, int)
            done += len(blobs)
    el = time.perf_counter() - t0
    return done * CHUNK_BYTES / el / 1e9, done


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_gpus():
    """Number of GPUs this process may use, counted WITHOUT the HIP runtime (the launching
    parent must not touch the GPU): the KFD topology's GPU nodes (simd_count > 0), filtered
    by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as the runtime
    filters them.  HSDS_KFD_TOPOLOGY overrides the topology directory (tests)."""
    import glob
    topo = os.environ.get("HSDS_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    n = 0
    for props in sorted(glob.glob(os.path.join(topo, "*", "properties"))):
        try:
            kv = dict(line.split(None, 1) for line in open(props) if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def launch_ranks(n, argv, dry_run=False):
    """Start one bench.py rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in each
    child's environment), forward their output, return the worst exit status.  The parent
    never imports torch.cuda's runtime: GPUs are counted from the KFD topology
    (visible_gpus), and every rank checks its own device once it starts."""
    import subprocess
    if not dry_run:
        have = visible_gpus()
        if n > have:
            print(f"bench.py: --gpus {n} but {have} visible GPU(s)", file=sys.stderr, flush=True)
            return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def dry_run_rank(args):
    """--dry-run: the rank layout alone over gloo (CPU tests): one JSON line from rank 0
    with the world the collective backend sees."""
    import datetime
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
        t = __import__("torch").tensor([rank])
        dist.all_reduce(t)
        seen = dist.get_world_size()
        assert int(t) == world * (world - 1) // 2
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "rccl_world": seen, "gpus_arg": args.gpus}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", type=int, default=0, help="1: rank layout only, gloo, no GPU (CPU tests)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=4096)
    ap.add_argument("--unique", type=int, default=1024)
    ap.add_argument("--f2", type=int, default=1, help="also measure F2 (HDF5 zlib+shuffle) chunks")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel-timing", type=int, default=0)
    ap.add_argument("--copy-ceiling", type=int, default=1, help="measure the HIP streaming-copy ceiling (2 GiB)")
    ap.add_argument("--e2e", type=int, default=1, help="also measure the PCIe-inclusive rate (N=1)")
    ap.add_argument("--e2e-sub", type=int, default=8, help="PCIe-inclusive rate: pipelined sub-batches")
    ap.add_argument("--cfg3", type=int, default=1, help="also measure configs[2] decode+select (N=1)")
    ap.add_argument("--lz4", type=int, default=1, help="also measure Blosc-lz4 1 MiB chunks (N=1)")
    ap.add_argument("--bshuf", type=int, default=1, help="also measure bitshuffle+LZ4 1 MiB f32 chunks (N=1)")
    ap.add_argument("--cfg1", type=int, default=1, help="also measure configs[0] uncompressed read selection (N=1)")
    ap.add_argument("--zstd", type=int, default=1, help="also measure Blosc-zstd 1 MiB chunks (N=1; needs the image's libblosc)")
    ap.add_argument("--cfg5", type=int, default=1, help="also measure configs[4] scatter+encode (N=1)")
    ap.add_argument("--cfg5w", type=int, default=1, help="configs[4] through the sharded write path (all N)")
    ap.add_argument("--cfg5-steps", type=int, default=3)
    ap.add_argument("--cfg5w-variants", default="full,offset_100_100",
                    help="cfg5w requests: full (aligned), offset_100_100 (edge RMW); the offset one reads its "
                         "edge chunks from the objects the first variant stored")
    ap.add_argument("--cfg4", type=int, default=1,
                    help="configs[3] sharded decode+select (+RCCL gather when N > 1)")
    ap.add_argument("--cfg4-steps", type=int, default=3)
    ap.add_argument("--cfg4-unique", type=int, default=256)
    ap.add_argument("--cfg4-scale", type=int, default=1, help="divide the cfg4 dataset extents (local checks)")
    ap.add_argument("--cfg4-full", type=int, default=1,
                    help="configs[3] full-extent read through GET_Value pagination (gather and no-gather modes)")
    ap.add_argument("--max-request-size", type=int, default=100 << 20, help="SN max_request_size (config.yml: 100m)")
    ap.add_argument("--headline", type=int, default=1,
                    help="0: skip the configs[1] headline and print only the selected legs (profiling passes)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], dry_run=bool(args.dry_run)))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry_run:
        dry_run_rank(args)
        return

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible", file=sys.stderr,
              flush=True)
        sys.exit(2)
    if world > 1:
        import datetime
        torch.distributed.init_process_group("nccl", timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    if not args.headline:
        legs = {}
        if world == 1 and args.cfg3:
            legs["cfg3"] = run_cfg3(args, dev)
        if world == 1 and args.cfg1:
            legs["cfg1"] = run_cfg1(args, dev)
        if world == 1 and args.cfg5:
            legs["cfg5"] = run_cfg5(args, dev, rank)
        if args.cfg5w:
            legs["cfg5_sharded_write"] = run_cfg5_sharded(args, dev, rank, world)
        if args.cfg4 == 1:
            legs["cfg4"] = run_cfg4(args, dev, rank, world)
        if args.cfg4_full:
            legs["cfg4_full"] = run_cfg4_full(args, dev, rank, world)
        if rank == 0:
            print(json.dumps({"metric": "profiling pass (no headline)", "legs": legs}), flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    r1 = run_format("F1", args, dev, rank, world)
    r2 = run_format("F2", args, dev, rank, world) if args.f2 else None

    total_dec = r1["dec_bytes"] * world
    ms_per_step = r1["elapsed_s"] / args.steps * 1e3
    value = total_dec * args.steps / r1["elapsed_s"] / 1e9
    launch_bytes = r1["comp_bytes"] + r1["dec_bytes"]
    achieved = launch_bytes / (r1["kernel_ms"] / 1e3) / 1e9
    out = {
        "metric": "GB/s device-resident chunk decode (shuffle+deflate 1 MiB f32) at 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "rccl_world": torch.distributed.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic smooth f32 round(cumsum(N(0,1)),2), {args.unique} distinct chunks/rank "
                f"stored {args.chunks // args.unique}x at distinct HBM addresses",
        "config": {"workload": "configs[1]: F1 HSDS Blosc-zlib L4 frames, 1 MiB f32 chunks, "
                               f"{args.chunks}-chunk batch per GPU, device-resident",
                   "chunks_per_gpu": args.chunks, "chunk_bytes": CHUNK_BYTES,
                   "compressed_bytes_per_gpu": r1["comp_bytes"], "parallelism": f"chunk-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "inflate2_kernel", "kernel_ms": round(r1["kernel_ms"], 3),
                     "bytes_per_launch": launch_bytes},
    }
    if args.copy_ceiling:
        cc = copy_ceiling(dev)
        out["roofline"]["copy_ceiling_GBps"] = max(cc.values())
        out["roofline"]["copy_ceiling"] = cc
    tr = load_traffic(args, world)
    if tr is not None:
        out["roofline"]["traffic"] = tr["bytes_per_launch"]
        out["roofline"]["traffic_undoubled"] = tr.get("bytes_per_launch_undoubled")
        out["roofline"]["traffic_source"] = tr["source"]
    if r2 is not None:
        v2 = r2["dec_bytes"] * world * args.steps / r2["elapsed_s"] / 1e9
        out["f2"] = {"value": round(v2, 2), "unit": "GB/s", "format": "HDF5 chunk: zlib L4 of byte-shuffled f32",
                     "compressed_bytes_per_gpu": r2["comp_bytes"], "inflate_kernel_ms": round(r2["kernel_ms"], 3)}
    if world == 1 and args.lz4:
        r3 = run_format("LZ4", args, dev, rank, world)
        v3 = r3["dec_bytes"] * args.steps / r3["elapsed_s"] / 1e9
        out["lz4"] = {"value": round(v3, 2), "unit": "GB/s", "format": "Blosc-lz4 frames (typesize 1, 128 KiB blocks)",
                      "compressed_bytes_per_gpu": r3["comp_bytes"], "lz_kernel_ms": round(r3["kernel_ms"], 3),
                      "algorithmic_GBps": round((r3["comp_bytes"] + r3["dec_bytes"]) / (r3["kernel_ms"] / 1e3) / 1e9, 2)}
        if args.cpu_seconds > 0:
            threads = box_threads()
            v, n, ver = cpu_baseline_libblosc(r3["blobs"][:256], min(args.cpu_seconds, 4.0), threads)
            vo, no_ = cpu_baseline(r3["blobs"][:256], min(args.cpu_seconds, 2.0), threads, compressor="lz4")
            out["lz4"]["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
                                          "sample": f"{n} x 1 MiB Blosc-lz4 chunk decodes by libblosc {ver} "
                                                    f"blosc_decompress_ctx (the reference's c-blosc), {threads} threads",
                                          "oracle_port": round(vo, 3)}
        del r3
    if world == 1 and args.e2e:
        out["e2e_pcie"] = run_e2e(r1, args, dev, nsub=args.e2e_sub)
    if world == 1 and args.zstd:
        try:
            zu = args.unique
            args.unique = min(args.unique, 256)
            r4 = run_format("ZSTD", args, dev, rank, world)
            args.unique = zu
            out["zstd"] = {"value": round(r4["dec_bytes"] * args.steps / r4["elapsed_s"] / 1e9, 2), "unit": "GB/s",
                           "format": "Blosc-zstd frames from libblosc 1.21 (level 5, typesize 1)",
                           "compressed_bytes_per_gpu": r4["comp_bytes"], "zstd_kernel_ms": round(r4["kernel_ms"], 3)}
            if args.cpu_seconds > 0:
                threads = box_threads()
                v, n, ver = cpu_baseline_libblosc(r4["blobs"][:64], min(args.cpu_seconds, 4.0), threads)
                vo, no_ = cpu_baseline(r4["blobs"][:64], min(args.cpu_seconds, 2.0), threads, compressor="zstd")
                out["zstd"]["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads,
                                               "kind": "reference",
                                               "sample": f"{n} x 1 MiB Blosc-zstd chunk decodes by libblosc {ver} "
                                                         f"blosc_decompress_ctx (the reference's c-blosc), "
                                                         f"{threads} threads",
                                               "oracle_port": round(vo, 3)}
            del r4
        except Exception as e:   # corpus writer unavailable: the headline stands
            out["zstd"] = {"error": f"{type(e).__name__}: {e}"[:200]}
    if world == 1 and args.bshuf:
        bu = args.unique
        args.unique = min(args.unique, 256)
        r5 = run_format("BSHUF", args, dev, rank, world)
        args.unique = bu
        out["bshuf"] = {"value": round(r5["dec_bytes"] * args.steps / r5["elapsed_s"] / 1e9, 2), "unit": "GB/s",
                        "format": "bitshuffle+LZ4 objects (shuffle=2, f32, 2048-element blocks, 12-byte header)",
                        "compressed_bytes_per_gpu": r5["comp_bytes"], "bshuf_kernel_ms": round(r5["kernel_ms"], 3)}
        if args.cpu_seconds > 0:
            threads = box_threads()
            v, n = cpu_baseline_bshuf(r5["blobs"][:64], min(args.cpu_seconds, 4.0), threads)
            out["bshuf"]["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads, "kind": "port",
                                            "sample": f"{n} x 1 MiB bitshuffle+LZ4 chunk decodes, oracle, "
                                                      f"{threads} threads"}
        del r5
    if world == 1 and args.cfg1:
        out["cfg1"] = run_cfg1(args, dev)
    if world == 1 and args.cfg3:
        out["cfg3"] = run_cfg3(args, dev)
    if world == 1 and args.cfg5:
        out["cfg5"] = run_cfg5(args, dev, rank)
    if args.cfg5w:
        try:
            out["cfg5_sharded_write"] = run_cfg5_sharded(args, dev, rank, world)
        except Exception as e:   # the headline stands even if this leg fails
            out["cfg5_sharded_write"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if args.cfg4 == 1:
        try:
            out["cfg4"] = run_cfg4(args, dev, rank, world)
        except Exception as e:   # the headline stands even if this leg fails
            out["cfg4"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if args.cfg4_full == 1:
        try:
            out["cfg4_full"] = run_cfg4_full(args, dev, rank, world)
        except Exception as e:   # the headline stands even if this leg fails
            out["cfg4_full"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        threads = box_threads()
        sample = r1["blobs"][:256]
        v, n, ver = cpu_baseline_libblosc(sample, args.cpu_seconds, threads)
        v1, n1, _ = cpu_baseline_libblosc(sample[:32], min(3.0, args.cpu_seconds / 4), 1)
        vo, no_ = cpu_baseline(sample, min(4.0, args.cpu_seconds / 2), threads)
        cal = calibration()
        out["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
                               "cpu_model": cpu_model(), "per_core": round(v1, 4),
                               "sample": f"{n} x 1 MiB F1 chunk decodes (256 distinct) in ~{args.cpu_seconds:.0f}s by "
                                         f"libblosc {ver} blosc_decompress_ctx (the c-blosc the reference's numcodecs "
                                         f"vendors; zlib codec), {threads} threads (the box's CPU share); "
                                         f"per_core: {n1} decodes on 1 thread",
                               "oracle_port": round(vo, 3)}
        if cal:
            # oracle / shimmed-reference ratio measured in the build container
            # (tools/calibrate_cpu.py -> profiles/r2_cpu_calibration.json)
            out["cpu_baseline"]["oracle_reference_equiv"] = round(vo / cal["ratio_oracle_over_reference_8"], 3)
            out["cpu_baseline"]["calibration"] = "profiles/r2_cpu_calibration.json"
        if "e2e_pcie" in out:
            # the reference's path starts and ends in host memory too: the same CPU decode
            out["e2e_pcie"]["cpu_baseline"] = dict(out["cpu_baseline"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
