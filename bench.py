"""Headline benchmark: GB/s of device-resident chunk decode (shuffle+deflate L4, 1 MiB
float32 chunks) -- BASELINE.json `metric`, configs[1] (4096-chunk batch per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

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
    else:
        shuf = [np.frombuffer(orc.shuffle(r, 4), np.uint8) for r in raw]
        blobs = orc.encode_batch(shuf, op="zlib", clevel=4, nthreads=threads)
    return raw, blobs


def run_format(fmt, args, dev, rank, world):
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    threads = min(16, os.cpu_count() or 1)
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

    def step():
        eng.decode(d_src, d_desc, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4, stream=stream)

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


def cpu_baseline(blobs, seconds, threads):
    """Oracle decode (c-blosc frame walk + libz, same as the reference path) on the
    box's host cores, bounded to about `seconds` of wall time."""
    from oracle import oracle as orc
    exp = [CHUNK_BYTES] * len(blobs)
    out = [np.empty(CHUNK_BYTES, np.uint8) for _ in blobs]
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, status = orc.uncompress_batch(blobs, exp, "zlib", 1, 4, nthreads=threads, out=out)
        assert (status == CHUNK_BYTES).all()
        done += len(blobs)
    el = time.perf_counter() - t0
    return done * CHUNK_BYTES / el / 1e9, done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=4096)
    ap.add_argument("--unique", type=int, default=1024)
    ap.add_argument("--f2", type=int, default=1, help="also measure F2 (HDF5 zlib+shuffle) chunks")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel-timing", type=int, default=0)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.distributed.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

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
                     "kernel": "inflate_kernel", "kernel_ms": round(r1["kernel_ms"], 3),
                     "bytes_per_launch": launch_bytes},
    }
    if r2 is not None:
        v2 = r2["dec_bytes"] * world * args.steps / r2["elapsed_s"] / 1e9
        out["f2"] = {"value": round(v2, 2), "unit": "GB/s", "format": "HDF5 chunk: zlib L4 of byte-shuffled f32",
                     "compressed_bytes_per_gpu": r2["comp_bytes"], "inflate_kernel_ms": round(r2["kernel_ms"], 3)}
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        threads = min(16, os.cpu_count() or 1)
        sample = r1["blobs"][:256]
        v, n = cpu_baseline(sample, args.cpu_seconds, threads)
        out["cpu_baseline"] = {"value": round(v, 3), "unit": "GB/s", "cores": threads, "kind": "port",
                               "sample": f"{n} x 1 MiB F1 chunk decodes (256 distinct) in ~{args.cpu_seconds:.0f}s, "
                                         f"oracle c-blosc frame walk + libz inflate, {threads} threads"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
