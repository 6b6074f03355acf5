"""CPU-baseline calibration, build container only.

Times the reference's own storUtil._uncompress (imported through tests/golden/refshim.py:
numcodecs re-expressed over the image's libblosc 1.21.0) against the oracle's C restatement
(oracle/oracle.c orc_uncompress_batch) on the same F1 corpus (1 MiB smooth f32, Blosc-zlib
L4, typesize 1, byte shuffle), at 1 core and at 8 cores.  The reference is one process per
core (HSDS data nodes are single-threaded asyncio processes), the oracle one thread per
core.  Writes profiles/r2_cpu_calibration.json; the ratio converts the on-box oracle
cpu_baseline into the reference's rate.  Never runs on the GPU box."""
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CHUNK = 1 << 20
NCHUNK = 64


def corpus():
    from oracle import oracle as orc
    out = []
    for i in range(NCHUNK):
        g = np.random.default_rng(20261015 + i)
        raw = np.round(np.cumsum(g.normal(size=CHUNK // 4)), 2).astype(np.float32).view(np.uint8)
        out.append(np.frombuffer(orc.blosc_encode(raw.tobytes(), typesize=1, clevel=4, shuffle=1), np.uint8))
    return out


def _ref_worker(args):
    blobs, seconds = args
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import refshim  # noqa: F401
    from hsds.util import storUtil as su
    dt = np.dtype("<f4")
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for b in blobs:
            out = su._uncompress(b.tobytes(), compressor="deflate", shuffle=1, dtype=dt, chunk_shape=(CHUNK // 4,))
            assert len(out) == CHUNK
            n += 1
    return n, time.perf_counter() - t0


def ref_rate(blobs, procs, seconds):
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_ref_worker, [(blobs, seconds)] * procs)
    return sum(n for n, _ in res) * CHUNK / max(t for _, t in res) / 1e9


def oracle_rate(blobs, threads, seconds):
    from oracle import oracle as orc
    out = [np.empty(CHUNK, np.uint8) for _ in blobs]
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, st = orc.uncompress_batch(blobs, [CHUNK] * len(blobs), "zlib", 1, 4, nthreads=threads, out=out)
        assert (st == CHUNK).all()
        n += len(blobs)
    return n * CHUNK / (time.perf_counter() - t0) / 1e9


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    blobs = corpus()
    res = {"cpu_model": cpu_model(), "cpus": os.cpu_count(), "chunks": NCHUNK, "chunk_bytes": CHUNK,
           "format": "F1 Blosc-zlib L4, typesize 1, byte shuffle, smooth f32", "unit": "GB/s decoded"}
    for cores in (1, 8):
        r = ref_rate(blobs, cores, 6.0)
        o = oracle_rate(blobs, cores, 6.0)
        res[f"reference_{cores}"] = round(r, 4)
        res[f"oracle_{cores}"] = round(o, 4)
        res[f"ratio_oracle_over_reference_{cores}"] = round(o / r, 3)
        print(cores, "cores: reference", round(r, 4), "oracle", round(o, 4), "ratio", round(o / r, 3), flush=True)
    with open(os.path.join(ROOT, "profiles", "r2_cpu_calibration.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
