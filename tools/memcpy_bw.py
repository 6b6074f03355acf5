"""Diagnostic: host copy rate of N ~0.6 MB bytes objects into one page-locked buffer by a
thread pool of T workers (the DN read path's staging step), for a few T."""
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def main():
    n, sz = 256, 600_000
    blobs = [os.urandom(sz) for _ in range(n)]
    host = torch.empty(n * sz, dtype=torch.uint8, pin_memory=True)
    h = host.numpy()

    def put(k0, k1):
        for k in range(k0, k1):
            h[k * sz:(k + 1) * sz] = np.frombuffer(blobs[k], np.uint8)
    for t in (1, 4, 8, 16, 32):
        pool = ThreadPoolExecutor(max_workers=t)
        parts = max(t, 32)
        cuts = [n * i // parts for i in range(parts + 1)]
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            list(pool.map(lambda i: put(cuts[i], cuts[i + 1]), range(parts)))
            best = min(best, time.perf_counter() - t0)
        print(f"threads {t:3d}: {n * sz / best / 1e9:6.1f} GB/s ({best * 1e3:.2f} ms for {n * sz / 1e6:.0f} MB)")
        pool.shutdown()


if __name__ == "__main__":
    main()
