"""Diagnostic: pinned host <-> device copy rates on this box (the DN read path's PCIe
ceiling), for a few sizes, one stream and H2D || D2H on two streams."""
import time

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    dev = torch.device("cuda", 0)
    for mb in (16, 64, 256):
        n = mb << 20
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        h2d = rate(lambda: d.copy_(h, non_blocking=True), n)
        d2h = rate(lambda: h.copy_(d, non_blocking=True), n)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d2 = torch.empty(n, dtype=torch.uint8, device=dev)

        def both():
            with torch.cuda.stream(s1):
                d.copy_(h, non_blocking=True)
            with torch.cuda.stream(s2):
                h2.copy_(d2, non_blocking=True)
        bi = rate(both, 2 * n)
        print(f"{mb:4d} MiB  H2D {h2d:6.1f} GB/s  D2H {d2h:6.1f} GB/s  both {bi:6.1f} GB/s (sum)")
    # 150 MB host-to-device in pieces (the read batch's staged upload)
    n = 150 << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for parts in (1, 4, 16, 64, 256):
        cuts = [n * i // parts for i in range(parts + 1)]

        def pieces():
            for i in range(parts):
                d[cuts[i]:cuts[i + 1]].copy_(h[cuts[i]:cuts[i + 1]], non_blocking=True)
        print(f"150 MiB H2D in {parts:3d} pieces: {rate(pieces, n):6.1f} GB/s")


if __name__ == "__main__":
    main()
