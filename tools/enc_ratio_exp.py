"""CPU-emulation size experiment for the deflate parse (test infrastructure): first-column
and spread chunks of a cfg5-like slab, emulator stream size / CPython zlib size at L4,
per 256 KiB split.  Usage: python tools/enc_ratio_exp.py [chain ...]"""
import ctypes, os, sys, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, os.environ.get("EMU_LIB", "tests/emu/libdeflate_emu.so")))
L.emu_deflate_far.restype = ctypes.c_int64
L.emu_deflate_far.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int]
rng = np.random.default_rng(7)
cols = 512 * 4
rows = 512
walk = np.round(np.cumsum(rng.normal(size=(rows, cols)), axis=1), 2).astype(np.float32)
first = [walk[:, 0:512].copy().tobytes()]
spread = [walk[:, 512 * k:512 * (k + 1)].copy().tobytes() for k in (2, 3)]
def emu(b, chain, far):
    a = np.frombuffer(b, np.uint8)
    out = np.zeros(len(b) // 4 + 1024, np.uint32)
    r = L.emu_deflate_far(a.ctypes.data, len(b), out.ctypes.data, len(b) + 4096, 4, chain, far)
    assert r > 0 and zlib.decompress(out.view(np.uint8)[:r].tobytes()) == b
    return r
S = 1 << 18
for spec in (sys.argv[1:] or ["4"]):
    chain, far = (int(spec.rstrip("f")), 1) if spec.endswith("f") else (int(spec), 0)
    res = []
    for name, cs in (("first", first), ("spread", spread)):
        ours = ref = 0
        for c in cs:
            for o in range(0, len(c), S):
                ours += emu(c[o:o + S], chain, far)
                ref += len(zlib.compress(c[o:o + S], 4))
        res.append(f"{name} {ours / ref:.4f}")
    print(f"chain {spec:>4s}: " + ", ".join(res), flush=True)
