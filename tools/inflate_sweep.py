"""CPU sweep of the inflate kernel's window parameters through the single-source
emulator (tests/emu/inflate_emu.cpp): builds one emulator per -D variant and reports
decode correctness plus the per-window work model (speculative steps of the slowest
lane, repair rounds, windows) on the bench's F1 chunk generator.  Development tool.

  python tools/inflate_sweep.py "HZ_CMAX=256" "HZ_CMAX=288" --tune 384,96,1,288,4
"""
import argparse
import ctypes
import os
import subprocess
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(defs, out):
    flags = [f"-D{d}" for d in defs if d]
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", *flags, "-o", out,
                    os.path.join(ROOT, "tests", "emu", "inflate_emu.cpp"), "-lz"], check=True)
    lib = ctypes.CDLL(out)
    lib.emu_inflate.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_void_p]
    return lib


def chunks(n, seed=0, shuffled=True):
    """bench.py's F2 streams (smooth f32 chunks, byte-shuffled, zlib level 4) or,
    unshuffled, the F1 payload"""
    from bench import smooth_chunk
    out = []
    for i in range(n):
        raw = smooth_chunk(seed + i).view(np.uint8)
        raw = (raw.reshape(-1, 4).T if shuffled else raw).tobytes()
        out.append((raw, zlib.compress(raw, 4)))
    return out


def run(lib, data, tune):
    tot = np.zeros(14, np.uint64)
    for raw, comp in data:
        src = np.frombuffer(comp, np.uint8)
        dst = np.zeros(len(raw), np.uint8)
        st = np.zeros(14, np.uint64)
        r = lib.emu_inflate(src.ctypes.data, len(comp), dst.ctypes.data, len(raw), *tune, st.ctypes.data)
        if r != 0 or dst.tobytes() != raw:
            return None
        tot += st
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+", help="comma-separated -D lists, e.g. HZ_CMAX=288,HZ_SLOTS=52")
    ap.add_argument("--tune", action="append", default=None, help="L0,W,adapt,C,rounds (repeatable)")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--raw", action="store_true", help="unshuffled payload (F1-like)")
    a = ap.parse_args()
    tunes = [tuple(int(x) for x in t.split(",")) for t in (a.tune or ["384,96,1,192,4"])]
    data = chunks(a.chunks, shuffled=not a.raw)
    nbytes = sum(len(r) for r, _ in data)
    for k, v in enumerate(a.variants):
        lib = build(v.split(","), f"/tmp/libinflate_sweep{k}.so")
        for t in tunes:
            s = run(lib, data, t)
            if s is None:
                print(f"{v:36s} {t} DECODE MISMATCH")
                continue
            win, smax, rep, rmax = int(s[0]), int(s[9]), int(s[11]), int(s[5])
            print(f"{v:36s} {str(t):24s} windows {win:6d} B/win {nbytes / win:7.0f} "
                  f"steps_max/win {smax / win:6.1f} repairs/win {rep / win:5.2f} rsteps/win {rmax / win:6.1f} "
                  f"work/KB {(smax + rmax) * 1024 / nbytes:6.2f}")


if __name__ == "__main__":
    main()
