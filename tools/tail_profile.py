"""Diagnostic: wave-level load balance of inflate2_kernel at the bench configuration
(HZ_PROFILE build, tools/libhsds_prof.so).  From the 100 MHz real-time clock: kernel span
(first wave start -> last wave end), mean and earliest wave end, the waves' summed stream
decode time against span x waves (the busy fraction), and the longest single stream."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from hsds_amd import _native  # noqa: E402

_native.LIB_PATH = os.environ.get("HZ_PROF_LIB") or os.path.join(ROOT, "tools", "libhsds_prof.so")
L = _native.lib()
L.hsds_debug_tail.argtypes = [ctypes.c_void_p, ctypes.c_int]
from bench import make_corpus, CHUNK_BYTES  # noqa: E402
from hsds_amd.engine import ChunkEngine, pack_chunks  # noqa: E402


def run(fmt, n, unique):
    raw, blobs = make_corpus(fmt, unique, 20261015, 16)
    src, descs, ext = pack_chunks([blobs[i % unique] for i in range(n)], [CHUNK_BYTES] * n)
    dev = torch.device("cuda", 0)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.empty(ext, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    buf = (ctypes.c_ulonglong * 8)()
    for rep in range(3):
        L.hsds_debug_tail(buf, 1)
        eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=1, itemsize=4)
        torch.cuda.synchronize()
        L.hsds_debug_tail(buf, 0)
        t0, t1, sum_end, waves, busy, longest, min_end = buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6]
        span = (t1 - t0) / 1e5          # ms
        mean_end = (sum_end / waves - t0) / 1e5
        print(f"{fmt} n={n} waves={waves} kernel={eng.last_inflate_ms():.2f} ms span={span:.2f} ms "
              f"first wave end={(min_end - t0) / 1e5:.2f} ms mean wave end={mean_end:.2f} ms "
              f"busy={busy / (waves * (t1 - t0)):.3f} longest stream={longest / 1e5:.3f} ms")
    assert (d_st.cpu().numpy() == 0).all()


if __name__ == "__main__":
    run("F1", int(os.environ.get("HZ_TAIL_N", "4096")), 1024)
    run("F2", int(os.environ.get("HZ_TAIL_N", "4096")), 1024)
