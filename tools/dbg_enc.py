"""debug: codec._shuffle(2, ...) over the bitshuffle golden cases, one at a time"""
import ctypes
import json
import os
import sys
import numpy as np
sys.path.insert(0, os.getcwd())
import torch  # noqa: F401
from hsds_amd import codec
hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p
meta = json.load(open("tests/golden/bitshuffle_cases.json"))
arrs = np.load("tests/golden/bitshuffle_cases.npz")
for c in meta["cases"]:
    if c["status"] != "ok" or c["block"] != 2048:
        continue
    raw = arrs[c["name"] + "__raw"].tobytes()
    dt = np.dtype("S%d" % c["itemsize"]) if c["itemsize"] not in (1, 2, 4, 8, 16) else np.dtype({1: "u1", 2: "<u2", 4: "<u4", 8: "<u8", 16: "<c16"}[c["itemsize"]])
    try:
        got = codec._shuffle(2, raw, chunk_shape=(c["nbytes"] // c["itemsize"],), dtype=dt)
        print("ok", c["name"], len(got), flush=True)
    except Exception as e:
        print("ERR", c["name"], c["nbytes"], c["itemsize"], e, hip.hipGetErrorString(hip.hipGetLastError()), flush=True)
        break
