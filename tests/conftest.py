import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "codec_cases.json")))
    arrs = np.load(os.path.join(ROOT, "tests", "golden", "codec_cases.npz"))
    return d, arrs


@pytest.fixture(scope="session")
def golden2():
    """lz4 / lz4hc / blosclz / zstd Blosc objects (tests/golden/make_codec2_golden.py)"""
    import json
    import numpy as np
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "codec2_cases.json")))
    arrs = np.load(os.path.join(ROOT, "tests", "golden", "codec2_cases.npz"))
    return d, arrs


@pytest.fixture(scope="session")
def bshuf_golden():
    """bitshuffle+LZ4 HSDS frames (tests/golden/make_bitshuffle_golden.py)"""
    import json
    import numpy as np
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "bitshuffle_cases.json")))
    arrs = np.load(os.path.join(ROOT, "tests", "golden", "bitshuffle_cases.npz"))
    return d, arrs


@pytest.fixture(scope="session")
def selection_golden():
    import json
    return json.load(open(os.path.join(ROOT, "tests", "golden", "selection_cases.json")))


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as orc
    orc.lib()
    return orc


@pytest.fixture(scope="session")
def blosc_bit_golden():
    """Blosc frames with the bitshuffle flag (tests/golden/make_blosc_bitshuffle_golden.py)"""
    import json
    import numpy as np
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "blosc_bitshuffle_cases.json")))
    arrs = np.load(os.path.join(ROOT, "tests", "golden", "blosc_bitshuffle_cases.npz"))
    return d, arrs
