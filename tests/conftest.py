import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    # Build the in-tree library and the CPU oracle if this checkout has not been built yet.
    lib = os.path.join(ROOT, "rustnetworkstack_amd", "librns_checksum.so")
    orc = os.path.join(ROOT, "oracle", "build", "libcsum_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.check_call(["make", "-s", "-C", ROOT, "-j8"])


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import get_oracle
    return get_oracle()


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def sweep():
    import json
    with open(os.path.join(GOLDEN, "sweep_vectors.json")) as f:
        return json.load(f)


def expand_fragment(spec: str) -> bytes:
    """Fixture fragment notation: hex string, or REPEAT:<hex>:<count>."""
    if spec.startswith("REPEAT:"):
        _, hx, cnt = spec.split(":")
        return bytes.fromhex(hx) * int(cnt)
    return bytes.fromhex(spec)


def sweep_arena(sweep):
    """Rebuild the arena a sweep fixture was generated over (see tests/golden/make_golden.py)."""
    import numpy as np

    from oracle.oracle import splitmix64_bytes
    rnd = splitmix64_bytes(sweep["seed"], sweep["random_bytes"])
    e = sweep["edge_bytes"]
    return np.concatenate([rnd, np.zeros(e, dtype=np.uint8), np.full(e, 0xFF, dtype=np.uint8)])
