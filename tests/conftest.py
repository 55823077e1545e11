"""Shared fixtures.  ``-m gpu`` tests need a gfx950 device; everything else runs on CPU."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle.oracle import OracleLib
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return OracleLib(path)


@pytest.fixture(scope="session")
def random_golden():
    """F3/F5 fixture: 4096 tuples x 4 keys with reference hashes and sweep queues."""
    d = np.load(os.path.join(GOLDEN, "random_tuples.npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    out["ports"] = (((out["sport"] & 0xFFFF) << 16) | (out["dport"] & 0xFFFF)).astype(np.uint32)
    out["tuples"] = np.stack([out["sip"], out["dip"], out["ports"]], axis=1).astype(np.uint32)
    out["key_list"] = [[int(x) for x in out["keys"][k][:out["key_len"][k]]] for k in range(4)]
    with open(os.path.join(GOLDEN, "sweep_counts.json")) as f:
        out["sweep_counts"] = json.load(f)
    return out


@pytest.fixture(scope="session")
def example_key():
    with open(os.path.join(GOLDEN, "example_input", "hash_key.txt")) as f:
        return [int(x, 16) for x in f.read().split(":")]


@pytest.fixture(scope="session")
def edge_cases():
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        return json.load(f)
