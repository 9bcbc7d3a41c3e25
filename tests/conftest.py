"""Shared test setup.

* `gpu` marker: tests that need an MI355X (run with `-m gpu` on the GPU box).
* Puts the repo root (for `oracle`) and shuffle-coding_amd/ (for `ans_amd`) on sys.path
  and builds the in-tree libraries if they are missing (CPU-only build works here).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "shuffle-coding_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

if not os.path.exists(os.path.join(PKG, "lib", "libshufflecoding_amd.so")):
    subprocess.check_call(["make", "-s", "-C", PKG])
if not os.path.exists(os.path.join(ROOT, "oracle", "build", "libans_oracle.so")):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def multiset_masses():
    return np.asarray(load_json("masses_multiset.json")["masses"], dtype=np.uint64)


@pytest.fixture(scope="session")
def multiset_vectors():
    """The reference's fixtures multiset-data/{1000,10000,100000}.txt (src/multiset.rs:161-166)."""
    import ans_amd
    return {n: np.asarray(ans_amd.read_multiset(os.path.join(GOLDEN, f"multiset_{n}.txt")), dtype=np.uint32)
            for n in (1000, 10000, 100000)}


@pytest.fixture(scope="session")
def golden_multiset():
    return load_json("golden_multiset.json")


@pytest.fixture(scope="session")
def golden_small():
    return load_json("golden_small.json")["cases"]
