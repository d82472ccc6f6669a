"""Shared fixtures.  `-m gpu` tests need a HIP device and call the product
through the C ABI (libgx_amd.so); the CPU oracle (oracle/) is the checker."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "genomics-rs_amd"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
FASTA = os.path.join(GOLDEN, "fasta")
COMPARISON = os.path.join(GOLDEN, "comparison_data")

# config.toml:1-5 and tests/test_alignment.rs:4-11
CONFIG_SCORES = (1, -2, -1, -5)
TEST_SCORES = (1, -2, -2, -5)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); calls the HIP product")
    config.addinivalue_line("markers", "slow: large inputs (30k x 30k)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.build()
    o.load()
    return o


@pytest.fixture(scope="session")
def gx():
    import gxamd
    return gxamd


@pytest.fixture(scope="session")
def ctx(gx):
    c = gx.Context(0)
    yield c
    c.close()


def read_fasta_records(path):
    """Oracle-side FASTA parse (from_fasta restatement) -> [(name, seq bytes)]."""
    import oracle as o
    with open(path, "rb") as f:
        return o.fasta_parse(f.read())
