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

# Hardware queues per process for the GPU tests (read when HIP initialises,
# before any test touches the device).  The library's pipelines put fills,
# walks and copies on up to five streams; with HIP's default of 4 queues two
# of them share a queue, which orders their work as if it were one stream
# and hides missing stream waits.  With 8 every stream has a queue of its own
# (tests/test_gpu_atsize.py test_overlapped_alternating_sets fails on a build
# without the overlapped pipeline's walk wait only then:
# profiles/r05_mutation_nowait.txt).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

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
