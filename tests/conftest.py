import os
import sys

import pytest

try:  # load torch's own HIP runtime before libmtg_boss loads /opt/rocm's: a torch device first used
    import torch  # noqa: F401  after the library initialised the GPU reports no device
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture(scope="session")
def transcripts_1000():
    import seq_io  # tests/seq_io.py: the test-side FASTA reader
    return seq_io.read_sequences(os.path.join(GOLDEN, "transcripts_1000.fa"))
