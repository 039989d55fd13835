import os
import sys

import pytest

# the library reads its NGT_AMD_* test knobs only with the master switch set
# (ngt_amd/csrc/knobs.h); tests that force a path set the knob itself
os.environ.setdefault("NGT_AMD_TEST_KNOBS", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(HERE, "golden")
