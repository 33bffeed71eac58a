import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


# Core parity evidence first: a failure in a feature test (graph replay, pool,
# BC / PPO) under `-x` must not leave the oracle comparison of the hot path
# unreached (round-4 verdict).  Stable within a file.
_FIRST = ("test_gpu_parity.py", "test_gpu_split.py", "test_gpu_full_scale.py", "test_gpu_rows_shapes.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)
    items[:] = [it for _, it in sorted(enumerate(items), key=lambda t: (rank(t[1]), t[0]))]


def golden_cases():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f[0] == "c")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
