import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


class DPCases:
    """tests/golden/dp_cases.npz, produced from the reference by make_golden.py."""

    def __init__(self):
        self.d = np.load(os.path.join(GOLDEN, "dp_cases.npz"))
        self.n = int(self.d["n_cases"])

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        p = f"c{i:03d}_"
        return {k[len(p):]: self.d[k] for k in self.d.files if k.startswith(p)}


@pytest.fixture(scope="session")
def dp_cases():
    return DPCases()
