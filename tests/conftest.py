import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "alphazero-gnn_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds on CPU")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def split_weights(z, prefix):
    return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


@pytest.fixture(scope="session")
def c4_gnn_weights():
    from azhip.weights import gnn_spec, synthetic_state_dict
    seed = int(golden("c4_gnn.npz")["seed"])
    return synthetic_state_dict(gnn_spec(3136, 2), seed)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
