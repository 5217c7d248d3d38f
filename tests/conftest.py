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
    config.addinivalue_line("markers", "nn_failures_expected: the test injects network "
                                       "failures on purpose (skips the zero-fallback check)")


@pytest.fixture(autouse=True)
def _no_silent_nn_fallbacks(request):
    """the reference silently degrades a failed network call to uniform priors
    and v=0 (MCTS.py:195-200).  Every such event is counted (nn_fallback); a test that ends
    with a non-zero count fails, so a broken kernel cannot pass as degraded play."""
    import nn_fallback
    nn_fallback.reset()
    yield
    if request.node.get_closest_marker("nn_failures_expected") is None:
        assert nn_fallback.total() == 0, f"network fallbacks occurred: {nn_fallback.counts()}"
    nn_fallback.reset()


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def split_weights(z, prefix):
    return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


@pytest.fixture(scope="session")
def c4_gnn_weights():
    from azhip.weights import gnn_spec, synthetic_state_dict
    seed = int(golden("c4_gnn.npz")["seed"])
    return synthetic_state_dict(gnn_spec(3136, 2), seed)


def report(name, **fields):
    """Append one JSON line to $AZ_REPORT_DIR/margins.jsonl (no-op without the variable)."""
    d = os.environ.get("AZ_REPORT_DIR")
    if d:
        import json
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "margins.jsonl"), "a") as f:
            f.write(json.dumps({"check": name, **fields}) + "\n")


def assert_close(name, got, ref, tol=1e-5, rel_floor=None):
    """max |got - ref| <= tol (or, with rel_floor, max |got - ref| / max(rel_floor, |ref|) <=
    tol: used for log-probabilities, whose magnitude reaches hundreds on trained weights, where
    one fp32 ulp is already > 1e-5).  Records the error and the margin tol / error."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    if rel_floor is not None:
        err = err / np.maximum(np.abs(ref), rel_floor)
    worst = float(err.max()) if err.size else 0.0
    report(name, max_err=worst, tol=tol, margin=(tol / worst if worst > 0 else float("inf")),
           n=int(err.size), relative=rel_floor is not None)
    assert worst <= tol, (name, worst, tol)
    return worst


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
