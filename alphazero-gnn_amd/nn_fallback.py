"""Process-wide accounting of network-failure fallbacks (failure detection).

The reference degrades a failed leaf evaluation to uniform priors over the valid moves and a
value of 0, and only logs it (MCTS.py:195-200).  Every search path here keeps that behaviour
(the Python MCTS, the lock-step drivers, the native engine, the arena players), but each
degraded leaf is also counted here, so that a kernel which starts raising cannot hide behind
plausible-looking self-play throughput:

* tests/conftest.py fails every test that ends with a non-zero count (unless the test injects
  failures on purpose and says so with @pytest.mark.nn_failures_expected);
* bench.py reports the count of its self-play leg and fails when it is non-zero;
* AZ_STRICT_NN=1 turns the degradation into an exception at the site (NNFailure).

The root `predict` of expand_tree is unguarded in the reference (MCTS.py:108-113): a failure
there propagates, here too, and is not a fallback.
"""
import logging
import os
import threading

log = logging.getLogger("nn_fallback")

_lock = threading.Lock()
_counts = {}


class NNFailure(RuntimeError):
    """Raised at a fallback site under AZ_STRICT_NN=1."""


def strict():
    return os.environ.get("AZ_STRICT_NN", "0") not in ("", "0")


def record(site, exc, leaves=1):
    """`leaves` leaf evaluations at `site` fell back to uniform priors / v=0 because of `exc`."""
    leaves = int(leaves)
    with _lock:
        _counts[site] = _counts.get(site, 0) + leaves
    log.error("Error in neural network prediction (%s: %d leaf evaluation(s) degraded to "
              "uniform priors, value 0): %r", site, leaves, exc)
    if strict():
        raise NNFailure(f"{site}: network evaluation failed ({exc!r})") from exc


def total():
    with _lock:
        return sum(_counts.values())


def counts():
    with _lock:
        return dict(_counts)


def reset():
    with _lock:
        _counts.clear()
