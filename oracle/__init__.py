"""ORACLE — TEST INFRASTRUCTURE ONLY.

A plain numpy (and, for gradients, torch-CPU-fp32) restatement of the reference
andrpac/alphazero-gnn hot path.  Every function cites the reference file:line it follows.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``
may import anything from here, and only as the checker / the timed CPU baseline.
The product (``alphazero-gnn_amd/``) never imports it: its compute runs on the HIP
library and fails loudly when that library or a GPU is missing.

Parity pinning: the restatement is checked against golden vectors captured from the
reference itself in the build container (``tests/golden/make_goldens.py``), see
``tests/test_oracle_golden.py``.
"""
