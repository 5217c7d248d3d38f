"""A/B of the 256x128 LDS-DMA tile variants on the output_transform shape (each run in its own
subprocess): AZ_GEMM_RING = 2 (default 2-buffer), 3 (3-buffer ring), 4 (ring + stagger),
5 / 6 (the same two with the 32x32x2 MFMA).
    python tools/ring_probe.py [M ...]"""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep import run  # noqa: E402

Ms = [int(a) for a in sys.argv[1:]] or [512, 768, 1024, 65536]
RINGS = os.environ.get("RINGS", "2,3,4,5,6").split(",")
for M in Ms:
    for rep in range(2):
        for ring in RINGS:
            r = run({"AZ_GEMM_RING": ring}, M=M)
            print(json.dumps({"M": M, "ring": ring, **r}), flush=True)
for K in (3100, 1000):                 # partial last k-tile of a split (A's tail zeroed)
    for ring in RINGS:
        print(json.dumps({"M": 512, "K": K, "ring": ring,
                          **run({"AZ_GEMM_RING": ring}, 512, 3136, K)}), flush=True)
