"""A/B of the 256x128 LDS-DMA tile with a 2-buffer (default) vs 3-buffer LDS ring
(AZ_GEMM_RING=3) on the output_transform shape at several M (each in its own subprocess).
    python tools/ring_probe.py [M ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep import run  # noqa: E402

Ms = [int(a) for a in sys.argv[1:]] or [512, 768, 1024, 2048, 65536]
for M in Ms:
    for ring in ("2", "3", "2", "3"):
        env = {"AZ_GEMM_RING": ring}
        r = run(env, M=M)
        print(json.dumps({"M": M, "ring": ring, **r}), flush=True)
for K in (3100, 1000):                 # partial last k-tile of a split (A's tail zeroed)
    for ring in ("2", "3"):
        print(json.dumps({"M": 512, "K": K, "ring": ring, **run({"AZ_GEMM_RING": ring}, 512, 3136, K)}),
              flush=True)
