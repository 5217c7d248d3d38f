"""fp16-form GEMM on pre-split planes (tuning tile 16; with AZ_P3_REUSE=1 the planes are split
once, so the call is the tile kernel + reduce) vs the product fp16 form splitting in the tile
(tuning tile 1): HIP-event time per call, error vs float64, a hash of the output bits.  One
process per tile (the dispatch reads its environment once):
    AZ_TUNING_LIB=1 AZ_GEMM_X3=16 AZ_P3_REUSE=1 python tools/p2h_probe.py 512,4096 [reps]"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402

Ms = [int(m) for m in sys.argv[1].split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
N = K = 3136
g = torch.Generator(device="cuda").manual_seed(0)
w = (torch.rand((N, K), device="cuda", generator=g) * 2 - 1) / K ** 0.5
if os.environ.get("AZ_PROBE_REGISTER", "1") == "1":      # as parameter storage: W's planes cached
    from azhip import _lib
    _lib.check(_lib.load().az_weights_register(w.data_ptr(), w.numel() * 4), "az_weights_register")
b = torch.rand((N,), device="cuda", generator=g)
for M in Ms:
    x = torch.rand((M, K), device="cuda", generator=g) * 2 - 1
    y = torch.empty((M, N), device="cuda")
    for _ in range(30):
        ops.linear(x, w, b, act=1, out=y)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        ops.linear(x, w, b, act=1, out=y)
    ev[1].record()
    torch.cuda.synchronize()
    ref = (x.double() @ w.double().T + b.double()).clamp_min(0)
    print(json.dumps({"M": M, "tile": os.environ.get("AZ_GEMM_X3"),
                      "us": round(ev[0].elapsed_time(ev[1]) / reps * 1e3, 2),
                      "maxerr": float((y.double() - ref).abs().max()),
                      "hash": hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:12]}),
          flush=True)
