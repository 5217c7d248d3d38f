"""Time ops.linear (output_transform shape, 3136 x 3136, bias + ReLU) at the given M values with
HIP events: python tools/gemm_ab.py M1,M2,... [reps]  (one JSON line per M)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402

Ms = [int(m) for m in sys.argv[1].split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
N = K = 3136
w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
if os.environ.get("AZ_PROBE_REGISTER", "1") == "1":      # as parameter storage (the product path)
    from azhip import _lib
    _lib.check(_lib.load().az_weights_register(w.data_ptr(), w.numel() * 4), "az_weights_register")
b = torch.rand((N,), device="cuda")
for M in Ms:
    x = torch.rand((M, K), device="cuda") * 2 - 1
    y = torch.empty((M, N), device="cuda")
    for _ in range(3):
        ops.linear(x, w, b, act=1, out=y)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        ops.linear(x, w, b, act=1, out=y)
    e[1].record()
    torch.cuda.synchronize()
    us = e[0].elapsed_time(e[1]) / reps * 1e3
    print(json.dumps({"M": M, "us": round(us, 2), "fp32_equiv_tflops": round(2 * M * N * K / us / 1e6, 1),
                      "bf16_frac": round(6 * 2 * M * N * K / us / 1e6 / 2516.6, 4),
                      "lib": os.environ.get("AZ_AB_LIB", "libaz_hip.so")}), flush=True)
