"""Run one GEMM shape repeatedly (for rocprofv3 counter passes): python tools/gemm_one.py M N K reps"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402

M, N, K, reps = (int(a) for a in sys.argv[1:5])
x = torch.rand((M, K), device="cuda") * 2 - 1
w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
b = torch.rand((N,), device="cuda")
y = torch.empty((M, N), device="cuda")
for _ in range(reps):
    ops.linear(x, w, b, act=1, out=y)
torch.cuda.synchronize()
print("ok")
