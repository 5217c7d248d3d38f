"""GEMV timing for the small-batch evaluation: y = relu(x W^T + b), W 3136 x 3136, M = 1..8 rows,
events over 200 back-to-back launches; AZ_GEMV_ROWS (tuning build) picks the gemv_rows shape."""
import json
import os
import sys

os.environ.setdefault("AZ_TUNING_LIB", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
import torch  # noqa: E402
from azhip import ops  # noqa: E402

N = K = 3136
g = torch.Generator().manual_seed(0)
w = ((torch.rand((N, K), generator=g) * 2 - 1) / K ** 0.5).cuda()
b = torch.rand((N,), generator=g).cuda()
x = torch.rand((8, K), generator=g).cuda()
out = {"rows": os.environ.get("AZ_GEMV_ROWS", "default")}
for M in range(1, 9):
    xm = x[:M].contiguous()
    y = torch.empty((M, N), device="cuda")
    for _ in range(20):
        ops.linear(xm, w, b, act=1, out=y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        ops.linear(xm, w, b, act=1, out=y)
    e1.record()
    torch.cuda.synchronize()
    out[M] = round(e0.elapsed_time(e1) / 200 * 1e3, 2)
print(json.dumps(out), flush=True)
