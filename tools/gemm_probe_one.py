"""20 launches of the B = 512 output_transform GEMM (512 x 3136 x 3136, bias + ReLU) for
counter collection: `python3 tools/gemm_probe_one.py [kslice|tile]` (kslice = gemm_kslice via
the tuning build's AZ_GEMM_KSLICE; tile = the default split-K tile path)."""
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "kslice":
    os.environ["AZ_TUNING_LIB"] = "1"
    os.environ["AZ_GEMM_KSLICE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
import torch  # noqa: E402
from azhip import ops  # noqa: E402

M = N = K = 3136
M = 512
x = torch.rand((M, K), device="cuda") * 2 - 1
w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
b = torch.rand((N,), device="cuda")
y = torch.empty((M, N), device="cuda")
for _ in range(20):
    ops.linear(x, w, b, act=1, out=y)
torch.cuda.synchronize()
print("ok", flush=True)
