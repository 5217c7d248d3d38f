"""The stream-K heads path at self-play batch sizes: ops.linear_heads(want_y=False) on
output_transform.2's shape (3136 x 3136, 7 actions) at each M given, REPS calls each, so a
rocprofv3 kernel trace / PMC pass sees gemm_x3_csk<..., HEADS> + heads_tiles_finalize_kernel<true>
per M (grid size tells the M apart).   python tools/csk_heads_probe.py 800,1576,3150 50"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402

Ms = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "800,1576,3150").split(",")]
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
g = torch.Generator(device="cuda").manual_seed(0)
F, A = 3136, 7
w = torch.randn(F, F, device="cuda", generator=g) * F ** -0.5
b = torch.randn(F, device="cuda", generator=g) * 0.01
wp = torch.randn(A, F, device="cuda", generator=g) * F ** -0.5
bp = torch.zeros(A, device="cuda")
wv = torch.randn(1, F, device="cuda", generator=g) * F ** -0.5
bv = torch.zeros(1, device="cuda")
for M in Ms:
    x = torch.relu(torch.randn(M, F, device="cuda", generator=g))
    for _ in range(REPS):
        ops.linear_heads(x, w, b, wp, bp, wv, bv, want_y=False)
    torch.cuda.synchronize()
    print(f"M={M} done", flush=True)
