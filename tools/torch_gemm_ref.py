"""Vendor-library reference point (not product code): torch.nn.functional.linear in fp32 on
the GPU box (rocBLAS / hipBLASLt) at the shapes az_gemm_f32 is tuned for."""
import json
import torch

torch.backends.cuda.matmul.allow_tf32 = False
for (M, N, K) in [(512, 3136, 3136), (256, 3136, 3136), (4096, 3136, 3136), (4096, 4096, 4096)]:
    x = torch.rand((M, K), device="cuda") * 2 - 1
    w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
    b = torch.rand((N,), device="cuda")
    for _ in range(5):
        y = torch.nn.functional.linear(x, w, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        y = torch.nn.functional.linear(x, w, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(json.dumps({"M": M, "N": N, "K": K, "us": round(us, 1),
                      "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
