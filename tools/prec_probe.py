"""x3 (bf16, six products) vs h3 (fp16, three products) GEMM forms, tuning build: time ops.linear
(output_transform shape 3136 x 3136, bias + ReLU) per M under AZ_GEMM_PREC, each form in its own
subprocess, and check the result against float64 (error / sum|a*b| per element, all rows, 512
random columns).  ReLU'd-feature-like A (x >= 0, 30 % zeros) and uniform W.
    python tools/prec_probe.py M1,M2,... [rounds]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch
sys.path.insert(0, "%s/alphazero-gnn_amd")
from azhip import ops
M, N, K = %d, 3136, 3136
g = torch.Generator(device="cuda").manual_seed(M)
x = torch.relu(torch.randn((M, K), device="cuda", generator=g) * 2 - 0.5)
w = (torch.rand((N, K), device="cuda", generator=g) * 2 - 1) / K ** 0.5
b = torch.rand((N,), device="cuda", generator=g) - 0.5
y = torch.empty((M, N), device="cuda")
for _ in range(20):
    ops.linear(x, w, b, act=1, out=y)
torch.cuda.synchronize()
reps = 30
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
for i in range(reps):
    ev[2 * i].record()
    ops.linear(x, w, b, act=1, out=y)
    ev[2 * i + 1].record()
torch.cuda.synchronize()
ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(reps))
us = sum(ts) / reps
cols = torch.randperm(N, device="cuda", generator=g)[:512]
xd, wd = x.double(), w[cols].double()
rows = torch.arange(M, device="cuda") if M <= 8192 else torch.randperm(M, device="cuda", generator=g)[:4096]
ref = torch.relu(xd[rows] @ wd.T + b[cols].double())
scale = xd[rows].abs() @ wd.abs().T + b[cols].double().abs()
err = ((y[rows][:, cols].double() - ref).abs() / (scale + 1e-300))
print(json.dumps({"us": round(us, 2), "us_med": round(ts[reps // 2], 2),
                  "fp32_equiv_tflops": round(2 * M * N * K / us / 1e6, 1),
                  "rel_err_max": float(err.max()), "rel_err_mean": float(err.mean())}))
'''


def run(M, prec):
    env = dict(os.environ, AZ_TUNING_LIB="1", AZ_GEMM_PREC=prec)
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, M)], env=env, capture_output=True,
                       text=True, timeout=300)
    if r.returncode != 0:
        return {"error": r.stderr[-600:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    Ms = [int(m) for m in sys.argv[1].split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    for _ in range(rounds):
        for M in Ms:
            for prec in ("x3", "h3"):
                print(json.dumps({"M": M, "prec": prec, **run(M, prec)}), flush=True)
