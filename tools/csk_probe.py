"""Cycled stream-K A/B (tuning build): time ops.linear (output_transform shape, 3136 x 3136,
bias + ReLU) at self-play M values under AZ_CSK plans, each plan in its own subprocess (the
override is read once), and check every result against float64 (error / sum|a*b| per element).

    python tools/csk_probe.py "M:plan;plan|M:plan..."   plan = off | auto | an,bf,at,bt
"""
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
x = torch.rand((M, K), device="cuda", generator=g) * 2 - 1
w = (torch.rand((N, K), device="cuda", generator=g) * 2 - 1) / K ** 0.5
b = torch.rand((N,), device="cuda", generator=g)
y = torch.empty((M, N), device="cuda")
for _ in range(30):
    ops.linear(x, w, b, act=1, out=y)
torch.cuda.synchronize()
reps = 40
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
for i in range(reps):
    ev[2 * i].record()
    ops.linear(x, w, b, act=1, out=y)
    ev[2 * i + 1].record()
torch.cuda.synchronize()
ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(reps))
us = sum(ts) / reps
xd, wd = x.double(), w.double()
ref = torch.relu(xd @ wd.T + b.double())
scale = xd.abs() @ wd.abs().T + b.double().abs()
err = float(((y.double() - ref).abs() / (scale + 1e-30)).max())
y2 = torch.empty_like(y)
ops.linear(x, w, b, act=1, out=y2)
torch.cuda.synchronize()
print(json.dumps({"us": round(us, 2), "us_min": round(ts[0], 2), "us_med": round(ts[reps // 2], 2),
                  "bf16_frac": round(6 * 2 * M * N * K / us / 1e6 / 2516.6, 4),
                  "rel_err": err, "deterministic": bool(torch.equal(y, y2))}))
'''


def run(M, plan):
    env = dict(os.environ, AZ_TUNING_LIB="1", AZ_CSK_PRINT="1")
    if plan != "auto":
        env["AZ_CSK"] = plan
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, M)], env=env, capture_output=True,
                       text=True, timeout=300)
    info = [l for l in r.stderr.splitlines() if l.startswith("csk ")]
    if r.returncode != 0:
        return {"error": r.stderr[-400:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["plan_used"] = info[-1] if info else "gemm_x3_sk (no csk)"
    return out


if __name__ == "__main__":
    spec = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    for _ in range(rounds):
        for part in spec.split("|"):
            M, plans = part.split(":")
            for plan in plans.split(";"):
                res = run(int(M), plan)
                print(json.dumps({"M": int(M), "plan": plan, **res}), flush=True)
