import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import os, sys, time, json, torch
sys.path.insert(0, "/root/repo/alphazero-gnn_amd")
from azhip import ops
n = 119645192
p = torch.randn(n, device="cuda"); g = torch.randn(n, device="cuda")
m = torch.zeros(n, device="cuda"); v = torch.zeros(n, device="cuda")
for step in range(1, 4): ops.adam(p, g, m, v, 1e-3, step)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for step in range(4, 24): ops.adam(p, g, m, v, 1e-3, step)
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(json.dumps({"U": os.environ.get("AZ_ADAM_U"), "us": round(us, 1), "GBps": round(28 * n / us / 1e3, 1)}))
