"""Time az_gnn_aggregate_fwd on the config-5 per-GPU shard (512 32x32 grids, F=64) under the
AZ_AGG_CFG tuning variants (each in its own process: the override is read once)."""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch
sys.path.insert(0, "%s"); sys.path.insert(0, "%s/alphazero-gnn_amd")
import bench
from azhip import ops
r = bench.aggregate_roofline(torch, ops, torch.device("cuda", 0), graphs=%d, full_graphs=0)
print(json.dumps(r))
'''
for graphs in (512, 4096):
    for cfg in sys.argv[1].split(",") if len(sys.argv) > 1 else ("0", "1", "2"):
        e = dict(os.environ, AZ_AGG_CFG=cfg)
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, ROOT, graphs)], env=e,
                           capture_output=True, text=True, timeout=300)
        out = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-300:]
        print(json.dumps({"graphs": graphs, "cfg": cfg, "res": out}), flush=True)
