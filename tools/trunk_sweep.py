"""Time az_c4_trunk_fwd and the heads entry points at B = 512 / 4096 under AZ_TRUNK_NB
variants (each in its own process: the override is read once)."""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch, numpy as np
sys.path.insert(0, "%s/alphazero-gnn_amd")
from azhip import ops
from azhip.weights import connect4_net_spec, synthetic_state_dict
B = %d
W = {k: torch.from_numpy(v).cuda() for k, v in synthetic_state_dict(connect4_net_spec(7), 1).items()}
boards = torch.from_numpy(np.random.default_rng(0).integers(-1, 2, (B, 7, 7)).astype(np.int8)).cuda()
feat = torch.empty((B, 3136), device="cuda")
def t(fn, reps=50):
    for _ in range(5): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
tr = t(lambda: ops.c4_trunk(boards, W, out=feat))
hd = t(lambda: ops.heads(feat, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"], W["fc_value.bias"]))
print(json.dumps({"trunk_us": tr, "heads_us": hd}))
'''
for B in (512, 4096):
    for nb in sys.argv[1].split(","):
        e = dict(os.environ)
        if nb != "auto":
            e["AZ_TRUNK_NB"] = nb
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, B)], env=e, capture_output=True,
                           text=True, timeout=300)
        out = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-300:]
        print(json.dumps({"B": B, "nb": nb, "res": out}), flush=True)
