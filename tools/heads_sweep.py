"""Trunk (AZ_TRUNK_NB) and heads (AZ_HEADS_R) variants at the batch sizes the bench and the
self-play rounds run (each variant in its own process; the overrides are read once).  Also checks
that every heads variant returns the default's bits.   python tools/heads_sweep.py"""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")
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
out = ops.heads(feat, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"], W["fc_value.bias"])
hd = t(lambda: ops.heads(feat, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"], W["fc_value.bias"]))
np.save("%s", torch.cat([o.reshape(B, -1) for o in out], 1).cpu().numpy())
print(json.dumps({"trunk_us": tr, "heads_us": hd}))
'''


def run(env, B, tag):
    e = dict(os.environ)
    e.update(env)
    path = f"/tmp/heads_{tag}.npy"
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, B, path)], env=e,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}, None
    import numpy as np
    return json.loads(r.stdout.strip().splitlines()[-1]), np.load(path)


if __name__ == "__main__":
    import numpy as np
    # python tools/heads_sweep.py [B,B,...] [all|twopass|trunk]
    Bs = [int(b) for b in sys.argv[1].split(",")] if len(sys.argv) > 1 else [512, 1024, 1576, 2048, 4096]
    which = sys.argv[2] if len(sys.argv) > 2 else "all"
    envs = ([{"AZ_HEADS_TWOPASS": "1"}] if which == "twopass" else
            [{"AZ_TRUNK_NB": str(n)} for n in (1, 2, 3, 4, 5, 6, 7, 8)] if which == "trunk" else
            [{"AZ_HEADS_R": "2"}, {"AZ_HEADS_R": "4"}, {"AZ_HEADS_R": "8"}, {"AZ_TRUNK_NB": "1"},
             {"AZ_TRUNK_NB": "2"}, {"AZ_TRUNK_NB": "4"}, {"AZ_TRUNK_NB": "8"},
             {"AZ_HEADS_TWOPASS": "1"}])
    for B in Bs:
        base, ref = run({}, B, "base")
        print(json.dumps({"B": B, "variant": "default", **base}), flush=True)
        for env in envs:
            res, out = run(env, B, "v")
            same = bool(out is not None and ref is not None and np.array_equal(out, ref))
            print(json.dumps({"B": B, "variant": env, "bit_identical": same, **res}), flush=True)
