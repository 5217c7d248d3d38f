"""az_c4_trunk_heads_fwd at the given B under env variants (each in its own process; tuning
build): time per call and bit-identity of (feat, logp, pi, v) with the default.
  python tools/trunk_heads_probe.py B1,B2,..."""
import json
import os
import subprocess
import sys

os.environ.setdefault("AZ_TUNING_LIB", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch, numpy as np
sys.path.insert(0, "%s/alphazero-gnn_amd")
from azhip import ops
from azhip.weights import connect4_net_spec, synthetic_state_dict
B = %d
W = {k: torch.from_numpy(v).cuda() for k, v in synthetic_state_dict(connect4_net_spec(7), 1).items()}
boards = torch.from_numpy(np.random.default_rng(0).integers(-1, 2, (B, 7, 7)).astype(np.int8)).cuda()
out = ops.c4_trunk_heads(boards, W)
for _ in range(5): ops.c4_trunk_heads(boards, W)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): ops.c4_trunk_heads(boards, W)
e1.record(); torch.cuda.synchronize()
np.save("%s", torch.cat([o.reshape(B, -1) for o in out], 1).cpu().numpy())
print(json.dumps({"us": e0.elapsed_time(e1) / 50 * 1e3}))
'''


def run(env, B, tag):
    e = dict(os.environ)
    e.update(env)
    path = f"/tmp/th_{tag}.npy"
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, B, path)], env=e,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}, None
    import numpy as np
    return json.loads(r.stdout.strip().splitlines()[-1]), np.load(path)


if __name__ == "__main__":
    import numpy as np
    for B in [int(b) for b in sys.argv[1].split(",")]:
        base, ref = run({}, B, "base")
        print(json.dumps({"B": B, "variant": "default", **base}), flush=True)
        for env in ({"AZ_TRUNK_HEADS_FUSED": "1"}, {"AZ_TRUNK_HEADS_FUSED": "2"}):
            res, o = run(env, B, "v")
            same = bool(o is not None and ref is not None and np.array_equal(o, ref))
            print(json.dumps({"B": B, "variant": env, "bit_identical": same, **res}), flush=True)
