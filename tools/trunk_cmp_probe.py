"""Probe: Connect4 trunk determinism and agreement -- c4_gnn_eval's trunk (split-A form) vs
az_c4_trunk_fwd with registered / unregistered weights, three repeats each, and the rows that
differ against the oracle.  AZ_TUNING_LIB=1 AZ_TRUNK_NB=<n> forces the boards per block.
    python tools/trunk_cmp_probe.py [B,B,...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    from azhip import ops
    from azhip.nets import C4Evaluator
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from oracle import nets as O
    Wnp = synthetic_state_dict(connect4_net_spec(7), 1)
    ev = C4Evaluator(Wnp, synthetic_state_dict(gnn_spec(3136, 2), 2), device=torch.device("cuda"))
    Wn, Gn = ev.nnet.params, ev.gnn.params
    Wc = {k: Wn[k].clone() for k in Wn.keys()}
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "512,1576,3150").split(",")]
    for B in Bs:
        rng = np.random.default_rng(B)
        bnp = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
        boards = torch.from_numpy(bnp).cuda()
        outs = {}
        for rep in range(3):
            feat = torch.empty((B, 3136), device="cuda")
            hidden = torch.empty((B, 3136), device="cuda")
            ops.c4_gnn_eval(boards, Wn, Gn, feat=feat, hidden=hidden)
            outs[f"eval{rep}"] = feat
            outs[f"reg{rep}"] = ops.c4_trunk(boards, Wn)
            outs[f"unreg{rep}"] = ops.c4_trunk(boards, Wc)
        torch.cuda.synchronize()
        base = outs["unreg0"]
        bad = set()
        line = []
        for k, f in outs.items():
            rows = torch.nonzero((f != base).any(1)).flatten().cpu().numpy()
            bad.update(rows.tolist())
            line.append(f"{k}:{len(rows)}")
        err = {}
        if bad:
            sel = np.array(sorted(bad))[:16]
            ref = O.c4_features(bnp[sel], {k: np.asarray(v, np.float64) for k, v in Wnp.items()})
            for k, f in outs.items():
                err[k] = float(np.abs(f[torch.from_numpy(sel).cuda()].double().cpu().numpy() - ref).max())
        if bad:
            r0 = sorted(bad)[0]
            for k, f in outs.items():
                dif = torch.nonzero(f[r0] != base[r0]).flatten().cpu().numpy()
                if len(dif):
                    co, p = dif // 49, dif % 49
                    print(f"  row {r0} {k}: {len(dif)} values differ, channels {sorted(set(co.tolist()))[:20]}"
                          f" positions {sorted(set(p.tolist()))[:20]}", flush=True)
                    break
        print(f"B={B} nb={os.environ.get('AZ_TRUNK_NB', 'model')} rows differing from unreg0: "
              + " ".join(line), "first", sorted(bad)[:8],
              "max err vs oracle on them:", {k: round(v, 5) for k, v in err.items()}, flush=True)


if __name__ == "__main__":
    main()
