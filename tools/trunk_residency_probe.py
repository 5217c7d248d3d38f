"""Probe: the Connect4 trunk with two blocks per CU (AZ_AB_LIB=libaz_hip_exp.so, a tuning build
with -DAZ_TRUNK_SMALL_UNION) -- rows that differ from the float64 oracle over repeats, and the
kernel time, for AZ_TRUNK_NB / AZ_TRUNK_DYN_LDS set by the caller.
    python tools/trunk_residency_probe.py [B,B,...]"""
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
    Wn = ev.nnet.params
    W64 = {k: np.asarray(v, np.float64) for k, v in Wnp.items()}
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1576").split(",")]
    tag = f"nb={os.environ.get('AZ_TRUNK_NB', 'model')} dyn={os.environ.get('AZ_TRUNK_DYN_LDS', '0')}"
    for B in Bs:
        rng = np.random.default_rng(B)
        bnp = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
        boards = torch.from_numpy(bnp).cuda()
        ref = torch.from_numpy(O.c4_features(bnp, W64)).cuda()
        bad_runs = []
        first = None
        for rep in range(8):
            f = ops.c4_trunk(boards, Wn)
            torch.cuda.synchronize()
            err = (f.double() - ref).abs().amax(1)
            rows = torch.nonzero(err > 1e-4).flatten().cpu().numpy()
            bad_runs.append(len(rows))
            if first is None and len(rows):
                first = rows[:8].tolist()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            ops.c4_trunk(boards, Wn)
        e0.record()
        for _ in range(20):
            ops.c4_trunk(boards, Wn)
        e1.record()
        torch.cuda.synchronize()
        print(f"B={B} {tag}: bad rows per run {bad_runs} first {first} "
              f"us/call {e0.elapsed_time(e1) * 1e3 / 20:.1f}", flush=True)


if __name__ == "__main__":
    main()
