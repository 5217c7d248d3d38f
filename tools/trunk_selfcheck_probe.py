"""Probe: where the two-blocks-per-CU trunk goes wrong.  Runs c4_trunk (AZ_TRUNK_NB boards per
block) on libaz_hip_exp.so built with -DAZ_TRUNK_SMALL_UNION -DAZ_TRUNK_SELFCHECK: every thread
re-derives conv1 items and compares them with the planes image in LDS right after it is written
(phase 0: own item, 1: another wave's) and at the end of the block (phase 2); mismatches are
logged with the block, thread and HW_ID.  Also counts output rows that differ from the oracle.
    AZ_AB_LIB=libaz_hip_exp.so AZ_TUNING_LIB=1 AZ_TRUNK_NB=1 python tools/trunk_selfcheck_probe.py [B,...]"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    from azhip import ops
    from azhip._lib import lib
    from azhip.nets import C4Evaluator
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from oracle import nets as O
    Wnp = synthetic_state_dict(connect4_net_spec(7), 1)
    ev = C4Evaluator(Wnp, synthetic_state_dict(gnn_spec(3136, 2), 2), device=torch.device("cuda"))
    Wn = ev.nnet.params
    W64 = {k: np.asarray(v, np.float64) for k, v in Wnp.items()}
    log = torch.zeros(64 + 48 * 2048, dtype=torch.int32, device="cuda")
    L = lib()
    L.az_debug_trunk_chk.argtypes = [ctypes.c_void_p]
    assert L.az_debug_trunk_chk(ctypes.c_void_p(log.data_ptr())) == 0
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "512,1576").split(",")]
    for B in Bs:
        rng = np.random.default_rng(B)
        bnp = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
        boards = torch.from_numpy(bnp).cuda()
        ref = torch.from_numpy(O.c4_features(bnp, W64)).cuda()
        for rep in range(6):
            log.zero_()
            f = ops.c4_trunk(boards, Wn)
            torch.cuda.synchronize()
            err = (f.double() - ref).abs().amax(1)
            rows = torch.nonzero(err > 1e-4).flatten().cpu().numpy()
            lg = log.cpu().numpy().view(np.uint32)
            n = int(lg[0])
            ent = lg[64:64 + 48 * min(n, 2048)].reshape(-1, 48)
            ph = collections.Counter(ent[:, 3].tolist())
            blocks = sorted(set(ent[:, 0].tolist()))
            nconv = int((ent[:, 5] > 0).sum())
            print(f"B={B} rep {rep}: bad rows {len(rows)} {rows[:6].tolist()} | c1 mismatches {n} "
                  f"by phase {dict(ph)} conv1-recompute mismatches {nconv} blocks {blocks[:8]}",
                  flush=True)
            if n and rep < 2:
                for e in ent[:10]:
                    hw = int(e[6])
                    wave, simd, cu, sh, se = hw & 15, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
                    print(f"   blk {e[0]} tid {e[1]} (wave {e[1] // 64} lane {e[1] % 64}) item {e[2]} "
                          f"phase {e[3]} words {e[4]} conv {e[5]} sa {e[7:8].view(np.float32)[0]} "
                          f"hw wave {wave} simd {simd} cu {cu} se {se}", flush=True)
                    print("      image", " ".join(f"{x:08x}" for x in e[8:16]),
                          "\n      split", " ".join(f"{x:08x}" for x in e[16:24]),
                          "\n      v    ", e[24:32].view(np.float32).tolist(),
                          "\n      v2   ", e[32:40].view(np.float32).tolist(), flush=True)
                bad_items = collections.Counter((int(e[2]) for e in ent))
                lanes = collections.Counter((int(e[1]) % 64 for e in ent))
                hw_waves = collections.Counter((int(e[6]) & 15 for e in ent))
                print("   items", sorted(bad_items)[:40], "lanes", sorted(lanes)[:64],
                      "hw wave ids", dict(hw_waves), flush=True)


if __name__ == "__main__":
    main()
