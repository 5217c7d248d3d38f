"""GEMM tuning sweep on the GPU box: time az_gemm_f32 for the output_transform shape under
tile/split overrides (each variant in its own subprocess since the overrides are read once)."""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch
sys.path.insert(0, "%s/alphazero-gnn_amd")
from azhip import ops
M, N, K = %d, %d, %d
x = torch.rand((M, K), device="cuda") * 2 - 1
w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
b = torch.rand((N,), device="cuda")
y = torch.empty((M, N), device="cuda")
for _ in range(5):
    ops.linear(x, w, b, act=1, out=y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 50
e0.record()
for _ in range(reps):
    ops.linear(x, w, b, act=1, out=y)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
ref = torch.relu(x.double() @ w.double().T + b.double())
scale = x.double().abs() @ w.double().abs().T
err = float(((y.double() - ref).abs() / (scale + 1e-30)).max())
print(json.dumps({"us": us, "tflops": 2 * M * N * K / us / 1e6, "rel_err": err}))
'''


def run(env, M=512, N=3136, K=3136):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, M, N, K)], env=e,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "sweep"
    if mode == "quick":
        for (M, N, K) in [(512, 3136, 3136), (4096, 3136, 3136), (64, 3136, 3136)]:
            for cfg in ("0", "1", "2", "3", "4", "5"):
                for sk in ("0", "1"):
                    res = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_STREAMK": sk}, M, N, K)
                    print(json.dumps({"M": M, "cfg": cfg, "streamk": sk, **res}), flush=True)
        sys.exit(0)
    if mode == "quickcheck":      # one small run per glds config: correctness before the sweep
        for cfg in sys.argv[2].split(",") if len(sys.argv) > 2 else ("6", "7", "8", "9"):
            for (M, N, K) in [(100, 200, 96), (100, 200, 100), (512, 3136, 3136)]:
                res = run({"AZ_GEMM_CFG": cfg}, M, N, K)
                print(json.dumps({"M": M, "N": N, "K": K, "cfg": cfg, **res}), flush=True)
                if "error" in res or res.get("rel_err", 1) > 1e-5:
                    sys.exit(3)
        sys.exit(0)
    if mode == "glds":
        cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ("0", "6", "7", "8", "9")
        splits = sys.argv[3].split(",") if len(sys.argv) > 3 else ("", "2", "3", "4", "5", "6",
                                                                   "8")
        for (M, N, K) in [(512, 3136, 3136), (256, 3136, 3136), (4096, 3136, 3136)]:
            for cfg in cfgs:
                for sp in splits:
                    env = {"AZ_GEMM_CFG": cfg}
                    if sp == "auto":
                        sp = ""
                    if sp:
                        env["AZ_GEMM_SPLITS"] = sp
                    res = run(env, M, N, K)
                    print(json.dumps({"M": M, "cfg": cfg, "splits": sp or "auto", **res}),
                          flush=True)
        sys.exit(0)
    if mode == "tall":         # config-5 GNN layer shapes: M = V of 512 grids, K <= 128
        for (M, N, K) in [(524288, 256, 64), (524288, 64, 64), (524288, 64, 128)]:
            for cfg in sys.argv[2].split(","):
                env = {"AZ_GEMM_CFG": cfg} if cfg != "auto" else {}
                res = run(env, M, N, K)
                print(json.dumps({"M": M, "N": N, "K": K, "cfg": cfg, **res}), flush=True)
        sys.exit(0)
    if mode == "tallabl":      # epilogue-store ablation on the tall shapes (results wrong by design)
        for (M, N, K) in [(524288, 256, 64), (524288, 64, 64)]:
            for cfg in sys.argv[2].split(","):
                for abl in ("0", "4"):
                    res = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_ABLATE": abl}, M, N, K)
                    print(json.dumps({"M": M, "N": N, "K": K, "cfg": cfg, "ablate": abl, **res}),
                          flush=True)
        sys.exit(0)
    if mode == "longk":        # steady state: K 10x longer, fixed splits (per-block overhead amortised)
        for cfg in sys.argv[2].split(","):
            for abl in sys.argv[3].split(","):
                res = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_ABLATE": abl, "AZ_GEMM_SPLITS": "5"},
                          512, 3136, 31360)
                print(json.dumps({"M": 512, "K": 31360, "cfg": cfg, "ablate": abl, **res}),
                      flush=True)
        sys.exit(0)
    if mode == "tallk":        # gemm_tall (default dispatch) vs the tile kernels (AZ_GEMM_NOTALL)
        for (M, N, K) in [(524288, 256, 64), (524288, 64, 64), (524288, 64, 128),
                          (524288, 128, 64), (20007, 64, 64)]:
            for env in ({}, {"AZ_GEMM_NOTALL": "1"}, {"AZ_GEMM_ABLATE": "4"},
                        {"AZ_GEMM_ABLATE": "8"}):
                res = run(env, M, N, K)
                print(json.dumps({"M": M, "N": N, "K": K, "env": env, **res}), flush=True)
        sys.exit(0)
    if mode == "kslice":       # gemm_kslice (M = 512) vs the split-K tile (default dispatch)
        for env in ({"AZ_GEMM_KSLICE": "1"}, {}):
            print(json.dumps({"env": env, **run(env)}), flush=True)
        sys.exit(0)
    if mode == "mgrid":        # default dispatch vs cfg x split at given M (self-play batch sizes)
        Ms = [int(x) for x in sys.argv[2].split(",")]
        cfgs = sys.argv[3].split(",")
        splits = sys.argv[4].split(",")
        for M in Ms:
            print(json.dumps({"M": M, "cfg": "default", **run({}, M=M)}), flush=True)
            for cfg in cfgs:
                for sp in splits:
                    r = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_SPLITS": sp}, M=M)
                    print(json.dumps({"M": M, "cfg": cfg, "splits": sp, **r}), flush=True)
        sys.exit(0)
    if mode == "bigm":         # large-batch output_transform (also B = 65,536)
        M = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
        for cfg in sys.argv[2].split(","):
            r = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_SPLITS": "1"}, M=M)
            print(json.dumps({"M": M, "cfg": cfg, **r}), flush=True)
        sys.exit(0)
    if mode == "x3":           # fp32 on the bf16 matrix cores (gemm_x3) vs the fp32 MFMA tiles
        # argv: Ms  tiles  splits ("auto" = the dispatch's own choice)
        shapes = [tuple(int(v) for v in (x + ":3136:3136").split(":")[:3])
                  for x in sys.argv[2].split(",")]     # "M" or "M:N:K"
        tiles = sys.argv[3].split(",")
        splits = sys.argv[4].split(",")
        for (M, N, K) in shapes:
            print(json.dumps({"M": M, "N": N, "K": K, "x3": "off",
                              **run({"AZ_GEMM_X3": "0"}, M, N, K)}), flush=True)
            for t in tiles:
                for sp in splits:
                    env = {"AZ_GEMM_X3": t}
                    if sp != "auto":
                        env["AZ_GEMM_SPLITS"] = sp
                    print(json.dumps({"M": M, "N": N, "K": K, "x3": t, "splits": sp,
                                      **run(env, M, N, K)}), flush=True)
        sys.exit(0)
    if mode == "ablate":       # glds2 timing ablations (results wrong by design)
        cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ("15", "16")
        abls = sys.argv[3].split(",") if len(sys.argv) > 3 else ("0", "1", "2", "3")
        for (M, N, K) in [(512, 3136, 3136), (4096, 3136, 3136)]:
            for cfg in cfgs:
                for abl in abls:
                    res = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_ABLATE": abl}, M, N, K)
                    print(json.dumps({"M": M, "cfg": cfg, "ablate": abl, **res}), flush=True)
        sys.exit(0)
    shapes = [(512, 3136, 3136), (4096, 3136, 3136), (64, 3136, 3136), (64, 6272, 3136),
              (4096, 256, 64)]
    for (M, N, K) in shapes:
        for cfg in ("0", "1", "2", "3", "4", "5"):
            for sk in ("0", "1"):
                res = run({"AZ_GEMM_CFG": cfg, "AZ_GEMM_STREAMK": sk}, M, N, K)
                print(json.dumps({"M": M, "N": N, "K": K, "cfg": cfg, "streamk": sk, **res}),
                      flush=True)
        print(json.dumps({"M": M, "N": N, "K": K, "cfg": "auto", **run({}, M, N, K)}), flush=True)
