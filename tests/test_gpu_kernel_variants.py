"""The A/B kernel variants compute the same bits as the default path.  The switches exist only in
the tuning build (libaz_hip_tuning.so, AZ_TUNING_LIB=1; the product library ignores the
environment); each switch is read once per process, so every variant runs in a child process of
its own on the same inputs, and the product library's default run is compared too:
  - heads: one launch with 2 rows per block (default) vs chunk partials + finalize
    (AZ_HEADS_TWOPASS=1) -- Connect4GNN.py:48-57;
  - the GNN tail's split-K heads: rowsw (default) vs one row per block
    (AZ_SPLITK_HEADS_MODE=rows) vs chunk partials + finalize (=chunks) -- gnn_utils.py:115;
  - the split-K reduce: float4 (default) vs scalar (AZ_GEMM_NOVEC=1);
  - the split-K heads' rows per block: 1 (default) vs 2 / 4 (AZ_SPLITK_HEADS_R);
  - the fp16-form GEMM on pre-split planes (default for registered weights) vs splitting in the
    tile (AZ_GEMM_NOP2=1, and weights outside registered storage), and output_transform.0's
    fused reduce + split of .2's operand vs the plain reduce (AZ_NO_PRESPLIT=1);
  - the fp32 MFMA 256x128 GEMM tile (AZ_GEMM_X3=0, the path before gemm_x3 took these shapes):
    2-buffer vs 3-buffer ring and its stagger (AZ_GEMM_RING=3 / 4): the same k order, so the same
    sums (compared with the fp32 tile's own default, since gemm_x3 sums differently)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1] + "/alphazero-gnn_amd")
import os
from azhip import ops, _lib
out = {}
reg = os.environ.get("AZ_TEST_REGISTER", "1") == "1"   # weights as registered parameter storage
keep = []   # registered weights stay allocated: a freed one's address must not come back as new
F, A = 3136, 8
for B in (33, 100, 512):
    g = torch.Generator().manual_seed(B)
    x = torch.rand((B, F), generator=g) * 2 - 1
    w0 = (torch.rand((F, F), generator=g) * 2 - 1) / F ** 0.5
    w2 = (torch.rand((F, F), generator=g) * 2 - 1) / F ** 0.5
    b0 = (torch.rand((F,), generator=g) - 0.5) * 0.1
    b2 = (torch.rand((F,), generator=g) - 0.5) * 0.1
    wp = (torch.rand((A, F), generator=g) * 2 - 1) / F ** 0.5
    wv = (torch.rand((1, F), generator=g) * 2 - 1) / F ** 0.5
    bp, bv = torch.rand((A,), generator=g) - 0.5, torch.rand((1,), generator=g) - 0.5
    c = [t.cuda() for t in (x, w0, b0, w2, b2, wp, bp, wv, bv)]
    keep.append(c)
    if reg:
        for t in (c[1], c[3]):
            _lib.check(_lib.load().az_weights_register(t.data_ptr(), t.numel() * 4), "register")
    logp, pi, v, y, hid = ops.transform_heads(*c)
    hl, hp_, hv_ = ops.heads(c[0], c[5], c[6], c[7], c[8])
    tl, tp, tv, _, th = ops.transform_heads(*c, want_y=False)   # heads from the GEMM tiles
    for k, t in (("logp", logp), ("pi", pi), ("v", v), ("y", y), ("hid", hid),
                 ("h_logp", hl), ("h_pi", hp_), ("h_v", hv_), ("t_logp", tl), ("t_pi", tp),
                 ("t_v", tv), ("t_hid", th)):
        out["%s_%d" % (k, B)] = t.cpu().numpy()
np.savez(sys.argv[2], **out)
print("ok")
'''

VARIANTS = {
    "default": {},
    "twopass_chunks": {"AZ_HEADS_TWOPASS": "1", "AZ_SPLITK_HEADS_MODE": "chunks"},
    "rows": {"AZ_SPLITK_HEADS_MODE": "rows"},
    "novec": {"AZ_GEMM_NOVEC": "1"},
    "heads_r2": {"AZ_SPLITK_HEADS_R": "2"},
    "heads_r4": {"AZ_SPLITK_HEADS_R": "4"},
    "nop2": {"AZ_GEMM_NOP2": "1"},
    "no_presplit": {"AZ_NO_PRESPLIT": "1"},
    "unregistered": {"AZ_TEST_REGISTER": "0"},
}
FP32_VARIANTS = {
    "fp32": {"AZ_GEMM_X3": "0"},
    "ring3": {"AZ_GEMM_X3": "0", "AZ_GEMM_RING": "3"},
    "ring_stagger": {"AZ_GEMM_X3": "0", "AZ_GEMM_RING": "4"},
    "fp32_novec": {"AZ_GEMM_X3": "0", "AZ_GEMM_NOVEC": "1"},
}


def _run(tmp_path, name, env_extra, tuning=True):
    env = dict(os.environ)
    env.pop("AZ_TUNING_LIB", None)
    if tuning:
        env["AZ_TUNING_LIB"] = "1"
    for k in ("AZ_HEADS_TWOPASS", "AZ_SPLITK_HEADS_MODE", "AZ_GEMM_NOVEC", "AZ_GEMM_RING",
              "AZ_GEMM_X3", "AZ_SPLITK_HEADS_R", "AZ_GEMM_NOP2", "AZ_NO_PRESPLIT",
              "AZ_TEST_REGISTER"):
        env.pop(k, None)
    env.update(env_extra)
    path = str(tmp_path / f"{name}.npz")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(np.load(path))


@pytest.mark.timeout(600)
def test_kernel_variants_bit_identical(tmp_path):
    ref = _run(tmp_path, "default", VARIANTS["default"])
    prod = _run(tmp_path, "product", {}, tuning=False)
    for k, a in ref.items():
        assert np.array_equal(a, prod[k]), f"product library: {k} differs"
    for name, env in VARIANTS.items():
        if name == "default":
            continue
        got = _run(tmp_path, name, env)
        for k, a in ref.items():
            assert np.array_equal(a, got[k]), f"{name}: {k} differs"
    ref32 = _run(tmp_path, "fp32", FP32_VARIANTS["fp32"])
    for name, env in FP32_VARIANTS.items():
        if name == "fp32":
            continue
        got = _run(tmp_path, name, env)
        for k, a in ref32.items():
            assert np.array_equal(a, got[k]), f"{name}: {k} differs"
