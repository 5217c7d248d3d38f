"""CPU checks of the drop-in boundary: libaz_hip.so builds, loads without a GPU and exports
every entry point include/az_hip.h declares; the ctypes binding covers exactly those."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "az_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(az_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def built():
    from azhip.build import build
    return build(verbose=False)


def test_header_declares_entry_points():
    names = declared()
    for must in ("az_gemm_f32", "az_c4_trunk_fwd", "az_heads_fwd", "az_gnn_aggregate_fwd",
                 "az_gnn_attn_score_fwd", "az_gnn_layer_fwd", "az_mlp2_fwd", "az_adam_f32"):
        assert must in names


def test_library_exports_every_declared_symbol(built):
    lib = ctypes.CDLL(built)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_matches_header(built):
    from azhip import _lib
    assert sorted(_lib.SIGNATURES) == declared()
    L = _lib.load()
    assert L.az_abi_version() == 2
    assert L.az_last_error() == b""


def test_struct_layouts_match_header(built, tmp_path):
    """ctypes mirrors of az_gemm_desc / az_graph / az_gnn_layer_w: every field offset and the
    struct sizes agree with what a C compiler makes of include/az_hip.h."""
    import shutil
    import subprocess
    from azhip import _lib
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    structs = {"az_gemm_desc": _lib.GemmDesc, "az_graph": _lib.Graph, "az_gnn_layer_w": _lib.LayerW,
               "az_c4_eval": _lib.C4Eval}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(){"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run([cc, str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                 check=True).stdout.splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_ops_fail_loudly_without_gpu(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from azhip import _lib
    with pytest.raises(RuntimeError, match="no HIP device"):
        _lib.lib()


def test_host_side_validation_without_gpu(built):
    """Argument checks of the leaf-evaluation entry points run on the host before any HIP call:
    B = 0 is a no-op, bad shapes / null pointers return AZ_EINVAL with a message (the
    reference's exceptions become status codes at this boundary)."""
    from azhip import _lib
    L = _lib.load()
    AZ_OK, AZ_EINVAL = 0, -1
    d = _lib.C4Eval()
    d.max_B = 4
    assert L.az_c4_eval_fwd(ctypes.byref(d), None, 0, None, None, None, None, None) == AZ_OK
    assert L.az_c4_eval_fwd(ctypes.byref(d), None, 5, None, None, None, None, None) == AZ_EINVAL
    assert b"max_B" in L.az_last_error()
    assert L.az_c4_eval_fwd(ctypes.byref(d), None, 1, None, None, None, None, None) == AZ_EINVAL
    assert b"null" in L.az_last_error()
    args = [None] * 6 + [None, None, 8, None, None] + [None] * 4 + [None, 0, None]
    assert L.az_c4_trunk_heads_fwd(None, 0, *args[2:]) == AZ_OK
    assert L.az_c4_trunk_heads_fwd(None, 3, *args[2:]) == AZ_EINVAL
    bad_a = list(args[2:])
    bad_a[6] = 40                                     # A > 32
    assert L.az_c4_trunk_heads_fwd(None, 3, *bad_a) == AZ_EINVAL
    assert b"A=40" in L.az_last_error()
    assert L.az_host_free(None) == AZ_OK


def test_unsupported_action_size_rejected_up_front():
    """A board whose action size exceeds the heads kernels' limit (TicTacToe n >= 6: A = 37) is
    rejected when the wrapper is built, with a clear error -- not per predict, where MCTS would
    swallow it and play a whole iteration on uniform priors (MCTS.py:195-200)."""
    from tictactoe.TicTacToeGNN import TicTacToeGNNWrapper
    from tictactoe.TicTacToeGame import TicTacToeGame
    with pytest.raises(ValueError, match="action size 37"):
        TicTacToeGNNWrapper(TicTacToeGame(6), {"use_gnn": True, "gnn_layers": 2})


def _device_code_objects(so_path):
    """The gfx950 code objects inside a HIP shared library: its .hip_fatbin section is one
    clang offload bundle per translation unit (-fno-gpu-rdc), each a header of (offset, size,
    target triple) entries."""
    import struct
    import subprocess
    import tempfile
    objcopy = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", so_path, os.devnull],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], blob.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(magic, pos + 32)
    return out


@pytest.mark.parametrize("name", ["libaz_hip.so", "libaz_hip_tuning.so"])
def test_device_code_has_no_packed_fp32(built, name, tmp_path):
    """Regression guard for the round-6 finding (azhip/build.py NO_PK_F32): packed-FP32
    VALU instructions (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) returned wrong low elements in
    lanes 48-63 on MI355X while another workgroup shared the CU, so no kernel may contain one."""
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("no ROCm llvm-objdump")
    so = os.path.join(os.path.dirname(built), name)
    cos = _device_code_objects(so)
    assert len(cos) >= 7, f"{name}: {len(cos)} gfx950 code objects"   # every kernel source
    total = 0
    for i, co in enumerate(cos):
        p = tmp_path / f"co{i}.o"
        p.write_bytes(co)
        dis = subprocess.run([objdump, "-d", str(p)], capture_output=True, text=True,
                             check=True).stdout
        assert "v_mfma" in dis or "s_endpgm" in dis
        total += len(re.findall(r"\bv_pk_(?:fma|mul|add|mov)_f32\b", dis))
    assert total == 0, f"{name}: {total} packed-FP32 instructions"
