"""ctypes binding of libaz_hip.so (the C-ABI declared in include/az_hip.h).

The library is loaded AFTER ``import torch`` so that it binds to the HIP runtime torch
already mapped (both carry the SONAME libamdhip64.so.7): device pointers from torch tensors
and torch's streams are then valid inside the library.  There is no fallback: when the
library is missing or no gfx950 device is visible, every op raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# AZ_TUNING_LIB=1 selects the tuning build (A/B-experiment switches + slower variants; tools/
# and the kernel-variant test only)
LIB_PATH = os.path.join(HERE, "libaz_hip_tuning.so" if os.environ.get("AZ_TUNING_LIB") == "1"
                        else "libaz_hip.so")
# AZ_AB_LIB=<file in azhip/>: an A/B build of the same sources at another revision (tools/
# ab_lib.sh writes libaz_hip_base.so), timed beside the current one in the same GPU session
if os.environ.get("AZ_AB_LIB"):
    LIB_PATH = os.path.join(HERE, os.path.basename(os.environ["AZ_AB_LIB"]))

c_int, c_float, c_double, c_void_p, c_int64, c_size_t = (
    ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t)
c_char_p = ctypes.c_char_p

ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, ACT_DRELU = 0, 1, 2, 3, 4


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("A", c_void_p), ("lda", c_int), ("a_kmajor", c_int),
        ("A2", c_void_p), ("lda2", c_int), ("K0", c_int),
        ("a_rows", c_void_p),
        ("B", c_void_p), ("ldb", c_int), ("b_kmajor", c_int),
        ("b_rows", c_void_p),
        ("bias", c_void_p),
        ("act", c_int),
        ("R", c_void_p), ("ldr", c_int),
        ("G", c_void_p), ("ldg", c_int),
        ("beta", c_float),
        ("C", c_void_p), ("ldc", c_int),
        ("c_rows", c_void_p),
        ("C2", c_void_p), ("ldc2", c_int),
        ("ws", c_void_p), ("ws_bytes", c_size_t),
    ]


class Graph(ctypes.Structure):
    _fields_ = [("V", c_int), ("E", c_int), ("rowptr", c_void_p), ("col", c_void_p),
                ("edge_dst", c_void_p), ("D", c_int), ("dst_rows", c_void_p),
                ("src_rowptr", c_void_p), ("src_edges", c_void_p), ("dst_index", c_void_p),
                ("max_deg", c_int), ("band", c_int)]


LAYER_FIELDS = ("att_w1", "att_b1", "att_w2", "att_b2", "upd_w1", "upd_b1", "upd_w2", "upd_b2",
                "gate_w", "gate_b")


class LayerW(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in LAYER_FIELDS]


class LayerGrads(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in LAYER_FIELDS]


class C4Eval(ctypes.Structure):
    """az_c4_eval (include/az_hip.h)."""
    _fields_ = [("conv1_w", c_void_p), ("conv1_b", c_void_p), ("conv2_w", c_void_p),
                ("conv2_b", c_void_p), ("fc_policy_w", c_void_p), ("fc_policy_b", c_void_p),
                ("fc_value_w", c_void_p), ("fc_value_b", c_void_p), ("A", c_int),
                ("ot0_w", c_void_p), ("ot0_b", c_void_p), ("ot2_w", c_void_p),
                ("ot2_b", c_void_p), ("max_B", c_int), ("feat", c_void_p), ("hidden", c_void_p),
                ("y", c_void_p), ("logp", c_void_p), ("glogp", c_void_p), ("ws", c_void_p),
                ("ws_bytes", c_size_t), ("sync", c_void_p), ("err", c_void_p)]


# name -> (restype, argtypes); every symbol here must be declared in include/az_hip.h
SIGNATURES = {
    "az_abi_version": (c_int, []),
    "az_last_error": (c_char_p, []),
    "az_check_device": (c_int, []),
    "az_host_alloc": (c_void_p, [c_size_t]),
    "az_host_free": (c_int, [c_void_p]),
    "az_gemm_f32": (c_int, [ctypes.POINTER(GemmDesc), c_void_p]),
    "az_c4_trunk_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    "az_conv3x3_relu_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                    c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "az_heads_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "az_c4_eval_fwd": (c_int, [ctypes.POINTER(C4Eval), c_void_p, c_int, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    "az_c4_trunk_heads_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                      c_void_p]),
    "az_heads_fwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                             c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_size_t, c_void_p]),
    "az_gnn_attn_score_fwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "az_gnn_aggregate_fwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int, c_void_p,
                                     c_void_p, c_int, c_void_p]),
    "az_gnn_layer_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "az_gnn_layer_infer_ws_bytes": (c_size_t, [ctypes.POINTER(Graph), c_int, c_int]),
    "az_gnn_layer_infer": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int,
                                   ctypes.POINTER(LayerW), c_void_p, c_void_p, c_size_t,
                                   c_void_p]),
    "az_gnn_layer_ot_infer_ws_bytes": (c_size_t, [ctypes.POINTER(Graph), c_int, c_int]),
    "az_gnn_layer_ot_infer": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int,
                                      ctypes.POINTER(LayerW), c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "az_gnn_source_proj_fwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int,
                                       ctypes.POINTER(LayerW), c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    "az_gnn_layer_fused_fwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_void_p, c_int, c_int,
                                       ctypes.POINTER(LayerW), c_void_p, c_void_p]),
    "az_gnn_layer_fwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int,
                                 ctypes.POINTER(LayerW), c_void_p, c_void_p, c_size_t, c_void_p]),
    "az_gnn_node_update_ws_bytes": (c_size_t, [c_int, c_int]),
    "az_gnn_node_update_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    "az_gnn_node_update_bwd_ws_bytes": (c_size_t, [c_int, c_int]),
    "az_gnn_node_update_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    "az_mlp2_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "az_transform_heads_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "az_linear_heads_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "az_transform_heads_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "az_heads_loss_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "az_heads_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                             c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_int, c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "az_colsum_ws_bytes": (c_size_t, [c_int, c_int]),
    "az_colsum": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_float, c_void_p, c_size_t,
                          c_void_p]),
    "az_dropout_mask": (c_int, [c_void_p, c_int64, c_double, ctypes.c_uint64, c_void_p]),
    "az_mask_scale": (c_int, [c_void_p, c_void_p, c_float, c_int64, c_void_p, c_void_p]),
    "az_nchw_drelu_to_pm": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_int,
                                    c_void_p, c_void_p]),
    "az_im2col3x3": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                             c_void_p]),
    "az_col2im3x3_drelu": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                   c_void_p, c_void_p]),
    "az_gnn_layer_bwd_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "az_gnn_layer_bwd": (c_int, [ctypes.POINTER(Graph), c_void_p, c_int, c_int,
                                 ctypes.POINTER(LayerW), c_void_p, c_void_p, c_void_p,
                                 ctypes.POINTER(LayerGrads), c_void_p, c_size_t, c_void_p]),
    "az_mlp2_bwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_size_t, c_void_p]),
    "az_adam_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_double, c_double,
                            c_double, c_double, c_int, c_void_p]),
    "az_adam_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_double, c_double,
                             c_double, c_double, c_int, c_void_p]),
    "az_weights_changed": (c_int, []),
    "az_weights_register": (c_int, [c_void_p, c_size_t]),
    "az_weights_unregister": (c_int, [c_void_p]),
    "az_gemm_form": (c_int, [c_int, c_int, c_int, c_size_t]),
}

_lib = None


def load(path=LIB_PATH):
    """Load and type the library (no GPU needed; the CPU tests use this to check exports)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (map torch's HIP runtime first)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -m azhip.build` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.az_abi_version() != 2:
        raise RuntimeError("libaz_hip.so ABI mismatch")
    _lib = L
    return L


_device_checked = False


def lib():
    """The library, after checking that torch sees a gfx950 device."""
    global _device_checked
    L = load()
    if not _device_checked:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("azhip: no HIP device visible; this framework runs its compute "
                               "only on MI355X (gfx950) and has no CPU fallback")
        torch.cuda.init()
        check(L.az_check_device(), "az_check_device")
        _device_checked = True
    return L


def check(rc, what):
    if rc != 0:
        msg = load().az_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")
