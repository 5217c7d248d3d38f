"""Build the in-tree libraries (no torch involved in any build):

    libaz_hip.so          hipcc --offload-arch=gfx950   the device kernels + C-ABI (include/az_hip.h)
    libaz_hip_tuning.so   the same with -DAZ_TUNING: the A/B-experiment switches and the measured-
                          slower kernel variants (tools/ and tests/test_gpu_kernel_variants.py load
                          it with AZ_TUNING_LIB=1; the product library has neither)
    libaz_mcts.so         g++ -fopenmp                  the native MCTS engine (include/az_mcts.h)

    python -m azhip.build [--force]     # from alphazero-gnn_amd/

force=True recompiles every object from source (the driver's build() does); BUILD_INFO.json
beside the libraries records the compiler, flags and a hash of every source.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(HERE, "libaz_hip.so")
TUNING_OUT = os.path.join(HERE, "libaz_hip_tuning.so")
INFO = os.path.join(HERE, "BUILD_INFO.json")
HOST_OUT = os.path.join(HERE, "libaz_mcts.so")
HOST_SOURCES = ["az_mcts.cpp"]
# -ffp-contract=off: no FMA contraction, so the float64/float32 search arithmetic rounds
# exactly like the reference's NumPy operations.
HOST_FLAGS = ["-O3", "-fPIC", "-shared", "-std=c++17", "-fopenmp", "-ffp-contract=off",
              "-Wall", "-Wl,-z,defs"]
OBJ = os.path.join(CSRC, "build")
SOURCES = ["az_runtime.hip", "az_gemm.hip", "az_trunk.hip", "az_gnn.hip", "az_gnn_fused.hip",
           "az_gnn_band.hip", "az_optim.hip", "az_backward.hip"]
# No packed-FP32 VALU code (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): on MI355X a packed op
# gave wrong low-element results in lanes 48-63 when another workgroup shared the CU (round 6:
# tools/trunk_selfcheck_probe.py, profiles/r06/trunk_packed_fp32/).  The feature is
# a device target feature; the host compile ignores it with a one-line note.
# tests/test_lib_abi.py::test_device_code_has_no_packed_fp32 disassembles both libraries.
NO_PK_F32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall",
         "-Wno-unused-function", "-fno-gpu-rdc"] + NO_PK_F32


def hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c


def _flags_current(odir):
    """True when the objects in odir were compiled with today's FLAGS (a flag change rebuilds)."""
    stamp = os.path.join(odir, "FLAGS")
    return os.path.exists(stamp) and open(stamp).read() == " ".join(FLAGS)


def _stamp_flags(odir):
    with open(os.path.join(odir, "FLAGS"), "w") as f:
        f.write(" ".join(FLAGS))


def _compile(src, force=False, tuning=False):
    odir = os.path.join(OBJ, "tuning") if tuning else OBJ
    obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
    s = os.path.join(CSRC, src)
    deps = [s, os.path.join(os.path.dirname(PKG), "include", "az_hip.h")] + \
        [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if not force and os.path.exists(obj) and _flags_current(odir) and \
            all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc()] + FLAGS + (["-DAZ_TUNING"] if tuning else []) + ["-c", s, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def _link(objs, out, force):
    if not force and os.path.exists(out) and \
            all(os.path.getmtime(out) >= os.path.getmtime(o) for o in objs):
        return False
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o", out] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return True


def _build_info():
    import hashlib
    import json
    import time
    ver = subprocess.run([hipcc(), "--version"], capture_output=True, text=True).stdout
    srcs = {}
    for f in sorted(os.listdir(CSRC)):
        p = os.path.join(CSRC, f)
        if os.path.isfile(p):
            srcs[f] = hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]
    hdr = os.path.join(os.path.dirname(PKG), "include")
    for f in sorted(os.listdir(hdr)):
        srcs["include/" + f] = hashlib.sha256(open(os.path.join(hdr, f), "rb").read()).hexdigest()[:16]
    info = {"built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
            "hipcc": [l for l in ver.splitlines() if l.strip()][:2], "flags": FLAGS,
            "host_flags": HOST_FLAGS, "sources_sha256_16": srcs}
    with open(INFO, "w") as f:
        json.dump(info, f, indent=1)


def build(verbose=True, force=False, tuning=True):
    """Compile libaz_hip.so (and libaz_hip_tuning.so unless tuning=False) for gfx950."""
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.join(OBJ, "tuning"), exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    jobs = [(s, False) for s in srcs] + ([(s, True) for s in srcs] if tuning else [])
    with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        objs = list(ex.map(lambda j: _compile(j[0], force, j[1]), jobs))
    _stamp_flags(OBJ)
    if tuning:
        _stamp_flags(os.path.join(OBJ, "tuning"))
    changed = _link(objs[:len(srcs)], OUT, force)
    if tuning:
        changed |= _link(objs[len(srcs):], TUNING_OUT, force)
    if changed or force or not os.path.exists(INFO):
        _build_info()
    if verbose and changed:
        print(f"built {OUT}" + (f" and {os.path.basename(TUNING_OUT)}" if tuning else ""))
    return OUT


def build_host(verbose=True, force=False):
    srcs = [os.path.join(CSRC, f) for f in HOST_SOURCES]
    deps = srcs + [os.path.join(os.path.dirname(PKG), "include", "az_mcts.h")]
    if not force and os.path.exists(HOST_OUT) and \
            all(os.path.getmtime(HOST_OUT) >= os.path.getmtime(d) for d in deps):
        return HOST_OUT
    cmd = ["g++"] + HOST_FLAGS + srcs + ["-o", HOST_OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed for libaz_mcts.so:\n{r.stderr}")
    if verbose:
        print(f"built {HOST_OUT}")
    return HOST_OUT


if __name__ == "__main__":
    f = "--force" in sys.argv
    build_host(force=f)
    build(force=f)
    sys.exit(0)
