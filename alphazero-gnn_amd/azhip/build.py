"""Build the two in-tree libraries (no torch involved in either build):

    libaz_hip.so   hipcc --offload-arch=gfx950   the device kernels + C-ABI (include/az_hip.h)
    libaz_mcts.so  g++ -fopenmp                  the native MCTS engine (include/az_mcts.h)

    python -m azhip.build          # from alphazero-gnn_amd/
"""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(HERE, "libaz_hip.so")
HOST_OUT = os.path.join(HERE, "libaz_mcts.so")
HOST_SOURCES = ["az_mcts.cpp"]
# -ffp-contract=off: no FMA contraction, so the float64/float32 search arithmetic rounds
# exactly like the reference's NumPy operations.
HOST_FLAGS = ["-O3", "-fPIC", "-shared", "-std=c++17", "-fopenmp", "-ffp-contract=off",
              "-Wall", "-Wl,-z,defs"]
OBJ = os.path.join(CSRC, "build")
SOURCES = ["az_runtime.hip", "az_gemm.hip", "az_trunk.hip", "az_gnn.hip", "az_gnn_fused.hip",
           "az_optim.hip", "az_backward.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall",
         "-Wno-unused-function", "-fno-gpu-rdc"]


def hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c


def _compile(src):
    obj = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    s = os.path.join(CSRC, src)
    deps = [s, os.path.join(CSRC, "az_common.h"), os.path.join(CSRC, "az_heads.h"),
            os.path.join(os.path.dirname(PKG), "include", "az_hip.h")]
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc()] + FLAGS + ["-c", s, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(o) for o in objs):
        return OUT
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o", OUT] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {OUT}")
    return OUT


def build_host(verbose=True):
    srcs = [os.path.join(CSRC, f) for f in HOST_SOURCES]
    deps = srcs + [os.path.join(os.path.dirname(PKG), "include", "az_mcts.h")]
    if os.path.exists(HOST_OUT) and all(os.path.getmtime(HOST_OUT) >= os.path.getmtime(d)
                                        for d in deps):
        return HOST_OUT
    cmd = ["g++"] + HOST_FLAGS + srcs + ["-o", HOST_OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed for libaz_mcts.so:\n{r.stderr}")
    if verbose:
        print(f"built {HOST_OUT}")
    return HOST_OUT


if __name__ == "__main__":
    build_host()
    build()
    sys.exit(0)
