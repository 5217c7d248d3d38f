"""Build libaz_hip.so in-tree with hipcc for gfx950 (no torch involved in the build).

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
OBJ = os.path.join(CSRC, "build")
SOURCES = ["az_runtime.hip", "az_gemm.hip", "az_trunk.hip", "az_gnn.hip", "az_optim.hip",
           "az_backward.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall",
         "-Wno-unused-function", "-fno-gpu-rdc"]


def hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c


def _compile(src):
    obj = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    s = os.path.join(CSRC, src)
    deps = [s, os.path.join(CSRC, "az_common.h"),
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


if __name__ == "__main__":
    build()
    sys.exit(0)
