"""Probe: where a gemm_p3 block's time goes.  libaz_hip_exp.so = az_gemm.hip built with
-DAZ_TUNING -DAZ_P3_STAMPS (linked with the tuning objects): lane 0 of every wave stamps
s_memrealtime (100 MHz) at the body's start, after the prologue's DMA issue, before each stage's
wait and after its barrier, at the loop's end and after the epilogue.  Runs ops.linear at M
(the product dispatch: split-K gemm_p3 at M = 512) and prints per-phase medians over blocks /
waves and the spread of block start and end times.
    AZ_AB_LIB=libaz_hip_exp.so AZ_TUNING_LIB=1 python tools/p3_stamp_probe.py [M]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def main():
    from azhip import ops, _lib
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    L = _lib.load()
    N = K = 3136
    w = (torch.rand((N, K), device="cuda") * 2 - 1) / K ** 0.5
    _lib.check(L.az_weights_register(w.data_ptr(), w.numel() * 4), "register")
    b = torch.rand((N,), device="cuda")
    x = torch.rand((M, K), device="cuda") * 2 - 1
    y = torch.empty((M, N), device="cuda")
    for _ in range(50):
        ops.linear(x, w, b, act=1, out=y)
    blocks, NW, SL = 2048, 8, 72
    buf = torch.zeros(blocks * NW * SL, dtype=torch.int64, device="cuda")
    L.az_debug_p3_stamps.argtypes = [ctypes.c_void_p]
    reps = []
    for rep in range(5):
        buf.zero_()
        assert L.az_debug_p3_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
        ops.linear(x, w, b, act=1, out=y)
        torch.cuda.synchronize()
        assert L.az_debug_p3_stamps(ctypes.c_void_p(0)) == 0
        for _ in range(5):
            ops.linear(x, w, b, act=1, out=y)
        torch.cuda.synchronize()
        reps.append(buf.cpu().numpy().reshape(blocks, NW, SL).copy())
    for a in reps:
        used = a[:, 0, 0] > 0
        s = a[used].astype(np.float64)
        nb = int(used.sum())
        t0 = s[:, :, 0].min()
        ns = lambda v: (v) * 10.0        # 100 MHz ticks -> ns
        nk = int(((s[0, 0, 2:66:2] > 0)).sum())
        start = ns(s[:, :, 0] - t0)
        end = ns(s[:, :, 67] - t0)
        prol = ns(s[:, :, 2] - s[:, :, 0])                      # body start -> first wait
        first = ns(s[:, :, 3] - s[:, :, 2])                     # stage 0's wait + barrier
        waits = np.stack([ns(s[:, :, 3 + 2 * k] - s[:, :, 2 + 2 * k]) for k in range(1, nk)], -1)
        bodies = np.stack([ns(s[:, :, 2 + 2 * (k + 1)] - s[:, :, 3 + 2 * k]) for k in range(nk - 1)], -1)
        last = ns(s[:, :, 66] - s[:, :, 3 + 2 * (nk - 1)])
        epi = ns(s[:, :, 67] - s[:, :, 66])
        cyc = (s[:, :, 69] - s[:, :, 68]) / np.maximum(1, (s[:, :, 67] - s[:, :, 0]) * 10.0)
        med = lambda v: round(float(np.median(v)), 1)
        print(json.dumps({
            "M": M, "blocks": nb, "stages": nk,
            "kernel_span_ns": med(end.max()) , "block_start_ns": {"min": med(start.min()), "median": med(start), "max": med(start.max())},
            "block_end_ns": {"min": med(end.min()), "median": med(end), "max": med(end.max())},
            "prologue_ns": med(prol), "stage0_wait_ns": med(first),
            "stage_body_ns": med(bodies), "stage_body_ns_by_k": [med(bodies[:, :, k]) for k in range(nk - 1)],
            "stage_wait_ns": med(waits), "stage_wait_ns_by_k": [med(waits[:, :, k]) for k in range(nk - 1)],
            "last_stage_ns": med(last), "epilogue_ns": med(epi),
            "clock_GHz": med(cyc), "waves_0_3_vs_4_7_body_ns": [med(bodies[:, :4]), med(bodies[:, 4:])]}))


if __name__ == "__main__":
    main()
