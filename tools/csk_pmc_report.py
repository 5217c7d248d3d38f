"""Summary of tools/gpu_csk_pmc.sh: per (config, M), the GEMM kernel's HBM bytes per dispatch
(FETCH_SIZE x 2 on gfx950 for 16-B streaming reads -- MI355X_MICROARCH.md -- + WRITE_SIZE), L2 hit
rate, clock, MFMA busy, and the kernel / fix-up durations.
    python tools/csk_pmc_report.py gpurun_out/cskpmc_TAG [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

ALG = lambda M: (M * 3136 + 3136 * 3136 + M * 3136) * 4 + 3136 * 4   # A + W read, C written, bias


def counters(d, sub):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(f):
        return out
    for r in csv.DictReader(open(f)):
        out[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    root = sys.argv[1]
    res = []
    for d in sorted(glob.glob(os.path.join(root, "*_*"))):
        cfg, M = os.path.basename(d).split("_")
        M = int(M)
        kt = {}
        f = os.path.join(d, "kt", "run_kernel_stats.csv")
        if os.path.exists(f):
            for r in csv.DictReader(open(f)):
                kt[r["Name"].split("(")[0]] = (float(r["AverageNs"]), int(r["Calls"]))
        fe, wr, tc, sq = (counters(d, s) for s in ("fetch", "write", "tcc", "sq"))
        gemm = [k for k in fe if "gemm_x3" in k or "gemm_p3" in k]
        fix = [k for k in fe if "fixup" in k]
        if not gemm:
            continue
        g = gemm[0]
        mean = lambda x: sum(x) / len(x) if x else None
        fetch = mean(fe[g]["FETCH_SIZE"]) * 1024 * 2          # KB -> B, gfx950 x2
        write = mean(wr[g]["WRITE_SIZE"]) * 1024
        row = {"config": cfg, "M": M, "kernel": g.split("::")[-1][:60],
               "hbm_bytes_per_dispatch": round(fetch + write),
               "fetch_bytes_x2": round(fetch), "write_bytes": round(write),
               "algorithmic_bytes": ALG(M),
               "ratio_to_algorithmic": round((fetch + write) / ALG(M), 2)}
        if fix:
            ff = mean(fe[fix[0]]["FETCH_SIZE"]) * 1024 * 2 + mean(wr[fix[0]]["WRITE_SIZE"]) * 1024
            row["fixup_bytes"] = round(ff)
        h, m = mean(tc[g]["TCC_HIT_sum"]), mean(tc[g]["TCC_MISS_sum"])
        if h is not None and m:
            row["l2_hit"] = round(h / (h + m), 3)
        ns = next((v[0] for k, v in kt.items() if "gemm_x3" in k or "gemm_p3" in k), None)
        fns = next((v[0] for k, v in kt.items() if "fixup" in k), None)
        row["kernel_us"] = round(ns / 1e3, 2) if ns else None
        row["fixup_us"] = round(fns / 1e3, 2) if fns else None
        gui = mean(tc[g]["GRBM_GUI_ACTIVE"])
        if gui and ns:
            row["clk_GHz"] = round(gui / 8 / ns, 3)
            mb = mean(sq[g]["SQ_VALU_MFMA_BUSY_CYCLES"])
            if mb:
                row["mfma_busy"] = round(mb / (gui / 8 * 1024), 3)
        res.append(row)
        print(json.dumps(row))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
