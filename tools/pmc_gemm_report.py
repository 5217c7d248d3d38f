"""Per-kernel averages of the counter passes written by tools/gpu_gemm_pmc.sh."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for cdir in sorted(glob.glob(os.path.join(d, "c*_p1"))):
    c = os.path.basename(cdir)[:-3]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("p1", "p2"):
        f = os.path.join(d, f"{c}_{p}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if "gemm" not in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0][-60:]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kt = {}
    f = os.path.join(d, f"{c}_kt", "run_kernel_stats.csv")
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            kt[r["Name"].split("(")[0][-60:]] = float(r["AverageNs"])
    for k, cs in vals.items():
        a = {n: sum(v) / len(v) for n, v in cs.items()}
        ns = kt.get(k)
        line = f"{c} {k} ns={ns}"
        if ns and "GRBM_GUI_ACTIVE" in a:
            line += f" clk_GHz={a['GRBM_GUI_ACTIVE'] / 8 / ns:.3f}"
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in a:
                    line += f" {n[3:]}={a[n] / wc:.3f}"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
            line += (f" mfma_busy/(gui*1024/8)="
                     f"{a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
        if "SQ_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
            line += f" sq_busy/gui={a['SQ_BUSY_CYCLES'] / a['GRBM_GUI_ACTIVE']:.3f}"
        if "TCC_HIT_sum" in a:
            line += f" L2hit={a['TCC_HIT_sum'] / max(1, a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.3f}"
        line += " " + " ".join(f"{n}={v:.4g}" for n, v in sorted(a.items()))
        print(line)
