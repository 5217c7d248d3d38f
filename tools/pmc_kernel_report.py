"""Per-kernel averages of the counter passes of tools/gpu_kernel_pmc.sh:
    python tools/pmc_kernel_report.py gpurun_out/kpmc_TAG [kernel-substring]"""
import collections
import csv
import os
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2", "p3"):
    f = os.path.join(d, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        if want not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0][-70:]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
kt = {}
f = os.path.join(d, "kt", "run_kernel_stats.csv")
if os.path.exists(f):
    for r in csv.DictReader(open(f)):
        kt[r["Name"].split("(")[0][-70:]] = float(r["AverageNs"])
for k, cs in vals.items():
    a = {n: sum(v) / len(v) for n, v in cs.items()}
    ns = kt.get(k)
    out = [f"{k} ns={ns}"]
    wc = a.get("SQ_WAVE_CYCLES")
    if ns and "GRBM_GUI_ACTIVE" in a:
        gui = a["GRBM_GUI_ACTIVE"]
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; the quotient reads high for dispatches shorter
        # than ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back) and is only a clock below ~2.5 GHz
        clk = gui / 8 / ns
        out.append(f"clk_GHz={clk:.3f}" if ns >= 3e5 and clk < 2.6 else
                   f"clk_GHz=n/a(dispatch {ns / 1e3:.0f} us: GUI_ACTIVE/8/ns = {clk:.2f})")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            out.append(f"mfma_busy={a['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * 1024):.3f}")
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if n in a:
                out.append(f"{n[3:]}={a[n] / wc:.3f}")
    if "TCC_HIT_sum" in a:
        out.append(f"L2hit={a['TCC_HIT_sum'] / max(1, a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.3f}")
    out += [f"{n}={v:.4g}" for n, v in sorted(a.items())]
    print(" ".join(out))
