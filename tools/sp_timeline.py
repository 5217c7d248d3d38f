"""GPU timeline of a traced self-play leg (tools/gpu_sp_trace.sh): busy fraction of the GPU over
the leg (union of kernel and copy intervals), per-batch GPU span, and the gaps between batches.

    python tools/sp_timeline.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


def main(d):
    ks = load(d, "*kernel_trace.csv")
    cs = load(d, "*memory_copy_trace.csv")
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "")) for r in ks]
    iv += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", ""), "") for r in cs]
    iv.sort()
    # the self-play leg: the longest run of trunk launches (c4_trunk*) -- from the first trunk
    # kernel after the warm-up to the last
    trunk = [x for x in iv if "c4_trunk" in x[2]]
    if not trunk:
        print("no trunk kernels")
        return
    # split trunk launches into clusters separated by > 0.5 s: the leg is the largest cluster
    clusters, cur = [], [trunk[0]]
    for a, b in zip(trunk, trunk[1:]):
        if b[0] - a[1] > 5e8:
            clusters.append(cur)
            cur = []
        cur.append(b)
    clusters.append(cur)
    leg = max(clusters, key=lambda c: c[-1][1] - c[0][0])   # the longest span
    t0, t1 = leg[0][0], leg[-1][1]
    sel = [x for x in iv if x[0] >= t0 and x[1] <= t1 + 5e6]
    busy, end = 0, t0
    for a, b, _, _ in sel:
        if b <= end:
            continue
        busy += b - max(a, end)
        end = b
    wall = end - t0
    print(f"leg: {len(leg)} batches, wall {wall/1e9:.3f} s, GPU busy (union) {busy/1e9:.3f} s = {busy/wall:.3f}")
    tot = {}
    for a, b, n, _ in sel:
        k = n.split("(")[0][:60]
        tot[k] = tot.get(k, 0) + (b - a)
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
        print(f"  {k:60s} {v/1e9:7.3f} s")
    # gaps: idle intervals between consecutive busy spans, histogram
    gaps, end = [], sel[0][1]
    for a, b, _, _ in sel[1:]:
        if a > end:
            gaps.append(a - end)
        end = max(end, b)
    gaps.sort()
    if gaps:
        import statistics
        print(f"idle gaps: {len(gaps)}, total {sum(gaps)/1e9:.3f} s, median {statistics.median(gaps)/1e3:.1f} us, "
              f"p90 {gaps[int(0.9*len(gaps))]/1e3:.1f} us, > 100 us: {sum(g for g in gaps if g > 1e5)/1e9:.3f} s")


if __name__ == "__main__":
    main(sys.argv[1])
