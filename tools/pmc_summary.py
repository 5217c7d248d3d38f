"""Summarise the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu_profile.sh into
profiles/<tag>_pmc_hbm.csv and profiles/pmc.json (what bench.py reports as roofline.traffic).

    python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>

HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024: on gfx950 FETCH_SIZE counts
half of the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section).  The bench's
output_transform call is one az_gemm_f32 = the tile kernel plus, when split-K is used, the
split-K reduce kernel dispatched right after it; both are charged to that call.
"""
import csv
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                         int(r["Grid_Size"])))
    rows.sort()
    return rows


def main(d, tag):
    fetch = load(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    per = collections.defaultdict(lambda: [[], []])
    for i, rows in enumerate((fetch, write)):
        for _, name, kb, _ in rows:
            per[name][i].append(kb)
    out = os.path.join(ROOT, "profiles", f"{tag}_pmc_hbm.csv")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KB_avg", "WRITE_SIZE_KB_avg",
                    "hbm_bytes_corrected (2*FETCH + WRITE)"])
        for name, (fe, wr) in sorted(per.items(), key=lambda kv: -sum(kv[1][0])):
            if not fe or not wr:
                continue
            fa, wa = sum(fe) / len(fe), sum(wr) / len(wr)
            w.writerow([name, len(fe), round(fa, 1), round(wa, 1), int((2 * fa + wa) * 1024)])

    def call_bytes(rows, tile_pred):
        """per az_gemm_f32 call: the tile kernel + the reduce that immediately follows it (+ from
        round 4 the A row-scale launch right before it: the fp16 form, az_gemm.hip)"""
        tile, red, scl = [], [], []
        for i, (_, name, kb, _) in enumerate(rows):
            nxt = rows[i + 1][1] if i + 1 < len(rows) else ""
            prv = rows[i - 1][1] if i > 0 else ""
            # output_transform.0 = the tile kernel followed by its splitk_reduce_kernel (the
            # second GEMM's slabs go to splitk_heads_partial_kernel instead)
            # (the standalone call; the bench step's output_transform.0 hands its slabs to
            # splitk_reduce_split_kernel, which also splits the next GEMM's A: not matched)
            if tile_pred(name) and ("splitk_reduce4_kernel" in nxt or
                                    "splitk_reduce_kernel" in nxt):
                tile.append(kb)
                red.append(rows[i + 1][2])
                scl.append(rows[i - 1][2] if ("row_scale_kernel" in prv or
                                              "h3_split_rows_kernel" in prv) else 0.0)
        n = max(1, len(tile))
        return sum(tile) / n, sum(red) / n, len(tile), sum(scl) / n

    # the forward Linear path of the bench GEMMs (gemm_x3 from r02m on)
    is_fwd_gemm = lambda n: "gemm_f32_glds" in n or "gemm_x3" in n or "gemm_p3" in n
    ft, fr, nf, fs = call_bytes(fetch, is_fwd_gemm)
    wt, wr, _, ws = call_bytes(write, is_fwd_gemm)
    gemm_tile = int((2 * ft + wt) * 1024)
    gemm_red = int((2 * fr + wr) * 1024)
    gemm_scale = int((2 * fs + ws) * 1024)
    # the 512-grid shard launches (grid = V * 8 lanes); the 4096-grid full-config ones excluded
    shard = 512 * 1024 * 8
    agg = [kb for _, n, kb, gs in fetch if "aggregate_small_kernel" in n and gs == shard]
    aggw = [kb for _, n, kb, gs in write if "aggregate_small_kernel" in n and gs == shard]
    B, F = 512, 3136
    res = {
        "round": 1, "tag": tag,
        "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                  f"`python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train` "
                  f"(tools/gpu_profile.sh {tag}); per-kernel averages over all dispatches; "
                  f"bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 (gfx950 FETCH_SIZE reports "
                  f"half of wide reads, MI355X_MICROARCH.md HBM section)",
        "gemm": {"kernel": "az_gemm_f32 output_transform.0 call (%s%s tile kernel + "
                           "splitk_reduce4_kernel)" % (
                               ("h3_split_rows_kernel + " if any("gemm_p3" in r[1] for r in fetch)
                                else "row_scale_kernel + ") if gemm_scale else "",
                               "gemm_p3" if any("gemm_p3" in r[1] for r in fetch) else
                               "gemm_x3" if any("gemm_x3" in r[1] for r in fetch)
                               else "gemm_f32_glds2"),
                 "dispatches": nf,
                 "hbm_bytes_per_launch": gemm_tile + gemm_red + gemm_scale,
                 "gemm_kernel_bytes": gemm_tile, "reduce_kernel_bytes": gemm_red,
                 "row_scale_kernel_bytes": gemm_scale,
                 "algorithmic_bytes": 4 * (B * F + F * F + F + B * F), "tag": tag},
    }
    if agg and aggw:
        V, E = 512 * 1024, 512 * 3968
        res["aggregate"] = {"kernel": "aggregate_small_kernel<8,2,1,NT> (512 32x32 grids, F=64)",
                            "hbm_bytes_per_launch": int((2 * sum(agg) / len(agg)
                                                         + sum(aggw) / len(aggw)) * 1024),
                            "algorithmic_bytes": V * 64 * 4 * 2 + E * 8 + (V + 1) * 4}
    # round 2: the fused eval-mode GNN layer and its source projection (tools/fused_probe.py one:
    # 512 grids, x warm from the previous launch as in the bench's "warm" figure)
    ff, fw = (os.path.join(d, "ffetch", "run_counter_collection.csv"),
              os.path.join(d, "fwrite", "run_counter_collection.csv"))
    if os.path.exists(ff) and os.path.exists(fw):
        fe2, wr2 = load(ff, "FETCH_SIZE"), load(fw, "WRITE_SIZE")
        V, E = 512 * 1024, 512 * 3968
        for key, pred, alg in (
                ("gnn_layer_fused", lambda n: "gnn_layer_fused_kernel" in n,
                 V * 1024 + 4 * E + 4 * (V + 1)),
                ("gnn_source_proj", lambda n: "gemm_tall" in n or "gemm_f32" in n,
                 V * 64 * 4 + 128 * 64 * 4 + V * 128 * 4),
                # round 3 (tools/band_probe.py): the band-mode layer, one launch per layer (x read
                # once, x_out written, the CSR); OT = the last layer with output_transform fused
                ("gnn_layer_band", lambda n: "gnn_layer_band_kernel<0, false>" in n,
                 V * 64 * 4 * 2 + 4 * E + 4 * (V + 1)),
                ("gnn_layer_band_ot", lambda n: "gnn_layer_band_kernel<0, true>" in n,
                 V * 64 * 4 * 2 + 4 * E + 4 * (V + 1))):
            if key == "gnn_source_proj" and tag >= "r03":   # no source projection in band mode
                continue
            a = [kb for _, n, kb, _ in fe2 if pred(n)]
            b = [kb for _, n, kb, _ in wr2 if pred(n)]
            if a and b:
                res[key] = {"kernel": key, "dispatches": len(a),
                            "hbm_bytes_per_launch": int((2 * sum(a) / len(a) + sum(b) / len(b))
                                                        * 1024),
                            "algorithmic_bytes": alg,
                            "tag": tag,
                            "note": "512 32x32 grids, back-to-back launches (x partly "
                                    "Infinity-Cache resident between them)"}
    res["round"] = int(tag[1:3]) if tag[:3] in ("r02", "r03", "r04", "r05", "r06") else res["round"]
    # keep the entries of earlier passes this one did not measure (e.g. the fused-layer probe)
    path = os.path.join(ROOT, "profiles", "pmc.json")
    try:
        old = json.load(open(path))
    except (OSError, ValueError):
        old = {}
    for k, v in old.items():
        if k == "gnn_source_proj" and tag >= "r03":
            continue
        if isinstance(v, dict) and k not in res:
            v.setdefault("tag", old.get("tag"))
            res[k] = v
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
