"""Per-grid-size HBM bytes of aggregate_small_kernel from tools/gpu_agg_pmc.sh:
bytes = (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024 (MI355X_MICROARCH.md HBM section), per dispatch,
grouped by grid size (512-grid shard vs all 4096 grids), vs the algorithmic bytes."""
import collections
import csv
import sys

d = sys.argv[1]


def load(sub, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter and "aggregate_small_kernel" in r["Kernel_Name"]:
            out[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return out


f, w = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
for grid in sorted(f):
    graphs = 512 if grid < 10_000_000 else 4096
    V, E = graphs * 1024, graphs * 3968
    alg = V * 64 * 4 * 2 + E * 8 + (V + 1) * 4
    fb = sum(f[grid]) / len(f[grid])
    wb = sum(w.get(grid, [0])) / max(1, len(w.get(grid, [])))
    hbm = (2 * fb + wb) * 1024
    print(f"grid_size={grid} graphs~{graphs} dispatches={len(f[grid])} FETCH_KB={fb:.0f} "
          f"WRITE_KB={wb:.0f} hbm_bytes={hbm:.4g} algorithmic={alg:.4g} ratio={hbm / alg:.3f}")
