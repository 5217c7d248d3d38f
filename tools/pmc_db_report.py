"""Per-kernel averages of a rocprofv3 --pmc run's counters, read from its sqlite output
(`-o run` -> <dir>/run_results.db): each dispatch's counter summed over its instances, then
averaged over the dispatches of each kernel.  Usage: pmc_db_report.py DB [name-substring ...]"""
import sqlite3
import sys


def report(db, pats=()):
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, avg(v), count(*) from (select dispatch_id, kernel_name,"
         " counter_name, sum(value) v from counters_collection group by dispatch_id, counter_name)"
         " group by kernel_name, counter_name order by kernel_name, counter_name")
    out = {}
    for name, ctr, v, n in c.execute(q):
        if pats and not any(p in name for p in pats):
            continue
        out.setdefault(name, {"dispatches": n})[ctr] = v
    return out


if __name__ == "__main__":
    for name, d in report(sys.argv[1], sys.argv[2:]).items():
        print(name[:110])
        for k, v in d.items():
            print(f"    {k:28s} {v:.4g}")
        if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_INSTS_LDS"):
            print(f"    conflict cycles / LDS instruction {d['SQ_LDS_BANK_CONFLICT'] / d['SQ_INSTS_LDS']:.3f}")
