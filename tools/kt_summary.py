"""Summarise a rocprofv3 --kernel-trace --stats CSV: total, share, calls and average per kernel.
    python tools/kt_summary.py <..._kernel_stats.csv> [top]"""
import csv
import sys


def main():
    rows = list(csv.reader(open(sys.argv[1])))[1:]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 18
    tot = sum(float(r[2]) for r in rows) / 1e6
    print(f"total {tot:.1f} ms of kernel time")
    for r in rows[:top]:
        ms = float(r[2]) / 1e6
        print(f"{ms:9.1f} ms {ms / tot * 100:5.1f}%  {r[1]:>6} x {float(r[3]) / 1e3:7.1f} us  {r[0][:96]}")


if __name__ == "__main__":
    main()
