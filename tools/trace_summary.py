#!/usr/bin/env python3
"""Markdown summary of a rocprofv3 --kernel-trace CSV: per kernel the dispatch count, the median
duration (robust to first-launch outliers that skew run_kernel_stats.csv's average) and the mean
after dropping the first quarter of dispatches.

usage: trace_summary.py <run_kernel_trace.csv> [title line ...] > summary.md"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        by[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for line in sys.argv[2:]:
        print(line)
    print()
    print("| kernel | dispatches | median us | mean (after warm-up quarter) us |")
    print("|---|---|---|---|")
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:12]:
        tail = d[len(d) // 4:] or d
        print(f"| `{name[:120]}` | {len(d)} | {statistics.median(d) / 1e3:.1f} | "
              f"{sum(tail) / len(tail) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
