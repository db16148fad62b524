#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 --kernel-trace results database (the rocpd SQLite file
ROCm 7 writes by default).  Prints the per-kernel-name table --stats gives (calls, total, average,
min, max), then the ebpf dispatches split into runs of consecutive launches with the same name
and grid, so that each bench.py line (C4, then every --also config) gets its own average.
Usage: kt_db_summary.py <results.db>"""
import sqlite3
import sys
from collections import OrderedDict


def stats(v):
    v = sorted(v)
    return len(v), sum(v), sum(v) / len(v), v[len(v) // 2], v[0], v[-1]


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, grid_x, workgroup_x, lds_size from kernels "
                     "order by start").fetchall()
    by = OrderedDict()
    for name, s, e, *_ in rows:
        by.setdefault(name, []).append((e - s) / 1e3)
    print("%-48s %6s %12s %10s %10s %10s %10s" % ("kernel", "calls", "total_us", "avg_us",
                                                   "median_us", "min_us", "max_us"))
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        n, tot, avg, med, lo, hi = stats(v)
        print("%-48s %6d %12.1f %10.2f %10.2f %10.2f %10.2f" % (name[:48], n, tot, avg, med, lo, hi))
    print()
    print("ebpf dispatch runs (consecutive launches, same kernel and grid):")
    runs = []
    for name, s, e, gx, wx, lds in rows:
        if "ebpf" not in name:
            continue
        key = (name, gx, wx, lds)
        if runs and runs[-1][0] == key:
            runs[-1][1].append((e - s) / 1e3)
        else:
            runs.append((key, [(e - s) / 1e3]))
    for (name, gx, wx, lds), v in runs:
        if len(v) < 3:
            continue
        n, tot, avg, med, lo, hi = stats(v)
        print("  %-24s grid %9d wg %4d lds %6d  n=%4d avg %9.2f med %9.2f min %9.2f max %9.2f us"
              % (name[:24], gx, wx, lds, n, avg, med, lo, hi))


if __name__ == "__main__":
    main()
