#!/usr/bin/env python3
"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace CSV, grouped by kernel name
and by position within a repeating launch sequence (e.g. the bucketed C5 launch: bucket_count,
bucket_scatter, then one ebpf_jit_gen per length class).  Usage: kt_summary.py <dir> [period]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    f = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ebpf = [r for r in rows if "ebpf" in r["Kernel_Name"] or "bucket" in r["Kernel_Name"]]
    by = defaultdict(list)
    for r in ebpf:
        by[r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in by.items():
        v = sorted(v)
        print("%-40s n=%4d median %9.2f us  min %9.2f" % (k, len(v), v[len(v) // 2], v[0]))
    if len(sys.argv) > 2:
        p = int(sys.argv[2])
        seqs = defaultdict(list)
        names = {}
        for i, r in enumerate(ebpf):
            seqs[i % p].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            names[i % p] = r["Kernel_Name"][:30]
        for j in range(p):
            v = sorted(seqs[j])
            print("position %d %-30s median %9.2f us" % (j, names[j], v[len(v) // 2]))
        # gaps: from the first dispatch's start to the last's end per sequence
        spans = []
        for s in range(0, len(ebpf) - p + 1, p):
            spans.append((int(ebpf[s + p - 1]["End_Timestamp"]) - int(ebpf[s]["Start_Timestamp"])) / 1e3)
        spans.sort()
        print("sequence span median %.2f us" % spans[len(spans) // 2])


if __name__ == "__main__":
    main()
