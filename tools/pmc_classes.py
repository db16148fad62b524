#!/usr/bin/env python3
"""Per-dispatch PMC counters of a repeating launch sequence (rocprofv3 --pmc CSVs under <dir>/p*/),
averaged per position in the sequence (the bucketed launch: one ebpf_jit_gen per length class).
Usage: pmc_classes.py <dir> <period>"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, period = sys.argv[1], int(sys.argv[2])
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(
                r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ids = sorted(per)
        for i, did in enumerate(ids):
            for c, v in per[did].items():
                acc[i % period][c].append(v)
    for pos in sorted(acc):
        print("position %d" % pos)
        for c in sorted(acc[pos]):
            v = acc[pos][c]
            print("  %-34s %16.1f" % (c, sum(v) / len(v)))


if __name__ == "__main__":
    main()
