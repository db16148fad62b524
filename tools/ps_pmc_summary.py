"""Per-dispatch counters of tools/ps_pmc.sh: for each mode and pass, the counters of the last
step's compiled-kernel dispatches (path-sorted: classifying run, then main run), per 64-packet
group of the 4M-packet C5 batch where that reads better."""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ps_pmc"
GROUPS = (1 << 22) / 64
for mode in ("on", "off"):
    disp = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(ROOT, mode + "_*", "*counter_collection.csv"))):
        p = os.path.basename(os.path.dirname(f))
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        byd = defaultdict(lambda: defaultdict(float))
        for r in rows:
            byd[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        ids = sorted(byd)
        last = ids[-2:] if mode == "on" else ids[-1:]
        for k, i in enumerate(last):
            disp[k].update(byd[i])
    for k in sorted(disp):
        c = disp[k]
        name = ("classify" if k == 0 else "main") if mode == "on" else "plain"
        print("%-4s %-8s " % (mode, name) + " ".join(
            "%s=%.1f" % (n, v / GROUPS) if n.startswith("SQ_INSTS") else "%s=%.3g" % (n, v)
            for n, v in sorted(c.items())))
