"""Summarise bench.py JSON lines (one per file) of an A/B directory: kernel ms, frac, step ms."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        r = d.get("roofline", {})
        print("%-26s kernel_ms %.4f frac %.3f ms_per_step %.4f verified %s" % (
            f.split("/")[-1], r.get("kernel_ms", 0), r.get("frac", 0), d["ms_per_step"], d.get("verified")))
    except Exception as e:  # noqa: BLE001 (a failed run leaves an empty file)
        print(f, "unreadable:", e)
