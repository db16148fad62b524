#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-dispatch averages of each counter for the interpreter
kernel, HBM traffic per launch with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md,
HBM section: FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read; FETCH_SIZE /
WRITE_SIZE are in KiB).  Writes profiles/<round>/pmc_<cfg>.json.  (bench.py measures its own
roofline.traffic with two rocprofv3 --pmc child passes; this summarises wider counter sets.)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                if "ebpf_interp" not in kn and "ebpf_jit" not in kn:
                    continue
                vals[(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), xs in vals.items():
        per[name].append(sum(xs))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    T, rnd = sys.argv[1], sys.argv[2]
    cfgs = sys.argv[3:]
    cfgs = [c for c in cfgs if not c.startswith("--")]
    for cfg in cfgs:
        c = {}
        bench = None
        for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", T, "pmc_%s_*" % cfg))):
            c.update(load(d))
            try:
                bench = json.load(open(os.path.join(d, "bench.json")))
            except Exception:  # noqa: BLE001
                pass
        out = {"config": cfg, "counters_per_dispatch": c}
        note = ("FETCH_SIZE x2 (gfx950 16-B/lane streaming-read correction); WRITE_SIZE as "
                "reported (8-B/lane stores: calibrate against c0, whose writes are exactly "
                "8 B per packet)")
        if "FETCH_SIZE" in c:
            out["fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
            if cfg == "c4h" and bench:
                # only the packet DMA is a 16-B/lane streaming read: its known bytes get the
                # correction, the random table probes are taken as reported (doubling them too
                # would put the launch above the chip's read bandwidth)
                pk = bench["config"]["packets_per_gpu"] * 64
                out["fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 + pk / 2
                note = ("FETCH_SIZE as reported + half the packet bytes (the 16-B/lane streaming "
                        "packet DMA is undercounted by half on gfx950; the random table probes "
                        "are not corrected); WRITE_SIZE as reported")
        if "WRITE_SIZE" in c:
            out["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            out["hbm_bytes_per_launch"] = out["fetch_bytes_corrected"] + out["write_bytes"]
        if bench:
            out["algorithmic_bytes_per_launch"] = bench["roofline"]["algorithmic_bytes_per_launch"]
            out["packets_per_launch"] = bench["config"]["packets_per_gpu"]
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    out[k + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
        out["note"] = note
        os.makedirs(os.path.join(ROOT, "profiles", rnd), exist_ok=True)
        with open(os.path.join(ROOT, "profiles", rnd, "pmc_%s.json" % cfg), "w") as f:
            json.dump(out, f, indent=1)
        print(cfg, json.dumps({k: v for k, v in out.items() if k != "counters_per_dispatch"}))
        print("  ", {k: round(v) for k, v in c.items()})


if __name__ == "__main__":
    main()
