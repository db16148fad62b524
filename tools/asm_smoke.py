#!/usr/bin/env python3
"""Small first-contact run of the assembly interpreter: golden vectors through variant 0 and
variant 1, mismatches printed per case (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

pkgload.load()
import goldens  # noqa: E402
from helpers import device_run  # noqa: E402
from generic_ebpf_amd import native  # noqa: E402

env = native.Env()
names = sys.argv[1:] or ["kat", "workloads", "rand"]
for g in names:
    for c in goldens.load(os.path.join(goldens.GOLDEN_DIR, g + ".npz")):
        for variant in [int(x) for x in os.environ.get("VARIANTS", "0").split(",")]:
            try:
                ret, faults, after = device_run(native, env, c, variant)
            except Exception as e:  # noqa: BLE001
                print("ERR", c.name, variant, e, flush=True)
                continue
            bad = np.nonzero(ret != c.expect_r0)[0]
            fl = np.unique(faults)
            ok = len(bad) == 0 and not faults.any() and np.array_equal(after, c.expect_data)
            if not ok:
                print("FAIL %s v%d: %d/%d mismatches first=%s got=%s want=%s faults=%s data_eq=%s" % (
                    c.name, variant, len(bad), c.count, bad[:3], ret[bad[:3]], c.expect_r0[bad[:3]],
                    fl, np.array_equal(after, c.expect_data)), flush=True)
            else:
                print("ok   %s v%d" % (c.name, variant), flush=True)
print("env destroy", env.destroy())
