#!/usr/bin/env python3
"""Device parity of the golden cases (tests/golden/*.npz) for the current build and environment
(EBPF_CC_OFF etc.): prints the failing cases.  Quick bisection aid; tests/ holds the real tests."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pkgload  # noqa: E402

pkgload.load()
import goldens  # noqa: E402
from generic_ebpf_amd import native  # noqa: E402


def main():
    env = native.Env()
    bad = []
    total = 0
    for fn in goldens.all_golden_files():
        for c in goldens.load(fn):
            maps = [native.Map(env, me, vs) for vs, me, _ in c.maps]
            for m, (vs, me, data) in zip(maps, c.maps):
                m.fill(data)
            p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
            data = np.ascontiguousarray(c.data.copy())
            ret, faults, _ = p.run_batch(data, c.count, c.stride, c.offsets)
            total += 1
            if not (np.array_equal(ret, c.expect_r0) and not faults.any()):
                bad.append((c.name, int(np.count_nonzero(ret != c.expect_r0)), int(np.count_nonzero(faults))))
            p.destroy()
            for m in maps:
                m.destroy()
    print("EBPF_CC_OFF=%s: %d/%d bad %s" % (os.environ.get("EBPF_CC_OFF", ""), len(bad), total, bad[:6]), flush=True)


if __name__ == "__main__":
    main()
