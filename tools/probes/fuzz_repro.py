"""Reproduce one reference-mode fuzz case (tools/fuzz_gpu.py case()) on the device, several times,
and print how the device differs from the oracle: which packets, their results, fault codes,
packet bytes and maps.  Usage: fuzz_repro.py SEED K LAYOUT VARIANT [REPEATS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fuzz_gpu  # noqa: E402
from fuzz_gpu import native  # noqa: E402


def main():
    seed, k, layout, variant = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    c = fuzz_gpu.case(k, seed, layout)
    print("program: %d slots, %d packets, maps %s" % (len(c.code) // 8, c.count,
                                                      [(m[0], m[1]) for m in c.maps]))
    want, wf, wdata, wmaps = fuzz_gpu.oracle(c)
    env = native.Env()
    for r in range(reps):
        got, gf, gdata, gmaps = fuzz_gpu.device(env, c, variant, extents=bool(k & 2))
        bad = np.nonzero((want != got) | (wf != gf))[0]
        print("run %d: %d packets differ (results/faults), data equal %s, maps equal %s" % (
            r, len(bad), np.array_equal(wdata, gdata), wmaps == gmaps))
        for i in bad[:8]:
            print("  packet %d: want %#x fault %d, got %#x fault %d" % (i, want[i], wf[i], got[i], gf[i]))
        if wmaps != gmaps:
            for mi, (a, b) in enumerate(zip(wmaps, gmaps)):
                if a != b:
                    ab, bb = np.frombuffer(a, np.uint8), np.frombuffer(b, np.uint8)
                    d = np.nonzero(ab != bb)[0]
                    print("  map %d: %d bytes differ, first at %s" % (mi, len(d), d[:16]))
        if not np.array_equal(wdata, gdata):
            d = np.nonzero(wdata != gdata)[0]
            print("  packet bytes: %d differ, first at %s" % (len(d), d[:16]))
    code = np.frombuffer(c.code, dtype=np.uint8).reshape(-1, 8)
    np.save(os.path.join(ROOT, "gpurun_out", "repro_code.npy"), code)
    env.destroy()


if __name__ == "__main__":
    main()
