#!/usr/bin/env python3
"""Golden vectors for the hashtable maps' key hash, from the reference's own ebpf_jhash.h
(compiled as is by oracle/Makefile's _ref/jhash_harness; container only).  Writes
tests/golden/maps/jhash.npz: keys (concatenated), key offsets, misalignment, initval, expected hash."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/jhash_harness"])
    g = np.random.default_rng(2024)
    keys, lines, meta = [], [], []
    for i in range(600):
        n = int(g.integers(0, 80)) if i >= 100 else i % 40
        key = g.integers(0, 256, n, dtype=np.uint8).tobytes()
        off = int(g.integers(0, 4))
        init = int(g.integers(0, 2**32)) if i % 3 == 0 else 0
        keys.append(key)
        meta.append((off, init))
        lines.append("%d %d %s" % (init, off, key.hex() or "-"))
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "jhash_harness")],
                         input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    hashes = [int(x) for x in out.stdout.split()]
    assert len(hashes) == len(keys)
    offs = np.zeros(len(keys) + 1, dtype=np.int64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "maps", "jhash.npz"),
                        data=np.frombuffer(b"".join(keys), dtype=np.uint8), offsets=offs,
                        misalign=np.array([m[0] for m in meta], dtype=np.int64),
                        initval=np.array([m[1] for m in meta], dtype=np.uint32),
                        expect=np.array(hashes, dtype=np.uint32))
    print("wrote %d jhash vectors" % len(keys))


if __name__ == "__main__":
    sys.exit(main())
