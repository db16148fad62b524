"""Randomised parity sweep on the GPU (a longer run than tests/test_gpu_parity.py): seeded random
programs (generic-ebpf_amd/randprog.py: every opcode and reference quirk) on the device against the
oracle, for every device variant, on both kernels: 64-B packets (staged) and packets of random
length 16..79 at CSR offsets (general kernels, short packets fault), and with regrouping forced
(EBPF_CC_REGROUP=1, size thresholds 2 and 1: most random programs get regroup points, so random
subtrees are queued and batched).
Odd-numbered programs also call map_update_elem / map_delete_elem (the device batch semantics).
Compares results, fault codes, post-run packet bytes and the maps after the batch.

  python tools/fuzz_gpu.py [--programs N] [--seed S] [--out DIR]
Prints one line per configuration and exits 1 on any mismatch (the failing seeds are listed)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import pkgload  # noqa: E402

pkgload.load()
import goldens  # noqa: E402
import pyoracle  # noqa: E402
from helpers import make_maps  # noqa: E402
from generic_ebpf_amd import native, randprog, workloads  # noqa: E402


def ragged_packets(n, seed):
    g = np.random.default_rng(seed)
    sizes = g.integers(16, 80, n).astype(np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
    return data, offs


def case(k, seed, layout):
    g = np.random.default_rng(seed * 7919 + k)
    vs = int(g.choice([8, 16]))
    me = int(g.choice([16, 256]))
    lay = randprog.random_program(seed * 100000 + k, length=int(g.integers(10, 120)), nmaps=2,
                                  map_value_size=vs, writes=bool(k & 1))
    maps = [(vs, me, g.integers(0, 256, vs * me, dtype=np.uint8).tobytes()) for _ in range(2)]
    n = int(g.choice([1, 63, 64, 65, 777, 2048]))
    if layout == "staged":
        return goldens.Case("r%d" % k, lay.code, lay.relocs, maps,
                            workloads.packets_random(n, 64, seed=k), n, 64, None)
    data, offs = ragged_packets(n, seed * 31 + k)
    return goldens.Case("r%d" % k, lay.code, lay.relocs, maps, data, n, 0, offs)


def oracle(c):
    """(ret, faults, packet bytes after, map bytes after the batch)"""
    op = pyoracle.OracleProgram(c.code, c.relocs, c.maps)
    ret, faults, data, _ = op.run(c.data, c.count, c.stride, c.offsets, nthreads=8)
    return ret, faults, data, [op.map_bytes(i) for i in range(len(c.maps))]


def device(env, c, variant):
    maps = make_maps(native, env, c)
    p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        native.set_variant(variant)
        data = np.ascontiguousarray(c.data.copy())
        ret, faults, _ = p.run_batch(data, c.count, c.stride, c.offsets)
        after = [b"".join(m.lookup(i)[1] for i in range(m.max_entries)) for m in maps]
        return ret, faults, data, after
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--programs", type=int, default=500)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    env = native.Env()
    failed = False
    configs = [(v, lay, 0) for v in (0, 1, 2) for lay in ("staged", "general")]
    configs += [(0, "general", 2), (0, "general", 1)]   # regrouping, size threshold 2 / 1
    for variant, layout, rg in configs:
        if rg:
            os.environ["EBPF_CC_REGROUP"] = "1"
            os.environ["EBPF_CC_RG_MIN"] = str(rg)
        t0 = time.time()
        bad, faults = [], 0
        for k in range(a.programs):
            c = case(k, a.seed, layout)
            want, wf, wdata, wmaps = oracle(c)
            got, gf, gdata, gmaps = device(env, c, variant)
            faults += int(np.count_nonzero(wf))
            if not (np.array_equal(want, got) and np.array_equal(wf, gf) and
                    np.array_equal(wdata, gdata) and wmaps == gmaps):
                bad.append(k)
        os.environ.pop("EBPF_CC_REGROUP", None)
        os.environ.pop("EBPF_CC_RG_MIN", None)
        print("variant %d %-7s%s: %d programs, %d faulted packets, %d mismatches %s (%.0f s)" % (
            variant, layout, " regroup>=%d" % rg if rg else "", a.programs, faults, len(bad), bad[:20],
            time.time() - t0), flush=True)
        failed = failed or bool(bad)
    env.destroy()
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main()
