#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the GENUINE reference interpreter (container only).

The reference libebpf.so is the one the survey built from /root/reference in a scratch copy
(/tmp/refbuild); this script does not build or copy the reference.  It
compiles oracle/refgen/ref_harness.c against it (outputs only under oracle/_ref/), writes each
case to a binary case file, runs the harness (every packet twice under two stack poisons), and
keeps a case only if no packet read undefined state.

Usage: python tools/gen_golden.py [--quick] [--rand N] [--pkts N]
"""
import argparse
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pkgload  # noqa: E402
import goldens  # noqa: E402

pkg = pkgload.load()
isa, layout, workloads = pkg.isa, pkg.layout, pkg.workloads
from generic_ebpf_amd import randprog  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def write_case(path, c):
    with open(path, "wb") as f:
        f.write(struct.pack("<IIII", 0x43504245, 1, len(c.code), len(c.maps)))
        for vs, me, d in c.maps:
            assert len(d) == vs * me
            f.write(struct.pack("<II", vs, me))
            f.write(d)
        f.write(struct.pack("<I", len(c.relocs)))
        for s, m in c.relocs:
            f.write(struct.pack("<II", s, m))
        f.write(c.code)
        f.write(struct.pack("<QII", c.count, c.stride, 0 if c.offsets is None else 1))
        if c.offsets is not None:
            f.write(np.asarray(c.offsets, dtype=np.uint64).tobytes())
        f.write(struct.pack("<Q", len(c.data)))
        f.write(c.data.tobytes())


def run_reference(c, tmp):
    cp, op = os.path.join(tmp, "case.bin"), os.path.join(tmp, "out.bin")
    write_case(cp, c)
    subprocess.check_call([HARNESS, cp, op])
    raw = open(op, "rb").read()
    n = c.count
    r0 = np.frombuffer(raw[:8 * n], dtype=np.uint64).copy()
    undef = np.frombuffer(raw[8 * n: 9 * n], dtype=np.uint8).copy()
    after = np.frombuffer(raw[9 * n:], dtype=np.uint8).copy()
    return r0, undef, after


# ----------------------------------------------------------------------------- cases

def raw_prog(slots):
    """slots: dict slot -> (op, dst, src, off, imm); holes get MOV r0, 0x5eed (never executed
    if the stepping rule is honoured — a wrong stepper returns 0x5eed-derived values)."""
    n = max(slots) + 1
    b = bytearray()
    for i in range(n):
        if i in slots:
            b += isa.encode(*slots[i])
        else:
            b += isa.encode(isa.OPS["mov_imm"], 0, 0, 0, 0x5eed)
    return bytes(b)


def kat_cases():
    O = isa.OPS
    pk = np.zeros(64, dtype=np.uint8)
    pk[:8] = [0x00, 0x12, 0x24, 0x36, 0x48, 0x5a, 0x6c, 0x7e]
    progs = {
        "kat_cumulative_pc": {0: (O["mov_imm"], 0, 0, 0, 1), 1: (O["add_imm"], 0, 0, 0, 1),
                              2: (O["add_imm"], 0, 0, 0, 1), 3: (O["exit"], 0, 0, 0, 0)},
        "kat_mov64_adds": {0: (O["mov_imm"], 0, 0, 0, 5), 1: (O["mov64_imm"], 0, 0, 0, 3),
                           3: (O["exit"], 0, 0, 0, 0)},
        "kat_neg32": {0: (O["mov_imm"], 0, 0, 0, 5), 1: (O["neg"], 0, 0, 0, 7),
                      3: (O["exit"], 0, 0, 0, 0)},
        "kat_neg64": {0: (O["mov_imm"], 0, 0, 0, 5), 1: (O["neg64"], 0, 0, 0, 7),
                      3: (O["exit"], 0, 0, 0, 0)},
        "kat_arsh32_logical": {0: (O["mov_imm"], 0, 0, 0, -16), 1: (O["arsh_imm"], 0, 0, 0, 2),
                               3: (O["exit"], 0, 0, 0, 0)},
        "kat_lddw_arsh64": {0: (O["lddw"], 0, 0, 0, 0), 1: (0, 0, 0, 0, isa.s32(0x80000000)),
                            2: (O["arsh64_imm"], 0, 0, 0, 4), 5: (O["exit"], 0, 0, 0, 0)},
        "kat_lsh32_mask": {0: (O["mov_imm"], 0, 0, 0, 1), 1: (O["lsh_imm"], 0, 0, 0, 33),
                           3: (O["exit"], 0, 0, 0, 0)},
        "kat_lsh64_mask": {0: (O["mov_imm"], 0, 0, 0, 1), 1: (O["lsh64_imm"], 0, 0, 0, 65),
                           3: (O["exit"], 0, 0, 0, 0)},
        "kat_ja_fwd": {0: (O["mov_imm"], 0, 0, 0, 7), 1: (O["ja"], 0, 0, 2, 0),
                       5: (O["exit"], 0, 0, 0, 0)},
        "kat_ja_back": {0: (O["mov_imm"], 0, 0, 0, 1), 1: (O["add_imm"], 0, 0, 0, 2),
                        3: (O["ja"], 0, 0, -2, 0), 4: (O["exit"], 0, 0, 0, 0)},
        "kat_jeq_sext": {0: (O["mov_imm"], 0, 0, 0, -1), 1: (O["jeq_imm"], 0, 0, 1, -1),
                         3: (O["exit"], 0, 0, 0, 0), 4: (O["mov_imm"], 0, 0, 0, 0x55),
                         8: (O["exit"], 0, 0, 0, 0)},
        "kat_ldxdw_be32": {0: (O["ldxdw"], 0, 1, 0, 0), 1: (O["be"], 0, 0, 0, 32),
                           3: (O["exit"], 0, 0, 0, 0)},
        "kat_stdw_ldxb": {0: (O["stdw"], 10, 0, -8, -2), 1: (O["ldxb"], 0, 10, -8, 0),
                          3: (O["exit"], 0, 0, 0, 0)},
    }
    out = []
    for name, sl in progs.items():
        out.append(goldens.Case(name, raw_prog(sl), [], [], pk.copy(), 1, 64, None))
    return out


def map_bytes(values, vs):
    return b"".join(int(v).to_bytes(8, "little")[:vs].ljust(vs, b"\0") for v in values)


def rand_cases(n, seed0):
    out = []
    g = np.random.default_rng(seed0)
    for k in range(n):
        vs = int(g.choice([8, 16, 32]))
        me = int(g.choice([8, 256, 300]))
        lay = randprog.random_program(seed0 + k, length=int(g.integers(10, 60)), nmaps=2,
                                      map_value_size=vs)
        maps = [(vs, me, g.integers(0, 256, vs * me, dtype=np.uint8).tobytes()) for _ in range(2)]
        pk = workloads.packets_random(64, 64, seed=seed0 + 1000 + k)
        out.append(goldens.Case("rand_%d" % (seed0 + k), lay.code, lay.relocs, maps, pk, 64, 64,
                                None))
    return out


def workload_cases(n):
    out = []
    c2 = workloads.prog_c2()
    out.append(goldens.Case("c2", c2.code, [], [], workloads.packets_random(n, 64, 2), n, 64, None))
    c3 = workloads.prog_c3()
    out.append(goldens.Case("c3", c3.code, [], [], workloads.packets_l2l3(n, 64, 3), n, 64, None))
    c4 = workloads.prog_c4()
    vals = workloads.c4_map_values()
    out.append(goldens.Case("c4", c4.code, c4.relocs, [(8, 256, map_bytes(vals, 8))],
                            workloads.packets_l2l3(n, 64, 3), n, 64, None))
    c5 = workloads.prog_c5()
    m = max(64, n // 4)
    data, offs, _ = workloads.packets_imix(m, seed=5)
    out.append(goldens.Case("c5", c5.code, [], [], data, m, 0, offs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--rand", type=int, default=200, help="random-program cases")
    ap.add_argument("--pkts", type=int, default=2048, help="packets per workload case")
    args = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_harness"])
    os.makedirs(goldens.GOLDEN_DIR, exist_ok=True)
    groups = {
        "kat": kat_cases(),
        "rand": rand_cases(40 if args.quick else args.rand, 1000),
        "workloads": workload_cases(512 if args.quick else args.pkts),
    }
    with tempfile.TemporaryDirectory() as tmp:
        for gname, cases in groups.items():
            keep = []
            for c in cases:
                r0, undef, after = run_reference(c, tmp)
                if undef.any():
                    print("drop %s: %d packets read undefined state" % (c.name, int((undef != 0).sum())))
                    continue
                c.expect_r0, c.expect_data = r0, after
                keep.append(c)
            path = os.path.join(goldens.GOLDEN_DIR, gname + ".npz")
            goldens.save(path, keep)
            print("%s: %d cases -> %s (%d bytes)" % (gname, len(keep), path, os.path.getsize(path)))


if __name__ == "__main__":
    main()
