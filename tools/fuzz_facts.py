"""Value-range fuzzing of the compiled path (round 6, after tools/fuzz_gpu.py seed 91 found a
packet load fused with a wider BE32 given the load's own width): straight-line reference-semantics
programs made of what the code generator keeps facts about — packet loads of every width (some
followed by BE16 / BE32 / BE64 / LE on the same register: the fused forms), 32- and 64-bit ALU
with immediates and registers, shifts by any amount, multiplies, NEG, MOV (64-bit MOV adds, as in
the reference) — ending in a fold of every register into r0 with 64-bit multiplies, so that any
wrong bit anywhere shows in the result.  Results and fault codes against the oracle, 64-B staged
packets.

--maps: stack stores with loads of other widths, and array lookups keyed by registers.
--general: ragged packets at CSR offsets (the general kernels: staged headers, short lanes).
--standard: the same programs under standard eBPF semantics (laid out slot after slot).

  python tools/fuzz_facts.py [--programs N] [--seed S] [--variants 0,2] [--maps]"""
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
from generic_ebpf_amd import isa, layout, native, workloads  # noqa: E402

I = isa.Insn
ALU = ["add", "sub", "mul", "or", "and", "xor", "lsh", "rsh", "arsh"]


def program(seed, maps=False, standard=False):
    """maps: also stack stores and loads at other widths (the generator's stack forwarding) and
    array lookups keyed by a register (map 0: 16 x 8 B; the key masked to 15 or not, so the
    lookup's NULL check may be proven away or not) with loads through the result"""
    g = np.random.default_rng(seed)
    regs = list(range(2, 10))
    body = []
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef

    def load(r):
        z = int(g.choice([1, 2, 4, 8]))
        off = int(g.integers(0, 64 - z + 1))
        body.append(I({1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[z], r, 1, off))
        if g.random() < 0.5:   # a swap right after: the fused forms
            body.append(I(str(g.choice(["be", "le"])), r, imm=int(g.choice([16, 32, 64]))))

    if maps:   # (the context pointer, reloaded after each lookup: LDDW r1 replaces it; the
        # stack slots the loads read start defined)
        body.append(I("stxdw", 10, 1, -64))
        body += [I("stdw", 10, 0, -8 * j, int(g.integers(-2**31, 2**31))) for j in range(2, 6)]
    for r in regs:
        if g.random() < 0.7:
            load(r)
        else:
            body.append(I("mov_imm", r, imm=int(g.integers(-2**31, 2**31))))
    for _ in range(int(g.integers(10, 41))):
        d = int(g.choice(regs))
        u = g.random()
        if u < 0.15:
            load(d)
        elif u < 0.2:
            body.append(I(str(g.choice(["be", "le"])), d, imm=int(g.choice([16, 32, 64]))))
        elif u < 0.25:
            body.append(I(str(g.choice(["neg", "neg64"])), d))
        elif maps and u < 0.33:   # a stack store, and a load of another width somewhere in it
            zs, zl = int(g.choice([1, 2, 4, 8])), int(g.choice([1, 2, 4, 8]))
            slot = -8 * int(g.integers(2, 6))
            body.append(I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[zs], 10, int(g.choice(regs)), slot))
            body.append(I({1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[zl], d, 10,
                          slot + int(g.integers(0, 8 - zl + 1))))
        elif maps and u < 0.38:   # an array lookup keyed by a register, a load through it
            k = int(g.choice(regs))
            if g.random() < 0.6:
                body.append(I("and_imm", k, imm=15))
            body += [I("stxw", 10, k, -4), LdDw(1, MapRef(0)), I("mov_imm", 2, imm=0),
                     I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
                     Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=0x5a5a), I("exit")]),
                     I("ldxdw", 1, 10, -64), I("mov_imm", 2, imm=int(g.integers(0, 2**31)))]
            z = int(g.choice([1, 2, 4, 8]))
            body.append(I({1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[z], d, 0,
                          int(g.integers(0, 8 - z + 1))))
        else:
            op = str(g.choice(ALU + ["mov"]))
            w64 = g.random() < 0.6
            name = op + ("64" if w64 else "")
            if g.random() < 0.5:
                if op in ("lsh", "rsh", "arsh"):
                    imm = int(g.integers(0, 70))
                else:
                    imm = int(g.choice([int(g.integers(-2**31, 2**31)), int(g.integers(0, 256)),
                                        int(g.integers(-256, 0)), 1 << int(g.integers(0, 31))]))
                body.append(I(name + "_imm", d, imm=imm))
            else:
                body.append(I(name + "_reg", d, int(g.choice(regs))))
    body += [I("mov_imm", 0, imm=0)]
    for r in regs:
        body += [I("xor64_reg", 0, r), I("mul64_imm", 0, imm=625341585)]
    body.append(I("exit"))
    if standard:   # (straight-line, slot after slot: standard eBPF's own layout)
        return b"".join(x.encode() for x in body), []
    lay = layout.assemble(body)
    return lay.code, lay.relocs


def ragged(n, seed):
    """n packets of 40..80 bytes at CSR offsets (the general kernels; a load past a short
    packet's end faults MEM)"""
    g = np.random.default_rng(seed)
    sizes = g.integers(40, 81, n).astype(np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    return g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8), offs


def _run(env, code, relocs, specs, c, variant, standard):
    import pyoracle
    op = pyoracle.OracleProgram(code, relocs, specs, semantics=1 if standard else 0)
    want, wf, _, _ = op.run(c.data, c.count, c.stride, c.offsets, nthreads=4)
    maps = []
    for vs, me, d in specs:
        m = native.Map(env, me, vs)
        m.fill(d)
        maps.append(m)
    p = native.Prog(env, native.patch_relocs(code, relocs, [m.handle for m in maps]))
    try:
        if standard:
            p.set_semantics(native.SEM_STANDARD)
        native.set_variant(variant)
        got, gf, _ = p.run_batch(np.ascontiguousarray(c.data.copy()), c.count, c.stride, c.offsets)
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()
    return want, wf, got, gf


def campaign(env, programs, seed, variants=(0,), maps=False, general=False, standard=False):
    """True when any program's results or faults differ from the oracle's (one line a variant);
    general: ragged packets at CSR offsets (the general kernels) instead of 64-B staged ones;
    standard: standard eBPF semantics (straight-line, no maps)"""
    failed = False
    for variant in variants:
        t0, bad = time.time(), []
        for k in range(programs):
            code, relocs = program(seed * 1000003 + k, maps=maps and not standard, standard=standard)
            specs = [(8, 16, np.random.default_rng(k).integers(0, 256, 128, dtype=np.uint8).tobytes())] \
                if maps and not standard else []
            if general:
                data, offs = ragged(256, k)
                c = goldens.Case("f%d" % k, code, relocs, specs, data, 256, 0, offs)
            else:
                pk = workloads.packets_random(256, 64, seed=k)
                c = goldens.Case("f%d" % k, code, relocs, specs, pk.reshape(-1), 256, 64, None)
            want, wf, got, gf = _run(env, code, relocs, specs, c, variant, standard)
            if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
                bad.append(k)
            if k % 1000 == 999:
                print("  ... %d programs, %d mismatches" % (k + 1, len(bad)), flush=True)
        print("facts%s%s%s variant %d: %d programs, %d mismatches %s (%.0f s)" % (
            " (maps)" if maps and not standard else "", " general" if general else "",
            " standard" if standard else "", variant, programs, len(bad), bad[:20], time.time() - t0),
            flush=True)
        failed = failed or bool(bad)
    return failed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--programs", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--maps", action="store_true", help="stack forwarding and array lookups too")
    ap.add_argument("--general", action="store_true", help="ragged packets: the general kernels")
    ap.add_argument("--standard", action="store_true", help="standard eBPF semantics (no maps)")
    a = ap.parse_args()
    env = native.Env()
    failed = campaign(env, a.programs, a.seed, tuple(int(v) for v in a.variants.split(",")), a.maps,
                      a.general, a.standard)
    env.destroy()
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main()
