"""Randomised parity sweep on the GPU (a longer run than tests/test_gpu_parity.py): seeded random
programs (generic-ebpf_amd/randprog.py: every opcode and reference quirk) on the device against the
oracle, for every device variant, on both kernels: 64-B packets (staged) and packets of random
length 16..79 at CSR offsets (general kernels, short packets fault).
Odd-numbered programs also call map_update_elem / map_delete_elem (the device batch semantics).
Compares results, fault codes, post-run packet bytes and the maps after the batch.
--hash: the programs' two maps are hashtables instead (4-byte keys, a random live subset of a
key universe the programs' keys hit and miss, capacity 16 or 256 so that inserts can hit EBUSY):
lookups, updates and deletes against the oracle's replay model; the tables are compared through
get_next_key's walk (order and values).

--loopwrites --hash: loop programs mixing counters (fetched or not), stores, loads back and
update calls in one hashtable's values (round 6: its counter updates are counted records).

  python tools/fuzz_gpu.py [--programs N] [--seed S] [--hash | --standard | --mutate | --loopwrites |
                                                      --manywrites]
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


def hash_spec(g, vs):
    cap = int(g.choice([16, 256]))
    universe = np.unique(np.concatenate([np.arange(8), g.integers(0, 256, 64),
                                         g.integers(0, 2**32, 64)]).astype(np.uint64))
    keys = g.permutation(universe)[:int(g.integers(0, cap + 1))]
    items = [(int(x).to_bytes(4, "little"), g.bytes(vs)) for x in keys]
    return pyoracle.HashSpec(4, vs, items=items, capacity=cap)


def case(k, seed, layout, hashed=False, writes=None, many=False):
    g = np.random.default_rng(seed * 7919 + k)
    vs = int(g.choice([8, 16, 72, 200]))   # (> 64: no inline constant, round 5)
    me = int(g.choice([16, 256]))
    lay = randprog.random_program(seed * 100000 + k, length=int(g.integers(10, 120)), nmaps=2,
                                  map_value_size=vs,
                                  writes=(bool(k & 1) or hashed) if writes is None else writes,
                                  many_writes=many)
    if hashed:
        maps = [hash_spec(g, vs) for _ in range(2)]
    else:
        maps = [(vs, me, g.integers(0, 256, vs * me, dtype=np.uint8).tobytes()) for _ in range(2)]
    n = int(g.choice([1, 63, 64, 65, 777, 2048]))
    if layout == "staged":
        c = goldens.Case("r%d" % k, lay.code, lay.relocs, [] if hashed else maps,
                         workloads.packets_random(n, 64, seed=k), n, 64, None)
    else:
        data, offs = ragged_packets(n, seed * 31 + k)
        c = goldens.Case("r%d" % k, lay.code, lay.relocs, [] if hashed else maps, data, n, 0, offs)
    if hashed:
        c.maps = maps
    return c


def oracle(c):
    """(ret, faults, packet bytes after, maps after the batch: array bytes / hashtable items)"""
    op = pyoracle.OracleProgram(c.code, c.relocs, c.maps)
    ret, faults, data, _ = op.run(c.data, c.count, c.stride, c.offsets, nthreads=8)
    return ret, faults, data, [op.hash_models[i].items() if isinstance(m, pyoracle.HashSpec)
                               else op.map_bytes(i) for i, m in enumerate(c.maps)]


def walk(m):
    """A device-side hashtable through the host API: get_next_key's walk with the values."""
    import ctypes
    out, prev = [], None
    while True:
        nk = ctypes.create_string_buffer(m.key_size)
        k = None if prev is None else ctypes.create_string_buffer(prev, m.key_size)
        if native.lib().ebpf_map_get_next_key_from_user(m.ptr, k, nk) != 0:
            return out
        prev = nk.raw
        out.append((prev, m.lookup(prev)[1]))


def device(env, c, variant, extents=False):
    """extents: the CSR offsets handed over as (start, end) pairs (EBPF_BATCH_EXTENTS), the
    same packets: the results must not change."""
    if isinstance(c.maps[0], pyoracle.HashSpec):
        maps = []
        for spec in c.maps:
            m = native.HashMap(env, spec.key_size, spec.value_size, spec.capacity)
            for kk, vv in spec.items:
                assert m.update(kk, vv) == 0
            maps.append(m)
    else:
        maps = make_maps(native, env, c)
    p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        native.set_variant(variant)
        data = np.ascontiguousarray(c.data.copy())
        if extents and c.offsets is not None:
            o = np.asarray(c.offsets, dtype=np.uint64)
            ext = np.stack([o[:-1], o[1:]], axis=1).reshape(-1)
            ret, faults, _ = p.run_batch(data, c.count, 0, ext, extents=True)
        else:
            ret, faults, _ = p.run_batch(data, c.count, c.stride, c.offsets)
        after = [walk(m) if isinstance(m, native.HashMap) else
                 b"".join(m.lookup(i)[1] for i in range(m.max_entries)) for m in maps]
        return ret, faults, data, after
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


def standard(a, env):
    """--standard: random programs under standard eBPF semantics (tests/stdprogs.py: loop-free
    programs with every ALU op, JMP32, stack, packet and array-lookup access; programs with counted
    loops; cursor walks over the packet) against the oracle's run_std, 64-B packets (staged) and
    72-B (general kernels)."""
    import stdprogs
    failed = False
    for variant in getattr(a, "variants", (0, 1, 2)):
        for stride in (64, 72):
            t0, bad = time.time(), []
            for k in range(a.programs):
                seed = a.seed * 100000 + k
                g = np.random.default_rng(seed)
                specs = []
                if k % 4 == 3:   # a packet walk with a cursor (loads at run-time offsets)
                    code, rel = stdprogs.gen_cursor_program(seed)
                elif k % 2:
                    code, rel = stdprogs.gen_loop_program(seed, length=int(g.integers(10, 40)))
                else:
                    code, rel = stdprogs.gen_program(seed, length=int(g.integers(10, 80)), with_map=k % 4 == 0)
                    if k % 4 == 0:
                        specs = [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())]
                n = int(g.choice([1, 64, 65, 777, 2048]))
                pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
                if a.mutate and k % 2:
                    continue  # (loop programs: an edit can make a loop run to the 2^20 budget on
                              # every packet, minutes of oracle time; mutated runs take loop-free ones)
                if a.mutate:  # (forward offsets only: a new backward edge would loop to the budget)
                    code = mutate(code, np.random.default_rng(seed + 1), forward=True)
                    outs = []
                    for si in (0, 0xa5):
                        r, f, _, _ = pyoracle.OracleProgram(code, rel, specs, semantics=1, stack_init=si,
                                                            track_undef=True).run(pk.reshape(-1), n, stride, nthreads=8)
                        outs.append((r.tobytes(), f.tobytes(), bool((f == 100).any())))
                    if outs[0][2] or outs[0] != outs[1]:
                        continue
                want, wf, _, _ = pyoracle.OracleProgram(code, rel, specs, semantics=1).run(
                    pk.reshape(-1), n, stride, nthreads=8)
                maps = []
                for vs, me, d in specs:
                    m = native.Map(env, me, vs)
                    m.fill(d)
                    maps.append(m)
                p = native.Prog(env, native.patch_relocs(code, rel, [m.handle for m in maps]))
                try:
                    p.set_semantics(native.SEM_STANDARD)
                    native.set_variant(variant)
                    got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, stride)
                finally:
                    native.set_variant(0)
                    p.destroy()
                    for m in maps:
                        m.destroy()
                if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
                    bad.append(k)
                if k % 100 == 99:
                    print("  ... %d programs, %d mismatches" % (k + 1, len(bad)), flush=True)
            print("standard%s variant %d stride %d: %d programs, %d mismatches %s (%.0f s)" % (
                " mutated" if a.mutate else "", variant, stride, a.programs, len(bad), bad[:20],
                time.time() - t0), flush=True)
            failed = failed or bool(bad)
    return failed


def mutate(code, g, forward=False):
    """4-15 random edits of a program (reference semantics): a conditional jump's offset set to 0
    or to a small value, a slot replaced by JA +0 / JA +1, an immediate changed."""
    b = bytearray(code)
    n = len(b) // 8
    conds = [i for i in range(n) if (b[8 * i] & 7) == 5 and b[8 * i] not in (0x05, 0x85, 0x95)]
    for _ in range(int(g.integers(4, 16))):
        kind = int(g.integers(0, 4))
        if kind <= 1 and conds:
            i = int(g.choice(conds))
            off = 0 if kind == 0 else int(g.integers(0 if forward else -3, 4))
            b[8 * i + 2:8 * i + 4] = (off & 0xffff).to_bytes(2, "little")
        elif kind == 2:
            i = int(g.integers(0, n))
            b[8 * i:8 * i + 8] = bytes([0x05, 0]) + int(g.integers(0, 2)).to_bytes(2, "little") + bytes(4)
        else:
            i = int(g.integers(0, n))
            if b[8 * i] != 0x18 and (i == 0 or b[8 * i - 8] != 0x18):
                b[8 * i + 4:8 * i + 8] = int(g.integers(-2**31, 2**31)).to_bytes(4, "little", signed=True)
    return bytes(b)


def defined(c):
    """The oracle's results do not depend on the uninitialised stack or on addresses
    (track_undef, two stack fills, two thread counts)."""
    outs = []
    for si, nt in ((0, 1), (0xa5, 3)):
        op = pyoracle.OracleProgram(c.code, c.relocs, c.maps, stack_init=si, track_undef=True)
        ret, faults, data, _ = op.run(c.data, c.count, c.stride, c.offsets, nthreads=nt)
        if (faults == 100).any():
            return False
        outs.append((ret.tobytes(), faults.tobytes(), data.tobytes()))
    return outs[0] == outs[1]


def mutated(a, env):
    """--mutate: random programs edited at random (zero and small jump offsets, JA +0 / +1 slots,
    new immediates), kept only when the oracle finds them defined, on every variant and both
    kernels."""
    failed = False
    for variant, layout in [(v, lay) for v in getattr(a, "variants", (0, 1, 2))
                            for lay in ("staged", "general")]:
        t0, bad, kept = time.time(), [], 0
        for k in range(a.programs):
            # (seed 1 keeps the round-3 campaign's programs; other seeds mix in map writes)
            c = case(k, a.seed, layout, writes=bool(k & 1) if a.seed != 1 else False)
            c.code = mutate(c.code, np.random.default_rng(a.seed * 7777 + k))
            if not defined(c):
                continue
            kept += 1
            want, wf, wdata, wmaps = oracle(c)
            try:
                got, gf, gdata, gmaps = device(env, c, variant)
            except Exception as e:  # noqa: BLE001
                bad.append((k, str(e)[:60]))
                continue
            if not (np.array_equal(want, got) and np.array_equal(wf, gf) and
                    np.array_equal(wdata, gdata) and wmaps == gmaps):
                bad.append(k)
            if k % 500 == 499:
                print("  ... %d programs, %d kept, %d mismatches" % (k + 1, kept, len(bad)), flush=True)
        print("mutated variant %d %-7s: %d programs, %d defined, %d mismatches %s (%.0f s)" % (
            variant, layout, a.programs, kept, len(bad), bad[:20], time.time() - t0), flush=True)
        failed = failed or bool(bad)
    return failed


def reference(a, env):
    """Random programs under the reference's semantics (array maps, or hashtables with --hash)
    on every variant and both kernels; returns True on any mismatch.  --manywrites: every
    program's main path ends with 17..60 stores into a map value or 17..40 map_update_elem calls
    (randprog bulk_writes: a loop-free program has no write limit)."""
    failed = False
    many = getattr(a, "manywrites", False)
    for variant in getattr(a, "variants", (0, 1, 2)):
        for layout in ("staged", "general"):
            t0 = time.time()
            bad, faults = [], 0
            for k in range(a.programs):
                c = case(k, a.seed, layout, a.hash, many=many)
                want, wf, wdata, wmaps = oracle(c)
                # (every other general-kernel case hands its packets over as extents)
                got, gf, gdata, gmaps = device(env, c, variant, extents=bool(k & 2))
                faults += int(np.count_nonzero(wf))
                if not (np.array_equal(want, got) and np.array_equal(wf, gf) and
                        np.array_equal(wdata, gdata) and wmaps == gmaps):
                    bad.append(k)
                if k % 100 == 99:
                    print("  ... %d programs, %d mismatches" % (k + 1, len(bad)), flush=True)
            print("%s%svariant %d %-7s: %d programs, %d faulted packets, %d mismatches %s (%.0f s)" % (
                "hash " if a.hash else "", "many-writes " if many else "", variant, layout, a.programs,
                faults, len(bad), bad[:20], time.time() - t0), flush=True)
            failed = failed or bool(bad)
    return failed


def loop_writes(a, env):
    """--loopwrites: random standard programs that write maps inside loops
    (stdprogs.gen_loop_write_program: stores, loads back, updates, and every third program
    counter updates — read back, XADD with BPF_FETCH and live idiom registers, with --fetched;
    trip counts up to 24, so packets pass the 16 logged writes (or the 32 words of the view)
    and fault WRITES) on every variant, staged 64-B packets; results, faults and both maps
    against the oracle's batch mode."""
    import stdprogs
    failed = False
    hashed = getattr(a, "hash", False)
    for variant in getattr(a, "variants", (0, 1, 2)):
        t0, bad, faults = time.time(), [], 0
        for k in range(a.programs):
            seed = a.seed * 100000 + k
            g = np.random.default_rng(seed)
            # (every third program counts; with --fetched, the counters are read back; with
            # --hash map 0 is a hashtable and every program mixes counters, fetched or not,
            # stores, loads back and updates of map 1 in its values)
            fetched = k % 3 == 2 and getattr(a, "fetched", False)
            code, rel = stdprogs.gen_loop_write_program(seed, counters=k % 3 == 2, fetched=fetched,
                                                        mixed=hashed)
            vs0 = 32 if fetched else 16
            arr = (8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())
            if hashed:   # (a random subset of the 16 keys the programs look up; capacity 16)
                keys = g.permutation(16)[:int(g.integers(0, 17))]
                specs = [pyoracle.HashSpec(4, 16, items=[(int(x).to_bytes(4, "little"), g.bytes(16))
                                                         for x in keys], capacity=16), arr]
            else:
                specs = [(vs0, 16, g.integers(0, 256, 16 * vs0, dtype=np.uint8).tobytes()), arr]
            n = int(g.choice([1, 64, 65, 777, 4099]))
            pk = g.integers(0, 256, (n, 64), dtype=np.uint8)
            op = pyoracle.OracleProgram(code, rel, specs, semantics=1)
            want, wf, _, _ = op.run(pk.reshape(-1), n, 64, nthreads=8)
            faults += int(np.count_nonzero(wf))
            maps = []
            for spec in specs:
                if isinstance(spec, pyoracle.HashSpec):
                    m = native.HashMap(env, 4, spec.value_size, spec.capacity)
                    for kk, vv in spec.items:
                        assert m.update(kk, vv) == 0
                else:
                    vs, me, d = spec
                    m = native.Map(env, me, vs)
                    m.fill(d)
                maps.append(m)
            p = native.Prog(env, native.patch_relocs(code, rel, [m.handle for m in maps]))
            try:
                p.set_semantics(native.SEM_STANDARD)
                native.set_variant(variant)
                got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, 64)
                after = [walk(m) if isinstance(m, native.HashMap) else
                         b"".join(m.lookup(key)[1] for key in range(m.max_entries)) for m in maps]
            finally:
                native.set_variant(0)
                p.destroy()
                for m in maps:
                    m.destroy()
            want0 = op.hash_models[0].items() if hashed else op.map_bytes(0)
            if not (np.array_equal(want, got) and np.array_equal(wf, gf) and
                    after[0] == want0 and after[1] == op.map_bytes(1)):
                bad.append(k)
            if k % 100 == 99:
                print("  ... %d programs, %d mismatches" % (k + 1, len(bad)), flush=True)
        print("loop writes%s%s variant %d: %d programs, %d faulted packets, %d mismatches %s (%.0f s)" % (
            " (fetched)" if getattr(a, "fetched", False) else "", " (hashtable)" if hashed else "",
            variant, a.programs, faults, len(bad), bad[:20], time.time() - t0), flush=True)
        failed = failed or bool(bad)
    return failed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--programs", type=int, default=500)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--hash", action="store_true", help="hashtable maps (lookups and writes)")
    ap.add_argument("--standard", action="store_true", help="standard eBPF semantics (loops too)")
    ap.add_argument("--mutate", action="store_true", help="randomly edited programs (defined ones)")
    ap.add_argument("--loopwrites", action="store_true", help="map writes inside loops (standard)")
    ap.add_argument("--fetched", action="store_true",
                    help="with --loopwrites: the counter programs read their counters back")
    ap.add_argument("--manywrites", action="store_true",
                    help="reference programs with more than 16 map writes on one path")
    ap.add_argument("--variants", default="0,1,2", help="device variants to run (e.g. 0: compiled only)")
    a = ap.parse_args()
    a.variants = tuple(int(v) for v in a.variants.split(","))
    env = native.Env()
    if a.loopwrites:
        failed = loop_writes(a, env)
    elif a.manywrites:
        failed = reference(a, env)
    elif a.mutate and not a.standard:
        failed = mutated(a, env)
    elif a.standard:
        failed = standard(a, env)
    else:
        failed = reference(a, env)
    env.destroy()
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main()
