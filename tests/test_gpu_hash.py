"""Device hashtable lookups (read-only device table, dprog.h dp_map) against the oracle's
hashtable_map_lookup_elem restatement: every device variant, the staged and the general kernels,
key sizes 1..40, keys on the stack or in the packet, NULL keys, faults, two hashtables in one
program, table refresh after host updates, and a large table with long probe chains."""
import numpy as np
import pytest

import hashprogs
import pyoracle
from test_maps_hash import HCASES, hcase

pytestmark = pytest.mark.gpu

VARIANTS = [0, 1, 2]   # compiled, portable HIP, asm interpreter


def run_device(native, env, lay, specs, data, count, stride, offsets=None, variant=0, max_entries=64):
    maps = [hashprogs.NativeHash(native, env, s.key_size, s.value_size, max_entries, s.items)
            for s in specs]
    p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        native.set_variant(variant)
        d = np.ascontiguousarray(data.copy())
        ret, faults, _ = p.run_batch(d, count, stride, offsets)
        return ret, faults
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 80])
def test_hash_cases_vs_oracle(gpu, env, variant, stride):
    bad = []
    for k in range(len(HCASES)):
        rng = np.random.default_rng(300 + k)
        lay, specs, pk = hcase(k, rng, n=4096, size=stride)
        want, wf, _ = hashprogs.oracle(lay, specs, pk.reshape(-1), len(pk), stride)
        got, gf = run_device(gpu, env, lay, specs, pk.reshape(-1), len(pk), stride, variant=variant)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad.append((k, int(np.count_nonzero(want != got)), int(np.count_nonzero(wf != gf))))
    assert not bad, bad


@pytest.mark.parametrize("variant", VARIANTS)
def test_hash_value_store_read_back(gpu, env, variant):
    """A store into a hashtable value through the lookup result, then a load of it: the packet
    reads its own store (no MAP_WRITE fault since round 4)."""
    rng = np.random.default_rng(5)
    items, keys = hashprogs.make_table(rng, 4, 8, 40)
    lay = hashprogs.lookup_program(4, "stack", 0, store=True)
    specs = [pyoracle.HashSpec(4, 8, items)]
    pk = hashprogs.packets_with_keys(rng, 2048, 64, keys, 0, 4)
    want, wf, _ = hashprogs.oracle(lay, specs, pk.reshape(-1), len(pk), 64)
    got, gf = run_device(gpu, env, lay, specs, pk.reshape(-1), len(pk), 64, variant=variant)
    assert not wf.any() and (want == 0xdead).any() and (want != 0xdead).any()
    assert np.array_equal(want, got) and np.array_equal(wf, gf)


@pytest.mark.parametrize("variant", [0, 2])
def test_hash_offsets_batch(gpu, env, variant):
    """Ragged packets (CSR offsets): keys in the packet, some packets too short for the key."""
    rng = np.random.default_rng(9)
    items, keys = hashprogs.make_table(rng, 6, 8, 200)
    lay = hashprogs.lookup_program(6, "packet", 10)
    n = 3000
    lens = rng.integers(8, 120, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    for i in range(n):
        if lens[i] >= 16:
            k = keys[int(rng.integers(0, len(keys)))]
            data[int(offs[i]) + 10:int(offs[i]) + 16] = np.frombuffer(k, dtype=np.uint8)
    specs = [pyoracle.HashSpec(6, 8, items)]
    want, wf, _ = hashprogs.oracle(lay, specs, data, n, 0, offs)
    got, gf = run_device(gpu, env, lay, specs, data, n, 0, offs, variant=variant, max_entries=256)
    assert wf.any() and (want == 0xdead).any()
    assert np.array_equal(want, got) and np.array_equal(wf, gf)


@pytest.mark.parametrize("variant", VARIANTS)
def test_hash_table_refresh_after_updates(gpu, env, variant):
    """Host updates, deletes and replacements between batches reach the device table."""
    rng = np.random.default_rng(11)
    items, keys = hashprogs.make_table(rng, 4, 8, 50)
    lay = hashprogs.lookup_program(4, "stack", 0)
    pk = hashprogs.packets_with_keys(rng, 4096, 64, keys, 0, 4)
    m = hashprogs.NativeHash(gpu, env, 4, 8, 100, items)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    try:
        gpu.set_variant(variant)
        live = dict(items)
        for rnd in range(4):
            d = np.ascontiguousarray(pk.reshape(-1).copy())
            got, gf, _ = p.run_batch(d, len(pk), 64)
            want, wf, _ = hashprogs.oracle(lay, [pyoracle.HashSpec(4, 8, list(live.items()))],
                                           pk.reshape(-1), len(pk), 64)
            assert np.array_equal(want, got) and np.array_equal(wf, gf), rnd
            for k in list(live)[:10]:
                m.delete(k)
                del live[k]
            for k in keys[50 + 10 * rnd:60 + 10 * rnd]:
                v = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
                m.update(k, v)
                live[k] = v
            k0 = next(iter(live))
            live[k0] = b"\x01" * 8
            m.update(k0, live[k0])
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


@pytest.mark.parametrize("variant", [0, 1])
def test_hash_large_table(gpu, env, variant):
    """200k entries of 8-byte keys (a 512k-slot device table), 1M packets, half hits."""
    rng = np.random.default_rng(13)
    n_items = 200_000
    keys = np.unique(rng.integers(0, 2**63, 2 * n_items + 1000, dtype=np.uint64))[:2 * n_items]
    rng.shuffle(keys)
    kb = keys.view(np.uint8).reshape(-1, 8)
    vals = rng.integers(0, 2**63, n_items, dtype=np.uint64)
    items = [(kb[i].tobytes(), vals[i].tobytes()) for i in range(n_items)]
    lay = hashprogs.lookup_program(8, "packet", 16)
    n = 1 << 20
    pk = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    pk[:, 16:24] = kb[rng.integers(0, len(kb), n)]
    # expected: a numpy join instead of the oracle's linear scan (same semantics, fast)
    lut = dict(zip(keys[:n_items].tolist(), vals.tolist()))
    pkeys = pk[:, 16:24].copy().view(np.uint64).reshape(-1)
    want = np.array([lut.get(k, 0xdead) for k in pkeys.tolist()], dtype=np.uint64)
    got, gf = run_device(gpu, env, lay, [pyoracle.HashSpec(8, 8, items)], pk.reshape(-1), n, 64,
                         variant=variant, max_entries=n_items)
    assert not gf.any()
    assert np.array_equal(want, got)


@pytest.mark.parametrize("variant", [0, 2])
def test_c4h_full_size(gpu, env, variant):
    """The C4H bench workload at its full size (64M packets tiled from 1M distinct over the
    1M-entry table): device result of packet i == the oracle's for the distinct packet it tiles."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4h()
    universe, keys, values = workloads.c4h_table()
    distinct, tiles = 1 << 20, 64
    pk = workloads.packets_c4h(distinct, universe)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [pyoracle.HashSpec(4, 8, keys=keys, values=values)])
    want, wf, _, _ = op.run(pk.reshape(-1), distinct, 64, None, nthreads=8)
    assert not wf.any()
    assert (want == 2).any()      # misses take the NULL branch (exit 2) ...
    m = gpu.HashMap(env, 4, 8, len(keys))
    m.fill(keys, values)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    try:
        gpu.set_variant(variant)
        data = np.tile(pk.reshape(-1), tiles)
        got, gf, _ = p.run_batch(data, distinct * tiles, 64)
        assert not gf.any()
        np.testing.assert_array_equal(got.reshape(tiles, distinct),
                                      np.broadcast_to(want, (tiles, distinct)))
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


@pytest.mark.parametrize("knob", ["EBPF_CC_HSPEC", "EBPF_CC_DEFER_DMA"])
def test_hash_cases_specialised_lookup(gpu, env, monkeypatch, knob):
    """The code generator's opt-in hashtable paths against the oracle, on every case with a key
    of at most 8 bytes in the frame and on the C4H program: the inline probe (EBPF_CC_HSPEC=1)
    and the next group's packet DMA issued behind the first probe (EBPF_CC_DEFER_DMA=1)."""
    monkeypatch.setenv(knob, "1")
    bad = []
    for k in range(len(HCASES)):
        rng = np.random.default_rng(900 + k)
        lay, specs, pk = hcase(k, rng, n=4096, size=64)
        want, wf, _ = hashprogs.oracle(lay, specs, pk.reshape(-1), len(pk), 64)
        got, gf = run_device(gpu, env, lay, specs, pk.reshape(-1), len(pk), 64, variant=0)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad.append(k)
    assert not bad, bad
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4h()
    universe, keys, values = workloads.c4h_table(entries=1 << 16)
    pk = workloads.packets_c4h(1 << 18, universe)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [pyoracle.HashSpec(4, 8, keys=keys, values=values)])
    want, wf, _, _ = op.run(pk.reshape(-1), len(pk), 64, None, nthreads=8)
    m = gpu.HashMap(env, 4, 8, len(keys))
    m.fill(keys, values)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    try:
        got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), len(pk), 64)
        assert not gf.any() and np.array_equal(want, got)
    finally:
        p.destroy()
        m.destroy()


def _runtime_map_program(sel_mask=1, scale=None):
    """r1 = map 0 + sel * (map 1 - map 0), sel = pkt[5] & sel_mask: the lookup's map is known only
    at run time (sel_mask 3 also makes r1 = map 0 + 2 * (map 1 - map 0) and + 3 *: not maps,
    BAD_MAP); key = the packet's first 4 bytes on the stack; r0 = the value's first 8 bytes or
    0xdead."""
    from generic_ebpf_amd import isa
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef, assemble
    I = isa.Insn
    nodes = [I("mov_imm", 6, imm=0), I("mov64_reg", 6, 1), I("ldxw", 9, 6, 0), I("stxw", 10, 9, -8),
             I("ldxb", 7, 6, 5), I("and_imm", 7, imm=sel_mask),
             LdDw(1, MapRef(0)), LdDw(8, MapRef(1)), I("sub64_reg", 8, 1), I("mul64_reg", 8, 7),
             I("add64_reg", 1, 8),
             I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-8),
             I("call", imm=0),
             Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=0xdead), I("exit")]),
             I("ldxdw", 0, 0, 0), I("exit")]
    return assemble(nodes)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("second", ["hash", "array"])
@pytest.mark.parametrize("sel_mask", [1, 3])
def test_hash_lookup_map_known_at_run_time(gpu, env, variant, second, sel_mask):
    """The lookup's map is a run-time value: hashtable A, or hashtable / array B, or (sel_mask 3)
    not a map at all (BAD_MAP), per packet — the translator's compare chain on r1 against the
    oracle, whose helper resolves r1 at run time like the reference."""
    rng = np.random.default_rng(91)
    items_a, keys_a = hashprogs.make_table(rng, 4, 8, 40)
    items_b, keys_b = hashprogs.make_table(rng, 4, 8, 40)
    n = 4096
    keys = keys_a + keys_b + [bytes([k, 0, 0, 0]) for k in range(16)]
    pk = hashprogs.packets_with_keys(rng, n, 64, keys, 0, 4)
    lay = _runtime_map_program(sel_mask)
    spec_a = pyoracle.HashSpec(4, 8, items=items_a)
    arr = rng.integers(0, 256, 16 * 8, dtype=np.uint8).tobytes()
    spec_b = pyoracle.HashSpec(4, 8, items=items_b) if second == "hash" else (8, 16, arr)
    want, wf, _ = hashprogs.oracle(lay, [spec_a, spec_b], pk.reshape(-1), n, 64)
    ma = hashprogs.NativeHash(gpu, env, 4, 8, 64, items_a)
    if second == "hash":
        mb = hashprogs.NativeHash(gpu, env, 4, 8, 64, items_b)
    else:
        mb = gpu.Map(env, 16, 8)
        mb.fill(arr)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [ma.handle, mb.handle]))
    try:
        gpu.set_variant(variant)
        got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        np.testing.assert_array_equal(gf, wf)
        np.testing.assert_array_equal(got, want)
        assert (wf == 10).any() == (sel_mask == 3)
    finally:
        gpu.set_variant(0)
        p.destroy()
        ma.destroy()
        mb.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("ks,src,stride", [(300, "stack", 512), (600, "packet", 1024),
                                           (257, "packet", 320)])
def test_hash_long_keys(gpu, env, variant, ks, src, stride):
    """Keys of hundreds of bytes (device slots of 512 B to 1 KB): on the stack and in the packet."""
    rng = np.random.default_rng(ks)
    items, keys = hashprogs.make_table(rng, ks, 8, 24)
    n = 1024
    pk = hashprogs.packets_with_keys(rng, n, stride, keys, 8, ks)
    lay = hashprogs.lookup_program(ks, src, key_off=8)
    spec = pyoracle.HashSpec(ks, 8, items=items)
    want, wf, _ = hashprogs.oracle(lay, [spec], pk.reshape(-1), n, stride)
    got, gf = run_device(gpu, env, lay, [spec], pk.reshape(-1), n, stride, variant=variant)
    np.testing.assert_array_equal(gf, wf)
    np.testing.assert_array_equal(got, want)
    assert (want != 0xdead).any() and (want == 0xdead).any()


def _forward_alias_program():
    """Hashtable value forwarding (asm_cc.cpp AHF_HLOOKUP) must not reuse a register whose value
    another name still reaches: r7 is dead after the lookup as a register, but the key's stack
    word was stored from it and a later stack load is forwarded from r7.  Reusing r7 for the
    probe's value bytes dropped that forwarding in the final pass only, so the exit the
    liveness pass had proven constant read a register it had removed the code for (fuzz_gpu.py
    --hash case 126, shrunk)."""
    I, Branch, LdDw, MapRef, assemble = hashprogs._mods()
    R0, R1, R2, R3, R6, R7, R8, R9, R10 = 0, 1, 2, 3, 6, 7, 8, 9, 10
    nodes = [
        I("ldxb", R8, R1, 3), I("ldxb", R9, R1, 4),   # live across the lookup
        I("mov_imm", R7, imm=3), I("stxw", R10, R7, -4),
        LdDw(R1, MapRef(0)),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
        I("call", imm=0),
        Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=1), I("exit")]),
        I("ldxb", R6, R0, 5),
        Branch(I("jeq_reg", R8, R9), [I("mov_reg", R0, R6), I("exit")]),
        # r0 = a constant + the key's low byte, read back through the stack (forwarded from r7)
        I("mov_imm", R0, imm=0x5bd1e995), I("ldxb", R3, R10, -4), I("add64_reg", R0, R3),
        I("exit"),
    ]
    return assemble(nodes)


@pytest.mark.parametrize("variant", VARIANTS)
def test_hash_forwarding_register_alias(gpu, env, variant):
    lay = _forward_alias_program()
    rng = np.random.default_rng(126)
    items = [(int(k).to_bytes(4, "little"), rng.bytes(8)) for k in range(8) if k != 5]
    spec = pyoracle.HashSpec(4, 8, items=items, capacity=16)
    n = 777
    pk = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    pk[::3, 4] = pk[::3, 3]   # both exits taken
    want, wf, _ = hashprogs.oracle(lay, [spec], pk.reshape(-1), n, 64)
    got, gf = run_device(gpu, env, lay, [spec], pk.reshape(-1), n, 64, variant=variant, max_entries=16)
    assert not wf.any()
    assert np.array_equal(wf, gf)
    assert np.array_equal(want, got), int((want != got).sum())
