"""Programs, maps and packets for the hashtable-lookup parity tests (test infrastructure).

A case = a stepping-aware program (layout.assemble) that builds a key, calls
map_lookup_elem on a hashtable (helper 0, ebpf_map.c:77-84 -> ebpf_map_hashtable.c:285-301),
NULL-checks the result and reads the value; a seeded key universe half of which is in the map;
packets that carry one key each.  The oracle (oracle/pyoracle.py HashSpec) and the device run
the same case; the device map is a real hashtable built through the C-ABI."""
import ctypes

import numpy as np

import pyoracle

R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)


def _mods():
    from generic_ebpf_amd import isa
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef, assemble
    return isa.Insn, Branch, LdDw, MapRef, assemble


def key_nodes(ks, src, key_off, stk_off, I):
    """r2 = the key: copied from the packet to the stack, or a pointer into the packet, or NULL."""
    nodes = []
    if src == "stack":
        for b in range(ks):
            nodes += [I("ldxb", R7, R6, key_off + b), I("stxb", R10, R7, stk_off + b)]
        nodes += [I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=stk_off)]
    elif src == "packet":
        nodes += [I("mov_imm", R2, imm=0), I("mov64_reg", R2, R6), I("add64_imm", R2, imm=key_off)]
    elif src == "null":
        nodes += [I("mov_imm", R2, imm=0)]
    else:
        raise ValueError(src)
    return nodes


def lookup_program(ks, src="stack", key_off=0, stk_off=None, read=(8, 0), miss=0xdead,
                   store=False, second=None):
    """r0 = value bytes [read[1], read[1] + read[0]) of map 0's value for the packet's key, or
    `miss`.  store: write the packet's first 8 bytes into the value first (read back by the
    load: the packet's own store, ebpf_gpu.h "Stores into map values").  second:
    (ks2, key_off2) looks up map 1 too and XORs its first 8 value bytes in (or 0x77 on a miss)."""
    I, Branch, LdDw, MapRef, assemble = _mods()
    if stk_off is None:
        stk_off = -((ks + 7) & ~7)
    ldx = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[read[0]]
    nodes = [I("mov_imm", R6, imm=0), I("mov64_reg", R6, R1)]
    nodes += key_nodes(ks, src, key_off, stk_off, I)
    nodes += [LdDw(R1, MapRef(0)), I("call", imm=0),
              Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=miss), I("exit")])]
    if store:
        nodes += [I("ldxdw", R9, R6, 0), I("stxdw", R0, R9, 0)]
    nodes += [I(ldx, R8, R0, read[1])]
    if second is not None:
        ks2, off2 = second
        so2 = -64 - ((ks2 + 7) & ~7)
        nodes += key_nodes(ks2, "stack", off2, so2, I)
        nodes += [LdDw(R1, MapRef(1)), I("call", imm=0),
                  Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=0x77), I("exit")]),
                  I("ldxdw", R9, R0, 0), I("xor64_reg", R8, R9)]
    nodes += [I("mov_imm", R0, imm=0), I("mov64_reg", R0, R8), I("exit")]
    return assemble(nodes)


def make_table(rng, ks, vs, n_items, universe=None):
    """(items, universe): n_items (key, value) pairs and a key universe twice that size
    (distinct keys; the first n_items are the map's)."""
    u = universe or 2 * n_items
    keys, seen = [], set()
    space = 256 ** ks
    while len(keys) < min(u, space):
        k = rng.integers(0, 256, ks, dtype=np.uint8).tobytes()
        if k not in seen:
            seen.add(k)
            keys.append(k)
    items = [(k, rng.integers(0, 256, vs, dtype=np.uint8).tobytes()) for k in keys[:n_items]]
    return items, keys


def packets_with_keys(rng, n, size, keys, key_off, ks):
    pk = rng.integers(0, 256, (n, size), dtype=np.uint8)
    idx = rng.integers(0, len(keys), n)
    for i in range(n):
        pk[i, key_off:key_off + ks] = np.frombuffer(keys[idx[i]], dtype=np.uint8)
    return pk


class NativeHash:
    """A hashtable created and filled through the C-ABI."""

    def __init__(self, native, env, ks, vs, max_entries, items, type=2):
        self.L = native.lib()
        self.ks, self.vs = ks, vs
        self.ptr = ctypes.c_void_p()
        attr = native.MapAttr(type, ks, vs, max_entries, 0)
        rc = self.L.ebpf_map_create(env.ptr, ctypes.byref(self.ptr), ctypes.byref(attr))
        assert rc == 0, rc
        for k, v in items:
            self.update(k, v)

    def update(self, k, v, flags=0):
        rc = self.L.ebpf_map_update_elem_from_user(self.ptr, ctypes.create_string_buffer(k, self.ks),
                                                   ctypes.create_string_buffer(v, self.vs), flags)
        assert rc == 0, rc

    def delete(self, k):
        assert self.L.ebpf_map_delete_elem_from_user(self.ptr, ctypes.create_string_buffer(k, self.ks)) == 0

    @property
    def handle(self):
        return self.ptr.value

    def destroy(self):
        self.L.ebpf_map_destroy(self.ptr)


def oracle(lay, specs, data, count, stride, offsets=None):
    op = pyoracle.OracleProgram(lay.code, lay.relocs, specs)
    ret, faults, after, _ = op.run(data, count, stride, offsets, nthreads=4)
    return ret, faults, after
