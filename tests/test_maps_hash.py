"""Hashtable and percpu-hashtable maps through the C-ABI (host side).

Re-expresses the reference's tests/ebpf_map_tests/{,percpu_}hashtable_map_*_test.cpp and checks
the things those tests leave open against the oracle's model of
sys/dev/ebpf/ebpf_map_hashtable.c (oracle/pyoracle.py HashtableModel): the exact get_next_key
order (which pins the bucket hash, jhash), replacement moving a key to the head of its bucket,
EBUSY at capacity, the spare-element swap, and programs doing hashtable lookups through
ebpf_prog_run.  Device batches reject programs that load a hashtable (EOPNOTSUPP).
"""
import ctypes
import errno
import os
import struct
import subprocess

import numpy as np
import pytest

import pyoracle

HT, PHT = 2, 3
NCPU = os.sysconf("SC_NPROCESSORS_ONLN")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "maps", "jhash.npz")


class HMap:
    """Byte-keyed view of one map (key/value sizes as created)."""

    def __init__(self, native, env, type, key_size, value_size, max_entries):
        self.native, self.ks, self.vs = native, key_size, value_size
        self.percpu = type == PHT
        self.ptr = ctypes.c_void_p()
        attr = native.MapAttr(type, key_size, value_size, max_entries, 0)
        rc = native.lib().ebpf_map_create(env.ptr, ctypes.byref(self.ptr), ctypes.byref(attr))
        assert rc == 0, rc
        self.L = native.lib()

    def update(self, key, value, flags=0):
        k = ctypes.create_string_buffer(key, self.ks)
        v = ctypes.create_string_buffer(value, self.vs)
        return self.L.ebpf_map_update_elem_from_user(self.ptr, k, v, flags)

    def lookup(self, key):
        k = ctypes.create_string_buffer(key, self.ks)
        n = self.vs * (NCPU if self.percpu else 1)
        v = ctypes.create_string_buffer(n)
        rc = self.L.ebpf_map_lookup_elem_from_user(self.ptr, k, v)
        if rc:
            return rc, None
        if self.percpu:
            return 0, [v.raw[i * self.vs:(i + 1) * self.vs] for i in range(NCPU)]
        return 0, v.raw

    def delete(self, key):
        return self.L.ebpf_map_delete_elem_from_user(self.ptr, ctypes.create_string_buffer(key, self.ks))

    def next_key(self, key):
        out = ctypes.create_string_buffer(self.ks)
        k = None if key is None else ctypes.create_string_buffer(key, self.ks)
        rc = self.L.ebpf_map_get_next_key_from_user(self.ptr, k, out)
        return rc, (out.raw if rc == 0 else None)

    def walk(self):
        keys, rc, k = [], 0, None
        while True:
            rc, k = self.next_key(k)
            if rc:
                assert rc == errno.ENOENT
                return keys
            keys.append(k)
            assert len(keys) <= 1 << 20

    def destroy(self):
        self.L.ebpf_map_destroy(self.ptr)


@pytest.fixture(params=[HT, PHT], ids=["hashtable", "percpu_hashtable"])
def hmap(request, native, env):
    m = HMap(native, env, request.param, 4, 4, 100)
    yield m
    m.destroy()


def u32(x):
    return struct.pack("<I", x)


# ---- jhash: the oracle's restatement against vectors from the reference's own header ----

def test_oracle_jhash_matches_reference_vectors():
    z = np.load(GOLDEN)
    d, o = z["data"].tobytes(), z["offsets"]
    for i in range(len(o) - 1):
        assert pyoracle.jhash(d[o[i]:o[i + 1]], int(z["initval"][i])) == int(z["expect"][i]), i


def test_oracle_c_jhash_matches_reference_vectors():
    z = np.load(GOLDEN)
    d, o = z["data"].tobytes(), z["offsets"]
    L = pyoracle.lib()
    for i in range(len(o) - 1):
        k = d[o[i]:o[i + 1]]
        assert L.oracle_jhash(k, len(k), int(z["initval"][i])) == int(z["expect"][i]), i


def test_product_jhash_header_matches_reference_vectors(tmp_path):
    """csrc/jhash.h (shared by host maps and device code) compiled on its own, every golden
    vector at its recorded misalignment."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "t.cpp"
    src.write_text(
        '#include "jhash.h"\n#include <cstdio>\n#include <cstring>\n#include <cstdlib>\n'
        'int main(){unsigned init,off;char hex[1024];static unsigned char buf[600];\n'
        'while(scanf("%u %u %1023s",&init,&off,hex)==3){size_t n=0;\n'
        'if(strcmp(hex,"-"))for(;hex[2*n];n++){unsigned b;sscanf(hex+2*n,"%2x",&b);buf[off+n]=b;}\n'
        'printf("%u\\n",ebpf_jhash(buf+off,n,init));}}\n')
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "generic-ebpf_amd", "csrc"),
                           str(src), "-o", str(exe)])
    z = np.load(GOLDEN)
    d, o = z["data"].tobytes(), z["offsets"]
    lines = ["%d %d %s" % (int(z["initval"][i]), int(z["misalign"][i]), d[o[i]:o[i + 1]].hex() or "-")
             for i in range(len(o) - 1)]
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split()
    assert [int(x) for x in out] == [int(x) for x in z["expect"]]


# ---- the reference's map tests (hashtable_map_*_test.cpp, percpu_hashtable_map_*_test.cpp) ----

def test_correct_update(hmap):
    assert hmap.update(u32(50), u32(100)) == 0


def test_update_more_than_max_entries(hmap):
    for i in range(100):
        assert hmap.update(u32(i), u32(i)) == 0
    assert hmap.update(u32(100), u32(100)) == errno.EBUSY
    # replacing an existing key at capacity still works (spare element / in place)
    assert hmap.update(u32(7), u32(70)) == 0
    rc, v = hmap.lookup(u32(7))
    assert rc == 0 and (v == [u32(70)] * NCPU if hmap.percpu else v == u32(70))


def test_update_flags(hmap):
    assert hmap.update(u32(50), u32(100), pyoracle.EBPF_EXIST) == errno.ENOENT
    assert hmap.update(u32(50), u32(100), pyoracle.EBPF_NOEXIST) == 0
    assert hmap.update(u32(50), u32(100), pyoracle.EBPF_NOEXIST) == errno.EEXIST
    assert hmap.update(u32(50), u32(101), pyoracle.EBPF_EXIST) == 0
    rc, v = hmap.lookup(u32(50))
    assert rc == 0 and (v == [u32(101)] * NCPU if hmap.percpu else v == u32(101))


def test_lookup(hmap):
    assert hmap.update(u32(50), u32(100)) == 0
    assert hmap.lookup(u32(51)) == (errno.ENOENT, None)
    rc, v = hmap.lookup(u32(50))
    assert rc == 0
    assert v == ([u32(100)] * NCPU if hmap.percpu else u32(100))


def test_delete(hmap):
    assert hmap.delete(u32(50)) == 0          # absent key: still 0
    assert hmap.update(u32(50), u32(1)) == 0
    assert hmap.delete(u32(50)) == 0
    assert hmap.lookup(u32(50))[0] == errno.ENOENT
    assert hmap.walk() == []


def test_get_first_key(hmap):
    assert hmap.next_key(None) == (errno.ENOENT, None)
    assert hmap.update(u32(100), u32(200)) == 0
    assert hmap.next_key(None) == (0, u32(100))


def test_get_next_key_walks_every_key_in_reference_order(hmap):
    model = pyoracle.HashtableModel(100, percpu=hmap.percpu, ncpu=NCPU)
    for i in range(100):
        assert hmap.update(u32(i), u32(i)) == 0
        assert model.update(u32(i), u32(i)) == 0
    got = hmap.walk()
    assert sorted(got) == sorted(u32(i) for i in range(100))
    assert got == model.keys_in_order()
    # an absent key restarts from the first bucket (:518-520)
    assert hmap.next_key(u32(12345)) == model.get_next_key(u32(12345))


@pytest.mark.parametrize("key_size,max_entries,seed", [(1, 200, 1), (3, 50, 2), (8, 1000, 3),
                                                       (13, 300, 4), (40, 64, 5)])
def test_random_operations_match_model(native, env, key_size, max_entries, seed):
    """Random update/delete/lookup streams (flags included), then the full get_next_key walk:
    return codes, values and iteration order all equal the model's."""
    rng = np.random.default_rng(seed)
    for typ in (HT, PHT):
        m = HMap(native, env, typ, key_size, 12, max_entries)
        model = pyoracle.HashtableModel(max_entries, percpu=typ == PHT, ncpu=NCPU)
        universe = [rng.integers(0, 256, key_size, dtype=np.uint8).tobytes()
                    for _ in range(min(256 ** key_size, max_entries * 2))]
        try:
            for step in range(max_entries * 4):
                k = universe[int(rng.integers(0, len(universe)))]
                op = int(rng.integers(0, 10))
                if op < 6:
                    v = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
                    fl = int(rng.integers(0, 3))
                    assert m.update(k, v, fl) == model.update(k, v, fl), step
                elif op < 8:
                    assert m.delete(k) == model.delete(k) == 0
                else:
                    rc, v = m.lookup(k)
                    mv = model.lookup(k)
                    assert (rc == 0) == (mv is not None)
                    if mv is not None:
                        assert v == mv
            assert m.walk() == model.keys_in_order()
        finally:
            m.destroy()


def test_percpu_hashtable_reuses_elements_lifo(native, env):
    """A deleted element goes back to the head of the free list and is the next one allocated
    (ebpf_allocator.c:80-144): observable as a fresh key inheriting nothing but working."""
    m = HMap(native, env, PHT, 4, 8, 4)
    try:
        for i in range(4):
            assert m.update(u32(i), struct.pack("<Q", i)) == 0
        assert m.update(u32(9), struct.pack("<Q", 9)) == errno.EBUSY
        assert m.delete(u32(2)) == 0
        assert m.update(u32(9), struct.pack("<Q", 9)) == 0
        assert m.lookup(u32(9)) == (0, [struct.pack("<Q", 9)] * NCPU)
        assert m.update(u32(10), struct.pack("<Q", 9)) == errno.EBUSY
    finally:
        m.destroy()


def test_hashtable_create_limits(native, env):
    em = ctypes.c_void_p()
    big = native.MapAttr(HT, 0xfffffff0, 0x10, 4, 0)       # key + value + linkage > UINT32_MAX
    assert native.lib().ebpf_map_create(env.ptr, ctypes.byref(em), ctypes.byref(big)) == errno.E2BIG


# ---- programs using a hashtable ----

def _lookup_prog(native):
    """r0 = value(u32 at packet[0]) or 0xdead when absent — through helper 0 (map_lookup_elem)."""
    from generic_ebpf_amd import isa
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef, assemble
    I = isa.Insn
    nodes = [I("ldxw", 6, 1, 0), I("stxw", 10, 6, -4), LdDw(1, MapRef(0)),
             I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
             Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=0xdead), I("exit")]),
             I("ldxdw", 0, 0, 0), I("exit")]
    return assemble(nodes)


@pytest.mark.parametrize("typ", [HT, PHT], ids=["hashtable", "percpu_hashtable"])
def test_prog_run_with_hashtable_lookup(native, env, typ):
    m = HMap(native, env, typ, 4, 8, 64)
    p = None
    try:
        for k in range(0, 64, 2):
            assert m.update(u32(k * 1000), struct.pack("<Q", k * 7 + 1)) == 0
        lay = _lookup_prog(native)
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.ptr.value]))
        for k in range(64):
            r, _ = p.run_cpu(u32(k * 1000) + bytes(60))
            assert r == (k * 7 + 1 if k % 2 == 0 else 0xdead), k
    finally:
        if p is not None:
            p.destroy()
        m.destroy()


def test_device_translation_of_hashtable_programs(native, env):
    """Hashtable lookups translate for the device (both code layouts compile): a statically
    known map, percpu hashtables, keys of hundreds of bytes, and lookups whose map is known only
    at run time (a compare chain on r1 over the program's hashtables).  Keys over 65535 bytes
    have no device form (EOPNOTSUPP; the program still runs through ebpf_prog_run)."""
    from generic_ebpf_amd import isa
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef, assemble
    I = isa.Insn
    ht = HMap(native, env, HT, 4, 8, 64)
    pht = HMap(native, env, PHT, 4, 8, 64)
    progs, extra = [], []
    try:
        lay = _lookup_prog(native)
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [ht.ptr.value]))
        progs.append(p)
        i = native.DprogInfo()
        assert native.lib().ebpf_prog_device_info(p.ptr, ctypes.byref(i)) == 0
        assert i.nmaps == 1
        for layout in (0, 1):
            assert len(p.device_code(layout)) > 0
        p2 = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [pht.ptr.value]))
        progs.append(p2)
        assert native.lib().ebpf_prog_device_info(p2.ptr, ctypes.byref(i)) == 0   # percpu: the caller's CPU copy
        big = HMap(native, env, HT, 300, 8, 4)      # long keys: slots of 512 bytes
        extra.append(big)
        p4 = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [big.ptr.value]))
        progs.append(p4)
        assert native.lib().ebpf_prog_device_info(p4.ptr, ctypes.byref(i)) == 0
        huge = HMap(native, env, HT, 65536, 8, 2)   # past the device table's key-size field
        extra.append(huge)
        p5 = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [huge.ptr.value]))
        progs.append(p5)
        assert native.lib().ebpf_prog_device_info(p5.ptr, ctypes.byref(i)) == errno.EOPNOTSUPP
        assert "no device form" in native.last_error()
        # r1 = the hashtable's handle plus a packet byte: resolved at run time
        nodes = [I("ldxw", 6, 1, 0), I("stxw", 10, 6, -4), I("ldxb", 7, 1, 4), LdDw(1, MapRef(0)),
                 I("add64_reg", 1, 7), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                 I("call", imm=0), I("exit")]
        lay3 = assemble(nodes)
        p3 = native.Prog(env, native.patch_relocs(lay3.code, lay3.relocs, [ht.ptr.value]))
        progs.append(p3)
        assert native.lib().ebpf_prog_device_info(p3.ptr, ctypes.byref(i)) == 0
        for layout in (0, 1):
            assert len(p3.device_code(layout)) > 0
    finally:
        for p in progs:
            p.destroy()
        ht.destroy()
        pht.destroy()
        for m in extra:
            m.destroy()


# ---- the oracle's hashtable lookups against the CPU path (ebpf_prog_run over the host table) ----

HCASES = [  # (ks, vs, key source, key offset, read (size, off), store, second map)
    (4, 8, "stack", 0, (8, 0), False, None),
    (1, 8, "stack", 5, (4, 4), False, None),
    (3, 16, "packet", 7, (8, 8), False, None),
    (8, 8, "stack", 2, (2, 6), False, None),
    (13, 12, "packet", 20, (4, 8), False, None),
    (16, 8, "stack", 16, (8, 0), False, (4, 40)),
    (40, 24, "stack", 0, (8, 16), False, None),
    (4, 8, "stack", 0, (8, 4), False, None),      # crosses the value end: fault
    (4, 8, "null", 0, (8, 0), False, None),       # NULL key: r0 = NULL
    (8, 8, "packet", 60, (8, 0), False, None),    # key runs off the packet: fault
]


def hcase(k, rng, n=128, size=64):
    import hashprogs
    ks, vs, src, off, read, store, second = HCASES[k]
    items, keys = hashprogs.make_table(rng, ks, vs, 40)
    lay = hashprogs.lookup_program(ks, src, off, read=read, store=store, second=second)
    specs = [pyoracle.HashSpec(ks, vs, items)]
    if second:
        items2, keys2 = hashprogs.make_table(rng, second[0], 8, 30)
        specs.append(pyoracle.HashSpec(second[0], 8, items2))
    pk = hashprogs.packets_with_keys(rng, n, size, keys, min(off, size - ks), ks)
    if second:
        pk2 = hashprogs.packets_with_keys(rng, n, size, keys2, second[1], second[0])
        pk[:, second[1]:second[1] + second[0]] = pk2[:, second[1]:second[1] + second[0]]
    return lay, specs, pk


@pytest.mark.parametrize("k", range(len(HCASES)))
def test_oracle_hash_lookups_match_cpu_path(native, env, k):
    import hashprogs
    rng = np.random.default_rng(100 + k)
    lay, specs, pk = hcase(k, rng)
    want, wf, _ = hashprogs.oracle(lay, specs, pk.reshape(-1), len(pk), pk.shape[1])
    maps = [hashprogs.NativeHash(native, env, s.key_size, s.value_size, 64, s.items) for s in specs]
    p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        for i in range(len(pk)):
            if wf[i]:
                continue      # (the reference's behaviour there is a crash or a stray read)
            r, _ = p.run_cpu(pk[i].tobytes())
            assert r == int(want[i]), (i, hex(r), hex(int(want[i])))
        if HCASES[k][2] != "null" and k != 7 and k != 9:
            assert not wf.any()
            assert (want != 0xdead).any() and (want == 0xdead).any()   # hits and misses
        if k in (7, 9):
            assert wf.any()
    finally:
        p.destroy()
        for m in maps:
            m.destroy()
