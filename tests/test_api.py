"""Re-expression of the reference's own API tests (tests/ebpf_prog_tests/prog_load_test.cpp,
tests/ebpf_map_tests/{map_*,array_map_*}_test.cpp) against the engine's libebpf.so, plus the
drop-in ABI: struct layouts and every exported symbol the headers declare."""
import os
import ctypes
import errno
import struct

import pytest

from generic_ebpf_amd import isa


def test_exports_every_declared_symbol(native):
    L = native.lib()
    for name in native.FUNCS:
        assert hasattr(L, name), name
    for name in native.DATA_SYMBOLS:
        assert native.addr_of(name) != 0, name
    hdr = open(native.HERE + "/../include/ebpf.h").read() + \
        open(native.HERE + "/../include/ebpf_gpu.h").read()
    import re
    declared = set(re.findall(r"^\w[\w \*]*?\b(ebpf_\w+)\(", hdr, re.M))
    assert declared <= set(native.FUNCS), declared - set(native.FUNCS)


def test_exports_nothing_else(native):
    """The dynamic symbol table holds exactly the headers' functions and data symbols
    (generic-ebpf_amd/libebpf.map): no embedded code objects, no C++ runtime instantiations."""
    import subprocess
    path = os.path.join(native.HERE, "lib", "libebpf.so")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    # (+ ebpf_prog_attach_map: not in the public header, but the reference's libebpf.so exports
    # it, sys/dev/ebpf/ebpf_prog.c:84-109)
    want = set(native.FUNCS) | set(native.DATA_SYMBOLS) | {"ebpf_prog_attach_map"}
    assert exported == want, exported ^ want


def test_abi_layouts(native):
    assert ctypes.sizeof(native.ProgAttr) == 32
    assert native.ProgAttr.prog_len.offset == 16 and native.ProgAttr.data.offset == 24
    assert ctypes.sizeof(native.MapAttr) == 20
    assert ctypes.sizeof(native.Config) == 1544
    assert native.Config.helper_types.offset == 1024
    assert native.Config.preprocessor_type.offset == 1536
    # emt_* = name[64] + 9 function pointers; eht_* = name[64] + fn
    assert ctypes.c_char.in_dll(native.lib(), "emt_array")
    assert ctypes.string_at(native.addr_of("emt_array")) == b"array"
    assert ctypes.string_at(native.addr_of("eht_map_lookup_elem")) == b"map_lookup_elem"


# ---- prog_load_test.cpp:29-103 ----------------------------------------------------------
EXIT = isa.encode(isa.OPS["exit"])


def _create(native, env_ptr, epp, type_, prog, plen):
    buf = ctypes.create_string_buffer(prog, max(len(prog), 1)) if prog is not None else None
    attr = native.ProgAttr(type_, ctypes.addressof(buf) if buf is not None else None, plen, None)
    return native.lib().ebpf_prog_create(env_ptr, epp, ctypes.byref(attr))


def test_load_with_null_prog_pointer(native, env):
    assert _create(native, env.ptr, None, 0, EXIT, 1) == errno.EINVAL


@pytest.mark.parametrize("t", [64, 65])
def test_load_with_invalid_prog_type(native, env, t):
    ep = ctypes.c_void_p()
    assert _create(native, env.ptr, ctypes.byref(ep), t, EXIT, 1) == errno.EINVAL


def test_load_with_zero_len(native, env):
    ep = ctypes.c_void_p()
    assert _create(native, env.ptr, ctypes.byref(ep), 0, EXIT, 0) == errno.EINVAL


def test_load_with_null_prog(native, env):
    ep = ctypes.c_void_p()
    assert _create(native, env.ptr, ctypes.byref(ep), 0, None, 1) == errno.EINVAL


def test_correct_load_and_env_busy(native, env):
    ep = ctypes.c_void_p()
    assert _create(native, env.ptr, ctypes.byref(ep), 0, EXIT, 1) == 0
    assert native.lib().ebpf_env_destroy(env.ptr) == errno.EBUSY  # ebpf_env.c:44-45
    native.lib().ebpf_prog_destroy(ep)


def test_unset_prog_type(native, env):
    ep = ctypes.c_void_p()
    assert _create(native, env.ptr, ctypes.byref(ep), 5, EXIT, 1) == errno.EINVAL


# ---- map_create_test.cpp ----------------------------------------------------------------
def _map_create(native, env, attr, null_out=False):
    em = ctypes.c_void_p()
    err = native.lib().ebpf_map_create(env.ptr, None if null_out else ctypes.byref(em),
                                       ctypes.byref(attr))
    if err == 0:
        native.lib().ebpf_map_destroy(em)
    return err


@pytest.mark.parametrize("attr,null_out", [
    ((0, 4, 4, 100), True), ((64, 4, 4, 100), False), ((65, 4, 4, 100), False),
    ((0, 0, 4, 100), False), ((0, 4, 0, 100), False), ((0, 4, 4, 0), False)])
def test_map_create_invalid(native, env, attr, null_out):
    a = native.MapAttr(*attr, 0)
    assert _map_create(native, env, a, null_out) == errno.EINVAL


def test_map_create_ok(native, env):
    assert _map_create(native, env, native.MapAttr(0, 4, 4, 100, 0)) == 0


@pytest.fixture()
def amap(native, env):
    m = native.Map(env, 100, 4)
    yield m
    m.destroy()


# ---- map_lookup_test.cpp / map_update_test.cpp / map_delete_test.cpp / get_next_key --------
def test_lookup_null_map(native, amap):
    k = ctypes.c_uint32(50)
    assert native.lib().ebpf_map_lookup_elem(None, ctypes.byref(k)) is None


def test_lookup_null_key(native, amap):
    assert native.lib().ebpf_map_lookup_elem(amap.ptr, None) is None


def test_lookup_past_max(native, amap):
    k = ctypes.c_uint32(100)
    assert native.lib().ebpf_map_lookup_elem(amap.ptr, ctypes.byref(k)) is None


def test_update_invalid_args(native, amap):
    L = native.lib()
    k, v = ctypes.c_uint32(1), ctypes.c_uint32(1)
    assert L.ebpf_map_update_elem(None, ctypes.byref(k), ctypes.byref(v), 0) == errno.EINVAL
    assert L.ebpf_map_update_elem(amap.ptr, None, ctypes.byref(v), 0) == errno.EINVAL
    assert L.ebpf_map_update_elem(amap.ptr, ctypes.byref(k), None, 0) == errno.EINVAL
    assert L.ebpf_map_update_elem(amap.ptr, ctypes.byref(k), ctypes.byref(v), 3) == errno.EINVAL


def test_delete_invalid_args(native, amap):
    k = ctypes.c_uint32(100)
    assert native.lib().ebpf_map_delete_elem(None, ctypes.byref(k)) == errno.EINVAL
    assert native.lib().ebpf_map_delete_elem(amap.ptr, None) == errno.EINVAL


def test_get_next_key_args(native, amap):
    L = native.lib()
    k, nk = ctypes.c_uint32(50), ctypes.c_uint32(0)
    assert L.ebpf_map_get_next_key_from_user(None, ctypes.byref(k), ctypes.byref(nk)) == errno.EINVAL
    assert L.ebpf_map_get_next_key_from_user(amap.ptr, None, ctypes.byref(nk)) != errno.EINVAL
    assert L.ebpf_map_get_next_key_from_user(amap.ptr, ctypes.byref(k), None) == errno.EINVAL


# ---- array_map_*_test.cpp -----------------------------------------------------------------
def test_array_delete(native, amap):
    k = ctypes.c_uint32(50)
    assert amap.update(50, struct.pack("<I", 100)) == 0
    assert native.lib().ebpf_map_delete_elem_from_user(amap.ptr, ctypes.byref(k)) == errno.EINVAL


def test_array_get_next_key(native, amap):
    L = native.lib()
    nk = ctypes.c_uint32(7)
    k = ctypes.c_uint32(99)
    assert L.ebpf_map_get_next_key_from_user(amap.ptr, ctypes.byref(k), ctypes.byref(nk)) == errno.ENOENT
    assert L.ebpf_map_get_next_key_from_user(amap.ptr, None, ctypes.byref(nk)) == 0 and nk.value == 0
    k = ctypes.c_uint32(50)
    assert L.ebpf_map_get_next_key_from_user(amap.ptr, ctypes.byref(k), ctypes.byref(nk)) == 0
    assert nk.value == 51


def test_array_lookup_from_user(native, env):
    m = native.Map(env, 100, 8)
    try:
        assert m.update(50, struct.pack("<Q", 100)) == 0
        assert m.lookup(100)[0] == errno.EINVAL
        assert m.lookup(102)[0] == errno.EINVAL
        err, v = m.lookup(50)
        assert err == 0 and struct.unpack("<Q", v)[0] == 100
    finally:
        m.destroy()


def test_array_update(native, amap):
    assert amap.update(100, struct.pack("<I", 100)) == errno.EINVAL
    assert amap.update(50, struct.pack("<I", 100)) == 0
    assert amap.update(50, struct.pack("<I", 101)) == 0
    for i in range(100):
        assert amap.update(i, struct.pack("<I", 100)) == 0
    assert amap.update(100, struct.pack("<I", 100)) == errno.EINVAL
    assert amap.update(50, struct.pack("<I", 100), flags=1) == errno.EEXIST


def test_percpu_array_roundtrip(native, env):
    import os
    m = native.Map(env, 10, 8, type=native.MAP_TYPE_PERCPU_ARRAY)
    try:
        assert m.update(3, struct.pack("<Q", 77)) == 0
        ncpu = os.sysconf("SC_NPROCESSORS_ONLN")
        k = ctypes.c_uint32(3)
        buf = ctypes.create_string_buffer(8 * ncpu)
        assert native.lib().ebpf_map_lookup_elem_from_user(m.ptr, ctypes.byref(k), buf) == 0
        assert set(struct.unpack("<%dQ" % ncpu, buf.raw)) == {77}
    finally:
        m.destroy()



def test_time_next_launch_argument_checks(native):
    """ebpf_gpu_time_next_launch (include/ebpf_gpu.h): both events or neither; no HIP call."""
    L = native.lib()
    assert L.ebpf_gpu_time_next_launch(ctypes.c_void_p(16), None) == errno.EINVAL
    assert L.ebpf_gpu_time_next_launch(None, ctypes.c_void_p(16)) == errno.EINVAL
    assert L.ebpf_gpu_time_next_launch(None, None) == 0


def test_batch_flags_validation(native, env):
    """batch->flags: only EBPF_BATCH_HIST_OVERWRITE, and only on the device entry point; the
    check comes before any device work, so it holds without a GPU."""
    from generic_ebpf_amd import isa
    code = isa.encode(isa.OPS["mov_imm"], 0, imm=1) + isa.encode(isa.OPS["exit"])
    p = native.Prog(env, code)
    try:
        L = native.lib()
        bad = native.PktBatch(16, None, 1, 64, 0x2)
        assert L.ebpf_prog_run_batch_dev(p.ptr, 0, ctypes.byref(bad), 16, None, None,
                                         None) == errno.EINVAL
        host = native.PktBatch(16, None, 1, 64, native.BATCH_HIST_OVERWRITE)
        ret = (ctypes.c_uint64 * 1)()
        assert L.ebpf_prog_run_batch(p.ptr, ctypes.byref(host), ret, None, None) == errno.EINVAL
    finally:
        p.destroy()


def test_bench_issue_roofline():
    """bench.py's VALU-issue roofline (general kernels): SQ_INSTS_VALU x 4 cycles over 1,024
    SIMDs at 2.4 GHz, per group and as a fraction of the kernel time."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    r = b.issue_roofline({"SQ_INSTS_VALU": 1024 * 2.4e6 / 4, "SQ_INSTS_SALU": 100.0,
                          "SQ_INSTS_VMEM_RD": 10.0}, kern_ms=2.0, groups=10)
    assert r["bound"] == "valu-issue" and abs(r["floor_ms"] - 1.0) < 1e-9
    assert r["frac"] == 0.5 and r["salu_per_group"] == 10.0 and r["vmem_rd_per_group"] == 1.0
    assert b.issue_roofline({}, 1.0, 1) is None
