"""Counter updates through a PACKET pointer: the translator fuses
`LDX X = [r1 + off]; ADD X, y; STX [r1 + off] = X` into one counter-update entry and decodes
standard-semantics XADD to another, whatever the base register.  On the packet these are plain
read-modify-write stores (the reference writes the packet in place, ebpf_interpreter.c:343-366),
so a later load of the same word must read the new value: the program may not run in the staged
kernel (packet bytes copied into registers / LDS) nor with the general kernels' staged headers.

CPU: the oracle against hand-computed answers.  GPU: every variant, 64-B fixed-stride batches
(the staged kernel's shape) and CSR offsets batches (general kernels, short packets faulting
MEM), results, faults and packet bytes against the oracle."""
import os

import numpy as np
import pytest

import pyoracle
import stdprogs

R0, R1, R2, R3, R4, R5, R6, R7 = range(8)
VARIANTS = [int(v) for v in os.environ.get("EBPF_TEST_VARIANTS", "0,1,2").split(",")]


def _ref(nodes):
    from generic_ebpf_amd import layout
    lay = layout.assemble(nodes)
    return lay.code, lay.relocs


def prog_w32():
    """pkt[4..8) += 7 (32-bit), then r0 = the reloaded word + pkt[6] + pkt[40..44)."""
    from generic_ebpf_amd.isa import Insn as I
    return _ref([I("ldxw", R4, R1, 40), I("ldxw", R2, R1, 4), I("add_imm", R2, imm=7),
                 I("stxw", R1, R2, 4), I("ldxw", R0, R1, 4), I("ldxb", R3, R1, 6),
                 I("add64_reg", R0, R3), I("add64_reg", R0, R4), I("exit")])


def prog_dw64():
    """pkt[16..24) += pkt[0] (64-bit register addend), then r0 = the reloaded word ^ pkt[20..24)."""
    from generic_ebpf_amd.isa import Insn as I
    return _ref([I("ldxb", R5, R1, 0), I("ldxdw", R2, R1, 16), I("add64_reg", R2, R5),
                 I("stxdw", R1, R2, 16), I("ldxdw", R0, R1, 16), I("ldxw", R3, R1, 20),
                 I("xor64_reg", R0, R3), I("exit")])


def prog_xadd(width, fetch):
    """Standard semantics: XADD of pkt[1] into pkt[8..8 + width), then r0 = the reloaded word
    (+ the fetched old value)."""
    I = stdprogs.I
    op = 0xdb if width == 8 else 0xc3
    ld = "ldxdw" if width == 8 else "ldxw"
    items = [I("ldxb", 7, 1, 1), I("mov64_reg", 6, 7), (op, 1, 7, 8, 1 if fetch else 0),
             I(ld, 0, 1, 8)]
    if fetch:
        items.append(I("add64_reg", 0, 7))
    items.append(I("exit"))
    return stdprogs.asm(items)


def _u(b, at, w):
    return int.from_bytes(bytes(b[at:at + w]), "little")


def expect(name, pk):
    ret, after = [], pk.copy()
    for i, p in enumerate(pk):
        q = after[i]
        if name == "w32":
            x = (_u(p, 4, 4) + 7) & 0xffffffff
            q[4:8] = np.frombuffer(x.to_bytes(4, "little"), dtype=np.uint8)
            ret.append((x + int(q[6]) + _u(p, 40, 4)) & (2**64 - 1))
        elif name == "dw64":
            x = (_u(p, 16, 8) + int(p[0])) & (2**64 - 1)
            q[16:24] = np.frombuffer(x.to_bytes(8, "little"), dtype=np.uint8)
            ret.append(x ^ _u(q, 20, 4))
        else:
            w, fetch = int(name[4]), name.endswith("f")
            old = _u(p, 8, w)
            x = (old + int(p[1])) & ((1 << (8 * w)) - 1)
            q[8:8 + w] = np.frombuffer(x.to_bytes(w, "little"), dtype=np.uint8)
            ret.append((x + (old if fetch else 0)) & (2**64 - 1))
    return np.array(ret, dtype=np.uint64), after


PROGS = {"w32": (prog_w32, 0), "dw64": (prog_dw64, 0), "xadd4": (lambda: prog_xadd(4, False), 1),
         "xadd8": (lambda: prog_xadd(8, False), 1), "xadd8f": (lambda: prog_xadd(8, True), 1)}


def _packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


@pytest.mark.parametrize("name", sorted(PROGS))
def test_oracle_packet_counters_known_answers(name):
    mk, sem = PROGS[name]
    code, rel = mk()
    pk = _packets(1000, 31)
    op = pyoracle.OracleProgram(code, rel, [], semantics=sem)
    ret, faults, data, _ = op.run(pk.reshape(-1), len(pk), 64)
    want, after = expect(name, pk)
    assert not faults.any()
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(data.reshape(pk.shape), after)


def _offsets_batch(n, seed):
    """CSR packets of 9..79 bytes back to back: some end before the counter word (MEM)."""
    g = np.random.default_rng(seed)
    lens = g.integers(9, 80, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    return data, offs


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", sorted(PROGS))
@pytest.mark.parametrize("shape", ["stride64", "offsets"])
def test_device_packet_counters_vs_oracle(gpu, env, variant, name, shape):
    mk, sem = PROGS[name]
    code, rel = mk()
    n = (1 << 15) + 13
    if shape == "stride64":
        data, offs, stride = np.ascontiguousarray(_packets(n, 32).reshape(-1)), None, 64
    else:
        (data, offs), stride = _offsets_batch(n, 33), 0
    op = pyoracle.OracleProgram(code, rel, [], semantics=sem)
    want, wf, wdata, _ = op.run(data, n, stride, offs, nthreads=8)
    if shape == "offsets":
        assert wf.any() and (wf == 0).any()
    p = gpu.Prog(env, code)
    try:
        if sem:
            p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(variant)
        got_data = data.copy()
        ret, faults, _ = p.run_batch(got_data, n, stride, offs)
    finally:
        gpu.set_variant(0)
        p.destroy()
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(got_data, wdata)
