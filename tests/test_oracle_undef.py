"""The oracle's track_undef mode (test tooling for the fuzz shrinker and the mutation fuzzer,
oracle/ebpf_oracle.c taint_pre): a result that depends on the reference's uninitialised stack or
on an address faults with code 100; defined programs run as before."""
import numpy as np

import pyoracle
from generic_ebpf_amd import isa

E = isa.encode


def _run(code, relocs=(), maps=()):
    pk = np.zeros((4, 64), dtype=np.uint8)
    op = pyoracle.OracleProgram(code, list(relocs), list(maps), track_undef=True)
    return op.run(pk.reshape(-1), 4, 64)[:2]


def test_defined_program_unchanged():
    # r0 = 7; r0 += pkt[3]; exit  (slots 0, 1, 3 under the reference's stepping)
    code = b"".join([E(0xb4, 0, 0, 0, 7), E(0x71, 2, 1, 3, 0), E(0xb4, 9, 0, 0, 1),
                     E(0x0f, 0, 2, 0, 0), E(0xb4, 9, 0, 0, 1), E(0xb4, 9, 0, 0, 1), E(0x95)])
    ret, faults = _run(code)
    assert not faults.any() and (ret == 7).all()


def test_uninitialised_stack_read():
    # r0 = *(u32 *)(r10 - 4) without a store: undefined
    code = b"".join([E(0x61, 0, 10, -4, 0), E(0x95), E(0x95)])
    ret, faults = _run(code)
    assert (faults == 100).all()


def test_stored_then_read_is_defined():
    # *(u32 *)(r10 - 4) = 9; r0 = *(u32 *)(r10 - 4)
    code = b"".join([E(0x62, 10, 0, -4, 9), E(0x61, 0, 10, -4, 0), E(0xb4, 9, 0, 0, 1), E(0x95)])
    ret, faults = _run(code)
    assert not faults.any() and (ret == 9).all()


def test_address_result():
    # r0 = r10 (MOV64 adds in the reference: r0 = 0 + r10); exit with an address
    code = b"".join([E(0xbf, 0, 10, 0, 0), E(0x95), E(0x95)])
    ret, faults = _run(code)
    assert (faults == 100).all()


def test_address_difference_is_defined():
    # r2 = r10; r2 -= r10 (an address minus an address); r0 += r2 -> 0
    code = b"".join([E(0xbf, 2, 10, 0, 0), E(0x1f, 2, 10, 0, 0), E(0xb4, 9, 0, 0, 1),
                     E(0x0f, 0, 2, 0, 0), E(0xb4, 9, 0, 0, 1), E(0xb4, 9, 0, 0, 1), E(0x95)])
    ret, faults = _run(code)
    assert not faults.any() and (ret == 0).all()


def test_wrapping_address_faults_mem():
    # r2 = -4 (all ones but the low bits); r0 = *(u64 *)(r2 + 0): an access whose end wraps past
    # 2^64 is no region's (MEM), in the shadow bookkeeping too (it crashed the tracker once)
    code = b"".join([E(0xb7, 2, 0, 0, -4), E(0x79, 0, 2, 0, 0), E(0xb4, 9, 0, 0, 1), E(0x95)])
    pk = np.zeros((4, 64), dtype=np.uint8)
    for sem in (0, 1):
        op = pyoracle.OracleProgram(code, [], [], track_undef=True, semantics=sem)
        ret, faults = op.run(pk.reshape(-1), 4, 64)[:2]
        assert (faults == 3).all()
