"""The CPU oracle is pinned to the GENUINE reference: every golden vector (generated from the
reference libebpf.so by tools/gen_golden.py) must reproduce bit for bit, r0 and packet bytes."""
import numpy as np
import pytest

import goldens
from helpers import oracle_run

CASES = [c for f in goldens.all_golden_files() for c in goldens.load(f)]


def test_golden_files_present():
    names = {c.name for c in CASES}
    assert {"c2", "c3", "c4", "c5", "kat_cumulative_pc"} <= names
    assert sum(1 for n in names if n.startswith("rand_")) >= 40


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_oracle_matches_reference(case):
    ret, faults, after, _ = oracle_run(case)
    assert not faults.any()
    np.testing.assert_array_equal(ret, case.expect_r0)
    np.testing.assert_array_equal(after, case.expect_data)


# SURVEY.md Appendix A known answers, as reproduced by the genuine reference (kat.npz).
KAT = {
    "kat_cumulative_pc": 2, "kat_mov64_adds": 8, "kat_neg32": 0xfffffff9,
    "kat_neg64": 0xfffffffffffffffe, "kat_arsh32_logical": 0x3ffffffc,
    "kat_lddw_arsh64": 0x0800000000000000, "kat_lsh32_mask": 2, "kat_lsh64_mask": 2,
    "kat_ja_fwd": 7, "kat_ja_back": 3, "kat_jeq_sext": 0xffffffff, "kat_ldxdw_be32": 0x122436,
    "kat_stdw_ldxb": 0xfe,
}


def test_known_answers():
    got = {c.name: int(c.expect_r0[0]) for c in CASES if c.name.startswith("kat_")}
    assert got == KAT


def test_oracle_fault_codes():
    """Undefined-in-the-reference behaviours map to the documented fault codes."""
    import pyoracle
    from generic_ebpf_amd import isa
    O = isa.OPS
    e = isa.encode
    pk = np.zeros(64, np.uint8)

    def run(code):
        op = pyoracle.OracleProgram(code)
        r, f, _, _ = op.run(pk, 1, 64)
        return int(f[0])

    assert run(e(O["mov_imm"], 0, imm=1) + e(O["div_imm"], 0, imm=0)) == 2
    assert run(e(0x06) + e(O["exit"])) == 1                                  # JMP32 class
    assert run(e(O["ldxw"], 0, 1, 62) + e(O["exit"])) == 3                   # past 64 B
    assert run(e(O["mov_imm"], 0, imm=1) + e(O["mov_imm"], 0, imm=2)) == 4   # falls off
    assert run(e(O["call"], imm=5) + e(O["exit"])) == 5                      # unset helper
    assert run(e(O["call"], imm=3) + e(O["exit"])) == 6                      # no device form
    assert run(e(O["mov_imm"], 12, imm=1) + e(O["exit"])) == 7               # r12
    assert run(e(O["ja"], off=-1) + e(O["exit"])) == 8                       # (0,1) self-loop
    from generic_ebpf_amd import layout
    bad_map = layout.assemble([layout.LdDw(1, 0x1234), isa.Insn("mov_imm", 2, imm=8),
                               isa.Insn("call", imm=0), isa.Insn("exit")]).code
    assert run(bad_map) == 10                                                # r1 not a map
