"""Host-side translation (reference stepping → device program) and the stepping-aware
assembler.  No GPU needed: ebpf_prog_device_info only translates."""
import numpy as np

import goldens
from generic_ebpf_amd import isa, layout, workloads


def test_assembler_triangular_stepping():
    slots, how = layout.simulate_slots(workloads.prog_c2().code)
    assert how == "exit" and slots == [0, 1, 3, 6, 10, 15, 21, 28]


def test_assembler_main_path_counts():
    assert workloads.prog_c2().main_path_steps == 8
    assert workloads.prog_c3().main_path_steps == 64
    assert workloads.prog_c4().main_path_steps >= 64
    assert workloads.prog_c5().main_path_steps == 256


def _info(native, env, code):
    p = native.Prog(env, code)
    try:
        return p.info()
    finally:
        p.destroy()


def test_translation_sizes(native, env):
    i = _info(native, env, workloads.prog_c2().code)
    assert (i.nslots, i.nentries) == (29, 8)
    lay = workloads.prog_c3()
    i = _info(native, env, lay.code)
    assert i.nslots == lay.nslots
    # JA stride resets are folded away: fewer entries than executed-path instructions+resets
    assert 60 <= i.nentries < 200


def test_translation_faults_are_entries(native, env):
    O = isa.OPS
    e = isa.encode
    # falls off the end, self-loop, invalid opcode: each becomes a (shared) FAULT entry
    for code in (e(O["mov_imm"], 0, imm=1) + e(O["mov_imm"], 0, imm=1),
                 e(O["ja"], off=-1) + e(O["exit"]),
                 e(0x06) + e(O["exit"])):
        assert _info(native, env, code).nentries >= 1


def test_translation_resolves_maps(native, env):
    lay = workloads.prog_c4()
    m = native.Map(env, 256, 8)
    try:
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        i = p.info()
        assert i.nmaps == 1 and i.max_stack == 4
        p.destroy()
    finally:
        m.destroy()


def test_all_goldens_translate(native, env):
    for f in goldens.all_golden_files():
        for c in goldens.load(f):
            assert _info(native, env, c.code).nentries >= 1


def test_literal_slot_programs_execute_the_stepped_slots():
    """SURVEY.md §8(d) literal N-slot variants: 64 slots execute 11, 256 execute 23 (slots
    0, 1, 3, 6, ... under cumulative stepping), ending in EXIT."""
    from generic_ebpf_amd import layout, workloads
    for n, k in ((64, 11), (256, 23)):
        lay = workloads.prog_literal(n)
        seq, how = layout.simulate_slots(lay.code)
        assert len(lay.code) == 8 * n and how == "exit" and len(seq) == k == lay.main_path_steps
        assert seq == [i * (i + 1) // 2 for i in range(k)]
