"""ebpf_prog_run (single packet, CPU entry point of the drop-in API) against the genuine
reference's golden vectors."""
import numpy as np
import pytest

import goldens
from helpers import make_maps

CASES = [c for f in goldens.all_golden_files() for c in goldens.load(f)]


@pytest.mark.parametrize("case", CASES[:80], ids=[c.name for c in CASES[:80]])
def test_single_packet_matches_reference(native, env, case):
    maps = make_maps(native, env, case)
    p = native.Prog(env, native.patch_relocs(case.code, case.relocs, [m.handle for m in maps]))
    try:
        for i in range(min(case.count, 32)):
            if case.offsets is not None:
                lo, hi = int(case.offsets[i]), int(case.offsets[i + 1])
            else:
                lo, hi = i * case.stride, (i + 1) * case.stride
            r, after = p.run_cpu(case.data[lo:hi].tobytes())
            assert r == case.expect_r0[i]
            assert after == case.expect_data[lo:hi].tobytes()
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


def test_random_and_mutated_programs_match_oracle(native, env):
    """ebpf_prog_run (the API's CPU entry point, interp_cpu.cpp) against the oracle on random
    stepping-aware programs and randomly edited ones (tools/fuzz_gpu.py's generator and mutator,
    kept when the oracle's track_undef finds them defined), on the packets that do not fault
    (the reference has no error channel: a faulting packet crashes it, and this entry point
    keeps that)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    argv, sys.argv = sys.argv, sys.argv[:1]
    try:
        import fuzz_gpu as F
    finally:
        sys.argv = argv
    checked, bad = 0, []
    for k in range(240):
        c = F.case(k, 6, "staged", writes=False)
        if k % 2:
            c.code = F.mutate(c.code, np.random.default_rng(6 * 7777 + k))
            if not F.defined(c):
                continue
        want, wf, wdata, _ = F.oracle(c)
        maps = make_maps(native, env, c)
        p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
        try:
            pk = c.data.reshape(c.count, 64)
            after = wdata.reshape(c.count, 64)
            for i in range(min(c.count, 16)):
                if wf[i]:
                    continue
                r, out = p.run_cpu(pk[i].tobytes())
                checked += 1
                if r != want[i] or out != after[i].tobytes():
                    bad.append((k, i))
                    break
        finally:
            p.destroy()
            for m in maps:
                m.destroy()
    assert checked > 1000 and not bad, (checked, bad[:10])
