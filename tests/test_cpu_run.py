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
