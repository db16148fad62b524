"""Shared helpers: run a golden/generated case on the oracle and on the device."""
import numpy as np

import pyoracle


def oracle_run(case, nthreads=4):
    op = pyoracle.OracleProgram(case.code, case.relocs, case.maps)
    return op.run(case.data, case.count, case.stride, case.offsets, nthreads=nthreads)


def make_maps(native, env, case):
    maps = []
    for vs, me, d in case.maps:
        m = native.Map(env, me, vs)
        m.fill(d)
        maps.append(m)
    return maps


def device_run(native, env, case, variant=0):
    """Host-buffer batch run on the GPU.  Returns (ret, faults, data_after)."""
    maps = make_maps(native, env, case)
    code = native.patch_relocs(case.code, case.relocs, [m.handle for m in maps])
    p = native.Prog(env, code)
    try:
        native.set_variant(variant)
        data = np.ascontiguousarray(case.data.copy())
        ret, faults, _ = p.run_batch(data, case.count, case.stride, case.offsets)
        return ret, faults, data
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()
