"""ebpf_prog_run_batch_async / ebpf_batch_wait (include/ebpf_gpu.h): the host-buffer batch without
blocking the caller (a NIC-ring consumer overlapping its next segment).
CPU: argument errors and ENODEV with no GPU.  GPU: several jobs in flight at once, each equal to
the oracle, and a failing batch's error surfacing at the wait."""
import ctypes
import errno

import numpy as np
import pytest

import goldens
from helpers import oracle_run


def _prog(native, env):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c3()
    return lay, native.Prog(env, lay.code)


def test_async_argument_errors(native, env):
    lay, p = _prog(native, env)
    try:
        b = native.PktBatch(None, None, 0, 64, 0)
        h = ctypes.c_void_p()
        assert native.lib().ebpf_prog_run_batch_async(p.ptr, ctypes.byref(b), None, None,
                                                      ctypes.byref(h)) == errno.EINVAL
        assert native.lib().ebpf_prog_run_batch_async(p.ptr, ctypes.byref(b), None, None,
                                                      None) == errno.EINVAL
        assert native.lib().ebpf_batch_wait(None, None) == errno.EINVAL
        if native.gpu_count() == 0:
            ret = np.zeros(1, dtype=np.uint64)
            assert native.lib().ebpf_prog_run_batch_async(
                p.ptr, ctypes.byref(b), ret.ctypes.data, None, ctypes.byref(h)) == errno.ENODEV
            assert h.value is None
    finally:
        p.destroy()


@pytest.mark.gpu
def test_async_jobs_in_flight_vs_oracle(gpu, env):
    from generic_ebpf_amd import workloads
    lay, p = _prog(gpu, env)
    try:
        jobs, cases = [], []
        for k in range(4):
            n = (1 << 20) + 997 * k
            if k % 2:   # offsets form, packets cut to 20..64 B (short ones fault MEM)
                lens = np.random.default_rng(k).integers(20, 65, n)
                frames = workloads.packets_l2l3(n, 64, seed=20 + k)
                data = np.ascontiguousarray(frames[np.arange(64)[None, :] < lens[:, None]])
                offs = np.zeros(n + 1, dtype=np.uint64)
                np.cumsum(lens, out=offs[1:])
                c = goldens.Case("a%d" % k, lay.code, [], [], data, n, 0, offs)
                jobs.append(p.run_batch_async(data, n, 0, offs))
            else:
                data = workloads.packets_l2l3(n, 64, seed=20 + k).reshape(-1)
                c = goldens.Case("a%d" % k, lay.code, [], [], data, n, 64, None)
                jobs.append(p.run_batch_async(data, n, 64))
            cases.append(c)
        for c, j in zip(cases, jobs):
            got, gf, st = j.wait()
            want, wf, _, _ = oracle_run(c, nthreads=8)
            np.testing.assert_array_equal(wf, gf)
            np.testing.assert_array_equal(want, got)
            assert st.packets == c.count
    finally:
        p.destroy()


@pytest.mark.gpu
def test_async_error_surfaces_at_wait(gpu, env):
    """A batch the pipeline refuses (no packet data) is still a job: its error is the wait's."""
    lay, p = _prog(gpu, env)
    try:
        b = gpu.PktBatch(None, None, 10, 64, 0)
        ret = np.zeros(10, dtype=np.uint64)
        h = ctypes.c_void_p()
        rc = gpu.lib().ebpf_prog_run_batch_async(p.ptr, ctypes.byref(b), ret.ctypes.data, None,
                                                 ctypes.byref(h))
        assert rc == 0 and h.value
        assert gpu.lib().ebpf_batch_wait(h, None) == errno.EINVAL
    finally:
        p.destroy()
