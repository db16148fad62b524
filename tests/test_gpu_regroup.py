"""Regrouping (compiled programs, general kernels; gen_interp.py "Regrouping", asm_cc.cpp
cc_regroup_plan): lanes that reach the head of a heavy subtree are queued and run later in
batches of 64 lanes that all take that subtree.  The results, fault codes and verdict histogram
must be what running every packet on its own gives (the oracle, restating ebpf_interpreter.c),
whatever the batch size: partial batches at the end of a wave's groups, faults inside queued
subtrees, packets of any length at any offset."""
import numpy as np
import pytest

import goldens
from helpers import device_run, oracle_run

PUSH = bytes.fromhex("7e0db5be")   # s_bcnt1_i32_b64 s53, exec: the head of a queue push


def _prog(body):
    from generic_ebpf_amd import workloads
    return workloads.assemble(workloads._c5_nodes(3, body))


def _packets(n, seed=21):
    """Packets of any length 20..1599 at unaligned offsets; bytes 16-17 (the IPv4 total length
    the program branches on) random, so a lane's size class says nothing about its real length
    and the subtrees' loads fault (MEM) on short packets."""
    g = np.random.default_rng(seed)
    sizes = g.integers(20, 1600, n).astype(np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
    return data, offs


def _points(native, env, code, layout=0):
    p = native.Prog(env, code)
    try:
        return p.device_code(layout).count(PUSH)
    finally:
        p.destroy()


def test_plan_picks_the_c5_leaves(native, env, monkeypatch):
    """C5's twelve leaves (three size classes x a depth-2 tree) become the regroup points of the
    general kernel; none in the staged kernel (64-B packets: no general kernel) or when disabled."""
    from generic_ebpf_amd import workloads
    code = workloads.prog_c5().code
    assert _points(native, env, code) == 0          # (opt-in)
    monkeypatch.setenv("EBPF_CC_REGROUP", "1")
    assert _points(native, env, code) == 12
    assert _points(native, env, _prog(120).code) == 12


def test_plan_skips_programs_without_divergent_heavy_paths(native, env, monkeypatch):
    from generic_ebpf_amd import workloads
    monkeypatch.setenv("EBPF_CC_REGROUP", "1")
    for cfg in ("c2", "c3", "c0"):
        assert _points(native, env, workloads.CONFIGS[cfg]["prog"]().code) == 0, cfg


@pytest.fixture()
def regroup(monkeypatch):
    monkeypatch.setenv("EBPF_CC_REGROUP", "1")


@pytest.mark.gpu
def test_regrouped_results_faults_ragged(gpu, env, regroup):
    lay = _prog(120)
    assert _points(gpu, env, lay.code) == 12
    for n in (1, 63, 64, 65, 1000, 4097, 100003):
        data, offs = _packets(n, seed=n)
        c = goldens.Case("rg", lay.code, [], [], data, n, 0, offs)
        want, wf, _, _ = oracle_run(c, nthreads=8)
        got, gf, _ = device_run(gpu, env, c, 0)
        assert (wf != 0).any() or n < 100, "the case should fault some packets"
        np.testing.assert_array_equal(wf, gf, err_msg="n=%d" % n)
        np.testing.assert_array_equal(want, got, err_msg="n=%d" % n)


@pytest.mark.gpu
def test_regrouped_histogram_device_resident(gpu, env, regroup):
    """Device-resident launch with a verdict histogram (exits of queued lanes count in their
    batch, faults in bin 256) and an overwrite launch after it on the same stream."""
    import torch
    lay = _prog(120)
    n = 300007
    data, offs = _packets(n, seed=5)
    c = goldens.Case("rg", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    h = np.zeros(257, dtype=np.int64)
    ok = wf == 0
    np.add.at(h, np.minimum(want[ok], 255).astype(np.int64), 1)
    h[256] = int((~ok).sum())
    p = gpu.Prog(env, lay.code)
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(data).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream()
        for _ in range(2):
            p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(),
                            d_flt.data_ptr(), d_hist.data_ptr(), st.cuda_stream, hist_overwrite=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
        np.testing.assert_array_equal(d_flt.cpu().numpy(), wf)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
    finally:
        p.destroy()


@pytest.mark.gpu
def test_regroup_on_off_agree_c5(gpu, env, regroup, monkeypatch):
    """C5 on IMIX packets, regrouped and not: bit-identical (and equal to the oracle)."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = 1 << 17
    data, offs, _ = workloads.packets_imix(n)
    c = goldens.Case("c5", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    got, gf, _ = device_run(gpu, env, c, 0)
    monkeypatch.delenv("EBPF_CC_REGROUP")
    got2, gf2, _ = device_run(gpu, env, c, 0)
    np.testing.assert_array_equal(want, got)
    np.testing.assert_array_equal(got, got2)
    np.testing.assert_array_equal(wf, gf)
    np.testing.assert_array_equal(gf, gf2)
