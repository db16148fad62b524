"""Length-bucketed launches of mixed-size batches (gpu_runtime.cpp launch_bucketed, bucket.hip,
the span-staged kernels of gen_interp.py and asm_cc.cpp mode 2).

A batch in offsets form of at least 64K packets, run by a compiled program that loads past the
packets' first 64 bytes, is sorted into length classes on the device; class 0 (short, jumbo or
unaligned packets) runs on the general kernels, the others with each packet staged whole in LDS.
Per packet the semantics are those of ebpf_prog_run (ebpf_interpreter.c:327-338 loads at
r + off): the results, fault codes and the verdict histogram must equal the oracle's for every
mix of classes — IMIX, ragged counts, random lengths with aligned and unaligned starts, loads
that straddle 16-B blocks, generic (pointer-arithmetic) loads and lanes that fault."""
import numpy as np
import pytest

import goldens
from helpers import oracle_run

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bucketing_on(monkeypatch):
    monkeypatch.setenv("EBPF_BUCKET", "1")

R0, R1, R2, R3, R4, R5, R6 = range(7)


def _pointer_prog():
    """r2 = r1 + (pkt[16..17] & 0x7ff) (a data-dependent offset: generic, region-checked loads
    through the LDS aperture), r0 = u32 at r2 + 3 xor u16 at r1 + 130 (constant offset, past the
    header) xor u64 at r1 + 70 (straddles two 16-B blocks); lanes past their packet fault MEM."""
    from generic_ebpf_amd import isa, layout
    I = isa.Insn
    return layout.assemble([
        I("ldxh", R3, R1, 16), I("and_imm", R3, imm=0x7ff),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R1), I("add64_reg", R2, R3),
        I("ldxw", R0, R2, 3),
        I("ldxh", R4, R1, 130), I("xor64_reg", R0, R4),
        I("ldxdw", R5, R1, 70), I("xor64_reg", R0, R5),
        I("exit")])


def _batch(kind, n, seed):
    """(data, offsets) of n packets."""
    from generic_ebpf_amd import workloads
    g = np.random.default_rng(seed)
    if kind == "imix":
        data, offs, _ = workloads.packets_imix(n, seed=seed)
        return data, offs
    lens = g.integers(1, 2000, n)
    if kind == "aligned":       # every start on a 16-B boundary: classes 0, 1, 2 and jumbo
        pad = (lens + 15) // 16 * 16
    elif kind == "unaligned":   # back to back: most starts unaligned (class 0)
        pad = lens
    else:                       # half and half
        pad = np.where(g.random(n) < 0.5, (lens + 15) // 16 * 16, lens)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(pad, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    return data, offs


def _check(gpu, env, lay, data, offs, n):
    c = goldens.Case("b", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=16)
    p = gpu.Prog(env, lay.code)
    try:
        ret, faults, st = p.run_batch(np.ascontiguousarray(data.copy()), n, 0, offs)
        exec_name, layout, _, _ = p.exec_info(0)
    finally:
        p.destroy()
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    np.testing.assert_array_equal(np.array(st.hist[:], dtype=np.int64),
                                  np.bincount(bins, minlength=257))
    return layout


@pytest.mark.parametrize("kind", ["imix", "aligned", "unaligned", "mixed"])
@pytest.mark.parametrize("prog", ["c5", "c5s8", "pointer"])
def test_bucketed_vs_oracle(gpu, env, kind, prog):
    from generic_ebpf_amd import workloads
    lay = {"c5": workloads.prog_c5, "c5s8": lambda: workloads.prog_c5(seed=8),
           "pointer": _pointer_prog}[prog]()
    n = (1 << 17) + 13
    data, offs = _batch(kind, n, 31)
    layout = _check(gpu, env, lay, data, offs, n)
    assert layout == 2   # the bucketed launch ran


@pytest.mark.parametrize("seed", [9, 10, 11])
def test_bucketed_c5_variants_truncated(gpu, env, seed):
    """Other C5 programs over IMIX packets cut at random lengths and zero-padded to a multiple
    of 16 bytes (CSR has no gaps: the padding is part of the packet; every start stays 16-B
    aligned, so the span classes take them): lanes end inside runs of hoisted LDS loads and
    fault there."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=seed)
    n = 1 << 17
    data, offs, sizes = workloads.packets_imix(n, seed=seed)
    g = np.random.default_rng(seed)
    lens = sizes.astype(np.int64)
    cut = g.random(n) < 0.4
    lens[cut] = g.integers(18, lens[cut] + 1)
    starts = offs[:-1].astype(np.int64)
    pad = (lens + 15) // 16 * 16
    new_offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(pad, out=new_offs[1:])
    new_data = np.zeros(int(new_offs[-1]), dtype=np.uint8)
    for i in range(n):
        new_data[int(new_offs[i]):int(new_offs[i]) + lens[i]] = data[starts[i]:starts[i] + lens[i]]
    layout = _check(gpu, env, lay, new_data, new_offs, n)
    assert layout == 2


def test_bucketed_device_resident_hist_modes(gpu, env):
    """The device-resident path: three launches of one IMIX batch in add mode give 3x the
    oracle's histogram (the class launches add, only the first of an overwrite launch stores)."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = (1 << 18) + 5
    data, offs = _batch("imix", n, 41)
    c = goldens.Case("b", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=16)
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    h = np.bincount(bins, minlength=257)
    p = gpu.Prog(env, lay.code)
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(data).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_hist = torch.full((257,), 9, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(),
                        d_flt.data_ptr(), d_hist.data_ptr(), st, hist_overwrite=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
        for _ in range(2):
            p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(),
                            d_flt.data_ptr(), d_hist.data_ptr(), st)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_hist.cpu().numpy(), 3 * h)
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
        np.testing.assert_array_equal(d_flt.cpu().numpy(), wf)
        assert p.exec_info(0)[1] == 2
    finally:
        p.destroy()
