"""Path-sorted launches (gpu_runtime.cpp launch_pathsorted, asm_jit.cpp asm_pathsort_prefix,
asm_cc.cpp cc_pathsort_plan, bucket.hip path classes).

A batch in offsets form of at least 64K packets, run by a compiled program whose tree splits into
heavy subtrees, runs in three steps: the program's prefix classifies every packet by the subtree
it reaches (cut points retire with fault code 64 + q), the packet indices are sorted by that
class, and the whole program runs over the sorted order, each packet keeping its own result,
fault and verdict.  Per packet the semantics are ebpf_prog_run's (ebpf_interpreter.c:23-372):
results, fault codes and histograms must equal the oracle's — IMIX, truncated packets that fault
inside the prefix and inside subtrees, random programs with random cut points (every class
mixture, small batches forced through the path), device-resident histogram modes."""
import numpy as np
import pytest

import goldens
from helpers import oracle_run

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _pathsort_on(monkeypatch):
    monkeypatch.setenv("EBPF_PATHSORT", "1")


def _check(gpu, env, lay, data, offs, n, relocs=(), maps=()):
    c = goldens.Case("p", lay.code if hasattr(lay, "code") else lay, list(relocs), list(maps), data, n, 0, offs)
    want, wf, wdata, _ = oracle_run(c, nthreads=16)
    from helpers import make_maps
    mp = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in mp]))
    try:
        d = np.ascontiguousarray(data.copy())
        ret, faults, st = p.run_batch(d, n, 0, offs)
        layout = p.exec_info(0)[1]
    finally:
        p.destroy()
        for m in mp:
            m.destroy()
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(d, wdata)
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    np.testing.assert_array_equal(np.array(st.hist[:], dtype=np.int64), np.bincount(bins, minlength=257))
    return layout


def _truncated_imix(n, seed, frac=0.4):
    """IMIX packets cut at random lengths (CSR, back to back): lanes fault in the prefix (the
    length field or a tested byte past the end) and inside the subtrees."""
    from generic_ebpf_amd import workloads
    data, offs, sizes = workloads.packets_imix(n, seed=seed)
    g = np.random.default_rng(seed)
    lens = sizes.astype(np.int64)
    cut = g.random(n) < frac
    lens[cut] = g.integers(1, lens[cut] + 1)
    starts = offs[:-1].astype(np.int64)
    new_offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=new_offs[1:])
    idx = np.concatenate([np.arange(s, s + l) for s, l in zip(starts, lens)])
    return np.ascontiguousarray(data[idx]), new_offs


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_pathsorted_c5_imix(gpu, env, seed):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=seed)
    n = (1 << 17) + 13
    data, offs, _ = workloads.packets_imix(n, seed=seed + 100)
    assert _check(gpu, env, lay, data, offs, n) == 3   # the path-sorted launch ran


@pytest.mark.parametrize("seed", [7, 10])
def test_pathsorted_c5_truncated(gpu, env, seed):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=seed)
    n = 1 << 17
    data, offs = _truncated_imix(n, seed)
    assert _check(gpu, env, lay, data, offs, n) == 3


def test_pathsort_off_is_plain(gpu, env, monkeypatch):
    from generic_ebpf_amd import workloads
    monkeypatch.setenv("EBPF_PATHSORT", "0")
    lay = workloads.prog_c5()
    n = 1 << 17
    data, offs, _ = workloads.packets_imix(n, seed=3)
    assert _check(gpu, env, lay, data, offs, n) == 0


def test_pathsorted_random_programs(gpu, env, monkeypatch):
    """Random stepping-aware programs with two array maps (lookups, stack traffic, every ALU and
    jump quirk) on ragged packets, with the cut threshold at 2 entries and the batch threshold
    at 1 packet: most programs get cut points anywhere in their trees."""
    from generic_ebpf_amd import randprog
    monkeypatch.setenv("EBPF_PATHSORT_MIN", "2")
    monkeypatch.setenv("EBPF_PATHSORT_MINBATCH", "1")
    sorted_runs = 0
    for k in range(60):
        g = np.random.default_rng(5000 + k)
        lay = randprog.random_program(77000 + k, length=int(g.integers(20, 120)), nmaps=2,
                                      map_value_size=8)
        maps = [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes()) for _ in range(2)]
        n = int(g.choice([1, 63, 64, 65, 777, 3000]))
        sizes = g.integers(16, 80, n).astype(np.uint64)
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(sizes, out=offs[1:])
        data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
        layout = _check(gpu, env, lay, data, offs, n, lay.relocs, maps)
        sorted_runs += layout == 3
    assert sorted_runs >= 20, sorted_runs


def test_pathsorted_device_resident_hist_modes(gpu, env):
    """Device-resident: an overwrite launch then two add launches give 3x the oracle's
    histogram; results and fault bytes are the oracle's."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = (1 << 18) + 5
    data, offs = _truncated_imix(n, 41, frac=0.1)
    c = goldens.Case("p", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=16)
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    h = np.bincount(bins, minlength=257)
    p = gpu.Prog(env, lay.code)
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(data).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_flt = torch.full((n,), 77, dtype=torch.uint8, device=dev)
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
        assert p.exec_info(0)[1] == 3
    finally:
        p.destroy()
