"""Window launches (gpu_runtime.cpp launch_windowed, gen_interp.py "Window mode", asm_jit.cpp cut
code, asm_cc.cpp cc_cut_plan cut points).

A batch in offsets form run by a compiled program that reads past the first 64 bytes goes
through the span image in windows: up to 256 packets staged in LDS by one contiguous DMA, every
packet run to its exit or to the head of a heavy subtree (phase A), the cut packets sorted by
subtree in LDS and run again from the start 64 per group (phase C).  Packets that cannot open a
window (not 16-B aligned, longer than a window) run next on the general kernels.  Per packet the
semantics are ebpf_prog_run's (ebpf_interpreter.c:23-372): results, fault codes and histograms
must equal the oracle's — IMIX, truncated packets that fault in phase A and in phase C, unaligned
and oversized packets (the overflow path), out-of-order offsets, random programs, device-resident
histogram modes."""
import numpy as np
import pytest

import goldens
from helpers import oracle_run

pytestmark = pytest.mark.gpu

WINDOW = 4   # ebpf_prog_device_exec layout of a window launch


@pytest.fixture(autouse=True)
def _window_on(monkeypatch):
    monkeypatch.setenv("EBPF_WINDOW", "1")


def _check(gpu, env, lay, data, offs, n, relocs=(), maps=()):
    c = goldens.Case("w", lay.code if hasattr(lay, "code") else lay, list(relocs), list(maps), data, n, 0, offs)
    want, wf, wdata, _ = oracle_run(c, nthreads=16)
    from helpers import make_maps
    mp = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in mp]))
    try:
        d = np.ascontiguousarray(data.copy())
        ret, faults, st = p.run_batch(d, n, 0, offs)
        layout = p.exec_info(0)[1]
        # device-resident, results and fault bytes pre-filled with sentinels: a packet whose
        # result is never stored cannot pass on what an earlier batch left in a pooled buffer
        if n:
            import torch
            dev = torch.device("cuda:0")
            d_pk = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
            d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
            d_ret = torch.full((n,), 0x5eed, dtype=torch.int64, device=dev)
            d_flt = torch.full((n,), 77, dtype=torch.uint8, device=dev)
            d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
            p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(),
                            d_flt.data_ptr(), d_hist.data_ptr(), torch.cuda.current_stream().cuda_stream,
                            hist_overwrite=True)
            torch.cuda.synchronize()
            dev_ret = d_ret.cpu().numpy().view(np.uint64)
            dev_flt = d_flt.cpu().numpy()
            dev_hist = d_hist.cpu().numpy()
    finally:
        p.destroy()
        for m in mp:
            m.destroy()
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(d, wdata)
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    np.testing.assert_array_equal(np.array(st.hist[:], dtype=np.int64), np.bincount(bins, minlength=257))
    if n:
        np.testing.assert_array_equal(dev_flt, wf)
        np.testing.assert_array_equal(dev_ret, want)
        np.testing.assert_array_equal(dev_hist, np.bincount(bins, minlength=257))
    return layout


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_window_c5_imix(gpu, env, seed):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=seed)
    n = (1 << 17) + 13
    data, offs, _ = workloads.packets_imix(n, seed=seed + 100)
    assert _check(gpu, env, lay, data, offs, n) == WINDOW


@pytest.mark.parametrize("seed", [7, 10])
def test_window_c5_truncated(gpu, env, seed):
    """Back-to-back CSR packets of random lengths (mostly not 16-B aligned: the overflow path)."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=seed)
    n = 1 << 17
    data, offs, sizes = workloads.packets_imix(n, seed=seed)
    g = np.random.default_rng(seed)
    lens = sizes.astype(np.int64)
    cut = g.random(n) < 0.4
    lens[cut] = g.integers(1, lens[cut] + 1)
    starts = offs[:-1].astype(np.int64)
    new_offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=new_offs[1:])
    idx = np.concatenate([np.arange(s, s + l) for s, l in zip(starts, lens)])
    assert _check(gpu, env, lay, np.ascontiguousarray(data[idx]), new_offs, n) == WINDOW


def test_window_c5_aligned_truncated(gpu, env):
    """Packets cut short to a multiple of 16 bytes, back to back (every packet 16-B aligned, so
    every packet windows; the cut ones fault at the bytes they lost, in phase A or phase C)."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5(seed=11)
    n = 1 << 17
    data, offs, sizes = workloads.packets_imix(n, seed=12)
    g = np.random.default_rng(12)
    lens = sizes.astype(np.int64)
    cut = g.random(n) < 0.3
    lens[cut] = (g.integers(1, lens[cut] + 1) + 15) // 16 * 16
    lens = np.minimum(lens, (sizes.astype(np.int64) + 15) // 16 * 16)
    starts = offs[:-1].astype(np.int64)
    new_offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=new_offs[1:])
    idx = np.concatenate([np.arange(s, s + l) for s, l in zip(starts, lens)])
    assert _check(gpu, env, lay, np.ascontiguousarray(data[idx]), new_offs, n) == WINDOW


def test_window_overflow_packets(gpu, env, monkeypatch):
    """Jumbo packets longer than a window and unaligned packets between aligned ones: the
    overflow list and its general-kernel launch, mixed with windows."""
    from generic_ebpf_amd import workloads
    monkeypatch.setenv("EBPF_WIN_BYTES", "8192")
    lay = workloads.prog_c5(seed=7)
    g = np.random.default_rng(3)
    n = 20000
    sizes = g.choice([64, 576, 1500, 9000, 20000], size=n, p=[0.5, 0.3, 0.15, 0.04, 0.01])
    shift = np.where(g.random(n) < 0.1, g.integers(1, 16, n), 0)   # some start unaligned
    offs = np.zeros(n + 1, dtype=np.uint64)
    cur = 0
    for i in range(n):
        cur += int(shift[i])
        offs[i] = cur
        cur += int((sizes[i] + 63) // 64 * 64)
    offs[n] = cur
    data = g.integers(0, 256, cur + 64, dtype=np.uint8)
    base = offs[:-1].astype(np.int64)
    data[base + 12] = 0x08
    data[base + 13] = 0
    data[base + 14] = 0x45
    tot = sizes - 14
    data[base + 16] = (tot >> 8) & 0xff
    data[base + 17] = tot & 0xff
    assert _check(gpu, env, lay, data, offs, n) == WINDOW


def test_window_off_is_plain(gpu, env, monkeypatch):
    from generic_ebpf_amd import workloads
    monkeypatch.setenv("EBPF_WINDOW", "0")
    lay = workloads.prog_c5()
    n = 1 << 17
    data, offs, _ = workloads.packets_imix(n, seed=3)
    assert _check(gpu, env, lay, data, offs, n) == 0


def test_window_random_programs(gpu, env, monkeypatch):
    """Random stepping-aware programs with two array maps (lookups, stack traffic, every ALU and
    jump quirk) on packets of random sizes, 16-B aligned or not, with the cut threshold at 2
    entries and the batch threshold at 1 packet: cut points anywhere in the trees.  Every fourth
    program stores into its packets (no window: the plain launch)."""
    from generic_ebpf_amd import randprog
    monkeypatch.setenv("EBPF_WIN_CUT_MIN", "2")
    monkeypatch.setenv("EBPF_WINDOW_MINBATCH", "1")
    windowed = 0
    for k in range(60):
        g = np.random.default_rng(6000 + k)
        lay = randprog.random_program(78000 + k, length=int(g.integers(20, 120)), nmaps=2,
                                      map_value_size=8, pkt_stores=k % 4 == 3)
        maps = [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes()) for _ in range(2)]
        n = int(g.choice([1, 63, 64, 65, 257, 777, 3000]))
        sizes = g.integers(16, 200, n).astype(np.uint64)
        if k % 2 == 0:   # 16-B aligned rows: most packets window
            sizes = (sizes + 15) // 16 * 16
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(sizes, out=offs[1:])
        data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
        layout = _check(gpu, env, lay, data, offs, n, lay.relocs, maps)
        windowed += layout == WINDOW
    assert windowed >= 20, windowed


def test_window_device_resident_hist_modes(gpu, env):
    """Device-resident: an overwrite launch then two add launches give 3x the oracle's
    histogram; results and fault bytes are the oracle's."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = (1 << 18) + 5
    data, offs, sizes = workloads.packets_imix(n, seed=41)
    c = goldens.Case("w", lay.code, [], [], data, n, 0, offs)
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
        assert p.exec_info(0)[1] == WINDOW
    finally:
        p.destroy()
