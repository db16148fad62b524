"""Multi-GPU sharding of one batch.

* In the library: ebpf_prog_run_batch_multi (host buffers, one thread per shard; a device may
  repeat, which is how one GPU box exercises N shards) and ebpf_prog_run_batch_multi_dev
  (device-resident, RCCL all-reduce of the verdict histograms).
* Across processes (the bench's layout): 2 ranks on cuda:0 with gloo, the concatenated
  shard results and the summed histogram equal ONE launch over the whole batch
  (tests/shard_worker.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import goldens
from helpers import make_maps, oracle_run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c4_case(n, seed=3):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4()
    pk = workloads.packets_l2l3(n, 64, seed=seed)
    return goldens.Case("c4", lay.code, lay.relocs,
                        [(8, 256, workloads.c4_map_values().tobytes())], pk.reshape(-1), n, 64, None)


def test_multi_rejects_bad_devices(env):
    """No GPU here: every device index is out of range (ENODEV); bad lists are EINVAL."""
    import errno
    from generic_ebpf_amd import native
    c = _c4_case(64)
    maps = make_maps(native, env, c)
    p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        with pytest.raises(native.EbpfError) as ei:
            p.run_batch_multi([], np.ascontiguousarray(c.data), 64, 64)
        assert ei.value.code == errno.EINVAL
        if native.gpu_count() == 0:
            with pytest.raises(native.EbpfError) as ei:
                p.run_batch_multi([0], np.ascontiguousarray(c.data), 64, 64)
            assert ei.value.code == errno.ENODEV
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


def test_dev_init(native):
    """ebpf_dev_init: ENODEV with no GPU or more devices than visible; on a GPU
    host every visible device loads its kernels."""
    import errno
    n = native.gpu_count()
    with pytest.raises(native.EbpfError) as ei:
        native.dev_init(n + 1)
    assert ei.value.code == errno.ENODEV
    if n == 0:
        with pytest.raises(native.EbpfError) as ei:
            native.dev_init(0)
        assert ei.value.code == errno.ENODEV
    else:
        native.dev_init(0)
        native.dev_init(1)


@pytest.mark.gpu
def test_dev_init_gpu(gpu):
    gpu.dev_init(0)
    gpu.dev_init(gpu.gpu_count())


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [1, 2, 3])
def test_run_batch_multi_host_buffers(gpu, env, ndev):
    """Shards on one GPU (repeated device index): results, faults and the summed histogram equal
    the oracle's; a ragged count leaves uneven shards."""
    n = (1 << 20) + 37
    c = _c4_case(n)
    want, wf, _, _ = oracle_run(c, nthreads=16)
    maps = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        ret, faults, st = p.run_batch_multi([0] * ndev, np.ascontiguousarray(c.data), n, 64)
        np.testing.assert_array_equal(ret, want)
        np.testing.assert_array_equal(faults, wf)
        h = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257)
        np.testing.assert_array_equal(np.array(st.hist[:], dtype=np.int64), h)
        assert st.packets == n and st.faulted == 0
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
def test_run_batch_multi_imix(gpu, env):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = 1 << 16
    data, offs, _ = workloads.packets_imix(n, seed=9)
    c = goldens.Case("c5", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=16)
    p = gpu.Prog(env, c.code)
    try:
        ret, faults, st = p.run_batch_multi([0, 0], np.ascontiguousarray(data), n, 0, offs)
        np.testing.assert_array_equal(ret, want)
        np.testing.assert_array_equal(faults, wf)
    finally:
        p.destroy()


@pytest.mark.gpu
def test_run_batch_multi_dev_rccl(gpu, env, monkeypatch):
    """Device-resident multi launch through the RCCL all-reduce (forced at one device: the
    communicator, the grouped all-reduce and the dlopen of RCCL all run), histogram exact in
    overwrite mode and in add mode over three consecutive calls (the caller's earlier counts are
    added to, never multiplied by the collective)."""
    import torch
    monkeypatch.setenv("EBPF_FORCE_RCCL", "1")
    n = 1 << 20
    c = _c4_case(n, seed=21)
    want, _, _, _ = oracle_run(c, nthreads=16)
    h = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257)
    maps = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(c.data).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_hist = torch.full((257,), 5, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        p.run_batch_multi_dev([0], [(d_pk.data_ptr(), n, 64, None)], [d_ret.data_ptr()],
                              hists=[d_hist.data_ptr()], streams=[st], hist_overwrite=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
        d_hist.fill_(5)
        for _ in range(3):
            p.run_batch_multi_dev([0], [(d_pk.data_ptr(), n, 64, None)], [d_ret.data_ptr()],
                                  hists=[d_hist.data_ptr()], streams=[st])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_hist.cpu().numpy(), 5 + 3 * h)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("same_stream", [False, True])
def test_run_batch_multi_dev_shards_one_device(gpu, env, same_stream):
    """Two shards on one device (a repeated device index): each caller histogram receives the
    SUM over both shards, added to what it held (three calls in add mode: 3x the oracle's plus
    the initial counts) or set (overwrite); shards on two streams join and fork correctly."""
    import torch
    n = (1 << 20) + 333
    c = _c4_case(n, seed=22)
    want, _, _, _ = oracle_run(c, nthreads=16)
    h = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257)
    maps = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(c.data).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        h0 = torch.full((257,), 7, dtype=torch.int64, device=dev)
        h1 = torch.full((257,), 11, dtype=torch.int64, device=dev)
        s0 = torch.cuda.Stream()
        s1 = s0 if same_stream else torch.cuda.Stream()
        torch.cuda.synchronize()
        half = n // 2
        shards = [(d_pk.data_ptr(), half, 64, None),
                  (d_pk.data_ptr() + half * 64, n - half, 64, None)]
        rets = [d_ret.data_ptr(), d_ret.data_ptr() + half * 8]
        for _ in range(3):
            p.run_batch_multi_dev([0, 0], shards, rets, hists=[h0.data_ptr(), h1.data_ptr()],
                                  streams=[s0.cuda_stream, s1.cuda_stream])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
        np.testing.assert_array_equal(h0.cpu().numpy(), 7 + 3 * h)
        np.testing.assert_array_equal(h1.cpu().numpy(), 11 + 3 * h)
        p.run_batch_multi_dev([0, 0], shards, rets, hists=[h0.data_ptr(), h1.data_ptr()],
                              streams=[s0.cuda_stream, s1.cuda_stream], hist_overwrite=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(h0.cpu().numpy(), h)
        np.testing.assert_array_equal(h1.cpu().numpy(), h)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
def test_entry_points_keep_current_device(gpu, env):
    """A C library must not change its caller's current device: after every entry point the
    thread's device is the one it set (on a box with several GPUs the caller sits on the last
    one and the library works on device 0)."""
    import torch
    nd = torch.cuda.device_count()
    mine = nd - 1
    torch.cuda.set_device(mine)
    n = 4096
    c = _c4_case(n, seed=23)
    maps = make_maps(gpu, env, c)
    p = gpu.Prog(env, gpu.patch_relocs(c.code, c.relocs, [m.handle for m in maps]))
    try:
        gpu.dev_init(0)
        assert torch.cuda.current_device() == mine
        p.prepare(0)
        assert torch.cuda.current_device() == mine
        ret, faults, st = p.run_batch(np.ascontiguousarray(c.data), n, 64)
        assert torch.cuda.current_device() == mine
        p.run_batch_multi([0, 0], np.ascontiguousarray(c.data), n, 64)
        assert torch.cuda.current_device() == mine
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(c.data).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        torch.cuda.set_device(mine)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), hist_ptr=d_hist.data_ptr())
        assert torch.cuda.current_device() == mine
        p.run_batch_multi_dev([0], [(d_pk.data_ptr(), n, 64, None)], [d_ret.data_ptr()],
                              hists=[d_hist.data_ptr()])
        assert torch.cuda.current_device() == mine
        torch.cuda.synchronize(dev)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()
        torch.cuda.set_device(0)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,total", [("c4", (1 << 22) + 4099), ("c5", 200001)])
def test_two_ranks_gloo_equal_one_launch(gpu, cfg, total):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(29611 + (cfg == "c5")),
           os.path.join(ROOT, "tests", "shard_worker.py"), cfg, str(total)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout.decode()[-2000:], r.stderr.decode()[-3000:])
    assert '"hist_equal": true' in r.stdout.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("launcher", ["torchrun", "self"])
def test_bench_two_ranks_gloo(launcher):
    """bench.py's own N > 1 path (the driver's scaling run uses it with RCCL on 8 GPUs): two
    ranks on cuda:0 over gloo, strong sharding of one C4 batch; rank 0 prints one verified line
    counting both shards, with C5 (BASELINE config 5) measured the same way under "also".
    "self": plain `bench.py --gpus 2` with no launcher around it starts its own two ranks."""
    import json
    total = (1 << 21) + 77
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
            "--packets", str(total), "--no-cpu-baseline", "--no-pmc", "--also", "c5"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", "--master-port", "29631"] + args
    else:
        cmd = [sys.executable] + args
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="4", EBPF_BENCH_BACKEND="gloo")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout.decode()[-2000:], r.stderr.decode()[-3000:])
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout.decode()[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["verified"] is True and d["scaling"] == "strong"
    assert d["config"]["packets_total"] == total
    assert d["config"]["packets_per_gpu"] == (total + 1) // 2
    # BASELINE config 5 in the same run, sharded the same way
    c5 = d["also"]["c5"]
    assert c5["verified"] is True and c5["packets_total"] == 1 << 22, c5


def _bench_rc(args, **extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120, env=env)
    return r.returncode, r.stderr.decode()


def test_bench_gpus_checks():
    """`bench.py --gpus N` refuses to run a line it cannot honour (CPU here: no GPU visible):
    fewer visible GPUs than N, and a launcher whose WORLD_SIZE disagrees with --gpus."""
    import torch
    if torch.cuda.device_count() == 0:
        rc, err = _bench_rc(["--gpus", "2", "--steps", "1", "--warmup", "0"])
        assert rc == 2 and "--gpus 2 but 0 GPU(s) visible" in err, err
    rc, err = _bench_rc(["--gpus", "2", "--steps", "1"], WORLD_SIZE="1")
    assert rc == 2 and "WORLD_SIZE=1 but --gpus 2" in err, err
    rc, err = _bench_rc(["--gpus", "1", "--steps", "1"], WORLD_SIZE="4")
    assert rc == 2 and "WORLD_SIZE=4 but --gpus 1" in err, err
