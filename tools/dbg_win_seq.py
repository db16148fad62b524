"""Replay tests/test_gpu_window.py::test_window_random_programs in one Env, printing every
program's outcome; at a mismatch, rerun that program plain, without cut points and on the
interpreter, in the same Env."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import pkgload  # noqa: E402
pkgload.load()
import numpy as np  # noqa: E402
import goldens  # noqa: E402
from helpers import oracle_run, make_maps  # noqa: E402
from generic_ebpf_amd import randprog, native  # noqa: E402

os.environ["EBPF_WIN_CUT_MIN"] = "2"
os.environ["EBPF_WINDOW_MINBATCH"] = "1"
env = native.Env()


def run(c, data, offs, n, envs, variant=0):
    saved = {k: os.environ.get(k) for k in envs}
    os.environ.update({k: v for k, v in envs.items() if v is not None})
    for k, v in envs.items():
        if v is None:
            os.environ.pop(k, None)
    mp = make_maps(native, env, c)
    p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in mp]))
    native.set_variant(variant)
    d = np.ascontiguousarray(data.copy())
    ret, faults, st = p.run_batch(d, n, 0, offs)
    lay = p.exec_info(0)[:2]
    native.set_variant(0)
    p.destroy()
    for m in mp:
        m.destroy()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    return ret, faults, lay


for k in range(int(sys.argv[1]), int(sys.argv[2])):
    g = np.random.default_rng(6000 + k)
    lay = randprog.random_program(78000 + k, length=int(g.integers(20, 120)), nmaps=2,
                                  map_value_size=8, pkt_stores=k % 4 == 3)
    maps = [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes()) for _ in range(2)]
    n = int(g.choice([1, 63, 64, 65, 257, 777, 3000]))
    sizes = g.integers(16, 200, n).astype(np.uint64)
    if k % 2 == 0:
        sizes = (sizes + 15) // 16 * 16
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
    c = goldens.Case("w", lay.code, list(lay.relocs), maps, data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=4)
    ret, flt, ly = run(c, data, offs, n, {"EBPF_WINDOW": "1"})
    bad = int((ret != want).sum()) + int((flt != wf).sum())
    print(k, n, ly, "bad", bad, flush=True)
    if bad:
        import torch
        dev = torch.device("cuda:0")
        mp = make_maps(native, env, c)
        p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in mp]))
        os.environ["EBPF_WINDOW"] = "1"
        d_pk = torch.from_numpy(data).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_ret = torch.full((n,), 0x5555, dtype=torch.int64, device=dev)
        d_flt = torch.full((n,), 77, dtype=torch.uint8, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        stq = torch.cuda.current_stream().cuda_stream
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(),
                        d_flt.data_ptr(), d_hist.data_ptr(), stq, hist_overwrite=True)
        torch.cuda.synchronize()
        r = d_ret.cpu().numpy().view(np.uint64)
        print("  dev-resident: ret values", np.unique(r)[:5], "faults", np.unique(d_flt.cpu().numpy()),
              "hist nonzero", {int(i): int(v) for i, v in enumerate(d_hist.cpu().numpy()) if v})
        p.destroy()
        for m in mp:
            m.destroy()
        i = int(np.nonzero((ret != want) | (flt != wf))[0][0])
        print("  first", i, "want", want[i], wf[i], "got", ret[i], flt[i])
        for name, envs, var in (("again", {"EBPF_WINDOW": "1"}, 0), ("plain", {"EBPF_WINDOW": "0"}, 0),
                                ("nohoist", {"EBPF_WINDOW": "1", "EBPF_CC_NOHOIST": "1"}, 0),
                                ("norunmask", {"EBPF_WINDOW": "1", "EBPF_CC_NORUNMASK": "1"}, 0),
                                ("nocc", {"EBPF_WINDOW": "1", "EBPF_JIT_NOCC": "1"}, 0),
                                ("wg1", {"EBPF_WINDOW": "1", "EBPF_WIN_WG": "1"}, 0),
                                ("again2", {"EBPF_WINDOW": "1"}, 0),
                                ("nocut", {"EBPF_WINDOW": "1", "EBPF_WINDOW_NOCUT": "1"}, 0),
                                ("interp", {"EBPF_WINDOW": "0"}, 2)):
            r2, f2, l2 = run(c, data, offs, n, envs, var)
            print("  ", name, l2, "bad", int((r2 != want).sum()) + int((f2 != wf).sum()), r2[i], flush=True)
