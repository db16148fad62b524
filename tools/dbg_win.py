"""Debug one random program of tests/test_gpu_window.py::test_window_random_programs: the oracle,
the plain launch, the window launch (with and without cut points), the interpreter variants."""
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

k = int(sys.argv[1])
g = np.random.default_rng(6000 + k)
lay = randprog.random_program(78000 + k, length=int(g.integers(20, 120)), nmaps=2, map_value_size=8,
                              pkt_stores=k % 4 == 3)
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
print("oracle", want[:4], wf[:4])
os.environ["EBPF_WIN_CUT_MIN"] = "2"
os.environ["EBPF_WINDOW_MINBATCH"] = "1"
for name, envs, variant in (("plain", {"EBPF_WINDOW": "0"}, 0), ("window", {"EBPF_WINDOW": "1"}, 0),
                            ("window-nocut", {"EBPF_WINDOW": "1", "EBPF_WINDOW_NOCUT": "1"}, 0),
                            ("interp", {"EBPF_WINDOW": "0"}, 2), ("hip", {"EBPF_WINDOW": "0"}, 1)):
    os.environ.update(envs)
    os.environ.pop("EBPF_WINDOW_NOCUT", None) if "EBPF_WINDOW_NOCUT" not in envs else None
    env = native.Env()
    mp = make_maps(native, env, c)
    p = native.Prog(env, native.patch_relocs(c.code, c.relocs, [m.handle for m in mp]))
    native.set_variant(variant)
    d = np.ascontiguousarray(data.copy())
    ret, faults, st = p.run_batch(d, n, 0, offs)
    print(name, p.exec_info(0)[:2], ret[:4], faults[:4], "mismatch", int((ret != want).sum()),
          int((faults != wf).sum()))
    native.set_variant(0)
    p.destroy()
    for m in mp:
        m.destroy()
