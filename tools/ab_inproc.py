#!/usr/bin/env python3
"""In-process A/B timing of compiled programs on one GPU: the boxes differ by several percent in
HBM throughput, so relative costs (C4 over the c0 floor, optimiser on/off) are measured by
alternating the candidates inside one process, many rounds, and reporting the median kernel time.

  python3 tools/ab_inproc.py c0 c4 c4:nocc c3 ...     (":nocc" = compiled with EBPF_JIT_NOCC=1)
  python3 tools/ab_inproc.py ab/k4.so@c0 ab/k4.so@c4 ab/k8.so@c4   (a build of the library per
                                                                   candidate, all in one process)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from generic_ebpf_amd import native, workloads  # noqa: E402


def main():
    import torch
    names = sys.argv[1:] or ["c0", "c4"]
    rounds, launches = 7, 20
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("AB_PACKETS", 1 << 26))
    pk = workloads.packets_l2l3(1 << 22, 64, seed=3)
    d_l2 = torch.from_numpy(pk.reshape(-1)).to(dev).repeat(-(-n >> 22))
    rnd = workloads.packets_random(1 << 22, 64, seed=2)
    d_rnd = torch.from_numpy(rnd.reshape(-1)).to(dev).repeat(-(-n >> 22))
    d_ret = torch.empty(n, dtype=torch.int64, device=dev)
    n5 = min(n, 1 << 22)
    imix, imix_offs, _ = workloads.packets_imix(n5, seed=5)
    d_imix = torch.from_numpy(imix).to(dev)
    d_imix_offs = torch.from_numpy(imix_offs.view(np.int64)).to(dev)
    d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    cands = []
    libs = {}

    def select(path):
        # one CDLL per library build (RTLD_LOCAL: each resolves its own symbols)
        if path not in libs:
            native._lib = None
            native.LIB_PATH = path
            libs[path] = native.lib()
        native._lib = libs[path]

    default_lib = native.LIB_PATH
    envs = {}
    for nm in names:
        path, _, spec = nm.rpartition("@")
        path = os.path.join(ROOT, path) if path else default_lib
        select(path)
        if path not in envs:
            envs[path] = (native.Env(), {})
        env, maps = envs[path]
        cfg, _, opt = spec.partition(":")
        lay = workloads.CONFIGS[cfg]["prog"]()
        handles = []
        if cfg == "c4h":
            # ":eNN" = a table of 2^NN entries instead of the bench's 1M (footprint probe)
            ent = 1 << int(opt[1:]) if opt.startswith("e") else workloads.C4H_ENTRIES
            key = "c4h%d" % ent
            if key not in maps:
                universe, hk, hv = workloads.c4h_table(entries=ent)
                hm = native.HashMap(env, 4, 8, len(hk))
                hm.fill(hk, hv)
                maps[key] = hm
                maps[key + "_pk"] = torch.from_numpy(
                    workloads.packets_c4h(1 << 22, universe).reshape(-1)).to(dev).repeat(-(-n >> 22))
            handles = [maps[key].handle]
        if cfg == "c4":
            if "c4" not in maps:
                m = native.Map(env, 256, 8)
                m.fill(workloads.c4_map_values().tobytes())
                maps["c4"] = m
            handles = [maps["c4"].handle]
        if opt == "nocc":
            os.environ["EBPF_JIT_NOCC"] = "1"
        if opt == "nohoist":
            os.environ["EBPF_CC_NOHOIST"] = "1"
        if opt == "noshort":
            os.environ["EBPF_CC_NOSHORT"] = "1"
        if opt == "nohfwd":
            os.environ["EBPF_CC_NOHFWD"] = "1"
        if opt == "defer":
            os.environ["EBPF_CC_DEFER_DMA"] = "1"
        if opt.startswith("off"):
            os.environ["EBPF_CC_OFF"] = opt[3:]
        if opt.startswith("salu") or opt.startswith("valu"):   # issue-port probes
            os.environ["EBPF_CC_PAD_" + opt[:4].upper()] = opt[4:]
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, handles))
        p.prepare(0)
        data = d_rnd if cfg in ("c0", "c2") else d_l2
        if cfg == "c4h":
            data = maps["c4h%d_pk" % (1 << int(opt[1:]) if opt.startswith("e") else workloads.C4H_ENTRIES)]
        if opt == "l2":      # the same program over the other packet buffer (placement check)
            data = d_l2
        elif opt == "rnd":
            data = d_rnd
        # the program is compiled at its first launch
        if cfg == "c5":
            data = d_imix
            p.run_batch_dev(0, data.data_ptr(), 64, 0, d_ret.data_ptr(), d_imix_offs.data_ptr(),
                            None, None, stream.cuda_stream)
        else:
            p.run_batch_dev(0, data.data_ptr(), 64, 64, d_ret.data_ptr(), None, None, None,
                            stream.cuda_stream)
        torch.cuda.synchronize()
        os.environ.pop("EBPF_JIT_NOCC", None)
        os.environ.pop("EBPF_CC_NOHOIST", None)
        os.environ.pop("EBPF_CC_OFF", None)
        os.environ.pop("EBPF_CC_DEFER_DMA", None)
        os.environ.pop("EBPF_CC_NOHFWD", None)
        os.environ.pop("EBPF_CC_NOSHORT", None)
        os.environ.pop("EBPF_CC_PAD_SALU", None)
        os.environ.pop("EBPF_CC_PAD_VALU", None)
        launch_env = {}
        if opt.startswith("wg"):   # workgroups per CU cap at launch (occupancy / tail probe)
            launch_env["EBPF_WG_PER_CU"] = opt[2:]
        if opt.startswith("sb"):   # superblock size at launch
            launch_env["EBPF_SUPERBLOCK"] = opt[2:]
        cands.append((nm, p, data, path, launch_env))
    times = {nm: [] for nm in names}

    def launch(p, data, path, launch_env):
        select(path)
        for k in ("EBPF_WG_PER_CU", "EBPF_SUPERBLOCK"):
            if k in launch_env:
                os.environ[k] = launch_env[k]
            else:
                os.environ.pop(k, None)
        if data is d_imix:
            p.run_batch_dev(0, data.data_ptr(), n5, 0, d_ret.data_ptr(), d_imix_offs.data_ptr(), None,
                            d_hist.data_ptr(), stream.cuda_stream)
            return
        p.run_batch_dev(0, data.data_ptr(), n, 64, d_ret.data_ptr(), None, None, d_hist.data_ptr(),
                        stream.cuda_stream)

    for nm, p, data, path, le in cands:  # warm
        for _ in range(3):
            launch(p, data, path, le)
    torch.cuda.synchronize()
    for r in range(rounds):
        for nm, p, data, path, le in cands:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(launches):
                launch(p, data, path, le)
            b.record(stream)
            torch.cuda.synchronize()
            times[nm].append(a.elapsed_time(b) / launches)
    base = float(np.median(times[names[0]]))
    for nm in names:
        t = float(np.median(times[nm]))
        npk = n5 if nm.endswith("c5") or "c5:" in nm else n
        print("%-10s %.4f ms  %.1f Gpkt/s  frac %.4f  x%.3f of %s   (min %.4f max %.4f)" % (
            nm, t, npk / t / 1e6, npk * 64 / (t * 1e-3) / 8e12, t / base, names[0],
            min(times[nm]), max(times[nm])), flush=True)


if __name__ == "__main__":
    main()
