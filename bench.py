#!/usr/bin/env python3
"""Device-resident batch eBPF throughput on MI355X (BASELINE.json metric).

One step = one launch of the engine over the rank's whole device-resident shard of the batch
(the workload named by --config; default C4: the 64-insn VALE-BPF-style classify + one
array-map lookup per packet over 64M x 64 B synthetic packets) plus, when N > 1, the per-step
verdict histogram all-reduce (RCCL).  Packets are synthetic (seeded generator) and resident in
HBM before timing starts.

Multi-GPU (one process per GPU, torch.distributed.run): by default the config's batch is
SHARDED (--scaling strong: C4's 64M packets split in contiguous shards over the N ranks,
shard.shard_bounds, as BASELINE config 4 states); --scaling weak gives every rank a batch of
the config's size.  The only collective is the 257-bin histogram all-reduce, issued
asynchronously so that it runs under the next step's kernel.

After the timed loop the LAST timed launch is verified: its per-packet results (the whole
shard, on the GPU) and the reduced verdict histogram are compared with the CPU oracle
(oracle/, the restatement of the reference interpreter) on the distinct packets the shard
tiles; any mismatch prints the line with "verified": false and exits 1.

roofline.kernel_ms is the engine's kernel alone: HIP events that the library records on the
launch stream just before and after that kernel (ebpf_gpu_time_next_launch), so it compares
with the kernel's average in a rocprofv3 --kernel-trace --stats summary.  Every 2nd timed step
carries the events (--time-every; 10 samples in the driver's 20-step run) and kernel_ms is their
MEDIAN (the mean, min and max are in the line too; a median above ms_per_step is flagged).  roofline.traffic is measured by THIS run: two child passes
of this script under rocprofv3 --pmc (FETCH_SIZE, then WRITE_SIZE) on the same workload, after
the timed region (null if rocprofv3 is unavailable or fails; --no-pmc skips them).  Programs on
the general kernel (divergent, any packet size: C5) get a third pass (SQ_INSTS_VALU / _SALU /
_VMEM_RD) for roofline.issue, the VALU-issue floor that divergence puts under such a launch, and
a fourth (TCP tag accesses, L1->L2 requests, TD busy, GRBM active) for roofline.gather, the floor
its per-lane loads meet at the rate tools/ubench/gather.hip sustains on C5's address shape.

The same run also measures the other BASELINE configs (--also, default c2,c3,c5,c4h: C2 the
8-insn ALU program over 1M packets, C3 the 64-insn classifier over 16M, C5 the 256-insn filter over
IMIX packets, C4H the classifier with a hashtable lookup), each sharded and verified the same way and
reported under "also" with its own roofline -- so the driver's 1/2/4/8-GPU runs carry every config
at every N.

`bench.py --gpus N` with N > 1 and no launcher around it starts its N ranks itself
(torch.distributed.run in a child process, self_launch); under a launcher WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pkgload  # noqa: E402

pkg = pkgload.load()
from generic_ebpf_amd import native, shard, workloads  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SIMDS, CLOCK_GHZ, VALU_ISSUE_CYCLES = 256 * 4, 2.4, 4  # MI355X: 256 CUs x 4 SIMD16, wave64 VALU
ISSUE_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD")
# the gather roofline of a general-kernel line (per-lane loads at run-time addresses): TCP tag
# accesses (a lane's load is one per 128-B line it touches), L1->L2 read requests, TD busy
# cycles (summed over the 256 TDs) and GRBM active cycles (summed over the 8 XCDs), one pass
GATHER_COUNTERS = ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TD_TD_BUSY_sum",
                   "GRBM_GUI_ACTIVE")
# Tag accesses per CU cycle the chip sustains on C5's address shape with every lane active:
# tools/ubench/gather.hip mode 'i' (IMIX 64/576/1500 B packets, 26 loads of 1-8 B per lane at
# per-class offsets drawn as C5's leaves draw theirs, no divergence, no other work), best
# occupancy (4 waves per CU: 0.511-0.545 over 7 launches, median 0.517); 16-24 waves per CU,
# where more lines miss L1, sustain 0.37-0.42 (profiles/r06/gather/README.md)
GATHER_ACCESSES_PER_CU_CYCLE = 0.517
CUS = 256
METRIC = "Mpkt/s device-resident (64-insn filter, 64B pkts); achieved HBM GB/s vs peak"
# Round-1 calibration in the build container, C4, 1 thread: the genuine reference libebpf.so
# 9.1 Mpkt/s, this oracle (port) 7.6 Mpkt/s
PORT_VS_REFERENCE = round(7.6 / 9.1, 3)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c4", choices=sorted(workloads.CONFIGS))
    ap.add_argument("--packets", type=int, default=0,
                    help="packets of the whole batch (strong) or per GPU (weak); default per config")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the batch is sharded over the ranks (default); weak: each rank its own batch")
    ap.add_argument("--variant", type=int, default=0,
                    help="0 = compiled (default), 1 = portable HIP, 2 = assembly interpreter")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU baseline budget (half all-threads, half one pinned thread)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the oracle check (PMC child passes)")
    ap.add_argument("--no-pmc", action="store_true", help="no rocprofv3 --pmc passes for roofline.traffic")
    ap.add_argument("--pmc-dir", default="", help="where the PMC passes write (default: a temp dir)")
    ap.add_argument("--time-every", type=int, default=2,
                    help="event-time the kernel of every k-th timed step (default 2: the events come from the kernel's own dispatch packet, ebpf_gpu_time_next_launch, so a timed step costs no extra GPU-side marker)")
    ap.add_argument("--sync-each", action="store_true",
                    help="diagnostics: synchronise after every step (launches never queue)")
    ap.add_argument("--also", default="c2,c3,c5,c4h,c4c,c3l",
                    help="comma-separated further configs measured in the same run (sharded the same way) "
                         "and reported under 'also' (default: every other BASELINE config -- C2, C3, C5 "
                         "the IMIX filter -- C4H, the hashtable form of C4, C4C, C4 with a per-key "
                         "counter update, and C3L, a bounded loop under standard semantics); '' for none")
    ap.add_argument("--also-min-ms", type=float, default=60.0,
                    help="an --also config whose --steps would time less than this many ms runs more "
                         "steps (up to --also-max-steps; its line says how many): a 20-step timed region "
                         "of a 15-us launch is 0.3 ms, where one host hiccup or the first launch's "
                         "latency decides the number")
    ap.add_argument("--also-max-steps", type=int, default=4000)
    ap.add_argument("--launch", default="eager", choices=["graph", "eager"],
                    help="eager: direct launches (default); graph: each step replays a captured HIP graph (measured 1.6%% slower on C2-C4, profiles/r01/graph_ab)")
    return ap.parse_args(argv)


DEFAULT_PACKETS = {"nop200": 1 << 24, "alu200": 1 << 24, "c0": 1 << 26, "c2": 1 << 20, "c3": 1 << 24,
                   "c4": 1 << 26, "c4c": 1 << 26, "c3l": 1 << 24, "c5": 1 << 22, "c4h": 1 << 26, "c3lit": 1 << 24,
                   "c5lit": 1 << 22, "c5d0": 1 << 22, "c5d1": 1 << 22, "c5ms": 1 << 22,
                   "c5b2": 1 << 22, "c5b0": 1 << 22}
# C4H: bytes one lookup must move.  The device table's slot is 32 B (u32 used | u32 hash | 4-B key
# 8-B padded | 8-B value), but a random probe cannot fetch less than one 64-B line from HBM: the
# PMC passes measured 64 B per lookup (FETCH_SIZE, profiles/r02/s3/all/bench_c4h_slots8.json:
# 7.79 GB per launch = 4.29 GB packets + 0.54 GB results + 64 B x 46.1M lookups), so the roofline
# counts the line (round 2 counted the slot's 32 B)
C4H_PROBE_BYTES = 64
DISTINCT = 1 << 22  # distinct synthetic packets generated on the host, tiled in HBM


class Workload:
    """The rank's part [lo, hi) of the global batch.  Fixed-size configs: global packet g is
    distinct[g % D] (D distinct packets generated once, the same on every rank).  C5: an
    IMIX stream generated in blocks, so a shard is the same bytes whatever N."""

    def __init__(self, cfg, lo, hi, total):
        self.cfg, self.lo, self.hi = cfg, lo, hi
        self.n = hi - lo
        self.lay = workloads.CONFIGS[cfg]["prog"]()
        # 0: the reference's stepping; 1: standard eBPF (ebpf_prog_set_semantics: C3L's loop)
        self.semantics = workloads.CONFIGS[cfg].get("semantics", 0)
        self.maps = []
        self.offs = None
        if workloads.CONFIGS[cfg]["pkt"] == "imix":
            self.pk, self.offs, _ = workloads.packets_imix_range(lo, hi, seed=5)
            if cfg == "c5ms":  # (probe: the melded leaves' operand table)
                t = workloads.c5meldsim_table()
                self.maps = [(4 * t.shape[1], 16, t.tobytes())]
            self.D = self.n
            return
        self.D = min(total, DISTINCT)
        if cfg == "c4":
            self.maps = [(8, 256, workloads.c4_map_values().tobytes())]
        if cfg == "c4c":  # + the per-key packet counters, from zero
            self.maps = [(8, 256, workloads.c4_map_values().tobytes()), (8, 256, bytes(8 * 256))]
        if cfg == "c4h":  # ("hash", key_size, value_size, max_entries, keys, values)
            universe, keys, values = workloads.c4h_table()
            self.maps = [("hash", 4, 8, len(keys), keys, values)]
            self.pk = workloads.packets_c4h(self.D, universe, seed=4)
            return
        if cfg == "c3l":
            self.pk = workloads.packets_ipv4opt(self.D)
            return
        rnd = cfg in ("c0", "c2", "nop200", "alu200")
        gen = workloads.packets_random if rnd else workloads.packets_l2l3
        self.pk = gen(self.D, 64, seed=2 if rnd else 3)

    def device_packets(self, torch, dev):
        """(packets on dev, offsets on dev or None) for this shard."""
        if self.offs is not None:
            return (torch.from_numpy(self.pk).to(dev),
                    torch.from_numpy(self.offs.view(np.int64)).to(dev))
        base = torch.from_numpy(self.pk).to(dev)           # D x 64
        s = self.lo % self.D
        if s:
            base = torch.cat([base[s:], base[:s]])
        reps = (self.n + self.D - 1) // self.D
        d_pk = (base.repeat(reps, 1)[: self.n] if reps > 1 else base[: self.n]).contiguous()
        return d_pk.reshape(-1), None

    def algorithmic_bytes(self):
        if self.offs is not None:
            # sum of min(len, W) rounded up to 64 B (W = the program's largest
            # load extent; C5 reads anywhere in its packets) + the offsets array
            lens = np.diff(self.offs)
            w = workloads.CONFIGS[self.cfg].get("extent")
            if w is not None:
                lens = np.minimum(lens, (w + 63) // 64 * 64)
            return int(lens.sum()) + 8 * (self.n + 1)
        b = self.n * 64
        if self.cfg == "c4h":  # + one table line per packet that reaches the lookup (IPv4, not ICMP)
            pk = self.pk
            et = (pk[:, 12].astype(np.uint32) << 8) | pk[:, 13]
            reach = float(np.mean((et == 0x0800) & (pk[:, 23] != 1)))
            b += int(round(self.n * reach) * C4H_PROBE_BYTES)
        return b

    def oracle_maps(self):
        import pyoracle
        return [pyoracle.HashSpec(m[1], m[2], keys=m[4], values=m[5]) if m[0] == "hash" else m
                for m in self.maps]


def make_maps(env, spec):
    maps = []
    for s in spec:
        if s[0] == "hash":
            _, ks, vs, me, keys, values = s
            m = native.HashMap(env, ks, vs, me)
            m.fill(keys, values)
        else:
            vs, me, d = s
            m = native.Map(env, me, vs)
            m.fill(d)
        maps.append(m)
    return maps


def oracle_threads():
    """Host threads for the oracle: the CPU share this process may use (OMP_NUM_THREADS is set
    to the box's share on the GPU pool; else the affinity mask)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(aff, int(env))) if env.isdigit() and int(env) > 0 else aff


def verify(w, torch, d_ret, d_hist_total, world, dev):
    """Compare the last launch's results on the device with the oracle.  Returns (ok, info)."""
    import pyoracle
    op = pyoracle.OracleProgram(w.lay.code, w.lay.relocs, w.oracle_maps(), checked=True,
                                semantics=w.semantics)
    thr = oracle_threads()
    if w.offs is not None:
        want, wf, _, _ = op.run(w.pk, w.n, 0, w.offs, nthreads=thr)
    else:
        want, wf, _, _ = op.run(w.pk, w.D, 64, None, nthreads=thr)
    # per-packet results: a fixed-size config's shard tiles want[] starting at lo % D; an IMIX
    # shard is its own packets (D = n: no rotation, whatever lo)
    wt = torch.from_numpy(want.view(np.int64)).to(dev)
    s = w.lo % w.D if w.offs is None else 0
    if s:
        wt = torch.cat([wt[s:], wt[:s]])
    got = d_ret[: w.n]
    k, r = divmod(w.n, w.D)
    bad = 0
    if k:
        bad += int((got[: k * w.D].view(k, w.D) != wt.unsqueeze(0)).sum())
    if r:
        bad += int((got[k * w.D:] != wt[:r]).sum())
    # histogram of the shard: bin min(r0, 255), faulted packets in bin 256
    cnt = np.full(w.D, k, dtype=np.int64)
    cnt[(s + np.arange(r)) % w.D] += 1
    bins = np.where(wf != 0, 256, np.minimum(want, 255)).astype(np.int64)
    exp = np.bincount(bins, weights=cnt, minlength=257).astype(np.int64)
    exp_t = torch.from_numpy(exp).to(dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(exp_t)
        b = torch.tensor([bad], dtype=torch.int64, device=dev)
        dist.all_reduce(b)
        bad = int(b[0])
    hist_bad = int((d_hist_total != exp_t).sum())
    info = {"verified": bad == 0 and hist_bad == 0, "ret_mismatches": bad,
            "hist_mismatched_bins": hist_bad,
            "oracle_packets": int(w.n if w.offs is not None else w.D)}
    return info["verified"], info


def verify_counters(w, maps, launches):
    """C4C: the counters map after `launches` launches over the shard equals the oracle's count of
    the packets that reached the counter update (ebpf_gpu.h: counter updates are additions, so
    the map ends as the reference's sequential run leaves it), for every key."""
    import pyoracle
    s, (k, r) = w.lo % w.D, divmod(w.n, w.D)

    def once(pk):
        spec = [w.maps[0], (8, 256, bytes(8 * 256))]
        op = pyoracle.OracleProgram(w.lay.code, w.lay.relocs, spec)
        op.run(pk, len(pk), 64, nthreads=oracle_threads())
        return np.frombuffer(op.map_bytes(1), dtype=np.uint64).astype(object)
    per = once(w.pk) * k if k else 0
    if r:
        per = per + once(w.pk[(s + np.arange(r)) % w.D])
    want = [int(x) * launches % (1 << 64) for x in per]
    got = [int(np.frombuffer(maps[1].lookup(key)[1], dtype=np.uint64)[0]) for key in range(256)]
    return {"counters_verified": got == want, "counted_per_launch": int(sum(int(x) for x in per)),
            "counter_mismatches": sum(1 for a, b in zip(got, want) if a != b)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w, budget_s):
    """The oracle (the CPU restatement of the reference interpreter in raw-pointer mode, the
    reference's cost model) on a bounded sample of the same workload, run in place on
    preallocated buffers: (i) every thread of this process's CPU share, contiguous shards
    (OpenMP static schedule); (ii) one thread pinned to one core."""
    import pyoracle
    if w.offs is not None:
        n = min(w.n, 1 << 18)
        data = np.ascontiguousarray(w.pk[: int(w.offs[n])])
        offsets = np.ascontiguousarray(w.offs[: n + 1], dtype=np.uint64)
        stride = 0
    else:
        n = min(w.D, 1 << 20)
        data = np.ascontiguousarray(w.pk[:n].reshape(-1))
        offsets, stride = None, 64
    # no configured program stores to packet bytes, so passes over the same buffer are identical
    op = pyoracle.OracleProgram(w.lay.code, w.lay.relocs, w.oracle_maps(), checked=False,
                                semantics=w.semantics)
    ret = np.zeros(n, dtype=np.uint64)

    def timed(threads, seconds):
        op.run_inplace(data, n, stride, offsets, ret, None, threads)  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            op.run_inplace(data, n, stride, offsets, ret, None, threads)
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return n * passes / el / 1e6, passes, el

    thr = oracle_threads()
    multi, mp, mel = timed(thr, budget_s / 2)
    old = os.sched_getaffinity(0)
    core = min(old)
    try:
        os.sched_setaffinity(0, {core})
        single, sp, sel = timed(1, budget_s / 2)
    finally:
        os.sched_setaffinity(0, old)
    return {"value": round(multi, 2), "unit": "Mpkt/s", "cores": thr, "kind": "port",
            "single_thread_value": round(single, 2), "single_thread_core": core,
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "port_vs_reference": PORT_VS_REFERENCE,
            "sample": "%d %s packets (%s) run in place: %d passes on %d threads in %.1f s; "
                      "%d passes on 1 thread pinned to CPU %d in %.1f s" % (
                          n, w.cfg.upper(), "IMIX" if offsets is not None else "64 B",
                          mp, thr, mel, sp, core, sel)}


DIST_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def pmc_traffic(a, w, total, layout, cfg=None):
    """HBM bytes per launch of the engine's kernel, from two rocprofv3 --pmc child passes of
    this script on the same workload (each counter group in a run of its own, kernel trace
    only besides --pmc: MI355X_MICROARCH.md, HBM/rocprofv3).  FETCH_SIZE/WRITE_SIZE are KiB;
    gfx950's FETCH_SIZE reports half of a 16-B/lane streaming read, so the staged kernels'
    packet DMA (layout 1) gets its other half added back."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    cfg = cfg or a.config
    out = a.pmc_dir or tempfile.mkdtemp(prefix="ebpf_pmc_")
    child = [sys.executable, os.path.abspath(__file__), "--config", cfg, "--packets",
             str(total), "--steps", "2", "--warmup", "1", "--variant", str(a.variant),
             "--no-cpu-baseline", "--no-pmc", "--no-verify", "--also="]
    vals = {}
    # general kernels (divergent programs): also the instruction counts of the issue roofline
    passes = [("FETCH_SIZE",), ("WRITE_SIZE",)]
    if layout == 0:
        passes += [ISSUE_COUNTERS, GATHER_COUNTERS]
    for group in passes:
        counter = group[0]
        d = os.path.join(out, "pmc_%s_%s" % (cfg, counter))
        os.makedirs(d, exist_ok=True)
        cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc"] + list(group) + ["--kernel-trace",
               "--kernel-include-regex", "ebpf_(interp|jit)", "--output-format", "csv",
               "-d", d, "-o", "pmc", "--"] + child
        # (a single-process child: at N > 1 rank 0 measures its own shard's launch on its GPU, so
        # the launcher's rendezvous variables are not passed on)
        env = {k: v for k, v in os.environ.items() if k not in DIST_ENV and not k.startswith("TORCHELASTIC_")}
        env["TMPDIR"] = os.environ.get("TMPDIR", "/tmp")
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
        if r.returncode != 0:
            return None, "%s pass exited %d: %s" % (counter, r.returncode,
                                                     r.stderr.decode(errors="replace")[-300:])
        for c in group:
            per = {}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        kn = row.get("Kernel_Name", "")
                        if row.get("Counter_Name") != c or not (
                                "ebpf_interp" in kn or "ebpf_jit" in kn):
                            continue
                        per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
            if not per:
                return None, "%s pass recorded no engine dispatch" % c
            vals[c] = sum(per.values()) / len(per) * (1024.0 if c.endswith("_SIZE") else 1.0)
    fetch = vals["FETCH_SIZE"]
    note = "FETCH_SIZE + WRITE_SIZE per launch, this run"
    if layout == 1:
        fetch += w.n * 64 / 2.0
        note += "; staged 64-B packet DMA: half its bytes added (gfx950 16-B/lane undercount)"
    return {"bytes": fetch + vals["WRITE_SIZE"], "fetch_reported": vals["FETCH_SIZE"],
            "write": vals["WRITE_SIZE"], "note": note,
            "insts": {c: vals[c] for c in ISSUE_COUNTERS + GATHER_COUNTERS if c in vals}}, None


def issue_roofline(insts, kern_ms, groups):
    """The second roofline of a divergent program (general kernels): VALU issue.  A wave64
    VALU instruction occupies its SIMD (16 lanes wide) for 4 cycles, so the launch cannot
    finish before SQ_INSTS_VALU x 4 / (SIMDs x clock) (MI355X: 256 CUs x 4 SIMDs, 2.4 GHz
    peak engine clock; MI355X_MICROARCH.md).  Divergence multiplies the VALU count: every path
    a 64-packet group takes is issued once for the whole wave."""
    valu = insts.get("SQ_INSTS_VALU")
    if not valu:
        return None
    floor_ms = valu * VALU_ISSUE_CYCLES / (SIMDS * CLOCK_GHZ * 1e9) * 1e3
    return {"bound": "valu-issue", "valu_insts": int(valu),
            "valu_per_group": round(valu / max(1, groups), 1),
            "salu_per_group": round(insts.get("SQ_INSTS_SALU", 0) / max(1, groups), 1),
            "vmem_rd_per_group": round(insts.get("SQ_INSTS_VMEM_RD", 0) / max(1, groups), 1),
            "floor_ms": round(floor_ms, 4), "kernel_ms": round(kern_ms, 4),
            "frac": round(floor_ms / kern_ms, 4) if kern_ms > 0 else None,
            "model": "SQ_INSTS_VALU x %d cycles / (%d SIMDs x %.1f GHz), this run's PMC pass" % (
                VALU_ISSUE_CYCLES, SIMDS, CLOCK_GHZ)}


def gather_roofline(insts, kern_ms, groups):
    """The roofline of per-lane gathers (general kernels): a launch cannot
    finish before its TCP tag accesses pass at the rate the chip sustains on the same address
    shape with every lane active and nothing else to do (GATHER_ACCESSES_PER_CU_CYCLE, measured
    by tools/ubench/gather.hip), at the peak engine clock on every CU.  Beside it: how busy the
    texture data path was (TD busy cycles per TD / GRBM active cycles per XCD), the L1 miss ratio
    and the accesses per 64-packet group."""
    acc = insts.get("TCP_TOTAL_CACHE_ACCESSES_sum")
    if not acc:
        return None
    floor_ms = acc / (GATHER_ACCESSES_PER_CU_CYCLE * CUS * CLOCK_GHZ * 1e9) * 1e3
    grbm = insts.get("GRBM_GUI_ACTIVE", 0) / 8.0
    td = insts.get("TD_TD_BUSY_sum", 0) / CUS
    req = insts.get("TCP_TCC_READ_REQ_sum", 0)
    return {"bound": "gather", "tag_accesses": int(acc), "accesses_per_group": round(acc / max(1, groups), 1),
            "l1_miss_ratio": round(req / acc, 4), "td_busy": round(td / grbm, 4) if grbm else None,
            "accesses_per_cu_cycle": round(acc / (grbm * CUS), 4) if grbm else None,
            "floor_ms": round(floor_ms, 4), "kernel_ms": round(kern_ms, 4),
            "frac": round(floor_ms / kern_ms, 4) if kern_ms > 0 else None,
            "model": "TCP_TOTAL_CACHE_ACCESSES / (%.3f per CU cycle x %d CUs x %.1f GHz): "
                     "tools/ubench/gather.hip mode i, this run's PMC pass" % (
                         GATHER_ACCESSES_PER_CU_CYCLE, CUS, CLOCK_GHZ)}


def measure(a, cfg, packets, torch, dist, world, rank, local, dev, also=False):
    """One configuration on this rank: build its shard, warm up, time a.steps launches (barrier
    and max over ranks), verify the last launch.  Returns the numbers of the JSON line.  An
    --also config (also=True) times at least --also-min-ms of steps (see parse)."""
    size = packets or DEFAULT_PACKETS[cfg]
    if a.scaling == "strong":
        total = size
        lo, hi = shard.shard_bounds(total, rank, world)
    else:
        total = size * world
        lo, hi = rank * size, (rank + 1) * size
    w = Workload(cfg, lo, hi, size if a.scaling == "weak" else total)
    n = w.n

    env = native.Env()
    maps = make_maps(env, w.maps)
    prog = native.Prog(env, native.patch_relocs(w.lay.code, w.lay.relocs, [m.handle for m in maps]))
    if w.semantics:
        prog.set_semantics(native.SEM_STANDARD)
    native.set_variant(a.variant)
    prog.prepare(local)

    d_pk, d_offs = w.device_packets(torch, dev)
    bytes_per_launch = w.algorithmic_bytes()
    d_ret = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    # two histogram buffers: the all-reduce of step i (N > 1) overlaps the launch of step i + 1
    hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(2)]
    red = shard.OverlappedHistReduce(hists)
    stream = torch.cuda.current_stream()
    # the launch sets its histogram to this batch's counts (no memset first)
    launch = prog.launcher(local, d_pk.data_ptr(), n, 64, d_ret.data_ptr(),
                           None if d_offs is None else d_offs.data_ptr(), None,
                           stream.cuda_stream, hist_overwrite=True)
    hptr = [h.data_ptr() for h in hists]

    # HIP graphs (one per histogram buffer): the launch replays as one submission
    graphs = None
    if a.launch == "graph":
        launch(hptr[0])  # map mirrors uploaded, program compiled
        torch.cuda.synchronize()
        try:
            graphs = []
            for p in hptr:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    prog.run_batch_dev(local, d_pk.data_ptr(), n, 64, d_ret.data_ptr(),
                                       None if d_offs is None else d_offs.data_ptr(), None, p,
                                       torch.cuda.current_stream().cuda_stream,
                                       hist_overwrite=True)
                graphs.append(g)
        except Exception as e:  # capture unsupported: eager launches, said in the bench line
            print("graph capture failed (%s); eager launches" % e, file=sys.stderr)
            graphs = None
            torch.cuda.synchronize()

    def step(i, ev=None):
        b = red.acquire(i)
        if graphs is not None:  # events around the replay
            if ev is not None:
                ev[0].record(stream)
            graphs[b].replay()
            if ev is not None:
                ev[1].record(stream)
        else:
            if ev is not None:  # the library records them around the engine's kernel alone
                native.time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
            launch(hptr[b])
        red.issue(b)
        if a.sync_each:
            torch.cuda.synchronize()

    for i in range(a.warmup):
        step(i)
    red.finish()
    torch.cuda.synchronize()
    steps = a.steps
    if also and a.also_min_ms > 0:
        # a few more warm steps estimate the step; the count is the same on every rank (max)
        t_est = time.perf_counter()
        for i in range(10):
            step(i)
        red.finish()
        torch.cuda.synchronize()
        est_ms = (time.perf_counter() - t_est) * 1e3 / 10
        want = int(np.ceil(a.also_min_ms / max(est_ms, 1e-3)))
        steps = max(a.steps, min(a.also_max_steps, want))
        if world > 1:
            t = torch.tensor([steps], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            steps = int(t[0])
    timed = list(range(0, steps, max(1, a.time_every)))  # steps whose kernel is event-timed
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in timed]
    for e0, e1 in evs:  # torch creates its events at their first record
        e0.record(stream)
        e1.record(stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 0
    for i in range(steps):
        if k < len(timed) and timed[k] == i:
            step(i, evs[k])
            k += 1
        else:
            step(i)
    d_hist = red.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_samples = [s.elapsed_time(e) for s, e in evs]
    kern_ms = float(np.median(kern_samples))
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])
    ms_per_step = el * 1e3 / steps
    value = total * steps / el / 1e6
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    exec_name, layout, translate_ms, build_ms = prog.exec_info(local)

    hist = d_hist.cpu().numpy()
    faulted = int(hist[256])
    vinfo = {"verified": None}
    ok = True
    if not a.no_verify:  # the last timed launch against the oracle (outside the timing)
        ok, vinfo = verify(w, torch, d_ret, d_hist, world, dev)
        if cfg == "c4c":
            c = verify_counters(w, maps, a.warmup + steps + (10 if also and a.also_min_ms > 0 else 0) +
                                (1 if graphs is not None else 0))
            vinfo.update(c)
            ok = ok and c["counters_verified"]
            vinfo["verified"] = ok
    elif int(hist.sum()) != total:
        ok = False
        vinfo = {"verified": False, "hist_total": int(hist.sum())}
    info = prog.info()
    prog.destroy()
    for m in maps:
        m.destroy()
    env.destroy()
    return dict(w=w, n=n, total=total, value=value, ms_per_step=ms_per_step, kern_ms=kern_ms,
                achieved=achieved, bytes_per_launch=bytes_per_launch, exec_name=exec_name,
                layout=layout, translate_ms=translate_ms, build_ms=build_ms, faulted=faulted,
                vinfo=vinfo, ok=ok, nentries=info.nentries, graph=graphs is not None,
                samples=len(evs), kern_stats=kernel_stats(kern_samples, ms_per_step), steps=steps)


def kernel_stats(samples, ms_per_step):
    """The event-timed kernel durations of this rank: how many, their mean / min / max, and
    whether the median exceeds the step (it cannot, for back-to-back launches on one stream,
    unless the sample is unrepresentative)."""
    med = float(np.median(samples))
    return {"n": len(samples), "median": round(med, 4), "mean": round(float(np.mean(samples)), 4),
            "min": round(float(np.min(samples)), 4), "max": round(float(np.max(samples)), 4),
            "median_exceeds_step": bool(med > ms_per_step)}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(a):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N ranks, one process per
    GPU, as `python -m torch.distributed.run --nproc-per-node N bench.py ...` in a fresh child
    process (nothing here has touched the GPU yet: torch.cuda.device_count() does not initialise
    it), let rank 0's JSON line through on the inherited stdout and return the child's exit
    code.  Fewer visible GPUs than N is an error, except in the gloo rehearsal
    (EBPF_BENCH_BACKEND=gloo), where the ranks share the visible GPUs."""
    import torch
    ngpu = torch.cuda.device_count()
    backend = os.environ.get("EBPF_BENCH_BACKEND", "nccl")
    if ngpu < a.gpus and not (backend == "gloo" and ngpu >= 1):
        print("bench.py: --gpus %d but %d GPU(s) visible" % (a.gpus, ngpu), file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % a.gpus, "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(self_launch(a))
    if world_env is not None and int(world_env) != a.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (world_env, a.gpus), file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("EBPF_BENCH_BACKEND", "nccl")
    if world > 1 and backend == "gloo":   # rehearsal of N > 1 with every rank on one GPU
        local = local % max(1, torch.cuda.device_count())
    # the rank's GPU is bound before the process group exists, so that RCCL's communicator and
    # its barrier use this device (not a guess from the rank number)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # nccl (= RCCL) on the node; EBPF_BENCH_BACKEND=gloo rehearses N > 1 on one GPU
        dist.init_process_group(backend)
    R = measure(a, a.config, a.packets, torch, dist, world, rank, local, dev)
    ok = R["ok"]
    w, n, total, layout, kern_ms = R["w"], R["n"], R["total"], R["layout"], R["kern_ms"]
    cfg = a.config
    # further BASELINE configurations measured in the same run, sharded the same way (a line of
    # their own under "also"; a failed check there is reported, it does not void the line)
    also = {}
    for c in [x for x in a.also.split(",") if x and x != cfg]:
        try:
            S = measure(a, c, 0, torch, dist, world, rank, local, dev, also=True)
        except Exception as e:  # reported in the line; the primary measurement stands
            also[c] = {"error": "%s: %s" % (type(e).__name__, e)}
            continue
        if rank == 0 and not a.no_pmc:  # the same PMC passes as the primary line
            t, err = pmc_traffic(a, S["w"], S["n"] if world > 1 else S["total"], S["layout"], c)
            S["traffic"], S["traffic_note"] = (t["bytes"], t["note"]) if t else (None, err)
            S["issue"] = (issue_roofline(t["insts"], S["kern_ms"], (S["n"] + 63) // 64)
                          if t and t["insts"] else None)
            S["gather"] = (gather_roofline(t["insts"], S["kern_ms"], (S["n"] + 63) // 64)
                           if t and t["insts"] else None)
        also[c] = {"value": round(S["value"], 1), "unit": "Mpkt/s", "ms_per_step": round(S["ms_per_step"], 4),
                   "steps": S["steps"], "warmup": a.warmup + 10,
                   "packets_total": S["total"], "packets_per_gpu": S["n"], "verified": S["vinfo"].get("verified"),
                   "check": S["vinfo"], "exec": S["exec_name"],
                   "kernel_layout": "staged64" if S["layout"] == 1 else "general",
                   "roofline": {"bound": "hbm", "achieved": round(S["achieved"], 1), "peak": PEAK_HBM_GBS,
                                "unit": "GB/s", "frac": round(S["achieved"] / PEAK_HBM_GBS, 4),
                                "kernel_ms": round(S["kern_ms"], 4), "kernel_ms_stats": S["kern_stats"],
                                "traffic": S.get("traffic"),
                                "traffic_note": S.get("traffic_note", "disabled (--no-pmc)"),
                                "algorithmic_bytes_per_launch": S["bytes_per_launch"],
                                "issue": S.get("issue"), "gather": S.get("gather")},
                   "desc": workloads.CONFIGS[c]["desc"]}

    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(w, a.cpu_seconds)
        traffic, pmc_note = None, "disabled (--no-pmc)"
        issue = gather = None
        if not a.no_pmc:   # (N > 1: rank 0's shard, one launch on its GPU, as the roofline's)
            t, err = pmc_traffic(a, w, n if world > 1 else total, layout)
            traffic, pmc_note = (t["bytes"], t["note"]) if t else (None, err)
            if t and t["insts"]:
                issue = issue_roofline(t["insts"], kern_ms, (n + 63) // 64)
                gather = gather_roofline(t["insts"], kern_ms, (n + 63) // 64)
        out = {
            "metric": METRIC,
            "value": round(R["value"], 1), "unit": "Mpkt/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(R["ms_per_step"], 4), "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "verified": R["vinfo"].get("verified"),
            "config": {"workload": cfg, "desc": workloads.CONFIGS[cfg]["desc"],
                       "packets_total": total, "packets_per_gpu": n,
                       "packet_bytes": 64 if w.offs is None else "IMIX",
                       "main_path_insns": w.lay.main_path_steps, "prog_slots": w.lay.nslots,
                       "dprog_entries": R["nentries"], "variant": a.variant,
                       "exec": R["exec_name"], "kernel_layout": "staged64" if layout == 1 else "general",
                       "translate_ms": round(R["translate_ms"], 3), "build_ms": round(R["build_ms"], 3),
                       "parallelism": "dp%d" % world,
                       "launch": "graph" if R["graph"] else "eager",
                       "faulted_packets": R["faulted"]},
            "check": R["vinfo"],
            "roofline": {"bound": "hbm", "achieved": round(R["achieved"], 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(R["achieved"] / PEAK_HBM_GBS, 4),
                         "traffic": traffic, "traffic_note": pmc_note,
                         "kernel_ms": round(kern_ms, 4), "kernel_ms_samples": R["samples"],
                         "kernel_ms_stats": R["kern_stats"],
                         "algorithmic_bytes_per_launch": R["bytes_per_launch"],
                         "issue": issue, "gather": gather},
            "cpu_baseline": cpu,
            "also": also,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
