"""Debug: device hashtable writes vs oracle, mismatches by (op, sel, exists)."""
import sys, collections
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import pkgload
pkgload.load()
import numpy as np
import pyoracle
import test_hash_writes as T
from generic_ebpf_amd import native as gpu

env = gpu.Env()
for ks in (4, 12):
    for variant in (1, 2, 0):
        n = 1 << 14
        spec = T._table(ks, 71, 30, 40)
        lay = T.prog_hash_writes(ks)
        op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
        pk = T._packets(n, 72)
        want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
        hm = T._device_map(gpu, env, spec)
        p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [hm.handle]))
        gpu.set_variant(variant)
        ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        gpu.set_variant(0)
        snap = spec.model()
        c = collections.Counter()
        for i in np.nonzero((ret != want) | (faults != wf))[0]:
            pp = pk[i]
            k = T._key(int.from_bytes(pp[0:4].tobytes(), "little") & 63, ks)
            o, sel = int(pp[1]) & 7, int(pp[2]) & 3
            c[(o, sel, snap.lookup(k) is not None, int(want[i]) & 0xff, int(ret[i]) & 0xff,
               int(want[i]) >> 8 == int(ret[i]) >> 8, int(wf[i]), int(faults[i]))] += 1
        walk_ok = T._walk(gpu, hm) == op.hash_models[0].items()
        print("ks", ks, "variant", variant, "mismatch", sum(c.values()), "walk_ok", walk_ok, flush=True)
        for kk, v in sorted(c.items(), key=lambda x: -x[1])[:12]:
            print("   (op, sel, exists, want_rc, got_rc, hi_ok, wf, f)", kk, v)
        p.destroy(); hm.destroy()
