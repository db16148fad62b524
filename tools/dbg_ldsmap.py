"""Round-5 debug: compiled LDS map reads in the general kernels (c5ms probe mismatch).  r8 = the
sum of table row 0's first N words (LDXMAP through a lookup with key 0), packet loads (LDXPKC)
optionally interleaved; device r0 vs the exact sum, for several N, strides and variants."""
import sys; sys.path[:0] = ['/root/repo', '/root/repo/tests', '/root/repo/oracle']
import pkgload; pkgload.load()
import numpy as np
import stdprogs
from generic_ebpf_amd import native
I = stdprogs.I
env = native.Env()
g = np.random.default_rng(1)
for N in (8, 16, 17, 24, 32, 48, 64, 72):
    for inter in (False, True):
        for vs_words in (N, 72):
            table = g.integers(0, 2**20, (16, vs_words), dtype=np.uint32)
            items = [I("mov64_reg", 7, 1), I("mov64_imm", 5, imm=0), I("stxw", 10, 5, -4),
                     ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                     I("call", imm=0), I("mov64_imm", 8, imm=0)]
            for k in range(N):
                items += [I("ldxw", 4, 0, 4 * k), I("add64_reg", 8, 4)]
                if inter and k % 3 == 0:
                    items += [I("ldxb", 6, 7, 20 + k % 40), I("and64_imm", 6, imm=0), I("add64_reg", 8, 6)]
            items += [I("mov64_reg", 0, 8), I("exit")]
            code, rel = stdprogs.asm(items)
            want = int(table[0, :N].astype(np.uint64).sum())
            res = []
            for stride in (64, 72):
                m = native.Map(env, 16, 4 * vs_words)
                m.fill(table.tobytes())
                p = native.Prog(env, native.patch_relocs(code, rel, [m.handle]))
                p.set_semantics(native.SEM_STANDARD)
                n = 4096
                data = np.zeros(n * stride, dtype=np.uint8)
                r, f, _ = p.run_batch(data, n, stride)
                vals = np.unique(r)
                res.append("s%d:%s%s" % (stride, "ok" if (r == want).all() else "BAD", "" if (r == want).all() else
                           " got %s" % [hex(int(x)) for x in vals[:3]]))
                p.destroy()
                m.destroy()
            print("N=%d inter=%d vs=%d want=%#x %s" % (N, inter, 4 * vs_words, want, " ".join(res)), flush=True)
