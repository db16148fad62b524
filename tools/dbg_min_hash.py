"""Debug: shrink a variant-0 mismatch of the hashtable fuzz mode (tools/fuzz_gpu.py --hash) to a
small program by replacing slots with the reference's no-op (LE r0, 64) while the mismatch stays.

  python tools/dbg_min_hash.py K [staged|general]
Prints the shrunk program (one slot per line, hex) and the device / oracle results."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
k = int(sys.argv[1])
lay = sys.argv[2] if len(sys.argv) > 2 else "staged"
sys.argv = sys.argv[:1]
import numpy as np  # noqa: E402
import fuzz_gpu as F  # noqa: E402
from generic_ebpf_amd import native, isa  # noqa: E402

env = native.Env()
NOP = isa.encode(0xd4, 0, 0, 0, 64)  # LE r0, 64


def defined(c):
    """no result depends on the initial stack or registers (the reference leaves them undefined)"""
    import pyoracle
    outs, keep = [], []
    # (thread count: the stack slices and the packet copy move, so a result that depends on a
    # stack or packet address changes too)
    for si, ri, nt in ((0, 0, 1), (0xa5, 0, 2), (0, 0x77, 3)):
        op = pyoracle.OracleProgram(c.code, c.relocs, c.maps, stack_init=si, reg_init=ri,
                                    track_undef=True)
        ret, faults, data, _ = op.run(c.data, c.count, c.stride, c.offsets, nthreads=nt)
        if (faults == 100).any():
            return False
        keep.append(data)
        outs.append((ret.tobytes(), faults.tobytes(), data.tobytes()))
    return outs[0] == outs[1] == outs[2]


def bad(c):
    if not defined(c):
        return False
    want, wf, wdata, wmaps = F.oracle(c)
    try:
        got, gf, gdata, gmaps = F.device(env, c, 0)
    except Exception as e:  # noqa: BLE001
        return False
    return not (np.array_equal(want, got) and np.array_equal(wf, gf) and
                np.array_equal(wdata, gdata) and wmaps == gmaps)


c = F.case(k, 1, lay, True)
assert bad(c), "case does not fail"
code = bytearray(c.code)
relocs = list(c.relocs)
nslots = len(code) // 8
changed = True
while changed:
    changed = False
    for i in range(nslots):
        if code[8 * i:8 * i + 8] == NOP:
            continue
        if any(r[0] == i or r[0] + 1 == i for r in relocs if isinstance(r, tuple)):
            continue
        old = bytes(code[8 * i:8 * i + 8])
        code[8 * i:8 * i + 8] = NOP
        c.code = bytes(code)
        if bad(c):
            changed = True
        else:
            code[8 * i:8 * i + 8] = old
c.code = bytes(code)
print("relocs", relocs)
for i in range(nslots):
    s = code[8 * i:8 * i + 8]
    if s != NOP:
        print("%3d %s" % (i, s.hex()))
want, wf, _, wm = F.oracle(c)
got, gf, _, gm = F.device(env, c, 0)
d = np.nonzero(want != got)[0]
print("count", c.count, "mismatching", len(d))
for i in d[:4]:
    print("pkt %d want %x got %x" % (i, int(want[i]), int(got[i])))
print("maps equal", wm == gm, "faults want", np.unique(wf, return_counts=True), "got",
      np.unique(gf, return_counts=True))
with open("gpurun_out/min_%d_%s.bin" % (k, lay), "wb") as fh:
    fh.write(c.code)
