"""Packet loads at run-time offsets (LDXPKTV) at every width, offset and alignment, against the
oracle (round 5: the compiled staged form, asm_cc.cpp ldxpktv_staged).  A program reads byte 1
of its packet as an offset t (& 63: unknown to the translator, so the load is LDXPKTV), then
loads z bytes at packet + t + K.  Batches where every packet has the same t take the compiled
code's register path (every running lane at one offset: the bytes straight from the staged
packet registers through GPR indexing); batches with random t take the LDS path (the
transposed packet buffer); offsets past the packet's end take the generic load and fault MEM,
as the reference's bounds check would (here: the oracle's checked mode).  Staged (64-B) and
general (72-B stride) kernels, every device variant."""
import numpy as np
import pytest

import pyoracle
import stdprogs

pytestmark = pytest.mark.gpu

I = stdprogs.I
VARIANTS = [0, 1, 2]
LDX = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}


def prog(z, K):
    """r0 = *(u{z} *)(r1 + (pkt[1] & 63) + K) ^ (pkt[1] << 56)."""
    return stdprogs.asm([
        I("ldxb", 3, 1, 1), I("mov64_reg", 4, 3), I("and64_imm", 3, imm=63),
        I("mov64_reg", 2, 1), I("add64_reg", 2, 3), I(LDX[z], 0, 2, K),
        I("lsh64_imm", 4, imm=56), I("xor64_reg", 0, 4), I("exit")])


def batches(stride, seed):
    """(name, packets): one uniform batch per offset t in 0..63 (t in byte 1 of every packet),
    and a batch with a random t per packet; 200 packets each (a partial last group)."""
    g = np.random.default_rng(seed)
    n = 200
    out = []
    for t in range(64):
        pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
        pk[:, 1] = (pk[:, 1] & 0xc0) | t
        out.append(("t=%d" % t, pk))
    out.append(("random", g.integers(0, 256, (n, stride), dtype=np.uint8)))
    return out


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 72])
@pytest.mark.parametrize("z", [1, 2, 4, 8])
def test_pktv_offsets_widths_vs_oracle(gpu, env, variant, stride, z):
    bad, faulted, clean = [], 0, 0
    for K in (0, 3, 17):
        code, rel = prog(z, K)
        p = gpu.Prog(env, code)
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            for name, pk in batches(stride, 1000 * z + K + stride):
                n = len(pk)
                want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(
                    pk.reshape(-1), n, stride, nthreads=4)
                got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, stride)
                faulted += int(np.count_nonzero(wf))
                clean += int(np.count_nonzero(wf == 0))
                if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
                    bad.append((K, name, int((want != got).sum()), int((wf != gf).sum())))
        finally:
            gpu.set_variant(0)
            p.destroy()
    assert not bad, bad
    assert faulted and clean
