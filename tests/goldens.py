"""Golden-vector fixtures: cases (program + maps + packets) with the GENUINE reference's results.

A case holds the unpatched bytecode plus LDDW map relocations [(slot, map)], because the
reference has no relocation step: a program carries raw ``struct ebpf_map*`` values in its LDDW
immediates (ebpf.h:91-98 declares resolve_map_desc, nothing calls it).  Each executor (genuine
reference, oracle, device) patches in its own map handles.

Fixtures are written by tools/gen_golden.py (container only) and stored as .npz (arrays only,
loaded with allow_pickle=False).
"""
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Case:
    def __init__(self, name, code, relocs, maps, data, count, stride, offsets,
                 expect_r0=None, expect_data=None):
        self.name = name
        self.code = bytes(code)
        self.relocs = [tuple(int(x) for x in r) for r in relocs]
        self.maps = [(int(vs), int(me), bytes(d)) for vs, me, d in maps]
        self.data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8).reshape(-1))
        self.count = int(count)
        self.stride = int(stride)
        self.offsets = None if offsets is None else np.asarray(offsets, dtype=np.uint64)
        self.expect_r0 = None if expect_r0 is None else np.asarray(expect_r0, dtype=np.uint64)
        self.expect_data = None if expect_data is None else np.asarray(expect_data,
                                                                       dtype=np.uint8)


def _cat(parts, dtype):
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    for i, p in enumerate(parts):
        offs[i + 1] = offs[i] + len(p)
    allv = np.concatenate([np.asarray(p, dtype=dtype).reshape(-1) for p in parts]) if parts \
        else np.zeros(0, dtype=dtype)
    return allv, offs


def save(path, cases):
    codes, code_off = _cat([np.frombuffer(c.code, dtype=np.uint8) for c in cases], np.uint8)
    data, data_off = _cat([c.data for c in cases], np.uint8)
    edata, _ = _cat([c.expect_data for c in cases], np.uint8)
    r0, r0_off = _cat([c.expect_r0 for c in cases], np.uint64)
    offs, offs_off = _cat([c.offsets if c.offsets is not None else np.zeros(0, np.uint64)
                           for c in cases], np.uint64)
    rel = np.array([(i, s, m) for i, c in enumerate(cases) for s, m in c.relocs],
                   dtype=np.int64).reshape(-1, 3)
    mrow = [(i, k, vs, me) for i, c in enumerate(cases) for k, (vs, me, _) in enumerate(c.maps)]
    mdat, mdat_off = _cat([np.frombuffer(d, dtype=np.uint8) for c in cases for (_, _, d) in c.maps],
                          np.uint8)
    np.savez_compressed(
        path, names=np.array([c.name for c in cases]), code=codes, code_off=code_off,
        data=data, data_off=data_off, expect_data=edata, expect_r0=r0, r0_off=r0_off,
        offsets=offs, offsets_off=offs_off,
        has_offsets=np.array([c.offsets is not None for c in cases]),
        count=np.array([c.count for c in cases], dtype=np.int64),
        stride=np.array([c.stride for c in cases], dtype=np.int64),
        relocs=rel, maps=np.array(mrow, dtype=np.int64).reshape(-1, 4), map_data=mdat,
        map_data_off=mdat_off)


def load(path):
    z = np.load(path, allow_pickle=False)
    out = []
    maps_rows = z["maps"]
    mi = 0
    for i, name in enumerate(z["names"]):
        c0, c1 = z["code_off"][i], z["code_off"][i + 1]
        d0, d1 = z["data_off"][i], z["data_off"][i + 1]
        r0a, r0b = z["r0_off"][i], z["r0_off"][i + 1]
        maps = []
        while mi < len(maps_rows) and maps_rows[mi][0] == i:
            _, k, vs, me = maps_rows[mi]
            m0, m1 = z["map_data_off"][mi], z["map_data_off"][mi + 1]
            maps.append((int(vs), int(me), z["map_data"][m0:m1].tobytes()))
            mi += 1
        rel = [(int(s), int(m)) for (ci, s, m) in z["relocs"] if ci == i]
        offsets = None
        if z["has_offsets"][i]:
            o0, o1 = z["offsets_off"][i], z["offsets_off"][i + 1]
            offsets = z["offsets"][o0:o1]
        out.append(Case(str(name), z["code"][c0:c1].tobytes(), rel, maps, z["data"][d0:d1],
                        z["count"][i], z["stride"][i], offsets, z["expect_r0"][r0a:r0b],
                        z["expect_data"][d0:d1]))
    return out


def all_golden_files():
    if not os.path.isdir(GOLDEN_DIR):
        return []
    return sorted(os.path.join(GOLDEN_DIR, f) for f in os.listdir(GOLDEN_DIR)
                  if f.endswith(".npz"))
