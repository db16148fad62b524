"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/ebpf_oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker or the
timed CPU baseline; the product (generic-ebpf_amd/) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

HELPER_UNSET, HELPER_MAP_LOOKUP, HELPER_OTHER = 0, 1, 2


class _Map(ctypes.Structure):
    _fields_ = [("handle", ctypes.c_uint64), ("data", ctypes.c_void_p),
                ("value_size", ctypes.c_uint32), ("max_entries", ctypes.c_uint32)]


class _Prog(ctypes.Structure):
    _fields_ = [("insns", ctypes.c_void_p), ("nslots", ctypes.c_uint64),
                ("helper_kind", ctypes.c_uint8 * 64), ("maps", ctypes.c_void_p),
                ("nmaps", ctypes.c_uint32), ("reg_init", ctypes.c_uint64),
                ("stack_init", ctypes.c_uint8), ("checked", ctypes.c_uint8)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.oracle_run_batch.restype = ctypes.c_uint64
        _lib.oracle_run_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int]
    return _lib


# Fake but distinct LDDW handles for oracle maps (the reference uses struct ebpf_map* values).
def oracle_handle(k):
    return 0x00007f5e00001000 + 0x100 * k


class OracleProgram:
    """A program + its maps, ready to run on the oracle.  ``code`` is unpatched; relocations
    [(slot, map_index)] are patched with oracle handles here."""

    def __init__(self, code, relocs=(), maps=(), helper_kinds=None, checked=True,
                 reg_init=0, stack_init=0):
        b = bytearray(code)
        for slot, k in relocs:
            h = oracle_handle(k)
            b[slot * 8 + 4: slot * 8 + 8] = (h & 0xffffffff).to_bytes(4, "little")
            b[slot * 8 + 12: slot * 8 + 16] = (h >> 32).to_bytes(4, "little")
        self.code = np.frombuffer(bytes(b), dtype=np.uint8).copy()
        self.map_data = [np.ascontiguousarray(np.frombuffer(bytes(d), dtype=np.uint8)).copy()
                         for (_, _, d) in maps]
        self.maps_arr = (_Map * max(1, len(maps)))()
        for k, (vs, me, _) in enumerate(maps):
            self.maps_arr[k].handle = oracle_handle(k)
            self.maps_arr[k].data = self.map_data[k].ctypes.data
            self.maps_arr[k].value_size = vs
            self.maps_arr[k].max_entries = me
        self.p = _Prog()
        self.p.insns = self.code.ctypes.data
        self.p.nslots = len(self.code) // 8
        kinds = helper_kinds or {0: HELPER_MAP_LOOKUP, 1: HELPER_OTHER, 2: HELPER_OTHER}
        for i, v in kinds.items():
            self.p.helper_kind[i] = v
        self.p.maps = ctypes.addressof(self.maps_arr)
        self.p.nmaps = len(maps)
        self.p.reg_init = reg_init
        self.p.stack_init = stack_init
        self.p.checked = 1 if checked else 0

    def run(self, data, count, stride=0, offsets=None, nthreads=1):
        """Runs in place on a COPY of ``data``; returns (ret u64[count], faults u8[count],
        data_after u8[...], executed_instructions)."""
        work = np.ascontiguousarray(np.array(data, dtype=np.uint8, copy=True).reshape(-1))
        ret = np.zeros(count, dtype=np.uint64)
        faults = np.zeros(count, dtype=np.uint8)
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        steps = lib().oracle_run_batch(ctypes.addressof(self.p), work.ctypes.data,
                                       None if offs is None else offs.ctypes.data,
                                       count, stride, ret.ctypes.data, faults.ctypes.data,
                                       nthreads)
        return ret, faults, work, int(steps)
