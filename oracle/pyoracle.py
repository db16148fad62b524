"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/ebpf_oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker or the
timed CPU baseline; the product (generic-ebpf_amd/) never imports this module.
"""
import copy
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

HELPER_UNSET, HELPER_MAP_LOOKUP, HELPER_OTHER, HELPER_MAP_UPDATE, HELPER_MAP_DELETE = 0, 1, 2, 3, 4
# the engine's Env (generic_ebpf_amd.native): helpers 0..2 = lookup / update / delete as in the
# reference tests' config (tests/test_common.hpp:69-73), 3 = a helper with no device form
DEFAULT_HELPER_KINDS = {0: HELPER_MAP_LOOKUP, 1: HELPER_MAP_UPDATE, 2: HELPER_MAP_DELETE,
                        3: HELPER_OTHER}


class _Map(ctypes.Structure):
    _fields_ = [("handle", ctypes.c_uint64), ("data", ctypes.c_void_p),
                ("value_size", ctypes.c_uint32), ("max_entries", ctypes.c_uint32),
                ("kind", ctypes.c_uint32), ("key_size", ctypes.c_uint32),
                ("keys", ctypes.c_void_p), ("nbuckets", ctypes.c_uint32),
                ("bucket_head", ctypes.c_void_p), ("bucket_next", ctypes.c_void_p),
                ("capacity", ctypes.c_uint32)]


class HashSpec:
    """A hashtable map for the oracle: ``items`` = [(key bytes, value bytes)] (live entries), or
    ``keys``/``values`` as uint8 arrays [n, key_size] / [n, value_size] (large tables);
    ``capacity`` = the map's max_entries (None: the entries given, i.e. a full table)."""

    def __init__(self, key_size, value_size, items=None, keys=None, values=None, capacity=None):
        self.key_size, self.value_size = key_size, value_size
        self.capacity = capacity
        if items is not None:
            items = [(bytes(k), bytes(v)) for k, v in items]
            assert all(len(k) == key_size and len(v) == value_size for k, v in items)
            keys = np.frombuffer(b"".join(k for k, _ in items), dtype=np.uint8)
            values = np.frombuffer(b"".join(v for _, v in items), dtype=np.uint8)
        self.keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint8).reshape(-1, key_size))
        self.values = np.ascontiguousarray(np.asarray(values, dtype=np.uint8).reshape(-1, value_size))
        assert len(self.keys) == len(self.values)

    @property
    def items(self):
        return [(self.keys[i].tobytes(), self.values[i].tobytes()) for i in range(len(self.keys))]

    def __len__(self):
        return len(self.keys)

    def model(self):
        """The table as a HashtableModel (entries inserted in order, as a test fills the
        engine's map; a spec made by from_model: that model)."""
        if getattr(self, "_model", None) is not None:
            return copy.deepcopy(self._model)
        m = HashtableModel(self.capacity or max(1, len(self)))
        for k, v in self.items:
            m.update(k, v)
        return m

    @classmethod
    def from_model(cls, model, key_size, value_size):
        """The model's live entries (the table a next batch starts from)."""
        spec = cls(key_size, value_size, items=model.items(), capacity=model.cap)
        spec._model = copy.deepcopy(model)
        return spec


class _LazyModels(dict):
    """{map index: HashtableModel}, each built from its HashSpec when first asked for."""

    def __init__(self, specs):
        super().__init__()
        self.specs = specs

    def __missing__(self, k):
        m = self[k] = self.specs[k].model()
        return m


class _Prog(ctypes.Structure):
    _fields_ = [("insns", ctypes.c_void_p), ("nslots", ctypes.c_uint64),
                ("helper_kind", ctypes.c_uint8 * 64), ("maps", ctypes.c_void_p),
                ("nmaps", ctypes.c_uint32), ("reg_init", ctypes.c_uint64),
                ("stack_init", ctypes.c_uint8), ("checked", ctypes.c_uint8),
                ("semantics", ctypes.c_uint8), ("track_undef", ctypes.c_uint8),
                ("sequential", ctypes.c_uint8)]


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
        _lib.oracle_run_batch_hlog.restype = ctypes.c_uint64
        _lib.oracle_run_batch_hlog.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_void_p]
        _lib.oracle_hash_build.restype = None
        _lib.oracle_hash_build.argtypes = [ctypes.c_void_p]
        _lib.oracle_jhash.restype = ctypes.c_uint32
        _lib.oracle_jhash.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
    return _lib


# Fake but distinct LDDW handles for oracle maps (the reference uses struct ebpf_map* values).
def oracle_handle(k):
    return 0x00007f5e00001000 + 0x100 * k


class OracleProgram:
    """A program + its maps, ready to run on the oracle.  ``code`` is unpatched; relocations
    [(slot, map_index)] are patched with oracle handles here."""

    def __init__(self, code, relocs=(), maps=(), helper_kinds=None, checked=True,
                 reg_init=0, stack_init=0, semantics=0, track_undef=False, sequential=False):
        b = bytearray(code)
        for slot, k in relocs:
            h = oracle_handle(k)
            b[slot * 8 + 4: slot * 8 + 8] = (h & 0xffffffff).to_bytes(4, "little")
            b[slot * 8 + 12: slot * 8 + 16] = (h >> 32).to_bytes(4, "little")
        self.code = np.frombuffer(bytes(b), dtype=np.uint8).copy()
        u8 = lambda d: np.ascontiguousarray(np.frombuffer(bytes(d) or b"\0", dtype=np.uint8)).copy()
        self.map_data, self.map_keys, self.map_index = [], [], []
        self.specs = list(maps)
        # k -> HashtableModel: the hashtables after the batches run so far (built on first use)
        self.hash_models = _LazyModels(self.specs)
        self.maps_arr = (_Map * max(1, len(maps)))()
        for k, m in enumerate(maps):
            self.maps_arr[k].handle = oracle_handle(k)
            if isinstance(m, HashSpec):
                self.map_data.append(u8(m.values.tobytes()))
                self.map_keys.append(u8(m.keys.tobytes()))
                self.maps_arr[k].kind = 1
                self.maps_arr[k].key_size = m.key_size
                self.maps_arr[k].keys = self.map_keys[-1].ctypes.data
                self.maps_arr[k].value_size = m.value_size
                self.maps_arr[k].max_entries = len(m)
                self.maps_arr[k].capacity = m.capacity or len(m)
                # the reference's bucket index (nbuckets = entries rounded up to a power of two)
                nb = 1
                while nb < max(1, len(m)):
                    nb <<= 1
                head = np.zeros(nb, dtype=np.int32)
                nxt = np.zeros(max(1, len(m)), dtype=np.int32)
                self.map_index.append((head, nxt))
                self.maps_arr[k].nbuckets = nb
                self.maps_arr[k].bucket_head = head.ctypes.data
                self.maps_arr[k].bucket_next = nxt.ctypes.data
                lib().oracle_hash_build(ctypes.byref(self.maps_arr[k]))
            else:
                vs, me, d = m
                self.map_data.append(u8(d))
                self.maps_arr[k].value_size = vs
                self.maps_arr[k].max_entries = me
            self.maps_arr[k].data = self.map_data[k].ctypes.data
        self.p = _Prog()
        self.p.insns = self.code.ctypes.data
        self.p.nslots = len(self.code) // 8
        kinds = helper_kinds or DEFAULT_HELPER_KINDS
        for i, v in kinds.items():
            self.p.helper_kind[i] = v
        # does the program call a map-writing helper (a CALL whose id is one) on a hashtable?
        ins = self.code[: len(self.code) // 8 * 8].reshape(-1, 8)
        ids = ins[ins[:, 0] == 0x85, 4:8].copy().view(np.int32).reshape(-1)
        # (or a store into a hashtable value: any checked program with a hashtable may make one)
        self.hash_writes = any(isinstance(m, HashSpec) for m in maps) and (checked or any(
            kinds.get(int(i)) in (HELPER_MAP_UPDATE, HELPER_MAP_DELETE) for i in ids))
        self.p.maps = ctypes.addressof(self.maps_arr)
        self.p.nmaps = len(maps)
        self.p.reg_init = reg_init
        self.p.stack_init = stack_init
        self.p.checked = 1 if checked else 0
        self.p.semantics = semantics
        self.p.track_undef = 1 if track_undef else 0
        # the reference's own run, one packet after the other: stores into map values and array
        # map_update_elem land at once (ebpf_oracle.h); batches run on one thread
        self.p.sequential = 1 if sequential else 0

    def run(self, data, count, stride=0, offsets=None, nthreads=1):
        """Runs in place on a COPY of ``data``; returns (ret u64[count], faults u8[count],
        data_after u8[...], executed_instructions).  Map writes (map_update_elem) are applied
        to this object's array-map data after the batch, in packet order (ebpf_oracle.h);
        ``map_bytes(k)`` reads them back."""
        work = np.ascontiguousarray(np.array(data, dtype=np.uint8, copy=True).reshape(-1))
        ret = np.zeros(count, dtype=np.uint64)
        faults = np.zeros(count, dtype=np.uint8)
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        args = (ctypes.addressof(self.p), work.ctypes.data, None if offs is None else offs.ctypes.data,
                count, stride, ret.ctypes.data, faults.ctypes.data, nthreads)
        if not self.hash_writes:
            steps = lib().oracle_run_batch(*args)
            return ret, faults, work, int(steps)
        # hashtable writes: the batch-start table stays in the oracle's maps (every packet sees
        # it); the successful calls come back in (packet, call) order and are replayed on
        # hash_models (a replay that fails leaves the model unchanged)
        used = ctypes.c_uint64(0)
        rmax = max(8 + m.key_size + m.value_size for m in self.specs if isinstance(m, HashSpec))
        cap = max(4096, 16 * count * rmax)   # (16 hashtable writes per packet; else run again)
        buf = np.zeros(cap, dtype=np.uint8)
        # (the run applies its array-map writes: kept to run again from the same start)
        arrays = {k: self.map_data[k].copy() for k, m in enumerate(self.specs)
                  if not isinstance(m, HashSpec)}
        steps = lib().oracle_run_batch_hlog(*args, buf.ctypes.data, cap, ctypes.byref(used))
        if used.value > cap:   # (a loop-free path with more writes: the same run, a larger buffer)
            cap = int(used.value)
            buf = np.zeros(cap, dtype=np.uint8)
            work[:] = np.asarray(data, dtype=np.uint8).reshape(-1)
            for k, d in arrays.items():
                self.map_data[k][:] = d
            steps = lib().oracle_run_batch_hlog(*args, buf.ctypes.data, cap, ctypes.byref(used))
        if used.value > cap:
            raise RuntimeError("oracle: more hashtable writes than the replay buffer holds")
        self.last_hlog = []
        if used.value:
            raw, pos = buf[:used.value].tobytes(), 0
            while pos < len(raw):
                k = int.from_bytes(raw[pos:pos + 4], "little")
                word = int.from_bytes(raw[pos + 4:pos + 8], "little")
                spec = self.specs[k]
                key = raw[pos + 8:pos + 8 + spec.key_size]
                val = raw[pos + 8 + spec.key_size:pos + 8 + spec.key_size + spec.value_size]
                pos += 8 + spec.key_size + spec.value_size
                self.last_hlog.append((k, word & 0xff, word >> 8, key, val))
                op = word & 0xff
                if op == 1:
                    self.hash_models[k].update(key, val, word >> 8)
                elif op == 2:
                    self.hash_models[k].delete(key)
                else:   # a store into the element's value (3), or a counter update (4)
                    size, off = (word >> 8) & 0xff, word >> 16
                    self.hash_models[k].store(key, off, val[:size], add=op == 4)
        return ret, faults, work, int(steps)

    def map_bytes(self, k):
        """Current bytes of map k (array maps: max_entries * value_size)."""
        return self.map_data[k].tobytes()

    def run_inplace(self, data, count, stride, offsets, ret, faults=None, nthreads=1):
        """Timed form for bench.py's cpu_baseline: runs on ``data`` itself (packet stores land
        in it) into caller-preallocated ``ret`` (u64[count]) / ``faults`` (u8[count] or None);
        no copy, no allocation.  ``offsets`` must already be a contiguous u64 array or None.
        Returns the executed-instruction count."""
        return int(lib().oracle_run_batch(ctypes.addressof(self.p), data.ctypes.data,
                                          None if offsets is None else offsets.ctypes.data,
                                          count, stride, ret.ctypes.data,
                                          None if faults is None else faults.ctypes.data,
                                          nthreads))


# ---- hashtable maps (host-side map API; small cases, pure Python) ----

def _rot(x, k):
    return ((x << k) | (x >> (32 - k))) & 0xffffffff


def jhash(key, initval=0):
    """Bob Jenkins' lookup3 hashlittle over ``key`` (bytes): the reference's
    ebpf_jenkins_hash() (sys/dev/ebpf/ebpf_jhash.h:159-330, bound on little-endian hosts by
    Linux/ebpf/user/ebpf_linux_user.c:204-208).  The reference's aligned 4-/2-/1-byte read paths
    all compute this value.  Pinned by tests/golden/maps/jhash.npz."""
    M = 0xffffffff
    n = len(key)
    a = b = c = (0xdeadbeef + n + initval) & M
    w = lambda p: int.from_bytes(key[p:p + 4].ljust(4, b"\0"), "little")
    i = 0
    while n - i > 12:
        a, b, c = (a + w(i)) & M, (b + w(i + 4)) & M, (c + w(i + 8)) & M
        a = ((a - c) & M) ^ _rot(c, 4); c = (c + b) & M
        b = ((b - a) & M) ^ _rot(a, 6); a = (a + c) & M
        c = ((c - b) & M) ^ _rot(b, 8); b = (b + a) & M
        a = ((a - c) & M) ^ _rot(c, 16); c = (c + b) & M
        b = ((b - a) & M) ^ _rot(a, 19); a = (a + c) & M
        c = ((c - b) & M) ^ _rot(b, 4); b = (b + a) & M
        i += 12
    if n == i:
        return c
    tail = key[i:].ljust(12, b"\0")
    a = (a + int.from_bytes(tail[0:4], "little")) & M
    b = (b + int.from_bytes(tail[4:8], "little")) & M
    c = (c + int.from_bytes(tail[8:12], "little")) & M
    c ^= b; c = (c - _rot(b, 14)) & M
    a ^= c; a = (a - _rot(c, 11)) & M
    b ^= a; b = (b - _rot(a, 25)) & M
    c ^= b; c = (c - _rot(b, 16)) & M
    a ^= c; a = (a - _rot(c, 4)) & M
    b ^= a; b = (b - _rot(a, 14)) & M
    c ^= b; c = (c - _rot(b, 24)) & M
    return c


EBPF_ANY, EBPF_NOEXIST, EBPF_EXIST = 0, 1, 2
_ENOENT, _EEXIST, _EBUSY = 2, 17, 16


class HashtableModel:
    """The reference's hashtable map as a CPU model (sys/dev/ebpf/ebpf_map_hashtable.c):
    nbuckets = max_entries rounded up to a power of two (:167), bucket = jhash(key) & (n-1)
    (:58-62), newest element first in its bucket (:380, :421), update flag checks (:88-100),
    EBUSY when the element pool is empty (:371-375), delete always 0 (:475-502) and
    get_next_key's bucket walk (:504-541).  Keys are bytes; values bytes (percpu: one per CPU)."""

    def __init__(self, max_entries, percpu=False, ncpu=1):
        self.nb = 1
        while self.nb < max_entries:
            self.nb <<= 1
        self.cap = max_entries
        self.percpu, self.ncpu = percpu, ncpu
        self.buckets = [[] for _ in range(self.nb)]   # newest first: [key, value(s)]

    def _find(self, key):
        bk = self.buckets[jhash(key) & (self.nb - 1)]
        for i, (k, _) in enumerate(bk):
            if k == key:
                return bk, i
        return bk, -1

    def __len__(self):
        return sum(len(b) for b in self.buckets)

    def lookup(self, key):
        bk, i = self._find(key)
        return None if i < 0 else bk[i][1]

    def update(self, key, value, flags=EBPF_ANY):
        bk, i = self._find(key)
        if i >= 0 and flags & EBPF_NOEXIST:
            return _EEXIST
        if i < 0 and flags & EBPF_EXIST:
            return _ENOENT
        if i >= 0:
            if self.percpu:       # in place (:405-407 / :452-455)
                bk[i][1] = [value] * self.ncpu
                return 0
            del bk[i]            # replaced by a new head element (:378-381)
        elif len(self) >= self.cap:
            return _EBUSY
        bk.insert(0, [key, [value] * self.ncpu if self.percpu else value])
        return 0

    def delete(self, key):
        bk, i = self._find(key)
        if i >= 0:
            del bk[i]
        return 0

    def store(self, key, off, data, add=False):
        """A program's store into the value of ``key`` through a lookup result, in place (the
        element keeps its place in its bucket); ``add``: a counter update adding ``data``
        (little-endian, mod 2^(8 len(data))).  No element: nothing (it was deleted before)."""
        bk, i = self._find(key)
        if i < 0:
            return
        cur = bk[i][1][0] if self.percpu else bk[i][1]
        v = bytearray(cur)
        n = len(data)
        if add:
            x = (int.from_bytes(v[off:off + n], "little") + int.from_bytes(data, "little")) % (1 << (8 * n))
            data = x.to_bytes(n, "little")
        v[off:off + n] = data
        if self.percpu:
            bk[i][1][0] = bytes(v)
        else:
            bk[i][1] = bytes(v)

    def get_next_key(self, key=None):
        start = 0
        if key is not None:
            bk, i = self._find(key)
            if i >= 0:
                if i + 1 < len(bk):
                    return 0, bk[i + 1][0]
                start = (jhash(key) & (self.nb - 1)) + 1
        for b in range(start, self.nb):
            if self.buckets[b]:
                return 0, self.buckets[b][0][0]
        return _ENOENT, None

    def keys_in_order(self):
        return [k for b in self.buckets for k, _ in b]

    def items(self):
        """(key, value) of every live entry in bucket order (percpu: CPU 0's value)."""
        return [(k, v[0] if self.percpu else v) for b in self.buckets for k, v in b]
