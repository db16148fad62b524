"""ctypes binding of the engine's C-ABI library (lib/libebpf.so).

The Python layer mirrors the reference's plugin interface: an ``Env`` owns a ``struct
ebpf_config`` laid out like tests/test_common.hpp:59-75 of the reference (program type 0
"test"; map types 0..3 = array, percpu array, hashtable, percpu hashtable; helpers 0..2 =
map_lookup_elem / map_update_elem / map_delete_elem), ``Map`` and ``Prog`` wrap the map and
program objects with the reference's errno conventions.  Batch runs go to the GPU through
include/ebpf_gpu.h; if the library is missing, loading fails loudly.
"""
import ctypes
import errno
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# EBPF_LIB: an alternative build of the same library (A/B experiments under tools/)
LIB_PATH = os.environ.get("EBPF_LIB") or os.path.join(HERE, "lib", "libebpf.so")

EBPF_TYPE_MAX = 64
EBPF_NAME_MAX = 64
EBPF_HIST_BINS = 257

MAP_TYPE_ARRAY, MAP_TYPE_PERCPU_ARRAY, MAP_TYPE_HASHTABLE, MAP_TYPE_PERCPU_HASHTABLE = range(4)
SEM_REFERENCE, SEM_STANDARD = 0, 1
HELPER_LOOKUP, HELPER_UPDATE, HELPER_DELETE, HELPER_OTHER = range(4)
EBPF_ANY, EBPF_NOEXIST, EBPF_EXIST = 0, 1, 2

FAULT_NAMES = ["NONE", "BAD_OPCODE", "DIV_ZERO", "MEM", "SLOT", "HELPER", "HELPER_UNSUPPORTED",
               "BAD_REG", "LOOP", "MAP_WRITE", "BAD_MAP", "WRITES"]


class ProgAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("prog", ctypes.c_void_p),
                ("prog_len", ctypes.c_uint32), ("data", ctypes.c_void_p)]


class MapAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("key_size", ctypes.c_uint32),
                ("value_size", ctypes.c_uint32), ("max_entries", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


_PREDFN = ctypes.CFUNCTYPE(ctypes.c_bool, ctypes.c_void_p)


class ProgType(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * EBPF_NAME_MAX), ("is_map_usable", _PREDFN),
                ("is_helper_usable", _PREDFN)]


class HelperType(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * EBPF_NAME_MAX), ("fn", ctypes.c_void_p)]


class Config(ctypes.Structure):
    _fields_ = [("prog_types", ctypes.c_void_p * EBPF_TYPE_MAX),
                ("map_types", ctypes.c_void_p * EBPF_TYPE_MAX),
                ("helper_types", ctypes.c_void_p * EBPF_TYPE_MAX),
                ("preprocessor_type", ctypes.c_void_p)]


class PktBatch(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("count", ctypes.c_uint64), ("stride", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class BatchStats(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("faulted", ctypes.c_uint64),
                ("hist", ctypes.c_uint64 * EBPF_HIST_BINS), ("kernel_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double)]


class DexecInfo(ctypes.Structure):
    _fields_ = [("exec", ctypes.c_int32), ("layout", ctypes.c_int32),
                ("translate_ms", ctypes.c_double), ("build_ms", ctypes.c_double)]


EXEC_NAMES = {0: "compiled", 1: "hip", 2: "interpreter"}


class PcapInfo(ctypes.Structure):
    _fields_ = [("linktype", ctypes.c_uint32), ("snaplen", ctypes.c_uint32),
                ("nanosecond", ctypes.c_uint32), ("byte_swapped", ctypes.c_uint32),
                ("truncated", ctypes.c_uint64), ("bytes", ctypes.c_uint64)]


class DprogInfo(ctypes.Structure):
    _fields_ = [("nslots", ctypes.c_uint32), ("nentries", ctypes.c_uint32),
                ("nmaps", ctypes.c_uint32), ("max_stack", ctypes.c_uint32)]


# Every function include/ebpf.h and include/ebpf_gpu.h declare: name -> (restype, argtypes)
_VP, _U32, _U64, _I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
FUNCS = {
    "ebpf_init": (_I, []), "ebpf_deinit": (_I, []),
    "ebpf_env_create": (_I, [_VP, _VP]), "ebpf_env_destroy": (_I, [_VP]),
    "ebpf_obj_acquire": (None, [_VP]), "ebpf_obj_release": (None, [_VP]),
    "ebpf_prog_create": (_I, [_VP, _VP, _VP]), "ebpf_prog_destroy": (None, [_VP]),
    "ebpf_prog_run": (_U64, [_VP, _VP]),
    "ebpf_map_create": (_I, [_VP, _VP, _VP]), "ebpf_map_lookup_elem": (_VP, [_VP, _VP]),
    "ebpf_map_update_elem": (_I, [_VP, _VP, _VP, _U64]),
    "ebpf_map_delete_elem": (_I, [_VP, _VP]),
    "ebpf_map_lookup_elem_from_user": (_I, [_VP, _VP, _VP]),
    "ebpf_map_update_elem_from_user": (_I, [_VP, _VP, _VP, _U64]),
    "ebpf_map_delete_elem_from_user": (_I, [_VP, _VP]),
    "ebpf_map_get_next_key_from_user": (_I, [_VP, _VP, _VP]),
    "ebpf_map_destroy": (None, [_VP]),
    # ebpf_gpu.h
    "ebpf_gpu_device_count": (_I, []), "ebpf_gpu_set_device": (_I, [_I]), "ebpf_dev_init": (_I, [_I]),
    "ebpf_gpu_set_variant": (_I, [_I]), "ebpf_gpu_time_next_launch": (_I, [_VP, _VP]), "ebpf_gpu_last_error": (ctypes.c_char_p, []),
    "ebpf_prog_prepare_device": (_I, [_VP, _I]),
    "ebpf_prog_run_batch": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "ebpf_prog_run_batch_dev": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP]),
    "ebpf_prog_run_batch_multi": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP]),
    "ebpf_prog_run_batch_multi_dev": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _VP]),
    "ebpf_prog_device_info": (_I, [_VP, _VP]),
    "ebpf_prog_device_exec": (_I, [_VP, _I, _VP]),
    "ebpf_prog_device_code": (_I, [_VP, _I, _VP, ctypes.POINTER(ctypes.c_size_t)]),
    "ebpf_prog_set_semantics": (_I, [_VP, _I]),
    "ebpf_pcap_batch": (_I, [_VP, ctypes.c_size_t, _I, _VP, _VP]),
    "ebpf_pcap_batch_free": (None, [_VP]),
    "ebpf_pcap_extents": (_I, [_VP, ctypes.c_size_t, _I, _VP, _VP]),
    "ebpf_prog_run_batch_async": (_I, [_VP, _VP, _VP, _VP, ctypes.POINTER(_VP)]),
    "ebpf_batch_wait": (_I, [_VP, _VP]),
}
DATA_SYMBOLS = ["emt_array", "emt_percpu_array", "emt_hashtable", "emt_percpu_hashtable",
                "eht_map_lookup_elem", "eht_map_update_elem", "eht_map_delete_elem"]

_lib = None


BATCH_HIST_OVERWRITE = 0x1  # include/ebpf_gpu.h EBPF_BATCH_HIST_OVERWRITE
BATCH_EXTENTS = 0x2         # EBPF_BATCH_EXTENTS: offsets holds (start, end) pairs


class _AsyncJob:
    """An ebpf_prog_run_batch_async job and the buffers it writes (see Prog.run_batch_async)."""

    def __init__(self, data, count, offsets, want_faults):
        self.data = data
        self.offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        self.ret = np.zeros(count, dtype=np.uint64)
        self.faults = np.zeros(count, dtype=np.uint8) if want_faults else None
        self.handle = None

    def wait(self):
        st = BatchStats()
        h, self.handle = self.handle, None
        _check(lib().ebpf_batch_wait(h, ctypes.byref(st)), "ebpf_batch_wait")
        return self.ret, self.faults, st


class PcapBatch:
    """ebpf_pcap_batch: a classic pcap capture (bytes) as a library-allocated batch in offsets
    form.  ``batch`` is the ebpf_pkt_batch to hand to the run functions; ``data()`` /
    ``offsets()`` copy it out; ``free()`` (or the context manager) releases it."""

    def __init__(self, capture, pinned=False, extents=False):
        # (extents: ebpf_pcap_extents, the batch is the capture itself; it is kept here)
        self.buf = np.frombuffer(bytes(capture), dtype=np.uint8)
        buf = self.buf
        self.batch = PktBatch()
        self.info = PcapInfo()
        fn = lib().ebpf_pcap_extents if extents else lib().ebpf_pcap_batch
        _check(fn(buf.ctypes.data if len(buf) else None, len(buf), 1 if pinned else 0,
                  ctypes.byref(self.batch), ctypes.byref(self.info)),
               "ebpf_pcap_extents" if extents else "ebpf_pcap_batch")

    @property
    def count(self):
        return int(self.batch.count)

    def offsets(self):
        n = 2 * self.count if self.batch.flags & BATCH_EXTENTS else self.count + 1
        return np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(
            self.batch.offsets)).copy()

    def data(self):
        if self.batch.flags & BATCH_EXTENTS:
            return self.buf.copy()
        n = int(self.info.bytes)
        if n == 0:
            return np.zeros(0, dtype=np.uint8)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(self.batch.data)).copy()

    def free(self):
        if self.batch.data is not None or self.batch.offsets is not None:
            lib().ebpf_pcap_batch_free(ctypes.byref(self.batch))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()


def lib():
    """Load lib/libebpf.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("native library not built: %s (run __graft_entry__.build())" % LIB_PATH)
        # torch (when installed) bundles its own HIP runtime under the same soname: loaded
        # first, it is the one the library binds to as well.  Loaded the other way round, a
        # process gets two HIP runtimes and whichever initialises second sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in FUNCS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def addr_of(symbol):
    return ctypes.addressof(ctypes.c_char.in_dll(lib(), symbol))


def last_error():
    return (lib().ebpf_gpu_last_error() or b"").decode()


class EbpfError(RuntimeError):
    def __init__(self, code, what):
        super().__init__("%s failed: %s (%d) %s" % (what, errno.errorcode.get(code, "?"), code,
                                                    last_error()))
        self.code = code


def _check(code, what):
    if code != 0:
        raise EbpfError(code, what)


_always = _PREDFN(lambda _p: True)


class Env:
    """ebpf_env with the reference test suite's configuration (tests/test_common.hpp:59-75),
    plus helper 3: a helper with no device implementation (CALL 3 faults HELPER_UNSUPPORTED
    on the device)."""

    def __init__(self, helpers=None):
        L = lib()
        self._ptype = ProgType(b"test", _always, _always)
        self._other = HelperType(b"other", None)
        self.config = Config()
        self.config.prog_types[0] = ctypes.addressof(self._ptype)
        for i, s in enumerate(["emt_array", "emt_percpu_array", "emt_hashtable",
                               "emt_percpu_hashtable"]):
            self.config.map_types[i] = addr_of(s)
        hl = helpers if helpers is not None else {
            HELPER_LOOKUP: addr_of("eht_map_lookup_elem"),
            HELPER_UPDATE: addr_of("eht_map_update_elem"),
            HELPER_DELETE: addr_of("eht_map_delete_elem"),
            HELPER_OTHER: ctypes.addressof(self._other)}
        for i, a in hl.items():
            self.config.helper_types[i] = a
        self.ptr = ctypes.c_void_p()
        _check(L.ebpf_env_create(ctypes.byref(self.ptr), ctypes.byref(self.config)),
               "ebpf_env_create")

    def destroy(self):
        return lib().ebpf_env_destroy(self.ptr)


class Map:
    def __init__(self, env, max_entries, value_size, key_size=4, type=MAP_TYPE_ARRAY):
        self.env = env
        self.value_size, self.max_entries = value_size, max_entries
        attr = MapAttr(type, key_size, value_size, max_entries, 0)
        self.ptr = ctypes.c_void_p()
        _check(lib().ebpf_map_create(env.ptr, ctypes.byref(self.ptr), ctypes.byref(attr)),
               "ebpf_map_create")

    @property
    def handle(self):
        return self.ptr.value

    def update(self, key, value_bytes, flags=EBPF_ANY):
        k = ctypes.c_uint32(key)
        v = ctypes.create_string_buffer(bytes(value_bytes), self.value_size)
        return lib().ebpf_map_update_elem_from_user(self.ptr, ctypes.byref(k), v, flags)

    def fill(self, data):
        """data: bytes of max_entries * value_size."""
        for k in range(self.max_entries):
            _check(self.update(k, data[k * self.value_size:(k + 1) * self.value_size]),
                   "map update")

    def lookup(self, key):
        k = ctypes.c_uint32(key)
        v = ctypes.create_string_buffer(self.value_size)
        err = lib().ebpf_map_lookup_elem_from_user(self.ptr, ctypes.byref(k), v)
        return err, v.raw

    def destroy(self):
        lib().ebpf_map_destroy(self.ptr)


class HashMap:
    """A hashtable (or percpu hashtable) map with byte-string keys (ebpf_map_hashtable.c)."""

    def __init__(self, env, key_size, value_size, max_entries, percpu=False):
        self.env = env
        self.key_size, self.value_size, self.max_entries = key_size, value_size, max_entries
        t = MAP_TYPE_PERCPU_HASHTABLE if percpu else MAP_TYPE_HASHTABLE
        attr = MapAttr(t, key_size, value_size, max_entries, 0)
        self.ptr = ctypes.c_void_p()
        _check(lib().ebpf_map_create(env.ptr, ctypes.byref(self.ptr), ctypes.byref(attr)),
               "ebpf_map_create")

    @property
    def handle(self):
        return self.ptr.value

    def update(self, key, value_bytes, flags=EBPF_ANY):
        k = ctypes.create_string_buffer(bytes(key), self.key_size)
        v = ctypes.create_string_buffer(bytes(value_bytes), self.value_size)
        return lib().ebpf_map_update_elem_from_user(self.ptr, k, v, flags)

    def fill(self, keys, values):
        """keys: uint8 [n, key_size]; values: uint8 [n, value_size] (EBPF_ANY updates)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, self.key_size)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1, self.value_size)
        f = lib().ebpf_map_update_elem_from_user
        kp, vp = keys.ctypes.data, values.ctypes.data
        for i in range(len(keys)):
            _check(f(self.ptr, kp + i * self.key_size, vp + i * self.value_size, EBPF_ANY),
                   "map update")

    def lookup(self, key):
        k = ctypes.create_string_buffer(bytes(key), self.key_size)
        v = ctypes.create_string_buffer(self.value_size)
        err = lib().ebpf_map_lookup_elem_from_user(self.ptr, k, v)
        return err, v.raw

    def delete(self, key):
        k = ctypes.create_string_buffer(bytes(key), self.key_size)
        return lib().ebpf_map_delete_elem_from_user(self.ptr, k)

    def destroy(self):
        lib().ebpf_map_destroy(self.ptr)


def patch_relocs(code, relocs, handles):
    b = bytearray(code)
    for slot, k in relocs:
        h = handles[k] & 0xffffffffffffffff
        b[slot * 8 + 4: slot * 8 + 8] = (h & 0xffffffff).to_bytes(4, "little")
        b[slot * 8 + 12: slot * 8 + 16] = (h >> 32).to_bytes(4, "little")
    return bytes(b)


class Prog:
    def __init__(self, env, code, prog_type=0):
        self.env = env
        self._buf = ctypes.create_string_buffer(bytes(code), len(code))
        attr = ProgAttr(prog_type, ctypes.addressof(self._buf), len(code), None)
        self.ptr = ctypes.c_void_p()
        _check(lib().ebpf_prog_create(env.ptr, ctypes.byref(self.ptr), ctypes.byref(attr)),
               "ebpf_prog_create")

    def destroy(self):
        lib().ebpf_prog_destroy(self.ptr)

    def info(self):
        i = DprogInfo()
        _check(lib().ebpf_prog_device_info(self.ptr, ctypes.byref(i)), "ebpf_prog_device_info")
        return i

    def exec_info(self, device=0):
        """What the last launch on ``device`` ran (ebpf_prog_device_exec): (exec name or None,
        layout, translate ms, build ms)."""
        i = DexecInfo()
        _check(lib().ebpf_prog_device_exec(self.ptr, device, ctypes.byref(i)),
               "ebpf_prog_device_exec")
        return EXEC_NAMES.get(i.exec), i.layout, i.translate_ms, i.build_ms

    def set_semantics(self, semantics):
        """SEM_REFERENCE (default) or SEM_STANDARD (ebpf_gpu.h ebpf_prog_set_semantics)."""
        _check(lib().ebpf_prog_set_semantics(self.ptr, semantics), "ebpf_prog_set_semantics")

    def prepare(self, device=0):
        _check(lib().ebpf_prog_prepare_device(self.ptr, device), "ebpf_prog_prepare_device")

    def run_cpu(self, packet):
        """Single packet through ebpf_prog_run (the API's per-packet CPU entry point)."""
        buf = ctypes.create_string_buffer(bytes(packet), len(packet))
        return lib().ebpf_prog_run(buf, self.ptr), buf.raw

    def run_batch(self, data, count, stride=0, offsets=None, want_faults=True, extents=False):
        """Host buffers: returns (ret u64[count], faults u8[count], stats).  ``data`` (a
        contiguous uint8 numpy array) is modified in place if the program stores to packets.
        ``extents``: ``offsets`` holds (start, end) pairs (EBPF_BATCH_EXTENTS)."""
        assert data.dtype == np.uint8 and data.flags["C_CONTIGUOUS"]
        ret = np.zeros(count, dtype=np.uint64)
        faults = np.zeros(count, dtype=np.uint8) if want_faults else None
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        b = PktBatch(data.ctypes.data, None if offs is None else offs.ctypes.data, count,
                     stride, BATCH_EXTENTS if extents else 0)
        st = BatchStats()
        _check(lib().ebpf_prog_run_batch(self.ptr, ctypes.byref(b), ret.ctypes.data,
                                         None if faults is None else faults.ctypes.data,
                                         ctypes.byref(st)), "ebpf_prog_run_batch")
        return ret, faults, st

    def run_batch_async(self, data, count, stride=0, offsets=None, want_faults=True):
        """ebpf_prog_run_batch_async: returns a job; job.wait() -> (ret, faults, stats) as
        run_batch.  ``data`` (and ``offsets``) must stay alive until the wait (the job keeps
        references)."""
        assert data.dtype == np.uint8 and data.flags["C_CONTIGUOUS"]
        job = _AsyncJob(data, count, offsets, want_faults)
        b = PktBatch(data.ctypes.data, None if job.offs is None else job.offs.ctypes.data, count,
                     stride, 0)
        h = ctypes.c_void_p()
        _check(lib().ebpf_prog_run_batch_async(self.ptr, ctypes.byref(b), job.ret.ctypes.data,
                                               None if job.faults is None else job.faults.ctypes.data,
                                               ctypes.byref(h)), "ebpf_prog_run_batch_async")
        job.handle = h
        return job

    def run_pcap(self, pcap, want_faults=True):
        """ebpf_prog_run_batch over a PcapBatch as the library built it (its own buffers, pinned
        or not).  Returns (ret, faults, stats) like run_batch."""
        ret = np.zeros(pcap.count, dtype=np.uint64)
        faults = np.zeros(pcap.count, dtype=np.uint8) if want_faults else None
        st = BatchStats()
        _check(lib().ebpf_prog_run_batch(self.ptr, ctypes.byref(pcap.batch), ret.ctypes.data,
                                         None if faults is None else faults.ctypes.data,
                                         ctypes.byref(st)), "ebpf_prog_run_batch")
        return ret, faults, st

    def run_batch_multi(self, devices, data, count, stride=0, offsets=None, want_faults=True,
                        extents=False):
        """ebpf_prog_run_batch_multi: host buffers sharded over ``devices`` (a list of device
        indices, repeats allowed).  Returns (ret, faults, stats) like run_batch."""
        assert data.dtype == np.uint8 and data.flags["C_CONTIGUOUS"]
        ret = np.zeros(count, dtype=np.uint64)
        faults = np.zeros(count, dtype=np.uint8) if want_faults else None
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        b = PktBatch(data.ctypes.data, None if offs is None else offs.ctypes.data, count,
                     stride, BATCH_EXTENTS if extents else 0)
        devs = (ctypes.c_int * len(devices))(*devices)
        st = BatchStats()
        _check(lib().ebpf_prog_run_batch_multi(self.ptr, len(devices), devs, ctypes.byref(b),
                                               ret.ctypes.data,
                                               None if faults is None else faults.ctypes.data,
                                               ctypes.byref(st)), "ebpf_prog_run_batch_multi")
        return ret, faults, st

    def run_batch_multi_dev(self, devices, shards, rets, faults=None, hists=None, streams=None,
                            hist_overwrite=False):
        """ebpf_prog_run_batch_multi_dev.  ``shards``: [(data_ptr, count, stride, offsets_ptr)]
        per device; ``rets`` / ``faults`` / ``hists`` / ``streams``: per-device pointers (ints)."""
        n = len(devices)
        arr = (PktBatch * n)()
        for d, (dp, cnt, stride, op) in enumerate(shards):
            arr[d] = PktBatch(dp, op, cnt, stride, BATCH_HIST_OVERWRITE if hist_overwrite else 0)
        P = ctypes.c_void_p * n
        _check(lib().ebpf_prog_run_batch_multi_dev(
            self.ptr, n, (ctypes.c_int * n)(*devices), arr, P(*rets),
            None if faults is None else P(*faults), None if hists is None else P(*hists),
            None if streams is None else P(*streams)), "ebpf_prog_run_batch_multi_dev")

    def device_code(self, layout=1):
        """The program compiled for variant 0 (raw gfx950 code bytes); works without a GPU."""
        n = ctypes.c_size_t(0)
        _check(lib().ebpf_prog_device_code(self.ptr, layout, None, ctypes.byref(n)),
               "ebpf_prog_device_code")
        buf = (ctypes.c_uint8 * max(1, n.value))()
        _check(lib().ebpf_prog_device_code(self.ptr, layout, buf, ctypes.byref(n)),
               "ebpf_prog_device_code")
        return bytes(buf)[: n.value]

    def run_batch_dev(self, device, data_ptr, count, stride, ret_ptr, offsets_ptr=None,
                      faults_ptr=None, hist_ptr=None, stream=None, hist_overwrite=False,
                      extents=False):
        """Device pointers (ints); asynchronous on ``stream`` (hipStream_t as int or None).
        ``hist_overwrite``: the histogram is set to this batch's counts instead of added to."""
        b = PktBatch(data_ptr, offsets_ptr, count, stride,
                     (BATCH_HIST_OVERWRITE if hist_overwrite else 0) |
                     (BATCH_EXTENTS if extents else 0))
        _check(lib().ebpf_prog_run_batch_dev(self.ptr, device, ctypes.byref(b), ret_ptr,
                                             faults_ptr, hist_ptr, stream),
               "ebpf_prog_run_batch_dev")


    def launcher(self, device, data_ptr, count, stride, ret_ptr, offsets_ptr=None,
                 faults_ptr=None, stream=None, hist_overwrite=False):
        """A prebound ebpf_prog_run_batch_dev for a bench loop: returns ``launch(hist_ptr)``
        whose only per-call work is the C call itself (batch descriptor and argument
        conversion done once here).  Raises EbpfError on a non-zero return."""
        b = PktBatch(data_ptr, offsets_ptr, count, stride,
                     BATCH_HIST_OVERWRITE if hist_overwrite else 0)
        f = lib().ebpf_prog_run_batch_dev
        args = (self.ptr, device, ctypes.byref(b), ret_ptr, faults_ptr)
        st = stream

        def launch(hist_ptr):
            rc = f(*args, hist_ptr, st)
            if rc:
                raise EbpfError(rc, "ebpf_prog_run_batch_dev")
        launch.batch = b  # keeps the descriptor alive with the closure
        return launch


def gpu_count():
    return lib().ebpf_gpu_device_count()


def dev_init(ndev=0):
    """ebpf_dev_init: load the kernels on devices 0..ndev-1 (0: all); raises EbpfError."""
    _check(lib().ebpf_dev_init(ndev), "ebpf_dev_init")


def time_next_launch(start_event, stop_event):
    """The calling thread's next run_batch_dev records these hipEvent_t handles (ints, or None
    to cancel) around the interpreter kernel alone (include/ebpf_gpu.h)."""
    _check(lib().ebpf_gpu_time_next_launch(start_event, stop_event), "ebpf_gpu_time_next_launch")


def set_variant(v):
    _check(lib().ebpf_gpu_set_variant(v), "ebpf_gpu_set_variant")
