"""A packet capture as a batch (include/ebpf_gpu.h ebpf_pcap_batch; SURVEY.md §8(f) rank 1: the
path starts in host memory, "a NIC ring or pcap buffer").  CPU: the classic libpcap format in
both byte orders and both timestamp units, zero-length and snaplen-truncated records, and the
malformed captures it must refuse.  GPU: a capture of L2/L3 frames of mixed lengths run through
ebpf_prog_run_batch from the library's own (pinned or pageable) buffers equals the oracle on
the same packets."""
import errno
import struct

import numpy as np
import pytest

from helpers import oracle_run

MAGIC_US, MAGIC_NS = 0xA1B2C3D4, 0xA1B23C4D


def make_pcap(packets, magic=MAGIC_US, big_endian=False, snaplen=65535, linktype=1, orig=None):
    e = ">" if big_endian else "<"
    out = [struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, snaplen, linktype)]
    for i, p in enumerate(packets):
        o = len(p) if orig is None else orig[i]
        out.append(struct.pack(e + "IIII", 1700000000 + i, 1000 * i, len(p), o))
        out.append(bytes(p))
    return b"".join(out)


def _packets(n, seed=1):
    g = np.random.default_rng(seed)
    return [g.integers(0, 256, int(g.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(n)]


@pytest.mark.parametrize("magic,big", [(MAGIC_US, False), (MAGIC_NS, False), (MAGIC_US, True),
                                       (MAGIC_NS, True)])
def test_pcap_batch_layout(native, magic, big):
    pk = _packets(300) + [b""]   # a zero-length record too
    with native.PcapBatch(make_pcap(pk, magic, big, linktype=113)) as b:
        assert b.count == len(pk)
        offs = b.offsets()
        assert offs[0] == 0 and np.array_equal(np.diff(offs), [len(p) for p in pk])
        assert b.data().tobytes() == b"".join(pk)
        assert b.info.linktype == 113 and b.info.snaplen == 65535
        assert b.info.nanosecond == (magic == MAGIC_NS) and b.info.byte_swapped == big
        assert b.info.truncated == 0 and b.info.bytes == sum(map(len, pk))


def test_pcap_batch_truncated_records_and_empty(native):
    pk = _packets(10, seed=2)
    orig = [len(p) + 7 * (i % 2) for i, p in enumerate(pk)]  # every other record cut by snaplen
    with native.PcapBatch(make_pcap(pk, orig=orig)) as b:
        assert b.info.truncated == 5 and b.count == 10
    with native.PcapBatch(make_pcap([])) as b:   # header only: an empty batch
        assert b.count == 0 and b.offsets().tolist() == [0]


def test_pcap_batch_large_capture_threaded(native):
    """A capture above 16 MB is gathered by several threads (contiguous packet ranges): the
    batch must be byte-identical to the records' concatenation."""
    g = np.random.default_rng(4)
    n = 150000
    lens = g.integers(0, 240, n)
    blob = g.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    ends = np.cumsum(lens)
    pk = [blob[e - l:e] for e, l in zip(ends, lens)]
    cap = make_pcap(pk)
    assert len(cap) > (16 << 20)
    with native.PcapBatch(cap) as b:
        assert b.count == n
        assert np.array_equal(b.offsets(), np.concatenate([[0], ends]).astype(np.uint64))
        assert b.data().tobytes() == blob


@pytest.mark.parametrize("bad", ["magic", "short_header", "record_header", "record_data",
                                 "empty"])
def test_pcap_batch_rejects(native, bad):
    good = make_pcap(_packets(4, seed=3), snaplen=256)
    cap = {"magic": b"\0\0\0\0" + good[4:], "short_header": good[:20],
           "record_header": good + b"\1\2\3", "record_data": good[:-1],
           "empty": b""}[bad]
    with pytest.raises(native.EbpfError) as ei:
        native.PcapBatch(cap)
    assert ei.value.code == errno.EINVAL
    if bad != "empty":
        assert "pcap" in native.last_error()


def test_pcap_records_longer_than_snaplen(native):
    """A record whose captured length exceeds the header's snaplen is cut to the snaplen (as
    libpcap's reader does) and counted as truncated; the records after it stay aligned."""
    pk = [b"a" * 300, b"b" * 100, bytes(range(256)) + b"c" * 44, b"", b"d" * 256]
    with native.PcapBatch(make_pcap(pk, snaplen=256)) as b:
        assert b.count == 5
        want = [p[:256] for p in pk]
        lens = [len(p) for p in want]
        assert np.array_equal(b.offsets(), np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64))
        assert b.data().tobytes() == b"".join(want)
        assert b.info.truncated == 2


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [True, False])
def test_pcap_batch_on_device_vs_oracle(gpu, env, pinned):
    """C3's classifier over a capture of L2/L3 frames cut to random lengths (14..128 B: some
    lanes fault MEM on their headers), straight from the library's buffers."""
    import goldens
    from generic_ebpf_amd import workloads
    n = 50000
    frames = workloads.packets_l2l3(n, 128, seed=9)
    lens = np.random.default_rng(10).integers(14, 129, n)
    cap = make_pcap([frames[i, :lens[i]].tobytes() for i in range(n)])
    lay = workloads.prog_c3()
    p = gpu.Prog(env, lay.code)
    try:
        with gpu.PcapBatch(cap, pinned=pinned) as b:
            got, gf, st = p.run_pcap(b)
            data, offs = b.data(), b.offsets()
    finally:
        p.destroy()
    c = goldens.Case("pcap", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    assert wf.any() and not wf.all()
    np.testing.assert_array_equal(wf, gf)
    np.testing.assert_array_equal(want, got)
    assert st.packets == n
