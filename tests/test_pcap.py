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


@pytest.mark.parametrize("magic,big", [(MAGIC_US, False), (MAGIC_NS, True)])
def test_pcap_extents_layout(native, magic, big):
    """ebpf_pcap_extents: the batch is the capture itself (no copy), offsets the (start, end) of
    every record's captured bytes in it (snaplen-truncated), flags EBPF_BATCH_EXTENTS; the same
    packets as ebpf_pcap_batch."""
    pk = _packets(300, seed=5) + [b"", b"x" * 300]
    cap = make_pcap(pk, magic, big, snaplen=256)
    with native.PcapBatch(cap, extents=True) as e, native.PcapBatch(cap) as g:
        assert e.batch.flags == native.BATCH_EXTENTS and e.count == g.count == len(pk)
        ext = e.offsets().reshape(-1, 2)
        raw = e.data()
        assert raw.tobytes() == cap
        assert b"".join(raw[s:t].tobytes() for s, t in ext) == g.data().tobytes()
        assert np.array_equal(ext[:, 1] - ext[:, 0], np.diff(g.offsets()))
        assert e.info.truncated == g.info.truncated == 1 and e.info.bytes == g.info.bytes


def test_pcap_extents_rejects(native):
    good = make_pcap(_packets(4, seed=3))
    with pytest.raises(native.EbpfError) as ei:
        native.PcapBatch(good[:-1], extents=True)
    assert ei.value.code == errno.EINVAL


def _gather(data, ext):
    """An extents batch as the offsets form the oracle takes (its packets' bytes concatenated)."""
    lens = (ext[:, 1] - ext[:, 0]).astype(np.int64)
    offs = np.zeros(len(ext) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    flat = np.concatenate([data[s:t] for s, t in ext]) if len(ext) else np.zeros(0, np.uint8)
    return flat.astype(np.uint8), offs


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_extents_batch_vs_oracle(gpu, env, variant):
    """EBPF_BATCH_EXTENTS on every variant: 40,000 packets of 0..127 bytes at random places in a
    buffer, in random order, with gaps, overlapping each other, some empty and some with an end
    below the start (length 0: every load faults MEM), against the oracle on the same packets
    gathered back to back; host buffers (chunked uploads of each chunk's span) and the
    device-resident entry point."""
    import torch
    from generic_ebpf_amd import workloads
    g = np.random.default_rng(31 + variant)
    n, size = 40000, 3 << 20
    data = g.integers(0, 256, size, dtype=np.uint8)
    frames = workloads.packets_l2l3(4096, 128, seed=3)
    starts = g.integers(0, size - 128, n).astype(np.uint64)
    lens = g.integers(0, 128, n).astype(np.uint64)
    for i in range(0, n, 7):   # real L2/L3 frames at some of the places
        data[int(starts[i]):int(starts[i]) + 128] = frames[i % 4096]
    ext = np.stack([starts, starts + lens], axis=1)
    bad = g.random(n) < 0.01
    ext[bad, 1] = ext[bad, 0] - 1          # an end below its start
    lay = workloads.prog_c3()
    good = np.where(bad[:, None], np.stack([starts, starts], axis=1), ext)
    flat, offs = _gather(data, good)
    want, wf, _, _ = oracle_run(__import__("goldens").Case("ext", lay.code, [], [], flat, n, 0, offs),
                                nthreads=8)
    assert (wf[~bad] == 0).any() and (wf[~bad] == 3).any()
    p = gpu.Prog(env, lay.code)
    try:
        gpu.set_variant(variant)
        got, gf, st = p.run_batch(np.ascontiguousarray(data), n, 0, ext.reshape(-1), extents=True)
        np.testing.assert_array_equal(gf, wf)
        np.testing.assert_array_equal(got, want)
        # device-resident
        d_data = torch.from_numpy(data).cuda()
        d_offs = torch.from_numpy(ext.reshape(-1).view(np.int64)).cuda()
        d_ret = torch.zeros(n, dtype=torch.int64, device="cuda")
        d_f = torch.zeros(n, dtype=torch.uint8, device="cuda")
        p.run_batch_dev(0, d_data.data_ptr(), n, 0, d_ret.data_ptr(), offsets_ptr=d_offs.data_ptr(),
                        faults_ptr=d_f.data_ptr(), extents=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_f.cpu().numpy(), wf)
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
    finally:
        gpu.set_variant(0)
        p.destroy()


@pytest.mark.gpu
def test_pcap_extents_on_device_vs_gathered(gpu, env):
    """The capture run in place (ebpf_pcap_extents, pinned offsets) gives the results of the
    gathered batch (ebpf_pcap_batch), which test_pcap_batch_on_device_vs_oracle pins to the
    oracle; also sharded over the device listed twice."""
    from generic_ebpf_amd import workloads
    n = 50000
    frames = workloads.packets_l2l3(n, 128, seed=9)
    lens = np.random.default_rng(10).integers(14, 129, n)
    cap = make_pcap([frames[i, :lens[i]].tobytes() for i in range(n)])
    lay = workloads.prog_c3()
    p = gpu.Prog(env, lay.code)
    try:
        with gpu.PcapBatch(cap, pinned=True) as b, gpu.PcapBatch(cap, pinned=True, extents=True) as e:
            want, wf, _ = p.run_pcap(b)
            got, gf, st = p.run_pcap(e)
            raw, ext = e.data(), e.offsets()
        mg, mf, _ = p.run_batch_multi([0, 0], np.ascontiguousarray(raw), n, 0, ext, extents=True)
    finally:
        p.destroy()
    assert wf.any() and not wf.all()
    np.testing.assert_array_equal(gf, wf)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(mf, wf)
    np.testing.assert_array_equal(mg, want)
    assert st.packets == n
