"""The reference's ISA construction macros (sys/sys/ebpf_vm_isa.h:107-143) in the drop-in header
include/ebpf_vm_isa.h: same bytes as the reference's own header for every macro that compiles
there, the same compile failures for the ones that do not, and a C consumer (tests/c/
isa_macros_prog.c) that builds a program with them, links lib/libebpf.so and runs it through
ebpf_prog_run (CPU, here) and ebpf_prog_run_batch (GPU, -m gpu)."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "generic-ebpf_amd", "lib")
REF_HDR = "/root/reference/sys/sys/ebpf_vm_isa.h"
NSLOTS = 60


def _cc(args, tmp_path, name):
    exe = str(tmp_path / name)
    r = subprocess.run(["gcc", "-std=gnu11", "-O1", "-Wall", "-o", exe] + args,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    return r, exe


def _bytes_with(header, tmp_path, name):
    r, exe = _cc(["-DEBPF_ISA_HEADER=\"%s\"" % header, "-I", INC,
                  os.path.join(ROOT, "tests", "c", "isa_macros_bytes.c")], tmp_path, name)
    assert r.returncode == 0, r.stderr.decode()
    return subprocess.run([exe], stdout=subprocess.PIPE, check=True).stdout


def test_macro_encodings(tmp_path):
    b = _bytes_with(os.path.join(INC, "ebpf_vm_isa.h"), tmp_path, "ours")
    ins = np.frombuffer(b, dtype=np.uint8).reshape(-1, 8)
    # EBPF_ALU_REG(EBPF_SUB, 2, 3): the reference sets SRC_IMM -> opcode 0x14 (SUB_IMM), src 3
    assert ins[2][0] == 0x14 and ins[2][1] == 0x32
    # EBPF_ALU64_REG(EBPF_MOV, 5, 6) -> 0xb7 (MOV64_IMM), src nibble 6
    assert ins[6][0] == 0xb7 and ins[6][1] == 0x65
    assert ins[-1][0] == 0x95 and ins[-3][0] == 0x85  # EXIT, CALL
    assert int.from_bytes(ins[12][2:4].tobytes(), "little", signed=True) == -3


@pytest.mark.skipif(not os.path.exists(REF_HDR), reason="reference tree not present")
def test_macro_bytes_match_reference_header(tmp_path):
    # the reference header needs <stdint.h> first (it includes nothing itself); compiled from
    # where it lies, nothing copied
    ours = _bytes_with(os.path.join(INC, "ebpf_vm_isa.h"), tmp_path, "ours")
    ref = _bytes_with(REF_HDR, tmp_path, "ref")
    assert ours == ref


@pytest.mark.parametrize("use", ["EBPF_LDX(EBPF_SIZE_B, 0, 1, 0)", "EBPF_STX(EBPF_SIZE_W, 10, 1, -4)",
                                 "EBPF_LDDW(0, 5)", "EBPF_PSEUDO_MAP_LD(1, 0)", "EBPF_JMP_JA(2)"])
def test_reference_macros_that_do_not_compile(tmp_path, use):
    """These do not compile against the reference header either (undefined EBPF_SRC_MEM /
    EBPF_DW, a missing comma, an undeclared `imm`): a consumer sees the same error."""
    src = tmp_path / "bad.c"
    src.write_text('#include <stdint.h>\n#include "ebpf_vm_isa.h"\n'
                   "struct ebpf_inst p[] = { %s };\nint main(void) { return p[0].opcode; }\n" % use)
    r, _ = _cc(["-I", INC, str(src)], tmp_path, "bad")
    assert r.returncode != 0


def build_consumer(tmp_path):
    r, exe = _cc(["-I", INC, os.path.join(ROOT, "tests", "c", "isa_macros_prog.c"),
                  "-L", LIBDIR, "-Wl,-rpath," + LIBDIR, "-lebpf"], tmp_path, "consumer")
    assert r.returncode == 0, r.stderr.decode()
    return exe


def run_consumer(exe, mode, n, tmp_path):
    out = str(tmp_path / ("out_%s.bin" % mode))
    r = subprocess.run([exe, mode, str(n), out], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr.decode())
    raw = open(out, "rb").read()
    return raw[: NSLOTS * 8], np.frombuffer(raw[NSLOTS * 8:], dtype=np.uint64)


def expected(n):
    i = np.arange(n, dtype=np.uint64)
    pk = ((i[:, None] * 7 + np.arange(64, dtype=np.uint64)[None, :] * 13) & 0xff).astype(np.uint8)
    b = pk[:, 0].astype(np.uint64)
    closed = np.where(b <= 0x70, 0x71, np.where(b > 0xc0, 0x170, 0x70)).astype(np.uint64)
    return pk, closed


def check(code, got, n):
    pk, closed = expected(n)
    np.testing.assert_array_equal(got, closed)
    want, wf, _, _ = pyoracle.OracleProgram(code).run(pk, n, 64)
    assert not wf.any()
    np.testing.assert_array_equal(got, want)


def test_consumer_program_cpu(tmp_path):
    exe = build_consumer(tmp_path)
    code, got = run_consumer(exe, "cpu", 4096, tmp_path)
    check(code, got, 4096)


@pytest.mark.gpu
def test_consumer_program_batch_gpu(tmp_path):
    exe = build_consumer(tmp_path)
    n = (1 << 20) + 13
    code, got = run_consumer(exe, "batch", n, tmp_path)
    check(code, got, n)


def _build_pcap_consumer(tmp_path):
    r, exe = _cc(["-I", INC, os.path.join(ROOT, "tests", "c", "pcap_async_consumer.c"),
                  "-L", LIBDIR, "-Wl,-rpath," + LIBDIR, "-lebpf"], tmp_path, "pcap_async")
    assert r.returncode == 0, r.stderr.decode()
    return exe


def test_pcap_consumer_c_cpu(tmp_path):
    """include/ebpf_gpu.h's pcap entry point from C: a capture built in memory becomes a batch
    whose offsets and bytes are the records'."""
    exe = _build_pcap_consumer(tmp_path)
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 0 and r.stdout.decode().strip() == "ok", (r.stdout, r.stderr)


@pytest.mark.gpu
def test_pcap_async_consumer_c_gpu(tmp_path):
    """The same C consumer runs a program over the capture with ebpf_prog_run_batch_async /
    ebpf_batch_wait and checks every verdict and MEM fault."""
    exe = _build_pcap_consumer(tmp_path)
    r = subprocess.run([exe, "gpu"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 0 and r.stdout.decode().strip() == "ok", (r.stdout, r.stderr)
