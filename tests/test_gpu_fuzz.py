"""The GPU fuzzer (tools/fuzz_gpu.py) inside the suite, on seeds the fixed-seed parity tests do
not use: random programs under the reference's semantics with array maps (every variant, staged
and general kernels) and with hashtables, standard-semantics programs (loop-free,
counted loops, cursor walks), programs that write maps inside loops (round 5), reference
programs with more than 16 map writes on one path and loop programs mixing every kind of write
in one hashtable's values (round 6), and randomly
edited programs the oracle finds defined.  Each mode
compares results, fault codes, packet bytes after the batch and the maps with the oracle.  The
long campaigns (thousands of programs per configuration) stay in tools/fuzz_gpu.py; their logs
are under profiles/r03/fuzz/."""
import argparse
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _args(**kw):
    a = argparse.Namespace(programs=150, seed=11, hash=False, standard=False, mutate=False)
    a.__dict__.update(kw)
    return a


@pytest.fixture(scope="module")
def fuzz(gpu):
    import fuzz_gpu
    return fuzz_gpu


@pytest.mark.parametrize("maps", [False, True])
def test_value_range_campaign(gpu, env, maps):
    """tools/fuzz_facts.py (round 6): straight-line programs aimed at the compiled code's
    value-range facts (loads, fused swaps, ALU, shifts, multiplies; with maps: stack forwarding
    and register-keyed lookups) on the compiled path and the assembly interpreter"""
    import fuzz_facts
    assert not fuzz_facts.campaign(env, 300, 161 + int(maps), (0, 2), maps)


@pytest.mark.parametrize("mode", ["reference", "hash", "standard", "mutate", "loopwrites",
                                  "loopfetched", "loophash", "manywrites"])
def test_fuzz_campaign(fuzz, env, mode):
    if mode == "reference":
        failed = fuzz.reference(_args(seed=11), env)
    elif mode == "hash":
        failed = fuzz.reference(_args(seed=12, hash=True), env)
    elif mode == "standard":
        failed = fuzz.standard(_args(seed=13, programs=80, standard=True), env)
    elif mode == "loopwrites":
        failed = fuzz.loop_writes(_args(seed=15, programs=40), env)
    elif mode == "loopfetched":   # (counters read back inside loops: 40 of them fetch)
        failed = fuzz.loop_writes(_args(seed=17, programs=120, fetched=True), env)
    elif mode == "loophash":   # (hashtable counters, stores, loads and updates inside loops)
        failed = fuzz.loop_writes(_args(seed=18, programs=60, hash=True), env)
    elif mode == "manywrites":   # (more than 16 writes on a loop-free path: no limit)
        failed = fuzz.reference(_args(seed=16, programs=60, manywrites=True), env)
    else:
        failed = fuzz.mutated(_args(seed=14, programs=200, mutate=True), env)
    assert not failed, "mismatches (see the captured output for the failing program numbers)"
