#!/usr/bin/env python3
"""Generate the hand-written gfx950 (CDNA4) assembly interpreter for the device program.

Output: <out>.s (the code object source: two interpreter kernels sharing one handler set, the
handler linker kernel, the handler offset table) and <out>.h (handler family ids for the host
lowering in asm_runtime.cpp).

Execution model (one lane = one packet, wavefront-lockstep dispatch):
  * eBPF register rK lives in v[2K:2K+1] (VGPRs, never memory);
  * every handler is specialised for its (operation, dst, src) so no register is indexed at
    run time; a dispatch is  s_load_dwordx8 entry -> s_waitcnt -> s_setpc_b64 handler;
  * the wave-uniform entry (32 B, dprog.h layout with `handler` linked to an absolute code
    address) is fetched with scalar loads (K$), so decoding costs no VALU;
  * in the staged kernel each lane's 64-B packet is loaded with 4 x global_load_dwordx4 into
    v22..v37 and packet loads at translation-time-known offsets read registers;
  * the 512-B eBPF stack lives in LDS (per-lane slice sized from the translated program);
  * lanes that disagree on a conditional jump are parked (v41 = their entry) and resumed after
    the running group retires; retirement writes r0, the fault code and an LDS histogram.
"""
import os
import re
import sys

NREG = 11
# cache policy of the streaming accesses (EBPF_ASM_NT bit 0 = ret stores nt, bit 1 = packet DMA
# loads nt).  Both nt by default: the once-read packet stream with nt DMA reads 6.75 TB/s against
# 6.06 TB/s default policy (tools/ubench/floor.hip, profiles/r01/ubench/)
_NT = int(os.environ.get("EBPF_ASM_NT", "3"))
ST_POLICY = " nt" if _NT & 1 else ""
LD_POLICY = " nt" if _NT & 2 else ""
# explicit cache-policy strings (A/B probes of the gfx950 sc0/sc1/nt bits), "+"-separated,
# e.g. EBPF_ASM_LDPOL=sc1+nt ("none" = no bits)
# hashtable probe loads (A/B: EBPF_ASM_PROBEPOL, same form; default policy)
PROBE_POLICY = ""
for _v, _n in (("EBPF_ASM_STPOL", "ST_POLICY"), ("EBPF_ASM_LDPOL", "LD_POLICY"),
               ("EBPF_ASM_PROBEPOL", "PROBE_POLICY")):
    if os.environ.get(_v):
        _p = os.environ[_v].replace("+", " ")
        globals()[_n] = "" if _p == "none" else " " + _p
# ---------------------------------------------------------------- register plan
PKT0 = 22            # v22..v37 staged packet dwords (staged kernel)
V_PKT = 38           # v[38:39] packet base address
V_LEN = 40           # packet length (bytes)
V_T = 41             # parked entry byte offset
V_STK = 42           # lane stack bottom (LDS byte address)
V_L16 = 43           # staged image: lane * 16 (LDS-DMA staging offset)
V_IDX = 43           # general image: the lane's packet index in the launch
# v[44:45] (RETK == 1) or v[64:64+2*RETK]: r0 of the lanes that retired, per group of the
# current superblock (stored together at the start of the next superblock)
H = [46, 47, 48, 49, 50, 51]         # handler temporaries
R = list(range(52, 63))              # routine temporaries
V_SEL = 63                           # v_perm selector 0x00010203 (byte swap)
# Results of RETK consecutive groups are kept in VGPRs and written as one RETK x 512-B burst
# (RETK > 1 adds 2*RETK VGPRs at v64).  Each wave walks superblocks of RETK consecutive groups.
# Default 8: one aligned 4-KB result burst per wave reads+writes at 5.6-5.7 TB/s against
# 5.1 TB/s for 512-B stores (floor.hip), worth the 6 instead of 8 waves per SIMD it costs.
# Two code objects are generated: the staged (fixed 64-B) kernels use RETK_STAGED, the general
# kernels (any stride / offsets: latency-bound per-packet loads, where the 8 waves per SIMD of
# RETK = 1 matter more than the store burst) use RETK = 1.
RETK_STAGED = int(os.environ.get("EBPF_ASM_RETK", "8"))
assert RETK_STAGED in (1, 2, 4, 8)


STAGED_IMAGE = True   # set per generated image (generate())

# Launch-private verdict partials (dp_launch.hist_rows, shared with asm_runtime.cpp): 8 replicas
# of EBPF_HIST_BINS u64 (bin 256 of replica 0 = the fault count), then the u32 arrival tickets:
# one per replica and a top one, each on a 64-B line of its own.
HIST_REPLICAS = 8
HIST_REPLICA_BYTES = 257 * 8
HIST_TICKET_OFF = HIST_REPLICAS * HIST_REPLICA_BYTES


def set_retk(k):
    global RETK, V_RB, NVGPR, SLOTS
    RETK = k
    V_RB = 44 if RETK == 1 else 64
    NVGPR = 64 if RETK == 1 else 64 + 2 * RETK
    # result slots: RETK, and 16 in the staged image with result bursts, whose wide kernel
    # (ebpf_jit_s64w) allocates the second 8 for write phasing (store_phased)
    SLOTS = 16 if RETK == 8 else RETK


set_retk(RETK_STAGED)

# SGPRs (next_free_sgpr 80 -> 8 waves per SIMD)
S_CB = 4             # s[4:5] code base (.Lcb): routines are reached at S_CB + (label - .Lcb)
S_ENT = 8            # s[8:15] current entry: s[8:9] handler, s[10:11] imm, s12 next, s13 target,
                     # s14 aux0, s15 aux1
S_ALIVE = 16         # s[16:17]
S_SAVE = 18          # s[18:19]
S_PROG, S_MAPS, S_DATA, S_OFFS, S_OFFBASE, S_RET, S_FAULTS, S_HIST = 20, 22, 24, 26, 28, 30, 32, 34
S_COUNT, S_STRIDE, S_START, S_NMAPS, S_NENT = 36, 38, 39, 40, 41
S_STKSTRIDE, S_LDSBASE = 42, 43      # dp_launch.stack_stride, .lds_stack_base
S_GROUP, S_GSTRIDE, S_NGROUPS, S_PKTLDS = 44, 45, 46, 47
S_MASK = 48          # s[48:49] temp mask
S_LINK = 50          # s[50:51] subroutine return address
S_CODE = 52          # fault code argument
S_T0, S_T1, S_T2, S_T3 = 53, 54, 55, 56
S_BYTES = 57         # check routine scratch
S_SHARED = 58        # s[58:59] src_shared_base
S_JUNK = 60          # s[60:61] scratch sdst
S_OK = 62            # s[62:63] check: accumulated ok lanes
S_REC = 64           # s[64:71] map record {handle, dev_base, value_size, max_entries, lds_off, pad}
S_PREVG = 72         # group whose results are still in V_RET (-1: none)
S_KMASK = 73         # superblock size - 1 of this launch (K' <= RETK, a power of two; host-chosen,
                     # dp_launch.total_waves bits 28..29 = log2 K'): small batches use shorter
                     # superblocks so that every wave gets work
S_WAVE = 3
NSGPR = 76           # + VCC, XNACK, FLAT_SCRATCH; s[74:75]: compiled programs' short-lane mask
                     # in the general image (asm_cc.cpp ldxpkc_general)
# general image: s[76:77] = the run mask of a compiled program's hoisted packet loads (asm_cc.cpp
# runmask: the running lanes whose packet holds every load of the run)
S_RUNMASK = 76
NSGPR_GEN = 88
# staged image: s[74:75] .. s[96:97] hold the taken-lane masks of a structured compiled program's
# pending branches (asm_jit.cpp; 12 levels); 98 SGPRs still allow the image's 6 waves per SIMD
S_JOIN = 74
JOIN_LEVELS = 12
# staged image with result bursts (RETK > 1): s98 = the result slots holding unwritten groups
# (bit k = slot k), s99 = dp_launch.wphase (store_phased)
S_PEND = S_JOIN + 2 * JOIN_LEVELS
S_WPHASE = S_PEND + 1
S_CLOCK = S_WPHASE + 1   # s[100:101]: the constant clock, read at the group's start
NSGPR_STAGED = S_CLOCK + 2
# (no join SGPRs in the general image: s74..s97 would overlap the run mask and the short-lane
# mask, and structured exits address the LDS histogram through lane 0 of v43, which the general
# image uses for V_IDX; AH_GEN_JOIN stays 0)
GEN_JOIN = 0
# general image: spare VGPRs v64.. for packet loads the code generator issues ahead (asm_cc.cpp
# hoist plan); 16 cost the general kernels 8 -> 6 waves per SIMD
GEN_HOIST_REGS = int(os.environ.get("EBPF_ASM_GENHOIST", "16"))
ALU64R = ["ADD", "SUB", "MUL", "OR", "AND", "XOR", "LSH", "RSH", "DIV", "MOD"]
ALU32R = ["ADD", "SUB", "MUL", "OR", "AND", "XOR", "LSH", "RSH", "MOV", "DIV", "MOD"]
ALU64I = ["ADD", "MUL", "OR", "AND", "XOR", "LSH", "RSH", "DIV", "MOD", "MOV"]   # MOV = LDDW
ALU32I = ["ADD", "SUB", "MUL", "OR", "AND", "XOR", "LSH", "RSH", "MOV", "DIV", "MOD"]
CONDS = ["JEQ", "JNE", "JGT", "JGE", "JLT", "JLE", "JSGT", "JSGE", "JSLT", "JSLE", "JSET"]
SIZES = [1, 2, 4, 8]

FAMILIES = []   # (name, arity) arity: 2 = (dst, src), 1 = (reg), 0


def fam(name, arity):
    FAMILIES.append((name, arity))


for o in ALU64R:
    fam("A64R_" + o, 2)
for o in ALU32R:
    fam("A32R_" + o, 2)
for c in CONDS:
    fam(c + "_R", 2)
for z in SIZES:
    fam("LDXGEN%d" % z, 2)
for z in SIZES:
    fam("STXGEN%d" % z, 2)
for z in SIZES:
    fam("LDXMAP%d" % z, 2)
for o in ALU64I:
    fam("A64I_" + o, 1)
for o in ALU32I:
    fam("A32I_" + o, 1)
for w in (16, 32, 64):
    fam("BSWAP%d" % w, 1)
for c in CONDS:
    fam(c + "_I", 1)
for z in SIZES:
    fam("LDXPKTG%d" % z, 1)
for z in SIZES:
    fam("LDXSTK%d" % z, 1)
for z in SIZES:
    fam("STXSTK%d" % z, 1)
for z in SIZES:
    fam("STGEN%d" % z, 1)
for z in SIZES:
    fam("STSTK%d" % z, 0)
for n in ("EXIT", "FAULT", "NOP", "LOOKUPSTK", "LOOKUPGEN"):
    fam(n, 0)
for z in SIZES:
    fam("LDXPKC%d" % z, 3)      # staged packet load at a constant byte offset: (dst, offset)
fam("HLOOKUP", 0)              # hashtable lookup, map known at translation time (s14 = record offset)
fam("UPDATE", 0)               # map_update_elem, map known (s14 = record offset, s15 = entry index)
for z in SIZES:
    fam("LDXHV%d" % z, 2)       # load from a hashtable value (lookup result), in range by provenance
# standard-eBPF semantics (ebpf_prog_set_semantics): the operations whose meaning differs from
# the reference's, and the JMP32 class
fam("MOV64R", 2)
fam("NEG64", 1)
fam("NEG32", 1)
fam("ARSH64I", 1)
fam("ARSH64R", 2)
fam("ARSH32I", 1)
fam("ARSH32R", 2)
for o in ("DIV64Z", "MOD64Z", "DIV32Z", "MOD32Z"):
    fam(o, 2)                  # register divisor; zero gives 0 (DIV) or dst (MOD)
for c in CONDS:
    fam("J32" + c[1:] + "_R", 2)
for c in CONDS:
    fam("J32" + c[1:] + "_I", 1)
# loops under standard semantics (dprog.h DK_LOOPINIT / DK_LOOPCNT): the lane's count of taken
# backward jumps in the first 4 bytes of its stack slice (below the frame the program addresses)
fam("LOOPINIT", 0)
fam("LOOPCNT", 0)
fam("HDELETE", 0)              # map_delete_elem on a hashtable known at translation time (s14, s15)
# interpreter superinstructions (asm_runtime.cpp asm_fuse_interp; staged kernels): a packet load at
# a constant offset fused with the BE16 / BE32 of its destination (dst, offset)
fam("LDXPKBE16", 3)
fam("LDXPKBE32", 3)
# stores into map values (ebpf_gpu.h "Stores into map values"; dprog.h DK_CNT_STORE / DK_XADD):
# the STX of a counter update (d = the pointer, s = the value), XADD (d = the pointer, s = the
# addend) and XADD | FETCH (d = the addend, which receives the old value; s = the pointer)
for z in (4, 8):
    fam("CNTST%d" % z, 2)
for z in (4, 8):
    fam("XADD%d" % z, 2)
for z in (4, 8):
    fam("XADDF%d" % z, 2)
fam("OVLINIT", 0)              # dprog.h DK_OVLINIT: the lane's overlay and write counts = 0
# a counter update the translator resolved completely (asm_runtime.cpp): an immediate addend
# (s[10:11]) into a DP_MAP_ATOMIC map's delta area at r_d + s14 (d = the value pointer, a
# non-NULL lookup result; s14 = the offset + the map's delta-area offset)
for z in (4, 8):
    fam("CNTAI%d" % z, 1)
# ... into the workgroup's LDS sums of a DP_MAP_LDSDELTA map: at (r_d - s15) + s14 (s15 = the
# mirror's address, low word; s14 = the offset + the table's LDS address)
for z in (4, 8):
    fam("CNTAL%d" % z, 1)
# a load through a packet pointer at an offset only known at run time (translate.cpp AV_CTXV:
# a cursor advanced in a loop): one bounds check against the lane's packet, one load; lanes whose
# address leaves the packet take the generic path (s[10:11] = the offset)
for z in SIZES:
    fam("LDXPKTV%d" % z, 2)
LOOP_BUDGET = 1 << 20          # dprog.h DP_LOOP_BUDGET
# the lane's stack slice below the frame (dprog.h DP_OVL_*): loop count, overlay count, the
# scratch a store into a map value is redirected to, the overlay entries
OVL_COUNT, VST_SCRATCH, WCOUNT, OVL_ENTRIES = 4, 8, 16, 24
WRITES_MAX = 16             # dprog.h DP_WRITES_MAX (dp_launch.vflags bit 4, DP_VF_WCAP)
FAULT_WRITES = 11           # include/ebpf_gpu.h EBPF_FAULT_WRITES
WPHASE_OFF = 0xd0              # dp_launch.wphase (store_phased)
VFLAGS_OFF = 0xcc              # dp_launch.vflags: bit 0 overlay, bit 1 value stores provided for
SPILL = 51                     # v51 (H[5]): .Lr_check's SGPR spill lanes around .Lr_vstore


def variants(arity):
    if arity == 3:
        return [(d, o) for o in range(64) for d in range(NREG)]
    if arity == 2:
        return [(d, s) for d in range(NREG) for s in range(NREG)]
    if arity == 1:
        return [(d, None) for d in range(NREG)]
    return [(None, None)]


def lo(r):
    return "v%d" % (2 * r)


def hi(r):
    return "v%d" % (2 * r + 1)


def pair(r):
    return "v[%d:%d]" % (2 * r, 2 * r + 1)


def v(i):
    return "v%d" % i


def vp(i):
    return "v[%d:%d]" % (i, i + 1)


def s(i):
    return "s%d" % i


def sp(i):
    return "s[%d:%d]" % (i, i + 1)


def dispatch(next_reg=12):
    """Fetch the entry at byte offset s[next_reg] (inside the entry being replaced: the offset
    is read when the load issues, and the code object is xnack-, so no replay can re-read it)
    and jump to its handler."""
    return ["s_load_dwordx8 s[8:15], s[%d:%d], s%d" % (S_PROG, S_PROG + 1, next_reg),
            "s_waitcnt lgkmcnt(0)",
            "s_setpc_b64 s[8:9]"]


_ENT_REF = re.compile(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]")


def early_fetch_point(body):
    """Interpreter image: where in a straight-line handler body the next entry's fetch can issue
    — right after the body's last reference to the entry SGPRs s[8:15] (the load overwrites them
    when it lands; its offset s12 is read at issue) — so that the fetch's latency overlaps the
    rest of the body.  None when the body branches, calls, or waits on a partial lgkmcnt."""
    last = -1
    for i, ln in enumerate(body):
        if ln.endswith(":") or ln.split(" ")[0] in ("s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz",
                                                    "s_cbranch_vccnz", "s_cbranch_execz",
                                                    "s_cbranch_execnz", "s_branch", "s_setpc_b64",
                                                    "s_swappc_b64"):
            return None
        for a, b, c in _ENT_REF.findall(ln):
            lo_, hi_ = (int(a), int(a)) if a else (int(b), int(c))
            if lo_ <= 15 and hi_ >= 8:
                last = i
    rest = body[last + 1:]
    if any("lgkmcnt(" in ln and "lgkmcnt(0)" not in ln for ln in rest):
        return None
    return last + 1


def raddr(label, pair_):
    return ["s_add_u32 %s, %s, %s-.Lcb" % (s(pair_), s(S_CB), label),
            "s_addc_u32 %s, %s, 0" % (s(pair_ + 1), s(S_CB + 1))]


def call(label):
    """Call a routine: its address is formed in the link pair, which the swap then
    overwrites with the return address (a routine that calls another saves its own link)."""
    return raddr(label, S_LINK) + ["s_swappc_b64 %s, %s" % (sp(S_LINK), sp(S_LINK))]


def goto(label):
    """Jump to a routine through the scratch pair (the link pair may be live: tail calls)."""
    return raddr(label, S_JUNK) + ["s_setpc_b64 %s" % sp(S_JUNK)]


def fault_mask(mask_sgpr_pair, code):
    """Retire the lanes in s[mask] with fault `code`; returns (or never, if none remain)."""
    out = []
    if mask_sgpr_pair != S_MASK:
        out.append("s_mov_b64 %s, %s" % (sp(S_MASK), sp(mask_sgpr_pair)))
    out += ["s_mov_b32 %s, %d" % (s(S_CODE), code)] + call(".Lr_fault")
    return out


# ---------------------------------------------------------------- handler bodies
def h_alu64r(op, d, sr):
    D0, D1, S0, S1 = lo(d), hi(d), lo(sr), hi(sr)
    t = H
    if op == "ADD":
        return ["v_lshl_add_u64 %s, %s, 0, %s" % (pair(d), pair(sr), pair(d))]
    if op == "SUB":
        return ["v_sub_co_u32 %s, vcc, %s, %s" % (D0, D0, S0),
                "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (D1, D1, S1)]
    if op == "MUL":
        return ["v_mad_u64_u32 %s, %s, %s, %s, 0" % (vp(t[0]), sp(S_JUNK), D0, S0),
                "v_mul_lo_u32 %s, %s, %s" % (v(t[2]), D0, S1),
                "v_mul_lo_u32 %s, %s, %s" % (v(t[3]), D1, S0),
                "v_add3_u32 %s, %s, %s, %s" % (D1, v(t[1]), v(t[2]), v(t[3])),
                "v_mov_b32 %s, %s" % (D0, v(t[0]))]
    if op in ("OR", "AND", "XOR"):
        m = {"OR": "v_or_b32", "AND": "v_and_b32", "XOR": "v_xor_b32"}[op]
        return ["%s %s, %s, %s" % (m, D0, D0, S0), "%s %s, %s, %s" % (m, D1, D1, S1)]
    if op == "LSH":
        return ["v_lshlrev_b64 %s, %s, %s" % (pair(d), S0, pair(d))]
    if op == "RSH":
        return ["v_lshrrev_b64 %s, %s, %s" % (pair(d), S0, pair(d))]
    if op in ("DIV", "MOD"):
        return divmod_body(d, sr, None, op, 64)
    raise ValueError(op)


def h_alu32r(op, d, sr):
    D0, D1, S0 = lo(d), hi(d), lo(sr)
    body = {
        "ADD": ["v_add_u32 %s, %s, %s" % (D0, D0, S0)],
        "SUB": ["v_sub_u32 %s, %s, %s" % (D0, D0, S0)],
        "MUL": ["v_mul_lo_u32 %s, %s, %s" % (D0, D0, S0)],
        "OR": ["v_or_b32 %s, %s, %s" % (D0, D0, S0)],
        "AND": ["v_and_b32 %s, %s, %s" % (D0, D0, S0)],
        "XOR": ["v_xor_b32 %s, %s, %s" % (D0, D0, S0)],
        "LSH": ["v_lshlrev_b32 %s, %s, %s" % (D0, S0, D0)],
        "RSH": ["v_lshrrev_b32 %s, %s, %s" % (D0, S0, D0)],
        "MOV": ["v_mov_b32 %s, %s" % (D0, S0)],
    }
    if op in ("DIV", "MOD"):
        return divmod_body(d, sr, None, op, 32)
    return body[op] + ["v_mov_b32 %s, 0" % D1]


def h_alu64i(op, d):
    D0, D1 = lo(d), hi(d)
    t = H
    if op == "ADD":
        return ["v_lshl_add_u64 %s, s[10:11], 0, %s" % (pair(d), pair(d))]
    if op == "MUL":
        return ["v_mad_u64_u32 %s, %s, %s, s10, 0" % (vp(t[0]), sp(S_JUNK), D0),
                "v_mul_lo_u32 %s, %s, s11" % (v(t[2]), D0),
                "v_mul_lo_u32 %s, %s, s10" % (v(t[3]), D1),
                "v_add3_u32 %s, %s, %s, %s" % (D1, v(t[1]), v(t[2]), v(t[3])),
                "v_mov_b32 %s, %s" % (D0, v(t[0]))]
    if op in ("OR", "AND", "XOR"):
        m = {"OR": "v_or_b32", "AND": "v_and_b32", "XOR": "v_xor_b32"}[op]
        return ["%s %s, s10, %s" % (m, D0, D0), "%s %s, s11, %s" % (m, D1, D1)]
    if op == "LSH":
        return ["v_lshlrev_b64 %s, s10, %s" % (pair(d), pair(d))]
    if op == "RSH":
        return ["v_lshrrev_b64 %s, s10, %s" % (pair(d), pair(d))]
    if op == "MOV":
        return ["v_mov_b32 %s, s10" % D0, "v_mov_b32 %s, s11" % D1]
    if op in ("DIV", "MOD"):
        return divmod_body(d, None, True, op, 64)
    raise ValueError(op)


def h_alu32i(op, d):
    D0, D1 = lo(d), hi(d)
    body = {
        "ADD": ["v_add_u32 %s, s10, %s" % (D0, D0)],
        "SUB": ["v_subrev_u32 %s, s10, %s" % (D0, D0)],
        "MUL": ["v_mul_lo_u32 %s, %s, s10" % (D0, D0)],
        "OR": ["v_or_b32 %s, s10, %s" % (D0, D0)],
        "AND": ["v_and_b32 %s, s10, %s" % (D0, D0)],
        "XOR": ["v_xor_b32 %s, s10, %s" % (D0, D0)],
        "LSH": ["v_lshlrev_b32 %s, s10, %s" % (D0, D0)],
        "RSH": ["v_lshrrev_b32 %s, s10, %s" % (D0, D0)],
        "MOV": ["v_mov_b32 %s, s10" % D0],
    }
    if op in ("DIV", "MOD"):
        return divmod_body(d, None, True, op, 32)
    return body[op] + ["v_mov_b32 %s, 0" % D1]


def divmod_body(d, sr, imm, op, bits, zero_ok=False):
    """Operands to R[0:1] (n) and R[2:3] (den); lanes with den == 0 fault DIV_ZERO (the
    reference raises SIGFPE), or with zero_ok (standard eBPF) get 0 (DIV) or n (MOD: the
    divider's remainder for a zero divisor is n); quotient / remainder from the shared
    restoring divider."""
    n0, n1, d0, d1 = v(R[0]), v(R[1]), v(R[2]), v(R[3])
    out = ["v_mov_b32 %s, %s" % (n0, lo(d))]
    out.append("v_mov_b32 %s, %s" % (n1, hi(d) if bits == 64 else "0"))
    if imm:
        out += ["v_mov_b32 %s, s10" % d0, "v_mov_b32 %s, %s" % (d1, "s11" if bits == 64 else "0")]
    else:
        out += ["v_mov_b32 %s, %s" % (d0, lo(sr)),
                "v_mov_b32 %s, %s" % (d1, hi(sr) if bits == 64 else "0")]
    if not imm and not zero_ok:  # (immediate zero divisors are resolved by the translator)
        out += ["v_cmp_eq_u64_e64 %s, %s, 0" % (sp(S_MASK), vp(R[2])),
                "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
                "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
                "s_cbranch_scc1 .Ldz_%s" % "{uid}"]
        out += fault_mask(S_MASK, 2)
        out.append(".Ldz_{uid}:")
    out += call(".Lr_udiv")
    q0, q1, r0, r1 = v(R[4]), v(R[5]), v(R[6]), v(R[7])
    if zero_ok and op == "DIV":
        out += ["v_cmp_eq_u64_e64 vcc, 0, %s" % vp(R[2]),
                "v_cndmask_b32_e64 %s, %s, 0, vcc" % (q0, q0),
                "v_cndmask_b32_e64 %s, %s, 0, vcc" % (q1, q1)]
    src = (q0, q1) if op == "DIV" else (r0, r1)
    out += ["v_mov_b32 %s, %s" % (lo(d), src[0]),
            "v_mov_b32 %s, %s" % (hi(d), src[1] if bits == 64 else "0")]
    return out


CMP = {"JEQ": "eq_u64", "JNE": "ne_u64", "JGT": "gt_u64", "JGE": "ge_u64", "JLT": "lt_u64",
       "JLE": "le_u64", "JSGT": "gt_i64", "JSGE": "ge_i64", "JSLT": "lt_i64", "JSLE": "le_i64"}


def h_cond(c, d, sr, imm):
    srcop = "s[10:11]" if imm else pair(sr)
    out = []
    if c == "JSET":
        if imm:
            out += ["v_and_b32 %s, s10, %s" % (v(H[0]), lo(d)),
                    "v_and_b32 %s, s11, %s" % (v(H[1]), hi(d))]
        else:
            out += ["v_and_b32 %s, %s, %s" % (v(H[0]), lo(d), lo(sr)),
                    "v_and_b32 %s, %s, %s" % (v(H[1]), hi(d), hi(sr))]
        out.append("v_cmp_ne_u64_e64 vcc, %s, 0" % vp(H[0]))
    else:
        out.append("v_cmp_%s_e64 vcc, %s, %s" % (CMP[c], pair(d), srcop))
    # (no lane taken, the usual uniform case, costs two scalar instructions: the AND's SCC says
    # whether any lane takes the branch)
    out += ["@CMPEND",
            "s_and_b64 %s, vcc, exec" % sp(S_MASK),
            "s_cbranch_scc0 .Lnt_{uid}",
            "s_cmp_eq_u64 %s, exec" % sp(S_MASK),
            "s_cbranch_scc1 .Ltk_{uid}",
            ] + goto(".Lr_diverge") + [
            ".Ltk_{uid}:"] + dispatch(13) + [".Lnt_{uid}:"] + dispatch(12)
    return out, True   # (body, has own dispatch)


CMP32 = {"JEQ": "eq_u32", "JNE": "ne_u32", "JGT": "gt_u32", "JGE": "ge_u32", "JLT": "lt_u32",
         "JLE": "le_u32", "JSGT": "gt_i32", "JSGE": "ge_i32", "JSLT": "lt_i32", "JSLE": "le_i32"}


def h_cond32(c, d, sr, imm):
    """JMP32: the compare of the low 32 bits (s10 = u32(imm) for the immediate form)."""
    srcop = "s10" if imm else lo(sr)
    if c == "JSET":
        out = ["v_and_b32 %s, %s, %s" % (v(H[0]), srcop, lo(d)),
               "v_cmp_ne_u32_e64 vcc, 0, %s" % v(H[0])]
    else:
        out = ["v_cmp_%s_e64 vcc, %s, %s" % (CMP32[c], lo(d), srcop)]
    body, own = h_cond(c, d, sr, imm)
    return out + body[body.index("@CMPEND"):], own


def h_std(name, d, sr):
    """Standard-eBPF operations (ebpf_gpu.h EBPF_SEM_STANDARD)."""
    D0, D1 = lo(d), hi(d)
    if name == "MOV64R":
        return ["v_mov_b64 %s, %s" % (pair(d), pair(sr))]
    if name == "NEG64":
        return ["v_sub_co_u32 %s, vcc, 0, %s" % (D0, D0),
                "v_subb_co_u32 %s, vcc, 0, %s, vcc" % (D1, D1)]
    if name == "NEG32":
        return ["v_sub_u32 %s, 0, %s" % (D0, D0), "v_mov_b32 %s, 0" % D1]
    if name == "ARSH64I":
        return ["v_ashrrev_i64 %s, s10, %s" % (pair(d), pair(d))]
    if name == "ARSH64R":
        return ["v_ashrrev_i64 %s, %s, %s" % (pair(d), lo(sr), pair(d))]
    if name == "ARSH32I":
        return ["v_ashrrev_i32 %s, s10, %s" % (D0, D0), "v_mov_b32 %s, 0" % D1]
    if name == "ARSH32R":
        return ["v_ashrrev_i32 %s, %s, %s" % (D0, lo(sr), D0), "v_mov_b32 %s, 0" % D1]
    op, bits = name[:3], int(name[3:5])
    return divmod_body(d, sr, None, op, bits, zero_ok=True)


def h_bswap(w, d):
    D0, D1 = lo(d), hi(d)
    if w == 16:
        return ["v_perm_b32 %s, 0, %s, v%d" % (D0, D0, V_SEL),
                "v_lshrrev_b32 %s, 16, %s" % (D0, D0), "v_mov_b32 %s, 0" % D1]
    if w == 32:
        return ["v_perm_b32 %s, 0, %s, v%d" % (D0, D0, V_SEL), "v_mov_b32 %s, 0" % D1]
    return ["v_perm_b32 %s, 0, %s, v%d" % (v(H[0]), D0, V_SEL),
            "v_perm_b32 %s, 0, %s, v%d" % (D0, D1, V_SEL),
            "v_mov_b32 %s, %s" % (D1, v(H[0]))]


def h_ldx_pkt_staged(z, d):
    """s10 = dword index k of the packet byte offset, s11 = byte shift (offset % 4)."""
    t0, t1, t2 = v(H[0]), v(H[1]), v(H[2])
    out = ["s_set_gpr_idx_on s10, gpr_idx(SRC0)",
           "v_mov_b32 %s, v%d" % (t0, PKT0),
           "v_mov_b32 %s, v%d" % (t1, PKT0 + 1)]
    if z == 8:
        out.append("v_mov_b32 %s, v%d" % (t2, PKT0 + 2))
    out.append("s_set_gpr_idx_off")
    D0, D1 = lo(d), hi(d)
    if z == 8:
        out += ["v_alignbyte_b32 %s, %s, %s, s11" % (D0, t1, t0),
                "v_alignbyte_b32 %s, %s, %s, s11" % (D1, t2, t1)]
    elif z == 4:
        out += ["v_alignbyte_b32 %s, %s, %s, s11" % (D0, t1, t0), "v_mov_b32 %s, 0" % D1]
    else:
        out += ["v_alignbyte_b32 %s, %s, %s, s11" % (t0, t1, t0),
                "v_and_b32 %s, %s, %s" % (D0, "0xff" if z == 1 else "0xffff", t0),
                "v_mov_b32 %s, 0" % D1]
    return out


def h_ldx_pkt_const(z, d, off):
    """Packet load at a translation-time byte offset from the packet bytes held in v22..v37,
    so 1-2 VALU (bit-field extract / byte align), no indexing.  Staged kernels: every packet is
    exactly 64 bytes.  General kernels (header staging, s7 bit 3): lanes whose packet is shorter
    than off + z fault MEM, lanes shorter than 64 bytes (not staged) load from memory."""
    if off + z > 64:
        return []          # never selected: the lowering faults such loads statically
    if not STAGED_IMAGE:
        out = ["v_cmp_gt_u32_e64 %s, %d, v%d" % (sp(S_MASK), off + z, V_LEN),
               "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
               "s_cbranch_scc0 .Lok_{uid}"] + fault_mask(S_MASK, 3) + [".Lok_{uid}:"]
        out += _pkc_extract(z, d, off)
        ld = {1: "global_load_ubyte", 2: "global_load_ushort", 4: "global_load_dword",
              8: "global_load_dwordx2"}[z]
        out += ["v_cmp_gt_u32_e64 %s, 64, v%d" % (sp(S_MASK), V_LEN),
                "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
                "s_cbranch_scc0 .Lst_{uid}",
                "s_mov_b64 %s, exec" % sp(S_JUNK),
                "s_mov_b64 exec, %s" % sp(S_MASK),
                "%s %s, v[%d:%d], off offset:%d" % (ld, pair(d) if z == 8 else lo(d), V_PKT,
                                                    V_PKT + 1, off),
                "s_waitcnt vmcnt(0)"]
        if z < 8:
            out.append("v_mov_b32 %s, 0" % hi(d))
        return out + ["s_mov_b64 exec, %s" % sp(S_JUNK), ".Lst_{uid}:"]
    return _pkc_extract(z, d, off)


def h_ldx_pkt_be(w, d, off):
    """LDXH / LDXW at a constant packet offset followed by BE16 / BE32 of the same register
    (ebpf_interpreter.c:327-338 then the byte swap of :164-185): one v_perm_b32 gathers the
    bytes in big-endian order from the staged packet dwords (staged kernels only)."""
    z = w // 8
    if not STAGED_IMAGE or off + z > 64:
        return []          # never selected
    k, sh = off >> 2, off & 3
    lo_ = "v%d" % (PKT0 + k)
    hi_ = "v%d" % (PKT0 + k + 1) if k + 1 < 16 else lo_   # (then no byte of it is selected)
    sel = 0
    for i in range(4):
        sel |= ((sh + z - 1 - i) if i < z else 0x0c) << (8 * i)
    return ["s_mov_b32 %s, 0x%x" % (s(S_JUNK), sel),
            "v_perm_b32 %s, %s, %s, %s" % (lo(d), hi_, lo_, s(S_JUNK)),
            "v_mov_b32 %s, 0" % hi(d)]


def _pkc_extract(z, d, off):
    k, sh = off >> 2, off & 3
    lo_, hi_ = "v%d" % (PKT0 + k), "v%d" % (PKT0 + k + 1) if k + 1 < 16 else None
    D0, D1 = lo(d), hi(d)
    if z == 1:
        return ["v_bfe_u32 %s, %s, %d, 8" % (D0, lo_, 8 * sh), "v_mov_b32 %s, 0" % D1]
    if z == 2:
        if sh <= 2:
            return ["v_bfe_u32 %s, %s, %d, 16" % (D0, lo_, 8 * sh), "v_mov_b32 %s, 0" % D1]
        return ["v_alignbyte_b32 %s, %s, %s, 3" % (D0, hi_, lo_),
                "v_bfe_u32 %s, %s, 0, 16" % (D0, D0), "v_mov_b32 %s, 0" % D1]
    if z == 4:
        if sh == 0:
            return ["v_mov_b32 %s, %s" % (D0, lo_), "v_mov_b32 %s, 0" % D1]
        return ["v_alignbyte_b32 %s, %s, %s, %d" % (D0, hi_, lo_, sh), "v_mov_b32 %s, 0" % D1]
    if sh == 0:
        if (PKT0 + k) % 2 == 0:
            return ["v_mov_b64 %s, v[%d:%d]" % (pair(d), PKT0 + k, PKT0 + k + 1)]
        return ["v_mov_b32 %s, %s" % (D0, lo_), "v_mov_b32 %s, %s" % (D1, hi_)]
    h2 = "v%d" % (PKT0 + k + 2)
    return ["v_alignbyte_b32 %s, %s, %s, %d" % (D0, hi_, lo_, sh),
            "v_alignbyte_b32 %s, %s, %s, %d" % (D1, h2, hi_, sh)]


LOADS = {1: "global_load_ubyte", 2: "global_load_ushort", 4: "global_load_dword",
         8: "global_load_dwordx2"}


def h_ldx_pkt_general(z, d):
    """s[10:11] = packet byte offset (>= 0); per-lane bound check against the packet length."""
    t = H
    out = ["v_mov_b32 %s, s10" % v(t[0]),
           "v_add_u32 %s, %d, %s" % (v(t[0]), z, v(t[0])),
           "v_cmp_gt_u32_e64 %s, %s, %s" % (sp(S_MASK), v(t[0]), v(V_LEN)),
           "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
           "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
           "s_cbranch_scc1 .Lok_{uid}"] + fault_mask(S_MASK, 3) + [".Lok_{uid}:"]
    out.append("v_lshl_add_u64 %s, s[10:11], 0, %s" % (vp(t[0]), vp(V_PKT)))
    if z == 8:
        out.append("%s %s, %s, off" % (LOADS[8], pair(d), vp(t[0])))
    else:
        out += ["%s %s, %s, off" % (LOADS[z], lo(d), vp(t[0])), "v_mov_b32 %s, 0" % hi(d)]
    out.append("s_waitcnt vmcnt(0)")
    return out


DS_R = {1: "ds_read_u8", 2: "ds_read_u16", 4: "ds_read_b32"}
DS_W = {1: "ds_write_b8", 2: "ds_write_b16", 4: "ds_write_b32"}


def h_ldx_stk(z, d):
    """s10 = LDS byte offset from the lane's stack bottom (aligned to min(z, 4))."""
    a = v(H[0])
    out = ["v_add_u32 %s, s10, v%d" % (a, V_STK)]
    if z == 8:
        out.append("ds_read2_b32 %s, %s offset1:1" % (pair(d), a))
    else:
        out += ["%s %s, %s" % (DS_R[z], lo(d), a), "v_mov_b32 %s, 0" % hi(d)]
    return out   # the dispatch's lgkmcnt(0) waits for the LDS read


def h_stx_stk(z, sr):
    a = v(H[0])
    out = ["v_add_u32 %s, s10, v%d" % (a, V_STK)]
    if z == 8:
        out.append("ds_write2_b32 %s, %s, %s offset1:1" % (a, lo(sr), hi(sr)))
    else:
        out.append("%s %s, %s" % (DS_W[z], a, lo(sr)))
    return out


def h_st_stk(z):
    """s[10:11] = value (sign-extended imm), s14 = LDS offset."""
    a, x0, x1 = v(H[0]), v(H[1]), v(H[2])
    out = ["v_add_u32 %s, s14, v%d" % (a, V_STK), "v_mov_b32 %s, s10" % x0]
    if z == 8:
        out += ["v_mov_b32 %s, s11" % x1, "ds_write2_b32 %s, %s, %s offset1:1" % (a, x0, x1)]
    else:
        out.append("%s %s, %s" % (DS_W[z], a, x0))
    return out


FLAT_LOAD = {1: "flat_load_ubyte", 2: "flat_load_ushort", 4: "flat_load_dword", 8: "flat_load_dwordx2"}


def gather(a0, acc, tmp, z, tag=None):
    """acc (two VGPRs) = the z bytes at the flat address v[a0:a0+1], little-endian.  z: an int
    (tmp a list of z VGPRs: when every running lane's address is z-aligned, one flat load of z
    bytes; else z byte loads issued together, one wait), or None for S_T0 bytes (4 or 8 at run
    time, byte by byte; tmp one VGPR, `tag` names the label)."""
    if z is not None:
        t = tmp
        out = []
        if z > 1:
            out += ["v_and_b32 %s, %d, %s" % (v(t[0]), z - 1, v(a0)),
                    "v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(t[0])),
                    "s_and_b64 %s, %s, exec" % (sp(S_JUNK), sp(S_JUNK)),
                    "s_cmp_eq_u64 %s, exec" % sp(S_JUNK),
                    "s_cbranch_scc0 .Lg_una_%s" % tag]
        out += ["%s %s, %s" % (FLAT_LOAD[z], vp(acc[0]) if z == 8 else v(acc[0]), vp(a0)),
                "s_waitcnt vmcnt(0) lgkmcnt(0)"]
        if z < 8:
            out.append("v_mov_b32 %s, 0" % v(acc[1]))
        if z == 1:
            return out
        out += ["s_branch .Lg_done_%s" % tag, ".Lg_una_%s:" % tag]
        out += ["flat_load_ubyte %s, %s offset:%d" % (v(t[b]), vp(a0), b) for b in range(z)]
        out += ["s_waitcnt vmcnt(0) lgkmcnt(0)",
                "v_mov_b32 %s, %s" % (v(acc[0]), v(t[0])), "v_mov_b32 %s, 0" % v(acc[1])]
        for b in range(1, z):
            tgt = v(acc[b // 4])
            out.append("v_lshl_or_b32 %s, %s, %d, %s" % (tgt, v(t[b]), 8 * (b % 4), tgt))
        out.append(".Lg_done_%s:" % tag)
        return out
    out = ["v_mov_b32 %s, 0" % v(acc[0]), "v_mov_b32 %s, 0" % v(acc[1])]
    for b in range(z or 8):
        if z is None and b == 4:
            out += ["s_cmp_le_u32 %s, %d" % (s(S_T0), b), "s_cbranch_scc1 .Lg_done_%s" % tag]
        out.append("flat_load_ubyte %s, %s offset:%d" % (v(tmp), vp(a0), b))
        out.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
        tgt = v(acc[b // 4])
        out.append("v_lshl_or_b32 %s, %s, %d, %s" % (tgt, v(tmp), 8 * (b % 4), tgt))
    if z is None:
        out.append(".Lg_done_%s:" % tag)
    return out


def vflags_test(bit, skip):
    """Branches to `skip` when dp_launch.vflags bit `bit` is clear (bit 0, the overlay: s7 bit 13,
    copied at kernel start; other bits: loaded, clobbering S_T3)."""
    if bit == 0:
        return ["s_bitcmp1_b32 s7, 13", "s_cbranch_scc0 %s" % skip]
    return ["s_load_dword %s, s[0:1], 0x%x" % (s(S_T3), VFLAGS_OFF),
            "s_waitcnt lgkmcnt(0)",
            "s_bitcmp1_b32 %s, %d" % (s(S_T3), bit),
            "s_cbranch_scc0 %s" % skip]


def h_ldx_gen(z, d, sr):
    """Generic load: address = r_src + sext(off) (s[10:11]); region check, then byte-wise
    flat loads (packet/map in global memory, stack in LDS via the shared aperture); a program
    that reads its own stores into map values (dp_launch.vflags bit 0) then takes the bytes it
    stored from its overlay (.Lr_ovlfix)."""
    a0 = H[0]
    out = ["v_lshl_add_u64 %s, s[10:11], 0, %s" % (vp(a0), pair(sr)),
           "s_mov_b32 %s, %d" % (s(S_T0), z), "s_mov_b32 %s, 0" % s(S_T1)] + call(".Lr_check")
    out += gather(a0, (H[2], H[3]), [H[4]] + R[:7], z, "{uid}")
    out += vflags_test(0, ".Lnovl_{uid}") + call(".Lr_ovlfix") + [".Lnovl_{uid}:"]
    out += ["v_mov_b32 %s, %s" % (lo(d), v(H[2])), "v_mov_b32 %s, %s" % (hi(d), v(H[3]))]
    return out


def dma_lane_offsets(dst, tmp):
    """dst = lane l's byte offset inside each 1-KB DMA block of a staged group: 64 (l & 15) +
    16 (l >> 4), so DMA q's lane l fetches chunk l >> 4 of packet 16 q + (l & 15) and the LDS
    block holds chunk c of its 16 packets as 256 contiguous bytes (packet m at 16 m).  Each DMA
    instruction still covers its own 1 KB (same cache lines, lanes permuted: the same DMA rate,
    profiles/r05/staging_layout/), and the staging reads of a chunk by 16 lanes are contiguous:
    no LDS bank conflicts (in the packets' own layout lanes 64 B apart collide)."""
    return ["v_bfe_u32 %s, v%d, 4, 4" % (dst, V_L16),
            "v_bfe_u32 %s, v%d, 8, 2" % (tmp, V_L16),
            "v_lshlrev_b32 %s, 4, %s" % (tmp, tmp),
            "v_lshl_or_b32 %s, %s, 6, %s" % (dst, dst, tmp)]


def lds_pkt_dwords(base, save_exec=None):
    """Write the lane's 64 staged bytes (v22..v37) into the wave's LDS packet buffer transposed:
    dword c of lane l at S_PKTLDS + 4 l + 256 c (VGPR `base` = S_PKTLDS + 4 l).  The loads at
    run-time offsets (lds_pkt_read) then read consecutive dwords across the lanes; in the DMA's
    layout (lane l's 64 bytes at S_PKTLDS + 64 l) every lane reading the same offset hit the same
    two banks (C3L: 112M conflict cycles per launch against 9M of LDS instructions)."""
    return ["ds_write_b32 %s, v%d offset:%d" % (base, PKT0 + c, 256 * c) for c in range(16)]


def lds_pkt_read(z, d, A, B, T):
    """d = the z bytes at byte offset T (a VGPR, <= 64 - z) of the lane's packet in the transposed
    LDS buffer (lds_pkt_dwords), A = S_PKTLDS + 4 lane (clobbered): the dwords around the bytes,
    then one byte align by T's low bits (any alignment, no branch; a dword past the lane's 64
    bytes is read but never selected).  Clobbers B, R[0..2]."""
    t0, t1, t2 = v(R[0]), v(R[1]), v(R[2])
    out = ["v_lshrrev_b32 %s, 2, %s" % (B, T),
           "v_lshl_add_u32 %s, %s, 8, %s" % (B, B, A)]
    if z == 1:
        out += ["ds_read_b32 %s, %s" % (t0, B)]
    else:
        out += ["ds_read2_b32 v[%d:%d], %s offset1:64" % (R[0], R[1], B)]
    if z == 8:
        out.append("ds_read_b32 %s, %s offset:512" % (t2, B))
    out += ["s_waitcnt lgkmcnt(0)",
            "v_alignbyte_b32 %s, %s, %s, %s" % (lo(d), t0 if z == 1 else t1, t0, T)]
    if z == 8:
        out.append("v_alignbyte_b32 %s, %s, %s, %s" % (hi(d), t2, t1, T))
    else:
        if z < 4:
            out.append("v_and_b32 %s, %s, %s" % (lo(d), "0xff" if z == 1 else "0xffff", lo(d)))
        out.append("v_mov_b32 %s, 0" % hi(d))
    return out


def h_ldx_pktv(z, d, sr):
    """LDXPKTV: address = r_src + sext(off); when every running lane's address holds z bytes of
    its own packet ([V_PKT, V_PKT + V_LEN)), one flat load (or z byte loads when unaligned) —
    in the staged kernel's keep mode from the LDS packet buffer instead; otherwise the generic
    load (region check, faults) for all of them."""
    a0 = H[0]
    out = ["v_lshl_add_u64 %s, s[10:11], 0, %s" % (vp(a0), pair(sr)),
           "v_sub_co_u32 %s, vcc, %s, v%d" % (v(H[2]), v(a0), V_PKT),
           "v_subb_co_u32 %s, vcc, %s, v%d, vcc" % (v(H[3]), v(a0 + 1), V_PKT + 1)]
    if STAGED_IMAGE:   # (every packet is 64 bytes: one unsigned 64-bit compare of the offset)
        out += ["v_cmp_ge_u64_e64 %s, %d, v[%d:%d]" % (sp(S_JUNK), 64 - z, H[2], H[3])]
    else:
        out += ["v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(H[3])),
                "v_subrev_u32 %s, %d, v%d" % (v(H[4]), z, V_LEN),
                "v_cmp_le_u32_e64 vcc, %s, %s" % (v(H[2]), v(H[4])),
                "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
                "v_cmp_le_u32_e64 vcc, %d, v%d" % (z, V_LEN),
                "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK))]
    out += ["s_and_b64 %s, %s, exec" % (sp(S_JUNK), sp(S_JUNK)),
            "s_cmp_eq_u64 %s, exec" % sp(S_JUNK),
            "s_cbranch_scc0 .Lpv_gen_{uid}"]
    A, B = v(H[4]), v(H[5])
    if STAGED_IMAGE:
        # keep mode (s7 bit 14): the group's packets stay in the wave's LDS packet buffer while
        # the program runs, transposed (lds_pkt_dwords), so read them there
        out += ["s_bitcmp1_b32 s7, 14",
                "s_cbranch_scc0 .Lpv_flat_{uid}",
                "v_lshrrev_b32 %s, 2, v%d" % (A, V_L16),
                "v_add_u32 %s, %s, %s" % (A, s(S_PKTLDS), A)]
    else:
        # general kernels with the headers kept in LDS (s7 bit 14, every lane's first 64 bytes,
        # transposed, when its packet is at least that long): when every running lane's bytes
        # lie in its first 64 and its packet has them staged, read them there
        out += ["s_bitcmp1_b32 s7, 14",
                "s_cbranch_scc0 .Lpv_flat_{uid}",
                "v_cmp_ge_u32_e64 vcc, %d, %s" % (64 - z, v(H[2])),
                "s_and_b64 %s, vcc, exec" % sp(S_MASK),
                "v_cmp_le_u32_e64 vcc, 64, v%d" % V_LEN,
                "s_and_b64 %s, %s, vcc" % (sp(S_MASK), sp(S_MASK)),
                "s_cmp_eq_u64 %s, exec" % sp(S_MASK),
                "s_cbranch_scc0 .Lpv_flat_{uid}",
                "v_mbcnt_lo_u32_b32 %s, -1, 0" % A,
                "v_mbcnt_hi_u32_b32 %s, -1, %s" % (A, A),
                "v_lshl_add_u32 %s, %s, 2, %s" % (A, A, s(S_PKTLDS))]
    out += lds_pkt_read(z, d, A, B, v(H[2]))
    out += ["s_branch .Lpv_done_{uid}", ".Lpv_flat_{uid}:"]
    out += gather(a0, (H[2], H[3]), [H[4]] + R[:7], z, "{uid}f")
    out += ["v_mov_b32 %s, %s" % (lo(d), v(H[2])), "v_mov_b32 %s, %s" % (hi(d), v(H[3])),
            "s_branch .Lpv_done_{uid}",
            ".Lpv_gen_{uid}:"]
    out += h_ldx_gen(z, d, sr)
    out.append(".Lpv_done_{uid}:")
    return out


def h_ldx_map(z, d, sr):
    """Load from an LDS-resident array-map value: r_src is (by pointer provenance) a lookup
    result of one map, i.e. NULL or dev_base + k*value_size + c.  s[10:11] = dev_base - off,
    s13 = map bytes - z (last valid byte offset), s14 = the map's LDS byte address.  Lanes whose
    address leaves the map (NULL, out of range) fault MEM; the rest read the LDS copy (aligned
    by construction: the host only selects this family when the access is)."""
    u0, u1, t = v(H[0]), v(H[1]), v(H[2])
    out = ["v_sub_co_u32 %s, vcc, %s, s10" % (u0, lo(sr)),
           "v_mov_b32 %s, s11" % t,
           "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (u1, hi(sr), t),
           "v_cmp_ge_u32_e64 %s, s13, %s" % (sp(S_MASK), u0),
           "v_cmp_eq_u32_e64 vcc, 0, %s" % u1,
           "s_and_b64 %s, %s, vcc" % (sp(S_MASK), sp(S_MASK)),
           "s_andn2_b64 %s, exec, %s" % (sp(S_MASK), sp(S_MASK)),
           "s_cbranch_scc0 .Lok_{uid}"] + fault_mask(S_MASK, 3) + [".Lok_{uid}:",
           "v_add_u32 %s, s14, %s" % (u0, u0)]
    if z == 8:
        out.append("ds_read2_b32 %s, %s offset1:1" % (pair(d), u0))
    else:
        out += ["%s %s, %s" % (DS_R[z], lo(d), u0), "v_mov_b32 %s, 0" % hi(d)]
    return out


def h_ldx_hv(z, d, sr):
    """Load from a hashtable value: r_src is (by pointer provenance) a lookup result of a
    hashtable map, i.e. NULL or a slot's value address, and the translator proved
    [off, off + z) inside the value (s14 = off, naturally aligned).  NULL lanes fault MEM;
    the rest do one global load (no region walk)."""
    ld = {1: "global_load_ubyte", 2: "global_load_ushort", 4: "global_load_dword",
          8: "global_load_dwordx2"}[z]
    a = vp(H[0])
    out = ["v_cmp_eq_u64_e64 %s, 0, %s" % (sp(S_MASK), pair(sr)),
           "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
           "s_cbranch_scc0 .Lok_{uid}"] + fault_mask(S_MASK, 3) + [".Lok_{uid}:",
           "v_add_co_u32 %s, vcc, s14, %s" % (v(H[0]), lo(sr)),
           "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(H[1]), hi(sr))]
    if z == 8:
        out += ["%s %s, %s, off" % (ld, pair(d), a)]
    else:
        out += ["%s %s, %s, off" % (ld, lo(d), a), "v_mov_b32 %s, 0" % hi(d)]
    return out + ["s_waitcnt vmcnt(0)"]


def store_bytes(a0, vals, z):
    out = []
    for b in range(z):
        src = vals[b // 4]
        if b % 4:
            out.append("v_lshrrev_b32 %s, %d, %s" % (v(H[4]), 8 * (b % 4), src))
            out.append("flat_store_byte %s, %s offset:%d" % (vp(a0), v(H[4]), b))
        else:
            out.append("flat_store_byte %s, %s offset:%d" % (vp(a0), src, b))
    out.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    return out


def h_stx_gen(z, d, sr, kind=1):
    """Generic store: the value in H[2:3] before the region check, which hands stores into map
    values to .Lr_vstore (kind 1: plain, 2: a counter update's STX) and points those lanes'
    address at their scratch; then byte-wise flat stores."""
    a0 = H[0]
    out = ["v_lshl_add_u64 %s, s[10:11], 0, %s" % (vp(a0), pair(d)),
           "v_mov_b32 %s, %s" % (v(H[2]), lo(sr)), "v_mov_b32 %s, %s" % (v(H[3]), hi(sr)),
           "s_mov_b32 %s, %d" % (s(S_T0), z), "s_mov_b32 %s, %d" % (s(S_T1), kind)] + call(".Lr_check")
    return out + store_bytes(a0, [v(H[2]), v(H[3])], z)


def h_xadd(z, p, x, fetch):
    """XADD: *(u32 / u64 *)(r_p + off) += r_x (fetch: r_x = the old value).  The check hands a
    map value's lanes to .Lr_vstore (kind 3), which leaves the old value the packet sees in the
    lane's scratch and points the address there; the read-modify-write below then serves every
    lane alike."""
    a0 = H[0]
    old, nv = (R[0], R[1]), (R[2], R[3])
    out = ["v_lshl_add_u64 %s, s[10:11], 0, %s" % (vp(a0), pair(p)),
           "v_mov_b32 %s, %s" % (v(H[2]), lo(x)), "v_mov_b32 %s, %s" % (v(H[3]), hi(x)),
           "s_mov_b32 %s, %d" % (s(S_T0), z), "s_mov_b32 %s, 3" % s(S_T1)] + call(".Lr_check")
    out += gather(a0, old, [H[4]] + R[4:11], z, "{uid}")
    out += ["v_lshl_add_u64 %s, %s, 0, %s" % (vp(nv[0]), vp(old[0]), vp(H[2]))]
    out += store_bytes(a0, [v(nv[0]), v(nv[1])], z)
    if fetch:
        out += ["v_mov_b32 %s, %s" % (lo(x), v(old[0])),
                "v_mov_b32 %s, %s" % (hi(x), v(old[1]) if z == 8 else "0")]
    return out


def h_st_gen(z, d):
    """s[10:11] = the value (sign-extended imm), s15 = the offset (aux1)."""
    a0 = H[0]
    out = ["s_ashr_i32 %s, s15, 31" % s(S_T3),
           "v_mov_b32 %s, s15" % v(H[2]), "v_mov_b32 %s, %s" % (v(H[3]), s(S_T3)),
           "v_lshl_add_u64 %s, %s, 0, %s" % (vp(a0), vp(H[2]), pair(d)),
           "v_mov_b32 %s, s10" % v(H[2]), "v_mov_b32 %s, s11" % v(H[3]),
           "s_mov_b32 %s, %d" % (s(S_T0), z), "s_mov_b32 %s, 1" % s(S_T1)] + call(".Lr_check")
    return out + store_bytes(a0, [v(H[2]), v(H[3])], z)


def h_lookup_stk():
    """r0 = lookup(map, *(u32*)(r10 + c)) with the map resolved at translation time:
    s[10:11] = device base of the map mirror, s13 = max_entries, s14 = key LDS offset,
    s15 = value_size (ebpf_map.c:77-84 -> ebpf_map_array.c:115-124)."""
    k, vs = v(H[0]), v(H[1])
    return ["v_add_u32 %s, s14, v%d" % (k, V_STK),
            "ds_read_b32 %s, %s" % (k, k),
            "v_mov_b32 %s, s15" % vs,
            "s_waitcnt lgkmcnt(0)",
            "v_cmp_gt_u32_e64 vcc, s13, %s" % k,
            "v_mad_u64_u32 %s, %s, %s, %s, s[10:11]" % (vp(H[2]), sp(S_JUNK), k, vs),
            "v_cndmask_b32 v0, 0, %s, vcc" % v(H[2]),
            "v_cndmask_b32 v1, 0, %s, vcc" % v(H[3])]


def _hl_word(dst, off, n):
    """dst = the little-endian key word at byte offset s[off] of the key at H[0:1], bytes at or
    past the key size (S_T0) read as 0 (jhash's zero-padded tail; the device table stores keys
    zero-padded the same way).  Clobbers R[8:10], H[3:5], S_BYTES, vcc."""
    t = [v(R[10]), v(H[3]), v(H[4]), v(H[5])]
    out = ["v_add_co_u32 %s, vcc, %s, %s" % (v(R[8]), s(off), v(H[0])),
           "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(R[9]), v(H[1]))]
    for j in range(4):
        out += ["s_add_u32 %s, %s, %d" % (s(S_BYTES), s(off), j + 1),
                "s_cmp_le_u32 %s, %s" % (s(S_BYTES), s(S_T0)),
                "s_cbranch_scc0 .Lhw_z%s_%d" % (n, j),
                "flat_load_ubyte %s, %s offset:%d" % (t[j], vp(R[8]), j),
                "s_branch .Lhw_d%s_%d" % (n, j),
                ".Lhw_z%s_%d:" % (n, j),
                "v_mov_b32 %s, 0" % t[j],
                ".Lhw_d%s_%d:" % (n, j)]
    out += ["s_waitcnt vmcnt(0) lgkmcnt(0)",
            "v_lshl_or_b32 %s, %s, 8, %s" % (dst, t[1], t[0]),
            "v_lshl_or_b32 %s, %s, 16, %s" % (dst, t[2], dst),
            "v_lshl_or_b32 %s, %s, 24, %s" % (dst, t[3], dst)]
    return out


def _rot(d, x, k):
    """d = rotl32(x, k)"""
    return ["v_alignbit_b32 %s, %s, %s, %d" % (d, x, x, 32 - k)]


def probe_wait(tag):
    """Wait for the hashtable probe load just issued."""
    return ["s_waitcnt vmcnt(0)"]


def hlookup_routine():
    """HLOOKUP (called): r0 = hashtable_map_lookup_elem(map, r2) for the map whose dp_map record
    is at byte offset s14 of the map table (ebpf_map.c:77-84 -> ebpf_map_hashtable.c:285-301).
    The key (key_size bytes at r2, anywhere a program may read) is region-checked like a load,
    hashed with jhash (ebpf_jhash.h hashlittle, initval 0) and probed linearly in the device
    table (dprog.h dp_map): a lane stops at its key (r0 = the slot's value) or at an empty slot
    (r0 = NULL).  r2 == 0 gives NULL with no access, as the reference's NULL-key check.
    Uses s[8:9] (return address), s[10:11] (entry exec), R[*], H[*]; compiled programs treat
    s10..s11 as clobbered after it."""
    L = [".Lr_hlookup:",
         "s_mov_b64 s[8:9], %s" % sp(S_LINK),
         "s_mov_b64 s[10:11], exec",
         "v_mov_b32 v0, 0", "v_mov_b32 v1, 0",
         "v_cmp_ne_u64_e64 vcc, 0, v[4:5]",
         "s_and_b64 exec, exec, vcc",              # NULL keys: r0 = NULL, nothing read
         "s_cbranch_execz .Lhl_ret"] + hprobe_body("") + [
         ".Lhl_ret:",
         # every lane that entered and did not fault (S_ALIVE lost the faulted ones)
         "s_and_b64 exec, s[10:11], %s" % sp(S_ALIVE),
         "s_setpc_b64 s[8:9]"]
    return L


def hprobe_body(tag):
    """The probe of HLOOKUP (shared with the hashtable path of UPDATE, whose labels carry `tag`):
    for the lanes in exec, v[0:1] = the value address of the key at r2 in the map at s14, or
    NULL; lanes whose key is not readable fault MEM.  Ends at .Lhl_ret<tag> (defined by the
    caller) with exec arbitrary.  Uses R[*], H[*], S_T*, S_OK, S_JUNK, s[64:71]."""
    a, b, c = v(R[0]), v(R[1]), v(R[2])
    t = v(R[3])
    T = tag
    L = ["s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
         "s_waitcnt lgkmcnt(0)",
         "s_and_b32 %s, s71, 0xffff" % s(S_T0),    # key size
         "s_mov_b32 %s, 0" % s(S_T1),
         "v_mov_b32 %s, v4" % v(H[0]), "v_mov_b32 %s, v5" % v(H[1])] + call(".Lr_check") + [
         # exec = the lanes whose key is readable (the others retired with a fault); a
         # structured compiled program may come back with none
         "s_cbranch_execz .Lhl_ret%s" % T,
         "s_mov_b64 %s, exec" % sp(S_MASK),
         "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
         "s_waitcnt lgkmcnt(0)",
         "s_and_b32 %s, s71, 0xffff" % s(S_T0),             # key size
         "s_bfe_u32 %s, s71, 0x50010" % s(S_T1),            # log2 slot stride (5 bits at 16)
         "s_sub_u32 s69, s69, 1",                            # slot mask
         "s_add_u32 s70, %s, 15" % s(S_T0),
         "s_and_b32 s70, s70, -8",                           # value offset 8 + round8(key size)
         # jhash: a = b = c = 0xdeadbeef + length (+ initval 0)
         "s_add_u32 %s, %s, 0xdeadbeef" % (s(S_JUNK), s(S_T0)),
         "v_mov_b32 %s, %s" % (a, s(S_JUNK)), "v_mov_b32 %s, %s" % (b, s(S_JUNK)),
         "v_mov_b32 %s, %s" % (c, s(S_JUNK)),
         "s_mov_b32 %s, 0" % s(S_T2),                       # byte offset
         "s_mov_b32 %s, %s" % (s(S_T3), s(S_T0)),           # bytes left
         ".Lhh_loop%s:" % T,
         "s_cmp_le_u32 %s, 12" % s(S_T3),
         "s_cbranch_scc1 .Lhh_tail%s" % T]
    n = [0]

    def add_words(keep=False):
        out = []
        for i, x in enumerate((a, b, c)):
            out += _hl_word(t, S_T2, "%s%d" % (T, n[0]))
            n[0] += 1
            out += ["v_add_u32 %s, %s, %s" % (x, x, t), "s_add_u32 %s, %s, 4" % (s(S_T2), s(S_T2))]
            if keep and i < 2:   # keys of <= 8 bytes: the tail's first two words are the key
                out.append("v_mov_b32 %s, %s" % (v(H[2]) if i == 0 else v(R[5]), t))
        return out
    L += add_words()
    for (x, y, z, k) in ((a, c, b, 4), (b, a, c, 6), (c, b, a, 8), (a, c, b, 16), (b, a, c, 19),
                         (c, b, a, 4)):
        # x -= y; x ^= rot(y, k); y += z
        L += ["v_sub_u32 %s, %s, %s" % (x, x, y)] + _rot(t, y, k) + \
             ["v_xor_b32 %s, %s, %s" % (x, x, t), "v_add_u32 %s, %s, %s" % (y, y, z)]
    L += ["s_sub_u32 %s, %s, 12" % (s(S_T3), s(S_T3)),
          "s_branch .Lhh_loop%s" % T,
          ".Lhh_tail%s:" % T]
    L += add_words(keep=True)
    for (x, y, k) in ((c, b, 14), (a, c, 11), (b, a, 25), (c, b, 16), (a, c, 4), (b, a, 14), (c, b, 24)):
        # x ^= y; x -= rot(y, k)
        L += ["v_xor_b32 %s, %s, %s" % (x, x, y)] + _rot(t, y, k) + ["v_sub_u32 %s, %s, %s" % (x, x, t)]
    # probe: slot i = hash & mask, then i + 1, ... until the key or an empty slot
    idx, sa, hd = v(R[3]), vp(R[4]), vp(R[6])
    # keys of up to 8 bytes: one 16-byte load per slot (used, hash, key) compared in registers
    k0, k1 = v(H[2]), v(H[3])
    L += ["s_cmp_le_u32 %s, 8" % s(S_T0),
          "s_cbranch_scc0 .Lhp_general%s" % T,
          "v_mov_b32 %s, %s" % (k1, v(R[5])),
          "v_and_b32 %s, s69, %s" % (idx, c),
          "s_mov_b64 %s, exec" % sp(S_OK),
          ".Lhq_loop%s:" % T,
          "v_mov_b32 %s, %s" % (v(R[4]), idx),
          "v_mov_b32 %s, 0" % v(R[5]),
          "v_lshlrev_b64 %s, %s, %s" % (sa, s(S_T1), sa),
          "v_lshl_add_u64 %s, %s, 0, s[66:67]" % (sa, sa),
          "global_load_dwordx4 v[%d:%d], %s, off%s" % (R[6], R[9], sa, PROBE_POLICY),
          # the slot's first 8 value bytes (value offset 16 for keys of <= 8 bytes), same line:
          # lanes that meet their key here keep them in v[50:51] for the code generator's
          # forwarded value loads (asm_cc.cpp AHF_LDXHV)
          "global_load_dwordx2 %s, %s, off offset:16%s" % (vp(H[4]), sa, PROBE_POLICY)] + probe_wait("hq" + T) + [
          "v_cmp_eq_u32_e64 vcc, 0, %s" % v(R[6]),           # empty slot: not found
          "s_andn2_b64 %s, %s, vcc" % (sp(S_OK), sp(S_OK)),
          "v_cmp_eq_u32_e64 %s, %s, %s" % (sp(S_JUNK), v(R[7]), c),
          "v_cmp_eq_u32_e64 vcc, %s, %s" % (v(R[8]), k0),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "v_cmp_eq_u32_e64 vcc, %s, %s" % (v(R[9]), k1),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_and_b64 exec, %s, %s" % (sp(S_JUNK), sp(S_OK)),  # found here
          "v_add_co_u32 v0, vcc, s70, %s" % v(R[4]),
          "v_addc_co_u32 v1, vcc, 0, %s, vcc" % v(R[5]),
          "s_andn2_b64 %s, %s, exec" % (sp(S_OK), sp(S_OK)),
          "s_mov_b64 exec, %s" % sp(S_OK),
          "s_cbranch_execz .Lhl_ret%s" % T,
          "v_add_u32 %s, 1, %s" % (idx, idx),
          "v_and_b32 %s, s69, %s" % (idx, idx),
          "s_branch .Lhq_loop%s" % T,
          ".Lhp_general%s:" % T]
    L += ["v_and_b32 %s, s69, %s" % (idx, c),
          "s_mov_b64 %s, exec" % sp(S_OK),                  # lanes still probing
          ".Lhp_loop%s:" % T,
          "v_mov_b32 %s, %s" % (v(R[4]), idx),
          "v_mov_b32 %s, 0" % v(R[5]),
          "v_lshlrev_b64 %s, %s, %s" % (sa, s(S_T1), sa),
          "v_lshl_add_u64 %s, %s, 0, s[66:67]" % (sa, sa),
          "global_load_dwordx2 %s, %s, off" % (hd, sa)] + probe_wait("hp" + T) + [
          "v_cmp_eq_u32_e64 vcc, 0, %s" % v(R[6]),          # empty slot: not found
          "s_andn2_b64 %s, %s, vcc" % (sp(S_OK), sp(S_OK)),
          "s_and_b64 exec, exec, %s" % sp(S_OK),
          "v_cmp_eq_u32_e64 vcc, %s, %s" % (v(R[7]), c),    # stored hash matches: compare keys
          "s_and_b64 exec, exec, vcc",
          "s_cbranch_execz .Lhp_next%s" % T,
          "s_mov_b32 %s, 0" % s(S_T2),
          ".Lhc_loop%s:" % T,
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_T0)),
          "s_cbranch_scc1 .Lhc_found%s" % T] + _hl_word(v(R[6]), S_T2, T + "99") + [
          "v_add_co_u32 %s, vcc, %s, %s" % (v(R[8]), s(S_T2), v(R[4])),
          "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(R[9]), v(R[5])),
          "global_load_dword %s, %s, off offset:8" % (v(R[7]), vp(R[8])),
          "s_waitcnt vmcnt(0)",
          "v_cmp_ne_u32_e64 vcc, %s, %s" % (v(R[6]), v(R[7])),
          "s_andn2_b64 exec, exec, vcc",
          "s_cbranch_execz .Lhp_next%s" % T,
          "s_add_u32 %s, %s, 4" % (s(S_T2), s(S_T2)),
          "s_branch .Lhc_loop%s" % T,
          ".Lhc_found%s:" % T,
          "v_add_co_u32 v0, vcc, s70, %s" % v(R[4]),
          "v_addc_co_u32 v1, vcc, 0, %s, vcc" % v(R[5]),
          "s_andn2_b64 %s, %s, exec" % (sp(S_OK), sp(S_OK)),
          ".Lhp_next%s:" % T,
          "s_mov_b64 exec, %s" % sp(S_OK),
          "s_cbranch_execz .Lhl_ret%s" % T,
          "v_add_u32 %s, 1, %s" % (idx, idx),
          "v_and_b32 %s, s69, %s" % (idx, idx),
          "s_branch .Lhp_loop%s" % T]
    return L


def log_record(T, word, ret):
    """For the lanes in exec: a slot in the launch's write log (one atomic add on its counter per
    wave), R[4:5] = the record's address (log + 64 + slot * stride), its first 16 bytes written:
    {u64 packet index, u32 entry | map << 20, u32 `word`}.  With dp_launch.vflags bit 4
    (DP_VF_WCAP) every lane first counts the write in its stack slice (DP_WCOUNT): a packet's
    write past WRITES_MAX faults it EBPF_FAULT_WRITES instead.  A full log (the host sizes it for
    the program's most writes per path: a library bug) faults MEM, loudly, rather than lose a
    write; exec empty after that branches to `ret`.  Uses R[0:7], S_T0..2, S_MASK, S_JUNK,
    s[64:69]."""
    return [
        "s_load_dword %s, s[0:1], 0x%x" % (s(S_T0), VFLAGS_OFF),
        "s_waitcnt lgkmcnt(0)",
        "s_bitcmp1_b32 %s, 4" % s(S_T0),
        "s_cbranch_scc0 .Lwc_ok%s" % T,
        "v_add_u32 %s, %d, v%d" % (v(R[0]), WCOUNT, V_STK),
        "v_mov_b32 %s, 1" % v(R[1]),
        "ds_add_rtn_u32 %s, %s, %s" % (v(R[2]), v(R[0]), v(R[1])),
        "s_waitcnt lgkmcnt(0)",
        "v_cmp_le_u32_e64 %s, %d, %s" % (sp(S_MASK), WRITES_MAX, v(R[2])),
        "s_and_b64 %s, %s, exec" % (sp(S_MASK), sp(S_MASK)),
        "s_cbranch_scc0 .Lwc_ok%s" % T,
        "s_mov_b32 %s, %d" % (s(S_CODE), FAULT_WRITES)] + call(".Lr_fault") + [
        "s_cbranch_execz %s" % ret,
        ".Lwc_ok%s:" % T,
        # a log slot per lane: one atomic add on the log's counter for the wave
        "s_load_dwordx4 s[64:67], s[0:1], 0x80",         # upd_log, upd_cap, upd_stride
        "s_load_dwordx2 s[68:69], s[0:1], 0x90",         # pkt_base
        "s_waitcnt lgkmcnt(0)",
        "s_bcnt1_i32_b64 %s, exec" % s(S_T0),
        "v_mbcnt_lo_u32_b32 %s, exec_lo, 0" % v(R[0]),
        "v_mbcnt_hi_u32_b32 %s, exec_hi, %s" % (v(R[0]), v(R[0])),
        "s_mov_b64 %s, exec" % sp(S_MASK),
        "s_ff1_i32_b64 %s, exec" % s(S_T1),
        "s_lshl_b64 exec, 1, %s" % s(S_T1),
        "v_mov_b32 %s, %s" % (v(R[1]), s(S_T0)),
        "v_mov_b32 %s, 0" % v(R[2]),
        "global_atomic_add %s, %s, %s, s[64:65] sc0" % (v(R[3]), v(R[2]), v(R[1])),
        "s_waitcnt vmcnt(0)",
        "v_readfirstlane_b32 %s, %s" % (s(S_T2), v(R[3])),
        "s_mov_b64 exec, %s" % sp(S_MASK),
        "v_add_u32 %s, %s, %s" % (v(R[0]), s(S_T2), v(R[0])),      # this lane's slot
        # (the host sizes the log for the program's most updates per path; a full log is a
        # library bug: MEM fault, loudly, rather than a lost write)
        "v_cmp_gt_u32_e64 vcc, s66, %s" % v(R[0]),
        "s_andn2_b64 %s, exec, vcc" % sp(S_MASK),
        "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
        "s_cbranch_scc1 .Lup_room%s" % T,
        "s_mov_b32 %s, 3" % s(S_CODE)] + call(".Lr_fault") + [
        "s_cbranch_execz %s" % ret,
        "s_load_dwordx4 s[64:67], s[0:1], 0x80",
        "s_load_dwordx2 s[68:69], s[0:1], 0x90",
        "s_waitcnt lgkmcnt(0)",
        ".Lup_room%s:" % T,
        # the record: log + 64 + slot * stride
        "s_add_u32 s64, s64, 64",
        "s_addc_u32 s65, s65, 0",
        "v_mov_b32 %s, s67" % v(R[1]),
        "v_mad_u64_u32 %s, %s, %s, %s, s[64:65]" % (vp(R[4]), sp(S_JUNK), v(R[0]), v(R[1])),
        # packet index (pkt_base = this launch's first packet in its batch)
    ] + lane_pkt_index(R[2]) + [
        "v_mov_b32 %s, s69" % v(R[3]),
        "v_add_co_u32 %s, vcc, s68, %s" % (v(R[2]), v(R[2])),
        "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(R[3]), v(R[3])),
        "global_store_dwordx2 %s, %s, off" % (vp(R[4]), vp(R[2])),
        "s_lshr_b32 %s, s14, 5" % s(S_T0),                  # map index
        "s_lshl_b32 %s, %s, 20" % (s(S_T0), s(S_T0)),
        "s_or_b32 %s, %s, s15" % (s(S_T0), s(S_T0)),        # | entry index
        "v_mov_b32 %s, %s" % (v(R[6]), s(S_T0)),
        "v_mov_b32 %s, %s" % (v(R[7]), word),
        "global_store_dwordx2 %s, %s, off offset:8" % (vp(R[4]), vp(R[6]))]


def copy_record(T, src, n, off):
    """Bytes [0, s[n]) at the flat address v[src:src+1] into the record at R[4:5] + s[off]
    (byte by byte: the source may be the stack, the packet or a map value).  Uses S_T0, S_T1,
    H[0], H[1], H[3:5], vcc."""
    return ["s_mov_b32 %s, 0" % s(S_T0),
            ".Lcp%s:" % T,
            "s_cmp_ge_u32 %s, %s" % (s(S_T0), s(n)),
            "s_cbranch_scc1 .Lcpe%s" % T,
            "v_add_co_u32 %s, vcc, %s, v%d" % (v(H[0]), s(S_T0), src),
            "v_addc_co_u32 %s, vcc, 0, v%d, vcc" % (v(H[1]), src + 1),
            "flat_load_ubyte %s, %s" % (v(H[3]), vp(H[0])),
            "s_add_u32 %s, %s, %s" % (s(S_T1), s(S_T0), s(off)),
            "v_add_co_u32 %s, vcc, %s, %s" % (v(H[4]), s(S_T1), v(R[4])),
            "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(H[5]), v(R[5])),
            "s_waitcnt vmcnt(0) lgkmcnt(0)",
            "global_store_byte %s, %s, off" % (vp(H[4]), v(H[3])),
            "s_add_u32 %s, %s, 1" % (s(S_T0), s(S_T0)),
            "s_branch .Lcp%s" % T,
            ".Lcpe%s:" % T]


def ovl_fix(T, acc):
    """The packet's own stores into map values over the z = S_T0 bytes just read at H[0:1] into
    acc (two VGPRs): every byte whose 8-byte word has an overlay entry (dprog.h DP_OVL_*) comes
    from that entry.  For the lanes in exec; clobbers R[6:10], H[4], S_T3, S_BYTES, S_MASK, vcc."""
    E, D0, D1, X, Y, C = R[10], R[6], R[7], R[8], R[9], H[4]   # (pairs start even: gfx950)
    L = ["v_add_u32 %s, %d, v%d" % (v(C), OVL_COUNT, V_STK),
         "ds_read_b32 %s, %s" % (v(C), v(C)),
         "s_mov_b32 %s, 0" % s(S_T3),
         ".Lof%s_loop:" % T,
         "s_waitcnt lgkmcnt(0)",
         "v_cmp_lt_u32_e64 vcc, %s, %s" % (s(S_T3), v(C)),
         "s_and_b64 vcc, vcc, exec",
         "s_cbranch_scc0 .Lof%s_done" % T,
         "s_mov_b64 %s, exec" % sp(S_MASK),
         "s_mov_b64 exec, vcc",
         "s_lshl_b32 %s, %s, 4" % (s(S_BYTES), s(S_T3)),
         "s_add_u32 %s, %s, %d" % (s(S_BYTES), s(S_BYTES), OVL_ENTRIES),
         "v_add_u32 %s, %s, v%d" % (v(E), s(S_BYTES), V_STK),
         "ds_read2_b32 %s, %s offset1:1" % (vp(D0), v(E)),          # the entry's word address
         "v_and_b32 %s, -8, %s" % (v(X), v(H[0])),
         "s_waitcnt lgkmcnt(0)",
         # d = entry word - (address & ~7): 0 or 8 when it is a word of this load
         "v_sub_co_u32 %s, vcc, %s, %s" % (v(D0), v(D0), v(X)),
         "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(D1), v(D1), v(H[1])),
         "v_cmp_ne_u32_e64 vcc, 0, %s" % v(D1),
         "v_cndmask_b32_e64 %s, %s, 16, vcc" % (v(D0), v(D0))]
    for b in range(8):
        if b in (1, 2, 4):
            L += ["s_cmp_le_u32 %s, %d" % (s(S_T0), b), "s_cbranch_scc1 .Lof%s_next" % T]
        k = 8 * (b % 4)
        a = v(acc[b // 4])
        L += ["v_and_b32 %s, 7, %s" % (v(X), v(H[0])),
              "v_add_u32 %s, %d, %s" % (v(X), b, v(X)),               # j = (a & 7) + b
              "v_and_b32 %s, 8, %s" % (v(Y), v(X)),                   # 8 * (j >> 3)
              "v_cmp_eq_u32_e64 vcc, %s, %s" % (v(Y), v(D0)),
              "v_and_b32 %s, 7, %s" % (v(X), v(X)),
              "v_add3_u32 %s, %s, %s, 8" % (v(X), v(X), v(E)),
              "ds_read_u8 %s, %s" % (v(Y), v(X)),
              "s_waitcnt lgkmcnt(0)",
              "v_lshlrev_b32 %s, %d, %s" % (v(Y), k, v(Y)),
              "v_and_b32 %s, 0x%x, %s" % (v(X), 0xffffffff ^ (0xff << k), a),
              "v_or_b32 %s, %s, %s" % (v(X), v(X), v(Y)),
              "v_cndmask_b32 %s, %s, %s, vcc" % (a, a, v(X))]
    L += [".Lof%s_next:" % T,
          "s_mov_b64 exec, %s" % sp(S_MASK),
          "s_add_u32 %s, %s, 1" % (s(S_T3), s(S_T3)),
          "s_branch .Lof%s_loop" % T,
          ".Lof%s_done:" % T]
    return L


def ovl_store(T, nv):
    """Remember, in the lanes' overlays, the z = S_T0 bytes of nv (two VGPRs) stored at H[0:1]:
    for each of the (one or two) 8-byte words the store touches, its entry — made on first use
    with the word's batch-start bytes from the mirror — gets the bytes.  A lane whose overlay is
    full (its entries = dp_launch.vflags bits 8..15; only a program with loops that reads its
    counters back fills it, ebpf_gpu.h) when the store needs a new entry gets OVF = 1 and
    stores nothing more.  For the lanes in exec; clobbers R[0:3], R[8:10], H[2:4], S_T3,
    S_BYTES, S_MASK, S_JUNK (saved exec), vcc."""
    W0, W1, CNT, IDX, E, X, Y, OVF = R[0], R[1], R[2], R[3], R[8], H[2], H[3], R[9]
    L = ["s_mov_b64 %s, exec" % sp(S_JUNK),
         "v_mov_b32 %s, 0" % v(OVF),
         "v_add_u32 %s, %d, v%d" % (v(X), OVL_COUNT, V_STK),
         "ds_read_b32 %s, %s" % (v(CNT), v(X)),
         "s_waitcnt lgkmcnt(0)"]
    for wi in (0, 1):
        t = "%s%d" % (T, wi)
        L += ["s_mov_b64 exec, %s" % sp(S_JUNK),
              "v_cmp_eq_u32_e64 vcc, 0, %s" % v(OVF),       # (not the lanes already full)
              "s_and_b64 exec, exec, vcc",
              "s_cbranch_execz .Los%s_end" % t]
        if wi:  # only lanes whose store reaches past its first word
            L += ["v_and_b32 %s, 7, %s" % (v(X), v(H[0])),
                  "v_add_u32 %s, %s, %s" % (v(X), s(S_T0), v(X)),
                  "v_cmp_lt_u32_e64 vcc, 8, %s" % v(X),
                  "s_and_b64 exec, exec, vcc",
                  "s_cbranch_execz .Los%s_end" % t]
        L += ["v_and_b32 %s, -8, %s" % (v(W0), v(H[0])),
              "v_mov_b32 %s, %s" % (v(W1), v(H[1]))]
        if wi:
            L += ["v_add_co_u32 %s, vcc, 8, %s" % (v(W0), v(W0)),
                  "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(W1), v(W1))]
        # the word's entry (IDX), if any
        L += ["v_mov_b32 %s, -1" % v(IDX),
              "s_mov_b32 %s, 0" % s(S_T3),
              ".Los%s_find:" % t,
              "v_cmp_lt_u32_e64 vcc, %s, %s" % (s(S_T3), v(CNT)),
              "s_and_b64 vcc, vcc, exec",
              "s_cbranch_scc0 .Los%s_found" % t,
              "s_mov_b64 %s, exec" % sp(S_MASK),
              "s_mov_b64 exec, vcc",
              "s_lshl_b32 %s, %s, 4" % (s(S_BYTES), s(S_T3)),
              "s_add_u32 %s, %s, %d" % (s(S_BYTES), s(S_BYTES), OVL_ENTRIES),
              "v_add_u32 %s, %s, v%d" % (v(E), s(S_BYTES), V_STK),
              "ds_read2_b32 %s, %s offset1:1" % (vp(X), v(E)),
              "v_mov_b32 %s, %s" % (v(E), s(S_T3)),
              "s_waitcnt lgkmcnt(0)",
              "v_cmp_eq_u64_e64 vcc, %s, %s" % (vp(X), vp(W0)),
              "v_cndmask_b32 %s, %s, %s, vcc" % (v(IDX), v(IDX), v(E)),
              "s_mov_b64 exec, %s" % sp(S_MASK),
              "s_add_u32 %s, %s, 1" % (s(S_T3), s(S_T3)),
              "s_branch .Los%s_find" % t,
              ".Los%s_found:" % t,
              # none: a new entry with the word's batch-start bytes (a full overlay: OVF)
              "v_cmp_eq_u32_e64 vcc, -1, %s" % v(IDX),
              "s_and_saveexec_b64 %s, vcc" % sp(S_MASK),
              "s_cbranch_execz .Los%s_have" % t,
              "s_load_dword %s, s[0:1], 0x%x" % (s(S_T3), VFLAGS_OFF),
              "s_waitcnt lgkmcnt(0)",
              "s_bfe_u32 %s, %s, 0x80008" % (s(S_T3), s(S_T3)),
              "v_cmp_le_u32_e64 vcc, %s, %s" % (s(S_T3), v(CNT)),
              "v_cndmask_b32_e64 %s, %s, 1, vcc" % (v(OVF), v(OVF)),
              "s_andn2_b64 exec, exec, vcc",
              "s_cbranch_execz .Los%s_have" % t,
              "v_mov_b32 %s, %s" % (v(IDX), v(CNT)),
              "v_add_u32 %s, 1, %s" % (v(CNT), v(CNT)),
              "v_lshl_add_u32 %s, %s, 4, v%d" % (v(E), v(IDX), V_STK),
              "v_add_u32 %s, %d, %s" % (v(E), OVL_ENTRIES, v(E)),
              "global_load_dwordx2 %s, %s, off" % (vp(X), vp(W0)),
              "ds_write2_b32 %s, %s, %s offset1:1" % (v(E), v(W0), v(W1)),
              "s_waitcnt vmcnt(0)",
              "ds_write2_b32 %s, %s, %s offset0:2 offset1:3" % (v(E), v(X), v(Y)),
              "v_add_u32 %s, %d, v%d" % (v(X), OVL_COUNT, V_STK),
              "ds_write_b32 %s, %s" % (v(X), v(CNT)),
              ".Los%s_have:" % t,
              "s_or_b64 exec, exec, %s" % sp(S_MASK),
              "v_cmp_eq_u32_e64 vcc, 0, %s" % v(OVF),
              "s_and_b64 exec, exec, vcc",
              "s_cbranch_execz .Los%s_end" % t,
              "v_lshl_add_u32 %s, %s, 4, v%d" % (v(E), v(IDX), V_STK),
              "v_add_u32 %s, %d, %s" % (v(E), OVL_ENTRIES + 8, v(E))]   # the entry's bytes
        # the bytes of the store that fall in this word
        for b in range(8):
            if b in (1, 2, 4):
                L += ["s_cmp_le_u32 %s, %d" % (s(S_T0), b), "s_cbranch_scc1 .Los%s_end" % t]
            L += ["v_and_b32 %s, 7, %s" % (v(X), v(H[0])),
                  "v_add_u32 %s, %d, %s" % (v(X), b, v(X)),          # j = (a & 7) + b
                  "v_and_b32 %s, 8, %s" % (v(Y), v(X)),
                  "v_cmp_eq_u32_e64 vcc, %d, %s" % (8 * wi, v(Y)),
                  "s_and_saveexec_b64 %s, vcc" % sp(S_MASK),
                  "v_and_b32 %s, 7, %s" % (v(X), v(X)),
                  "v_add_u32 %s, %s, %s" % (v(X), v(X), v(E)),
                  "v_lshrrev_b32 %s, %d, %s" % (v(Y), 8 * (b % 4), v(nv[b // 4])),
                  "ds_write_b8 %s, %s" % (v(X), v(Y)),
                  "s_or_b64 exec, exec, %s" % sp(S_MASK)]
        L += [".Los%s_end:" % t]
    L += ["s_mov_b64 exec, %s" % sp(S_JUNK),
          "s_waitcnt lgkmcnt(0)"]
    return L


def vstore_routine():
    """VSTORE (called by .Lr_check for the lanes of one map, exec = those lanes): a store into
    that map's values (ebpf_gpu.h "Stores into map values"), S_T1 = kind (1 a plain store of
    H[2:3]; 2 a counter update's STX of H[2:3]; 3 XADD of the addend H[2:3]), S_T0 = bytes,
    H[0:1] = the address, S_T2 = the map's index, s[64:71] its dp_map record.
      * kinds 2 and 3 read the value the packet sees there (L: the mirror's bytes under its
        overlay); kind 3 leaves L in the lane's scratch (the handler's own read-modify-write,
        pointed there, then fetches it); kind 2 adds X - L, kind 3 the addend;
      * the overlay (dp_launch.vflags bit 0) remembers the stored value;
      * an addition aligned to its width within the values of a DP_MAP_ATOMIC map goes into its
        delta area (a device atomic); everything else is a record in the batch's log
        {packet, map << 20 | DP_REC_VALUE | add << 16 | size, offset, data, hashtable slot}.
    Returns S_JUNK = the lanes to fault (code S_CODE): the log full, or value stores not provided
    for (vflags bit 1 clear: the translator saw none).  Preserves S_T0..S_T2 and v51 (SPILL);
    clobbers R[*], H[2:4], S_T3, S_BYTES, S_MASK, s[64:71], vcc."""
    L_, NV, OFF, VOFF, SLOT, WORD, ADD = (R[4], R[5]), (R[6], R[7]), R[0], R[2], R[3], R[8], R[10]
    L = [".Lr_vstore:",
         "v_writelane_b32 v%d, %s, 11" % (SPILL, s(S_LINK)),
         "v_writelane_b32 v%d, %s, 12" % (SPILL, s(S_LINK + 1)),
         "s_mov_b64 %s, 0" % sp(S_JUNK),
         "s_load_dword %s, s[0:1], 0x%x" % (s(S_T3), VFLAGS_OFF),
         "s_waitcnt lgkmcnt(0)",
         "s_bitcmp1_b32 %s, 1" % s(S_T3),
         "s_cbranch_scc1 .Lvs_go",
         "s_mov_b64 %s, exec" % sp(S_JUNK),
         "s_mov_b32 %s, 9" % s(S_CODE),          # EBPF_FAULT_MAP_WRITE
         "s_branch .Lvs_ret",
         ".Lvs_go:",
         "s_cmp_eq_u32 %s, 1" % s(S_T1),
         "s_cbranch_scc1 .Lvs_plain"] + gather(H[0], L_, H[4], None, "vs") + \
        vflags_test(0, ".Lvs_noovl") + ovl_fix("vs", L_) + [
         ".Lvs_noovl:",
         "s_cmp_eq_u32 %s, 3" % s(S_T1),
         "s_cbranch_scc0 .Lvs_cnt",
         # XADD: new = L + addend, L to the scratch, delta = the addend
         "v_lshl_add_u64 %s, %s, 0, %s" % (vp(NV[0]), vp(L_[0]), vp(H[2])),
         "v_add_u32 %s, %d, v%d" % (v(R[9]), VST_SCRATCH, V_STK),
         "ds_write2_b32 %s, %s, %s offset1:1" % (v(R[9]), v(L_[0]), v(L_[1])),
         "v_mov_b32 %s, %s" % (v(L_[0]), v(H[2])),
         "v_mov_b32 %s, %s" % (v(L_[1]), v(H[3])),
         "s_branch .Lvs_have",
         ".Lvs_cnt:",                             # a counter's STX: delta = X - L
         "v_mov_b32 %s, %s" % (v(NV[0]), v(H[2])),
         "v_mov_b32 %s, %s" % (v(NV[1]), v(H[3])),
         "v_sub_co_u32 %s, vcc, %s, %s" % (v(L_[0]), v(H[2]), v(L_[0])),
         "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(L_[1]), v(H[3]), v(L_[1])),
         "s_branch .Lvs_have",
         ".Lvs_plain:",
         "v_mov_b32 %s, %s" % (v(NV[0]), v(H[2])),
         "v_mov_b32 %s, %s" % (v(NV[1]), v(H[3])),
         "v_mov_b32 %s, 0" % v(L_[0]),
         "v_mov_b32 %s, 0" % v(L_[1]),
         ".Lvs_have:"] + vflags_test(0, ".Lvs_noovl2") + ovl_store("vs", NV) + [
         # (ovl_store kept exec there) lanes whose overlay was full fault WRITES, with nothing
         # of this store done
         "v_cmp_ne_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(R[9])),
         "s_andn2_b64 exec, exec, %s" % sp(S_JUNK),
         "s_mov_b32 %s, %d" % (s(S_CODE), FAULT_WRITES),
         "s_cbranch_execz .Lvs_ret",
         "s_branch .Lvs_ovl_done",
         ".Lvs_noovl2:",
         "s_mov_b64 %s, 0" % sp(S_JUNK),
         ".Lvs_ovl_done:",
         # offsets: OFF = address - the mirror (hashtables: SLOT, VOFF = in the value)
         "v_sub_co_u32 %s, vcc, %s, s66" % (v(OFF), v(H[0])),
         "v_mov_b32 %s, s67" % v(R[9]),
         "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[1]), v(H[1]), v(R[9])),
         "v_mov_b32 %s, %s" % (v(VOFF), v(OFF)),
         "v_mov_b32 %s, 0" % v(SLOT),
         "s_bitcmp1_b32 s71, 31",
         "s_cbranch_scc0 .Lvs_arr",
         "s_bfe_u32 %s, s71, 0x50010" % s(S_T3),                    # log2 of the slot stride
         "v_lshrrev_b64 %s, %s, %s" % (vp(R[8]), s(S_T3), vp(OFF)),
         "v_mov_b32 %s, %s" % (v(SLOT), v(R[8])),
         "s_lshl_b32 %s, 1, %s" % (s(S_BYTES), s(S_T3)),
         "s_sub_u32 %s, %s, 1" % (s(S_BYTES), s(S_BYTES)),
         "v_and_b32 %s, %s, %s" % (v(VOFF), s(S_BYTES), v(OFF)),
         "s_and_b32 %s, s71, 0xffff" % s(S_T3),                    # value offset in the slot:
         "s_add_u32 %s, %s, 15" % (s(S_T3), s(S_T3)),               # 8 + round8(key size)
         "s_and_b32 %s, %s, -8" % (s(S_T3), s(S_T3)),
         "v_subrev_u32 %s, %s, %s" % (v(VOFF), s(S_T3), v(VOFF)),
         ".Lvs_arr:",
         # ADD = an addition (kinds 2, 3) aligned to its width within the values
         "s_sub_u32 %s, %s, 1" % (s(S_T3), s(S_T0)),
         "v_and_b32 %s, %s, %s" % (v(ADD), s(S_T3), v(VOFF)),
         "v_cmp_eq_u32_e64 vcc, 0, %s" % v(ADD),
         "s_cmp_eq_u32 %s, 1" % s(S_T1),
         "s_cselect_b64 vcc, 0, vcc",
         "v_cndmask_b32_e64 %s, 0, 1, vcc" % v(ADD),
         # a DP_MAP_ATOMIC map: the additions into its delta area
         "s_bitcmp1_b32 s71, 30",
         "s_cbranch_scc0 .Lvs_rec",
         "s_and_saveexec_b64 %s, vcc" % sp(S_MASK),
         "s_cbranch_execz .Lvs_atom_done",
         # the workgroup's LDS sums (DP_MAP_LDSDELTA: table at s71 & 0xffff)
         "s_bitcmp1_b32 s71, 29",
         "s_cbranch_scc0 .Lvs_atom_g",
         "s_and_b32 %s, s71, 0xffff" % s(S_BYTES),
         "v_add_u32 %s, %s, %s" % (v(R[8]), s(S_BYTES), v(OFF)),
         "s_cmp_eq_u32 %s, 8" % s(S_T0),
         "s_cbranch_scc0 .Lvs_lds4",
         "ds_add_u64 %s, %s" % (v(R[8]), vp(L_[0])),
         "s_branch .Lvs_atom_done",
         ".Lvs_lds4:",
         "ds_add_u32 %s, %s" % (v(R[8]), v(L_[0])),
         "s_branch .Lvs_atom_done",
         ".Lvs_atom_g:",
         "s_mul_i32 %s, s68, s69" % s(S_BYTES),
         "s_add_u32 %s, %s, 63" % (s(S_BYTES), s(S_BYTES)),
         "s_and_b32 %s, %s, -64" % (s(S_BYTES), s(S_BYTES)),      # dprog.h dp_delta_off
         "v_lshl_add_u64 %s, %s, 0, s[66:67]" % (vp(R[8]), vp(OFF)),
         "v_add_co_u32 %s, vcc, %s, %s" % (v(R[8]), s(S_BYTES), v(R[8])),
         "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(R[9]), v(R[9])),
         "s_cmp_eq_u32 %s, 8" % s(S_T0),
         "s_cbranch_scc0 .Lvs_atom4",
         "global_atomic_add_x2 %s, %s, off" % (vp(R[8]), vp(L_[0])),
         "s_branch .Lvs_atom_done",
         ".Lvs_atom4:",
         "global_atomic_add %s, %s, off" % (vp(R[8]), v(L_[0])),
         ".Lvs_atom_done:",
         "s_waitcnt lgkmcnt(0)",
         "s_andn2_b64 exec, %s, exec" % sp(S_MASK),                # the lanes left: records
         ".Lvs_rec:",
         "s_cbranch_execz .Lvs_ret",
         # capped writes (vflags bit 4, DP_VF_WCAP): every record (the lanes here: a DP_MAP_ATOMIC
         # map's additions went to its delta area above) counts in the lane's slice; the one past
         # WRITES_MAX faults
         "s_load_dword %s, s[0:1], 0x%x" % (s(S_T3), VFLAGS_OFF),
         "s_waitcnt lgkmcnt(0)",
         "s_bitcmp1_b32 %s, 4" % s(S_T3),
         "s_cbranch_scc0 .Lvs_wc_ok",
         "s_mov_b64 %s, exec" % sp(S_MASK),
         "v_add_u32 %s, %d, v%d" % (v(R[1]), WCOUNT, V_STK),
         "v_mov_b32 %s, 1" % v(R[9]),
         "ds_add_rtn_u32 %s, %s, %s" % (v(R[9]), v(R[1]), v(R[9])),
         "s_waitcnt lgkmcnt(0)",
         "v_cmp_le_u32_e64 vcc, %d, %s" % (WRITES_MAX, v(R[9])),
         "s_and_b64 vcc, vcc, exec",              # (vcc = the lanes past the cap)
         "s_mov_b64 exec, %s" % sp(S_MASK),
         "s_andn2_b64 exec, exec, vcc",
         "s_or_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
         "s_mov_b32 %s, %d" % (s(S_CODE), FAULT_WRITES),
         "s_cbranch_execz .Lvs_ret",
         ".Lvs_wc_ok:",
         # the record's word and data (an addition: the addend; else the stored bytes)
         "s_lshl_b32 %s, %s, 20" % (s(S_T3), s(S_T2)),
         "s_or_b32 %s, %s, 0x%x" % (s(S_T3), s(S_T3), 0x80000),
         "s_or_b32 %s, %s, %s" % (s(S_T3), s(S_T3), s(S_T0)),
         "v_mov_b32 %s, %s" % (v(WORD), s(S_T3)),
         "v_cmp_ne_u32_e64 vcc, 0, %s" % v(ADD),
         "v_or_b32 %s, 0x%x, %s" % (v(R[9]), 0x10000, v(WORD)),
         "v_cndmask_b32 %s, %s, %s, vcc" % (v(WORD), v(WORD), v(R[9])),
         "v_cndmask_b32 %s, %s, %s, vcc" % (v(L_[0]), v(NV[0]), v(L_[0])),
         "v_cndmask_b32 %s, %s, %s, vcc" % (v(L_[1]), v(NV[1]), v(L_[1])),
         # a log slot per lane: one atomic add on the log's counter for the wave
         "s_load_dwordx4 s[64:67], s[0:1], 0x80",                # upd_log, upd_cap, upd_stride
         "s_load_dwordx2 s[68:69], s[0:1], 0x90",                # pkt_base
         "s_waitcnt lgkmcnt(0)",
         "s_cmp_eq_u64 s[64:65], 0",
         "s_cbranch_scc0 .Lvs_log",
         "s_or_b64 %s, %s, exec" % (sp(S_JUNK), sp(S_JUNK)),       # (no log: a library bug)
         "s_mov_b32 %s, 3" % s(S_CODE),
         "s_branch .Lvs_ret",
         ".Lvs_log:",
         "s_bcnt1_i32_b64 %s, exec" % s(S_T3),
         "v_mbcnt_lo_u32_b32 %s, exec_lo, 0" % v(OFF),
         "v_mbcnt_hi_u32_b32 %s, exec_hi, %s" % (v(OFF), v(OFF)),
         "s_mov_b64 %s, exec" % sp(S_MASK),
         "s_ff1_i32_b64 %s, exec" % s(S_BYTES),
         "s_lshl_b64 exec, 1, %s" % s(S_BYTES),
         "v_mov_b32 %s, %s" % (v(R[1]), s(S_T3)),
         "v_mov_b32 %s, 0" % v(R[9]),
         "global_atomic_add %s, %s, %s, s[64:65] sc0" % (v(R[6]), v(R[9]), v(R[1])),
         "s_waitcnt vmcnt(0)",
         "v_readfirstlane_b32 %s, %s" % (s(S_T3), v(R[6])),
         "s_mov_b64 exec, %s" % sp(S_MASK),
         "v_add_u32 %s, %s, %s" % (v(OFF), s(S_T3), v(OFF)),      # this lane's slot
         # a full log (the host sizes it for the program's records per path: a library bug)
         # faults MEM, loudly, rather than losing a write
         "v_cmp_gt_u32_e64 vcc, s66, %s" % v(OFF),
         "s_andn2_b64 %s, exec, vcc" % sp(S_MASK),
         "s_or_b64 %s, %s, %s" % (sp(S_JUNK), sp(S_JUNK), sp(S_MASK)),
         "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
         "s_cselect_b32 %s, %s, 3" % (s(S_CODE), s(S_CODE)),
         "s_and_b64 exec, exec, vcc",
         "s_cbranch_execz .Lvs_ret",
         # the record: log + 64 + slot * stride
         "s_add_u32 s64, s64, 64",
         "s_addc_u32 s65, s65, 0",
         "v_mov_b32 %s, s67" % v(R[1]),
         "v_mad_u64_u32 %s, vcc, %s, %s, s[64:65]" % (vp(NV[0]), v(OFF), v(R[1]))] + \
        lane_pkt_index(R[0]) + [
         "v_mov_b32 %s, s69" % v(R[1]),
         "v_add_co_u32 %s, vcc, s68, %s" % (v(R[0]), v(R[0])),
         "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(R[1]), v(R[1])),
         "global_store_dwordx2 %s, %s, off" % (vp(NV[0]), vp(R[0])),
         "v_mov_b32 %s, %s" % (v(R[9]), v(VOFF)),
         "global_store_dwordx2 %s, %s, off offset:8" % (vp(NV[0]), vp(WORD)),
         "global_store_dwordx2 %s, %s, off offset:16" % (vp(NV[0]), vp(L_[0])),
         "global_store_dword %s, %s, off offset:24" % (vp(NV[0]), v(SLOT)),
         ".Lvs_ret:",
         "v_readlane_b32 %s, v%d, 11" % (s(S_LINK), SPILL),
         "v_readlane_b32 %s, v%d, 12" % (s(S_LINK + 1), SPILL),
         "s_setpc_b64 %s" % sp(S_LINK)]
    return L


def update_routine():
    """UPDATE (called): r0 = map_update_elem(map, r2, r3, r4) for the map whose dp_map record is
    at byte offset s14 of the map table (ebpf_map.c:101-108 -> ebpf_map_array.c:185-211), with
    the device-batch semantics (ebpf_gpu.h "Map writes in a device batch"): the return code is
    the reference's (EINVAL for a NULL key / value or flags > EBPF_EXIST, EEXIST for
    EBPF_NOEXIST, EINVAL for a key >= max_entries, else 0) and the write itself goes to the
    launch's log (dp_launch.upd_log: {u64 packet, u32 entry | map << 20, u32 key, value}),
    applied after the batch in packet order.  Key and value are region-checked like loads.
    A hashtable (.Lup_hash): the return code against the batch-start table (EEXIST / ENOENT by
    the key's presence, ebpf_map_hashtable.c:87-100; EBUSY for a new key when the table was
    full, :371-377) and, for 0, a record {packet, entry | map << 20, flags << 8, key, value}
    replayed on the host after the batch.  Uses s[8:9] (return address), s[10:11] (entry exec),
    R[*], H[*], v63 (restored); compiled programs treat s10..s11 as clobbered after it."""
    key = v(H[2])
    L = [".Lr_update:",
         "s_mov_b64 s[8:9], %s" % sp(S_LINK),
         "s_mov_b64 s[10:11], exec",
         "v_mov_b32 v0, 22", "v_mov_b32 v1, 0",
         # NULL key / value or flags > EBPF_EXIST: EINVAL, nothing read (ebpf_map.c:101-107)
         "v_cmp_ne_u64_e64 %s, 0, v[4:5]" % sp(S_JUNK),
         "v_cmp_ne_u64_e64 vcc, 0, v[6:7]",
         "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
         "v_cmp_ge_u64_e64 vcc, 2, v[8:9]",
         "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
         "s_and_b64 exec, exec, %s" % sp(S_JUNK),
         "s_cbranch_execz .Lup_ret",
         "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
         "s_waitcnt lgkmcnt(0)",
         "s_bitcmp1_b32 s71, 31",
         "s_cbranch_scc1 .Lup_hash",
         # EBPF_NOEXIST: every key of an array exists -> EEXIST (ebpf_map_array.c:188-189)
         "v_and_b32 %s, 1, v8" % v(R[0]),
         "v_cmp_ne_u32_e64 vcc, 0, %s" % v(R[0]),
         "s_mov_b64 %s, exec" % sp(S_MASK),
         "s_and_b64 exec, exec, vcc",
         "v_mov_b32 v0, 17",
         "s_andn2_b64 exec, %s, vcc" % sp(S_MASK),
         "s_cbranch_execz .Lup_ret",
         # the key: 4 bytes at r2, region-checked like a load
         "v_mov_b32 %s, v4" % v(H[0]), "v_mov_b32 %s, v5" % v(H[1]),
         "s_mov_b32 %s, 4" % s(S_T0), "s_mov_b32 %s, 0" % s(S_T1)] + call(".Lr_check") + [
         "s_cbranch_execz .Lup_ret",
         "v_mov_b32 %s, 0" % key]
    for b in range(4):
        L += ["flat_load_ubyte %s, %s offset:%d" % (v(H[3]), vp(H[0]), b),
              "s_waitcnt vmcnt(0) lgkmcnt(0)",
              "v_lshl_or_b32 %s, %s, %d, %s" % (key, v(H[3]), 8 * b, key)]
    L += ["s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "v_cmp_gt_u32_e64 vcc, s69, %s" % key,          # key >= max_entries: EINVAL
          "s_and_b64 exec, exec, vcc",
          "s_cbranch_execz .Lup_ret",
          # the value: value_size bytes at r3, region-checked
          "v_mov_b32 %s, v6" % v(H[0]), "v_mov_b32 %s, v7" % v(H[1]),
          "s_mov_b32 %s, s68" % s(S_T0), "s_mov_b32 %s, 0" % s(S_T1)] + call(".Lr_check") + [
          "s_cbranch_execz .Lup_ret",
          "v_mov_b32 v0, 0"] + log_record("", key, ".Lup_ret") + [
          # the value, byte by byte (r3 may point at the stack, the packet or a map value)
          "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "s_mov_b32 %s, 0" % s(S_T0),
          ".Lup_copy:",
          "s_cmp_ge_u32 %s, s68" % s(S_T0),
          "s_cbranch_scc1 .Lup_ret",
          "v_add_co_u32 %s, vcc, %s, v6" % (v(H[0]), s(S_T0)),
          "v_addc_co_u32 %s, vcc, 0, v7, vcc" % v(H[1]),
          "flat_load_ubyte %s, %s" % (v(H[3]), vp(H[0])),
          "v_add_co_u32 %s, vcc, %s, %s" % (v(H[4]), s(S_T0), v(R[4])),
          "v_addc_co_u32 %s, vcc, 0, %s, vcc" % (v(H[5]), v(R[5])),
          "s_waitcnt vmcnt(0) lgkmcnt(0)",
          "global_store_byte %s, %s, off offset:16" % (vp(H[4]), v(H[3])),
          "s_add_u32 %s, %s, 1" % (s(S_T0), s(S_T0)),
          "s_branch .Lup_copy"]
    # hashtable: the lanes probing are marked in v63 (the probe leaves no mask register alone)
    L += [".Lup_hash:",
          "s_mov_b64 %s, exec" % sp(S_JUNK),
          "s_mov_b64 exec, s[10:11]",
          "v_mov_b32 v%d, 0" % V_SEL,
          "s_mov_b64 exec, %s" % sp(S_JUNK),
          "v_mov_b32 v%d, 1" % V_SEL,
          "v_mov_b32 v0, 0", "v_mov_b32 v1, 0"] + hprobe_body("U") + [
          ".Lhl_retU:",
          "s_and_b64 exec, s[10:11], %s" % sp(S_ALIVE),
          "v_cmp_eq_u32_e64 vcc, 1, v%d" % V_SEL,
          "s_and_b64 exec, exec, vcc",
          "s_cbranch_execz .Lup_hret",
          "v_cmp_ne_u64_e64 %s, 0, v[0:1]" % sp(S_MASK),         # the key is in the table
          "v_mov_b32 v0, 0", "v_mov_b32 v1, 0",
          "v_and_b32 %s, 1, v8" % v(R[0]),                        # EBPF_NOEXIST: EEXIST
          "v_cmp_ne_u32_e64 vcc, 0, %s" % v(R[0]),
          "s_and_b64 vcc, vcc, %s" % sp(S_MASK),
          "v_cndmask_b32_e64 v0, v0, 17, vcc",
          "v_and_b32 %s, 2, v8" % v(R[0]),                        # EBPF_EXIST: ENOENT
          "v_cmp_ne_u32_e64 vcc, 0, %s" % v(R[0]),
          "s_andn2_b64 vcc, vcc, %s" % sp(S_MASK),
          "v_cndmask_b32_e64 v0, v0, 2, vcc",
          # a new key with the table full (the trailer: live entries, max_entries): EBUSY
          "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "s_bfe_u32 %s, s71, 0x50010" % s(S_T1),
          "s_mov_b32 s64, s69",
          "s_mov_b32 s65, 0",
          "s_lshl_b64 s[64:65], s[64:65], %s" % s(S_T1),
          "s_add_u32 s64, s64, s66",
          "s_addc_u32 s65, s65, s67",
          "s_load_dwordx2 s[64:65], s[64:65], 0x0",
          "s_waitcnt lgkmcnt(0)",
          "s_cmp_lt_u32 s64, s65",
          "s_cbranch_scc1 .Lup_hroom",
          "v_cmp_eq_u32_e64 vcc, 0, v0",
          "s_andn2_b64 vcc, vcc, %s" % sp(S_MASK),
          "v_cndmask_b32_e64 v0, v0, 16, vcc",
          ".Lup_hroom:",
          "v_cmp_eq_u32_e64 vcc, 0, v0",
          "s_and_b64 exec, exec, vcc",
          "s_cbranch_execz .Lup_hret",
          # the value is read only by a call that succeeds (ebpf_map_hashtable.c:380-381)
          "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "v_mov_b32 %s, v6" % v(H[0]), "v_mov_b32 %s, v7" % v(H[1]),
          "s_mov_b32 %s, s68" % s(S_T0), "s_mov_b32 %s, 0" % s(S_T1)] + call(".Lr_check") + [
          "s_cbranch_execz .Lup_hret",
          "v_lshlrev_b32 %s, 8, v8" % v(H[2])] + log_record("h", v(H[2]), ".Lup_hret") + [
          "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "s_and_b32 %s, s71, 0xffff" % s(S_T2),                  # key size
          "s_mov_b32 %s, 16" % s(S_T3)] + copy_record("uk", 4, S_T2, S_T3) + [
          "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
          "s_waitcnt lgkmcnt(0)",
          "s_and_b32 %s, s71, 0xffff" % s(S_T3),
          "s_add_u32 %s, %s, 23" % (s(S_T3), s(S_T3)),
          "s_and_b32 %s, %s, -8" % (s(S_T3), s(S_T3)),            # 16 + round8(key size)
          "s_mov_b32 %s, s68" % s(S_T2)] + copy_record("uv", 6, S_T2, S_T3) + [
          ".Lup_hret:",
          "s_mov_b64 exec, s[10:11]",
          "v_mov_b32 v%d, 0x00010203" % V_SEL,
          ".Lup_ret:",
          # every lane that entered and did not fault (S_ALIVE lost the faulted ones)
          "s_and_b64 exec, s[10:11], %s" % sp(S_ALIVE),
          "s_setpc_b64 s[8:9]"]
    return L


def hdelete_routine():
    """HDELETE (called): r0 = map_delete_elem(map, r2) on the hashtable whose dp_map record is at
    s14 (ebpf_map.c:126-132 -> ebpf_map_hashtable.c:475-502): EINVAL for a NULL key, else 0 with
    the key region-checked (the reference hashes it) and a record {packet, entry | map << 20, 1,
    key} for the host's replay after the batch."""
    return [".Lr_hdelete:",
            "s_mov_b64 s[8:9], %s" % sp(S_LINK),
            "s_mov_b64 s[10:11], exec",
            "v_mov_b32 v0, 22", "v_mov_b32 v1, 0",
            "v_cmp_ne_u64_e64 vcc, 0, v[4:5]",
            "s_and_b64 exec, exec, vcc",
            "s_cbranch_execz .Lhd_ret",
            "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
            "s_waitcnt lgkmcnt(0)",
            "s_and_b32 %s, s71, 0xffff" % s(S_T0),
            "s_mov_b32 %s, 0" % s(S_T1),
            "v_mov_b32 %s, v4" % v(H[0]), "v_mov_b32 %s, v5" % v(H[1])] + call(".Lr_check") + [
            "s_cbranch_execz .Lhd_ret",
            "v_mov_b32 v0, 0",
            "v_mov_b32 %s, 1" % v(H[2])] + log_record("d", v(H[2]), ".Lhd_ret") + [
            "s_load_dwordx8 s[%d:%d], %s, s14" % (S_REC, S_REC + 7, sp(S_MAPS)),
            "s_waitcnt lgkmcnt(0)",
            "s_and_b32 %s, s71, 0xffff" % s(S_T2),
            "s_mov_b32 %s, 16" % s(S_T3)] + copy_record("dk", 4, S_T2, S_T3) + [
            ".Lhd_ret:",
            "s_and_b64 exec, s[10:11], %s" % sp(S_ALIVE),
            "s_setpc_b64 s[8:9]"]


# ---------------------------------------------------------------- handler emission
def handler_body(name, d, sr):
    """Returns (lines, has_dispatch)."""
    if name.startswith("A64R_"):
        return h_alu64r(name[5:], d, sr), False
    if name.startswith("A32R_"):
        return h_alu32r(name[5:], d, sr), False
    if name.startswith("A64I_"):
        return h_alu64i(name[5:], d), False
    if name.startswith("A32I_"):
        return h_alu32i(name[5:], d), False
    if name.startswith("BSWAP"):
        return h_bswap(int(name[5:]), d), False
    for c in CONDS:
        if name == c + "_R":
            return h_cond(c, d, sr, False)
        if name == c + "_I":
            return h_cond(c, d, None, True)
    if name.startswith("LDXPKC"):
        return h_ldx_pkt_const(int(name[6:]), d, sr), False
    if name.startswith("LDXPKBE"):
        return h_ldx_pkt_be(int(name[7:]), d, sr), False
    if name.startswith("LDXPKTG"):
        return h_ldx_pkt_general(int(name[7:]), d), False
    if name.startswith("LDXSTK"):
        return h_ldx_stk(int(name[6:]), d), False
    if name.startswith("STXSTK"):
        return h_stx_stk(int(name[6:]), d), False
    if name.startswith("STSTK"):
        return h_st_stk(int(name[5:])), False
    if name.startswith("LDXGEN"):
        return h_ldx_gen(int(name[6:]), d, sr), False
    if name.startswith("LDXPKTV"):
        return h_ldx_pktv(int(name[7:]), d, sr), False
    if name.startswith("LDXMAP"):
        return h_ldx_map(int(name[6:]), d, sr), False
    if name.startswith("LDXHV"):
        return h_ldx_hv(int(name[5:]), d, sr), False
    if name in ("MOV64R", "NEG64", "NEG32", "ARSH64I", "ARSH64R", "ARSH32I", "ARSH32R",
                "DIV64Z", "MOD64Z", "DIV32Z", "MOD32Z"):
        return h_std(name, d, sr), False
    if name.startswith("J32"):
        c = "J" + name[3:-2]
        return h_cond32(c, d, sr, name.endswith("_I"))
    if name.startswith("STXGEN"):
        return h_stx_gen(int(name[6:]), d, sr), False
    if name.startswith("CNTST"):
        return h_stx_gen(int(name[5:]), d, sr, kind=2), False
    if name.startswith("XADDF"):
        return h_xadd(int(name[5:]), sr, d, True), False
    if name.startswith("XADD"):
        return h_xadd(int(name[4:]), d, sr, False), False
    if name.startswith("STGEN"):
        return h_st_gen(int(name[5:]), d), False
    if name == "EXIT":
        return goto(".Lr_exit"), True
    if name == "FAULT":
        return ["s_mov_b32 %s, s14" % s(S_CODE), "s_mov_b64 %s, exec" % sp(S_MASK)] + \
            call(".Lr_fault") + ["s_endpgm"], True
    if name == "NOP":
        return [], False
    if name == "LOOKUPSTK":
        return h_lookup_stk(), False
    if name == "LOOKUPGEN":
        return goto(".Lr_lookup"), True
    if name == "HLOOKUP":
        return call(".Lr_hlookup"), False
    if name == "UPDATE":
        return call(".Lr_update"), False
    if name == "HDELETE":
        return call(".Lr_hdelete"), False
    if name.startswith("CNTAI"):
        z = int(name[5:])
        out = ["v_mov_b32 %s, s14" % v(H[2]), "v_mov_b32 %s, 0" % v(H[3]),
               "v_lshl_add_u64 %s, %s, 0, %s" % (vp(H[0]), vp(H[2]), pair(d)),
               "v_mov_b32 %s, s10" % v(H[2]), "v_mov_b32 %s, s11" % v(H[3])]
        if z == 8:
            return out + ["global_atomic_add_x2 %s, %s, off" % (vp(H[0]), vp(H[2]))], False
        return out + ["global_atomic_add %s, %s, off" % (vp(H[0]), v(H[2]))], False
    if name.startswith("CNTAL"):
        z = int(name[5:])
        out = ["v_subrev_u32 %s, s15, %s" % (v(H[0]), lo(d)),
               "v_add_u32 %s, s14, %s" % (v(H[0]), v(H[0])),
               "v_mov_b32 %s, s10" % v(H[2]), "v_mov_b32 %s, s11" % v(H[3])]
        if z == 8:
            return out + ["ds_add_u64 %s, %s" % (v(H[0]), vp(H[2]))], False
        return out + ["ds_add_u32 %s, %s" % (v(H[0]), v(H[2]))], False
    if name == "OVLINIT":   # the overlay's count and the logged-write count
        return ["v_mov_b32 %s, 0" % v(H[0]), "v_add_u32 %s, %d, v%d" % (v(H[1]), OVL_COUNT, V_STK),
                "ds_write_b32 %s, %s" % (v(H[1]), v(H[0])),
                "ds_write_b32 %s, %s offset:%d" % (v(H[1]), v(H[0]), WCOUNT - OVL_COUNT)], False
    if name == "LOOPINIT":
        return ["v_mov_b32 %s, 0" % v(H[0]), "ds_write_b32 v%d, %s" % (V_STK, v(H[0]))], False
    if name == "LOOPCNT":
        # count the taken backward jump; lanes past the budget fault LOOP (EBPF_FAULT_LOOP = 8)
        # (one LDS add returning the count before it: past the budget when that is >= budget)
        return ["v_mov_b32 %s, 1" % v(H[0]),
                "ds_add_rtn_u32 %s, v%d, %s" % (v(H[0]), V_STK, v(H[0])),
                "s_waitcnt lgkmcnt(0)",
                "v_cmp_le_u32_e32 vcc, %d, %s" % (LOOP_BUDGET, v(H[0])),
                "s_and_b64 %s, vcc, exec" % sp(S_MASK),
                "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
                "s_cbranch_scc1 .Lok_{uid}"] + fault_mask(S_MASK, 8) + [".Lok_{uid}:"], False
    raise ValueError(name)


# ---------------------------------------------------------------- shared routines
def routines():
    L = []

    # --- schedule: pick the parked group of the first live lane
    L += [".Lr_schedule:",
          "s_mov_b64 exec, %s" % sp(S_ALIVE),
          "s_cbranch_execz .Lgroup_done",
          "s_ff1_i32_b64 %s, exec" % s(S_T0),
          "v_readlane_b32 s6, v%d, %s" % (V_T, s(S_T0)),
          "v_cmp_eq_u32_e64 %s, s6, v%d" % (sp(S_MASK), V_T),
          "s_and_b64 exec, %s, %s" % (sp(S_MASK), sp(S_ALIVE)),
          "s_bitcmp1_b32 s7, 1",
          "s_cbranch_scc1 .Lsched_jit",
          "s_load_dwordx8 s[8:15], s[%d:%d], s6" % (S_PROG, S_PROG + 1),
          "s_waitcnt lgkmcnt(0)",
          "s_setpc_b64 s[8:9]",
          # compiled program: V_T is a code offset from .Lcb
          ".Lsched_jit:",
          "s_add_u32 s8, %s, s6" % s(S_CB),
          "s_addc_u32 s9, %s, 0" % s(S_CB + 1),
          "s_setpc_b64 s[8:9]"]
    # --- diverge: taken lanes (s[mask]) park at the target, the rest continue
    L += [".Lr_diverge:",
          "s_mov_b64 %s, exec" % sp(S_SAVE),
          "s_mov_b64 exec, %s" % sp(S_MASK),
          "v_mov_b32 v%d, s13" % V_T,
          "s_andn2_b64 exec, %s, %s" % (sp(S_SAVE), sp(S_MASK))] + dispatch(12)
    # EXIT: value r0 into V_RET (the group's results are stored together, see group code).
    # (the fault byte of every lane is zeroed when its group starts, and the LDS histogram is
    # kept whether or not the launch asked for one, so an exit does neither check)
    L += [".Lr_exit:"] + ret_slot_write("v0", "v1") + [
          "v_mov_b32 %s, 255" % v(R[8]),
          "v_mov_b32 %s, 0" % v(R[9]),
          "v_cmp_lt_u64_e64 vcc, v[0:1], %s" % vp(R[8]),
          "v_cndmask_b32 %s, %s, v0, vcc" % (v(R[8]), v(R[8])),
          # one LDS atomic per wave when every exiting lane has the same verdict (the usual
          # case); per-lane adds to one address would serialise.  (s_nop: a VALU write, then
          # v_readfirstlane of it, needs one wait state; without it the read can see the
          # previous value and every exit took the per-lane path)
          "s_nop 0",
          "v_readfirstlane_b32 %s, %s" % (s(S_BYTES), v(R[8])),
          "v_cmp_eq_u32_e64 %s, %s, %s" % (sp(S_MASK), s(S_BYTES), v(R[8])),
          "s_cmp_eq_u64 %s, exec" % sp(S_MASK),
          "s_cbranch_scc0 .Lex_lanes",
          # EXIT with r0 known at compile time (compiled programs): v[44:45] = r0 and S_BYTES =
          # its verdict bin are set by the caller, so the verdict needs no per-lane work
          ".Lr_exit_k:",
          ".Lex_uniform:",
          "s_bcnt1_i32_b64 %s, exec" % s(S_CODE),
          "s_lshl_b32 %s, %s, 2" % (s(S_BYTES), s(S_BYTES)),
          "s_mov_b64 %s, exec" % sp(S_SAVE),
          "s_mov_b64 exec, 1",
          "v_mov_b32 %s, %s" % (v(R[8]), s(S_BYTES)),
          "v_mov_b32 %s, %s" % (v(R[9]), s(S_CODE)),
          "ds_add_u32 %s, %s" % (v(R[8]), v(R[9])),
          "s_mov_b64 exec, %s" % sp(S_SAVE),
          "s_branch .Lex_nohist",
          ".Lex_lanes:",
          "v_lshlrev_b32 %s, 2, %s" % (v(R[8]), v(R[8])),
          "v_mov_b32 %s, 1" % v(R[9]),
          "ds_add_u32 %s, %s" % (v(R[8]), v(R[9])),
          ".Lex_nohist:",
          "s_andn2_b64 %s, %s, exec" % (sp(S_ALIVE), sp(S_ALIVE)),
          # structured compiled programs (s7 bit 2) call the exit and continue themselves
          "s_bitcmp1_b32 s7, 2",
          "s_cbranch_scc0 .Lex_sched",
          "s_setpc_b64 %s" % sp(S_LINK),
          ".Lex_sched:"] + goto(".Lr_schedule")
    # FAULT: lanes s[mask], code s[S_CODE]; returns via s[link] unless no lane remains
    L += [".Lr_fault:",
          "s_mov_b64 %s, exec" % sp(S_SAVE),
          "s_mov_b64 exec, %s" % sp(S_MASK),
          ] + ret_slot_write("0", "0") + [
          "s_cmp_eq_u64 %s, 0" % sp(S_FAULTS),
          "s_cbranch_scc1 .Lfl_nofault",
          ] + lane_pkt_index(R[9]) + [
          "v_mov_b32 %s, %s" % (v(R[8]), s(S_CODE)),
          "global_store_byte %s, %s, %s" % (v(R[9]), v(R[8]), sp(S_FAULTS)),
          ".Lfl_nofault:",
          # a program with map writes: the packet's bit in dp_launch.upd_faulted (its logged
          # writes do not land; map_writes.hip)
          "s_load_dwordx2 %s, s[0:1], 0xa8" % sp(S_JUNK),
          "s_load_dword %s, s[0:1], 0x90" % s(S_BYTES),            # pkt_base (low word)
          "s_waitcnt lgkmcnt(0)",
          "s_cmp_eq_u64 %s, 0" % sp(S_JUNK),
          "s_cbranch_scc1 .Lfl_nomark"] + lane_pkt_index(R[9]) + [
          "v_add_u32 %s, %s, %s" % (v(R[9]), s(S_BYTES), v(R[9])),
          "v_lshrrev_b32 %s, 5, %s" % (v(R[8]), v(R[9])),
          "v_lshlrev_b32 %s, 2, %s" % (v(R[8]), v(R[8])),
          "v_and_b32 %s, 31, %s" % (v(R[10]), v(R[9])),
          "v_lshlrev_b32_e64 %s, %s, 1" % (v(R[10]), v(R[10])),
          "global_atomic_or %s, %s, %s" % (v(R[8]), v(R[10]), sp(S_JUNK)),
          ".Lfl_nomark:",
          # bin 256 (faulted) goes straight to the global histogram: faults are rare, and the
          # LDS histogram then holds exactly 256 bins (1 KB)
          "s_cmp_eq_u64 %s, 0" % sp(S_HIST),
          "s_cbranch_scc1 .Lfl_nohist",
          "s_bcnt1_i32_b64 %s, exec" % s(S_BYTES),
          "s_mov_b64 exec, 1",     # lane 0 only (its operands set below, after the switch)
          "v_mov_b32 %s, %s" % (v(R[8]), s(S_BYTES)),
          "v_mov_b32 %s, 0" % v(R[9]),
          "v_mov_b32 %s, 0" % v(R[10]),
          "global_atomic_add_x2 %s, %s, %s offset:2048" % (v(R[10]), vp(R[8]), sp(S_HIST)),
          ".Lfl_nohist:",
          "s_andn2_b64 %s, %s, %s" % (sp(S_ALIVE), sp(S_ALIVE), sp(S_MASK)),
          "s_andn2_b64 exec, %s, %s" % (sp(S_SAVE), sp(S_MASK)),
          "s_cbranch_execz .Lfl_none",
          "s_setpc_b64 %s" % sp(S_LINK),
          ".Lfl_none:",
          # structured compiled programs continue with no lane (their join restores the rest)
          "s_bitcmp1_b32 s7, 2",
          "s_cbranch_scc0 .Lfl_sched",
          "s_setpc_b64 %s" % sp(S_LINK),
          ".Lfl_sched:"] + goto(".Lr_schedule")
    # UDIVMOD64: n = R[0:1], d = R[2:3] (non-zero) -> q = R[4:5], r = R[6:7]; clobbers R[8:9]
    n, dd, q, r = vp(R[0]), vp(R[2]), vp(R[4]), vp(R[6])
    L += [".Lr_udiv:",
          "v_mov_b32 %s, 0" % v(R[4]), "v_mov_b32 %s, 0" % v(R[5]),
          "v_mov_b32 %s, 0" % v(R[6]), "v_mov_b32 %s, 0" % v(R[7]),
          "s_mov_b32 %s, 64" % s(S_T2),
          ".Ludiv_loop:",
          "v_lshlrev_b64 %s, 1, %s" % (r, r),
          "v_lshrrev_b32 %s, 31, %s" % (v(R[8]), v(R[1])),
          "v_or_b32 %s, %s, %s" % (v(R[6]), v(R[6]), v(R[8])),
          "v_lshlrev_b64 %s, 1, %s" % (n, n),
          "v_lshlrev_b64 %s, 1, %s" % (q, q),
          "v_cmp_ge_u64_e64 vcc, %s, %s" % (r, dd),
          "v_sub_co_u32 %s, %s, %s, %s" % (v(R[8]), sp(S_JUNK), v(R[6]), v(R[2])),
          "v_subb_co_u32 %s, %s, %s, %s, %s" % (v(R[9]), sp(S_JUNK), v(R[7]), v(R[3]), sp(S_JUNK)),
          "v_cndmask_b32 %s, %s, %s, vcc" % (v(R[6]), v(R[6]), v(R[8])),
          "v_cndmask_b32 %s, %s, %s, vcc" % (v(R[7]), v(R[7]), v(R[9])),
          "v_cndmask_b32 %s, 0, 1, vcc" % v(R[8]),
          "v_or_b32 %s, %s, %s" % (v(R[4]), v(R[4]), v(R[8])),
          "s_sub_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_cmp_lg_u32 %s, 0" % s(S_T2),
          "s_cbranch_scc1 .Ludiv_loop",
          "s_setpc_b64 %s" % sp(S_LINK)]
    # CHECK: address H[0:1], size s[S_T0], write s[S_T1]; lanes outside every region fault
    # (MEM, or MAP_WRITE for a store into a map value); returns with exec = good lanes.
    ok = sp(S_OK)             # accumulated ok mask (the fault routine leaves it alone)
    L += [".Lr_check:",
          "s_mov_b64 %s, 0" % ok,
          # packet: u = a - pkt; u_hi == 0 && len >= size && u_lo <= len - size
          "v_sub_co_u32 %s, vcc, %s, v%d" % (v(R[0]), v(H[0]), V_PKT),
          "v_subb_co_u32 %s, vcc, %s, v%d, vcc" % (v(R[1]), v(H[1]), V_PKT + 1),
          "v_subrev_u32 %s, %s, v%d" % (v(R[2]), s(S_T0), V_LEN),
          "v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(R[1])),
          "v_cmp_ge_u32_e64 vcc, v%d, %s" % (V_LEN, s(S_T0)),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "v_cmp_le_u32_e64 vcc, %s, %s" % (v(R[0]), v(R[2])),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_or_b64 %s, %s, %s" % (ok, ok, sp(S_JUNK)),
          # stack: the reference's 512 bytes below r10 (generic accesses force a 516-byte slice,
          # the slice top is r10): u = a - {shared_hi : top - 512}; u_hi == 0 && u_lo <= 512 - size
          "s_sub_u32 %s, %s, 512" % (s(S_T3), s(S_STKSTRIDE)),
          "v_add_u32 %s, %s, v%d" % (v(R[4]), s(S_T3), V_STK),
          "v_sub_co_u32 %s, vcc, %s, %s" % (v(R[0]), v(H[0]), v(R[4])),
          "v_mov_b32 %s, %s" % (v(R[3]), s(S_SHARED + 1)),
          "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[1]), v(H[1]), v(R[3])),
          "s_sub_u32 %s, 512, %s" % (s(S_T3), s(S_T0)),
          "v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(R[1])),
          "v_cmp_ge_u32_e64 vcc, %s, %s" % (s(S_T3), v(R[0])),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_or_b64 %s, %s, %s" % (ok, ok, sp(S_JUNK)),
          # maps: for m in table (dp_map records of 32 B -> s[64:71])
          "s_mov_b32 %s, 0" % s(S_T2),
          ".Lck_map_loop:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_NMAPS)),
          "s_cbranch_scc1 .Lck_map_done",
          "s_lshl_b32 %s, %s, 5" % (s(S_T3), s(S_T2)),
          "s_load_dwordx8 s[%d:%d], %s, %s" % (S_REC, S_REC + 7, sp(S_MAPS), s(S_T3)),
          "s_waitcnt lgkmcnt(0)",
          "s_bitcmp1_b32 s71, 31",                 # hashtable record: its own rule below
          "s_cbranch_scc1 .Lck_hash",
          # s[66:67] = dev_base, s68 = value_size, s69 = max_entries
          "s_mul_i32 %s, s68, s69" % s(S_BYTES),
          "s_sub_u32 %s, %s, %s" % (s(S_T3), s(S_BYTES), s(S_T0)),
          "v_mov_b32 %s, s67" % v(R[3]),
          "v_sub_co_u32 %s, vcc, %s, s66" % (v(R[0]), v(H[0])),
          "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[1]), v(H[1]), v(R[3])),
          "v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_JUNK), v(R[1])),
          "v_cmp_ge_u32_e64 vcc, %s, %s" % (s(S_T3), v(R[0])),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_cmp_ge_u32 %s, %s" % (s(S_BYTES), s(S_T0)),
          "s_cselect_b64 %s, %s, 0" % (sp(S_JUNK), sp(S_JUNK)),
          ".Lck_map_tail:",
          "s_and_b64 %s, %s, exec" % (sp(S_JUNK), sp(S_JUNK)),
          "s_cmp_eq_u32 %s, 0" % s(S_T1),
          "s_cbranch_scc1 .Lck_map_ok",
          # a store into a map value (ebpf_gpu.h "Stores into map values"): .Lr_vstore for those
          # lanes (SGPRs it clobbers spilled to lanes of v51), whose address then points at the
          # lane's scratch, so the handler's own store leaves the map alone
          "s_cmp_eq_u64 %s, 0" % sp(S_JUNK),
          "s_cbranch_scc1 .Lck_map_next"]
    spill = [(S_LINK, 0), (S_LINK + 1, 1), ("exec_lo", 2), ("exec_hi", 3), (S_T0, 4), (S_T1, 5),
             (S_T2, 6), (S_OK, 7), (S_OK + 1, 8), (S_JUNK, 9), (S_JUNK + 1, 10)]
    L += ["v_writelane_b32 v%d, %s, %d" % (SPILL, r if isinstance(r, str) else s(r), k) for r, k in spill]
    L += ["s_mov_b64 exec, %s" % sp(S_JUNK)] + call(".Lr_vstore") + [
          # the lanes that stored: ok, their address the scratch
          "v_readlane_b32 %s, v%d, 9" % (s(S_MASK), SPILL),
          "v_readlane_b32 %s, v%d, 10" % (s(S_MASK + 1), SPILL),
          "s_andn2_b64 %s, %s, %s" % (sp(S_MASK), sp(S_MASK), sp(S_JUNK)),
          "v_readlane_b32 %s, v%d, 7" % (s(S_OK), SPILL),
          "v_readlane_b32 %s, v%d, 8" % (s(S_OK + 1), SPILL),
          "s_or_b64 %s, %s, %s" % (sp(S_OK), sp(S_OK), sp(S_MASK)),
          "s_mov_b64 exec, %s" % sp(S_MASK),
          "v_add_u32 %s, %d, v%d" % (v(H[0]), VST_SCRATCH, V_STK),
          "v_mov_b32 %s, %s" % (v(H[1]), s(S_SHARED + 1)),
          "v_readlane_b32 %s, v%d, 4" % (s(S_T0), SPILL),
          "v_readlane_b32 %s, v%d, 5" % (s(S_T1), SPILL),
          "v_readlane_b32 %s, v%d, 6" % (s(S_T2), SPILL),
          "v_readlane_b32 exec_lo, v%d, 2" % SPILL,
          "v_readlane_b32 exec_hi, v%d, 3" % SPILL,
          # the lanes .Lr_vstore could not serve fault (S_CODE)
          "s_cmp_eq_u64 %s, 0" % sp(S_JUNK),
          "s_cbranch_scc1 .Lck_vs_ok",
          "s_mov_b64 %s, %s" % (sp(S_MASK), sp(S_JUNK))] + call(".Lr_fault") + [
          ".Lck_vs_ok:",
          "v_readlane_b32 %s, v%d, 0" % (s(S_LINK), SPILL),
          "v_readlane_b32 %s, v%d, 1" % (s(S_LINK + 1), SPILL),
          "s_branch .Lck_map_next",
          ".Lck_map_ok:",
          "s_or_b64 %s, %s, %s" % (ok, ok, sp(S_JUNK)),
          ".Lck_map_next:",
          "s_add_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_branch .Lck_map_loop",
          # hashtable table (dprog.h dp_map): only [value, value + value_size) of a slot:
          # u = a - base < slots << lg, and (u mod stride) - value_off <= value_size - size
          ".Lck_hash:",
          "s_mov_b32 s64, s69",
          "s_mov_b32 s65, 0",
          "s_bfe_u32 s70, s71, 0x50010",
          "s_lshl_b64 s[64:65], s[64:65], s70",
          "v_mov_b32 %s, s67" % v(R[3]),
          "v_sub_co_u32 %s, vcc, %s, s66" % (v(R[0]), v(H[0])),
          "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[1]), v(H[1]), v(R[3])),
          "v_cmp_gt_u64_e64 %s, s[64:65], %s" % (sp(S_JUNK), vp(R[0])),
          "s_lshl_b32 %s, 1, s70" % s(S_BYTES),
          "s_sub_u32 %s, %s, 1" % (s(S_BYTES), s(S_BYTES)),
          "v_and_b32 %s, %s, %s" % (v(R[2]), s(S_BYTES), v(R[0])),
          "s_and_b32 %s, s71, 0xffff" % s(S_T3),
          "s_add_u32 %s, %s, 15" % (s(S_T3), s(S_T3)),
          "s_and_b32 %s, %s, -8" % (s(S_T3), s(S_T3)),
          "v_subrev_u32 %s, %s, %s" % (v(R[2]), s(S_T3), v(R[2])),
          "s_sub_u32 %s, s68, %s" % (s(S_BYTES), s(S_T0)),
          "s_cselect_b64 %s, 0, %s" % (sp(S_JUNK), sp(S_JUNK)),  # (scc: size > value_size)
          "v_cmp_ge_u32_e64 vcc, %s, %s" % (s(S_BYTES), v(R[2])),
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_branch .Lck_map_tail",
          ".Lck_map_done:",
          "s_andn2_b64 %s, exec, %s" % (sp(S_MASK), ok),
          "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
          "s_cbranch_scc1 .Lck_ret",
          "s_mov_b32 %s, 3" % s(S_CODE)] + goto(".Lr_fault") + [   # tail call: returns to our caller
          ".Lck_ret:",
          "s_setpc_b64 %s" % sp(S_LINK)]
    # LOOKUP (generic, entered by goto, leaves by dispatch): r0 = lookup(r1, r2) for any r1/r2
    # (NULL -> NULL, unknown map -> BAD_MAP).  Lanes with r1 == 0 or r2 == 0 get r0 = NULL and
    # are parked at the next entry (the scheduler resumes them after the running lanes).
    L += [".Lr_lookup:",
          "v_mov_b32 v0, 0", "v_mov_b32 v1, 0",
          "v_mov_b32 v%d, s12" % V_T,
          "v_cmp_ne_u64_e64 %s, v[2:3], 0" % sp(S_JUNK),
          "v_cmp_ne_u64_e64 vcc, v[4:5], 0",
          "s_and_b64 %s, %s, vcc" % (sp(S_JUNK), sp(S_JUNK)),
          "s_and_b64 exec, %s, exec" % sp(S_JUNK),
          "s_cbranch_execz .Llk_sched",
          # which lanes name a known map
          "s_mov_b64 %s, 0" % sp(S_OK),
          "s_mov_b32 %s, 0" % s(S_T2),
          ".Llk_scan:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_NMAPS)),
          "s_cbranch_scc1 .Llk_scan_done",
          "s_lshl_b32 %s, %s, 5" % (s(S_T3), s(S_T2)),
          "s_load_dwordx2 s[%d:%d], %s, %s" % (S_REC, S_REC + 1, sp(S_MAPS), s(S_T3)),
          "s_waitcnt lgkmcnt(0)",
          "v_cmp_eq_u64_e64 vcc, v[2:3], s[%d:%d]" % (S_REC, S_REC + 1),
          "s_or_b64 %s, %s, vcc" % (sp(S_OK), sp(S_OK)),
          "s_add_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_branch .Llk_scan",
          ".Llk_scan_done:",
          "s_andn2_b64 %s, exec, %s" % (sp(S_MASK), sp(S_OK)),
          "s_cmp_eq_u64 %s, 0" % sp(S_MASK),
          "s_cbranch_scc1 .Llk_known",
          "s_mov_b32 %s, 10" % s(S_CODE)] + call(".Lr_fault") + [
          ".Llk_known:",
          # key = *(u32*)r2, region checked
          "v_mov_b32 %s, v4" % v(H[0]), "v_mov_b32 %s, v5" % v(H[1]),
          "s_mov_b32 %s, 4" % s(S_T0), "s_mov_b32 %s, 0" % s(S_T1)] + call(".Lr_check")
    key = v(H[2])
    L += ["v_mov_b32 %s, 0" % key]
    for b in range(4):
        L += ["flat_load_ubyte %s, %s offset:%d" % (v(H[3]), vp(H[0]), b),
              "s_waitcnt vmcnt(0) lgkmcnt(0)",
              "v_lshl_or_b32 %s, %s, %d, %s" % (key, v(H[3]), 8 * b, key)]
    L += ["s_mov_b32 %s, 0" % s(S_T2),
          ".Llk_map:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_NMAPS)),
          "s_cbranch_scc1 .Llk_done",
          "s_lshl_b32 %s, %s, 5" % (s(S_T3), s(S_T2)),
          "s_load_dwordx8 s[%d:%d], %s, %s" % (S_REC, S_REC + 7, sp(S_MAPS), s(S_T3)),
          "s_waitcnt lgkmcnt(0)",
          "v_cmp_eq_u64_e64 %s, v[2:3], s[64:65]" % sp(S_JUNK),
          "v_cmp_gt_u32_e64 vcc, s69, %s" % key,
          "s_and_b64 vcc, vcc, %s" % sp(S_JUNK),
          "v_mov_b32 %s, s68" % v(H[3]),
          "v_mad_u64_u32 %s, %s, %s, %s, s[66:67]" % (vp(H[4]), sp(S_JUNK), key, v(H[3])),
          "v_cndmask_b32 v0, v0, %s, vcc" % v(H[4]),
          "v_cndmask_b32 v1, v1, %s, vcc" % v(H[5]),
          "s_add_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_branch .Llk_map",
          ".Llk_done:",
          "s_bitcmp1_b32 s7, 1",
          "s_cbranch_scc1 .Llk_jit"] + dispatch(12) + [
          ".Llk_jit:",     # compiled program: s12 = code offset of the next block
          "s_add_u32 %s, %s, s12" % (s(S_JUNK), s(S_CB)),
          "s_addc_u32 %s, %s, 0" % (s(S_JUNK + 1), s(S_CB + 1)),
          "s_setpc_b64 %s" % sp(S_JUNK)] + [
          ".Llk_sched:"] + goto(".Lr_schedule")
    L += hlookup_routine()
    L += update_routine()
    L += hdelete_routine()
    L += vstore_routine()
    # OVLFIX (called by generic loads when dp_launch.vflags bit 0): the packet's own stores over
    # the S_T0 bytes at H[0:1] just read into H[2:3]
    L += [".Lr_ovlfix:"] + ovl_fix("L", (H[2], H[3])) + ["s_setpc_b64 %s" % sp(S_LINK)]
    # PREFETCH (staged kernel): LDS-DMA the 4 KB of 64-B packets of group s[S_T0] into this
    # wave's packet buffer, coalesced (DMA q covers bytes q*1024 .. +1023, its lanes permuted:
    # dma_lane_offsets), lanes past the batch end masked off.  Clobbers s[64:68], m0, exec,
    # H[4:5].
    # The lane mask is a VALU compare, so it is computed under exec = all lanes, whatever exec
    # the caller arrives with (a compare under exec = 0 would DMA no chunk)
    L += [".Lr_prefetch:",
          "s_mov_b64 exec, -1",
          "s_cmp_ge_u32 %s, %s" % (s(S_T0), s(S_NGROUPS)),
          "s_cbranch_scc1 .Lpf_ret",
          "s_lshl_b32 s66, %s, 6" % s(S_T0),
          "s_sub_u32 s66, %s, s66" % s(S_COUNT),           # packets left from this group on
          "s_mov_b32 s64, %s" % s(S_T0),
          "s_mov_b32 s65, 0",
          "s_lshl_b64 s[64:65], s[64:65], 12",
          "s_add_u32 s64, s64, %s" % s(S_DATA),
          "s_addc_u32 s65, s65, %s" % s(S_DATA + 1),
          "s_mov_b32 s67, %s" % s(S_PKTLDS)] + dma_lane_offsets(v(H[4]), v(H[5]))
    for qq in range(4):
        # (lane l's bytes belong to packet 16 qq + (l & 15): inside the batch iff its offset,
        # 64 (l & 15) + 16 (l >> 4), is below 64 x the block's packets left)
        L += ["s_sub_i32 s68, s66, %d" % (16 * qq),
              "s_max_i32 s68, s68, 0",
              "s_min_u32 s68, s68, 16",
              "s_lshl_b32 s68, s68, 6",
              "v_cmp_gt_u32_e64 vcc, s68, %s" % v(H[4]),
              "s_mov_b64 exec, vcc",   # (a VALU write of EXEC would need 5 wait states here)
              "s_mov_b32 m0, s67",
              "s_nop 0",
              "global_load_lds_dwordx4 %s, s[64:65]%s" % (v(H[4]), LD_POLICY)]
        if qq < 3:
            L += ["s_add_u32 s64, s64, 1024", "s_addc_u32 s65, s65, 0",
                  "s_add_u32 s67, s67, 1024"]
    L += [".Lpf_ret:",
          "s_setpc_b64 %s" % sp(S_LINK)]
    return L


def kernel(name, staged, jit=False):
    k = "K%s%s" % ("s" if staged else "g", "j" if jit else "")
    L = [".globl %s" % name, ".p2align 8", ".type %s,@function" % name, "%s:" % name]
    if name == "ebpf_jit_s64" and phased() and SLOTS == 16:
        # the wide kernel: the same code with 16 result slots allocated (store_phased)
        L += [".globl ebpf_jit_s64w", ".type ebpf_jit_s64w,@function", "ebpf_jit_s64w:"]
    # v0 = workitem id; wave index within the 256-lane workgroup
    L += ["v_readfirstlane_b32 %s, v0" % s(S_WAVE),
          "s_lshr_b32 %s, %s, 6" % (s(S_WAVE), s(S_WAVE)),
          "s_load_dwordx16 s[%d:%d], s[0:1], 0x0" % (S_PROG, S_PROG + 15),
          "s_load_dwordx8 s[%d:%d], s[0:1], 0x40" % (S_COUNT, S_COUNT + 7),
          "s_load_dword %s, s[0:1], 0x60" % s(S_GSTRIDE),
          "s_load_dword %s, s[0:1], 0x64" % s(S_PKTLDS),
          "s_mov_b64 %s, src_shared_base" % sp(S_SHARED),
          "v_mov_b32 v%d, 0x00010203" % V_SEL,
          # code base: routines are addressed relative to .Lcb
          "s_getpc_b64 %s" % sp(S_CB),
          ".L%s_pc:" % k,
          "s_add_u32 %s, %s, .Lcb-.L%s_pc" % (s(S_CB), s(S_CB), k),
          "s_addc_u32 %s, %s, 0" % (s(S_CB + 1), s(S_CB + 1)),
          "v_mbcnt_lo_u32_b32 %s, -1, 0" % v(H[0]),
          "v_mbcnt_hi_u32_b32 %s, -1, %s" % (v(H[0]), v(H[0])),
          "v_lshlrev_b32 v%d, 4, %s" % (V_L16, v(H[0])),
          "s_mov_b32 %s, -1" % s(S_PREVG),
          "s_waitcnt lgkmcnt(0)",
          "s_mov_b32 s7, %d" % ((1 if staged else 0) | (2 if jit else 0)),
          # s7 bit 13: the program reads its own stores into map values (dp_launch.vflags bit 0)
          "s_load_dword %s, s[0:1], 0x%x" % (s(S_T3), VFLAGS_OFF)] + (
          # (the general kernels of a phased image leave write phasing off)
          ["s_load_dword %s, s[0:1], 0x%x" % (s(S_WPHASE), WPHASE_OFF) if staged else
           "s_mov_b32 %s, 0" % s(S_WPHASE),
           "s_mov_b32 %s, 0" % s(S_PEND)] if phased() else []) + [
          "s_waitcnt lgkmcnt(0)",
          "s_bitcmp1_b32 %s, 0" % s(S_T3),
          "s_cbranch_scc0 .L%s_noovl" % k,
          "s_or_b32 s7, s7, 0x2000",
          ".L%s_noovl:" % k,
          # s7 bit 15: dp_launch.offsets holds (start, end) pairs (vflags bit 2, DP_VF_EXTENTS)
          "s_bitcmp1_b32 %s, 2" % s(S_T3),
          "s_cbranch_scc0 .L%s_noext" % k,
          "s_or_b32 s7, s7, 0x8000",
          ".L%s_noext:" % k]
    if staged:
        # s7 bit 14 (keep mode): the program reads its packet at run-time offsets from the LDS
        # packet buffer (LDXPKTV), so the next group's DMA waits for the group's end.  Set by
        # the host in dp_launch.vflags (DP_VF_KEEP, still in S_T3) for compiled and interpreted
        # programs alike.  (Double-buffering the packets instead, two 4-KB buffers per wave,
        # measured slower on C3L: 0.294 against 0.284 ms, the LDS cutting 6 workgroups per CU
        # to 4; profiles/r05/keep2/)
        L += ["s_bitcmp1_b32 %s, 3" % s(S_T3),
              "s_cbranch_scc0 .L%s_nokeep" % k,
              "s_or_b32 s7, s7, 0x4000",
              ".L%s_nokeep:" % k]
    if not staged:   # header staging requested by the host (dp_launch.lds_pkt_base bit 31)
        L += ["s_bitcmp1_b32 %s, 31" % s(S_PKTLDS),
              "s_cbranch_scc0 .L%s_nogs" % k,
              "s_or_b32 s7, s7, 8",
              ".L%s_nogs:" % k,
              # bit 30: the staged headers are kept in the wave's LDS packet buffer too, for the
              # loads at run-time offsets (s7 bit 14 in the general kernels)
              "s_bitcmp1_b32 %s, 30" % s(S_PKTLDS),
              "s_cbranch_scc0 .L%s_nohl" % k,
              "s_or_b32 s7, s7, 0x4000",
              ".L%s_nohl:" % k,
              "s_and_b32 %s, %s, 0x3fffffff" % (s(S_PKTLDS), s(S_PKTLDS))]
    L += ["s_branch .Lprologue"]
    return L


V_RES = 44   # v[44:45]: r0 of the lanes that retired in the running group


def lane_index(dst):
    """dst = this lane's index in the wave (0..63)."""
    if STAGED_IMAGE:
        return ["v_lshrrev_b32 %s, 4, v%d" % (v(dst), V_L16)]
    return ["v_mbcnt_lo_u32_b32 %s, -1, 0" % v(dst), "v_mbcnt_hi_u32_b32 %s, -1, %s" % (v(dst), v(dst))]


def lane_pkt_index(dst):
    """dst = the packet index of this lane in the launch (general image: V_IDX)."""
    if STAGED_IMAGE:
        return ["v_lshrrev_b32 %s, 4, v%d" % (v(dst), V_L16),
                "v_lshl_add_u32 %s, %s, 6, %s" % (v(dst), s(S_GROUP), v(dst))]
    return ["v_mov_b32 %s, v%d" % (v(dst), V_IDX)]


def pkt_setup(idx, tag):
    """General kernels: V_PKT / V_LEN of the running lanes' packets (index in VGPR idx), and with
    header staging (s7 bit 3) their first 64 bytes into v22..v37.  Clobbers H[1], H[4:5], R[0],
    R[2], S_JUNK; leaves exec = the running lanes (s[S_MASK] holds them meanwhile)."""
    return ["s_mov_b64 %s, exec" % sp(S_MASK),
            "s_cmp_eq_u64 %s, 0" % sp(S_OFFS),
            "s_cbranch_scc0 .Lps_offsets_%s" % tag,
            "v_mov_b32 %s, %s" % (v(H[1]), s(S_STRIDE)),
            "v_mad_u64_u32 v[%d:%d], %s, v%d, %s, %s" % (V_PKT, V_PKT + 1, sp(S_JUNK), idx,
                                                         v(H[1]), sp(S_DATA)),
            "v_mov_b32 v%d, %s" % (V_LEN, s(S_STRIDE)),
            "s_branch .Lps_stage_%s" % tag,
            ".Lps_offsets_%s:" % tag,
            # offsets[i], offsets[i + 1]; extents batches (s7 bit 15): offsets[2i], offsets[2i + 1]
            "s_bitcmp1_b32 s7, 15",
            "s_cselect_b32 %s, 16, 8" % s(S_JUNK),
            "v_mov_b32 %s, %s" % (v(H[1]), s(S_JUNK)),
            "v_mad_u64_u32 %s, %s, v%d, %s, %s" % (vp(H[4]), sp(S_JUNK), idx, v(H[1]), sp(S_OFFS)),
            "global_load_dwordx2 %s, %s, off offset:8" % (vp(R[0]), vp(H[4])),
            "global_load_dwordx2 %s, %s, off" % (vp(H[4]), vp(H[4])),
            "s_waitcnt vmcnt(0)",
            # length = end - start; an end below its start or 4 GiB past it: length 0 (every load
            # of the packet faults MEM)
            "v_sub_co_u32 v%d, vcc, %s, %s" % (V_LEN, v(R[0]), v(H[4])),
            "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[1]), v(R[1]), v(H[5])),
            "v_cmp_ne_u32_e32 vcc, 0, %s" % v(R[1]),
            "v_cndmask_b32 v%d, v%d, 0, vcc" % (V_LEN, V_LEN),
            "v_mov_b32 %s, %s" % (v(R[2]), s(S_OFFBASE + 1)),
            "v_sub_co_u32 %s, vcc, %s, %s" % (v(H[4]), v(H[4]), s(S_OFFBASE)),
            "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(H[5]), v(H[5]), v(R[2])),
            "v_lshl_add_u64 v[%d:%d], %s, 0, %s" % (V_PKT, V_PKT + 1, vp(H[4]), sp(S_DATA)),
            ] + [
            # header staging: the first 64 bytes of every packet at least that long into
            # v22..v37 (what the staged kernels' LDS DMA provides)
            ".Lps_stage_%s:" % tag,
            "s_bitcmp1_b32 s7, 3",
            "s_cbranch_scc0 .Lps_done_%s" % tag,
            "v_cmp_lt_u32_e64 vcc, 63, v%d" % V_LEN,
            "s_and_b64 exec, %s, vcc" % sp(S_MASK),
            "s_cbranch_execz .Lps_done_%s" % tag] + [
            "global_load_dwordx4 v[%d:%d], v[%d:%d], off offset:%d" % (PKT0 + 4 * q, PKT0 + 4 * q + 3,
                                                                       V_PKT, V_PKT + 1, 16 * q)
            for q in range(4)] + [
            "s_waitcnt vmcnt(0)",
            # (s7 bit 14: the headers also into the wave's LDS packet buffer, transposed, for
            # loads at run-time offsets: h_ldx_pktv)
            "s_bitcmp1_b32 s7, 14",
            "s_cbranch_scc0 .Lps_done_%s" % tag,
            "v_mbcnt_lo_u32_b32 %s, -1, 0" % v(H[1]),
            "v_mbcnt_hi_u32_b32 %s, -1, %s" % (v(H[1]), v(H[1])),
            "v_lshl_add_u32 %s, %s, 2, %s" % (v(H[1]), v(H[1]), s(S_PKTLDS))] + lds_pkt_dwords(v(H[1])) + [
            ".Lps_done_%s:" % tag,
            "s_mov_b64 exec, %s" % sp(S_MASK)]


def ret_slot_write(x0, x1):
    """r0 of the retiring lanes into v[44:45]; a superblock kernel (RETK > 1) moves the whole
    group's results into its slot v[V_RB + 2k], k = group % RETK, once when the group is done
    (slot_commit), not at every exit."""
    return ["v_mov_b32 v%d, %s" % (V_RES, x0), "v_mov_b32 v%d, %s" % (V_RES + 1, x1)]


def phased():
    """The image's kernels keep result slots that store_phased can write (staged, RETK > 1)."""
    return STAGED_IMAGE and RETK > 1


def slot_commit():
    if RETK == 1:
        return []
    L = ["s_mov_b64 exec, -1",
         "s_and_b32 %s, %s, %s" % (s(S_BYTES), s(S_GROUP), s(S_KMASK))]
    if phased() and SLOTS == 16:
        # wide phasing (dp_launch.wphase bit 31, the 96-VGPR kernel): 16 slots, the superblocks
        # of a wave alternating between slots 0-7 and 8-15 (s98 bit 31 = the running half,
        # switched at each superblock's first group)
        L += ["s_cmp_eq_u32 %s, 0" % s(S_BYTES),
              "s_cbranch_scc0 .Lsc_half",
              "s_bitcmp1_b32 %s, 31" % s(S_WPHASE),
              "s_cbranch_scc0 .Lsc_half",
              "s_xor_b32 %s, %s, 0x80000000" % (s(S_PEND), s(S_PEND)),
              ".Lsc_half:",
              "s_lshr_b32 %s, %s, 28" % (s(S_T0), s(S_PEND)),
              "s_and_b32 %s, %s, 8" % (s(S_T0), s(S_T0)),
              "s_or_b32 %s, %s, %s" % (s(S_BYTES), s(S_BYTES), s(S_T0)),
              "s_bitset1_b32 %s, %s" % (s(S_PEND), s(S_BYTES))]
    elif phased():
        L.append("s_bitset1_b32 %s, %s" % (s(S_PEND), s(S_BYTES)))
    return L + [
            "s_lshl_b32 %s, %s, 1" % (s(S_BYTES), s(S_BYTES)),
            "s_set_gpr_idx_on %s, gpr_idx(DST)" % s(S_BYTES),
            "v_mov_b32 v%d, v%d" % (V_RB, V_RES),
            "v_mov_b32 v%d, v%d" % (V_RB + 1, V_RES + 1),
            "s_set_gpr_idx_off"]


def store_phased(tag, final):
    """Write phasing (dp_launch.wphase != 0, staged kernels with result slots): instead of one
    burst per superblock, a wave writes the slots of all its finished groups (S_PEND bits 0-15)
    when the GPU's constant clock is inside the write window, when the next group's slot still
    holds an unwritten group (all slots full), and at the end (`final`).  Every wave reads the same
    100-MHz counter, so the result writes of the whole GPU bunch into the windows and the packet
    reads run alone between them: HBM turns between reading and writing far less often (floor
    kernel, tools/ubench/phase.hip: 0.855 -> 0.773 ms for 64M packets).
    Slots: slot k = group & K'-1 of the wave's last superblocks; with wphase bit 31 (wide, the
    96-VGPR kernel) a wave's superblocks alternate between slots 0-7 and 8-15 (s98 bit 31 = the
    half of S_PREVG's superblock), so 16 groups fit (0.770 -> 0.753 ms, tools/ubench/phase2.hip).
    An unwritten slot of S_PREVG's half belongs to its superblock (index <= S_PREVG's) or to the
    one `back` (index above: two superblocks back when wide, one otherwise); a slot of the other
    half to the previous superblock.  Falls through to the superblock burst when wphase is 0;
    clobbers exec, S_T0..S_T3, S_BYTES, s[60:69], R[0], R[1]."""
    P = s(S_PEND)
    L = ["s_cmp_eq_u32 %s, 0" % s(S_WPHASE),
         "s_cbranch_scc1 .Lph_off_%s" % tag] + (
        ["s_waitcnt lgkmcnt(0)"] if not final else []) + [   # (the clock read)
         "s_and_b32 %s, %s, 0xffff" % (s(S_T0), P),
         "s_cbranch_scc0 .Lsp_none_%s" % tag]                   # nothing unwritten
    if not final:
        L += [# the next group's slot is taken: write now
              "s_and_b32 %s, %s, %s" % (s(S_T0), s(S_GROUP), s(S_KMASK)),
              "s_lshr_b32 %s, %s, 28" % (s(S_T1), P),
              "s_and_b32 %s, %s, 8" % (s(S_T1), s(S_T1)),
              "s_cmp_eq_u32 %s, 0" % s(S_T0),
              "s_cbranch_scc0 .Lph_nf_%s" % tag,
              "s_bitcmp1_b32 %s, 31" % s(S_WPHASE),
              "s_cbranch_scc0 .Lph_nf_%s" % tag,
              "s_xor_b32 %s, %s, 8" % (s(S_T1), s(S_T1)),           # (a new superblock's half)
              ".Lph_nf_%s:" % tag,
              "s_or_b32 %s, %s, %s" % (s(S_T0), s(S_T0), s(S_T1)),
              "s_bitcmp1_b32 %s, %s" % (P, s(S_T0)),
              "s_cbranch_scc1 .Lph_write_%s" % tag,
              "s_and_b32 %s, %s, 0x1f0000" % (s(S_T1), s(S_WPHASE)),   # width, offset 0
              "s_and_b32 %s, %s, 0xffff" % (s(S_T2), s(S_WPHASE)),
              "s_bfe_u32 %s, %s, %s" % (s(S_T0), s(S_CLOCK), s(S_T1)),
              "s_cmp_lt_u32 %s, %s" % (s(S_T0), s(S_T2)),
              "s_cbranch_scc0 .Lsp_none_%s" % tag,
              ".Lph_write_%s:" % tag]
    L += ["s_mov_b64 exec, -1",
          "v_lshrrev_b32 %s, 1, v%d" % (v(R[0]), V_L16),                # lane * 8
          "s_andn2_b32 %s, %s, %s" % (s(S_T1), s(S_PREVG), s(S_KMASK)),  # cur: S_PREVG's superblock
          "s_add_u32 %s, %s, %s" % (s(S_T2), s(S_GSTRIDE), s(S_KMASK)),  # superblock stride
          "s_sub_u32 %s, %s, %s" % (s(S_T0), s(S_T1), s(S_T2)),         # prev: the one before
          "s_bitcmp1_b32 %s, 31" % s(S_WPHASE),
          "s_cselect_b32 %s, %s, 0" % (s(S_T2), s(S_T2)),
          "s_sub_u32 %s, %s, %s" % (s(S_T2), s(S_T0), s(S_T2)),         # back
          "s_and_b32 %s, %s, %s" % (s(S_T3), s(S_PREVG), s(S_KMASK)),   # S_PREVG's slot index
          # every packet of cur (and so of the older ones) in the batch: no per-slot bounds (all
          # but a launch's last superblock)
          "s_lshr_b32 s66, %s, 6" % s(S_COUNT),
          "s_add_u32 s67, %s, %s" % (s(S_T1), s(S_KMASK)),
          "s_cmp_lt_u32 s67, s66",
          "s_cbranch_scc0 .Lph_ragged_%s" % tag]
    # result addresses of cur, prev and back: s[60:61], s[62:63], s[64:65]
    for lo, g in ((60, S_T1), (62, S_T0), (64, S_T2)):
        L += ["s_lshl_b32 s%d, %s, 9" % (lo, s(g)),
              "s_lshr_b32 s%d, %s, 23" % (lo + 1, s(g)),
              "s_add_u32 s%d, s%d, %s" % (lo, lo, s(S_RET)),
              "s_addc_u32 s%d, s%d, %s" % (lo + 1, lo + 1, s(S_RET + 1))]
    halves = [0] if RETK == SLOTS else [0, 1]

    def slots_of(half, ragged):
        """The writes for S_PREVG's half `half`: its own slots, then the other half's."""
        out = []
        for own in (True, False):
            h = half if own else 1 - half
            if h not in halves:
                continue
            for i in range(RETK):
                j = 8 * h + i
                sk = ".Lph_%s%d_%d_%s" % ("r" if ragged else "f", half, j, tag)
                out += ["s_bitcmp1_b32 %s, %d" % (P, j), "s_cbranch_scc0 %s" % sk]
                if not ragged:
                    if own:
                        out += ["s_cmp_ge_u32 %s, %d" % (s(S_T3), i),
                                "s_cselect_b64 s[66:67], s[60:61], s[64:65]"]
                    out.append("global_store_dwordx2 %s, v[%d:%d], s[%d:%d] offset:%d%s" % (
                        v(R[0]), V_RB + 2 * j, V_RB + 2 * j + 1, 66 if own else 62,
                        67 if own else 63, 512 * i, ST_POLICY))
                else:
                    if own:
                        out += ["s_cmp_ge_u32 %s, %d" % (s(S_T3), i),
                                "s_cselect_b32 %s, %s, %s" % (s(S_BYTES), s(S_T1), s(S_T2))]
                    else:
                        out.append("s_mov_b32 %s, %s" % (s(S_BYTES), s(S_T0)))
                    out += ["s_add_u32 %s, %s, %d" % (s(S_BYTES), s(S_BYTES), i),   # the group
                            "s_lshl_b32 s66, %s, 6" % s(S_BYTES),
                            "s_sub_u32 s66, %s, s66" % s(S_COUNT),                 # its packets
                            "v_cmp_gt_u32_e64 vcc, s66, %s" % v(R[1]),
                            "s_mov_b64 exec, vcc",
                            "s_lshl_b32 s66, %s, 9" % s(S_BYTES),
                            "s_lshr_b32 s67, %s, 23" % s(S_BYTES),
                            "s_add_u32 s66, s66, %s" % s(S_RET),
                            "s_addc_u32 s67, s67, %s" % s(S_RET + 1),
                            "global_store_dwordx2 %s, v[%d:%d], s[66:67]%s" % (
                                v(R[0]), V_RB + 2 * j, V_RB + 2 * j + 1, ST_POLICY),
                            "s_mov_b64 exec, -1"]
                out.append(sk + ":")
        return out

    for ragged in (False, True):
        if ragged:
            L += [".Lph_ragged_%s:" % tag,
                  "v_lshrrev_b32 %s, 4, v%d" % (v(R[1]), V_L16)]            # lane
        if len(halves) > 1:
            L += ["s_bitcmp1_b32 %s, 31" % P,
                  "s_cbranch_scc1 .Lph_%sh1_%s" % ("r" if ragged else "f", tag)]
        L += slots_of(0, ragged) + ["s_branch .Lph_done_%s" % tag]
        if len(halves) > 1:
            L += [".Lph_%sh1_%s:" % ("r" if ragged else "f", tag)] + slots_of(1, ragged) + [
                  "s_branch .Lph_done_%s" % tag]
    L += [".Lph_done_%s:" % tag,
          "s_and_b32 %s, %s, 0x80000000" % (P, P),                  # (keeps the half)
          "s_branch .Lsp_none_%s" % tag,
          ".Lph_off_%s:" % tag]
    return L


def store_prev_results(tag, final):
    """Write the result slots of the superblock that group S_PREVG ends (at the start of the
    next superblock, or at the end: `final`) as one burst of RETK x 512 B; clobbers exec.
    (With write phasing on, store_phased decides instead.)"""
    L = store_phased(tag, final) if phased() else []
    L += ["s_cmp_eq_u32 %s, -1" % s(S_PREVG),
         "s_cbranch_scc1 .Lsp_none_%s" % tag]
    if not final and RETK > 1:
        L += ["s_and_b32 %s, %s, %s" % (s(S_T0), s(S_PREVG), s(S_KMASK)),
              "s_cmp_lg_u32 %s, %s" % (s(S_T0), s(S_KMASK)),
              "s_cbranch_scc1 .Lsp_none_%s" % tag]
    # R0 = byte offset of the superblock's first packet result for this lane; R1 = its index
    # (all lanes: the current group's live mask says nothing about the stored groups)
    L += ["s_mov_b64 exec, -1",
          # (one result slot: the group itself, whatever the superblock size the host chose)
          "s_andn2_b32 %s, %s, %s" % (s(S_T0), s(S_PREVG), s(S_KMASK)) if RETK > 1 else
          "s_mov_b32 %s, %s" % (s(S_T0), s(S_PREVG)),
          ] + (["v_lshrrev_b32 %s, 4, v%d" % (v(R[1]), V_L16),
                "v_lshl_add_u32 %s, %s, 6, %s" % (v(R[1]), s(S_T0), v(R[1]))] if STAGED_IMAGE else
               ["v_mov_b32 %s, v%d" % (v(R[1]), V_IDX)]) + [
          "v_lshlrev_b32 %s, 3, %s" % (v(R[0]), v(R[1]))]
    for k in range(RETK):
        if k:
            L += ["s_cmp_lt_u32 %s, %d" % (s(S_KMASK), k),        # past this launch's K'
                  "s_cbranch_scc1 .Lsp_none_%s" % tag,
                  "v_add_u32 %s, 64, %s" % (v(R[1]), v(R[1]))]
        L += ["v_cmp_gt_u32_e64 vcc, %s, %s" % (s(S_COUNT), v(R[1])),
              "s_mov_b64 exec, vcc",
              "global_store_dwordx2 %s, v[%d:%d], %s offset:%d%s" % (
                  v(R[0]), V_RB + 2 * k, V_RB + 2 * k + 1, sp(S_RET), 512 * k, ST_POLICY)]
    L.append(".Lsp_none_%s:" % tag)
    return L


def next_group(dst):
    """dst = the group after S_GROUP in this wave's sequence (superblocks of RETK groups;
    S_GSTRIDE holds the jump to the next superblock's first group)."""
    return ["s_and_b32 %s, %s, %s" % (s(dst), s(S_GROUP), s(S_KMASK)),
            "s_cmp_eq_u32 %s, %s" % (s(dst), s(S_KMASK)),
            "s_cselect_b32 %s, %s, 1" % (s(dst), s(S_GSTRIDE)),
            "s_add_u32 %s, %s, %s" % (s(dst), s(dst), s(S_GROUP))]


def common_group_code():
    """Shared by all kernels (s7 bit 0: staged 64-B packets; bit 1: compiled program)."""
    L = [".Lcb:",
         "ebpf_cb:",
         ".Lprologue:"]
    # lane stack bottom = lds_base + (wave*64 + lane) * stride
    L += ["s_lshl_b32 %s, %s, 6" % (s(S_T0), s(S_WAVE)),
          "v_add_u32 %s, %s, %s" % (v(H[1]), s(S_T0), v(H[0])),          # tid
          "v_mul_lo_u32 %s, %s, %s" % (v(H[4]), v(H[1]), s(S_STKSTRIDE)),
          "v_add_u32 v%d, %s, %s" % (V_STK, s(S_LDSBASE), v(H[4]))]
    # zero the LDS verdict histogram (bins 0..255, one per lane of the 4 waves)
    L += ["v_lshlrev_b32 %s, 2, %s" % (v(H[2]), v(H[1])),
          "v_mov_b32 %s, 0" % v(H[3]),
          "ds_write_b32 %s, %s" % (v(H[2]), v(H[3]))]
    # copy the LDS-resident array maps (dp_map.lds_off != ~0) into LDS: 256 lanes x 4 B
    L += ["v_lshlrev_b32 %s, 2, %s" % (v(H[4]), v(H[1])),
          "s_mov_b32 %s, 0" % s(S_T2),
          ".Lmc_loop:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_NMAPS)),
          "s_cbranch_scc1 .Lmc_done",
          "s_lshl_b32 %s, %s, 5" % (s(S_T3), s(S_T2)),
          "s_load_dwordx8 s[%d:%d], %s, %s" % (S_REC, S_REC + 7, sp(S_MAPS), s(S_T3)),
          "s_waitcnt lgkmcnt(0)",
          "s_add_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_cmp_eq_u32 s70, -1",
          "s_cbranch_scc1 .Lmc_loop",
          "s_mul_i32 %s, s68, s69" % s(S_T1),
          "s_mov_b32 %s, 0" % s(S_T0),
          ".Lmc_chunk:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T0), s(S_T1)),
          "s_cbranch_scc1 .Lmc_zero",
          "v_add_u32 %s, %s, %s" % (v(H[5]), s(S_T0), v(H[4])),
          "v_cmp_gt_u32_e64 vcc, %s, %s" % (s(S_T1), v(H[5])),
          "s_mov_b64 exec, vcc",
          "global_load_dword %s, %s, s[66:67]" % (v(H[3]), v(H[5])),
          "s_waitcnt vmcnt(0)",
          "v_add_u32 %s, s70, %s" % (v(H[5]), v(H[5])),
          "ds_write_b32 %s, %s" % (v(H[5]), v(H[3])),
          "s_mov_b64 exec, -1",
          "s_add_u32 %s, %s, 1024" % (s(S_T0), s(S_T0)),
          "s_branch .Lmc_chunk",
          # a DP_MAP_LDSDELTA map: its workgroup sums start at zero
          ".Lmc_zero:",
          "s_bitcmp1_b32 s71, 29",
          "s_cbranch_scc0 .Lmc_loop",
          "s_and_b32 %s, s71, 0xffff" % s(S_T3),
          "v_mov_b32 %s, 0" % v(H[3]),
          "s_mov_b32 %s, 0" % s(S_T0),
          ".Lmc_zchunk:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T0), s(S_T1)),
          "s_cbranch_scc1 .Lmc_loop",
          "v_add_u32 %s, %s, %s" % (v(H[5]), s(S_T0), v(H[4])),
          "v_cmp_gt_u32_e64 vcc, %s, %s" % (s(S_T1), v(H[5])),
          "s_mov_b64 exec, vcc",
          "v_add_u32 %s, %s, %s" % (v(H[5]), s(S_T3), v(H[5])),
          "ds_write_b32 %s, %s" % (v(H[5]), v(H[3])),
          "s_mov_b64 exec, -1",
          "s_add_u32 %s, %s, 1024" % (s(S_T0), s(S_T0)),
          "s_branch .Lmc_zchunk",
          ".Lmc_done:",
          "s_waitcnt lgkmcnt(0)",
          "s_barrier"]
    # groups of 64 packets: group = workgroup*4 + wave, stride = total waves
    L += ["s_add_u32 %s, %s, 63" % (s(S_NGROUPS), s(S_COUNT)),
          "s_lshr_b32 %s, %s, 6" % (s(S_NGROUPS), s(S_NGROUPS)),
          # (an XCD-major logical workgroup order, each XCD one contiguous share of the
          # batch, measured 1-5% slower: profiles/r02/s3/ab_xcd_order.txt)
          "s_lshl_b32 %s, s2, 2" % s(S_GROUP),
          "s_add_u32 %s, %s, %s" % (s(S_GROUP), s(S_GROUP), s(S_WAVE)),
          # K' = superblock size of this launch (total_waves bits 28..29 = log2 K')
          "s_lshr_b32 %s, %s, 28" % (s(S_T1), s(S_GSTRIDE)),
          "s_and_b32 %s, %s, 0xffff" % (s(S_GSTRIDE), s(S_GSTRIDE)),
          "s_lshl_b32 %s, 1, %s" % (s(S_KMASK), s(S_T1)),
          "s_sub_u32 %s, %s, 1" % (s(S_KMASK), s(S_KMASK)),
          "s_lshl_b32 %s, %s, %s" % (s(S_GROUP), s(S_GROUP), s(S_T1)),
          ] + [
          # superblock jump: (total waves - 1) * K' + 1
          "s_lshl_b32 %s, %s, %s" % (s(S_GSTRIDE), s(S_GSTRIDE), s(S_T1)),
          "s_sub_u32 %s, %s, %s" % (s(S_GSTRIDE), s(S_GSTRIDE), s(S_KMASK)),
          # this wave's packet buffer (staged kernel); first group's prefetch
          "s_lshl_b32 %s, %s, 12" % (s(S_T0), s(S_WAVE)),
          "s_add_u32 %s, %s, %s" % (s(S_PKTLDS), s(S_PKTLDS), s(S_T0)),
          "s_bitcmp1_b32 s7, 0",
          "s_cbranch_scc0 .Lgroup_check",
          "s_mov_b32 %s, %s" % (s(S_T0), s(S_GROUP))] + call(".Lr_prefetch") + [
          "s_branch .Lgroup_check"]
    L += [".Lgroup_done:"]
    L += slot_commit() + next_group(S_T0) + [
          # keep mode (s7 bits 14 and 0: staged kernels): the next group's DMA, now that the
          # program is done with the packet buffer
          "s_and_b32 %s, s7, 0x4001" % s(S_BYTES),
          "s_cmp_eq_u32 %s, 0x4001" % s(S_BYTES),
          "s_cbranch_scc0 .Lgd_nokeep"] + call(".Lr_prefetch") + [
          ".Lgd_nokeep:",
          "s_mov_b32 %s, %s" % (s(S_GROUP), s(S_T0)),
          ".Lgroup_check:",
          "s_mov_b64 exec, -1",
          "s_cmp_lt_u32 %s, %s" % (s(S_GROUP), s(S_NGROUPS)),
          "s_cbranch_scc0 .Lfinish",
          ] + (
          # write phasing: the clock read for store_phased, early so that the group's staging
          # waits cover its latency
          ["s_cmp_eq_u32 %s, 0" % s(S_WPHASE),
           "s_cbranch_scc1 .Lgc_noclock",
           "s_memrealtime s[%d:%d]" % (S_CLOCK, S_CLOCK + 1),
           ".Lgc_noclock:"] if phased() else []) + lane_index(H[0]) + [
          "v_lshl_add_u32 v%d, %s, 6, %s" % (H[3], s(S_GROUP), v(H[0])),      # packet index
          "v_cmp_gt_u32_e64 %s, %s, v%d" % (sp(S_ALIVE), s(S_COUNT), H[3]),
          ] + [
          "s_bitcmp1_b32 s7, 0",
          "s_cbranch_scc0 .Lgs_general",
          # staged: this group's packets are (or are being) DMA'd into the packet buffer
          "s_waitcnt vmcnt(0)",
          # lane p's chunk c at 1024 (p >> 4) + 256 c + 16 (p & 15) (dma_lane_offsets):
          # 16 p + 3 x (16 p & 0x300), then 256 c per chunk
          "v_and_b32 %s, 0x300, v%d" % (v(H[1]), V_L16),
          "v_mad_u32_u24 %s, %s, 3, v%d" % (v(H[1]), v(H[1]), V_L16),
          "v_add_u32 %s, %s, %s" % (v(H[1]), s(S_PKTLDS), v(H[1]))]
    for q in range(4):
        L.append("ds_read_b128 v[%d:%d], %s offset:%d" % (PKT0 + 4 * q, PKT0 + 4 * q + 3,
                                                          v(H[1]), 256 * q))
    # next group's DMA: a full group (the common case) inline, with exec = all lanes and the
    # instruction offset stepping both the global and the LDS address (M0 set once); a partial
    # group through the masking routine.  (Keep mode, s7 bit 14: none here; .Lgroup_done
    # issues it once the program is done with the buffer)
    # (keep mode: the group's packets rewritten transposed for the program's loads at run-time
    # offsets, lds_pkt_dwords, once every lane's staging read has returned)
    L += ["s_waitcnt lgkmcnt(0)",
          "s_bitcmp1_b32 s7, 14",
          "s_cbranch_scc0 .Lgs_pf_dma",
          "v_lshrrev_b32 %s, 2, v%d" % (v(H[1]), V_L16),
          "v_add_u32 %s, %s, %s" % (v(H[1]), s(S_PKTLDS), v(H[1]))] + lds_pkt_dwords(v(H[1])) + [
          "s_branch .Lgs_pf_done",
          ".Lgs_pf_dma:"] + next_group(S_T0) + [
          "s_lshr_b32 %s, %s, 6" % (s(S_BYTES), s(S_COUNT)),        # full groups
          "s_cmp_lt_u32 %s, %s" % (s(S_T0), s(S_BYTES)),
          "s_cbranch_scc0 .Lgs_pf_slow",
          "s_lshr_b32 s65, %s, 20" % s(S_T0),
          "s_lshl_b32 s64, %s, 12" % s(S_T0),
          "s_add_u32 s64, s64, %s" % s(S_DATA),
          "s_addc_u32 s65, s65, %s" % s(S_DATA + 1),
          "s_mov_b64 exec, -1"] + dma_lane_offsets(v(H[4]), v(H[5])) + [
          "s_mov_b32 m0, %s" % s(S_PKTLDS),
          "s_nop 0"] + [
          "global_load_lds_dwordx4 %s, s[64:65] offset:%d%s" % (v(H[4]), 1024 * qq, LD_POLICY)
          for qq in range(4)] + [
          "s_branch .Lgs_pf_done",
          ".Lgs_pf_slow:"] + call(".Lr_prefetch") + [
          ".Lgs_pf_done:",
          # a compiled program computes the packet address itself if it needs it
          "s_bitcmp1_b32 s7, 1",
          "s_cbranch_scc1 .Lgs_init",
          "s_mov_b64 exec, %s" % sp(S_ALIVE),
          "v_mov_b32 %s, 64" % v(H[1]),
          "v_mad_u64_u32 v[%d:%d], %s, v%d, %s, %s" % (V_PKT, V_PKT + 1, sp(S_JUNK), H[3],
                                                       v(H[1]), sp(S_DATA)),
          "v_mov_b32 v%d, 64" % V_LEN,
          "s_branch .Lgs_init",
          ".Lgs_general:",
          "s_mov_b64 exec, %s" % sp(S_ALIVE)] + pkt_setup(H[3], "g") + [
          ".Lgs_init:"] + store_prev_results("g", False) + [
          "s_mov_b32 %s, %s" % (s(S_PREVG), s(S_GROUP))] + ([] if STAGED_IMAGE else [
          # V_IDX: this group's packet indices (after the previous group's store read them)
          "s_mov_b64 exec, -1",
          "v_mov_b32 v%d, v%d" % (V_IDX, H[3])]) + [
          "s_mov_b64 exec, %s" % sp(S_ALIVE),
          # fault code 0 for the whole group up front (a faulting lane overwrites its byte)
          "s_cmp_eq_u64 %s, 0" % sp(S_FAULTS),
          "s_cbranch_scc1 .Lgs_nofz",
          ] + lane_pkt_index(R[9]) + [
          "v_mov_b32 %s, 0" % v(R[8]),
          "global_store_byte %s, %s, %s" % (v(R[9]), v(R[8]), sp(S_FAULTS)),
          ".Lgs_nofz:",
          # a compiled program (s7 bit 1) starts at the head of its code area and sets up the
          # registers it reads itself (packet address, r1, r10, zeroes: asm_cc.cpp prologue)
          "s_bitcmp1_b32 s7, 1",
          "s_cbranch_scc0 .Lgs_interp"] + goto("ebpf_jit_area+16") + [
          ".Lgs_interp:"]
    # r0, r2..r9 start at zero
    for r in range(0, 20, 2):
        if r != 2:
            L.append("v_mov_b64 v[%d:%d], 0" % (r, r + 1))
    L += ["v_mov_b64 v[2:3], v[%d:%d]" % (V_PKT, V_PKT + 1),
          "v_add_u32 v20, %s, v%d" % (s(S_STKSTRIDE), V_STK),
          "v_mov_b32 v21, %s" % s(S_SHARED + 1),
          "s_lshl_b32 %s, %s, 5" % (s(S_T0), s(S_START)),
          "v_mov_b32 v%d, %s" % (V_T, s(S_T0))] + goto(".Lr_schedule")
    # finish: this workgroup's LDS histogram (u32 bins) goes into the launch's u64 partial
    # histograms with device-scope atomics, one replica per (workgroup & 7) so that the adds to
    # a hot bin spread over 8 lines; the workgroup whose ticket add returns nwg - 1 arrived last
    # and moves the 8 replicas (read-and-zero swaps) plus the fault count into the caller's
    # histogram (stored, or added), then re-arms the ticket.  One kernel per launch: no
    # second-stage reduce (hand-off form: 8-B agent atomics on both sides, MI355X_MICROARCH.md
    # "Valid forms")
    HR = HIST_REPLICA_BYTES
    L += [".Lfinish:"] + store_prev_results("f", True)
    L += [".Lfinish_body:",
          "s_mov_b64 exec, -1",
          "s_waitcnt vmcnt(0) lgkmcnt(0)",
          "s_barrier"]
    # DP_MAP_LDSDELTA maps: the workgroup's sums into the delta areas (a global atomic per
    # non-zero word; lane tid takes words tid, tid + 256, ...)
    L += lane_index(H[0]) + [
          "s_lshl_b32 %s, %s, 6" % (s(S_T0), s(S_WAVE)),
          "v_add_u32 %s, %s, %s" % (v(H[1]), s(S_T0), v(H[0])),       # tid
          "s_mov_b32 %s, 0" % s(S_T2),
          ".Lfd_loop:",
          "s_cmp_ge_u32 %s, %s" % (s(S_T2), s(S_NMAPS)),
          "s_cbranch_scc1 .Lfd_done",
          "s_lshl_b32 %s, %s, 5" % (s(S_T3), s(S_T2)),
          "s_load_dwordx8 s[%d:%d], %s, %s" % (S_REC, S_REC + 7, sp(S_MAPS), s(S_T3)),
          "s_waitcnt lgkmcnt(0)",
          "s_add_u32 %s, %s, 1" % (s(S_T2), s(S_T2)),
          "s_bitcmp1_b32 s71, 29",
          "s_cbranch_scc0 .Lfd_loop",
          "s_mul_i32 %s, s68, s69" % s(S_T1),                          # bytes
          "s_add_u32 %s, %s, 63" % (s(S_BYTES), s(S_T1)),
          "s_and_b32 %s, %s, -64" % (s(S_BYTES), s(S_BYTES)),          # dp_delta_off
          "s_add_u32 s66, s66, %s" % s(S_BYTES),
          "s_addc_u32 s67, s67, 0",                                    # the delta area
          "s_and_b32 %s, s71, 0xffff" % s(S_T3),                       # the LDS sums
          "s_bitcmp1_b32 s71, 28",
          "s_cselect_b32 %s, 3, 2" % s(S_CODE),                        # log2 of the word
          "v_lshlrev_b32 %s, %s, %s" % (v(H[2]), s(S_CODE), v(H[1])),  # first byte offset
          "s_lshl_b32 %s, 256, %s" % (s(S_BYTES), s(S_CODE)),          # bytes per round
          ".Lfd_word:",
          "v_cmp_gt_u32_e64 vcc, %s, %s" % (s(S_T1), v(H[2])),
          "s_and_saveexec_b64 %s, vcc" % sp(S_MASK),
          "s_cbranch_execz .Lfd_next",
          "v_add_u32 %s, %s, %s" % (v(H[3]), s(S_T3), v(H[2])),
          "v_mov_b32 %s, 0" % v(R[3]),
          "s_cmp_eq_u32 %s, 3" % s(S_CODE),
          "s_cbranch_scc0 .Lfd_r4",
          "ds_read_b64 %s, %s" % (vp(R[2]), v(H[3])),
          "s_branch .Lfd_r",
          ".Lfd_r4:",
          "ds_read_b32 %s, %s" % (v(R[2]), v(H[3])),
          ".Lfd_r:",
          "s_waitcnt lgkmcnt(0)",
          "v_cmp_ne_u64_e64 vcc, 0, %s" % vp(R[2]),
          "s_and_b64 exec, exec, vcc",
          "s_cbranch_execz .Lfd_next",
          "v_mov_b32 %s, %s" % (v(R[0]), v(H[2])),
          "s_cmp_eq_u32 %s, 3" % s(S_CODE),
          "s_cbranch_scc0 .Lfd_w4",
          "global_atomic_add_x2 %s, %s, s[66:67]" % (v(R[0]), vp(R[2])),
          "s_branch .Lfd_next",
          ".Lfd_w4:",
          "global_atomic_add %s, %s, s[66:67]" % (v(R[0]), v(R[2])),
          ".Lfd_next:",
          "s_mov_b64 exec, %s" % sp(S_MASK),
          "v_add_u32 %s, %s, %s" % (v(H[2]), s(S_BYTES), v(H[2])),
          "v_cmp_gt_u32_e64 vcc, %s, %s" % (s(S_T1), v(H[2])),
          "s_and_b64 vcc, vcc, exec",
          "s_cbranch_scc1 .Lfd_word",
          "s_mov_b64 exec, -1",
          "s_branch .Lfd_loop",
          ".Lfd_done:",
          "s_mov_b64 exec, -1",
          "s_cmp_eq_u64 %s, 0" % sp(S_HIST),
          "s_cbranch_scc1 .Lfin_end",
          ] + lane_index(H[0]) + [
          "s_lshl_b32 %s, %s, 6" % (s(S_T0), s(S_WAVE)),
          "v_add_u32 %s, %s, %s" % (v(H[1]), s(S_T0), v(H[0])),       # bin
          "v_lshlrev_b32 %s, 2, %s" % (v(H[2]), v(H[1])),
          "ds_read_b32 %s, %s" % (v(H[3]), v(H[2])),
          "s_load_dwordx2 %s, s[0:1], 0x68" % sp(S_REC),               # dp_launch.hist_rows
          "s_load_dwordx4 s[68:71], s[0:1], 0x70",     # hist_user, hist_flags, nwg
          "s_waitcnt lgkmcnt(0)",
          "s_cmp_eq_u64 %s, 0" % sp(S_REC),
          "s_cbranch_scc1 .Lfin_atomic",
          "s_and_b32 %s, s2, 7" % s(S_T1),
          "s_mul_i32 %s, %s, %d" % (s(S_T1), s(S_T1), HR),
          "v_lshlrev_b32 %s, 3, %s" % (v(R[0]), v(H[1])),
          "v_add_u32 %s, %s, %s" % (v(R[0]), s(S_T1), v(R[0])),
          "v_mov_b32 %s, %s" % (v(R[2]), v(H[3])),
          "v_mov_b32 %s, 0" % v(R[3]),
          "v_cmp_ne_u32_e64 vcc, 0, %s" % v(H[3]),
          "s_and_saveexec_b64 %s, vcc" % sp(S_SAVE),
          "s_cbranch_execz .Lfin_noadd",
          "global_atomic_add_x2 %s, %s, %s" % (v(R[0]), vp(R[2]), sp(S_REC)),
          ".Lfin_noadd:",
          "s_mov_b64 exec, -1",
          "s_waitcnt vmcnt(0)",          # this wave's adds (and its fault counts) performed
          "s_barrier",                   # ... and every wave's
          "s_cmp_eq_u32 %s, 0" % s(S_WAVE),
          "s_cbranch_scc0 .Lfin_flag",
          # two-level ticket (one hot word would serialise every workgroup's arrival): the
          # workgroups of replica r = wg & 7 count on ticket r; the last of them (its add
          # returns n_r - 1, n_r = (nwg - 1 - r) / 8 + 1) re-arms ticket r and counts on the
          # top ticket, whose last arrival (min(nwg, 8) - 1) is the launch's last workgroup
          "s_mov_b64 exec, 1",
          "s_and_b32 %s, s2, 7" % s(S_T1),
          "s_lshl_b32 %s, %s, 6" % (s(S_T0), s(S_T1)),
          "s_add_u32 %s, %s, %d" % (s(S_T0), s(S_T0), HIST_TICKET_OFF),
          "v_mov_b32 %s, %s" % (v(R[4]), s(S_T0)),
          "v_mov_b32 %s, 1" % v(R[5]),
          "global_atomic_add %s, %s, %s, %s sc0" % (v(R[6]), v(R[4]), v(R[5]), sp(S_REC)),
          "s_sub_u32 %s, s71, 1" % s(S_T3),
          "s_sub_u32 %s, %s, %s" % (s(S_T3), s(S_T3), s(S_T1)),
          "s_lshr_b32 %s, %s, 3" % (s(S_T3), s(S_T3)),        # n_r - 1
          "s_waitcnt vmcnt(0)",
          "v_readfirstlane_b32 %s, %s" % (s(S_T2), v(R[6])),
          "s_cmp_eq_u32 %s, %s" % (s(S_T2), s(S_T3)),
          "s_cselect_b32 %s, 1, 0" % s(S_T2),
          "s_cbranch_scc0 .Lfin_setflag",
          "v_mov_b32 %s, 0" % v(R[10]),
          "global_atomic_swap %s, %s, %s, %s sc0" % (v(R[8]), v(R[4]), v(R[10]), sp(S_REC)),
          "v_mov_b32 %s, %d" % (v(R[9]), HIST_TICKET_OFF + 64 * HIST_REPLICAS),
          "global_atomic_add %s, %s, %s, %s sc0" % (v(R[6]), v(R[9]), v(R[5]), sp(S_REC)),
          "s_min_u32 %s, s71, %d" % (s(S_T3), HIST_REPLICAS),
          "s_sub_u32 %s, %s, 1" % (s(S_T3), s(S_T3)),
          "s_waitcnt vmcnt(0)",
          "v_readfirstlane_b32 %s, %s" % (s(S_T2), v(R[6])),
          "s_cmp_eq_u32 %s, %s" % (s(S_T2), s(S_T3)),
          "s_cselect_b32 %s, 1, 0" % s(S_T2),
          ".Lfin_setflag:",
          "v_mov_b32 %s, %s" % (v(R[7]), s(S_T2)),
          "v_mov_b32 %s, 0" % v(R[8]),
          # LDS word 0 (bin 0, read by every wave before the barrier above) tells the others
          "ds_write_b32 %s, %s" % (v(R[8]), v(R[7])),
          "s_mov_b64 exec, -1",
          "s_waitcnt lgkmcnt(0)",
          ".Lfin_flag:",
          "s_barrier",
          "v_mov_b32 %s, 0" % v(R[8]),
          "ds_read_b32 %s, %s" % (v(R[7]), v(R[8])),
          "s_waitcnt lgkmcnt(0)",
          "v_readfirstlane_b32 %s, %s" % (s(S_T2), v(R[7])),
          "s_cmp_eq_u32 %s, 0" % s(S_T2),
          "s_cbranch_scc1 .Lfin_end",
          # the last workgroup: wave w moves bins 64w..64w+63 (v0..v15 results, v16..v23
          # addresses, v[24:25] = 0: the eBPF registers and staged packet are dead here)
          "v_lshlrev_b32 %s, 3, %s" % (v(R[0]), v(H[1])),
          "v_mov_b32 v24, 0",
          "v_mov_b32 v25, 0"]
    for r in range(HIST_REPLICAS):
        L += ["v_add_u32 v%d, %d, %s" % (16 + r, r * HR, v(R[0])),
              "global_atomic_swap_x2 v[%d:%d], v%d, v[24:25], %s sc0" % (2 * r, 2 * r + 1, 16 + r,
                                                                       sp(S_REC))]
    L += ["s_waitcnt vmcnt(0)"]
    for r in range(1, HIST_REPLICAS):
        L += ["v_lshl_add_u64 v[0:1], v[%d:%d], 0, v[0:1]" % (2 * r, 2 * r + 1)]
    L += ["s_bitcmp1_b32 s70, 0",                   # hist_flags bit 0: store (overwrite)
          "s_cbranch_scc0 .Lfin_add",
          "global_store_dwordx2 %s, v[0:1], s[68:69]" % v(R[0]),
          "s_branch .Lfin_faults",
          ".Lfin_add:",
          "global_atomic_add_x2 %s, v[0:1], s[68:69]" % v(R[0]),
          ".Lfin_faults:",
          "s_cmp_eq_u32 %s, 0" % s(S_WAVE),
          "s_cbranch_scc0 .Lfin_end",
          "s_mov_b64 exec, 1",                       # bin 256 (replica 0 only) and the ticket
          "v_mov_b32 v16, 2048",
          "global_atomic_swap_x2 v[2:3], v16, v[24:25], %s sc0" % sp(S_REC),
          "v_mov_b32 v17, %d" % (HIST_TICKET_OFF + 64 * HIST_REPLICAS),   # the top ticket
          "global_atomic_swap v18, v17, v24, %s sc0" % sp(S_REC),
          "s_waitcnt vmcnt(0)",
          "s_bitcmp1_b32 s70, 0",
          "s_cbranch_scc0 .Lfin_fadd",
          "global_store_dwordx2 v16, v[2:3], s[68:69]",
          "s_branch .Lfin_end",
          ".Lfin_fadd:",
          "global_atomic_add_x2 v16, v[2:3], s[68:69]",
          "s_branch .Lfin_end",
          # no partial buffer (variant-free fallback used by nothing today): per-bin atomics
          ".Lfin_atomic:",
          "v_cmp_ne_u32_e64 vcc, 0, %s" % v(H[3]),
          "s_and_saveexec_b64 %s, vcc" % sp(S_SAVE),
          "v_lshlrev_b32 %s, 3, %s" % (v(R[0]), v(H[1])),
          "v_mov_b32 %s, %s" % (v(R[2]), v(H[3])),
          "v_mov_b32 %s, 0" % v(R[3]),
          "global_atomic_add_x2 %s, %s, %s" % (v(R[0]), vp(R[2]), sp(S_HIST)),
          ".Lfin_end:",
          "s_waitcnt vmcnt(0)",
          "s_endpgm"]
    return L


def link_kernel():
    """ebpf_asm_link(dp_entry *e, uint32_t n): e[i].handler (= handler id) -> absolute address."""
    return [".globl ebpf_asm_link", ".p2align 8", ".type ebpf_asm_link,@function",
            "ebpf_asm_link:",
            "s_load_dwordx2 s[4:5], s[0:1], 0x0",
            "s_load_dword s6, s[0:1], 0x8",
            "s_getpc_b64 s[8:9]",
            ".Llink_base:",
            "s_add_u32 s10, s8, .Lhandler_table-.Llink_base",
            "s_addc_u32 s11, s9, 0",
            "v_lshl_add_u32 v1, s2, 6, v0",
            "s_waitcnt lgkmcnt(0)",
            "v_cmp_gt_u32_e64 vcc, s6, v1",
            "s_and_b64 exec, exec, vcc",
            "s_cbranch_execz .Llink_end",
            "v_mov_b32 v2, 32",
            "v_mad_u64_u32 v[2:3], s[12:13], v1, v2, s[4:5]",
            "global_load_dword v4, v[2:3], off",
            "s_waitcnt vmcnt(0)",
            "v_mov_b32 v6, 4",
            "v_mad_u64_u32 v[6:7], s[12:13], v4, v6, s[10:11]",
            "global_load_dword v8, v[6:7], off",
            "s_waitcnt vmcnt(0)",
            "v_ashrrev_i32 v9, 31, v8",
            "v_lshl_add_u64 v[10:11], v[8:9], 0, s[8:9]",
            "global_store_dwordx2 v[2:3], v[10:11], off",
            ".Llink_end:",
            "s_waitcnt vmcnt(0)",
            "s_endpgm"]


def kd(name, lds, vgprs, sgprs, kernarg, wgsize):
    return [".rodata", ".p2align 6", ".amdhsa_kernel %s" % name,
            ".amdhsa_group_segment_fixed_size %d" % lds,
            ".amdhsa_private_segment_fixed_size 0",
            ".amdhsa_kernarg_size %d" % kernarg,
            ".amdhsa_user_sgpr_count 2",
            ".amdhsa_user_sgpr_kernarg_segment_ptr 1",
            ".amdhsa_system_sgpr_workgroup_id_x 1",
            ".amdhsa_system_vgpr_workitem_id 0",
            ".amdhsa_next_free_vgpr %d" % vgprs,
            ".amdhsa_next_free_sgpr %d" % sgprs,
            ".amdhsa_accum_offset %d" % vgprs,
            ".amdhsa_reserve_vcc 1",
            ".amdhsa_reserve_xnack_mask 0",
            ".amdhsa_ieee_mode 0",
            ".amdhsa_dx10_clamp 0",
            ".end_amdhsa_kernel", ".text"]


def metadata(kernels):
    out = [".amdgpu_metadata", "---", "amdhsa.kernels:"]
    for name, kernarg, lds, vgprs, sgprs, wg in kernels:
        out += ["  - .args:",
                "      - .offset: 0",
                "        .size: %d" % kernarg,
                "        .value_kind: by_value",
                "    .group_segment_fixed_size: %d" % lds,
                "    .kernarg_segment_align: 8",
                "    .kernarg_segment_size: %d" % kernarg,
                "    .max_flat_workgroup_size: %d" % wg,
                "    .name: %s" % name,
                "    .private_segment_fixed_size: 0",
                "    .sgpr_count: %d" % sgprs,
                "    .symbol: %s.kd" % name,
                "    .vgpr_count: %d" % vgprs,
                "    .wavefront_size: 64"]
    out += ["amdhsa.target: amdgcn-amd-amdhsa--gfx950:xnack-", "amdhsa.version:", "  - 1", "  - 2",
            "...", ".end_amdgpu_metadata"]
    return out


JIT_AREA_BYTES = 512 * 1024
ENTRY_SGPR_RE = None


def entry_reads(lines):
    """6-bit mask of the entry SGPRs s10..s15 a handler body reads (compiled programs set
    exactly those before the copied body)."""
    import re
    global ENTRY_SGPR_RE
    if ENTRY_SGPR_RE is None:
        ENTRY_SGPR_RE = re.compile(r"(?<![\w\[:])s(1[0-5])(?![\w\]])|s\[(1[0-5]):(1[0-5])\]")
    m = 0
    for ln in lines:
        code = ln.split("//")[0]
        for x in ENTRY_SGPR_RE.finditer(code):
            if x.group(1):
                m |= 1 << (int(x.group(1)) - 10)
            else:
                for r in range(int(x.group(2)), int(x.group(3)) + 1):
                    m |= 1 << (r - 10)
    return m


def jit_templates():
    """Glue the host's copy-and-patch compiler stitches between copied handler bodies.  Never
    executed in place.  Literals 0x5eed5eed and branch offsets are patched per use."""
    L = [".p2align 2", "ebpf_jit_templates:"]
    for r in range(10, 16):
        L += [".Ljt_mov_s%d:" % r, "s_mov_b32 s%d, 0x5eed5eed" % r]
    # conditional tail, short form: no lane taken -> fall through (the common uniform case costs
    # two scalar instructions); all taken -> branch; mixed -> park the taken lanes at the taken
    # block (v41 = its code offset), continue with the rest
    L += [".Ljt_cs:",
          "s_and_b64 %s, vcc, exec" % sp(S_MASK),
          "s_cbranch_scc0 .Ljt_cs_end",
          "s_cmp_eq_u64 %s, exec" % sp(S_MASK),
          ".Ljt_cs_br:",
          "s_cbranch_scc1 .Ljt_cs_br",
          "s_mov_b64 %s, exec" % sp(S_SAVE),
          "s_mov_b64 exec, %s" % sp(S_MASK),
          ".Ljt_cs_vt:",
          "v_mov_b32 v%d, 0x5eed5eed" % V_T,
          "s_andn2_b64 exec, %s, %s" % (sp(S_SAVE), sp(S_MASK)),
          ".Ljt_cs_end:"]
    # long form (taken block beyond a 16-bit branch)
    L += [".Ljt_cl:",
          "s_and_b64 %s, vcc, exec" % sp(S_MASK),
          "s_cbranch_scc0 .Ljt_cl_end",
          "s_cmp_eq_u64 %s, exec" % sp(S_MASK),
          "s_cbranch_scc0 .Ljt_cl_skip",
          ".Ljt_cl_lit:",
          "s_add_u32 %s, %s, 0x5eed5eed" % (s(S_JUNK), s(S_CB)),
          "s_addc_u32 %s, %s, 0" % (s(S_JUNK + 1), s(S_CB + 1)),
          "s_setpc_b64 %s" % sp(S_JUNK),
          ".Ljt_cl_skip:",
          "s_mov_b64 %s, exec" % sp(S_SAVE),
          "s_mov_b64 exec, %s" % sp(S_MASK),
          ".Ljt_cl_vt:",
          "v_mov_b32 v%d, 0x5eed5eed" % V_T,
          "s_andn2_b64 exec, %s, %s" % (sp(S_SAVE), sp(S_MASK)),
          ".Ljt_cl_end:"]
    L += [".Ljt_wait:", "s_waitcnt lgkmcnt(0)",
          ".Ljt_br:", "s_branch .Ljt_br",
          ".Ljt_jl:",
          "s_add_u32 %s, %s, 0x5eed5eed" % (s(S_JUNK), s(S_CB)),
          "s_addc_u32 %s, %s, 0" % (s(S_JUNK + 1), s(S_CB + 1)),
          "s_setpc_b64 %s" % sp(S_JUNK),
          ".Ljt_jl_end:"]
    # offsets from .Lcb, read by asm_jit.cpp (order = enum jt_index there)
    names = [".Ljt_mov_s%d" % r for r in range(10, 16)] + [
        ".Ljt_cs", ".Ljt_cs_br", ".Ljt_cs_vt", ".Ljt_cs_end",
        ".Ljt_cl", ".Ljt_cl_lit", ".Ljt_cl_vt", ".Ljt_cl_end",
        ".Ljt_br", ".Ljt_jl", ".Ljt_jl_end", ".Ljt_wait", ".Lr_exit_k", ".Lr_exit", ".Lr_fault",
        ".Lr_hlookup", ".Lgroup_done",
        ".Lr_schedule",
        "ebpf_jit_area"]
    L += [".p2align 2", "ebpf_jit_tmpl:"] + ["  .long %s-.Lcb" % n for n in names]
    L += ["  .long %d" % JIT_AREA_BYTES]
    return L


# The staged image the assembly interpreter (variant 2) launches from (m3): one result group per
# burst (64 VGPRs) and an interpreter kernel that declares only the SGPRs the image's own code
# touches (s0..s73; compiled programs' join masks start at s74), so that 8 workgroups of 256
# lanes fit a CU (MI355X_MICROARCH.md "Residency": .sgpr_count <= 80 -> 8; 98 -> 6).  The
# interpreter is bound by its dependent dispatch chain (s_load -> s_waitcnt -> s_setpc per
# entry) and scales with resident waves (C4: 2 workgroups per CU 3.19 ms ... 6: 1.25 ms).
NSGPR_INTERP = S_JOIN
INTERP_IMAGE = False
RETK_INTERP = int(os.environ.get("EBPF_ASM_RETK_INTERP", "1"))
assert RETK_INTERP in (1, 2, 4, 8)


def main():
    """gen_interp.py <staged.s> <general.s> <staged-interpreter.s> <handlers.h>"""
    out_s1, out_s0, out_s3, out_h = sys.argv[1:5]
    header = None
    global NVGPR, INTERP_IMAGE
    for out_s, k, staged, interp in ((out_s1, RETK_STAGED, True, False),
                                     (out_s0, 1, False, False),
                                     (out_s3, RETK_INTERP, True, True)):
        set_retk(k)
        INTERP_IMAGE = interp
        if not staged:
            NVGPR += GEN_HOIST_REGS
        h = generate(out_s, staged)
        header = header or h
        assert h[:-2] == header[:-2]   # identical but for the RETK-dependent lines
    header = header[:-2] + ["#define AH_RET_GROUPS_STAGED %d  // groups per result burst, staged kernels"
                            % RETK_STAGED,
                            "#define AH_NVGPR_STAGED %d" % (64 if RETK_STAGED == 1 else 64 + 2 * RETK_STAGED),
                            "#define AH_RET_GROUPS_GENERAL 1",
                            "#define AH_NVGPR_STAGED_WIDE %d  // ebpf_jit_s64w: 16 result slots "
                            "(write phasing), 0 = none" % (96 if RETK_STAGED == 8 else 0),
                            "#define AH_NVGPR_GENERAL %d" % (64 + GEN_HOIST_REGS),
                            "#define AH_NVGPR_INTERP %d  // the interpreter's staged image (m3)"
                            % (64 if RETK_INTERP == 1 else 64 + 2 * RETK_INTERP),
                            "#define AH_RET_GROUPS_INTERP %d" % RETK_INTERP]
    with open(out_h, "w") as f:
        f.write("\n".join(header) + "\n")


def generate(out_s, staged_image):
    global STAGED_IMAGE
    STAGED_IMAGE = staged_image
    A = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950:xnack-"', ".amdhsa_code_object_version 5", ".text"]
    A += kernel("ebpf_interp_s64", True) + kernel("ebpf_interp_gen", False)
    A += kernel("ebpf_jit_s64", True, True) + kernel("ebpf_jit_gen", False, True)
    A += common_group_code() + routines()
    table = []
    meta = []
    reads = []
    conds = []
    hid = 0
    header = ["// generated by gen_interp.py — handler family ids for asm_runtime.cpp",
              "#pragma once", "#include <stdint.h>", "#define AH_NREGS %d" % NREG]
    fam_of, dst_of, src_of = [], [], []
    for fi, (name, arity) in enumerate(FAMILIES):
        header.append("#define AH_%s %d" % (name, hid))
        header.append("#define AHF_%s %d" % (name, fi))
        for d, sr in variants(arity):
            fam_of.append(fi)
            dst_of.append(255 if d is None else d)
            src_of.append(255 if sr is None else sr)
            label = "h_%d" % hid
            uid = "%d" % hid
            body, own = handler_body(name, d, sr)
            body = [ln.replace("{uid}", uid) for ln in body]
            A.append(".p2align 2")
            A.append("%s:" % label)
            is_cond = "@CMPEND" in body
            if is_cond:
                k = body.index("@CMPEND")
                copy = body[:k]
                A += copy + [".Lhe_%d:" % hid] + body[k + 1:]
            else:
                copy = body
                k = early_fetch_point(body) if (INTERP_IMAGE and not own) else None
                if k is not None and k < len(body):
                    # (this image never feeds the code generator, which copies label..Lhe_)
                    d = dispatch(12)
                    A += body[:k] + [d[0]] + body[k:] + [".Lhe_%d:" % hid] + d[1:]
                else:
                    A += body + [".Lhe_%d:" % hid]
                    if not own:
                        A += dispatch(12)
            m = entry_reads(copy)
            if name == "LOOKUPGEN":
                m |= 1 << 2      # the routine resumes at s12
            if name == "HLOOKUP":
                m |= 1 << 4      # the routine reads the map record offset from s14
            if name in ("UPDATE", "HDELETE"):
                m |= (1 << 4) | (1 << 5)   # map record offset (s14), entry index (s15)
            reads.append(m)
            # an LDS read whose result the interpreter's dispatch wait (lgkmcnt) covered
            last_ds = max([i for i, ln in enumerate(copy) if ln.startswith("ds_read")] or [-1])
            waits = [i for i, ln in enumerate(copy) if ln.startswith("s_waitcnt") and "lgkmcnt" in ln]
            needw = last_ds >= 0 and not any(i > last_ds for i in waits)
            conds.append((1 if is_cond else 0) | (2 if needw else 0))
            table.append(label)
            meta.append("  .long %s-.Lcb, .Lhe_%d-%s" % (label, hid, label))
            hid += 1
    header.append("#define AH_COUNT %d" % hid)
    header.append("// entry SGPRs (bit k = s(10+k)) each handler body reads")
    header.append("static const uint8_t ah_reads[AH_COUNT] = {%s};" % ",".join(map(str, reads)))
    header.append("// bit 0: conditional jump (copy the compare only); bit 1: body leaves an LDS read "
                  "outstanding")
    header.append("static const uint8_t ah_flags[AH_COUNT] = {%s};" % ",".join(map(str, conds)))
    header.append("// per handler: family (AHF_*), dst register, src register (LDXPKC: packet byte offset);")
    header.append("// 255 = none.  Read by the optimising code generator (asm_cc.cpp)")
    header.append("static const uint8_t ah_fam[AH_COUNT] = {%s};" % ",".join(map(str, fam_of)))
    header.append("static const uint8_t ah_dst[AH_COUNT] = {%s};" % ",".join(map(str, dst_of)))
    header.append("static const uint8_t ah_src[AH_COUNT] = {%s};" % ",".join(map(str, src_of)))
    header.append("#define AH_JIT_AREA_BYTES %d" % JIT_AREA_BYTES)
    header.append("#define AH_S_JOIN %d  // structured programs: taken-lane masks s[74:75]..  (staged image)" % S_JOIN)
    header.append("#define AH_JOIN_LEVELS %d" % JOIN_LEVELS)
    header.append("#define AH_GEN_JOIN %d  // the general image holds the join SGPRs too" % GEN_JOIN)
    header.append("#define AH_GEN_HOIST_BASE 64  // general image: spare VGPRs for hoisted loads")
    header.append("#define AH_GEN_HOIST_REGS %d" % GEN_HOIST_REGS)
    header.append("#define AH_S_RUNMASK %d  // general image: s[76:77], a hoisted-load run's lanes" % S_RUNMASK)
    header.append("#define AH_V_IDX %d  // general image: the lane's packet index" % V_IDX)
    header.append("#define AH_RET_GROUPS %d" % RETK)
    header.append("#define AH_NVGPR %d" % NVGPR)
    A += link_kernel()
    A += [".p2align 2", ".Lhandler_table:"]
    A += ["  .long %s-.Llink_base" % lab for lab in table]
    # compiled-program support: handler body table, glue templates, the patch area
    A += [".p2align 2", "ebpf_jit_meta:"] + meta
    A += jit_templates()
    A += [".p2align 8", "ebpf_jit_area:", "  .fill %d, 4, 0xbf810000" % (JIT_AREA_BYTES // 4)]
    # every VGPR the image's code names lies inside the kernels' allocation (a register past it
    # assembles but reads whatever the hardware holds there)
    vtop = 0
    for ln in A:
        code = ln.split(";")[0].split("//")[0]
        for a, b, c in re.findall(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]", code):
            vtop = max(vtop, int(a or c))
    vwide = V_RB + 2 * SLOTS if (staged_image and SLOTS == 16) else NVGPR
    assert vtop < max(NVGPR, vwide), "image code uses v%d, the kernels allocate %d VGPRs" % (
        vtop, max(NVGPR, vwide))
    kernarg = 232
    nsg = NSGPR_STAGED if (staged_image or GEN_JOIN) else NSGPR_GEN
    if INTERP_IMAGE:
        # the interpreter kernel declares s0..s73 only: check that the image's code uses no more
        top = 0
        for ln in A:
            for a, b, c in re.findall(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]", ln.split(";")[0].split("//")[0]):
                top = max(top, int(a or c))
        assert top < NSGPR_INTERP, "interpreter image uses s%d" % top
    ks = [("ebpf_interp_s64", kernarg, 0, NVGPR, NSGPR_INTERP if INTERP_IMAGE else nsg, 256),
          ("ebpf_interp_gen", kernarg, 0, NVGPR, nsg, 256),
          ("ebpf_jit_s64", kernarg, 0, NVGPR, nsg, 256),
          ("ebpf_jit_gen", kernarg, 0, NVGPR, nsg, 256),
          ("ebpf_asm_link", 16, 0, 16, 16, 64)]
    if vwide > NVGPR:
        ks.append(("ebpf_jit_s64w", kernarg, 0, vwide, nsg, 256))
    for name, ka, lds, vg, sg, wg in ks:
        A += kd(name, lds, vg, sg, ka, wg)
    md = metadata(ks)
    with open(out_s, "w") as f:
        f.write("\n".join(("\t" + x if not (x.endswith(":") or x.startswith(".") or x.startswith(" ")) else x)
                          for x in A) + "\n")
        f.write("\n".join(md) + "\n")
    return header


if __name__ == "__main__":
    main()
