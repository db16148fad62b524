// asm_cc.cpp — optimising gfx950 code generation for compiled programs (variant 0).
//
// asm_jit.cpp lays a lowered program (asm_lower) out as straight-line code; for each entry it
// can copy the interpreter's handler body verbatim.  Handler bodies are written for any register
// contents, so they pay for 64-bit generality everywhere: a 32-bit result re-zeroes its high
// half, a 64-bit multiply by a 32-bit constant multiplies by a zero high word, a compare of a
// loaded byte is a 64-bit compare against an SGPR pair set by two scalar moves, a map lookup
// re-reads its key from the stack and re-checks the result's range at every use.
//
// Here two forward passes and one backward pass over the state tree (the translator gives every
// entry one predecessor, so facts are exact per path) compile the hot families to hand-encoded
// gfx950 instructions instead:
//   facts (forward): per eBPF register, a known constant, the number of known leading zero bits,
//     non-NULL-ness, and for a map lookup result the map and the register holding its index;
//     per stack word, the register whose low bytes it holds (store-to-load forwarding);
//     compares against constants refine the facts on their taken / fall-through edges;
//   liveness (backward): pure operations (ALU, byte swaps, staged packet and stack loads,
//     lookups with a statically resolved map) whose result no path reads emit nothing, and the
//     group's register zeroing covers only the registers the program reads before writing;
//   emission (forward):
//   * constants fold (both operands known: a move of the result);
//   * high halves known zero are neither recomputed nor re-zeroed;
//   * 64-bit AND/OR/XOR/shift by constants become 32-bit operations where a half is unchanged
//     or zero, shifts by >= 32 become moves;
//   * MUL by a constant drops the partial products of known-zero words, multiplies by powers
//     of two become shifts;
//   * compares of values below 2^32 against constants below 2^32 are single VOPC e32
//     instructions with the constant as a literal; statically decided compares (including
//     NULL checks of lookups that cannot fail) become VCC = EXEC or 0;
//   * a staged packet load followed by BE16/BE32 of the same register is one v_perm_b32 that
//     picks the bytes in network order straight from the staged packet registers;
//   * stack stores/loads at known offsets are single LDS instructions with the offset folded in;
//     a load of a word stored from a register that is unchanged since reads the register;
//   * an array-map lookup whose key comes from a register proven below max_entries cannot
//     return NULL: r0 = base + key * value_size (one v_mad_u64_u32, or nothing if r0 is only
//     dereferenced), and loads through it read the workgroup's LDS copy of the map at
//     lds_off + key * value_size + off with no range check.
// Everything else (memory through unknown pointers, generic lookups, division, generic exits,
// faults) still copies the interpreter's handler body, so semantics there are unchanged.
//
// Encodings: VOP1/VOP2/VOPC (e32, literal allowed in src0), VOP3 (no literal on gfx9), SOP1,
// SOP2, DS.  Field layouts and opcodes are from llvm-mc -show-encoding for gfx950;
// tests/test_compile.py checks decoded forms.
#include <algorithm>

#include "asm_handlers.h"
#include "internal.h"

#include "asm_cc.h"

namespace {

// ---------------------------------------------------------------- encoder
enum : uint32_t {
	SRC_VCC = 106, SRC_EXEC = 126, SRC_LIT = 255, VGPR0 = 256,
};
// VOP2 opcodes (bits 30:25)
enum : uint32_t {
	V2_LSHRREV_B32 = 0x10, V2_LSHLREV_B32 = 0x12, V2_AND = 0x13, V2_OR = 0x14, V2_XOR = 0x15,
	V2_ADD_U32 = 0x34, V2_SUB_U32 = 0x35, V2_SUBREV_U32 = 0x36, V2_SUB_CO_U32 = 0x1a,
	V2_SUBB_CO_U32 = 0x1d,
};
// VOP1 opcodes (bits 16:9)
enum : uint32_t { V1_MOV_B32 = 0x01, V1_MOV_B64 = 0x38 };
// VOP3 opcodes (bits 25:16)
enum : uint32_t {
	V3_MAD_U32_U24 = 0x1c3, V3_BFE_U32 = 0x1c8, V3_ALIGNBYTE = 0x1cf, V3_MAD_U64_U32 = 0x1e8,
	V3_PERM_B32 = 0x1ed, V3_ADD3_U32 = 0x1ff, V3_LSHL_ADD_U64 = 0x208, V3_MUL_LO_U32 = 0x285,
	V3_LSHLREV_B64 = 0x28f, V3_LSHRREV_B64 = 0x290, V3_LSHL_ADD_U32 = 0x1fd,
};
// DS opcodes (bits 24:17)
enum : uint32_t {
	DS_WRITE_B32 = 0x0d, DS_WRITE2_B32 = 0x0e, DS_WRITE_B8 = 0x1e, DS_WRITE_B16 = 0x1f,
	DS_READ_B32 = 0x36, DS_READ2_B32 = 0x37, DS_READ_U8 = 0x3a, DS_READ_U16 = 0x3c,
};
// VOPC compare codes: base + {lt 1, eq 2, le 3, gt 4, ne 5, ge 6}
enum : uint32_t { VC_I32 = 0xc0, VC_U32 = 0xc8, VC_I64 = 0xe0, VC_U64 = 0xe8 };
enum { P_LT = 1, P_EQ = 2, P_LE = 3, P_GT = 4, P_NE = 5, P_GE = 6 };
const uint32_t S_WAITCNT_LGKM0 = 0xbf8cc07fu;
const int S_JUNK = 60; // s[60:61]: carry-out sink of v_mad_u64_u32 (gen_interp.py S_JUNK)
const int S_BYTES = 57, S_CB = 4;              // gen_interp.py S_BYTES, S_CB
const int T0 = 46, T1 = 47, T2 = 48, T3 = 49;  // handler temporaries (gen_interp.py H)
const int PKT0 = 22;                           // staged packet dwords v22..v37
const int V_STK = 42;                          // lane stack bottom (LDS byte address)
const int V_RES = 44;                          // v[44:45]: r0 of retiring lanes
const int V_SEL = 63;                          // v63 = 0x00010203 (byte reversal selector)

struct opnd {
	uint32_t code;
	uint32_t lit = 0;
};

bool
inline_i64(int64_t v, uint32_t *code)
{
	if (v >= 0 && v <= 64) {
		*code = 128 + (uint32_t)v;
		return true;
	}
	if (v >= -16 && v <= -1) {
		*code = 192 + (uint32_t)(-v);
		return true;
	}
	return false;
}

opnd
vreg(int n)
{
	return opnd{VGPR0 + (uint32_t)n};
}

// 32-bit constant for an e32 src0 / SOP source: inline constant or literal
opnd
k32(uint32_t v)
{
	uint32_t c;
	if (inline_i64((int64_t)(int32_t)v, &c))
		return opnd{c};
	return opnd{SRC_LIT, v};
}

// gfx9 (gfx950 included) VOP3 reads at most one SGPR (or VCC / EXEC / M0) through the constant
// bus; a second one reads garbage and no assembler stands between this encoder and the hardware.
// Every VOP3 the compiler emits is checked (cc_bus_violations, asm_jit_emit fails the build).
thread_local unsigned g_bus_violations = 0;

bool
is_sgpr_src(uint32_t c)
{
	return c <= 127 || (c >= 251 && c <= 253);
}

struct enc {
	std::vector<uint8_t> &b;
	void w(uint32_t x)
	{
		for (int i = 0; i < 4; i++)
			b.push_back((uint8_t)(x >> (8 * i)));
	}
	void lit(const opnd &s)
	{
		if (s.code == SRC_LIT)
			w(s.lit);
	}
	void vop2(uint32_t op, int vdst, opnd s0, int vsrc1)
	{
		w((op << 25) | ((uint32_t)vdst << 17) | ((uint32_t)vsrc1 << 9) | s0.code);
		lit(s0);
	}
	void vop1(uint32_t op, int vdst, opnd s0)
	{
		w((0x3fu << 25) | ((uint32_t)vdst << 17) | (op << 9) | s0.code);
		lit(s0);
	}
	void vopc(uint32_t op, opnd s0, int vsrc1)
	{
		w((0x3eu << 25) | (op << 17) | ((uint32_t)vsrc1 << 9) | s0.code);
		lit(s0);
	}
	// VOP3 (a and b forms); sources are 9-bit codes, never a literal on gfx9
	void vop3(uint32_t op, int vdst, uint32_t s0, uint32_t s1, uint32_t s2, int sdst = 0)
	{
		const uint32_t src[3] = {s0, s1, s2};
		// (two-source encodings: the compares, v_mul_lo_u32, the 64-bit shifts ignore src2)
		const int nsrc = (op < 0x100 || op == V3_MUL_LO_U32 || op == V3_LSHLREV_B64 ||
				  op == V3_LSHRREV_B64) ? 2 : 3;
		uint32_t bus = UINT32_MAX;
		for (int i = 0; i < nsrc; i++) {
			const uint32_t x = src[i];
			if (!is_sgpr_src(x) || x == bus)
				continue;
			if (bus != UINT32_MAX) {
				g_bus_violations++;
				if (getenv("EBPF_CC_BUS_DEBUG"))
					fprintf(stderr, "VOP3 op %#x reads SGPRs %u and %u\n", op, bus, x);
			}
			bus = x;
		}
		w((0x34u << 26) | (op << 16) | ((uint32_t)sdst << 8) | (uint32_t)vdst);
		w(s0 | (s1 << 9) | (s2 << 18));
	}
	void ds(uint32_t op, int addr, int data0, int data1, int vdst, uint32_t off0, uint32_t off1 = 0)
	{
		w((0x36u << 26) | (op << 17) | (off1 << 8) | off0);
		w((uint32_t)addr | ((uint32_t)data0 << 8) | ((uint32_t)data1 << 16) | ((uint32_t)vdst << 24));
	}
	void sop1(uint32_t op, int sdst, opnd s0)
	{
		w(0xbe800000u | ((uint32_t)sdst << 16) | (op << 8) | s0.code);
		lit(s0);
	}
	void sop2(uint32_t op, int sdst, opnd s0, opnd s1)
	{
		w(0x80000000u | (op << 23) | ((uint32_t)sdst << 16) | (s1.code << 8) | s0.code);
		lit(s0);
		lit(s1);
	}
	void wait_lgkm() { w(S_WAITCNT_LGKM0); }
};

// ---------------------------------------------------------------- facts
struct rf {
	bool c = false;   // known constant
	uint64_t v = 0;
	uint8_t lz = 0;   // known leading zero bits (64 if c && v == 0)
	bool nz = false;  // known non-zero (a lookup that cannot fail)
	int8_t mp = -1;   // >= 0: a pointer to map mp's value number u32(r[mreg]) (+0)
	int8_t mreg = -1;
	int8_t hfwd = -1; // >= 0: a hashtable lookup result whose value's first 8 bytes register
	                  // hfwd's VGPRs hold (loaded with the probe, see AHF_HLOOKUP)
};

inline int
clz64(uint64_t x)
{
	return x ? __builtin_clzll(x) : 64;
}

inline rf
kconst(uint64_t v)
{
	rf r;
	r.c = true;
	r.v = v;
	r.lz = (uint8_t)clz64(v);
	r.nz = v != 0;
	return r;
}

inline rf
kbits(int bits)
{
	rf r;
	r.lz = (uint8_t)(bits <= 0 ? 64 : bits >= 64 ? 0 : 64 - bits);
	return r;
}

inline int
bits_of(const rf &r)
{
	return 64 - r.lz;
}

// a stack word whose bytes are the low `size` bytes of register `reg` (unchanged since)
struct sslot {
	uint32_t off; // LDS offset from the lane's stack bottom (the lowered operand)
	uint8_t size;
	int8_t reg;
};

struct facts {
	rf r[AH_NREGS];
	bool pv[AH_NREGS] = {}; // the register's VGPRs hold its value (false: a dead write skipped)
	sslot st[8];
	uint8_t nst = 0;

	void def(int d, const rf &v, bool phys = true)
	{
		r[d] = v;
		pv[d] = phys;
		uint8_t k = 0;
		for (uint8_t i = 0; i < nst; i++)
			if (st[i].reg != d)
				st[k++] = st[i];
		nst = k;
		for (int q = 0; q < AH_NREGS; q++) {
			if (q != d && r[q].mreg == d) {
				r[q].mp = -1;
				r[q].mreg = -1;
			}
			if (r[q].hfwd == d)
				r[q].hfwd = -1;
		}
	}
	// d's VGPRs are overwritten with something else while its value facts stay true (a register
	// dead from here on, reused as a scratch): nothing may read those VGPRs for d any more
	void clobber_phys(int d)
	{
		pv[d] = false;
		uint8_t k = 0;
		for (uint8_t i = 0; i < nst; i++)
			if (st[i].reg != d)
				st[k++] = st[i];
		nst = k;
		for (int q = 0; q < AH_NREGS; q++) {
			if (r[q].mreg == d) {
				r[q].mp = -1;
				r[q].mreg = -1;
			}
			if (r[q].hfwd == d)
				r[q].hfwd = -1;
		}
	}
	void store(uint32_t off, int size, int reg)
	{
		uint8_t k = 0;
		for (uint8_t i = 0; i < nst; i++)
			if (st[i].off + st[i].size <= off || off + (uint32_t)size <= st[i].off)
				st[k++] = st[i];
		nst = k;
		if (reg >= 0 && nst < 8)
			st[nst++] = sslot{off, (uint8_t)size, (int8_t)reg};
	}
	bool nofwd = false;
	bool t2zero = false; // v48 (T2) holds 0 in this path's lanes (the multiply addend's low word)
	const sslot *slot(uint32_t off, int size) const
	{
		if (nofwd)
			return nullptr;
		for (uint8_t i = 0; i < nst; i++)
			if (st[i].off == off && st[i].size >= size)
				return &st[i];
		return nullptr;
	}
};

// EBPF_CC_OFF (debugging / A-B): bit 0 no dead-code removal, 1 zero every register at the start,
// 2 no stack forwarding, 3 no lookup specialisation, 4 no static branches, 5 no known-r0 exits
unsigned
cc_off()
{
	const char *e = getenv("EBPF_CC_OFF");
	return e ? (unsigned)strtoul(e, nullptr, 0) : 0u;
}

struct mapinfo {
	uint64_t dev_base;
	uint32_t value_size, max_entries, lds_off;
};

// ---------------------------------------------------------------- per-entry emission
struct emitter {
	cc_block &blk;
	enc E;
	facts &f;
	const std::vector<mapinfo> &maps;
	uint16_t used = 0; // registers this entry's code reads

	emitter(cc_block &b, facts &fa, const std::vector<mapinfo> &m) : blk(b), E{b.body}, f(fa), maps(m) {}

	static int L(int r) { return 2 * r; }
	static int Hi(int r) { return 2 * r + 1; }
	bool hz(int r) const { return f.r[r].lz >= 32; }
	void use(int r) { used |= (uint16_t)(1u << r); }

	// LDXPKTV in the staged kernels: d = the z bytes at r_sr + K of the lane's packet.
	// * every running lane at the same offset (a cursor advanced by constants: C3L's header
	//   words): from the packet dwords v22..v37 the staging left in registers, indexed by the
	//   offset's dword (s_set_gpr_idx_on, M0) and aligned by its low bits — no memory access;
	// * otherwise, in keep mode (s7 bit 14: gpu_runtime.cpp sets it for staged launches of
	//   programs with these loads), from the wave's transposed LDS packet buffer (gen_interp.py
	//   lds_pkt_read) when every running lane's bytes lie in its 64;
	// * else the interpreter's handler body h (generic load, faults), spliced in by the code
	//   generator.
	// (The handler's own fast path re-derives the address from s[10:11] and tests the keep flag
	// first: here r_sr is read directly and K folds into the bounds.)
	void ldxpktv_staged(int d, int sr, int z, uint32_t K, int h)
	{
		const int V_PKT = 38, V_L16 = 43, S_PKTLDS = 47, S_U = 60, S_M = 48;
		const int A = 50, B = 51, R0 = 52, R1 = 53, R2 = 54; // (gen_interp.py H[4], H[5], R[0..2])
		const uint32_t C = 64u - (uint32_t)z - K;            // last in-bounds offset T
		use(sr);
		auto sopc = [&](uint32_t op, uint32_t s0, uint32_t s1) {
			E.w(0xbf000000u | (op << 16) | (s1 << 8) | s0);
		};
		auto fwd = [&](uint32_t opw) { // a forward branch, patched by `to`
			const size_t at = E.b.size();
			E.w(opw);
			return at;
		};
		auto to = [&](size_t at) { // point the branch at `at` to here
			const uint32_t skip = (uint32_t)((E.b.size() - at - 4) / 4);
			E.b[at] = (uint8_t)skip;
			E.b[at + 1] = (uint8_t)(skip >> 8);
		};
		const uint32_t SCC0 = 0xbf840000u, SCC1 = 0xbf850000u, BR = 0xbf820000u;
		E.vop2(V2_SUB_CO_U32, T2, vreg(L(sr)), V_PKT);               // T = r - pkt (64-bit)
		E.vop2(V2_SUBB_CO_U32, T3, vreg(Hi(sr)), V_PKT + 1);
		E.vop1(0x02, S_U, vreg(T2));                                 // v_readfirstlane_b32
		E.vop1(0x02, S_U + 1, vreg(T3));
		E.vopc(VC_U64 + P_EQ, opnd{(uint32_t)S_U}, T2);              // vcc = T == T(first lane)
		E.sop2(0x13, S_M, opnd{SRC_EXEC}, opnd{SRC_VCC});            // s_andn2_b64: lanes differ
		const size_t to_lds = fwd(SCC1);
		sopc(0x07, S_U + 1, 128);                                    // s_cmp_lg_u32 hi, 0
		const size_t slow0 = fwd(SCC1);
		sopc(0x08, S_U, 128 + C);                                    // s_cmp_gt_u32 lo, C
		const size_t slow1 = fwd(SCC1);
		if (K)
			E.sop2(0x00, S_U, opnd{(uint32_t)S_U}, opnd{128 + K});  // s_add_u32
		E.sop2(0x1e, S_U + 1, opnd{(uint32_t)S_U}, opnd{128 + 2});  // s_lshr_b32: dword index
		// (VOP3 sources are indexed too: profiles/r05/c3l_pktv/)
		sopc(0x11, S_U + 1, 3);                                      // s_set_gpr_idx_on (SRC0, SRC1)
		E.vop3(V3_ALIGNBYTE, L(d), VGPR0 + PKT0 + 1, VGPR0 + PKT0, (uint32_t)S_U);
		if (z == 8)
			E.vop3(V3_ALIGNBYTE, Hi(d), VGPR0 + PKT0 + 2, VGPR0 + PKT0 + 1, (uint32_t)S_U);
		E.w(0xbf9c0000u);                                            // s_set_gpr_idx_off
		if (z < 4)
			E.vop2(V2_AND, L(d), k32(z == 1 ? 0xffu : 0xffffu), L(d));
		if (z < 8)
			hi0(d);
		const size_t done0 = fwd(BR);                                // (patched past the splice)
		to(to_lds);
		sopc(0x0d, 7, 128 + 14);                                     // s_bitcmp1_b32 s7, 14
		const size_t slow2 = fwd(SCC0);                              // no keep mode: the handler
		E.vopc(VC_U64 + P_GE, k32(C), T2);                           // vcc = T <= C
		E.sop2(0x13, S_JUNK, opnd{SRC_EXEC}, opnd{SRC_VCC});        // s_andn2_b64: lanes out
		const size_t slow3 = fwd(SCC1);
		E.vop2(V2_LSHRREV_B32, A, opnd{128 + 2}, V_L16);             // A = S_PKTLDS + 4 lane
		E.vop2(V2_ADD_U32, A, opnd{(uint32_t)S_PKTLDS}, A);
		if (K)
			E.vop2(V2_ADD_U32, T2, k32(K), T2);                  // T += K (<= 64 - z)
		E.vop2(V2_LSHRREV_B32, B, opnd{128 + 2}, T2);                // B = A + 256 (T >> 2)
		E.vop3(V3_LSHL_ADD_U32, B, VGPR0 + B, 128 + 8, VGPR0 + A);
		if (z == 1)
			E.ds(DS_READ_B32, B, 0, 0, R0, 0);
		else
			E.ds(DS_READ2_B32, B, 0, 0, R0, 0, 64);
		if (z == 8)
			E.ds(DS_READ_B32, B, 0, 0, R2, 0x200 & 0xff, 0x200 >> 8);
		E.wait_lgkm();
		E.vop3(V3_ALIGNBYTE, L(d), VGPR0 + (z == 1 ? R0 : R1), VGPR0 + R0, VGPR0 + T2);
		if (z == 8) {
			E.vop3(V3_ALIGNBYTE, Hi(d), VGPR0 + R2, VGPR0 + R1, VGPR0 + T2);
			f.def(d, rf());
		} else {
			if (z < 4)
				E.vop2(V2_AND, L(d), k32(z == 1 ? 0xffu : 0xffffu), L(d));
			hi0(d);
			f.def(d, kbits(8 * z));
		}
		const size_t done1 = fwd(BR);                                // (patched past the splice)
		// the slow branches, and both done branches, to the body's end: the splice starts there,
		// and the code generator moves the done branches past it
		for (size_t at : {slow0, slow1, slow2, slow3, done0, done1})
			to(at);
		blk.splice_h = h;
		blk.splice_at = (uint32_t)E.b.size();
		blk.splice_br[0] = (uint32_t)done0;
		blk.splice_br[1] = (uint32_t)done1;
		blk.splice_sval[0] = K;
		blk.splice_sval[1] = 0;
		f.t2zero = false;
	}
	// an SGPR holding the 32-bit constant v for this body (s13, s14, s15)
	uint32_t sconst(uint32_t v)
	{
		static const int regs[3] = {13, 14, 15};
		for (int r : regs)
			if ((blk.reads & (1u << (r - 10))) && blk.sval[r - 10] == v)
				return (uint32_t)r;
		for (int r : regs)
			if (!(blk.reads & (1u << (r - 10)))) {
				blk.reads |= (uint8_t)(1u << (r - 10));
				blk.sval[r - 10] = v;
				return (uint32_t)r;
			}
		return UINT32_MAX; // never: no body needs four constants
	}
	// the SGPR pair s[10:11] holding the 64-bit constant v
	uint32_t spair(uint64_t v)
	{
		blk.reads |= 3;
		blk.sval[0] = (uint32_t)v;
		blk.sval[1] = (uint32_t)(v >> 32);
		return 10;
	}
	uint32_t c3(uint32_t v)
	{
		uint32_t c;
		if (inline_i64((int64_t)(int32_t)v, &c))
			return c;
		return sconst(v);
	}
	// a 32-bit constant as a VOP3 source that does not use the constant bus: an inline
	// constant, or the literal moved into VGPR `tmp` first (for an instruction that already reads
	// an SGPR)
	uint32_t vconst(uint32_t v, int tmp)
	{
		uint32_t c;
		if (inline_i64((int64_t)(int32_t)v, &c))
			return c;
		mov32(tmp, v);
		return VGPR0 + (uint32_t)tmp;
	}
	uint32_t c64(uint64_t v)
	{
		uint32_t c;
		if (inline_i64((int64_t)v, &c))
			return c;
		return spair(v);
	}

	void mov32(int vd, uint32_t v) { E.vop1(V1_MOV_B32, vd, k32(v)); }
	// hi(d) = 0 after a write of lo(d) (d's previous value read or not)
	void hi0(int d)
	{
		if (!(f.pv[d] && hz(d)))
			mov32(Hi(d), 0);
	}
	// d = v (a constant), skipping halves the registers already hold
	void mov64(int d, uint64_t v)
	{
		const rf &o = f.r[d];
		const bool pv = f.pv[d];
		const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
		if (!(pv && o.c && (uint32_t)o.v == lo))
			mov32(L(d), lo);
		if (!(pv && ((o.c && (uint32_t)(o.v >> 32) == hi) || (hi == 0 && hz(d)))))
			mov32(Hi(d), hi);
		f.def(d, kconst(v));
	}
	// d = s (registers)
	void copy64(int d, int s)
	{
		if (d == s) {
			use(s);
			return;
		}
		if (f.r[s].c) {
			mov64(d, f.r[s].v);
			return;
		}
		use(s);
		if (hz(s)) {
			E.vop1(V1_MOV_B32, L(d), vreg(L(s)));
			hi0(d);
		} else {
			E.vop1(V1_MOV_B64, L(d), vreg(L(s)));
		}
		rf v = f.r[s];
		v.mp = -1; // (keep it simple: provenance stays with the original)
		v.mreg = -1;
		f.def(d, v);
	}

	// ---- ALU64 with a constant operand (d op= K)
	void add64i(int d, uint64_t K)
	{
		const rf x = f.r[d];
		if (K == 0) {
			use(d); // (a no-op passes d's value through)
			return;
		}
		if (x.c) {
			mov64(d, x.v + K);
			return;
		}
		use(d);
		E.vop3(V3_LSHL_ADD_U64, L(d), c64(K), 128, VGPR0 + L(d));
		f.def(d, (int64_t)K >= 0 ? kbits(std::max(bits_of(x), 64 - clz64(K)) + 1) : rf());
	}
	void or64i(int d, uint64_t K)
	{
		const rf x = f.r[d];
		if (x.c) {
			mov64(d, x.v | K);
			return;
		}
		if (K == 0) {
			use(d);
			return;
		}
		use(d);
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo)
			E.vop2(V2_OR, L(d), k32(lo), L(d));
		if (hi == 0xffffffffu)
			mov32(Hi(d), hi);
		else if (hi)
			E.vop2(V2_OR, Hi(d), k32(hi), Hi(d));
		rf v = kbits(std::max(bits_of(x), 64 - clz64(K)));
		v.nz = true;
		f.def(d, v);
	}
	void xor64i(int d, uint64_t K)
	{
		const rf x = f.r[d];
		if (x.c) {
			mov64(d, x.v ^ K);
			return;
		}
		if (K == 0) {
			use(d);
			return;
		}
		use(d);
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo)
			E.vop2(V2_XOR, L(d), k32(lo), L(d));
		if (hi)
			E.vop2(V2_XOR, Hi(d), k32(hi), Hi(d));
		f.def(d, kbits(std::max(bits_of(x), 64 - clz64(K))));
	}
	void and64i(int d, uint64_t K)
	{
		const rf x = f.r[d];
		if (x.c) {
			mov64(d, x.v & K);
			return;
		}
		if (K == ~0ull) {
			use(d);
			return;
		}
		if (K == 0) {
			mov64(d, 0);
			return;
		}
		use(d);
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo == 0)
			mov32(L(d), 0);
		else if (lo != 0xffffffffu)
			E.vop2(V2_AND, L(d), k32(lo), L(d));
		if (hi == 0)
			hi0(d);
		else if (hi != 0xffffffffu && !hz(d))
			E.vop2(V2_AND, Hi(d), k32(hi), Hi(d));
		f.def(d, kbits(std::min(bits_of(x), 64 - clz64(K))));
	}
	void lsh64i(int d, uint32_t c)
	{
		c &= 63;
		const rf x = f.r[d];
		if (c == 0) {
			use(d);
			return;
		}
		if (x.c) {
			mov64(d, x.v << c);
			return;
		}
		use(d);
		const int nb = std::min(64, bits_of(x) + (int)c);
		if (c >= 32) {
			if (c == 32)
				E.vop1(V1_MOV_B32, Hi(d), vreg(L(d)));
			else
				E.vop2(V2_LSHLREV_B32, Hi(d), opnd{128 + (c - 32)}, L(d));
			mov32(L(d), 0);
		} else if (nb <= 32) {
			E.vop2(V2_LSHLREV_B32, L(d), opnd{128 + c}, L(d));
		} else {
			E.vop3(V3_LSHLREV_B64, L(d), 128 + c, VGPR0 + L(d), 0);
		}
		f.def(d, kbits(nb));
	}
	void rsh64i(int d, uint32_t c)
	{
		c &= 63;
		const rf x = f.r[d];
		if (c == 0) {
			use(d);
			return;
		}
		if (x.c) {
			mov64(d, x.v >> c);
			return;
		}
		const int nb = std::max(0, bits_of(x) - (int)c);
		if (nb == 0) {
			mov64(d, 0);
			return;
		}
		use(d);
		if (c >= 32) {
			if (c == 32)
				E.vop1(V1_MOV_B32, L(d), vreg(Hi(d)));
			else
				E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + (c - 32)}, Hi(d));
			mov32(Hi(d), 0);
		} else if (hz(d)) {
			E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + c}, L(d));
		} else {
			E.vop3(V3_LSHRREV_B64, L(d), 128 + c, VGPR0 + L(d), 0);
		}
		f.def(d, kbits(nb));
	}
	void mul64i(int d, uint64_t K)
	{
		const rf x = f.r[d];
		if (x.c) {
			mov64(d, x.v * K);
			return;
		}
		if (K == 0) {
			mov64(d, 0);
			return;
		}
		if (K == 1) {
			use(d);
			return;
		}
		if ((K & (K - 1)) == 0) {
			lsh64i(d, (uint32_t)__builtin_ctzll(K));
			return;
		}
		use(d);
		const int nb = std::min(64, bits_of(x) + 64 - clz64(K));
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		const uint32_t klo = c3(lo);
		// d * K mod 2^64 = lo(d) * lo(K) + ((hi(d) * lo(K) + lo(d) * hi(K)) << 32): the cross
		// terms (low words only) go into the high word of the addend v[48:49] = {0, cross} of
		// one v_mad_u64_u32 that writes d in place
		if (hz(d) && hi == 0) {
			E.vop3(V3_MAD_U64_U32, L(d), VGPR0 + L(d), klo, 128, S_JUNK);
			f.def(d, kbits(nb));
			return;
		}
		if (!f.t2zero) {
			mov32(T2, 0);
			f.t2zero = true;
		}
		if (hi == 0) {
			E.vop3(V3_MUL_LO_U32, T3, VGPR0 + Hi(d), klo, 0);
		} else if (hz(d)) {
			E.vop3(V3_MUL_LO_U32, T3, VGPR0 + L(d), c3(hi), 0);
		} else {
			E.vop3(V3_MUL_LO_U32, T3, VGPR0 + Hi(d), klo, 0);
			E.vop3(V3_MUL_LO_U32, T1, VGPR0 + L(d), c3(hi), 0);
			E.vop2(V2_ADD_U32, T3, vreg(T3), T1);
		}
		E.vop3(V3_MAD_U64_U32, L(d), VGPR0 + L(d), klo, VGPR0 + T2, S_JUNK);
		f.def(d, kbits(nb));
	}

	// ---- ALU32 (lo op= k; hi = 0)
	// src >= 0: the operand is u32(r[src]) instead of r[d] (a 32-bit MOV d = src fused into
	// this operation by the caller)
	bool alu32i(int fam, int d, uint32_t k, int src = -1)
	{
		const int sr = src >= 0 ? src : d;
		const rf x = f.r[sr];
		const uint32_t a = (uint32_t)x.v;
		const int ab = std::min(32, bits_of(x));
		if (x.c || fam == AHF_A32I_MOV) {
			uint32_t r;
			switch (fam) {
			case AHF_A32I_ADD: r = a + k; break;
			case AHF_A32I_SUB: r = a - k; break;
			case AHF_A32I_MUL: r = a * k; break;
			case AHF_A32I_OR: r = a | k; break;
			case AHF_A32I_AND: r = a & k; break;
			case AHF_A32I_XOR: r = a ^ k; break;
			case AHF_A32I_LSH: r = a << (k & 31); break;
			case AHF_A32I_RSH: r = a >> (k & 31); break;
			case AHF_A32I_MOV: r = k; break;
			default: return false;
			}
			mov64(d, r);
			return true;
		}
		int nb = 32;
		const size_t at = blk.body.size();
		switch (fam) {
		case AHF_A32I_ADD:
			if (k)
				E.vop2(V2_ADD_U32, L(d), k32(k), L(sr));
			nb = k ? std::min(32, std::max(ab, 32 - __builtin_clz(k)) + 1) : ab;
			break;
		case AHF_A32I_SUB:
			if (k)
				E.vop2(V2_SUBREV_U32, L(d), k32(k), L(sr));
			nb = k ? 32 : ab;
			break;
		case AHF_A32I_MUL:
			E.vop3(V3_MUL_LO_U32, L(d), VGPR0 + L(sr), c3(k), 0);
			nb = k ? std::min(32, ab + 32 - __builtin_clz(k)) : 0;
			break;
		case AHF_A32I_OR:
			if (k)
				E.vop2(V2_OR, L(d), k32(k), L(sr));
			nb = std::max(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_AND:
			if (k != 0xffffffffu)
				E.vop2(V2_AND, L(d), k32(k), L(sr));
			nb = std::min(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_XOR:
			if (k)
				E.vop2(V2_XOR, L(d), k32(k), L(sr));
			nb = std::max(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_LSH:
			if (k & 31)
				E.vop2(V2_LSHLREV_B32, L(d), opnd{128 + (k & 31)}, L(sr));
			nb = std::min(32, ab + (int)(k & 31));
			break;
		case AHF_A32I_RSH:
			if (k & 31)
				E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + (k & 31)}, L(sr));
			nb = std::max(0, ab - (int)(k & 31));
			break;
		default:
			return false;
		}
		if (sr != d && blk.body.size() == at) // (an identity operation: the fused copy alone)
			E.vop1(V1_MOV_B32, L(d), vreg(L(sr)));
		use(sr);
		hi0(d);
		f.def(d, kbits(nb));
		return true;
	}
	bool alu32r(int fam, int d, int s)
	{
		if (f.r[s].c && fam != AHF_A32R_DIV && fam != AHF_A32R_MOD) {
			static const int to_i[] = {AHF_A32I_ADD, AHF_A32I_SUB, AHF_A32I_MUL, AHF_A32I_OR,
						   AHF_A32I_AND, AHF_A32I_XOR, AHF_A32I_LSH, AHF_A32I_RSH,
						   AHF_A32I_MOV};
			return alu32i(to_i[fam - AHF_A32R_ADD], d, (uint32_t)f.r[s].v);
		}
		const rf x = f.r[d];
		const int ab = std::min(32, bits_of(x)), sb = std::min(32, bits_of(f.r[s]));
		int nb = 32;
		switch (fam) {
		case AHF_A32R_ADD: E.vop2(V2_ADD_U32, L(d), vreg(L(d)), L(s)); nb = std::min(32, std::max(ab, sb) + 1); break;
		case AHF_A32R_SUB: E.vop2(V2_SUB_U32, L(d), vreg(L(d)), L(s)); break;
		case AHF_A32R_MUL: E.vop3(V3_MUL_LO_U32, L(d), VGPR0 + L(d), VGPR0 + L(s), 0); nb = std::min(32, ab + sb); break;
		case AHF_A32R_OR: E.vop2(V2_OR, L(d), vreg(L(s)), L(d)); nb = std::max(ab, sb); break;
		case AHF_A32R_AND: E.vop2(V2_AND, L(d), vreg(L(s)), L(d)); nb = std::min(ab, sb); break;
		case AHF_A32R_XOR: E.vop2(V2_XOR, L(d), vreg(L(s)), L(d)); nb = std::max(ab, sb); break;
		case AHF_A32R_LSH: E.vop2(V2_LSHLREV_B32, L(d), vreg(L(s)), L(d)); break;
		case AHF_A32R_RSH: E.vop2(V2_LSHRREV_B32, L(d), vreg(L(s)), L(d)); nb = ab; break;
		case AHF_A32R_MOV: E.vop1(V1_MOV_B32, L(d), vreg(L(s))); nb = sb; break;
		default: return false;
		}
		use(s);
		if (fam != AHF_A32R_MOV)
			use(d);
		if (d == s && (fam == AHF_A32R_SUB || fam == AHF_A32R_XOR))
			nb = 0;
		hi0(d);
		f.def(d, kbits(nb));
		return true;
	}
	bool alu64r(int fam, int d, int s)
	{
		const rf xs = f.r[s];
		const rf x = f.r[d];
		if (d == s) {
			switch (fam) {
			case AHF_A64R_ADD: lsh64i(d, 1); return true;
			case AHF_A64R_SUB: case AHF_A64R_XOR: mov64(d, 0); return true;
			case AHF_A64R_OR: case AHF_A64R_AND: use(d); return true;
			default: return false;
			}
		}
		if (xs.c) {
			switch (fam) {
			case AHF_A64R_ADD: add64i(d, xs.v); return true;
			case AHF_A64R_SUB: add64i(d, 0 - xs.v); return true;
			case AHF_A64R_MUL: mul64i(d, xs.v); return true;
			case AHF_A64R_OR: or64i(d, xs.v); return true;
			case AHF_A64R_AND: and64i(d, xs.v); return true;
			case AHF_A64R_XOR: xor64i(d, xs.v); return true;
			case AHF_A64R_LSH: lsh64i(d, (uint32_t)xs.v); return true;
			case AHF_A64R_RSH: rsh64i(d, (uint32_t)xs.v); return true;
			default: return false;
			}
		}
		if (x.c && x.v == 0 && (fam == AHF_A64R_ADD || fam == AHF_A64R_OR || fam == AHF_A64R_XOR)) {
			copy64(d, s);
			return true;
		}
		switch (fam) {
		case AHF_A64R_ADD:
			use(d);
			use(s);
			E.vop3(V3_LSHL_ADD_U64, L(d), VGPR0 + L(s), 128, VGPR0 + L(d));
			f.def(d, kbits(std::min(64, std::max(bits_of(x), bits_of(xs)) + 1)));
			return true;
		case AHF_A64R_OR:
		case AHF_A64R_XOR: {
			use(d);
			use(s);
			const uint32_t op = fam == AHF_A64R_OR ? V2_OR : V2_XOR;
			E.vop2(op, L(d), vreg(L(s)), L(d));
			if (!hz(s))
				E.vop2(op, Hi(d), vreg(Hi(s)), Hi(d));
			f.def(d, kbits(std::max(bits_of(x), bits_of(xs))));
			return true;
		}
		case AHF_A64R_AND:
			use(d);
			use(s);
			E.vop2(V2_AND, L(d), vreg(L(s)), L(d));
			if (hz(s))
				hi0(d);
			else if (!hz(d))
				E.vop2(V2_AND, Hi(d), vreg(Hi(s)), Hi(d));
			f.def(d, kbits(std::min(bits_of(x), bits_of(xs))));
			return true;
		default:
			return false;
		}
	}

	// ---- byte swaps (BE16/BE32 zero-extend; LE is lowered to AND)
	bool bswap(int fam, int d)
	{
		const rf x = f.r[d];
		if (fam == AHF_BSWAP16) {
			if (x.c) {
				mov64(d, __builtin_bswap16((uint16_t)x.v));
				return true;
			}
			use(d);
			E.vop3(V3_PERM_B32, L(d), 128, VGPR0 + L(d), sconst(0x0c0c0001u));
			hi0(d);
			f.def(d, kbits(16));
			return true;
		}
		if (fam == AHF_BSWAP32) {
			if (x.c) {
				mov64(d, __builtin_bswap32((uint32_t)x.v));
				return true;
			}
			use(d);
			E.vop3(V3_PERM_B32, L(d), 128, VGPR0 + L(d), VGPR0 + V_SEL);
			hi0(d);
			f.def(d, kbits(32));
			return true;
		}
		return false;
	}

	// ---- staged packet load at constant offset `off`, size z; swap_bytes = 0, 2 or 4 (a fused
	// BE16 / BE32 of the loaded register)
	// General kernels with header staging: the packet load at constant offset off < 64 from the
	// staged header registers, like the handler (h_ldx_pkt_const) but with its two per-load lane
	// compares replaced by one per-group mask: s[74:75] = lanes whose packet is shorter than 64
	// bytes (set by the prologue).  Only such lanes can fault (off + z > len) or need the load
	// from memory; when none is running the load is the extract alone.
	void ldxpkc_general(int d, int z, int off, uint32_t fault_off)
	{
		const int S_SHORT = 74, S_MASK = 48, S_CODE = 52, S_JUNK_ = 60, V_LEN = 40, V_PKT = 38;
		static const uint32_t gop[4] = {0x10, 0x12, 0x14, 0x15};
		const int zi = z == 1 ? 0 : z == 2 ? 1 : z == 4 ? 2 : 3;
		auto patch = [&](size_t at) { // branch at byte `at` jumps to here
			const uint32_t rel = (uint32_t)((blk.body.size() - at - 4) / 4);
			blk.body[at] = (uint8_t)(rel & 0xff);
			blk.body[at + 1] = (uint8_t)((rel >> 8) & 0xff);
		};
		E.sop2(0x0d, S_MASK, opnd{(uint32_t)S_SHORT}, opnd{SRC_EXEC});   // s_and_b64 (scc)
		const size_t to_fast = blk.body.size();
		E.w(0xbf840000u);                                                 // s_cbranch_scc0 fast
		E.vopc(VC_U32 + P_GT, k32((uint32_t)(off + z)), V_LEN);          // vcc = off+z > len
		E.sop2(0x0d, S_MASK, opnd{SRC_VCC}, opnd{SRC_EXEC});
		E.w(0xbf840000u | 5u);                                           // s_cbranch_scc0 +5
		E.sop1(0x00, S_CODE, opnd{128 + 3});                             // s_mov_b32 s52, 3 (MEM)
		call_routine(fault_off, 0);                                      // (4 dwords)
		const facts f0 = f; // (both paths emit the same extract from the same facts)
		ldxpkc(d, z, off, 0);
		E.sop2(0x0d, S_MASK, opnd{(uint32_t)S_SHORT}, opnd{SRC_EXEC});
		const size_t to_end1 = blk.body.size();
		E.w(0xbf840000u);                                                 // s_cbranch_scc0 end
		E.sop1(0x01, S_JUNK_, opnd{SRC_EXEC});                           // s_mov_b64 s60, exec
		E.sop1(0x01, 126, opnd{(uint32_t)S_MASK});                       // exec = short lanes
		E.w(0xdc008000u | (gop[zi] << 18) | (uint32_t)off);              // global_load_*
		E.w((uint32_t)V_PKT | (0x7fu << 16) | ((uint32_t)L(d) << 24));
		E.w(0xbf8c0f70u);                                                 // s_waitcnt vmcnt(0)
		if (z < 8)
			mov32(Hi(d), 0);
		E.sop1(0x01, 126, opnd{(uint32_t)S_JUNK_});                      // exec back
		const size_t to_end2 = blk.body.size();
		E.w(0xbf820000u);                                                 // s_branch end
		patch(to_fast);
		f = f0;
		ldxpkc(d, z, off, 0);
		patch(to_end1);
		patch(to_end2);
	}
	void ldxpkc(int d, int z, int off, int swap_bytes)
	{
		const int k = off >> 2, sh = off & 3;
		const int lo = PKT0 + k, nx = PKT0 + (k + 1 < 16 ? k + 1 : k);
		if (swap_bytes) {
			// result byte i = packet byte off + (W-1-i) for W-1-i < z
			uint32_t sel = 0;
			for (int i = 0; i < 4; i++) {
				const int j = swap_bytes - 1 - i;
				const uint32_t b = (i < swap_bytes && j < z) ? (uint32_t)(sh + j) : 0x0cu;
				sel |= b << (8 * i);
			}
			const uint32_t sc = sel == 0x00010203u ? VGPR0 + V_SEL : sconst(sel);
			E.vop3(V3_PERM_B32, L(d), VGPR0 + nx, VGPR0 + lo, sc);
			hi0(d);
			// (the loaded bytes land at the top of the swapped word: a byte under BE32 is b << 24,
			// so the value needs all 8 * W bits, not 8 * z)
			f.def(d, kbits(8 * swap_bytes));
			return;
		}
		if (z == 1) {
			E.vop3(V3_BFE_U32, L(d), VGPR0 + lo, 128 + 8 * sh, 128 + 8);
		} else if (z == 2) {
			if (sh <= 2)
				E.vop3(V3_BFE_U32, L(d), VGPR0 + lo, 128 + 8 * sh, 128 + 16);
			else
				E.vop3(V3_PERM_B32, L(d), VGPR0 + nx, VGPR0 + lo, sconst(0x0c0c0403u));
		} else if (z == 4) {
			if (sh == 0)
				E.vop1(V1_MOV_B32, L(d), vreg(lo));
			else
				E.vop3(V3_ALIGNBYTE, L(d), VGPR0 + nx, VGPR0 + lo, 128 + sh);
		} else {
			if (sh == 0) {
				if ((lo & 1) == 0) {
					E.vop1(V1_MOV_B64, L(d), vreg(lo));
				} else {
					E.vop1(V1_MOV_B32, L(d), vreg(lo));
					E.vop1(V1_MOV_B32, Hi(d), vreg(lo + 1));
				}
			} else {
				E.vop3(V3_ALIGNBYTE, L(d), VGPR0 + lo + 1, VGPR0 + lo, 128 + sh);
				E.vop3(V3_ALIGNBYTE, Hi(d), VGPR0 + lo + 2, VGPR0 + lo + 1, 128 + sh);
			}
			f.def(d, rf());
			return;
		}
		hi0(d);
		f.def(d, kbits(8 * z));
	}

	// ---- stack accesses at a known LDS offset `o` from the lane's stack bottom
	void stxstk(int z, int r, uint32_t o)
	{
		use(r);
		if (z == 8)
			E.ds(DS_WRITE2_B32, V_STK, L(r), Hi(r), 0, o / 4, o / 4 + 1);
		else
			E.ds(z == 4 ? DS_WRITE_B32 : z == 2 ? DS_WRITE_B16 : DS_WRITE_B8, V_STK, L(r), 0, 0, o);
		f.store(o, z, r);
	}
	// low z bytes of register s into d
	void low_bytes(int d, int s, int z)
	{
		if (z == 8) {
			copy64(d, s);
			return;
		}
		const rf xs = f.r[s];
		if (xs.c) {
			mov64(d, z == 4 ? (uint32_t)xs.v : xs.v & ((1ull << (8 * z)) - 1));
			return;
		}
		use(s);
		const int sb = std::min(bits_of(xs), 8 * z);
		if (bits_of(xs) <= 8 * z)
			E.vop1(V1_MOV_B32, L(d), vreg(L(s)));
		else if (z == 4)
			E.vop1(V1_MOV_B32, L(d), vreg(L(s)));
		else
			E.vop2(V2_AND, L(d), k32(z == 1 ? 0xffu : 0xffffu), L(s));
		hi0(d);
		f.def(d, kbits(sb));
	}
	void ldxstk(int z, int d, uint32_t o)
	{
		if (const sslot *sl = f.slot(o, z)) {
			low_bytes(d, sl->reg, z);
			return;
		}
		blk.stack_read = true;
		if (z == 8) {
			E.ds(DS_READ2_B32, V_STK, 0, 0, L(d), o / 4, o / 4 + 1);
			E.wait_lgkm();
			f.def(d, rf());
			return;
		}
		E.ds(z == 4 ? DS_READ_B32 : z == 2 ? DS_READ_U16 : DS_READ_U8, V_STK, 0, 0, L(d), o);
		E.wait_lgkm();
		hi0(d);
		f.def(d, kbits(8 * z));
	}

	// ---- array-map lookup resolved to map `mi` with the key at stack offset `o`: specialised
	// when the key is a register proven below max_entries (the lookup cannot return NULL)
	bool lookup_stk(int mi, uint32_t o)
	{
		if (mi < 0)
			return false;
		const mapinfo &m = maps[mi];
		const sslot *sl = f.slot(o, 4);
		if (!sl)
			return false;
		const int R = sl->reg;
		const rf xr = f.r[R];
		const uint64_t kmax = xr.c ? (uint32_t)xr.v : (bits_of(xr) >= 32 ? 0xffffffffull : (1ull << bits_of(xr)) - 1);
		if (kmax >= m.max_entries || m.max_entries > (1u << 24))
			return false;
		use(R);
		// (the map base is an SGPR pair: the value size must not be a second SGPR)
		E.vop3(V3_MAD_U64_U32, L(0), VGPR0 + L(R), vconst(m.value_size, T0), spair(m.dev_base), S_JUNK);
		rf v;
		v.nz = true;
		v.mp = (int8_t)mi;
		v.mreg = (int8_t)R;
		f.def(0, v);
		return true;
	}
	// LDXHV through a non-NULL hashtable lookup result whose value's first 8 bytes were
	// loaded with the probe into register D's VGPRs: an extract, no memory access
	bool ldxhv_fwd(int z, int d, int s, int32_t o)
	{
		const rf xs = f.r[s];
		if (xs.hfwd < 0 || !xs.nz || o < 0 || o + z > 8 || (o % z) != 0)
			return false;
		const int D = xs.hfwd;
		use(s);
		use(D);
		if (z == 8) {
			if (d != D)
				E.vop1(V1_MOV_B64, L(d), vreg(L(D)));
		} else if (z == 4) {
			E.vop1(V1_MOV_B32, L(d), vreg(L(D) + o / 4));
		} else {
			E.vop3(V3_BFE_U32, L(d), VGPR0 + L(D) + (uint32_t)(o / 4), 128 + 8 * (uint32_t)(o % 4),
			       128 + 8 * (uint32_t)z);
		}
		if (z < 8)
			mov32(Hi(d), 0);
		f.def(d, z == 8 ? rf() : kbits(8 * z));
		return true;
	}
	// LDXMAP through a pointer with known map and index register: the LDS copy, no check
	bool ldxmap(int z, int d, int s, uint64_t imm)
	{
		const rf xs = f.r[s];
		if (xs.mp < 0 || xs.mreg < 0 || !xs.nz)
			return false;
		const mapinfo &m = maps[xs.mp];
		if (m.lds_off == ~0u)
			return false;
		const int64_t c = (int64_t)(m.dev_base - imm); // the access offset within the value
		if (c < 0 || c + z > (int64_t)m.value_size)
			return false;
		const int R = xs.mreg;
		use(R);
		const uint32_t base = m.lds_off + (uint32_t)c;
		// (base >= the map area's LDS offset is never an inline constant: an SGPR, so a value
		// size that is none either goes through a VGPR)
		E.vop3(V3_MAD_U32_U24, T0, VGPR0 + L(R), vconst(m.value_size, T1), c3(base));
		if (z == 8) {
			E.ds(DS_READ2_B32, T0, 0, 0, L(d), 0, 1);
			E.wait_lgkm();
			f.def(d, rf());
			return true;
		}
		E.ds(z == 4 ? DS_READ_B32 : z == 2 ? DS_READ_U16 : DS_READ_U8, T0, 0, 0, L(d), 0);
		E.wait_lgkm();
		hi0(d);
		f.def(d, kbits(8 * z));
		return true;
	}

	// ---- EXIT with r0 known: result and verdict bin set here, then .Lr_exit_k (gen_interp.py)
	void exit_known(uint64_t r0, uint32_t exitk_off, bool call)
	{
		mov32(V_RES, (uint32_t)r0);
		mov32(V_RES + 1, (uint32_t)(r0 >> 32));
		if (call) {
			// structured programs: the verdict count inline (.Lr_exit_k's work): one LDS add
			// of popcount(exec) to bin min(r0, 255); the exiting lanes leave the alive mask
			// (lane 0's V_L16 = 0 addresses the bin through the instruction offset; the alive
			// mask is not read again before the group ends in a structured program)
			const int S_CODE = 52, S_SAVE = 18, R8 = 60, V_L16 = 43;
			const uint32_t bin = r0 < 255 ? (uint32_t)r0 : 255u;
			E.sop1(0x0d, S_CODE, opnd{SRC_EXEC});                         // s_bcnt1_i32_b64
			E.sop1(0x01, S_SAVE, opnd{SRC_EXEC});                         // s_mov_b64
			E.sop1(0x01, 126, opnd{128 + 1});                              // exec = lane 0
			E.vop1(V1_MOV_B32, R8, opnd{(uint32_t)S_CODE});
			E.ds(0x00, V_L16, R8, 0, 0, (bin * 4) & 0xff, (bin * 4) >> 8);  // ds_add_u32
			E.sop1(0x01, 126, opnd{(uint32_t)S_SAVE});
			(void)exitk_off;
			return;
		}
		E.sop1(0x00, S_BYTES, k32(r0 < 255 ? (uint32_t)r0 : 255u));   // s_mov_b32
		E.sop2(0x00, S_JUNK, opnd{(uint32_t)S_CB}, opnd{SRC_LIT, exitk_off}); // s_add_u32
		E.sop2(0x04, S_JUNK + 1, opnd{(uint32_t)S_CB + 1}, opnd{128});     // s_addc_u32
		E.sop1(0x1d, 0, opnd{(uint32_t)S_JUNK});                           // s_setpc_b64
	}
	// EXIT with r0 in registers (structured programs), inline: r0 into the result slot and one
	// LDS histogram add per lane at bin min(r0, 255) (what .Lr_exit does, without the call,
	// the return and the uniform-verdict test)
	void exit_inline()
	{
		const int R8 = 60, R9 = 61;
		use(0);
		E.vop1(V1_MOV_B32, V_RES, vreg(0));
		E.vop1(V1_MOV_B32, V_RES + 1, vreg(1));
		int bin = 0; // v0 holds the bin if r0 < 256
		if (f.r[0].lz < 56) {
			E.vop1(V1_MOV_B32, R8, k32(255));
			E.vop1(V1_MOV_B32, R9, opnd{128});
			E.vopc(VC_U64 + P_LT, vreg(0), R8);            // vcc = r0 < 255
			E.vop2(0x00, R8, vreg(R8), 0);                 // v_cndmask_b32 v60, v60, v0, vcc
			bin = R8;
		}
		E.vop2(V2_LSHLREV_B32, R8, opnd{128 + 2}, bin);
		E.vop1(V1_MOV_B32, R9, opnd{128 + 1});
		E.ds(0x00, R8, R9, 0, 0, 0);                        // ds_add_u32
	}
	// call a routine that returns (structured programs): the link pair s[50:51]
	void call_routine(uint32_t off, uint16_t reads)
	{
		const int S_LINK = 50;
		used |= reads;
		E.sop2(0x00, S_LINK, opnd{(uint32_t)S_CB}, opnd{SRC_LIT, off});     // s_add_u32
		E.sop2(0x04, S_LINK + 1, opnd{(uint32_t)S_CB + 1}, opnd{128});     // s_addc_u32
		E.sop1(0x1e, S_LINK, opnd{(uint32_t)S_LINK});                      // s_swappc_b64
	}
	// A packet load whose bytes were loaded ahead into VGPR `tmp` (general kernels, see
	// hoist plan in cc_compile): the bounds check at its own place (MEM fault for lanes whose
	// packet is shorter than off + z, like the handler), then wait for it (vmcnt <= the loads
	// issued after it) and copy.
	//
	// With the run mask (s[76:77], see cc_compile) the lanes in the mask hold the load already
	// and cannot fault on it; only when a running lane is outside the mask does the use compare:
	// fault the lanes past their packet's end, load for the others directly (and wait for it).
	void ldx_hoisted(int d, int z, uint32_t off, int tmp, uint32_t later, uint32_t fault_off,
			 bool runmask)
	{
		const int S_MASK = 48, S_CODE = 52, V_LEN = 40, S_JUNK_ = 60, V_PKT = 38;
		size_t br = 0, from = 0;
		if (runmask) {
			E.sop2(0x13, S_MASK, opnd{SRC_EXEC}, opnd{(uint32_t)AH_S_RUNMASK}); // s_andn2_b64
			br = E.b.size();
			E.w(0xbf840000u); // s_cbranch_scc0 over the block below (its length set at its end)
			from = E.b.size();
		}
		E.vopc(VC_U32 + P_GT, k32(off + (uint32_t)z), V_LEN);          // vcc = off + z > len
		E.sop2(0x0d, S_MASK, opnd{SRC_VCC}, opnd{SRC_EXEC});             // s_and_b64
		E.w(0xbf840000u | 5u);                                           // s_cbranch_scc0 +5
		E.sop1(0x00, S_CODE, opnd{128 + 3});                             // s_mov_b32 s52, 3
		call_routine(fault_off, 0);                                      // (4 dwords)
		if (runmask) {
			static const uint32_t gop[4] = {0x10, 0x12, 0x14, 0x15};
			const int zi = z == 1 ? 0 : z == 2 ? 1 : z == 4 ? 2 : 3;
			E.sop2(0x13, S_MASK, opnd{SRC_EXEC}, opnd{(uint32_t)AH_S_RUNMASK}); // in bounds, unmasked
			E.w(0xbf840000u | 6u);                                           // s_cbranch_scc0 +6
			E.sop1(0x01, S_JUNK_, opnd{SRC_EXEC});                           // s_mov_b64 s60, exec
			E.sop1(0x01, 126, opnd{(uint32_t)S_MASK});                       // s_mov_b64 exec, s48
			E.w(0xdc008000u | (gop[zi] << 18) | off);                        // global_load_* tmp
			E.w((uint32_t)V_PKT | (0x7fu << 16) | ((uint32_t)tmp << 24));
			E.w(0xbf8c0f70u);                                                // s_waitcnt vmcnt(0)
			E.sop1(0x01, 126, opnd{(uint32_t)S_JUNK_});                      // s_mov_b64 exec, s60
			const uint32_t skip = (uint32_t)((E.b.size() - from) / 4);
			E.b[br] = (uint8_t)skip;
			E.b[br + 1] = (uint8_t)(skip >> 8);
		}
		E.w(0xbf8c0000u | (later & 15u) | (7u << 4) | (15u << 8) | ((later >> 4) & 3u) << 14);
		if (z == 8) {
			E.vop1(V1_MOV_B64, L(d), vreg(tmp));
			f.def(d, rf());
		} else {
			E.vop1(V1_MOV_B32, L(d), vreg(tmp));
			hi0(d);
			f.def(d, kbits(8 * z));
		}
	}
	// FAULT entry (structured): fault every running lane with `code`
	void fault(uint32_t code, uint32_t fault_off)
	{
		const int S_MASK = 48, S_CODE = 52;
		E.sop1(0x00, S_CODE, k32(code));            // s_mov_b32 s52, code
		E.sop1(0x01, S_MASK, opnd{SRC_EXEC});       // s_mov_b64 s[48:49], exec
		call_routine(fault_off, 0);
	}

	// ---- conditional jumps: VCC = lanes taking the branch (the caller appends the tail)
	// c: 0 EQ, 1 NE, 2 GT, 3 GE, 4 LT, 5 LE, 6 SGT, 7 SGE, 8 SLT, 9 SLE, 10 SET
	static bool eval(int c, uint64_t a, uint64_t b)
	{
		const int64_t sa = (int64_t)a, sb = (int64_t)b;
		switch (c) {
		case 0: return a == b;
		case 1: return a != b;
		case 2: return a > b;
		case 3: return a >= b;
		case 4: return a < b;
		case 5: return a <= b;
		case 6: return sa > sb;
		case 7: return sa >= sb;
		case 8: return sa < sb;
		case 9: return sa <= sb;
		default: return (a & b) != 0;
		}
	}
	static int pred(int c) { static const int p[] = {P_EQ, P_NE, P_GT, P_GE, P_LT, P_LE, P_GT, P_GE, P_LT, P_LE}; return p[c]; }
	static int swapped(int p)
	{
		switch (p) {
		case P_GT: return P_LT;
		case P_GE: return P_LE;
		case P_LT: return P_GT;
		case P_LE: return P_GE;
		default: return p;
		}
	}
	// a compare decided at compile time: no code, the layout falls through or jumps
	unsigned off = 0;
	void decided(bool taken)
	{
		if ((off & 16) && taken) { // structured: s_mov_b64 vcc, exec (the split sends every lane)
			E.sop1(0x01, (int)SRC_VCC, opnd{SRC_EXEC});
			return;
		}
		// (structured and never taken: the code generator only empties the join mask)
		blk.sdir = taken ? 1 : 0;
	}
	void cond_imm(int c, int d, uint64_t K)
	{
		const rf &x = f.r[d];
		if (x.c) {
			decided(eval(c, x.v, K));
			return;
		}
		if (K == 0 && x.nz && (c == 0 || c == 1)) { // NULL check of a lookup that cannot fail
			decided(c == 1);
			return;
		}
		use(d);
		if (c == 10) { // JSET
			const uint32_t lo = (uint32_t)K, hi = hz(d) ? 0u : (uint32_t)(K >> 32);
			if (!lo && !hi) {
				decided(false);
				return;
			}
			if (!hi) {
				E.vop2(V2_AND, T0, k32(lo), L(d));
				E.vopc(VC_U32 + P_NE, opnd{128}, T0);
			} else {
				E.vop2(V2_AND, T0, k32(lo), L(d));
				E.vop2(V2_AND, T1, k32(hi), Hi(d));
				E.vopc(VC_U64 + P_NE, opnd{128}, T0);
			}
			return;
		}
		if (hz(d)) {
			// d in [0, 2^32): K outside that range decides statically (signed: d >= 0)
			if (K >> 32) {
				const bool kneg = (int64_t)K < 0;
				bool r;
				switch (c) {
				case 0: r = false; break;
				case 1: r = true; break;
				case 2: case 3: r = false; break;
				case 4: case 5: r = true; break;
				case 6: case 7: r = kneg; break;
				default: r = !kneg; break;
				}
				decided(r);
				return;
			}
			E.vopc(VC_U32 + swapped(pred(c)), k32((uint32_t)K), L(d));
			return;
		}
		const uint32_t base = c >= 6 ? VC_I64 : VC_U64;
		E.vopc(base + swapped(pred(c)), opnd{c64(K)}, L(d));
	}
	void cond_reg(int c, int d, int s)
	{
		if (f.r[s].c) {
			cond_imm(c, d, f.r[s].v);
			return;
		}
		use(d);
		use(s);
		if (c == 10) {
			E.vop2(V2_AND, T0, vreg(L(s)), L(d));
			if (hz(d) || hz(s)) {
				E.vopc(VC_U32 + P_NE, opnd{128}, T0);
			} else {
				E.vop2(V2_AND, T1, vreg(Hi(s)), Hi(d));
				E.vopc(VC_U64 + P_NE, opnd{128}, T0);
			}
			return;
		}
		if (hz(d) && hz(s)) {
			E.vopc(VC_U32 + pred(c), vreg(L(d)), L(s));
			return;
		}
		E.vopc((c >= 6 ? VC_I64 : VC_U64) + pred(c), vreg(L(d)), L(s));
	}
	// JMP32: compares of the low words
	static bool eval32(int c, uint32_t a, uint32_t b)
	{
		switch (c) {
		case 0: return a == b;
		case 1: return a != b;
		case 2: return a > b;
		case 3: return a >= b;
		case 4: return a < b;
		case 5: return a <= b;
		case 6: return (int32_t)a > (int32_t)b;
		case 7: return (int32_t)a >= (int32_t)b;
		case 8: return (int32_t)a < (int32_t)b;
		case 9: return (int32_t)a <= (int32_t)b;
		default: return (a & b) != 0;
		}
	}
	void cond32_imm(int c, int d, uint32_t K)
	{
		const rf &x = f.r[d];
		if (x.c) {
			decided(eval32(c, (uint32_t)x.v, K));
			return;
		}
		use(d);
		if (c == 10) {
			if (!K) {
				decided(false);
				return;
			}
			E.vop2(V2_AND, T0, k32(K), L(d));
			E.vopc(VC_U32 + P_NE, opnd{128}, T0);
			return;
		}
		E.vopc((c >= 6 ? VC_I32 : VC_U32) + swapped(pred(c)), k32(K), L(d));
	}
	void cond32_reg(int c, int d, int s)
	{
		if (f.r[s].c) {
			cond32_imm(c, d, (uint32_t)f.r[s].v);
			return;
		}
		use(d);
		use(s);
		if (c == 10) {
			E.vop2(V2_AND, T0, vreg(L(s)), L(d));
			E.vopc(VC_U32 + P_NE, opnd{128}, T0);
			return;
		}
		E.vopc((c >= 6 ? VC_I32 : VC_U32) + pred(c), vreg(L(d)), L(s));
	}
};

// the STX of a counter update, XADD (ebpf_gpu.h "Stores into map values"): generic stores
bool
is_value_store_fam(int fam)
{
	return fam == AHF_CNTST4 || fam == AHF_CNTST8 || fam == AHF_XADD4 || fam == AHF_XADD8 ||
	       fam == AHF_XADDF4 || fam == AHF_XADDF8;
}

bool
is_cond_fam(int fam)
{
	return (fam >= AHF_JEQ_R && fam <= AHF_JSET_R) || (fam >= AHF_JEQ_I && fam <= AHF_JSET_I) ||
	       (fam >= AHF_J32EQ_R && fam <= AHF_J32SET_R) || (fam >= AHF_J32EQ_I && fam <= AHF_J32SET_I);
}

// the register a copied handler body writes (-1: none)
int
written_reg(int fam, int d)
{
	switch (fam) {
	case AHF_LOOKUPSTK: case AHF_LOOKUPGEN: case AHF_HLOOKUP: case AHF_UPDATE: case AHF_HDELETE:
		return 0;
	case AHF_EXIT: case AHF_FAULT: case AHF_NOP:
	case AHF_STXGEN1: case AHF_STXGEN2: case AHF_STXGEN4: case AHF_STXGEN8:
	case AHF_STXSTK1: case AHF_STXSTK2: case AHF_STXSTK4: case AHF_STXSTK8:
	case AHF_STGEN1: case AHF_STGEN2: case AHF_STGEN4: case AHF_STGEN8:
	case AHF_STSTK1: case AHF_STSTK2: case AHF_STSTK4: case AHF_STSTK8:
	case AHF_CNTST4: case AHF_CNTST8: case AHF_XADD4: case AHF_XADD8: case AHF_OVLINIT:
	case AHF_CNTAI4: case AHF_CNTAI8: case AHF_CNTAL4: case AHF_CNTAL8:
		return -1;
	default:
		if (is_cond_fam(fam))
			return -1;
		return d < AH_NREGS ? d : -1;
	}
}

// registers a copied handler body reads
uint16_t
copied_uses(int fam, int d, int s)
{
	auto m = [](int r) -> uint16_t { return r < AH_NREGS ? (uint16_t)(1u << r) : 0; };
	switch (fam) {
	case AHF_EXIT: return 1;
	case AHF_LOOKUPGEN: return (1u << 1) | (1u << 2);
	case AHF_HLOOKUP: case AHF_HDELETE: return 1u << 2;
	case AHF_UPDATE: return (1u << 2) | (1u << 3) | (1u << 4);
	case AHF_FAULT: case AHF_NOP: case AHF_LOOKUPSTK: case AHF_OVLINIT: return 0;
	case AHF_STSTK1: case AHF_STSTK2: case AHF_STSTK4: case AHF_STSTK8: return 0;
	case AHF_LDXPKTG1: case AHF_LDXPKTG2: case AHF_LDXPKTG4: case AHF_LDXPKTG8: return 0;
	case AHF_LDXSTK1: case AHF_LDXSTK2: case AHF_LDXSTK4: case AHF_LDXSTK8: return 0;
	case AHF_LDXPKC1: case AHF_LDXPKC2: case AHF_LDXPKC4: case AHF_LDXPKC8: return 0;
	case AHF_A64I_MOV: return 0;
	case AHF_A32I_MOV: return 0;
	case AHF_A32R_MOV: case AHF_MOV64R: return m(s);
	default: return m(d) | m(s); // (LDX*: s = the address; ST*: d = base, s = value; ALU: both)
	}
}

// facts for a copied body's result
rf
copied_result(int fam)
{
	switch (fam) {
	case AHF_LDXGEN1: case AHF_LDXMAP1: case AHF_LDXPKTG1: case AHF_LDXSTK1: case AHF_LDXHV1:
	case AHF_LDXPKC1: case AHF_LDXPKTV1: return kbits(8);
	case AHF_LDXGEN2: case AHF_LDXMAP2: case AHF_LDXPKTG2: case AHF_LDXSTK2: case AHF_LDXHV2:
	case AHF_LDXPKC2: case AHF_LDXPKTV2: return kbits(16);
	case AHF_LDXGEN4: case AHF_LDXMAP4: case AHF_LDXPKTG4: case AHF_LDXSTK4: case AHF_LDXHV4:
	case AHF_LDXPKC4: case AHF_XADDF4: case AHF_LDXPKTV4: return kbits(32);
	default:
		if (fam >= AHF_A32R_ADD && fam <= AHF_A32R_MOD)
			return kbits(32);
		if (fam >= AHF_A32I_ADD && fam <= AHF_A32I_MOD)
			return kbits(32);
		return rf();
	}
}

// operations with no effect besides writing their destination register (no fault, no memory
// write): skipped when the destination is dead
bool
pure_fam(int fam, bool specialised_map_load)
{
	if (fam >= AHF_A64R_ADD && fam <= AHF_A64R_MOD)
		return fam != AHF_A64R_DIV && fam != AHF_A64R_MOD;
	if (fam >= AHF_A32R_ADD && fam <= AHF_A32R_MOD)
		return fam != AHF_A32R_DIV && fam != AHF_A32R_MOD;
	if ((fam >= AHF_A64I_ADD && fam <= AHF_A64I_MOV) || (fam >= AHF_A32I_ADD && fam <= AHF_A32I_MOD))
		return true; // immediate divisors are never zero here (the translator faults them)
	switch (fam) {
	case AHF_BSWAP16: case AHF_BSWAP32: case AHF_BSWAP64:
	case AHF_LDXPKC1: case AHF_LDXPKC2: case AHF_LDXPKC4: case AHF_LDXPKC8:
	case AHF_LDXSTK1: case AHF_LDXSTK2: case AHF_LDXSTK4: case AHF_LDXSTK8:
	case AHF_LOOKUPSTK:
		return true;
	case AHF_LDXMAP1: case AHF_LDXMAP2: case AHF_LDXMAP4: case AHF_LDXMAP8:
		return specialised_map_load;
	default:
		return false;
	}
}

// refine facts on the taken (taken = true) or fall-through edge of `d c K`
void
refine(facts &fa, int c, int d, uint64_t K, bool taken)
{
	rf &x = fa.r[d];
	if (x.c)
		return;
	if ((c == 0 && taken) || (c == 1 && !taken)) {
		const bool keep_map = K != 0 && x.mp >= 0;
		rf k = kconst(K);
		if (keep_map) {
			k.mp = x.mp;
			k.mreg = x.mreg;
		}
		x = k;
		return;
	}
	if (K == 0 && ((c == 1 && taken) || (c == 0 && !taken))) { // d != 0
		x.nz = true;
		return;
	}
	uint64_t B;
	bool ub = false;
	if ((c == 5 && taken) || (c == 2 && !taken)) { // d <= K (unsigned)
		B = K;
		ub = true;
	} else if (((c == 4 && taken) || (c == 3 && !taken)) && K) { // d < K
		B = K - 1;
		ub = true;
	}
	if (ub) {
		const int nb = 64 - clz64(B);
		if (64 - nb > x.lz)
			x.lz = (uint8_t)(64 - nb);
	}
}

} // namespace

void
cc_prologue(int mode, uint16_t live, bool needs_pkt, bool structured, std::vector<uint8_t> &out)
{
	enc P{out};
	if (structured)
		P.sop2(0x0e, 7, opnd{7}, opnd{128 + 4}); // s_or_b32 s7, s7, 4
	const int V_PKT = 38, V_LEN = 40, H1 = 47, H3 = 49, S_DATA = 24;
	if (mode == 1 && (needs_pkt || (live & (1u << 1)))) {
		// staged kernel: packet address = data + index * 64 (index in v49, gen_interp.py H[3])
		P.vop1(V1_MOV_B32, H1, opnd{128 + 64});
		P.vop3(V3_MAD_U64_U32, V_PKT, VGPR0 + H3, VGPR0 + H1, S_DATA, S_JUNK);
		P.vop1(V1_MOV_B32, V_LEN, opnd{128 + 64});
	}
	if (live & (1u << 1))
		P.vop1(V1_MOV_B64, 2, vreg(V_PKT));
	if (live & (1u << 10)) {
		const int S_STKSTRIDE = 42, S_SHARED_HI = 59;
		P.vop2(V2_ADD_U32, 20, opnd{(uint32_t)S_STKSTRIDE}, V_STK);
		P.vop1(V1_MOV_B32, 21, opnd{(uint32_t)S_SHARED_HI});
	}
	for (int r = 0; r < AH_NREGS; r++)
		if (r != 1 && r != 10 && (live & (1u << r)))
			P.vop1(V1_MOV_B64, 2 * r, opnd{128});
}

// VOP3 instructions this thread's compiler has emitted with two SGPR sources (a bug: see enc)
unsigned
cc_bus_violations()
{
	return g_bus_violations;
}

void
cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
	   const std::vector<char> &entry_point, int mode, bool structured, const cc_routines &rt,
	   const std::vector<dp_map> &table, std::vector<cc_block> &out)
{
	const size_t n = low.size();
	std::vector<mapinfo> maps(table.size());
	for (size_t i = 0; i < table.size(); i++)
		maps[i] = mapinfo{table[i].dev_base, table[i].value_size, table[i].max_entries, table[i].lds_off};
	// predecessors (the tree gives one; shared fault entries get no facts)
	std::vector<uint32_t> npred(n, 0);
	for (uint32_t e : order) {
		const uint32_t h = (uint32_t)low[e].handler;
		const int fam = ah_fam[h];
		if (fam == AHF_EXIT || fam == AHF_FAULT)
			continue;
		if (xl.entries[e].next < n)
			npred[xl.entries[e].next]++;
		if ((ah_flags[h] & 1) && xl.entries[e].target < n)
			npred[xl.entries[e].target]++;
	}
	// General kernels: packet loads at constant offsets (LDXPKTG, one memory round trip each)
	// are issued ahead at the head of the straight run that contains them, into the image's
	// spare VGPRs, so their latencies overlap.  A run ends at an entry point, a branch, a
	// non-fall-through successor, a store that may hit the packet or a scheduler hand-off.
	std::vector<int16_t> hoist_tmp(n, -1);
	std::vector<uint16_t> hoist_later(n, 0);
	std::vector<std::vector<uint32_t>> hoist_at(n);
	std::vector<uint32_t> hoist_next(n, UINT32_MAX); // the load to issue after this one is used
	// Run mask (general kernels: s[76:77]):
	// the run head tests every running lane against the run's largest load extent once (one
	// VALU compare into s[76:77]); the run's loads are issued for those lanes with no per-load
	// compare, and a use only compares (bounds check, fault, direct load) when some running
	// lane missed the mask.  Two VALU per hoisted load fewer; EBPF_CC_NORUNMASK=1 keeps the
	// per-load compares (A/B).
	const bool runmask = mode == 0 && getenv("EBPF_CC_NORUNMASK") == nullptr;
	std::vector<uint32_t> run_ext(n, 0); // run head: the largest off + size of its hoisted loads
	const int hoist_regs = AH_GEN_HOIST_REGS;
	const int slot_regs = 2;
	if (mode == 0 && hoist_regs > 0 && getenv("EBPF_CC_NOHOIST") == nullptr) {
		size_t k = 0;
		while (k < order.size()) {
			size_t j = k; // run [k, j]
			auto breaks_after = [&](uint32_t e) {
				const int fam = ah_fam[(uint32_t)low[e].handler];
				// (letting runs continue past conditionals along the fall-through edge, loads
				// issued for lanes that branch away, measured 3% slower on C5)
				return (ah_flags[(uint32_t)low[e].handler] & 1) || fam == AHF_EXIT ||
				       fam == AHF_FAULT || fam == AHF_LOOKUPGEN ||
				       (fam >= AHF_STXGEN1 && fam <= AHF_STXGEN8) ||
				       (fam >= AHF_STGEN1 && fam <= AHF_STGEN8) || is_value_store_fam(fam);
			};
			while (j + 1 < order.size() && !breaks_after(order[j]) &&
			       xl.entries[order[j]].next == order[j + 1] && !entry_point[order[j + 1]])
				j++;
			// the run's loads, issued through a ring of 2-VGPR slots: the first `slots` at the
			// run head, load i + slots right after load i is consumed (its slot is free again)
			std::vector<uint32_t> ld;
			for (size_t q = k; q <= j; q++) {
				const uint32_t e = order[q];
				const int fam = ah_fam[(uint32_t)low[e].handler];
				if (fam < AHF_LDXPKTG1 || fam > AHF_LDXPKTG8)
					continue;
				const int z = 1 << (fam - AHF_LDXPKTG1);
				if (low[e].imm + (uint64_t)z > 4095u)
					continue;
				ld.push_back(e);
			}
			if (ld.size() >= 2) {
				const size_t slots = (size_t)(hoist_regs / slot_regs);
				size_t issued = std::min(slots, ld.size());
				hoist_at[order[k]].assign(ld.begin(), ld.begin() + issued);
				for (uint32_t x : ld)
					run_ext[order[k]] = std::max<uint32_t>(
					    run_ext[order[k]],
					    (uint32_t)low[x].imm + (1u << (ah_fam[(uint32_t)low[x].handler] - AHF_LDXPKTG1)));
				for (size_t i = 0; i < ld.size(); i++) {
					hoist_tmp[ld[i]] = (int16_t)(AH_GEN_HOIST_BASE + slot_regs * (i % slots));
					hoist_later[ld[i]] = (uint16_t)(issued - 1 - i);
					if (i + slots < ld.size()) {
						hoist_next[ld[i]] = ld[i + slots];
						issued++;
					}
				}
			}
			k = j + 1;
		}
	}
	std::vector<uint16_t> uses(n, 0), live_out(n, 0xffff);
	std::vector<int8_t> defreg(n, -1);
	std::vector<char> pure(n, 0);
	uint16_t live_start = 0x7ff;
	const unsigned off = cc_off() | (structured ? 16u : 0u); // structured: compares leave VCC
	// general kernels (parking scheduler, no join SGPRs): s[74:75] is free for the short-lane
	// mask of the inline header loads (ldxpkc_general)
	const bool gen_short_mask = mode == 0 && !structured && !AH_GEN_JOIN &&
				    getenv("EBPF_CC_NOSHORT") == nullptr;
	bool uses_short_mask = false;

	for (int pass = 0; pass < 2; pass++) {
		const bool final_pass = pass == 1;
		out.assign(n, cc_block());
		std::vector<facts> in(n);
		std::vector<char> have(n, 0);
		if (xl.start < n) {
			facts f0; // r0, r2..r9 are zero at the start (the kernel, or the prologue below)
			for (int r = 0; r < AH_NREGS; r++) {
				f0.r[r] = (r == 1 || r == 10) ? rf() : kconst(0);
				f0.pv[r] = (live_start & (1u << r)) != 0;
			}
			in[xl.start] = f0;
			have[xl.start] = 1;
		}
		std::vector<char> fused(n, 0); // a BSWAP folded into the preceding packet load
		std::vector<int8_t> movfuse_src(n, -1);  // this entry reads a fused MOV's source
		std::vector<int16_t> movfuse_fam(n, -1); // ... as this 32-bit operation
		for (size_t k = 0; k < order.size(); k++) {
			const uint32_t e = order[k];
			const bool valid = have[e] && npred[e] == (e == xl.start ? 0u : 1u);
			facts f = valid ? in[e] : facts();
			if (!valid)
				for (bool &p : f.pv)
					p = true;
			cc_block &blk = out[e];
			const uint32_t h = (uint32_t)low[e].handler;
			const int fam = ah_fam[h], d = ah_dst[h], s = ah_src[h];
			const uint64_t K = low[e].imm;
			uint32_t aux0, aux1;
			memcpy(&aux0, reinterpret_cast<const uint8_t *>(&low[e]) + 24, 4);
			memcpy(&aux1, reinterpret_cast<const uint8_t *>(&low[e]) + 28, 4);
			f.nofwd = (off & 4) != 0;
			const facts before = f;
			emitter em(blk, f, maps);
			em.off = off;
			bool break_mov = false;
			// issue packet load x into its ring slot, for the lanes whose packet holds it
			// (masked: exec is already the lanes to load for, the run head's batch)
			auto issue = [&](enc &Hq, uint32_t x, bool masked = false) {
				const int S_JUNK_ = 60, V_LEN = 40, V_PKT = 38;
				const int fx = ah_fam[(uint32_t)low[x].handler];
				const int z = 1 << (fx - AHF_LDXPKTG1);
				const uint32_t K32 = (uint32_t)low[x].imm;
				static const uint32_t gop[4] = {0x10, 0x12, 0x14, 0x15};
				if (masked) {
				} else if (runmask) {
					Hq.sop1(0x20, S_JUNK_, opnd{(uint32_t)AH_S_RUNMASK}); // s_and_saveexec_b64
				} else {
					Hq.vopc(VC_U32 + P_LE, k32(K32 + (uint32_t)z), V_LEN); // vcc = off+z <= len
					Hq.sop1(0x20, S_JUNK_, opnd{SRC_VCC});                  // s_and_saveexec_b64
				}
				Hq.w(0xdc008000u | (gop[fx - AHF_LDXPKTG1] << 18) | K32);      // global_load_*
				Hq.w((uint32_t)V_PKT | (0x7fu << 16) | ((uint32_t)hoist_tmp[x] << 24));
				if (!masked)
					Hq.sop1(0x01, 126, opnd{(uint32_t)S_JUNK_});       // s_mov_b64 exec
			};
			if (!hoist_at[e].empty()) {
				enc Hq{blk.hoist};
				if (runmask) { // s[76:77] = the running lanes whose packet holds every load of the run
					Hq.vopc(VC_U32 + P_LE, k32(run_ext[e]), 40); // vcc = ext <= len (v40)
					Hq.sop1(0x01, AH_S_RUNMASK, opnd{SRC_VCC});    // s_mov_b64
					Hq.sop1(0x20, 60, opnd{SRC_VCC});            // s_and_saveexec_b64 s[60:61]
					for (uint32_t x : hoist_at[e])
						issue(Hq, x, true);
					Hq.sop1(0x01, 126, opnd{60u});               // s_mov_b64 exec, s[60:61]
				} else {
					for (uint32_t x : hoist_at[e])
						issue(Hq, x);
				}
			}
			bool ok = true, spec_map = false;
			// a 32-bit MOV d = s whose only successor operates on d with an immediate: the
			// successor reads s directly and the MOV emits nothing (one VALU move saved)
			if (fam == AHF_A32R_MOV && d != s && d < AH_NREGS && s < AH_NREGS && !(off & 1)) {
				const uint32_t nx = xl.entries[e].next;
				if (nx < n && k + 1 < order.size() && order[k + 1] == nx && !entry_point[nx] &&
				    npred[nx] == 1 && hoist_tmp[nx] < 0) {
					const uint32_t h2 = (uint32_t)low[nx].handler;
					const int f2 = ah_fam[h2];
					const uint32_t K2 = (uint32_t)low[nx].imm;
					int as32 = -1;
					if (ah_dst[h2] == d && f2 >= AHF_A32I_ADD && f2 <= AHF_A32I_RSH && f2 != AHF_A32I_MUL)
						as32 = f2; // (ADD, SUB, OR, AND, XOR, LSH, RSH: see alu32i)
					else if (ah_dst[h2] == d && f2 == AHF_A64I_RSH && K2 < 32)
						as32 = AHF_A32I_RSH; // (u32 >> c)
					else if (ah_dst[h2] == d && f2 == AHF_A64I_LSH && K2 < 32 &&
						 std::min(32, bits_of(f.r[s])) + (int)K2 <= 32)
						as32 = AHF_A32I_LSH; // (the result still fits 32 bits)
					if (as32 >= 0 && as32 != AHF_A32I_MUL && as32 != AHF_A32I_MOV) {
						movfuse_src[nx] = (int8_t)s;
						movfuse_fam[nx] = (int16_t)as32;
						em.use(s);
						break_mov = true;
					}
				}
			}
			if (break_mov) {
				// (nothing emitted; d keeps its old facts until the fused operation defines it)
			} else if (movfuse_src[e] >= 0) {
				ok = em.alu32i(movfuse_fam[e], d, (uint32_t)K, movfuse_src[e]);
			} else if (hoist_tmp[e] >= 0) {
				em.ldx_hoisted(d, 1 << (fam - AHF_LDXPKTG1), (uint32_t)K, hoist_tmp[e], hoist_later[e],
					       rt.fault, runmask);
				if (hoist_next[e] != UINT32_MAX)
					issue(em.E, hoist_next[e]);
			}
			switch ((hoist_tmp[e] >= 0 || break_mov || movfuse_src[e] >= 0) ? -1 : fam) {
			case -1: break;
			case AHF_NOP: break;
			case AHF_EXIT:
				if (f.r[0].c && !(off & 32))
					em.exit_known(f.r[0].v, rt.exit_k, structured);
				else if (structured && getenv("EBPF_CC_EXITCALL") == nullptr)
					em.exit_inline();
				else if (structured)
					em.call_routine(rt.exit, 1);
				else
					ok = false;
				break;
			case AHF_FAULT:
				if (structured)
					em.fault(aux0, rt.fault);
				else
					ok = false;
				break;
			case AHF_A64I_MOV: em.mov64(d, K); break;
			case AHF_A64I_ADD: em.add64i(d, K); break;
			case AHF_A64I_OR: em.or64i(d, K); break;
			case AHF_A64I_XOR: em.xor64i(d, K); break;
			case AHF_A64I_AND: em.and64i(d, K); break;
			case AHF_A64I_LSH: em.lsh64i(d, (uint32_t)K); break;
			case AHF_A64I_RSH: em.rsh64i(d, (uint32_t)K); break;
			case AHF_A64I_MUL: em.mul64i(d, K); break;
			case AHF_BSWAP16:
			case AHF_BSWAP32:
				if (fused[e]) {
					em.use(d); // the value the fused load produced
					break;
				}
				ok = em.bswap(fam, d);
				break;
			case AHF_LDXPKC1: case AHF_LDXPKC2: case AHF_LDXPKC4: case AHF_LDXPKC8: {
				if (mode == 0) { // general kernels: length checks against the short-lane mask
					ok = gen_short_mask && s + (1 << (fam - AHF_LDXPKC1)) <= 64;
					if (ok) {
						em.ldxpkc_general(d, 1 << (fam - AHF_LDXPKC1), s, rt.fault);
						uses_short_mask = true;
					}
					break;
				}
				const int z = 1 << (fam - AHF_LDXPKC1);
				int swap = 0;
				const uint32_t nx = xl.entries[e].next;
				if (mode == 1 && z <= 4 && nx < n && k + 1 < order.size() && order[k + 1] == nx &&
				    !entry_point[nx] && npred[nx] == 1) {
					const uint32_t h2 = (uint32_t)low[nx].handler;
					const int f2 = ah_fam[h2];
					if ((f2 == AHF_BSWAP16 || f2 == AHF_BSWAP32) && ah_dst[h2] == d) {
						swap = f2 == AHF_BSWAP16 ? 2 : 4;
						fused[nx] = 1;
					}
				}
				em.ldxpkc(d, z, s, swap);
				break;
			}
			case AHF_LDXPKTV1: case AHF_LDXPKTV2: case AHF_LDXPKTV4: case AHF_LDXPKTV8: {
				const int z = 1 << (fam - AHF_LDXPKTV1);
				const int64_t Ks = (int64_t)K;
				ok = mode == 1 && Ks >= 0 && Ks <= 64 - z && d < AH_NREGS && s < AH_NREGS &&
				     getenv("EBPF_CC_NOPKTV") == nullptr;
				if (ok) {
					em.ldxpktv_staged(d, s, z, (uint32_t)Ks, (int)h);
					em.used |= copied_uses(fam, d, s); // (the spliced slow path's reads)
				}
				break;
			}
			case AHF_STXSTK1: case AHF_STXSTK2: case AHF_STXSTK4: case AHF_STXSTK8:
				if (K + 8 <= 255 * 4)
					em.stxstk(1 << (fam - AHF_STXSTK1), d, (uint32_t)K);
				else
					ok = false;
				break;
			case AHF_LDXSTK1: case AHF_LDXSTK2: case AHF_LDXSTK4: case AHF_LDXSTK8:
				if (K + 8 <= 255 * 4)
					em.ldxstk(1 << (fam - AHF_LDXSTK1), d, (uint32_t)K);
				else
					ok = false;
				break;
			case AHF_LOOKUPSTK: {
				int mi = -1;
				for (size_t t = 0; t < maps.size(); t++)
					if (maps[t].dev_base == K && maps[t].max_entries == low[e].target &&
					    maps[t].value_size == aux1)
						mi = (int)t;
				ok = !(off & 8) && em.lookup_stk(mi, aux0);
				break;
			}
			case AHF_LDXMAP1: case AHF_LDXMAP2: case AHF_LDXMAP4: case AHF_LDXMAP8:
				ok = spec_map = em.ldxmap(1 << (fam - AHF_LDXMAP1), d, s, K);
				break;
			case AHF_HLOOKUP: {
				// (an inline jhash + home-slot probe, round 3, measured 3% slower than the
				// generic routine on C4H and was retired in round 5)
				const int mi = (int)(aux0 / 32);
				ok = false;
				// the generic routine, whose probe of a key of <= 8 bytes also loads the
				// slot's first 8 value bytes (v[50:51], gen_interp.py hlookup_routine): they
				// are kept in a register D dead from here on, so that loads through the
				// result (LDXHV) become register extracts (one memory round trip less)
				if (!ok && final_pass && mi < (int)table.size() && (table[mi].flags & DP_MAP_HASH) &&
				    dp_hash_key_size(table[mi].flags) <= 8 && getenv("EBPF_CC_NOHFWD") == nullptr) {
					// D must also be free of every fact that reads its VGPRs through another name
					// (a stack word forwarded from D, a map pointer indexed by D): dropping such a
					// fact here, where the pass that computed liveness kept it, changes the facts
					// downstream (a load forwarded there, a constant exit, dead code removed for
					// it) — found by the hashtable fuzz mode
					auto aliased = [&](int r) {
						for (uint8_t i = 0; i < f.nst; i++)
							if (f.st[i].reg == r)
								return true;
						for (int q = 0; q < AH_NREGS; q++)
							if (f.r[q].mreg == r)
								return true;
						return false;
					};
					int D = -1;
					for (int r = 9; r >= 2 && D < 0; r--)
						if (!(live_out[e] & (1u << r)) && !aliased(r))
							D = r;
					if (D >= 0) {
						blk.reads |= (uint8_t)(1u << 4); // s14 = the map record offset
						blk.sval[4] = aux0;
						em.use(2);
						em.call_routine(rt.hlookup, 0);
						em.E.vop1(V1_MOV_B64, 2 * D, vreg(50));
						f.def(0, rf());
						// (D's value facts stay: the liveness that picked D was computed with
						// them, so a compare they decided must stay decided — dropping them
						// made such a compare read D's VGPRs, now the forwarded value; with D
						// unaliased, clobber_phys drops nothing else)
						f.clobber_phys(D);
						f.r[0].hfwd = (int8_t)D;
						f.t2zero = false;
						ok = true;
					}
				}
				break;
			}
			case AHF_LDXHV1: case AHF_LDXHV2: case AHF_LDXHV4: case AHF_LDXHV8:
				ok = em.ldxhv_fwd(1 << (fam - AHF_LDXHV1), d, s, (int32_t)aux0);
				break;
			default:
				if (fam >= AHF_A32I_ADD && fam <= AHF_A32I_MOD)
					ok = em.alu32i(fam, d, (uint32_t)K);
				else if (fam >= AHF_A32R_ADD && fam <= AHF_A32R_MOD)
					ok = em.alu32r(fam, d, s);
				else if (fam >= AHF_A64R_ADD && fam <= AHF_A64R_MOD)
					ok = em.alu64r(fam, d, s);
				else if (fam >= AHF_JEQ_I && fam <= AHF_JSET_I)
					em.cond_imm(fam - AHF_JEQ_I, d, K);
				else if (fam >= AHF_JEQ_R && fam <= AHF_JSET_R)
					em.cond_reg(fam - AHF_JEQ_R, d, s);
				else if (fam >= AHF_J32EQ_I && fam <= AHF_J32SET_I)
					em.cond32_imm(fam - AHF_J32EQ_I, d, (uint32_t)K);
				else if (fam >= AHF_J32EQ_R && fam <= AHF_J32SET_R)
					em.cond32_reg(fam - AHF_J32EQ_R, d, s);
				else if (fam == AHF_MOV64R)
					em.copy64(d, s);
				else
					ok = false;
			}
			const int wr = written_reg(fam, d);
			if (ok) {
				blk.fast = true;
			} else {
				// the interpreter's body; the facts of what it writes are lost
				f = before;
				f.t2zero = false; // (handler bodies use v46..v51 freely)
				blk.fast = false;
				blk.body.clear();
				blk.splice_h = -1;
				blk.reads = 0;
				em.used = copied_uses(fam, d, s);
				if (wr >= 0)
					f.def(wr, copied_result(fam));
				// stores through unknown pointers may hit the stack
				if (fam >= AHF_STXGEN1 && fam <= AHF_STXGEN8)
					f.nst = 0;
				if ((fam >= AHF_STGEN1 && fam <= AHF_STGEN8) || is_value_store_fam(fam))
					f.nst = 0;
				if (fam >= AHF_STSTK1 && fam <= AHF_STSTK8)
					f.store(aux0, 1 << (fam - AHF_STSTK1), -1);
			}
			if (!final_pass) {
				uses[e] = em.used;
				defreg[e] = (int8_t)wr;
				pure[e] = (char)(pure_fam(fam, spec_map) && wr >= 0 &&
						 !(mode == 0 && fam >= AHF_LDXPKC1 && fam <= AHF_LDXPKC8));
			} else if (!(off & 1) && pure[e] && wr >= 0 && !(live_out[e] & (1u << wr))) {
				// dead: no code, the register's VGPRs do not hold the (unused) value
				blk.fast = true;
				blk.body.clear();
				blk.splice_h = -1;
				blk.reads = 0;
				f.pv[wr] = false;
				f.t2zero = before.t2zero; // (its code, which may have zeroed v48, is gone)
			}
			// successors
			if (fam == AHF_EXIT || fam == AHF_FAULT)
				continue;
			const uint32_t nx = xl.entries[e].next;
			const bool is_cond = (ah_flags[h] & 1) != 0;
			auto give = [&](uint32_t to, const facts &fo) {
				if (to >= n)
					return;
				in[to] = fo;
				have[to] = 1;
			};
			if (is_cond) {
				const uint32_t tk = xl.entries[e].target;
				const bool c64 = fam <= AHF_JSET_I; // (JMP32 edges refine nothing)
				const int c = fam >= AHF_JEQ_I ? fam - AHF_JEQ_I : fam - AHF_JEQ_R;
				const bool cimm = fam >= AHF_JEQ_I || f.r[s].c;
				const uint64_t cv = fam >= AHF_JEQ_I ? K : f.r[s].v;
				facts ft = f, fn = f;
				if (c64 && cimm && d < AH_NREGS) {
					refine(ft, c, d, cv, true);
					refine(fn, c, d, cv, false);
				}
				give(tk, ft);
				give(nx, fn);
			} else {
				give(nx, f);
			}
		}
		if (final_pass) {
			// the group set-up the kernel leaves to compiled programs: the packet address
			// (staged mode; the generic memory routines and r1 read it), r1, r10 and the
			// zeroing of r0, r2..r9 — each only if something reads it
			bool needs_pkt = (live_start & (1u << 1)) != 0;
			for (uint32_t e : order) {
				const int fam = ah_fam[(uint32_t)low[e].handler];
				if (!out[e].fast &&
				    ((fam >= AHF_LDXGEN1 && fam <= AHF_STXGEN8) || (fam >= AHF_LDXPKTG1 && fam <= AHF_LDXPKTG8) ||
				     (fam >= AHF_STGEN1 && fam <= AHF_STGEN8) || fam == AHF_LOOKUPGEN ||
				     is_value_store_fam(fam) || fam == AHF_UPDATE || fam == AHF_HDELETE))
					needs_pkt = true;
				// (compiled LDXPKTV reads the packet address too, and so does its spliced slow path)
				if (fam >= AHF_LDXPKTV1 && fam <= AHF_LDXPKTV8)
					needs_pkt = true;
			}
			// Dead stack stores: when no code of the program can read its stack frame — every
			// block is one of the families below, stack loads all forwarded from registers,
			// lookups compiled with their key in a register — the stores into the frame are
			// never observed, and emit nothing (C4: the key STXW, one LDS write per packet).
			// Anything that may read the frame (generic or run-time-offset loads, the lookup,
			// update and delete routines, hashtable probes, counters through pointers, a
			// copied handler body of a load or a lookup) keeps every store.
			if (getenv("EBPF_CC_KEEPSTORES") == nullptr) {
				bool frame_read = false;
				for (uint32_t e : order) {
					const int fam = ah_fam[(uint32_t)low[e].handler];
					const bool pure = (fam >= AHF_A64R_ADD && fam <= AHF_JSET_R) ||
							  (fam >= AHF_A64I_ADD && fam <= AHF_JSET_I) ||
							  (fam >= AHF_MOV64R && fam <= AHF_J32SET_I) ||
							  (fam >= AHF_STXSTK1 && fam <= AHF_STXSTK8) ||
							  (fam >= AHF_STSTK1 && fam <= AHF_STSTK8) ||
							  (fam >= AHF_LDXPKTG1 && fam <= AHF_LDXPKTG8) ||
							  (fam >= AHF_LDXPKC1 && fam <= AHF_LDXPKC8) ||
							  fam == AHF_LDXPKBE16 || fam == AHF_LDXPKBE32 || fam == AHF_EXIT ||
							  fam == AHF_FAULT || fam == AHF_NOP || fam == AHF_LOOPINIT ||
							  fam == AHF_LOOPCNT || fam == AHF_OVLINIT;
					const bool fast_ok = out[e].fast && !out[e].stack_read &&
							     ((fam >= AHF_LDXMAP1 && fam <= AHF_LDXMAP8) ||
							      (fam >= AHF_LDXSTK1 && fam <= AHF_LDXSTK8) || fam == AHF_LOOKUPSTK);
					if (!pure && !fast_ok) {
						frame_read = true;
						break;
					}
				}
				if (!frame_read)
					for (uint32_t e : order) {
						const int fam = ah_fam[(uint32_t)low[e].handler];
						if ((fam >= AHF_STXSTK1 && fam <= AHF_STXSTK8) ||
						    (fam >= AHF_STSTK1 && fam <= AHF_STSTK8)) {
							out[e].fast = true;
							out[e].body.clear();
							out[e].splice_h = -1;
							out[e].reads = 0;
						}
					}
			}
			if (xl.start < n) {
				cc_prologue(mode, live_start, needs_pkt, structured, out[xl.start].prologue);
				if (uses_short_mask) { // s[74:75] = lanes whose packet is shorter than 64 B
					enc P{out[xl.start].prologue};
					P.vop3(VC_U32 + P_GT, 74, 128 + 64, VGPR0 + 40, 0);
				}
			}
			break;
		}
		// liveness (backward over the tree: children come after their parent in `order`)
		std::vector<uint16_t> live_in(n, 0);
		for (size_t k = order.size(); k-- > 0;) {
			const uint32_t e = order[k];
			const uint32_t h = (uint32_t)low[e].handler;
			const int fam = ah_fam[h];
			uint16_t lo = 0;
			if (fam != AHF_EXIT && fam != AHF_FAULT) {
				const uint32_t nx = xl.entries[e].next;
				if (nx < n)
					lo |= npred[nx] == 1 ? live_in[nx] : 0x7ff;
				if ((ah_flags[h] & 1) && xl.entries[e].target < n) {
					const uint32_t tk = xl.entries[e].target;
					lo |= npred[tk] == 1 ? live_in[tk] : 0x7ff;
				}
			}
			live_out[e] = lo;
			uint16_t li = lo;
			if (defreg[e] >= 0 && !(uses[e] & (1u << defreg[e])))
				li &= (uint16_t)~(1u << defreg[e]);
			if (pure[e] && defreg[e] >= 0 && !(lo & (1u << defreg[e])))
				li = lo; // a dead pure operation reads nothing
			else
				li |= uses[e];
			live_in[e] = li;
		}
		live_start = xl.start < n ? live_in[xl.start] : 0x7ff;
		if (off & 3)
			live_start = 0x7ff;
	}
}
