// asm_cc.cpp — optimising gfx950 code generation for compiled programs (variant 0).
//
// asm_jit.cpp lays a lowered program (asm_lower) out as straight-line code and, for each entry,
// used to copy the interpreter's handler body verbatim.  Handler bodies are written for any
// register contents, so they pay for 64-bit generality everywhere: a 32-bit result re-zeroes
// its high half, a 64-bit multiply by a 32-bit constant multiplies by a zero high word, a
// compare of a loaded byte is a 64-bit compare against an SGPR pair set by two scalar moves.
//
// Here a forward dataflow over the state tree tracks, for every eBPF register, whether it holds
// a known constant and how many of its leading bits are known zero (the translator's tree gives
// every entry exactly one predecessor, so the facts are exact per path; taken/not-taken edges of
// compares against constants refine them).  With those facts the hot families are emitted as
// hand-encoded gfx950 instructions instead of the generic body:
//   * constants fold (both operands known: a move of the result);
//   * high halves known zero are neither recomputed nor re-zeroed;
//   * 64-bit AND/OR/XOR/shift by constants become 32-bit operations where a half is unchanged
//     or zero, shifts by >= 32 become moves;
//   * MUL by a constant drops the partial products of known-zero words (3 → 2 or 1 quarter-rate
//     multiplies), multiplies by powers of two become shifts;
//   * compares of values below 2^32 against constants below 2^32 are single VOPC e32
//     instructions with the constant as a literal (no scalar moves); statically decided
//     compares become VCC = EXEC or 0;
//   * a staged packet load followed by BE16/BE32 of the same register is one v_perm_b32 that
//     picks the bytes in network order straight from the staged packet registers.
// Everything else (memory through pointers, lookups, division, exits, faults) still copies the
// interpreter's handler body, so semantics there are unchanged by construction.
//
// Encodings: VOP1/VOP2/VOPC (e32, literal allowed in src0), VOP3 (no literal on gfx9), SOP1.
// Field layouts and opcodes were taken from llvm-mc -show-encoding for gfx950;
// tests/test_compile.py disassembles the generated code to check them.
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
	V2_CNDMASK = 0x00, V2_LSHRREV_B32 = 0x10, V2_ASHRREV_I32 = 0x11, V2_LSHLREV_B32 = 0x12,
	V2_AND = 0x13, V2_OR = 0x14, V2_XOR = 0x15, V2_ADD_CO = 0x19, V2_SUB_CO = 0x1a,
	V2_ADDC_CO = 0x1c, V2_SUBB_CO = 0x1d, V2_ADD_U32 = 0x34, V2_SUB_U32 = 0x35, V2_SUBREV_U32 = 0x36,
};
// VOP1 opcodes (bits 16:9)
enum : uint32_t { V1_MOV_B32 = 0x01, V1_NOT_B32 = 0x2b, V1_MOV_B64 = 0x38 };
// VOP3 opcodes (bits 25:16)
enum : uint32_t {
	V3_BFE_U32 = 0x1c8, V3_ALIGNBYTE = 0x1cf, V3_MAD_U64_U32 = 0x1e8, V3_PERM_B32 = 0x1ed,
	V3_ADD3_U32 = 0x1ff, V3_LSHL_ADD_U64 = 0x208, V3_MUL_LO_U32 = 0x285, V3_LSHLREV_B64 = 0x28f,
	V3_LSHRREV_B64 = 0x290,
};
// VOPC compare codes: base + {lt 1, eq 2, le 3, gt 4, ne 5, ge 6}
enum : uint32_t { VC_I32 = 0xc0, VC_U32 = 0xc8, VC_I64 = 0xe0, VC_U64 = 0xe8 };
enum { P_LT = 1, P_EQ = 2, P_LE = 3, P_GT = 4, P_NE = 5, P_GE = 6 };
const int S_JUNK = 60; // s[60:61]: carry-out sink of v_mad_u64_u32 (gen_interp.py S_JUNK)
const int T0 = 46, T1 = 47, T2 = 48, T3 = 49; // handler temporaries (gen_interp.py H)
const int PKT0 = 22;                          // staged packet dwords v22..v37
const int V_SEL = 63;                          // v63 = 0x00010203 (byte reversal selector)

// a source operand: 9-bit code, plus the literal when code == SRC_LIT
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

// 32-bit constant for an e32 src0: inline constant or literal
opnd
k32(uint32_t v)
{
	uint32_t c;
	if (inline_i64((int64_t)(int32_t)v, &c))
		return opnd{c};
	return opnd{SRC_LIT, v};
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
		w((0x34u << 26) | (op << 16) | ((uint32_t)sdst << 8) | (uint32_t)vdst);
		w(s0 | (s1 << 9) | (s2 << 18));
	}
	// s_mov_b64 vcc, exec | 0
	void vcc_all(bool all) { w(0xbe800000u | (SRC_VCC << 16) | (0x01u << 8) | (all ? SRC_EXEC : 128u)); }
};

// ---------------------------------------------------------------- facts
struct rf {
	bool c = false;  // known constant
	uint64_t v = 0;
	uint8_t lz = 0;  // known leading zero bits (64 if c && v == 0)
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

struct facts {
	rf r[AH_NREGS];
};

// ---------------------------------------------------------------- per-entry emission
struct emitter {
	cc_block &blk;
	enc E;
	facts &f;
	int next_s = 0; // constant SGPR allocation: s10/s11 (pair), s13, s14, s15

	emitter(cc_block &b, facts &fa) : blk(b), E{b.body}, f(fa) {}

	static int L(int r) { return 2 * r; }
	static int Hi(int r) { return 2 * r + 1; }
	bool hz(int r) const { return f.r[r].lz >= 32; }

	// an SGPR holding the 32-bit constant v for this body (s13, s14, s15)
	uint32_t sconst(uint32_t v)
	{
		static const int regs[3] = {13, 14, 15};
		for (int i = 0; i < 3; i++) {
			const int r = regs[i];
			if ((blk.reads & (1u << (r - 10))) && blk.sval[r - 10] == v)
				return (uint32_t)r;
		}
		for (int i = 0; i < 3; i++) {
			const int r = regs[i];
			if (!(blk.reads & (1u << (r - 10)))) {
				blk.reads |= (uint8_t)(1u << (r - 10));
				blk.sval[r - 10] = v;
				return (uint32_t)r;
			}
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
	// VOP3 source for a 32-bit constant
	uint32_t c3(uint32_t v)
	{
		uint32_t c;
		if (inline_i64((int64_t)(int32_t)v, &c))
			return c;
		return sconst(v);
	}
	// VOP3 / VOPC source for a 64-bit constant
	uint32_t c64(uint64_t v)
	{
		uint32_t c;
		if (inline_i64((int64_t)v, &c))
			return c;
		return spair(v);
	}

	void mov32(int vd, uint32_t v) { E.vop1(V1_MOV_B32, vd, k32(v)); }
	void hi0(int d)
	{
		if (!hz(d))
			mov32(Hi(d), 0);
	}
	// d = v (a constant), skipping halves already known to hold it
	void mov64(int d, uint64_t v)
	{
		const rf &o = f.r[d];
		const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
		if (!(o.c && (uint32_t)o.v == lo))
			mov32(L(d), lo);
		if (!((o.c && (uint32_t)(o.v >> 32) == hi) || (hi == 0 && hz(d))))
			mov32(Hi(d), hi);
		f.r[d] = kconst(v);
	}
	// d = s (registers)
	void copy64(int d, int s)
	{
		if (d == s)
			return;
		if (f.r[s].c) {
			mov64(d, f.r[s].v);
			return;
		}
		if (hz(s)) {
			E.vop1(V1_MOV_B32, L(d), vreg(L(s)));
			hi0(d);
		} else {
			E.vop1(V1_MOV_B64, L(d), vreg(L(s)));
		}
		f.r[d] = f.r[s];
	}

	// ---- ALU64 with a constant operand (d op= K)
	void add64i(int d, uint64_t K)
	{
		rf &x = f.r[d];
		if (K == 0)
			return;
		if (x.c) {
			mov64(d, x.v + K);
			return;
		}
		E.vop3(V3_LSHL_ADD_U64, L(d), c64(K), 128, VGPR0 + L(d));
		x = (int64_t)K >= 0 ? kbits(std::max(bits_of(x), 64 - clz64(K)) + 1) : rf();
	}
	void or64i(int d, uint64_t K)
	{
		rf &x = f.r[d];
		if (x.c) {
			mov64(d, x.v | K);
			return;
		}
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo)
			E.vop2(V2_OR, L(d), k32(lo), L(d));
		if (hi == 0xffffffffu)
			mov32(Hi(d), hi);
		else if (hi)
			E.vop2(V2_OR, Hi(d), k32(hi), Hi(d));
		x = kbits(std::max(bits_of(x), 64 - clz64(K)));
	}
	void xor64i(int d, uint64_t K)
	{
		rf &x = f.r[d];
		if (x.c) {
			mov64(d, x.v ^ K);
			return;
		}
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo)
			E.vop2(V2_XOR, L(d), k32(lo), L(d));
		if (hi)
			E.vop2(V2_XOR, Hi(d), k32(hi), Hi(d));
		x = kbits(std::max(bits_of(x), 64 - clz64(K)));
	}
	void and64i(int d, uint64_t K)
	{
		rf &x = f.r[d];
		if (x.c) {
			mov64(d, x.v & K);
			return;
		}
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		if (lo == 0)
			mov32(L(d), 0);
		else if (lo != 0xffffffffu)
			E.vop2(V2_AND, L(d), k32(lo), L(d));
		if (hi == 0)
			hi0(d);
		else if (hi != 0xffffffffu && !hz(d))
			E.vop2(V2_AND, Hi(d), k32(hi), Hi(d));
		x = kbits(std::min(bits_of(x), 64 - clz64(K)));
	}
	void lsh64i(int d, uint32_t c)
	{
		c &= 63;
		rf &x = f.r[d];
		if (c == 0)
			return;
		if (x.c) {
			mov64(d, x.v << c);
			return;
		}
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
		x = kbits(nb);
	}
	void rsh64i(int d, uint32_t c)
	{
		c &= 63;
		rf &x = f.r[d];
		if (c == 0)
			return;
		if (x.c) {
			mov64(d, x.v >> c);
			return;
		}
		const int nb = std::max(0, bits_of(x) - (int)c);
		if (nb == 0) {
			mov64(d, 0);
			return;
		}
		if (c >= 32) {
			if (c == 32)
				E.vop1(V1_MOV_B32, L(d), vreg(Hi(d)));
			else
				E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + (c - 32)}, Hi(d));
			hi0(d);
		} else if (hz(d)) {
			E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + c}, L(d));
		} else {
			E.vop3(V3_LSHRREV_B64, L(d), 128 + c, VGPR0 + L(d), 0);
		}
		f.r[d] = kbits(nb);
	}
	void mul64i(int d, uint64_t K)
	{
		rf &x = f.r[d];
		if (x.c) {
			mov64(d, x.v * K);
			return;
		}
		if (K == 0) {
			mov64(d, 0);
			return;
		}
		if (K == 1)
			return;
		if ((K & (K - 1)) == 0) {
			lsh64i(d, (uint32_t)__builtin_ctzll(K));
			return;
		}
		const int nb = std::min(64, bits_of(x) + 64 - clz64(K));
		const uint32_t lo = (uint32_t)K, hi = (uint32_t)(K >> 32);
		const uint32_t klo = c3(lo);
		if (hz(d) && hi == 0) {
			// d < 2^32: the full 64-bit product of two 32-bit words
			E.vop3(V3_MAD_U64_U32, T0, VGPR0 + L(d), klo, 128, S_JUNK);
			E.vop1(V1_MOV_B64, L(d), vreg(T0));
		} else if (hi == 0) {
			E.vop3(V3_MUL_LO_U32, T2, VGPR0 + Hi(d), klo, 0);
			E.vop3(V3_MAD_U64_U32, T0, VGPR0 + L(d), klo, 128, S_JUNK);
			E.vop2(V2_ADD_U32, Hi(d), vreg(T1), T2);
			E.vop1(V1_MOV_B32, L(d), vreg(T0));
		} else if (hz(d)) {
			E.vop3(V3_MUL_LO_U32, T2, VGPR0 + L(d), c3(hi), 0);
			E.vop3(V3_MAD_U64_U32, T0, VGPR0 + L(d), klo, 128, S_JUNK);
			E.vop2(V2_ADD_U32, Hi(d), vreg(T1), T2);
			E.vop1(V1_MOV_B32, L(d), vreg(T0));
		} else {
			E.vop3(V3_MUL_LO_U32, T2, VGPR0 + L(d), c3(hi), 0);
			E.vop3(V3_MUL_LO_U32, T3, VGPR0 + Hi(d), klo, 0);
			E.vop3(V3_MAD_U64_U32, T0, VGPR0 + L(d), klo, 128, S_JUNK);
			E.vop3(V3_ADD3_U32, Hi(d), VGPR0 + T1, VGPR0 + T2, VGPR0 + T3);
			E.vop1(V1_MOV_B32, L(d), vreg(T0));
		}
		x = kbits(nb);
	}

	// ---- ALU32 (lo op= k; hi = 0)
	bool alu32i(int fam, int d, uint32_t k)
	{
		rf &x = f.r[d];
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
		switch (fam) {
		case AHF_A32I_ADD:
			if (k)
				E.vop2(V2_ADD_U32, L(d), k32(k), L(d));
			nb = k ? std::min(32, std::max(ab, 32 - __builtin_clz(k)) + 1) : ab;
			break;
		case AHF_A32I_SUB:
			if (k)
				E.vop2(V2_SUBREV_U32, L(d), k32(k), L(d));
			nb = k ? 32 : ab;
			break;
		case AHF_A32I_MUL:
			E.vop3(V3_MUL_LO_U32, L(d), VGPR0 + L(d), c3(k), 0);
			nb = k ? std::min(32, ab + 32 - __builtin_clz(k)) : 0;
			break;
		case AHF_A32I_OR:
			if (k)
				E.vop2(V2_OR, L(d), k32(k), L(d));
			nb = std::max(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_AND:
			if (k != 0xffffffffu)
				E.vop2(V2_AND, L(d), k32(k), L(d));
			nb = std::min(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_XOR:
			if (k)
				E.vop2(V2_XOR, L(d), k32(k), L(d));
			nb = std::max(ab, k ? 32 - __builtin_clz(k) : 0);
			break;
		case AHF_A32I_LSH:
			if (k & 31)
				E.vop2(V2_LSHLREV_B32, L(d), opnd{128 + (k & 31)}, L(d));
			nb = std::min(32, ab + (int)(k & 31));
			break;
		case AHF_A32I_RSH:
			if (k & 31)
				E.vop2(V2_LSHRREV_B32, L(d), opnd{128 + (k & 31)}, L(d));
			nb = std::max(0, ab - (int)(k & 31));
			break;
		default:
			return false;
		}
		hi0(d);
		x = kbits(nb);
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
		rf &x = f.r[d];
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
		if (d == s && (fam == AHF_A32R_SUB || fam == AHF_A32R_XOR))
			nb = 0;
		hi0(d);
		x = kbits(nb);
		return true;
	}
	bool alu64r(int fam, int d, int s)
	{
		const rf xs = f.r[s];
		rf &x = f.r[d];
		if (d == s) {
			switch (fam) {
			case AHF_A64R_ADD: lsh64i(d, 1); return true;
			case AHF_A64R_SUB: case AHF_A64R_XOR: mov64(d, 0); return true;
			case AHF_A64R_OR: case AHF_A64R_AND: return true;
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
			E.vop3(V3_LSHL_ADD_U64, L(d), VGPR0 + L(s), 128, VGPR0 + L(d));
			x = kbits(std::min(64, std::max(bits_of(x), bits_of(xs)) + 1));
			return true;
		case AHF_A64R_OR:
		case AHF_A64R_XOR: {
			const uint32_t op = fam == AHF_A64R_OR ? V2_OR : V2_XOR;
			E.vop2(op, L(d), vreg(L(s)), L(d));
			if (!hz(s))
				E.vop2(op, Hi(d), vreg(Hi(s)), Hi(d));
			x = kbits(std::max(bits_of(x), bits_of(xs)));
			return true;
		}
		case AHF_A64R_AND:
			E.vop2(V2_AND, L(d), vreg(L(s)), L(d));
			if (hz(s))
				hi0(d);
			else if (!hz(d))
				E.vop2(V2_AND, Hi(d), vreg(Hi(s)), Hi(d));
			x = kbits(std::min(bits_of(x), bits_of(xs)));
			return true;
		default:
			return false;
		}
	}

	// ---- byte swaps (BE16/BE32 zero-extend; LE is lowered to AND)
	bool bswap(int fam, int d)
	{
		rf &x = f.r[d];
		if (fam == AHF_BSWAP16) {
			if (x.c) {
				mov64(d, __builtin_bswap16((uint16_t)x.v));
				return true;
			}
			E.vop3(V3_PERM_B32, L(d), 128, VGPR0 + L(d), sconst(0x0c0c0001u));
			hi0(d);
			x = kbits(16);
			return true;
		}
		if (fam == AHF_BSWAP32) {
			if (x.c) {
				mov64(d, __builtin_bswap32((uint32_t)x.v));
				return true;
			}
			E.vop3(V3_PERM_B32, L(d), 128, VGPR0 + L(d), VGPR0 + V_SEL);
			hi0(d);
			x = kbits(32);
			return true;
		}
		return false;
	}

	// ---- staged packet load at constant offset `off`, size z; swap_bytes = 0, 2 or 4 (a fused
	// BE16 / BE32 of the loaded register)
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
			f.r[d] = kbits(8 * std::min(z, swap_bytes));
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
			f.r[d] = rf();
			return;
		}
		hi0(d);
		f.r[d] = kbits(8 * z);
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
	// predicate of `d c x`, and of `x c' d` (operands swapped)
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
	void cond_imm(int c, int d, uint64_t K)
	{
		const rf &x = f.r[d];
		if (x.c) {
			E.vcc_all(eval(c, x.v, K));
			return;
		}
		if (c == 10) { // JSET
			const uint32_t lo = (uint32_t)K, hi = hz(d) ? 0u : (uint32_t)(K >> 32);
			if (!lo && !hi) {
				E.vcc_all(false);
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
				case 2: case 3: r = false; break;       // d > K (unsigned): K >= 2^32 > d
				case 4: case 5: r = true; break;
				case 6: case 7: r = kneg; break;        // d > K (signed)
				default: r = !kneg; break;              // d < K (signed)
				}
				E.vcc_all(r);
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
};

// registers a copied handler body may write
int
written_reg(int fam, int d)
{
	switch (fam) {
	case AHF_LOOKUPSTK:
	case AHF_LOOKUPGEN:
		return 0;
	case AHF_EXIT: case AHF_FAULT: case AHF_NOP:
	case AHF_STXGEN1: case AHF_STXGEN2: case AHF_STXGEN4: case AHF_STXGEN8:
	case AHF_STXSTK1: case AHF_STXSTK2: case AHF_STXSTK4: case AHF_STXSTK8:
	case AHF_STGEN1: case AHF_STGEN2: case AHF_STGEN4: case AHF_STGEN8:
	case AHF_STSTK1: case AHF_STSTK2: case AHF_STSTK4: case AHF_STSTK8:
		return -1;
	default:
		if (fam >= AHF_JEQ_R && fam <= AHF_JSET_R)
			return -1;
		if (fam >= AHF_JEQ_I && fam <= AHF_JSET_I)
			return -1;
		return d < AH_NREGS ? d : -1;
	}
}

// facts for a copied body's result
rf
copied_result(int fam)
{
	switch (fam) {
	case AHF_LDXGEN1: case AHF_LDXMAP1: case AHF_LDXPKTG1: case AHF_LDXSTK1: return kbits(8);
	case AHF_LDXGEN2: case AHF_LDXMAP2: case AHF_LDXPKTG2: case AHF_LDXSTK2: return kbits(16);
	case AHF_LDXGEN4: case AHF_LDXMAP4: case AHF_LDXPKTG4: case AHF_LDXSTK4: return kbits(32);
	default:
		if (fam >= AHF_A32R_ADD && fam <= AHF_A32R_MOD)
			return kbits(32);
		if (fam >= AHF_A32I_ADD && fam <= AHF_A32I_MOD)
			return kbits(32);
		return rf();
	}
}

// refine facts on the taken (taken = true) or fall-through edge of `d c K`
void
refine(facts &fa, int c, int d, uint64_t K, bool taken)
{
	rf &x = fa.r[d];
	if (x.c)
		return;
	// equality
	if ((c == 0 && taken) || (c == 1 && !taken)) {
		x = kconst(K);
		return;
	}
	// unsigned upper bounds: d <= B
	uint64_t B;
	bool ub = false;
	if ((c == 5 && taken) || (c == 2 && !taken)) { // d <= K
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
cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
	   const std::vector<char> &entry_point, int mode, std::vector<cc_block> &out)
{
	const size_t n = low.size();
	out.assign(n, cc_block());
	// predecessors (the tree gives one; shared fault entries and anything unexpected get none of
	// the facts)
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
	std::vector<facts> in(n);
	std::vector<char> have(n, 0);
	{
		facts f0; // the kernels zero r0, r2..r9 per group; r1 = packet, r10 = stack (unknown)
		for (int r = 0; r < AH_NREGS; r++)
			f0.r[r] = (r == 1 || r == 10) ? rf() : kconst(0);
		if (xl.start < n) {
			in[xl.start] = f0;
			have[xl.start] = 1;
		}
	}
	std::vector<char> fused(n, 0); // a BSWAP folded into the preceding packet load
	for (size_t k = 0; k < order.size(); k++) {
		const uint32_t e = order[k];
		// exact facts need the one predecessor (the start state: none)
		const bool valid = have[e] && npred[e] == (e == xl.start ? 0u : 1u);
		facts f = valid ? in[e] : facts();
		cc_block &blk = out[e];
		const uint32_t h = (uint32_t)low[e].handler;
		const int fam = ah_fam[h], d = ah_dst[h], s = ah_src[h];
		const uint64_t K = low[e].imm;
		emitter em(blk, f);
		bool ok = true;
		switch (fam) {
		case AHF_NOP: break;
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
			if (fused[e])
				break;
			ok = em.bswap(fam, d);
			break;
		case AHF_LDXPKC1: case AHF_LDXPKC2: case AHF_LDXPKC4: case AHF_LDXPKC8: {
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
			else
				ok = false;
		}
		if (ok) {
			blk.fast = true;
		} else {
			// the interpreter's body; the facts of what it writes are lost
			blk.fast = false;
			blk.body.clear();
			blk.reads = 0;
			const int wr = written_reg(fam, d);
			if (wr >= 0)
				f.r[wr] = copied_result(fam);
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
			const int c = fam >= AHF_JEQ_I ? fam - AHF_JEQ_I : fam - AHF_JEQ_R;
			const bool cimm = fam >= AHF_JEQ_I || f.r[s].c;
			const uint64_t cv = fam >= AHF_JEQ_I ? K : f.r[s].v;
			facts ft = f, fn = f;
			if (cimm && d < AH_NREGS) {
				refine(ft, c, d, cv, true);
				refine(fn, c, d, cv, false);
			}
			give(tk, ft);
			give(nx, fn);
		} else {
			give(nx, f);
		}
	}
}
