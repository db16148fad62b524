// interp_cpu.cpp — ebpf_prog_run: the single-packet entry point of the drop-in API.
//
// Replaces sys/dev/ebpf/ebpf_interpreter.c:23-372 for callers that run ONE packet per call on
// their own thread (a GPU launch costs microseconds; one packet costs ~20 ns on a CPU core, see
// SURVEY.md §3(E)).  Batches go to the GPU through ebpf_gpu.h; nothing in the batch path falls
// back to this function.
//
// Semantics are the reference's, quirks included: cumulative stepping (:39), 32-bit ops on
// truncated operands, MOV64 = add (:197-202), NEG ignores dst (:89-91), NEG64 = dst - imm
// (:182-184), logical ARSH (:110-115, :203-208), x86-masked shift counts, raw pointer memory
// access, CALL through the env helper table (:282-284), abort on an invalid opcode (:367-369).
// Instead of a 90-way switch it dispatches through a table of handlers indexed by opcode,
// built once.
//
// EBPF_SEM_STANDARD programs (ebpf_prog_set_semantics) run on a second table: sequential pc,
// MOV64 / NEG / NEG64 / ARSH with their standard meaning, DIV/MOD by zero defined (0 / dst
// unchanged) and the JMP32 class.  Same dispatch loop with `inst = prog + pc++`.
#include "internal.h"

#include <stdio.h>

namespace {

struct cpu_vm {
	uint64_t reg[EBPF_REG_MAX];
	const struct ebpf_inst *inst;
	uint32_t pc;
	const struct ebpf_helper_type *const *helpers;
};

using handler_fn = bool (*)(cpu_vm &, const struct ebpf_inst &); // false = EXIT

inline uint64_t &D(cpu_vm &v, const struct ebpf_inst &i) { return v.reg[i.dst]; }
inline uint64_t S(cpu_vm &v, const struct ebpf_inst &i) { return v.reg[i.src]; }
inline uint64_t SX(const struct ebpf_inst &i) { return (uint64_t)(int64_t)i.imm; }
inline uint32_t U(const struct ebpf_inst &i) { return (uint32_t)i.imm; }

template <typename T> inline T ld(uint64_t a) { T v; memcpy(&v, (const void *)(uintptr_t)a, sizeof v); return v; }
template <typename T> inline void st(uint64_t a, T v) { memcpy((void *)(uintptr_t)a, &v, sizeof v); }

#define H(name, body) \
	bool name(cpu_vm &v, const struct ebpf_inst &i) { body; return true; }

// ALU32: operands truncated to 32 bits, result zero-extended
H(add32r, D(v, i) = (uint32_t)((uint32_t)D(v, i) + (uint32_t)S(v, i)))
H(add32i, D(v, i) = (uint32_t)((uint32_t)D(v, i) + U(i)))
H(sub32r, D(v, i) = (uint32_t)((uint32_t)D(v, i) - (uint32_t)S(v, i)))
H(sub32i, D(v, i) = (uint32_t)((uint32_t)D(v, i) - U(i)))
H(mul32r, D(v, i) = (uint32_t)((uint32_t)D(v, i) * (uint32_t)S(v, i)))
H(mul32i, D(v, i) = (uint32_t)((uint32_t)D(v, i) * U(i)))
H(div32r, D(v, i) = (uint32_t)D(v, i) / (uint32_t)S(v, i))
H(div32i, D(v, i) = (uint32_t)D(v, i) / U(i))
H(or32r, D(v, i) = (uint32_t)D(v, i) | (uint32_t)S(v, i))
H(or32i, D(v, i) = (uint32_t)D(v, i) | U(i))
H(and32r, D(v, i) = (uint32_t)D(v, i) & (uint32_t)S(v, i))
H(and32i, D(v, i) = (uint32_t)D(v, i) & U(i))
H(lsh32r, D(v, i) = (uint32_t)((uint32_t)D(v, i) << (S(v, i) & 31)))
H(lsh32i, D(v, i) = (uint32_t)((uint32_t)D(v, i) << (U(i) & 31)))
H(rsh32r, D(v, i) = (uint32_t)D(v, i) >> (S(v, i) & 31))
H(rsh32i, D(v, i) = (uint32_t)D(v, i) >> (U(i) & 31))
H(neg32, D(v, i) = (uint32_t)(0u - U(i)))
H(mod32r, D(v, i) = (uint32_t)D(v, i) % (uint32_t)S(v, i))
H(mod32i, D(v, i) = (uint32_t)D(v, i) % U(i))
H(xor32r, D(v, i) = (uint32_t)D(v, i) ^ (uint32_t)S(v, i))
H(xor32i, D(v, i) = (uint32_t)D(v, i) ^ U(i))
H(mov32r, D(v, i) = (uint32_t)S(v, i))
H(mov32i, D(v, i) = U(i))
H(le, if (i.imm == 16) D(v, i) = (uint16_t)D(v, i); else if (i.imm == 32) D(v, i) = (uint32_t)D(v, i))
H(be, if (i.imm == 16) D(v, i) = __builtin_bswap16((uint16_t)D(v, i));
      else if (i.imm == 32) D(v, i) = __builtin_bswap32((uint32_t)D(v, i));
      else if (i.imm == 64) D(v, i) = __builtin_bswap64(D(v, i)))
// ALU64
H(add64r, D(v, i) += S(v, i))
H(add64i, D(v, i) += SX(i))
H(sub64r, D(v, i) -= S(v, i))
H(sub64i, D(v, i) -= SX(i))
H(mul64r, D(v, i) *= S(v, i))
H(mul64i, D(v, i) *= SX(i))
H(div64r, D(v, i) /= S(v, i))
H(div64i, D(v, i) /= SX(i))
H(or64r, D(v, i) |= S(v, i))
H(or64i, D(v, i) |= SX(i))
H(and64r, D(v, i) &= S(v, i))
H(and64i, D(v, i) &= SX(i))
H(lsh64r, D(v, i) <<= (S(v, i) & 63))
H(lsh64i, D(v, i) <<= (SX(i) & 63))
H(rsh64r, D(v, i) >>= (S(v, i) & 63))
H(rsh64i, D(v, i) >>= (SX(i) & 63))
H(neg64, D(v, i) -= SX(i))
H(mod64r, D(v, i) %= S(v, i))
H(mod64i, D(v, i) %= SX(i))
H(xor64r, D(v, i) ^= S(v, i))
H(xor64i, D(v, i) ^= SX(i))
// memory
H(ldxb, D(v, i) = ld<uint8_t>(S(v, i) + (uint64_t)(int64_t)i.offset))
H(ldxh, D(v, i) = ld<uint16_t>(S(v, i) + (uint64_t)(int64_t)i.offset))
H(ldxw, D(v, i) = ld<uint32_t>(S(v, i) + (uint64_t)(int64_t)i.offset))
H(ldxdw, D(v, i) = ld<uint64_t>(S(v, i) + (uint64_t)(int64_t)i.offset))
H(stb, st<uint8_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint8_t)i.imm))
H(sth, st<uint16_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint16_t)i.imm))
H(stw, st<uint32_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint32_t)i.imm))
H(stdw, st<uint64_t>(D(v, i) + (uint64_t)(int64_t)i.offset, SX(i)))
H(stxb, st<uint8_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint8_t)S(v, i)))
H(stxh, st<uint16_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint16_t)S(v, i)))
H(stxw, st<uint32_t>(D(v, i) + (uint64_t)(int64_t)i.offset, (uint32_t)S(v, i)))
H(stxdw, st<uint64_t>(D(v, i) + (uint64_t)(int64_t)i.offset, S(v, i)))
H(lddw, D(v, i) = (uint64_t)U(i) | ((uint64_t)(uint32_t)(&i + 1)->imm << 32); v.pc++)
// jumps: taken → pc += offset (u32 arithmetic)
#define J(name, cond) H(name, if (cond) v.pc += (uint32_t)(int32_t)i.offset)
J(ja, true)
J(jeqr, D(v, i) == S(v, i))
J(jeqi, D(v, i) == SX(i))
J(jgtr, D(v, i) > S(v, i))
J(jgti, D(v, i) > SX(i))
J(jger, D(v, i) >= S(v, i))
J(jgei, D(v, i) >= SX(i))
J(jsetr, (D(v, i) & S(v, i)) != 0)
J(jseti, (D(v, i) & SX(i)) != 0)
J(jner, D(v, i) != S(v, i))
J(jnei, D(v, i) != SX(i))
J(jsgtr, (int64_t)D(v, i) > (int64_t)S(v, i))
J(jsgti, (int64_t)D(v, i) > (int64_t)SX(i))
J(jsger, (int64_t)D(v, i) >= (int64_t)S(v, i))
J(jsgei, (int64_t)D(v, i) >= (int64_t)SX(i))
J(jltr, D(v, i) < S(v, i))
J(jlti, D(v, i) < SX(i))
J(jler, D(v, i) <= S(v, i))
J(jlei, D(v, i) <= SX(i))
J(jsltr, (int64_t)D(v, i) < (int64_t)S(v, i))
J(jslti, (int64_t)D(v, i) < (int64_t)SX(i))
J(jsler, (int64_t)D(v, i) <= (int64_t)S(v, i))
J(jslei, (int64_t)D(v, i) <= (int64_t)SX(i))
H(call, v.reg[0] = v.helpers[i.imm]->fn(v.reg[1], v.reg[2], v.reg[3], v.reg[4], v.reg[5]))
bool exit_(cpu_vm &, const struct ebpf_inst &) { return false; }
// standard semantics (where they differ from the reference's)
H(mov64r_std, D(v, i) = S(v, i))
H(mov64i_std, D(v, i) = SX(i))
H(neg32_std, D(v, i) = (uint32_t)(0u - (uint32_t)D(v, i)))
H(neg64_std, D(v, i) = 0 - D(v, i))
H(arsh32r_std, D(v, i) = (uint32_t)((int32_t)(uint32_t)D(v, i) >> (S(v, i) & 31)))
H(arsh32i_std, D(v, i) = (uint32_t)((int32_t)(uint32_t)D(v, i) >> (U(i) & 31)))
H(arsh64r_std, D(v, i) = (uint64_t)((int64_t)D(v, i) >> (S(v, i) & 63)))
H(arsh64i_std, D(v, i) = (uint64_t)((int64_t)D(v, i) >> (SX(i) & 63)))
H(div32r_std, D(v, i) = (uint32_t)S(v, i) ? (uint32_t)D(v, i) / (uint32_t)S(v, i) : 0)
H(div32i_std, D(v, i) = U(i) ? (uint32_t)D(v, i) / U(i) : 0)
H(mod32r_std, D(v, i) = (uint32_t)S(v, i) ? (uint32_t)D(v, i) % (uint32_t)S(v, i) : (uint32_t)D(v, i))
H(mod32i_std, D(v, i) = U(i) ? (uint32_t)D(v, i) % U(i) : (uint32_t)D(v, i))
H(div64r_std, D(v, i) = S(v, i) ? D(v, i) / S(v, i) : 0)
H(div64i_std, D(v, i) = SX(i) ? D(v, i) / SX(i) : 0)
H(mod64r_std, if (S(v, i)) D(v, i) %= S(v, i))
H(mod64i_std, if (SX(i)) D(v, i) %= SX(i))
inline uint32_t D32(cpu_vm &v, const struct ebpf_inst &i) { return (uint32_t)v.reg[i.dst]; }
inline uint32_t S32(cpu_vm &v, const struct ebpf_inst &i) { return (uint32_t)v.reg[i.src]; }
J(jeq32r, D32(v, i) == S32(v, i))
J(jeq32i, D32(v, i) == U(i))
J(jgt32r, D32(v, i) > S32(v, i))
J(jgt32i, D32(v, i) > U(i))
J(jge32r, D32(v, i) >= S32(v, i))
J(jge32i, D32(v, i) >= U(i))
J(jset32r, (D32(v, i) & S32(v, i)) != 0)
J(jset32i, (D32(v, i) & U(i)) != 0)
J(jne32r, D32(v, i) != S32(v, i))
J(jne32i, D32(v, i) != U(i))
J(jsgt32r, (int32_t)D32(v, i) > (int32_t)S32(v, i))
J(jsgt32i, (int32_t)D32(v, i) > (int32_t)U(i))
J(jsge32r, (int32_t)D32(v, i) >= (int32_t)S32(v, i))
J(jsge32i, (int32_t)D32(v, i) >= (int32_t)U(i))
J(jlt32r, D32(v, i) < S32(v, i))
J(jlt32i, D32(v, i) < U(i))
J(jle32r, D32(v, i) <= S32(v, i))
J(jle32i, D32(v, i) <= U(i))
J(jslt32r, (int32_t)D32(v, i) < (int32_t)S32(v, i))
J(jslt32i, (int32_t)D32(v, i) < (int32_t)U(i))
J(jsle32r, (int32_t)D32(v, i) <= (int32_t)S32(v, i))
J(jsle32i, (int32_t)D32(v, i) <= (int32_t)U(i))
bool invalid(cpu_vm &v, const struct ebpf_inst &)
{
	fprintf(stderr, "Invalid instruction at PC %u\n", v.pc);
	abort();
}

struct table {
	handler_fn f[256];
	table()
	{
		for (auto &x : f)
			x = invalid;
		const struct { uint8_t op; handler_fn fn; } ops[] = {
		    {0x0c, add32r}, {0x04, add32i}, {0x1c, sub32r}, {0x14, sub32i}, {0x2c, mul32r},
		    {0x24, mul32i}, {0x3c, div32r}, {0x34, div32i}, {0x4c, or32r}, {0x44, or32i},
		    {0x5c, and32r}, {0x54, and32i}, {0x6c, lsh32r}, {0x64, lsh32i}, {0x7c, rsh32r},
		    {0x74, rsh32i}, {0x84, neg32}, {0x9c, mod32r}, {0x94, mod32i}, {0xac, xor32r},
		    {0xa4, xor32i}, {0xbc, mov32r}, {0xb4, mov32i}, {0xcc, rsh32r}, {0xc4, rsh32i},
		    {0xd4, le}, {0xdc, be},
		    {0x0f, add64r}, {0x07, add64i}, {0x1f, sub64r}, {0x17, sub64i}, {0x2f, mul64r},
		    {0x27, mul64i}, {0x3f, div64r}, {0x37, div64i}, {0x4f, or64r}, {0x47, or64i},
		    {0x5f, and64r}, {0x57, and64i}, {0x6f, lsh64r}, {0x67, lsh64i}, {0x7f, rsh64r},
		    {0x77, rsh64i}, {0x87, neg64}, {0x9f, mod64r}, {0x97, mod64i}, {0xaf, xor64r},
		    {0xa7, xor64i}, {0xbf, add64r}, {0xb7, add64i}, {0xcf, rsh64r}, {0xc7, rsh64i},
		    {0x71, ldxb}, {0x69, ldxh}, {0x61, ldxw}, {0x79, ldxdw}, {0x72, stb}, {0x6a, sth},
		    {0x62, stw}, {0x7a, stdw}, {0x73, stxb}, {0x6b, stxh}, {0x63, stxw}, {0x7b, stxdw},
		    {0x18, lddw}, {0x05, ja}, {0x1d, jeqr}, {0x15, jeqi}, {0x2d, jgtr}, {0x25, jgti},
		    {0x3d, jger}, {0x35, jgei}, {0x4d, jsetr}, {0x45, jseti}, {0x5d, jner}, {0x55, jnei},
		    {0x6d, jsgtr}, {0x65, jsgti}, {0x7d, jsger}, {0x75, jsgei}, {0xad, jltr},
		    {0xa5, jlti}, {0xbd, jler}, {0xb5, jlei}, {0xcd, jsltr}, {0xc5, jslti},
		    {0xdd, jsler}, {0xd5, jslei}, {0x85, call}, {0x95, exit_},
		};
		for (const auto &o : ops)
			f[o.op] = o.fn;
	}
};

const table k_table;

struct std_table : table {
	std_table()
	{
		const struct { uint8_t op; handler_fn fn; } ops[] = {
		    {0xbf, mov64r_std}, {0xb7, mov64i_std}, {0x84, neg32_std}, {0x87, neg64_std},
		    {0xcc, arsh32r_std}, {0xc4, arsh32i_std}, {0xcf, arsh64r_std}, {0xc7, arsh64i_std},
		    {0x3c, div32r_std}, {0x34, div32i_std}, {0x9c, mod32r_std}, {0x94, mod32i_std},
		    {0x3f, div64r_std}, {0x37, div64i_std}, {0x9f, mod64r_std}, {0x97, mod64i_std},
		    {0x16, jeq32i}, {0x1e, jeq32r}, {0x26, jgt32i}, {0x2e, jgt32r}, {0x36, jge32i},
		    {0x3e, jge32r}, {0x46, jset32i}, {0x4e, jset32r}, {0x56, jne32i}, {0x5e, jne32r},
		    {0x66, jsgt32i}, {0x6e, jsgt32r}, {0x76, jsge32i}, {0x7e, jsge32r}, {0xa6, jlt32i},
		    {0xae, jlt32r}, {0xb6, jle32i}, {0xbe, jle32r}, {0xc6, jslt32i}, {0xce, jslt32r},
		    {0xd6, jsle32i}, {0xde, jsle32r},
		};
		for (const auto &o : ops)
			f[o.op] = o.fn;
	}
};

const std_table k_std_table;

} // namespace

EBPF_EXPORT uint64_t
ebpf_prog_run(void *ctx, struct ebpf_prog *ep)
{
	cpu_vm v;
	uint8_t stack[EBPF_STACK_SIZE];
	memset(v.reg, 0, sizeof(v.reg)); // the reference leaves these undefined
	v.reg[1] = (uint64_t)(uintptr_t)ctx;
	v.reg[10] = (uint64_t)(uintptr_t)(stack + EBPF_STACK_SIZE);
	v.helpers = ep->eo.eo_ee->ec->helper_types;
	v.inst = ep->prog;
	v.pc = 0;
	if (ep->semantics.load(std::memory_order_relaxed) == EBPF_SEM_STANDARD) {
		const uint32_t nslots = ep->prog_len / sizeof(struct ebpf_inst);
		for (;;) {
			if (v.pc >= nslots) // (a verifier would have refused the program)
				invalid(v, *ep->prog);
			v.inst = ep->prog + v.pc++;
			if (!k_std_table.f[v.inst->opcode](v, *v.inst))
				return v.reg[0];
		}
	}
	for (;;) {
		v.inst = v.inst + v.pc++;
		if (!k_table.f[v.inst->opcode](v, *v.inst))
			return v.reg[0];
	}
}
