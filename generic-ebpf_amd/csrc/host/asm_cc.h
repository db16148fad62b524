// asm_cc.h — optimising code generation for compiled programs (asm_cc.cpp), used by asm_jit.cpp.
#pragma once
#include <stdint.h>

#include <vector>

#include "internal.h"

// One entry's code.  fast: `body` is complete code for the entry, needing the scalar operand
// registers s(10+r) for each bit r of `reads` set to sval[r] before it; otherwise the compiler
// copies the interpreter's handler body (ah_reads / the lowered operands, as before).
// Conditional entries leave VCC = the lanes taking the branch (unless sdir >= 0: no code
// decides, the compiler falls through or jumps).
// prologue: code placed before everything else of the block (the start block's register
// zeroing: compiled programs zero only the registers they read before writing).
struct cc_block {
	bool fast = false;
	uint8_t reads = 0;
	uint32_t sval[6] = {};
	std::vector<uint8_t> body;
	std::vector<uint8_t> prologue;
	int8_t sdir = -1; // conditional decided at compile time: 0 never taken, 1 always taken
};

// low: the lowered entries (asm_lower); order: the layout order (depth-first, parents first);
// entry_point[e]: e can be entered other than by falling through from its layout predecessor.
// mode 1 = staged 64-B packets (packet loads read v22..v37).  exitk_off: offset of the
// .Lr_exit_k routine from .Lcb (EXIT with a known r0).  table: the program's maps.
void cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
		const std::vector<char> &entry_point, int mode, uint32_t exitk_off,
		const std::vector<dp_map> &table, std::vector<cc_block> &out);

// The group set-up a compiled program does itself (the kernel jumps straight to it): the packet
// address (staged mode), r1 = packet, r10 = stack top, zeroes for r0, r2..r9 — the registers in
// `live` (bit r), the packet address also if `needs_pkt` (generic memory routines read it).
void cc_prologue(int mode, uint16_t live, bool needs_pkt, std::vector<uint8_t> &out);
