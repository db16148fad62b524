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
	std::vector<uint8_t> hoist; // general kernels: packet loads issued ahead for this straight run
	int8_t sdir = -1; // conditional decided at compile time: 0 never taken, 1 always taken
	bool stack_read = false; // the fast body reads the lane's stack frame (an unforwarded LDX)
	// a fast body with a slow path: the interpreter's handler body `splice_h` (its operands
	// s10, s11 = splice_sval, then an lgkmcnt(0) wait) is inserted at body offset splice_at, and
	// the s_branches at body offsets splice_br[] (over the slow path; ~0 = none) grow by the
	// inserted bytes
	int32_t splice_h = -1;
	uint32_t splice_at = 0, splice_br[2] = {~0u, ~0u};
	uint32_t splice_sval[2] = {};
};

// Offsets from .Lcb of the interpreter routines compiled code calls or jumps to.
struct cc_routines {
	uint32_t exit_k; // EXIT with r0 known (v[44:45], s57 = verdict bin set by the caller)
	uint32_t exit;   // EXIT (r0 in v[0:1])
	uint32_t fault;  // fault the lanes s[48:49] with code s52
	uint32_t hlookup; // HLOOKUP: r0 = hashtable lookup (record offset s14, key at r2)
};

// low: the lowered entries (asm_lower); order: the layout order (depth-first, parents first);
// entry_point[e]: e can be entered other than by falling through from its layout predecessor.
// mode 1 = staged 64-B packets (packet loads read v22..v37).  structured: the program runs with
// structured control flow (asm_jit.cpp): exits and faults are calls that return, compares
// always leave VCC.  table: the program's maps.
// VOP3 instructions emitted with two SGPR sources so far on this thread (must stay 0)
unsigned cc_bus_violations();
void cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
		const std::vector<char> &entry_point, int mode, bool structured, const cc_routines &rt,
		const std::vector<dp_map> &table, std::vector<cc_block> &out);

// The group set-up a compiled program does itself (the kernel jumps straight to it): the packet
// address (staged mode), r1 = packet, r10 = stack top, zeroes for r0, r2..r9 — the registers in
// `live` (bit r), the packet address also if `needs_pkt` (generic memory routines read it).
// structured: also mark the wave's group as structured (s7 bit 2, read by the exit and fault
// routines).
void cc_prologue(int mode, uint16_t live, bool needs_pkt, bool structured, std::vector<uint8_t> &out);
