// asm_cc.h — optimising code generation for compiled programs (asm_cc.cpp), used by asm_jit.cpp.
#pragma once
#include <stdint.h>

#include <vector>

#include "internal.h"

// One entry's code.  fast: `body` is complete code for the entry, needing the scalar operand
// registers s(10+r) for each bit r of `reads` set to sval[r] before it; otherwise the compiler
// copies the interpreter's handler body (ah_reads / the lowered operands, as before).
// Conditional entries leave VCC = the lanes taking the branch either way.
struct cc_block {
	bool fast = false;
	uint8_t reads = 0;
	uint32_t sval[6] = {};
	std::vector<uint8_t> body;
};

// low: the lowered entries (asm_lower); order: the layout order (depth-first, parents first);
// entry_point[e]: e can be entered other than by falling through from its layout predecessor.
// mode 1 = staged 64-B packets (packet loads read v22..v37).
void cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
		const std::vector<char> &entry_point, int mode, std::vector<cc_block> &out);
