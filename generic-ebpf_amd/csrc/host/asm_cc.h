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
// regroup[e]: e is a regroup point (its code assumes nothing it did not compute itself).
void cc_compile(const dprog_host &xl, const std::vector<dp_entry> &low, const std::vector<uint32_t> &order,
		const std::vector<char> &entry_point, int mode, bool structured, const cc_routines &rt,
		const std::vector<dp_map> &table, const std::vector<char> &regroup,
		std::vector<cc_block> &out);

// Regrouping (gen_interp.py "Regrouping"; general kernels, unstructured compiled programs).
// A regroup point is the head of a subtree that both sides of a divergent conditional make
// heavy and that only computes (ALU, compares, packet loads at constant offsets, exits, faults:
// no stack, map or helper), so its lanes can run it later in another lane with their packet index
// and live registers restored.  cc_regroup_plan picks at most AH_RQ_MAX of them (the deepest,
// none inside another) and returns their live registers (<= 3, ascending), or no point at all
// when fewer than two qualify.
struct cc_regroup_point {
	uint32_t entry;
	std::vector<uint8_t> live;
};
void cc_regroup_plan(const dprog_host &xl, const std::vector<dp_entry> &low,
		     const std::vector<uint32_t> &order, std::vector<cc_regroup_point> &points);

// Path-sorted launches (gpu_runtime.cpp launch_pathsorted; general kernels, compiled programs):
// the cut points of the classifying run — heads of subtrees that both sides of a divergent
// conditional make heavy, the deepest, none inside another, at most max_cuts (the heaviest) —
// whose path from the start holds no store that may reach the packet or a map and no map write.
// Empty when fewer than two qualify.
void cc_pathsort_plan(const dprog_host &xl, const std::vector<dp_entry> &low,
		      const std::vector<uint32_t> &order, uint32_t max_cuts, std::vector<uint32_t> &cuts);

// Bytes of one queue: u32 packet indices [128], then u64 [128] per live-register slot.
inline uint32_t
cc_queue_bytes(uint32_t live_slots)
{
	return 512u + 1024u * live_slots;
}

// Code at the head of regroup point q: queue the running lanes (packet index, `live`) and leave
// the group (jump to the scheduler at sched_off from .Lcb).
void cc_push_code(int q, const std::vector<uint8_t> &live, uint32_t qbytes, uint32_t sched_off,
		  std::vector<uint8_t> &out);

// Window launches (gen_interp.py "Window mode"; span image): code at the head of cut point q,
// class cls = q + 1.  In phase A (s7 bit 12) the running lanes record their class and leave the
// group (.Lr_cut at cut_off from .Lcb); otherwise it falls through (2 SALU).  Cls <= 64.
void cc_cut_code(uint32_t cls, uint32_t cut_off, std::vector<uint8_t> &out);

// The drain code (entered at ebpf_jit_area + 0): run the first queue holding a batch (>= 64
// entries, or any with s7 bit 8) through .Lr_batch (batch_off) and its point's code (resume[q]),
// or return to the kernel (drain_ret_off) when none does.
void cc_drain_code(const std::vector<cc_regroup_point> &points, uint32_t qbytes,
		   const std::vector<uint32_t> &resume, uint32_t batch_off, uint32_t drain_ret_off,
		   std::vector<uint8_t> &out);

// The group set-up a compiled program does itself (the kernel jumps straight to it): the packet
// address (staged mode), r1 = packet, r10 = stack top, zeroes for r0, r2..r9 — the registers in
// `live` (bit r), the packet address also if `needs_pkt` (generic memory routines read it).
// structured: also mark the wave's group as structured (s7 bit 2, read by the exit and fault
// routines).
void cc_prologue(int mode, uint16_t live, bool needs_pkt, bool structured, std::vector<uint8_t> &out);
