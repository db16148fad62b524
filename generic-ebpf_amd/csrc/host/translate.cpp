// translate.cpp — reference bytecode → device program (dprog.h).
//
// The reference interpreter's next slot depends on (slot i, counter p):  "inst = inst + pc++"
// (sys/dev/ebpf/ebpf_interpreter.c:39), a taken jump adds its offset to p (:210 etc.) and LDDW
// adds one more (:341).  Starting from (0, 1) — the first fetch is slot 0 with pc already 1 —
//     plain:  (i, p) -> (i + p, p + 1)      LDDW: (i, p) -> (i + p + 1, p + 2)
//     taken:  (i, p) -> (i + p', p' + 1)    with p' = p + off  (u32 arithmetic)
// This file enumerates the reachable states and emits one dp_entry per state with explicit
// successors, so device code never does slot arithmetic.  Straight-line runs are emitted
// contiguously (fallthrough successor = index + 1) and taken sides after them.
//
// Under this rule a state (j, q) has exactly one possible predecessor slot (j - q + 1), so the
// state graph is a tree plus self-loops; a self-loop (a jump whose successor is its own state)
// is the only way the reference spins forever, and becomes an EBPF_FAULT_LOOP entry.
#include "internal.h"

#include <algorithm>
#include <array>

#include <unordered_map>

namespace {

bool
valid_op(uint8_t op)
{
	static const uint8_t ops[] = {
	    0x04, 0x0c, 0x14, 0x1c, 0x24, 0x2c, 0x34, 0x3c, 0x44, 0x4c, 0x54, 0x5c, 0x64, 0x6c,
	    0x74, 0x7c, 0x84, 0x94, 0x9c, 0xa4, 0xac, 0xb4, 0xbc, 0xc4, 0xcc, 0xd4, 0xdc, 0x07,
	    0x0f, 0x17, 0x1f, 0x27, 0x2f, 0x37, 0x3f, 0x47, 0x4f, 0x57, 0x5f, 0x67, 0x6f, 0x77,
	    0x7f, 0x87, 0x97, 0x9f, 0xa7, 0xaf, 0xb7, 0xbf, 0xc7, 0xcf, 0x61, 0x69, 0x71, 0x79,
	    0x62, 0x6a, 0x72, 0x7a, 0x63, 0x6b, 0x73, 0x7b, 0x18, 0x05, 0x15, 0x1d, 0x25, 0x2d,
	    0x35, 0x3d, 0x45, 0x4d, 0x55, 0x5d, 0x65, 0x6d, 0x75, 0x7d, 0x85, 0x95, 0xa5, 0xad,
	    0xb5, 0xbd, 0xc5, 0xcd, 0xd5, 0xdd};
	static bool tab[256];
	static bool init = [] {
		for (uint8_t o : ops)
			tab[o] = true;
		return true;
	}();
	(void)init;
	return tab[op];
}

bool
uses_dst(uint8_t op)
{
	return !(op == EBPF_OP_JA || op == EBPF_OP_CALL || op == EBPF_OP_EXIT);
}

bool
uses_src(uint8_t op)
{
	uint8_t cls = op & 7;
	if (cls == EBPF_CLS_LDX || cls == EBPF_CLS_STX)
		return true;
	if ((cls == EBPF_CLS_ALU || cls == EBPF_CLS_ALU64 || cls == EBPF_CLS_JMP) && (op & 0x08))
		return !(op == EBPF_OP_BE || op == EBPF_OP_CALL || op == EBPF_OP_EXIT);
	return false;
}

constexpr uint32_t kMaxEntries = 1u << 20;

struct Translator {
	const struct ebpf_inst *code;
	uint64_t nslots;
	const struct ebpf_config *ec;
	dprog_host &out;
	std::unordered_map<uint64_t, uint32_t> state_id;
	uint32_t fault_id[EBPF_FAULT_MAX];
	std::vector<std::pair<uint32_t, uint64_t>> pending; // (entry, state) to fill
	std::vector<std::pair<uint32_t, uint64_t>> loop_next; // (LOOPCNT entry, state it leads to)
	bool overflow = false;
	bool std_mode = false; // EBPF_SEM_STANDARD: sequential pc, the state is the slot alone

	Translator(const struct ebpf_inst *c, uint64_t n, const struct ebpf_config *e, dprog_host &o,
		   bool std_sem)
	    : code(c), nslots(n), ec(e), out(o), std_mode(std_sem)
	{
		for (auto &f : fault_id)
			f = UINT32_MAX;
	}

	static uint64_t key(uint64_t idx, uint32_t pc) { return (idx << 32) | pc; }

	uint32_t new_entry()
	{
		if (out.entries.size() >= kMaxEntries) {
			overflow = true;
			return 0;
		}
		dp_entry e;
		memset(&e, 0, sizeof(e));
		out.entries.push_back(e);
		return (uint32_t)(out.entries.size() - 1);
	}

	uint32_t fault(int code)
	{
		if (fault_id[code] == UINT32_MAX) {
			uint32_t id = new_entry();
			out.entries[id].kind = DK_FAULT;
			out.entries[id].aux = (uint16_t)code;
			fault_id[code] = id;
		}
		return fault_id[code];
	}

	// A taken backward jump to slot `idx` (standard semantics): a LOOPCNT entry on the edge,
	// which counts the jump and continues at the target's entry (resolved in run()).
	uint32_t loop_edge(uint64_t idx)
	{
		const uint32_t id = new_entry();
		out.entries[id].kind = DK_LOOPCNT;
		out.has_loops = true;
		if (idx >= nslots) { // (a jump before slot 0 wraps: past the program, not a state key)
			const uint32_t f = fault(EBPF_FAULT_SLOT);
			out.entries[id].next = f;
			return id;
		}
		loop_next.push_back({id, key(idx, 0)});
		return id;
	}

	// Entry for state (idx, pc), following JA chains.  New states are queued for filling.
	uint32_t get(uint64_t idx, uint32_t pc, bool *created)
	{
		*created = false;
		std::vector<uint64_t> aliases;
		uint32_t id = UINT32_MAX;
		for (uint64_t hops = 0;; hops++) {
			if (idx >= nslots) {
				id = fault(EBPF_FAULT_SLOT);
				break;
			}
			auto it = state_id.find(key(idx, pc));
			if (it != state_id.end()) {
				id = it->second;
				break;
			}
			const struct ebpf_inst &in = code[idx];
			if (std_mode && in.opcode == EBPF_OP_JA && hops <= nslots + 2) {
				aliases.push_back(key(idx, pc));
				const uint64_t nidx = idx + 1 + (uint64_t)(int64_t)in.offset;
				if (nidx == idx) {
					id = fault(EBPF_FAULT_LOOP);
					break;
				}
				if (in.offset < 0) { // a backward JA: counted
					id = loop_edge(nidx);
					break;
				}
				idx = nidx;
				continue;
			}
			if (in.opcode == EBPF_OP_JA && hops <= nslots + 2) {
				uint32_t np = pc + (uint32_t)(int32_t)in.offset;
				uint64_t nidx = idx + np;
				aliases.push_back(key(idx, pc));
				if (nidx == idx && np + 1 == pc) {
					id = fault(EBPF_FAULT_LOOP);
					break;
				}
				idx = nidx;
				pc = np + 1;
				continue;
			}
			if (in.opcode == EBPF_OP_JA) { // pathological chain
				id = fault(EBPF_FAULT_LOOP);
				break;
			}
			id = new_entry();
			state_id[key(idx, pc)] = id;
			pending.push_back({id, key(idx, pc)});
			*created = true;
			break;
		}
		for (uint64_t a : aliases)
			state_id[a] = id;
		return id;
	}

	// Standard semantics: entries for the operations whose meaning differs from the reference's
	// (returns true when `e` is complete; its successor is the next slot).
	bool std_rewrite(dp_entry &e, const struct ebpf_inst &in)
	{
		const uint8_t op = in.opcode;
		const uint64_t sx = (uint64_t)(int64_t)in.imm, zx = (uint64_t)(uint32_t)in.imm;
		switch (op) {
		case EBPF_OP_MOV64_IMM: e.kind = EBPF_OP_LDDW; e.imm = sx; return true;
		case EBPF_OP_MOV64_REG: e.kind = DK_MOV64R; return true;
		case EBPF_OP_NEG64: e.kind = DK_NEG64; return true;
		case EBPF_OP_NEG: e.kind = DK_NEG32; return true;
		case EBPF_OP_ARSH64_IMM: e.kind = DK_ARSH64I; e.imm = sx & 63; return true;
		case EBPF_OP_ARSH64_REG: e.kind = DK_ARSH64R; return true;
		case EBPF_OP_ARSH_IMM: e.kind = DK_ARSH32I; e.imm = zx & 31; return true;
		case EBPF_OP_ARSH_REG: e.kind = DK_ARSH32R; return true;
		case EBPF_OP_DIV64_REG: e.kind = DK_DIV64Z; return true;
		case EBPF_OP_MOD64_REG: e.kind = DK_MOD64Z; return true;
		case EBPF_OP_DIV_REG: e.kind = DK_DIV32Z; return true;
		case EBPF_OP_MOD_REG: e.kind = DK_MOD32Z; return true;
		case EBPF_OP_DIV64_IMM: // by a zero immediate: dst = 0
			if (sx != 0)
				return false;
			e.kind = EBPF_OP_LDDW;
			e.imm = 0;
			return true;
		case EBPF_OP_MOD64_IMM: // by a zero immediate: dst unchanged (dst += 0)
			if (sx != 0)
				return false;
			e.kind = EBPF_OP_ADD64_IMM;
			e.imm = 0;
			e.aux = 1; // (not an ADD of the program's: no counter update, fuse_counters)
			return true;
		case EBPF_OP_DIV_IMM: // 32-bit: dst = 0
			if (zx != 0)
				return false;
			e.kind = EBPF_OP_MOV_IMM;
			e.imm = 0;
			return true;
		case EBPF_OP_MOD_IMM: // 32-bit: dst = u32(dst)
			if (zx != 0)
				return false;
			e.kind = EBPF_OP_MOV_REG;
			e.src = e.dst;
			return true;
		default:
			return false;
		}
	}

	static bool valid_jmp32(uint8_t op)
	{
		switch (op & 0xf0) {
		case 0x10: case 0x20: case 0x30: case 0x40: case 0x50: case 0x60: case 0x70:
		case 0xa0: case 0xb0: case 0xc0: case 0xd0:
			return true;
		default:
			return false;
		}
	}

	// Fill one entry; returns the fallthrough successor if it was newly created (so the
	// caller continues the straight-line run), else UINT32_MAX.
	void fill(uint32_t id, uint64_t idx, uint32_t pc, std::vector<uint64_t> &deferred_taken,
		  std::vector<uint32_t> &deferred_taken_entry, uint32_t *next_new)
	{
		*next_new = UINT32_MAX;
		const struct ebpf_inst &in = code[idx];
		uint8_t op = in.opcode;
		dp_entry &e = out.entries[id];
		auto make_fault = [&](int c) {
			dp_entry &x = out.entries[id];
			x.kind = DK_FAULT;
			x.aux = (uint16_t)c;
		};
		const bool jmp32 = std_mode && (op & 7) == DP_CLS_JMP32;
		// XADD (standard semantics only: the reference has no case for it, ebpf_interpreter.c:
		// 367-369): imm BPF_ADD (0) or BPF_ADD | BPF_FETCH (1)
		const bool xadd = std_mode && (op == 0xc3 || op == 0xdb);
		if (jmp32 ? !valid_jmp32(op) : !(valid_op(op) || xadd) || (xadd && in.imm != 0 && in.imm != 1)) {
			make_fault(EBPF_FAULT_BAD_OPCODE);
			return;
		}
		if (jmp32 ? (in.dst >= EBPF_REG_MAX || ((op & 0x08) && in.src >= EBPF_REG_MAX))
			  : ((uses_dst(op) && in.dst >= EBPF_REG_MAX) ||
			     (uses_src(op) && in.src >= EBPF_REG_MAX))) {
			make_fault(EBPF_FAULT_BAD_REG);
			return;
		}
		e.kind = op;
		e.dst = in.dst;
		e.src = in.src;
		e.off = in.offset;
		uint8_t cls = op & 7;
		uint64_t sx = (uint64_t)(int64_t)in.imm;
		uint64_t zx = (uint64_t)(uint32_t)in.imm;
		uint64_t next_idx = std_mode ? idx + 1 : idx + pc;
		uint32_t next_pc = std_mode ? 0 : pc + 1;
		if (std_mode && std_rewrite(e, in)) {
			bool created;
			uint32_t n = get(next_idx, next_pc, &created);
			out.entries[id].next = n;
			if (created)
				*next_new = n;
			return;
		}
		if (jmp32)
			cls = EBPF_CLS_JMP; // (a conditional jump; the entry keeps its class-6 opcode)
		switch (cls) {
		case EBPF_CLS_ALU: {
			uint8_t alu = op & 0xf0;
			if ((alu == EBPF_DIV || alu == EBPF_MOD) && !(op & 0x08) && zx == 0) {
				make_fault(EBPF_FAULT_DIV_ZERO);
				return;
			}
			e.imm = (alu == EBPF_LSH || alu == EBPF_RSH || alu == EBPF_ARSH) && !(op & 0x08)
				    ? (zx & 31)
				    : zx;
			if (op == EBPF_OP_LE || op == EBPF_OP_BE)
				e.imm = sx;
			break;
		}
		case EBPF_CLS_ALU64: {
			uint8_t alu = op & 0xf0;
			if ((alu == EBPF_DIV || alu == EBPF_MOD) && !(op & 0x08) && sx == 0) {
				make_fault(EBPF_FAULT_DIV_ZERO);
				return;
			}
			e.imm = (alu == EBPF_LSH || alu == EBPF_RSH || alu == EBPF_ARSH) && !(op & 0x08)
				    ? (sx & 63)
				    : sx;
			break;
		}
		case EBPF_CLS_LD: // LDDW (the only LD-class opcode dispatched)
			if (idx + 1 >= nslots) {
				make_fault(EBPF_FAULT_SLOT);
				return;
			}
			e.imm = zx | ((uint64_t)(uint32_t)code[idx + 1].imm << 32);
			next_idx = std_mode ? idx + 2 : idx + pc + 1;
			next_pc = std_mode ? 0 : pc + 2;
			break;
		case EBPF_CLS_ST:
			e.imm = sx;
			if (in.dst != EBPF_R10)
				out.writes_memory = true;
			break;
		case EBPF_CLS_STX:
			if (in.dst != EBPF_R10)
				out.writes_memory = true;
			if (xadd) {
				e.kind = DK_XADD;
				e.aux = (uint16_t)((op == 0xdb ? 8 : 4) | (in.imm == 1 ? 0x100 : 0));
				out.writes_memory = true;
			}
			break;
		case EBPF_CLS_LDX:
			break;
		case EBPF_CLS_JMP:
			if (op == EBPF_OP_EXIT)
				return;
			if (op == EBPF_OP_CALL) {
				const struct ebpf_helper_type *h =
				    (in.imm >= 0 && in.imm < EBPF_TYPE_MAX) ? ec->helper_types[in.imm] : nullptr;
				if (h == nullptr) {
					make_fault(EBPF_FAULT_HELPER);
					return;
				}
				if (h == &eht_map_lookup_elem) {
					e.kind = DK_CALL_LOOKUP;
				} else if (h == &eht_map_update_elem || h == &eht_map_delete_elem) {
					// resolved against the map table after the dataflow pass
					e.kind = DK_CALL_UPDATE;
					e.aux = h == &eht_map_delete_elem ? 1 : 0;
				} else {
					make_fault(EBPF_FAULT_HELPER_UNSUPPORTED);
					return;
				}
				break;
			}
			e.imm = jmp32 ? zx : sx;
			{
				uint32_t np = pc + (uint32_t)(int32_t)in.offset;
				uint64_t tidx = std_mode ? idx + 1 + (uint64_t)(int64_t)in.offset : idx + np;
				uint32_t tpc = std_mode ? 0 : np + 1;
				if (tidx == idx && tpc == pc) {
					uint32_t f = fault(EBPF_FAULT_LOOP); // may grow entries: no `e` after this
					out.entries[id].target = f;
				} else if (tidx >= nslots) {
					// (before it becomes a state key: key() keeps 32 bits of the slot, and a
					// taken jump whose u32 pc wrapped lands 2^32 slots on — past the program)
					uint32_t f = fault(EBPF_FAULT_SLOT);
					out.entries[id].target = f;
				} else if (std_mode && in.offset < 0) {
					const uint32_t c = loop_edge(tidx); // (grows entries too)
					out.entries[id].target = c;
				} else {
					deferred_taken.push_back(key(tidx, tpc));
					deferred_taken_entry.push_back(id);
				}
			}
			break;
		default:
			make_fault(EBPF_FAULT_BAD_OPCODE);
			return;
		}
		bool created;
		uint32_t n = get(next_idx, next_pc, &created);
		out.entries[id].next = n;
		if (created)
			*next_new = n;
	}

	int run()
	{
		bool created;
		out.start = get(0, 1, &created);
		std::vector<uint64_t> dt;
		std::vector<uint32_t> dte;
		size_t pi = 0, di = 0, li = 0;
		while (!overflow) {
			// pending entries are processed in creation order; a straight run is filled
			// eagerly so fallthrough successors get consecutive indices.
			if (pi < pending.size()) {
				uint32_t id = pending[pi].first;
				uint64_t k = pending[pi].second;
				pi++;
				uint32_t nn;
				fill(id, k >> 32, (uint32_t)k, dt, dte, &nn);
				continue;
			}
			if (li < loop_next.size()) {
				const uint32_t from = loop_next[li].first;
				const uint64_t k = loop_next[li].second;
				li++;
				out.entries[from].next = get(k >> 32, (uint32_t)k, &created);
				continue;
			}
			if (di >= dt.size())
				break;
			uint64_t k = dt[di];
			uint32_t from = dte[di];
			di++;
			out.entries[from].target = get(k >> 32, (uint32_t)k, &created);
		}
		// A conditional jump of offset 0 goes to the same state taken or not (reference: pc += 0
		// leaves the next state (idx + pc, pc + 1) unchanged, ebpf_interpreter.c:209-211;
		// standard: pc + 1 + 0).  Its compare has no effect, so it becomes ADD64 dst, 0: the
		// state graph keeps one edge per entry (the device's structured control flow and every
		// pass that walks the tree rely on that; fuzz_gpu.py --standard found it).
		for (dp_entry &x : out.entries) {
			const uint8_t cls = x.kind < 0x100 ? (x.kind & 7) : 0xff;
			if ((cls == EBPF_CLS_JMP || cls == DP_CLS_JMP32) && x.kind != EBPF_OP_JA &&
			    x.kind != EBPF_OP_CALL && x.kind != EBPF_OP_EXIT && x.target == x.next) {
				x.kind = EBPF_OP_ADD64_IMM;
				x.imm = 0;
				x.src = 0;
				x.off = 0;
				x.aux = 1; // (not an ADD of the program's: no counter update, fuse_counters)
			}
		}
		if (!overflow && out.has_loops) { // every lane's loop count starts at 0
			const uint32_t init = new_entry();
			out.entries[init].kind = DK_LOOPINIT;
			out.entries[init].next = out.start;
			out.start = init;
		}
		if (overflow) {
			out.error = E2BIG;
			out.error_msg = "program state graph exceeds the device translation limit";
			return E2BIG;
		}
		return 0;
	}
};

// ---------------------------------------------------------------- pointer-provenance dataflow
av
mk(uint8_t kind, int64_t off = 0, int16_t map = -1)
{
	av a;
	a.kind = kind;
	a.off = off;
	a.map = map;
	return a;
}

bool
is_ptr(const av &a)
{
	return a.kind == AV_CTX || a.kind == AV_STACK || a.kind == AV_MAPVAL;
}

// a number (a constant or an AV_SCALAR): nothing in it came from a pointer
bool
is_num(const av &a)
{
	return a.kind == AV_CONST || a.kind == AV_SCALAR;
}

// dst + src for ADD64 / MOV64 (which adds, ebpf_interpreter.c:197-202)
av
add_av(const av &d, const av &s)
{
	if (d.kind == AV_CONST && s.kind == AV_CONST)
		return mk(AV_CONST, (int64_t)((uint64_t)d.off + (uint64_t)s.off));
	if (is_ptr(d) && s.kind == AV_CONST)
		return mk(d.kind, (int64_t)((uint64_t)d.off + (uint64_t)s.off), d.map);
	if (d.kind == AV_CONST && is_ptr(s))
		return mk(s.kind, (int64_t)((uint64_t)s.off + (uint64_t)d.off), s.map);
	// a packet pointer moved by a number no pointer went into (a TLV walk's length field) is
	// still a packet pointer; numbers combine into numbers
	const bool pd = d.kind == AV_CTX || d.kind == AV_CTXV, ps = s.kind == AV_CTX || s.kind == AV_CTXV;
	if ((pd && is_num(s)) || (is_num(d) && ps))
		return mk(AV_CTXV);
	if (is_num(d) && is_num(s))
		return mk(AV_SCALAR);
	return av();
}

// Two paths meet: the same value, two packet pointers (one with an unknown offset), two numbers,
// else unknown
av
meet_av(const av &a, const av &b)
{
	if (a == b)
		return a;
	const bool pa = a.kind == AV_CTX || a.kind == AV_CTXV, pb = b.kind == AV_CTX || b.kind == AV_CTXV;
	if (pa && pb)
		return mk(AV_CTXV);
	return is_num(a) && is_num(b) ? mk(AV_SCALAR) : av();
}

void
transfer(const dp_entry &e, const dprog_host &out, av r[EBPF_REG_MAX])
{
	const uint16_t k = e.kind;
	if (k == DK_FAULT || k == EBPF_OP_EXIT)
		return;
	if (k == DK_MOV64R) {
		r[e.dst] = r[e.src];
		return;
	}
	if (k >= DK_NEG64 && k <= DK_MOD32Z) { // (numbers stay numbers)
		const bool reads_src = k == DK_ARSH64R || k == DK_ARSH32R || k >= DK_DIV64Z;
		const bool num = is_num(r[e.dst]) && (!reads_src || is_num(r[e.src]));
		r[e.dst] = num ? mk(AV_SCALAR) : av();
		return;
	}
	if (k == DK_CALL_LOOKUP) {
		av res;
		if (r[1].kind == AV_CONST)
			for (size_t m = 0; m < out.maps.size(); m++)
				if ((uint64_t)r[1].off == (uint64_t)(uintptr_t)out.maps[m])
					res = mk(AV_MAPVAL_NULL, 0, (int16_t)m);
		r[0] = res; // r1..r5 keep their values (a plain C call in the reference)
		return;
	}
	if (k == DK_CALL_UPDATE) { // (update or, aux 1 before resolution, delete): an errno
		r[0] = av();
		return;
	}
	if (k == DK_LOOPINIT || k == DK_LOOPCNT || k == DK_OVLINIT)
		return;
	if (k == DK_CALL_HDELETE) {
		r[0] = av();
		return;
	}
	if (k == DK_CNT_STORE)
		return;
	if (k == DK_XADD) {
		if (e.aux & 0x100) // BPF_FETCH: src = the old value
			r[e.src] = av();
		return;
	}
	const uint8_t cls = k & 7;
	if (cls == EBPF_CLS_JMP || cls == DP_CLS_JMP32 || cls == EBPF_CLS_ST || cls == EBPF_CLS_STX)
		return;
	if (cls == EBPF_CLS_LDX) { // packet bytes are numbers; the stack and map values may hold pointers
		const uint8_t b = r[e.src].kind;
		r[e.dst] = (b == AV_CTX || b == AV_CTXV) ? mk(AV_SCALAR) : av();
		return;
	}
	if (k == EBPF_OP_LDDW) {
		r[e.dst] = mk(AV_CONST, (int64_t)e.imm);
		return;
	}
	const av s = (k & 0x08) ? r[e.src] : mk(AV_CONST, (int64_t)e.imm);
	av &d = r[e.dst];
	switch (k) {
	case EBPF_OP_ADD64_IMM: case EBPF_OP_ADD64_REG:
	case EBPF_OP_MOV64_IMM: case EBPF_OP_MOV64_REG:
		d = add_av(d, s);
		break;
	case EBPF_OP_SUB64_IMM: case EBPF_OP_SUB64_REG: case EBPF_OP_NEG64:
		if (s.kind == AV_CONST) {
			av neg = mk(AV_CONST, (int64_t)(0 - (uint64_t)s.off));
			d = add_av(d, neg);
		} else if (s.kind == AV_SCALAR && (d.kind == AV_CTX || d.kind == AV_CTXV || is_num(d))) {
			d = add_av(d, s); // (the sign does not matter to the kind)
		} else {
			d = av();
		}
		break;
	case EBPF_OP_MOV_IMM:
		d = mk(AV_CONST, (int64_t)(uint32_t)e.imm);
		break;
	case EBPF_OP_MOV_REG:
		d = s.kind == AV_CONST ? mk(AV_CONST, (int64_t)(uint32_t)s.off) : is_num(s) ? mk(AV_SCALAR) : av();
		break;
	case EBPF_OP_NEG:
		d = mk(AV_CONST, (int64_t)(uint32_t)(0u - (uint32_t)e.imm));
		break;
	default: // other ALU: numbers in, a number out
		d = is_num(d) && ((k & 0x08) == 0 || is_num(s)) ? mk(AV_SCALAR) : av();
		break;
	}
}

void
dataflow(dprog_host &out)
{
	const size_t n = out.entries.size();
	out.annot.assign(n, dp_annot());
	dp_annot init;
	for (auto &x : init.in)
		x = mk(AV_CONST, 0); // the device zeroes r0, r2..r9 (the reference leaves them undefined)
	init.in[1] = mk(AV_CTX, 0);
	init.in[10] = mk(AV_STACK, 0);
	init.reached = true;
	out.annot[out.start] = init;
	std::vector<uint32_t> work{out.start};
	std::vector<char> queued(n, 0);
	queued[out.start] = 1;
	while (!work.empty()) {
		uint32_t id = work.back();
		work.pop_back();
		queued[id] = 0;
		const dp_entry &e = out.entries[id];
		if (e.kind == DK_FAULT || e.kind == EBPF_OP_EXIT)
			continue;
		av r[EBPF_REG_MAX];
		for (int i = 0; i < EBPF_REG_MAX; i++)
			r[i] = out.annot[id].in[i];
		transfer(e, out, r);
		uint32_t succ[2] = {e.next, UINT32_MAX};
		if (e.kind < 0x100 && ((e.kind & 7) == EBPF_CLS_JMP || (e.kind & 7) == DP_CLS_JMP32))
			succ[1] = e.target;
		// the taken edge of "JEQ dst, imm" knows dst == imm (the 64-bit compare)
		av rt[EBPF_REG_MAX];
		for (int i = 0; i < EBPF_REG_MAX; i++)
			rt[i] = r[i];
		if (e.kind == EBPF_OP_JEQ_IMM && e.dst < EBPF_REG_MAX)
			rt[e.dst] = mk(AV_CONST, (int64_t)e.imm);
		// a NULL test of a lookup result: past it (JEQ 0 not taken, JNE 0 taken) it is non-NULL
		if ((e.kind == EBPF_OP_JEQ_IMM || e.kind == EBPF_OP_JNE_IMM) && e.imm == 0 &&
		    e.dst < EBPF_REG_MAX && r[e.dst].kind == AV_MAPVAL_NULL) {
			av nn = r[e.dst];
			nn.kind = AV_MAPVAL;
			if (e.kind == EBPF_OP_JEQ_IMM)
				r[e.dst] = nn; // (r feeds the fall-through edge below)
			else
				rt[e.dst] = nn;
		}
		for (int k = 0; k < 2; k++) {
			const uint32_t sx = succ[k];
			const av *re = k ? rt : r;
			if (sx == UINT32_MAX || sx >= n)
				continue;
			dp_annot &a = out.annot[sx];
			bool changed = false;
			if (!a.reached) {
				for (int i = 0; i < EBPF_REG_MAX; i++)
					a.in[i] = re[i];
				a.reached = true;
				changed = true;
			} else {
				for (int i = 0; i < EBPF_REG_MAX; i++) {
					const av m = meet_av(a.in[i], re[i]);
					if (m != a.in[i]) {
						a.in[i] = m;
						changed = true;
					}
				}
			}
			if (changed && !queued[sx]) {
				queued[sx] = 1;
				work.push_back(sx);
			}
		}
	}
}

// Successors of an entry in the state graph (UINT32_MAX: none).
uint32_t
succ_of(const dprog_host &out, uint32_t id, int k)
{
	const dp_entry &e = out.entries[id];
	if (e.kind == DK_FAULT || e.kind == EBPF_OP_EXIT)
		return UINT32_MAX;
	if (k == 0)
		return e.next;
	if (e.kind < 0x100 && ((e.kind & 7) == EBPF_CLS_JMP || (e.kind & 7) == DP_CLS_JMP32))
		return e.target;
	return UINT32_MAX;
}

// Counted loops whose budget cannot run out (standard semantics).  A program with one loop —
// one LOOPCNT entry L, reached from one conditional C on a counter X:
//   JNE X, 0 taken into L (the back edge), or JEQ X, 0 whose fall-through is L (exit test, JA back)
// — where every path from the loop head H = L.next to C decrements X by one exactly once
// (SUB64 X, 1 / ADD64 X, -1), nothing else on those paths writes X or calls a helper, and X
// enters the loop in [1, K]: the loop takes at most K - 1 backward jumps, so with K - 1 <=
// DP_LOOP_BUDGET no lane can reach EBPF_FAULT_LOOP and the count is dropped (C jumps to H
// directly; the oracle counts on and never faults either).  X's entry range comes from an
// interval pass over the loop-free graph (the back edge removed): constants, loads (0 ..
// 2^(8 size) - 1), AND / RSH / MOD / ADD / SUB with immediates, 64-bit compares with immediates
// on their edges.  Returns whether the loop count was dropped.
bool
elide_loop_count(dprog_host &out)
{
	const size_t n = out.entries.size();
	uint32_t L = UINT32_MAX;
	for (uint32_t i = 0; i < n; i++)
		if (out.entries[i].kind == DK_LOOPCNT && out.annot[i].reached) {
			if (L != UINT32_MAX)
				return false; // (several loops: their counts add up)
			L = i;
		}
	if (L == UINT32_MAX)
		return false;
	const uint32_t H = out.entries[L].next;
	if (H >= n || out.entries[H].kind == DK_FAULT)
		return false;
	// the one predecessor of L
	uint32_t C = UINT32_MAX;
	std::vector<std::vector<uint32_t>> preds(n);
	for (uint32_t i = 0; i < n; i++) {
		if (!out.annot[i].reached)
			continue;
		for (int k = 0; k < 2; k++) {
			const uint32_t s = succ_of(out, i, k);
			if (s >= n)
				continue;
			preds[s].push_back(i);
			if (s == L) {
				if (C != UINT32_MAX && C != i)
					return false;
				C = i;
			}
		}
	}
	if (C == UINT32_MAX)
		return false;
	const dp_entry &c = out.entries[C];
	const bool jne_form = c.kind == EBPF_OP_JNE_IMM && c.target == L && c.next != L;
	const bool jeq_form = c.kind == EBPF_OP_JEQ_IMM && c.next == L && c.target != L;
	if (!(jne_form || jeq_form) || c.imm != 0 || c.dst >= EBPF_REG_MAX)
		return false;
	const uint8_t X = c.dst;
	// the loop body: entries on a path H ->* C (not through L)
	std::vector<char> fwd(n, 0), bwd(n, 0);
	std::vector<uint32_t> st{H};
	fwd[H] = 1;
	while (!st.empty()) {
		const uint32_t i = st.back();
		st.pop_back();
		for (int k = 0; k < 2; k++) {
			const uint32_t s = succ_of(out, i, k);
			if (s < n && s != L && !fwd[s]) {
				fwd[s] = 1;
				st.push_back(s);
			}
		}
	}
	if (!fwd[C])
		return false;
	st.push_back(C);
	bwd[C] = 1;
	while (!st.empty()) {
		const uint32_t i = st.back();
		st.pop_back();
		if (i == H)
			continue;
		for (uint32_t p : preds[i])
			if (fwd[p] && !bwd[p] && p != L) {
				bwd[p] = 1;
				st.push_back(p);
			}
	}
	auto is_dec = [&](const dp_entry &e) {
		return e.dst == X && ((e.kind == EBPF_OP_SUB64_IMM && e.imm == 1) ||
				      (e.kind == EBPF_OP_ADD64_IMM && e.imm == ~0ull && e.aux == 0));
	};
	// (writes dst: ALU, ALU64, LDX, LDDW and the standard-semantics ALU kinds)
	auto writes = [&](const dp_entry &e, uint8_t r) {
		if (e.kind >= DK_MOV64R && e.kind <= DK_MOD32Z)
			return e.dst == r;
		if (e.kind >= 0x100)
			return true; // (calls, stores into maps, loop entries: not in a counted body)
		const uint8_t cls = e.kind & 7;
		return (cls == EBPF_CLS_ALU || cls == EBPF_CLS_ALU64 || cls == EBPF_CLS_LDX ||
			cls == EBPF_CLS_LD) && e.dst == r;
	};
	// decrements of X along the body's paths: every path H ->* C exactly one
	std::vector<int> ndec(n, -1); // -1 unknown, 0 or 1, 2 = inconsistent
	std::vector<uint32_t> order;  // topological over the body (a DAG: L is its only back edge)
	{
		std::vector<uint32_t> indeg(n, 0);
		for (uint32_t i = 0; i < n; i++)
			if (bwd[i])
				for (int k = 0; k < 2; k++) {
					const uint32_t s = succ_of(out, i, k);
					if (s < n && bwd[s] && s != H)
						indeg[s]++;
				}
		std::vector<uint32_t> q{H};
		while (!q.empty()) {
			const uint32_t i = q.back();
			q.pop_back();
			order.push_back(i);
			for (int k = 0; k < 2; k++) {
				const uint32_t s = succ_of(out, i, k);
				if (s < n && bwd[s] && s != H && --indeg[s] == 0)
					q.push_back(s);
			}
		}
	}
	size_t nbody = 0;
	for (uint32_t i = 0; i < n; i++)
		nbody += bwd[i] ? 1 : 0;
	if (order.size() != nbody)
		return false;
	ndec[H] = 0;
	for (uint32_t i : order) {
		const dp_entry &e = out.entries[i];
		int d = ndec[i];
		if (d < 0 || d > 1)
			return false;
		if (i != C) {
			if (is_dec(e))
				d++;
			else if (writes(e, X) || e.kind == DK_XADD)
				return false;
			if (e.kind == DK_CALL_LOOKUP || e.kind == DK_CALL_UPDATE || e.kind == DK_CALL_HDELETE)
				return false;
		}
		for (int k = 0; k < 2; k++) {
			const uint32_t s = succ_of(out, i, k);
			if (s >= n || !bwd[s] || s == H)
				continue;
			if (ndec[s] < 0)
				ndec[s] = d;
			else if (ndec[s] != d)
				return false;
		}
	}
	if (ndec[C] != 1)
		return false;
	// X's range on the way in: intervals over the graph without the back edge
	struct iv {
		uint64_t lo = 0, hi = ~0ull;
	};
	std::vector<std::array<iv, EBPF_REG_MAX>> in(n);
	std::vector<char> have(n, 0);
	std::vector<uint32_t> indeg(n, 0);
	for (uint32_t i = 0; i < n; i++)
		if (out.annot[i].reached)
			for (int k = 0; k < 2; k++) {
				const uint32_t s = succ_of(out, i, k);
				if (s < n && i != L)
					indeg[s]++;
			}
	for (auto &r : in[out.start]) {
		r.lo = 0;
		r.hi = 0; // (the device zeroes r0, r2..r9, as the dataflow assumes)
	}
	in[out.start][1] = iv();
	in[out.start][10] = iv();
	have[out.start] = 1;
	std::vector<uint32_t> q{out.start};
	auto join = [&](uint32_t s, const std::array<iv, EBPF_REG_MAX> &r) {
		if (!have[s]) {
			in[s] = r;
			have[s] = 1;
		} else {
			for (int k = 0; k < EBPF_REG_MAX; k++) {
				in[s][k].lo = std::min(in[s][k].lo, r[k].lo);
				in[s][k].hi = std::max(in[s][k].hi, r[k].hi);
			}
		}
	};
	while (!q.empty()) {
		const uint32_t i = q.back();
		q.pop_back();
		if (i == L)
			continue; // (the back edge)
		const dp_entry &e = out.entries[i];
		std::array<iv, EBPF_REG_MAX> r = in[i], t;
		const uint8_t d = e.dst < EBPF_REG_MAX ? e.dst : 0;
		const uint64_t K = e.imm;
		const uint8_t cls = e.kind < 0x100 ? (e.kind & 7) : 0xff;
		const iv full;
		auto set = [&](uint64_t lo, uint64_t hi) {
			r[d].lo = lo;
			r[d].hi = hi;
		};
		switch (e.kind) {
		case EBPF_OP_LDDW: set(K, K); break;
		case EBPF_OP_MOV_IMM: set((uint32_t)K, (uint32_t)K); break;
		case DK_MOV64R: r[d] = r[e.src]; break;
		case EBPF_OP_LDXB: set(0, 0xff); break;
		case EBPF_OP_LDXH: set(0, 0xffff); break;
		case EBPF_OP_LDXW: set(0, 0xffffffffull); break;
		case EBPF_OP_AND64_IMM: set(0, std::min(r[d].hi, K)); break;
		case EBPF_OP_AND_IMM: set(0, std::min<uint64_t>(r[d].hi, K & 0xffffffffull)); break;
		case EBPF_OP_RSH64_IMM: set(r[d].lo >> (K & 63), r[d].hi >> (K & 63)); break;
		case EBPF_OP_MOD64_IMM: set(0, K - 1); break; // (K != 0: MOD by 0 was rewritten)
		case EBPF_OP_ADD64_IMM:
			if ((int64_t)K >= 0 && r[d].hi <= ~0ull - K)
				set(r[d].lo + K, r[d].hi + K);
			else if ((int64_t)K < 0 && r[d].lo >= 0 - K)
				set(r[d].lo + K, r[d].hi + K);
			else
				r[d] = full;
			break;
		case EBPF_OP_SUB64_IMM:
			if ((int64_t)K >= 0 && r[d].lo >= K)
				set(r[d].lo - K, r[d].hi - K);
			else
				r[d] = full;
			break;
		default:
			if (e.kind >= DK_MOV64R && e.kind <= DK_MOD32Z)
				r[d] = full;
			else if (e.kind >= 0x100 && e.kind != DK_LOOPINIT && e.kind != DK_OVLINIT &&
				 e.kind != DK_LOOPCNT)
				for (auto &x : r)
					x = full; // (calls, XADD fetch, ...: nothing known after)
			else if (e.kind < 0x100 && writes(e, d))
				r[d] = (cls == EBPF_CLS_ALU) ? iv{0, 0xffffffffull} : full;
			break;
		}
		t = r;
		// 64-bit compares with an immediate refine their edges (taken: t, fall-through: r)
		if (cls == EBPF_CLS_JMP && !(e.kind & 0x08)) {
			iv &a = r[d], &b = t[d];
			switch (e.kind) {
			case EBPF_OP_JEQ_IMM: b.lo = std::max(b.lo, K); b.hi = std::min(b.hi, K); break;
			case EBPF_OP_JGT_IMM: b.lo = std::max(b.lo, K + 1); a.hi = std::min(a.hi, K); break;
			case EBPF_OP_JGE_IMM: b.lo = std::max(b.lo, K); if (K) a.hi = std::min(a.hi, K - 1); break;
			case EBPF_OP_JLT_IMM: if (K) b.hi = std::min(b.hi, K - 1); a.lo = std::max(a.lo, K); break;
			case EBPF_OP_JLE_IMM: b.hi = std::min(b.hi, K); a.lo = std::max(a.lo, K + 1); break;
			default: break;
			}
			if (e.kind == EBPF_OP_JGT_IMM && K == ~0ull)
				b = iv{1, 0}; // (never taken)
		}
		for (int k = 0; k < 2; k++) {
			const uint32_t s = succ_of(out, i, k);
			if (s >= n)
				continue;
			join(s, k ? t : r);
			if (--indeg[s] == 0)
				q.push_back(s);
		}
	}
	if (!have[H])
		return false;
	// H's range joined the entry edges only (the back edge was skipped); every predecessor
	// outside the loop must have been processed (indeg 0), else the graph has another cycle
	if (indeg[H] != 0)
		return false;
	const iv x = in[H][X];
	if (x.lo < 1 || x.hi - 1 > DP_LOOP_BUDGET)
		return false;
	dp_entry &cm = out.entries[C];
	if (jne_form)
		cm.target = H;
	else
		cm.next = H;
	return true;
}

// Counter updates (ebpf_gpu.h "Stores into map values"): three consecutive entries
//   LDX{W,DW} X = [P + off] (X != P);  ADD / SUB to X of an immediate or of a register other than
//   X (64-bit; 32-bit too for W; the reference's MOV64, which adds); STX [P + off] = X, same width
// make the STX a DK_CNT_STORE.  The pattern is on executed instructions, JA aside (the graph has
// JA folded): where the ALU or the STX entry has other predecessors (standard semantics), the
// pattern's path gets copies of its own.  Returns whether entries were added.
bool
fuse_counters(dprog_host &out, bool std_mode)
{
	const size_t n0 = out.entries.size();
	std::vector<uint32_t> preds(n0, 0);
	for (uint32_t i = 0; i < n0; i++) {
		if (!out.annot[i].reached)
			continue;
		for (int k = 0; k < 2; k++) {
			const uint32_t s = succ_of(out, i, k);
			if (s < n0)
				preds[s]++;
		}
	}
	bool grew = false;
	for (uint32_t i = 0; i < n0; i++) {
		const dp_entry e1 = out.entries[i];
		if (!out.annot[i].reached || !(e1.kind == EBPF_OP_LDXW || e1.kind == EBPF_OP_LDXDW) ||
		    e1.dst == e1.src)
			continue;
		const uint32_t w = e1.kind == EBPF_OP_LDXDW ? 8 : 4;
		const uint32_t j = e1.next;
		if (j >= n0)
			continue;
		const dp_entry e2 = out.entries[j];
		bool ok = false;
		if (e2.dst == e1.dst && e2.aux == 0)
			switch (e2.kind) {
			case EBPF_OP_ADD64_IMM: case EBPF_OP_SUB64_IMM: ok = true; break;
			case EBPF_OP_ADD64_REG: case EBPF_OP_SUB64_REG: ok = e2.src != e1.dst; break;
			case EBPF_OP_MOV64_IMM: ok = !std_mode; break; // (standard MOV64s are rewritten)
			case EBPF_OP_MOV64_REG: ok = !std_mode && e2.src != e1.dst; break;
			case EBPF_OP_ADD_IMM: case EBPF_OP_SUB_IMM: ok = w == 4; break;
			case EBPF_OP_ADD_REG: case EBPF_OP_SUB_REG: ok = w == 4 && e2.src != e1.dst; break;
			default: break;
			}
		if (!ok || e2.next >= n0)
			continue;
		const uint32_t k3 = e2.next;
		const dp_entry e3 = out.entries[k3];
		if (e3.kind != (w == 8 ? EBPF_OP_STXDW : EBPF_OP_STXW) || e3.dst != e1.src ||
		    e3.src != e1.dst || e3.off != e1.off)
			continue;
		dp_entry st = e3;
		st.kind = DK_CNT_STORE;
		st.aux = (uint16_t)w;
		// an immediate addend (the ALU's): aux bit 9, imm = what the update adds
		switch (e2.kind) {
		case EBPF_OP_ADD64_IMM: case EBPF_OP_MOV64_IMM: case EBPF_OP_ADD_IMM:
			st.imm = e2.imm;
			st.aux |= 0x200;
			break;
		case EBPF_OP_SUB64_IMM: case EBPF_OP_SUB_IMM:
			st.imm = 0 - e2.imm;
			st.aux |= 0x200;
			break;
		default:
			st.imm = 0;
			break;
		}
		if (preds[j] == 1 && preds[k3] == 1) {
			out.entries[k3] = st;
			continue;
		}
		// (a merge point under standard semantics: the pattern's own copies)
		dp_entry alu = e2;
		out.entries.push_back(st);
		alu.next = (uint32_t)(out.entries.size() - 1);
		out.entries.push_back(alu);
		out.entries[i].next = (uint32_t)(out.entries.size() - 1);
		grew = true;
	}
	return grew;
}

// Registers an entry reads and writes, for liveness (a read over-approximated, a write only where
// certain; an entry kind not listed reads every register).
void
reg_rw(const dp_entry &e, uint16_t *rd, uint16_t *wr)
{
	const uint16_t k = e.kind, d = (uint16_t)(1u << (e.dst & 15)), s = (uint16_t)(1u << (e.src & 15));
	*rd = 0;
	*wr = 0;
	switch (k) {
	case DK_FAULT: case DK_LOOPINIT: case DK_LOOPCNT: case DK_OVLINIT:
		return;
	case EBPF_OP_EXIT:
		*rd = 1;
		return;
	case DK_CALL_LOOKUP: case DK_CALL_HDELETE: // (map, key)
		*rd = 0x6;
		*wr = 1;
		return;
	case DK_CALL_UPDATE: // (map, key, value, flags)
		*rd = 0x1e;
		*wr = 1;
		return;
	case DK_CNT_STORE: case DK_XADD:
		*rd = d | s;
		return;
	case DK_MOV64R:
		*rd = s;
		*wr = d;
		return;
	case EBPF_OP_LDDW:
		*wr = d;
		return;
	default:
		break;
	}
	if (k >= DK_NEG64 && k <= DK_MOD32Z) {
		*rd = d | s;
		*wr = d;
		return;
	}
	if (k >= 0x100) {
		*rd = 0x7ff;
		return;
	}
	switch (k & 7) {
	case EBPF_CLS_LDX: *rd = s; *wr = d; return;
	case EBPF_CLS_ST: *rd = d; return;
	case EBPF_CLS_STX: *rd = d | s; return;
	case EBPF_CLS_JMP: case DP_CLS_JMP32: *rd = d | ((k & 0x08) ? s : 0); return;
	default: *rd = d | ((k & 0x08) ? s : 0); *wr = d; return; // ALU / ALU64
	}
}

// Registers live after each entry (a backward pass to a fixed point: the graph may have loops).
std::vector<uint16_t>
live_out(const dprog_host &out)
{
	const size_t n = out.entries.size();
	std::vector<uint16_t> rd(n), wr(n), lin(n, 0), lout(n, 0);
	for (size_t i = 0; i < n; i++)
		reg_rw(out.entries[i], &rd[i], &wr[i]);
	for (bool changed = true; changed;) {
		changed = false;
		for (size_t i = n; i-- > 0;) {
			uint16_t o = 0;
			for (int k = 0; k < 2; k++) {
				const uint32_t sx = succ_of(out, (uint32_t)i, k);
				if (sx < n)
					o |= lin[sx];
			}
			const uint16_t in = rd[i] | (uint16_t)(o & ~wr[i]);
			if (o != lout[i] || in != lin[i]) {
				lout[i] = o;
				lin[i] = in;
				changed = true;
			}
		}
	}
	return lout;
}

// ---- the slot graph of a standard-semantics program (ebpf_gpu.h "Stores into map values": the
// programs with loops that read their counter updates back).  A restatement of the contract on
// the bytecode itself, not on the state graph above, so that the decision depends on nothing but
// the program's bytes.

// A CALL of a helper the device runs (lookup, update, delete); 1 update, 2 the others, 0 none
int
std_slot_helper(const struct ebpf_config *ec, int32_t imm)
{
	const struct ebpf_helper_type *h = (imm >= 0 && imm < EBPF_TYPE_MAX) ? ec->helper_types[imm] : nullptr;
	if (h == &eht_map_update_elem)
		return 1;
	return (h != nullptr && (h == &eht_map_lookup_elem || h == &eht_map_delete_elem)) ? 2 : 0;
}

bool
std_slot_valid(const struct ebpf_inst &in)
{
	const uint8_t op = in.opcode;
	const bool jmp32 = (op & 7) == DP_CLS_JMP32;
	if (jmp32) {
		switch (op & 0xf0) {
		case 0x10: case 0x20: case 0x30: case 0x40: case 0x50: case 0x60: case 0x70:
		case 0xa0: case 0xb0: case 0xc0: case 0xd0:
			break;
		default:
			return false;
		}
		return !(in.dst >= EBPF_REG_MAX || ((op & 0x08) && in.src >= EBPF_REG_MAX));
	}
	const bool xadd = op == 0xc3 || op == 0xdb;
	if (!(valid_op(op) || xadd) || (xadd && in.imm != 0 && in.imm != 1))
		return false;
	return !((uses_dst(op) && in.dst >= EBPF_REG_MAX) || (uses_src(op) && in.src >= EBPF_REG_MAX));
}

// The slots execution may continue at after slot pc: both arms of a conditional jump (a target
// outside the program faults), LDDW over its second slot, none after EXIT or a faulting slot;
// a JA -1 spins (EBPF_FAULT_LOOP)
int
std_slot_succ(const struct ebpf_config *ec, const struct ebpf_inst *code, uint64_t n, uint64_t pc,
	      uint64_t succ[2])
{
	const struct ebpf_inst &in = code[pc];
	const uint8_t op = in.opcode;
	if (!std_slot_valid(in) || op == EBPF_OP_EXIT || (op == EBPF_OP_CALL && !std_slot_helper(ec, in.imm)))
		return 0;
	if (op == EBPF_OP_LDDW) {
		succ[0] = pc + 2;
		return 1;
	}
	const int64_t target = (int64_t)pc + 1 + in.offset;
	if (op == EBPF_OP_JA) {
		if (in.offset == -1 || target < 0)
			return 0;
		succ[0] = (uint64_t)target;
		return 1;
	}
	int k = 0;
	const uint8_t cls = op & 7;
	if ((cls == EBPF_CLS_JMP || cls == DP_CLS_JMP32) && op != EBPF_OP_CALL && target >= 0 &&
	    (uint64_t)target < n)
		succ[k++] = (uint64_t)target;
	succ[k++] = pc + 1;
	return k;
}

// Registers a standard-semantics slot reads / writes (a CALL reads its helper's arguments —
// lookup and delete r1, r2, update r1..r4 — and writes r0; EXIT reads r0)
void
std_slot_regs(const struct ebpf_config *ec, const struct ebpf_inst &in, uint16_t *rd, uint16_t *wr)
{
	const uint8_t op = in.opcode, cls = op & 7;
	const uint16_t d = (uint16_t)(1u << in.dst), s = (uint16_t)(1u << in.src);
	*rd = *wr = 0;
	if (!std_slot_valid(in))
		return;
	switch (cls) {
	case EBPF_CLS_LD:
		*wr = d;
		return;
	case EBPF_CLS_LDX:
		*rd = s;
		*wr = d;
		return;
	case EBPF_CLS_ST:
		*rd = d;
		return;
	case EBPF_CLS_STX:
		*rd = d | s;
		if ((op == 0xc3 || op == 0xdb) && in.imm == 1)
			*wr = s;
		return;
	case EBPF_CLS_JMP:
	case DP_CLS_JMP32:
		if (op == EBPF_OP_CALL) {
			*rd = std_slot_helper(ec, in.imm) == 1 ? 0x1e : 0x06;
			*wr = 1;
		} else if (op == EBPF_OP_EXIT) {
			*rd = 1;
		} else if (op != EBPF_OP_JA) {
			*rd = d | ((op & 0x08) ? s : 0);
		}
		return;
	default: // ALU / ALU64: MOV writes only (reg: reads src); NEG, LE / BE read dst only
		*wr = d;
		if ((op & 0xf0) == 0xb0)
			*rd = (op & 0x08) ? s : 0;
		else if ((op & 0xf0) == 0xd0 || (op & 0xf0) == 0x80)
			*rd = d;
		else
			*rd = d | ((op & 0x08) ? s : 0);
		return;
	}
}

// The slot execution continues at from pc, JA chains followed; n when none
uint64_t
std_slot_next_exec(const struct ebpf_inst *code, uint64_t n, uint64_t pc)
{
	for (uint64_t hops = 0; pc < n && hops <= n; hops++) {
		if (code[pc].opcode != EBPF_OP_JA)
			return pc;
		const int64_t t = (int64_t)pc + 1 + code[pc].offset;
		if (code[pc].offset == -1 || t < 0)
			return n;
		pc = (uint64_t)t;
	}
	return n;
}

// Does the program read its counter updates back?  A reachable XADD with BPF_FETCH, or a
// reachable counter idiom (LDX{W,DW} X = [P + off], X != P; then, JA aside, ADD / SUB to X of
// an immediate or of a register other than X, 64-bit or, for W, 32-bit; then STX [P + off] = X
// of the same width) whose X is live after its STX on the slot graph
bool
slot_reads_counters(const struct ebpf_config *ec, const struct ebpf_inst *code, uint64_t n)
{
	if (n == 0)
		return false;
	std::vector<char> seen(n, 0);
	std::vector<uint64_t> work{0};
	while (!work.empty()) {
		const uint64_t pc = work.back();
		work.pop_back();
		if (pc >= n || seen[pc])
			continue;
		seen[pc] = 1;
		uint64_t sx[2];
		const int k = std_slot_succ(ec, code, n, pc, sx);
		for (int i = 0; i < k; i++)
			work.push_back(sx[i]);
	}
	for (uint64_t i = 0; i < n; i++)
		if (seen[i] && (code[i].opcode == 0xc3 || code[i].opcode == 0xdb) && code[i].imm == 1)
			return true;
	std::vector<uint16_t> lin;
	for (uint64_t a = 0; a < n; a++) {
		const struct ebpf_inst &la = code[a];
		const uint8_t X = la.dst, P = la.src;
		if (!seen[a] || !(la.opcode == EBPF_OP_LDXW || la.opcode == EBPF_OP_LDXDW) || X == P)
			continue;
		const int size = la.opcode == EBPF_OP_LDXDW ? 8 : 4;
		const uint64_t b = std_slot_next_exec(code, n, a + 1);
		if (b >= n || code[b].dst != X)
			continue;
		const uint8_t bs = code[b].src;
		bool ok = false;
		switch (code[b].opcode) {
		case 0x07: case 0x17: ok = true; break;
		case 0x0f: case 0x1f: ok = bs != X; break;
		case 0x04: case 0x14: ok = size == 4; break;
		case 0x0c: case 0x1c: ok = size == 4 && bs != X; break;
		}
		if (!ok)
			continue;
		const uint64_t c = std_slot_next_exec(code, n, b + 1);
		if (c >= n)
			continue;
		const struct ebpf_inst &lc = code[c];
		if (lc.opcode != (size == 8 ? EBPF_OP_STXDW : EBPF_OP_STXW) || lc.dst != P || lc.src != X ||
		    lc.offset != la.offset)
			continue;
		if (lin.empty()) { // liveness to a fixed point: in = rd | (out & ~wr)
			lin.assign(n, 0);
			for (bool changed = true; changed;) {
				changed = false;
				for (uint64_t i = n; i-- > 0;) {
					uint16_t rd, wr, o = 0;
					std_slot_regs(ec, code[i], &rd, &wr);
					uint64_t sx[2];
					const int k = std_slot_succ(ec, code, n, i, sx);
					for (int j = 0; j < k; j++)
						if (sx[j] < n)
							o |= lin[sx[j]];
					const uint16_t in = (uint16_t)(rd | (o & ~wr));
					if (in != lin[i]) {
						lin[i] = in;
						changed = true;
					}
				}
			}
		}
		uint64_t sx[2];
		const int k = std_slot_succ(ec, code, n, c, sx);
		for (int j = 0; j < k; j++)
			if (sx[j] < n && ((lin[sx[j]] >> X) & 1))
				return true;
	}
	return false;
}

// Stores into map values (ebpf_gpu.h "Stores into map values"): which maps they may reach and
// how each written map's writes land (dprog_host upd_maps / hupd_maps / atomic_maps), whether
// the packet may read its own stores back (the overlay), and the write log's records per path.
int
analyze_writes(dprog_host &out)
{
	const size_t n = out.entries.size(), nm = out.maps.size();
	auto is_vsite = [&](size_t i, bool *add, av *base) {
		const dp_entry &e = out.entries[i];
		const uint8_t cls = e.kind < 0x100 ? (e.kind & 7) : 0xff;
		*add = e.kind == DK_CNT_STORE || e.kind == DK_XADD;
		if (!*add && cls != EBPF_CLS_ST && cls != EBPF_CLS_STX)
			return false;
		*base = out.annot[i].in[e.dst];
		// (the stack and the packet are never a map's values)
		return base->kind != AV_STACK && base->kind != AV_CTX && base->kind != AV_CTXV;
	};
	auto size_of = [](const dp_entry &e) -> uint32_t {
		if (e.kind == DK_CNT_STORE || e.kind == DK_XADD)
			return e.aux & 0xff;
		const uint32_t z = e.kind & 0x18;
		return z == 0x00 ? 4 : z == 0x08 ? 2 : z == 0x10 ? 1 : 8;
	};
	// per map: stores, counter updates, counter widths, and whether every counter update is
	// through that map's lookup result at an offset aligned for every key
	std::vector<uint32_t> nset(nm, 0), nadd(nm, 0), widths(nm, 0);
	std::vector<char> exact(nm, 1);
	out.vstore_sites = 0;
	for (size_t i = 0; i < n; i++) {
		bool add;
		av b;
		if (!out.annot[i].reached || !is_vsite(i, &add, &b))
			continue;
		out.vstore_sites++;
		const dp_entry &e = out.entries[i];
		const uint32_t w = size_of(e);
		const bool one = (b.kind == AV_MAPVAL || b.kind == AV_MAPVAL_NULL) && b.map >= 0 &&
				 (size_t)b.map < nm;
		for (size_t m = 0; m < nm; m++) {
			if (one && (size_t)b.map != m)
				continue;
			if (!add) {
				nset[m]++;
				continue;
			}
			nadd[m]++;
			widths[m] |= w;
			const int64_t o = b.off + e.off;
			if (!one || out.maps[m]->value_size % w || ((o % w) + w) % w)
				exact[m] = 0;
		}
	}
	for (size_t m = 0; m < nm; m++) {
		const uint16_t t = (uint16_t)m;
		const bool helper = std::find(out.upd_maps.begin(), out.upd_maps.end(), t) != out.upd_maps.end();
		const bool hash = out.maps[m]->is_hashtable();
		auto drop = [&](std::vector<uint16_t> &v) { v.erase(std::remove(v.begin(), v.end(), t), v.end()); };
		auto put = [&](std::vector<uint16_t> &v) {
			if (std::find(v.begin(), v.end(), t) == v.end())
				v.push_back(t);
		};
		if (nset[m] == 0 && nadd[m] == 0)
			continue;
		if (hash) {
			put(out.hupd_maps);
		} else if (nadd[m] == 0) {
			put(out.upd_maps); // stores (and update calls): byte winners on the device
			put(out.vstore_maps);
		} else if (nset[m] == 0 && !helper && exact[m] && (widths[m] == 4 || widths[m] == 8)) {
			put(out.atomic_maps);
			out.atomic_width.push_back((uint8_t)widths[m]);
		} else {
			drop(out.upd_maps);
			put(out.hupd_maps);
		}
	}
	// sites that log: every store, and counter updates unless all their maps are atomic
	auto logs = [&](size_t i) {
		const dp_entry &e = out.entries[i];
		if (e.kind == DK_CALL_UPDATE || e.kind == DK_CALL_HDELETE)
			return true;
		bool add;
		av b;
		if (!out.annot[i].reached || !is_vsite(i, &add, &b))
			return false;
		if (!add)
			return true;
		for (size_t m = 0; m < nm; m++) {
			if ((b.kind == AV_MAPVAL || b.kind == AV_MAPVAL_NULL) && b.map >= 0 && (size_t)b.map != m)
				continue;
			if (std::find(out.atomic_maps.begin(), out.atomic_maps.end(), (uint16_t)m) ==
			    out.atomic_maps.end())
				return true;
		}
		return false;
	};
	// may a load read a value the packet stored before it?  (a forward pass: `stored` after an
	// entry when any path to it passed a store into a map value)
	std::vector<char> stored(n, 0), seen(n, 0);
	{
		std::vector<uint32_t> work{out.start};
		seen[out.start] = 1;
		while (!work.empty()) {
			const uint32_t id = work.back();
			work.pop_back();
			bool add;
			av b;
			const char after = stored[id] || (out.annot[id].reached && is_vsite(id, &add, &b));
			for (int k = 0; k < 2; k++) {
				const uint32_t s = succ_of(out, id, k);
				if (s >= n)
					continue;
				if (!seen[s] || (after && !stored[s])) {
					seen[s] = 1;
					stored[s] = stored[s] || after;
					work.push_back(s);
				}
			}
		}
	}
	// A counter update whose register nobody reads after its STX needs no value the packet sees:
	// its addition is the same whatever was loaded, so neither it nor the idiom's LDX makes the
	// packet read its own stores back (the overlay)
	const std::vector<uint16_t> lout = live_out(out);
	auto cnt_dead = [&](size_t k) {
		const dp_entry &c = out.entries[k];
		return c.kind == DK_CNT_STORE && !((lout[k] >> c.src) & 1);
	};
	auto idiom_head_dead = [&](size_t i) { // LDX i -> ALU -> CNT_STORE with a dead register
		const dp_entry &e = out.entries[i];
		if (!(e.kind == EBPF_OP_LDXW || e.kind == EBPF_OP_LDXDW) || e.next >= n)
			return false;
		const uint32_t k = out.entries[e.next].next;
		if (k >= n)
			return false;
		const dp_entry &c = out.entries[k];
		return c.kind == DK_CNT_STORE && c.src == e.dst && c.dst == e.src && c.off == e.off && cnt_dead(k);
	};
	out.vstore_overlay = false;
	for (size_t i = 0; i < n && !out.vstore_overlay; i++) {
		const dp_entry &e = out.entries[i];
		if (!out.annot[i].reached || !stored[i])
			continue;
		if (e.kind == DK_CNT_STORE) {
			out.vstore_overlay = !cnt_dead(i); // (it loaded the value it adds to)
		} else if (e.kind == DK_XADD) {
			out.vstore_overlay = (e.aux & 0x100) != 0; // (BPF_FETCH returns the old value)
		} else if (e.kind < 0x100 && (e.kind & 7) == EBPF_CLS_LDX) {
			const av &b = out.annot[i].in[e.src];
			out.vstore_overlay = b.kind != AV_STACK && b.kind != AV_CTX && b.kind != AV_CTXV &&
					     !idiom_head_dead(i);
		}
	}
	// Programs with loops: a path has no bound on its writes.  Counter updates are device atomics
	// (an array only aligned counter updates of one width change) or records of a hashtable's
	// values, which count as logged writes like every other record; the logged writes are capped
	// per packet (DP_WRITES_MAX, the next one faults EBPF_FAULT_WRITES), which also bounds the
	// overlay (two words per store).  An array mixing counter updates with other writes is refused
	bool counters = false, atomic_cnt = false;
	for (size_t i = 0; i < n; i++) {
		const dp_entry &e = out.entries[i];
		if (!out.annot[i].reached || !(e.kind == DK_CNT_STORE || e.kind == DK_XADD))
			continue;
		counters = true;
		if (!out.has_loops)
			continue;
		const av &b = out.annot[i].in[e.dst];
		for (size_t m = 0; m < nm; m++) {
			if ((b.kind == AV_MAPVAL || b.kind == AV_MAPVAL_NULL) && b.map >= 0 && (size_t)b.map != m)
				continue;
			const bool atomic = std::find(out.atomic_maps.begin(), out.atomic_maps.end(), (uint16_t)m) !=
					    out.atomic_maps.end();
			atomic_cnt = atomic_cnt || atomic;
			if (!atomic && !out.maps[m]->is_hashtable()) {
				out.error = EOPNOTSUPP;
				out.error_msg = "in a program with loops, counter updates must go to a hashtable or to "
						"an array map that only aligned counter updates of one width change (run "
						"this one with ebpf_prog_run)";
				return EOPNOTSUPP;
			}
		}
	}
	// A program with loops that reads its counter updates back (slot_reads_counters: a live
	// idiom register, XADD with BPF_FETCH) keeps the packet's view of them in the overlay, 32
	// words (DP_OVL_MAX; the store that needs one more faults EBPF_FAULT_WRITES).  A read-back
	// of another form (a later load of a counter's word) is refused when device atomics take
	// counter updates (they are not counted, so nothing else bounds the overlay); a hashtable's
	// counter records are counted, so its overlay holds at most two words per logged write
	if (out.has_loops && counters && out.reads_counters) {
		out.vstore_overlay = true;
	} else if (out.has_loops && atomic_cnt && out.vstore_overlay) {
		out.error = EOPNOTSUPP;
		out.error_msg = "in a program with loops, the packet may read back the values its counter "
				"updates change only through the idiom's register or XADD with BPF_FETCH (run "
				"this one with ebpf_prog_run)";
		return EOPNOTSUPP;
	}
	// per path: records the log needs, stores the overlay holds
	std::vector<uint32_t> best(n, 0), bests(n, 0);
	std::vector<uint8_t> state(n, 0);
	std::vector<uint32_t> st{out.start};
	while (!st.empty()) {
		const uint32_t id = st.back();
		if (state[id] == 0) {
			state[id] = 1;
			for (int k = 0; k < 2; k++) {
				const uint32_t sx = succ_of(out, id, k);
				if (sx < n && state[sx] == 0)
					st.push_back(sx);
			}
			continue;
		}
		st.pop_back();
		if (state[id] == 2)
			continue;
		uint32_t m = 0, ms = 0;
		for (int k = 0; k < 2; k++) {
			const uint32_t sx = succ_of(out, id, k);
			if (sx < n) {
				m = std::max(m, best[sx]);
				ms = std::max(ms, bests[sx]);
			}
		}
		bool add;
		av b;
		best[id] = m + (logs(id) ? 1u : 0u);
		bests[id] = ms + (out.annot[id].reached && is_vsite(id, &add, &b) ? 1u : 0u);
		state[id] = 2;
	}
	out.max_updates = best[out.start];
	out.ovl_entries = out.vstore_overlay ? 2 * bests[out.start] : 0;
	// A loop-free program's log and overlay are sized by its path counts: every write it reaches
	// lands, as in the reference (ebpf_interpreter.c:343-366, ebpf_map.c:101-108).  Only a loop
	// has no per-path bound; its writes are capped (DP_WRITES_MAX)
	out.write_cap = false;
	if (out.has_loops) { // (the path counts above do not bound a loop)
		bool logging = false;
		for (size_t i = 0; i < n && !logging; i++)
			logging = out.annot[i].reached && logs(i);
		out.write_cap = logging;
		out.max_updates = logging ? DP_WRITES_MAX : 0;
		out.ovl_entries = out.vstore_overlay ? 2 * DP_WRITES_MAX : 0;
	}
	// (a loop-free path with more than DP_OVL_MAX / 2 stores read back runs on the portable
	// interpreter with its overlay spilled to memory, 16 B an entry per lane)
	if (out.ovl_entries > DP_OVL_SPILL_MAX) {
		out.error = EOPNOTSUPP;
		out.error_msg = "the program stores into map values and reads them back more often on one "
				"path than the device overlay holds (run it with ebpf_prog_run)";
		return EOPNOTSUPP;
	}
	return 0;
}

} // namespace

bool
prog_writes_maps(const dprog_host &xl)
{
	return xl.max_updates != 0 || !xl.atomic_maps.empty();
}

int
translate_program(struct ebpf_prog *ep, dprog_host &out)
{
	const struct ebpf_inst *code = ep->prog;
	uint64_t nslots = ep->prog_len / sizeof(struct ebpf_inst);
	const bool std_sem = ep->semantics.load() == EBPF_SEM_STANDARD;
	Translator t(code, nslots, ep->eo.eo_ee->ec, out, std_sem);
	int err = t.run();
	if (err)
		return err;
	if (const char *dump = getenv("EBPF_XLATE_DUMP")) { // (debugging: the entries, one a line)
		if (FILE *f = fopen(dump, "w")) {
			fprintf(f, "start %u\n", out.start);
			for (size_t i = 0; i < out.entries.size(); i++) {
				const dp_entry &e = out.entries[i];
				fprintf(f, "%zu kind %#x dst %u src %u off %d imm %#llx next %u target %u aux %u\n", i,
					e.kind, e.dst, e.src, e.off, (unsigned long long)e.imm, e.next, e.target, e.aux);
			}
			fclose(f);
		}
	}

	// Resolve LDDW immediates that are live maps of this env: the device map table.
	struct ebpf_env *ee = ep->eo.eo_ee;
	std::lock_guard<std::mutex> g(ee->lock);
	const struct ebpf_map *unsupported = nullptr;
	auto add_map = [&](struct ebpf_map *m) {
		if (map_device_layout_of(m).bytes == 0) {
			// device batches resolve array and hashtable maps (percpu ones included); a
			// map with no device form runs on the CPU path only (ebpf_prog_run)
			unsupported = m;
			return;
		}
		for (auto *x : out.maps)
			if (x == m)
				return;
		out.maps.push_back(m);
	};
	for (const dp_entry &e : out.entries) {
		if (e.kind == EBPF_OP_LDDW) {
			auto *cand = reinterpret_cast<struct ebpf_map *>((uintptr_t)e.imm);
			if (ee->maps.count(cand))
				add_map(cand);
		}
		if (e.kind == EBPF_OP_STXB || e.kind == EBPF_OP_STXH || e.kind == EBPF_OP_STXW ||
		    e.kind == EBPF_OP_STXDW || e.kind == EBPF_OP_STB || e.kind == EBPF_OP_STH ||
		    e.kind == EBPF_OP_STW || e.kind == EBPF_OP_STDW) {
			if (e.dst == EBPF_R10 && e.off < 0 && (uint32_t)(-e.off) > out.max_stack)
				out.max_stack = (uint32_t)(-e.off);
		}
	}
	for (uint32_t i = 0; i < ep->ndep_maps; i++)
		if (ee->maps.count(ep->dep_maps[i]))
			add_map(ep->dep_maps[i]);
	if (unsupported != nullptr) {
		out.error = EOPNOTSUPP;
		out.error_msg = std::string("the program uses a ") + unsupported->emt->name +
				" map with no device form (hashtable keys over 65535 bytes or a table over 64 GiB; "
				"run it with "
				"ebpf_prog_run)";
		out.maps.clear(); // (not pinned: nothing to release)
		return EOPNOTSUPP;
	}
	dataflow(out);
	// A hashtable lookup runs a probe specialised for its map.  A lookup whose map is known only
	// at run time, in a program with hashtables, becomes a compare chain on r1: one 64-bit JEQ
	// per hashtable of the table, taken into the lookup with that map known, ending in the
	// generic lookup (array maps, NULL, not a map).  Its successor then has several
	// predecessors: the dataflow runs again over the graph.
	bool any_hash = false;
	for (struct ebpf_map *m : out.maps)
		any_hash |= m->is_hashtable();
	if (any_hash) {
		const size_t n0 = out.entries.size();
		bool grew = false;
		for (size_t i = 0; i < n0; i++) {
			if (out.entries[i].kind != DK_CALL_LOOKUP || !out.annot[i].reached ||
			    out.annot[i].in[1].kind == AV_CONST)
				continue;
			const dp_entry call = out.entries[i];
			auto add = [&](const dp_entry &x) {
				out.entries.push_back(x);
				return (uint32_t)(out.entries.size() - 1);
			};
			uint32_t chain = add(call); // the generic lookup at the end of the chain
			for (size_t m = out.maps.size(); m-- > 0;) {
				if (!out.maps[m]->is_hashtable())
					continue;
				dp_entry j;
				memset(&j, 0, sizeof(j));
				j.kind = EBPF_OP_JEQ_IMM;
				j.dst = EBPF_R1;
				j.imm = (uint64_t)(uintptr_t)out.maps[m];
				j.next = chain;
				j.target = add(call);
				chain = add(j);
			}
			out.entries[i] = out.entries[chain]; // the first compare takes the call's place
			out.entries[chain].kind = DK_FAULT;   // (its copy is unreachable)
			out.entries[chain].aux = EBPF_FAULT_SLOT;
			grew = true;
		}
		if (out.entries.size() >= kMaxEntries) {
			out.error = E2BIG;
			out.error_msg = "program state graph exceeds the device translation limit";
			out.maps.clear();
			return E2BIG;
		}
		if (grew)
			dataflow(out);
	}
	// Map-writing helpers whose map is known only at run time (r1 not a translation-time
	// constant of the map table): a compare chain on r1 as for lookups, one 64-bit JEQ per map of the table taken
	// into a copy of the call with that map known; when none matches, the reference's argument
	// checks come first (ebpf_map.c:101-108: em, key or value NULL, or flags > EBPF_EXIST ->
	// EINVAL; delete :130-136: em or key NULL -> EINVAL), then the call dereferences a pointer
	// that is not a map of this env: EBPF_FAULT_BAD_MAP.
	{
		const size_t n0 = out.entries.size();
		bool grew = false;
		for (size_t i = 0; i < n0; i++) {
			if (out.entries[i].kind != DK_CALL_UPDATE || !out.annot[i].reached)
				continue;
			const av &r1 = out.annot[i].in[1];
			if (r1.kind == AV_CONST &&
			    std::any_of(out.maps.begin(), out.maps.end(), [&](const struct ebpf_map *m) {
				    return (uint64_t)r1.off == (uint64_t)(uintptr_t)m;
			    }))
				continue; // (resolved below)
			const dp_entry call = out.entries[i];
			const bool del = call.aux == 1;
			auto add = [&](const dp_entry &x) {
				out.entries.push_back(x);
				return (uint32_t)(out.entries.size() - 1);
			};
			dp_entry x;
			memset(&x, 0, sizeof(x));
			x.kind = EBPF_OP_LDDW; // r0 = EINVAL, then the call's successor
			x.imm = EINVAL;
			x.next = call.next;
			const uint32_t einval = add(x);
			memset(&x, 0, sizeof(x));
			x.kind = DK_FAULT;
			x.aux = EBPF_FAULT_BAD_MAP;
			uint32_t chain = add(x);
			auto cmp = [&](uint16_t kind, uint8_t reg, uint64_t imm, uint32_t taken, uint32_t next) {
				dp_entry j;
				memset(&j, 0, sizeof(j));
				j.kind = kind;
				j.dst = reg;
				j.imm = imm;
				j.target = taken;
				j.next = next;
				return add(j);
			};
			if (!del)
				chain = cmp(EBPF_OP_JGT_IMM, EBPF_R4, EBPF_EXIST, einval, chain);
			if (!del)
				chain = cmp(EBPF_OP_JEQ_IMM, EBPF_R3, 0, einval, chain);
			chain = cmp(EBPF_OP_JEQ_IMM, EBPF_R2, 0, einval, chain);
			chain = cmp(EBPF_OP_JEQ_IMM, EBPF_R1, 0, einval, chain);
			for (size_t m = out.maps.size(); m-- > 0;)
				chain = cmp(EBPF_OP_JEQ_IMM, EBPF_R1, (uint64_t)(uintptr_t)out.maps[m], add(call),
					    chain);
			out.entries[i] = out.entries[chain]; // the first compare takes the call's place
			out.entries[chain].kind = DK_FAULT;   // (its copy is unreachable)
			out.entries[chain].aux = EBPF_FAULT_SLOT;
			grew = true;
		}
		if (out.entries.size() >= kMaxEntries) {
			out.error = E2BIG;
			out.error_msg = "program state graph exceeds the device translation limit";
			out.maps.clear();
			return E2BIG;
		}
		if (grew)
			dataflow(out);
	}
	// Map-writing helpers, the map now a translation-time constant of the table.  delete on an
	// array map is EINVAL whatever its arguments (ebpf_map.c delete -> ebpf_map_array.c:
	// 246-250): a constant; on a hashtable it becomes DK_CALL_HDELETE.  update keeps its entry,
	// aux = the map's table index (its routine checks the arguments at run time).
	for (size_t i = 0; i < out.entries.size(); i++) {
		dp_entry &e = out.entries[i];
		if (e.kind != DK_CALL_UPDATE || !out.annot[i].reached)
			continue;
		const av &m1 = out.annot[i].in[1];
		int mi = -1;
		if (m1.kind == AV_CONST)
			for (size_t m = 0; m < out.maps.size(); m++)
				if ((uint64_t)m1.off == (uint64_t)(uintptr_t)out.maps[m])
					mi = (int)m;
		if (mi < 0) { // (a constant that is not a map of the table)
			e.kind = DK_FAULT;
			e.aux = EBPF_FAULT_BAD_MAP;
			continue;
		}
		if (e.aux == 1) { // delete
			if (out.maps[mi]->is_hashtable()) {
				e.kind = DK_CALL_HDELETE; // (the key is logged; the routine checks it)
				e.aux = (uint16_t)mi;
				if (std::find(out.hupd_maps.begin(), out.hupd_maps.end(), (uint16_t)mi) ==
				    out.hupd_maps.end())
					out.hupd_maps.push_back((uint16_t)mi);
			} else {
				e.kind = EBPF_OP_LDDW;
				e.dst = 0;
				e.imm = EINVAL;
			}
			continue;
		}
		e.aux = (uint16_t)mi;
		std::vector<uint16_t> &written = out.maps[mi]->is_hashtable() ? out.hupd_maps : out.upd_maps;
		if (std::find(written.begin(), written.end(), (uint16_t)mi) == written.end())
			written.push_back((uint16_t)mi);
	}
	// a counted loop that cannot reach the budget needs no count
	if (out.has_loops && getenv("EBPF_XLATE_KEEP_LOOPCNT") == nullptr && elide_loop_count(out))
		dataflow(out);
	// counter updates, then how the program's map writes land and the log's records per path
	if (fuse_counters(out, std_sem)) {
		if (out.entries.size() >= kMaxEntries) {
			out.error = E2BIG;
			out.error_msg = "program state graph exceeds the device translation limit";
			out.maps.clear();
			return E2BIG;
		}
		dataflow(out);
	}
	out.reads_counters = std_sem && out.has_loops && slot_reads_counters(ep->eo.eo_ee->ec, code, nslots);
	if (analyze_writes(out) != 0) {
		out.maps.clear();
		return out.error;
	}
	if (out.vstore_overlay || out.write_cap) { // every lane's overlay and write count start at 0
		dp_entry x;
		memset(&x, 0, sizeof(x));
		x.kind = DK_OVLINIT;
		x.next = out.start;
		out.entries.push_back(x);
		out.start = (uint32_t)(out.entries.size() - 1);
		dataflow(out);
	}
	// The program now pins its maps (released in prog_dtor): a device mirror must not outlive
	// its map while a later batch may still read it.
	for (struct ebpf_map *m : out.maps)
		m->eo.eo_ref.fetch_add(1);
	return 0;
}
