// asm_jit.cpp — copy-and-patch compilation of a translated program for gfx950.
//
// The interpreter (asm_runtime.cpp) pays one scalar dispatch per executed instruction: load the
// 32-B entry, wait, jump.  Here the same lowered entries (asm_lower) become straight-line code:
// for each entry, in depth-first order of the state tree (translate.cpp), the compiler emits
//   s_mov_b32 s10..s15, <operand>       only the entry registers the handler body reads
//   <handler body bytes>                copied from the assembled interpreter image
//   s_waitcnt lgkmcnt(0)                if the body leaves an LDS read outstanding
//   conditional tail / branch           see gen_interp.py jit_templates()
// into the reserved area of a private copy of the code object (ebpf_jit_area), which is then
// loaded as its own module.  Handler bodies reach the shared routines (fault, exit, udiv,
// check, lookup, schedule) relative to .Lcb, whose offset is the same in every copy, so the
// bytes need no relocation.  Divergence works as in the interpreter: lanes that take a branch
// the rest of the wave does not are parked with v41 = the code offset of their block, and the
// scheduler resumes them by jumping to .Lcb + v41 (s7 bit 1 selects that mode).
//
// The state graph is a tree, so every block is placed exactly once and each straight-line run
// falls through; only taken branches (and shared fault entries) need jumps.
#include <elf.h>
#include <hip/hip_runtime.h>

#include "asm_cc.h"
#include "asm_handlers.h"
#include "internal.h"

int asm_lower(const dprog_host &xl, int mode, const std::vector<dp_map> &table,
	      std::vector<dp_entry> &out, uint32_t *stack_stride, std::string *err);

namespace {

// Order of ebpf_jit_tmpl in gen_interp.py.
enum jt_index {
	JT_MOV_S10 = 0, // .. JT_MOV_S10 + 5
	JT_CS = 6, JT_CS_BR, JT_CS_VT, JT_CS_END,
	JT_CL, JT_CL_LIT, JT_CL_VT, JT_CL_END,
	JT_BR, JT_JL, JT_JL_END, JT_WAIT, JT_EXITK, JT_EXIT, JT_FAULT, JT_HLOOKUP, JT_GDONE,
	JT_SCHED, JT_AREA, JT_AREA_BYTES,
	JT_COUNT
};

struct jit_image {
	bool ok = false;
	std::string why;
	size_t cb = 0;                          // file offset of .Lcb
	std::vector<uint32_t> body_off, body_len; // per handler id, body offset from .Lcb, length
	uint32_t t[JT_COUNT] = {};
};

bool
find_symbols(const unsigned char *img, size_t len, const char *const *names, size_t nn,
	     size_t *file_off)
{
	if (len < sizeof(Elf64_Ehdr))
		return false;
	const Elf64_Ehdr *eh = reinterpret_cast<const Elf64_Ehdr *>(img);
	if (memcmp(eh->e_ident, ELFMAG, SELFMAG) != 0 || eh->e_ident[EI_CLASS] != ELFCLASS64 ||
	    eh->e_shoff + (uint64_t)eh->e_shnum * sizeof(Elf64_Shdr) > len)
		return false;
	const Elf64_Shdr *sh = reinterpret_cast<const Elf64_Shdr *>(img + eh->e_shoff);
	for (size_t i = 0; i < nn; i++)
		file_off[i] = 0;
	size_t found = 0;
	for (int si = 0; si < eh->e_shnum; si++) {
		if (sh[si].sh_type != SHT_SYMTAB || sh[si].sh_link >= eh->e_shnum)
			continue;
		const Elf64_Shdr &st = sh[si], &str = sh[st.sh_link];
		if (st.sh_offset + st.sh_size > len || str.sh_offset + str.sh_size > len)
			return false;
		const Elf64_Sym *sym = reinterpret_cast<const Elf64_Sym *>(img + st.sh_offset);
		const size_t ns = st.sh_size / sizeof(Elf64_Sym);
		for (size_t k = 0; k < ns; k++) {
			if (sym[k].st_name >= str.sh_size || sym[k].st_shndx == SHN_UNDEF ||
			    sym[k].st_shndx >= eh->e_shnum)
				continue;
			const char *nm = reinterpret_cast<const char *>(img + str.sh_offset + sym[k].st_name);
			for (size_t q = 0; q < nn; q++) {
				if (file_off[q] || strcmp(nm, names[q]) != 0)
					continue;
				const Elf64_Shdr &sec = sh[sym[k].st_shndx];
				file_off[q] = sec.sh_offset + (sym[k].st_value - sec.sh_addr);
				found++;
			}
		}
	}
	return found == nn;
}

const jit_image &
image_info(int mode)
{
	static jit_image info[kModes];
	static std::once_flag once[kModes];
	std::call_once(once[mode], [mode] {
		jit_image &I = info[mode];
		const unsigned char *img = asm_image(mode);
		const size_t len = asm_image_len(mode);
		const char *names[] = {"ebpf_cb", "ebpf_jit_meta", "ebpf_jit_tmpl"};
		size_t off[3];
		if (!find_symbols(img, len, names, 3, off)) {
			I.why = "code object lacks the compiled-program symbols";
			return;
		}
		I.cb = off[0];
		const unsigned char *meta = img + off[1];
		const unsigned char *tm = img + off[2];
		if (off[1] + 8ull * AH_COUNT > len || off[2] + 4ull * JT_COUNT > len) {
			I.why = "compiled-program tables out of range";
			return;
		}
		I.body_off.resize(AH_COUNT);
		I.body_len.resize(AH_COUNT);
		for (int h = 0; h < AH_COUNT; h++) {
			memcpy(&I.body_off[h], meta + 8 * h, 4);
			memcpy(&I.body_len[h], meta + 8 * h + 4, 4);
			if (I.cb + I.body_off[h] + I.body_len[h] > len) {
				I.why = "handler body out of range";
				return;
			}
		}
		memcpy(I.t, tm, sizeof(I.t));
		if (I.t[JT_AREA_BYTES] != AH_JIT_AREA_BYTES || I.cb + I.t[JT_AREA] + I.t[JT_AREA_BYTES] > len) {
			I.why = "compiled-program area out of range";
			return;
		}
		I.ok = true;
	});
	return info[mode];
}

inline bool
is_terminal(uint32_t h)
{
	return h == (uint32_t)AH_EXIT || h == (uint32_t)AH_FAULT;
}

inline bool
fits_simm16(int64_t bytes)
{
	const int64_t w = bytes / 4;
	return (bytes % 4) == 0 && w >= -32768 && w <= 32767;
}

// Layout order of the lowered entries: depth-first from the start, the not-taken successor
// falls through (parents before their children).
std::vector<uint32_t>
layout_order(const dprog_host &xl, const std::vector<dp_entry> &low)
{
	const size_t n = low.size();
	std::vector<uint32_t> order;
	order.reserve(n);
	std::vector<char> placed(n, 0);
	std::vector<uint32_t> stack{xl.start};
	while (!stack.empty()) {
		uint32_t cur = stack.back();
		stack.pop_back();
		while (cur < n && !placed[cur]) {
			placed[cur] = 1;
			order.push_back(cur);
			const uint32_t h = (uint32_t)low[cur].handler;
			if (is_terminal(h))
				break;
			if (ah_flags[h] & 1) {
				const uint32_t tk = xl.entries[cur].target;
				if (tk < n && !placed[tk])
					stack.push_back(tk);
			}
			cur = xl.entries[cur].next;
		}
	}
	return order;
}

} // namespace

// Compile the program for `mode` into a patched copy of the code object (*img) and return the
// emitted code bytes (*code).  Host only.  E2BIG: the code does not fit the reserved area.
// Area layout: +0 16 bytes never executed (s_endpgm), +16 the program's start block (where the kernel enters
// each group), then the blocks.
int
asm_jit_emit(const dprog_host &xl, int mode, const std::vector<dp_map> &table,
	     std::vector<unsigned char> *img_out, std::vector<unsigned char> *code,
	     uint32_t *stack_stride, std::string *err)
{
	const uint32_t HDR = 16;
	const jit_image &I = image_info(mode);
	if (!I.ok) {
		*err = I.why;
		return ENOSYS;
	}
	std::vector<dp_entry> low;
	int lerr = asm_lower(xl, mode, table, low, stack_stride, err);
	if (lerr)
		return lerr;
	const size_t n = low.size();
	const uint32_t *T = I.t;
	auto tsize = [&](int a, int b) { return T[b] - T[a]; };
	const uint32_t cs_len = tsize(JT_CS, JT_CS_END), cl_len = tsize(JT_CL, JT_CL_END);
	const uint32_t jl_len = tsize(JT_JL, JT_JL_END);

	const std::vector<uint32_t> order = layout_order(xl, low);
	std::vector<char> placed(n, 0);
	for (uint32_t e : order)
		placed[e] = 1;
	// successor that must follow each block (UINT32_MAX: none)
	auto succ = [&](uint32_t e) -> uint32_t {
		const uint32_t h = (uint32_t)low[e].handler;
		return is_terminal(h) ? UINT32_MAX : xl.entries[e].next;
	};
	std::vector<uint32_t> pos(n, 0), idx(n, UINT32_MAX);
	for (size_t k = 0; k < order.size(); k++)
		idx[order[k]] = (uint32_t)k;
	std::vector<char> long_cond(n, 0), long_br(n, 0);
	auto needs_branch = [&](uint32_t e) {
		const uint32_t sx = succ(e);
		if (sx == UINT32_MAX)
			return false;
		const uint32_t k = idx[e];
		return !(k + 1 < order.size() && order[k + 1] == sx);
	};
	// blocks that can be entered other than by falling through from their layout predecessor:
	// taken targets, branch targets, scheduler resume points after a lookup, the start
	std::vector<char> entry_point(n, 0);
	entry_point[xl.start] = 1;
	for (uint32_t e : order) {
		const uint32_t h = (uint32_t)low[e].handler;
		if (ah_flags[h] & 1)
			entry_point[xl.entries[e].target] = 1;
		if (h == (uint32_t)AH_LOOKUPGEN && xl.entries[e].next < n)
			entry_point[xl.entries[e].next] = 1;
		if (needs_branch(e))
			entry_point[succ(e)] = 1;
	}
	// Loop back edges (standard semantics: a conditional whose taken side is a LOOPCNT entry)
	// split the other way round: the lanes that stay in the loop continue, the lanes that leave
	// it park at the fall-through block, and when no lane loops any more the scheduler resumes
	// every parked lane of that exit together.  (The forward split would run the loop's tail
	// once per distinct trip count in the group.)  The fall-through block becomes an entry point.
	// (a loop whose count translate.cpp dropped jumps to its head directly: a loop head placed
	// before the conditional)
	std::vector<char> rev_cond(n, 0), loop_head(n, 0);
	for (uint32_t e = 0; e < n; e++)
		if (xl.entries[e].kind == DK_LOOPCNT && xl.entries[e].next < n)
			loop_head[xl.entries[e].next] = 1;
	if (getenv("EBPF_JIT_NOREVLOOP") == nullptr)
		for (uint32_t e : order) {
			const uint32_t h = (uint32_t)low[e].handler;
			if (!(ah_flags[h] & 1))
				continue;
			const uint32_t tk = xl.entries[e].target, nx = xl.entries[e].next;
			if (tk < n && nx < n && nx != tk &&
			    (xl.entries[tk].kind == DK_LOOPCNT || (loop_head[tk] && idx[tk] < idx[e]))) {
				rev_cond[e] = 1;
				entry_point[nx] = 1;
			}
		}
	const uint32_t RC = 48; // the reversed split up to its jump to the loop (see the emitter)
	// Structured control flow (staged programs without generic lookups): every conditional
	// splits exec into its fall-through lanes, which run first, and its taken lanes, whose mask
	// waits in s[74 + 2d] (d = branches pending on the path) and which run when the fall-through
	// subtree is done (the join at the head of the taken block).  A leaf (EXIT / FAULT) calls
	// its routine and continues at the innermost pending join (or ends the group).  No lane is
	// parked and nothing is scheduled; the interpreter's v41 parking remains for the rest.
	const uint32_t GROUP_END = UINT32_MAX;
	std::vector<uint32_t> cont(n, GROUP_END); // where a path through the entry continues
	std::vector<int> jdepth(n, 0);            // pending branches (join masks in use)
	std::vector<int> join_of(n, -1);          // entry e is the taken block of conditional k
	bool structured = (mode == 1 || AH_GEN_JOIN) && getenv("EBPF_JIT_NOSTRUCT") == nullptr &&
			  getenv("EBPF_JIT_NOCC") == nullptr;
	for (uint32_t e : order) {
		const uint32_t h = (uint32_t)low[e].handler;
		if (h == (uint32_t)AH_LOOKUPGEN)
			structured = false;
	}
	if (structured) {
		std::vector<char> seen(n, 0);
		seen[xl.start] = 1;
		for (uint32_t e : order) {
			if (!seen[e]) { // more than the tree: no structure
				structured = false;
				break;
			}
			const uint32_t h = (uint32_t)low[e].handler;
			if (is_terminal(h))
				continue;
			const uint32_t nx = xl.entries[e].next;
			if (ah_flags[h] & 1) {
				const uint32_t tk = xl.entries[e].target;
				if (jdepth[e] >= AH_JOIN_LEVELS || nx >= n || tk >= n || nx == tk || seen[nx] || seen[tk]) {
					structured = false;
					break;
				}
				jdepth[nx] = jdepth[e] + 1;
				cont[nx] = tk;
				jdepth[tk] = jdepth[e];
				cont[tk] = cont[e];
				join_of[tk] = (int)e;
				seen[nx] = seen[tk] = 1;
			} else if (nx < n) {
				if (seen[nx]) {
					structured = false;
					break;
				}
				jdepth[nx] = jdepth[e];
				cont[nx] = cont[e];
				seen[nx] = 1;
			}
		}
	}
	// per entry: optimised code (asm_cc.cpp) or the interpreter's handler body
	std::vector<cc_block> cb;
	const unsigned bus0 = cc_bus_violations();
	if (getenv("EBPF_JIT_NOCC") == nullptr) {
		cc_compile(xl, low, order, entry_point, mode, structured,
			   cc_routines{T[JT_EXITK], T[JT_EXIT], T[JT_FAULT], T[JT_HLOOKUP]}, table, cb);
	} else {
		cb.assign(n, cc_block()); // every body copied: full group set-up
		cc_prologue(mode, 0x7ff, true, false, cb[xl.start].prologue);
	}
	if (cc_bus_violations() != bus0) {
		*err = "internal error: the compiler emitted a VOP3 instruction reading two SGPRs";
		return EINVAL;
	}
	auto reads_of = [&](uint32_t e) -> uint8_t {
		return cb[e].fast ? cb[e].reads : ah_reads[(uint32_t)low[e].handler];
	};
	auto sval_of = [&](uint32_t e, int r) -> uint32_t {
		if (cb[e].fast)
			return cb[e].sval[r];
		uint32_t dw[8];
		memcpy(dw, &low[e], 32);
		return dw[2 + r];
	};
	// Operand registers s10..s15 a block must set: the ones its body reads, minus those that
	// provably already hold the value.  Values carry along a fall-through chain; a block that
	// can be entered any other way assumes nothing.
	std::vector<uint8_t> pre_mask(n, 0);
	{
		bool known[6] = {};
		uint32_t val[6] = {};
		for (size_t k = 0; k < order.size(); k++) {
			const uint32_t e = order[k];
			const bool fall = k > 0 && succ(order[k - 1]) == e && !needs_branch(order[k - 1]);
			if (!fall || entry_point[e])
				for (bool &x : known)
					x = false;
			const uint8_t rd = reads_of(e);
			uint8_t m = 0;
			for (int r = 0; r < 6; r++) {
				if (!(rd & (1u << r)))
					continue;
				const uint32_t v = sval_of(e, r);
				if (r == 2 || !known[r] || val[r] != v) {
					m |= (uint8_t)(1u << r);
					if (r != 2) {
						known[r] = true;
						val[r] = v;
					}
				}
			}
			pre_mask[e] = m;
			if (ah_fam[(uint32_t)low[e].handler] == AHF_HLOOKUP ||
			    ah_fam[(uint32_t)low[e].handler] == AHF_UPDATE ||
			    ah_fam[(uint32_t)low[e].handler] == AHF_HDELETE) // (their routines use s10/s11)
				for (bool &x : known)
					x = false;
		}
	}
	// s_mov_b32 s(10+r), v: 4 bytes with an inline constant, else 8 (s12, the resume offset,
	// is only known after layout: always the literal form)
	auto inline_code = [](uint32_t v, uint32_t *code) {
		const int32_t x = (int32_t)v;
		if (x >= 0 && x <= 64) {
			*code = 128 + (uint32_t)x;
			return true;
		}
		if (x >= -16 && x < 0) {
			*code = 192 + (uint32_t)(-x);
			return true;
		}
		return false;
	};
	auto pre_len = [&](uint32_t e) {
		uint32_t sz = 0, c;
		for (int r = 0; r < 6; r++)
			if (pre_mask[e] & (1u << r))
				sz += (r != 2 && inline_code(sval_of(e, r), &c)) ? 4 : 8;
		return sz;
	};
	// structured-mode glue (SALU, encoded here): join head, conditional split, leaf continuation
	std::vector<char> long_join(n, 0), long_leaf(n, 0);
	const uint32_t LJ = 16; // s_add_u32 (8) + s_addc_u32 + s_setpc_b64: a jump anywhere
	auto join_len = [&](uint32_t e) -> uint32_t {
		return (structured && join_of[e] >= 0) ? (long_join[e] ? 8 + LJ : 8) : 0;
	};
	auto leaf_jumps = [&](uint32_t e) -> bool { // a leaf whose continuation is not next in layout
		const uint32_t h = (uint32_t)low[e].handler;
		if (!structured || !is_terminal(h))
			return false;
		const uint32_t k = idx[e];
		const uint32_t nxt = k + 1 < order.size() ? order[k + 1] : GROUP_END;
		return cont[e] != nxt;
	};
	// a fast body's spliced slow path (cc_block.splice_h): operands, the handler body, a wait
	auto splice_len = [&](uint32_t e) -> uint32_t {
		return cb[e].splice_h < 0 ? 0 : 16 + I.body_len[(uint32_t)cb[e].splice_h] + 4;
	};
	auto block_size = [&](uint32_t e, uint32_t *pre, uint32_t *body_end) {
		const uint32_t h = (uint32_t)low[e].handler;
		uint32_t sz = join_len(e) + (uint32_t)cb[e].prologue.size() +
			      (uint32_t)cb[e].hoist.size() + pre_len(e);
		*pre = sz;
		if (cb[e].fast) {
			sz += (uint32_t)cb[e].body.size() + splice_len(e);
		} else {
			sz += I.body_len[h];
			if (ah_flags[h] & 2)
				sz += 4;
		}
		*body_end = sz;
		if (structured && (ah_flags[h] & 1) && cb[e].sdir == 0) {
			sz += 4; // s_mov_b64 s[Tk], 0: no lane takes it
		} else if (structured && (ah_flags[h] & 1)) {
			sz += long_cond[e] ? 12 + LJ : 12;
		} else if (ah_flags[h] & 1) {
			if (cb[e].sdir < 0 && rev_cond[e])
				sz += RC + (long_cond[e] ? LJ : 4);
			else if (cb[e].sdir < 0)
				sz += long_cond[e] ? cl_len : cs_len;
			else if (cb[e].sdir == 1)
				sz += long_cond[e] ? jl_len : 4; // always taken: a jump
		}
		if (needs_branch(e))
			sz += long_br[e] ? jl_len : 4;
		if (leaf_jumps(e))
			sz += long_leaf[e] ? LJ : 4;
		return sz;
	};
	// position of a continuation (GROUP_END: the block after the last one)
	uint32_t end_pos = 0;
	auto cont_pos = [&](uint32_t c) { return c == GROUP_END ? end_pos : pos[c]; };
	uint32_t total = 0;
	for (int iter = 0; iter < 8; iter++) {
		total = HDR;
		for (uint32_t e : order) {
			uint32_t pre, be;
			pos[e] = total;
			total += block_size(e, &pre, &be);
		}
		end_pos = total;
		if (structured)
			total += LJ; // the group end: jump to .Lgroup_done
		bool changed = false;
		for (uint32_t e : order) {
			uint32_t pre, be;
			block_size(e, &pre, &be);
			const uint32_t h = (uint32_t)low[e].handler;
			if (structured) {
				if (join_of[e] >= 0 && !long_join[e] &&
				    !fits_simm16((int64_t)cont_pos(cont[e]) - (int64_t)(pos[e] + 8))) {
					long_join[e] = 1;
					changed = true;
				}
				if ((ah_flags[h] & 1) && !long_cond[e] && cb[e].sdir != 0 &&
				    !fits_simm16((int64_t)pos[xl.entries[e].target] - (int64_t)(pos[e] + be + 12))) {
					long_cond[e] = 1;
					changed = true;
				}
				if (leaf_jumps(e) && !long_leaf[e]) {
					const uint32_t br_at = pos[e] + block_size(e, &pre, &be) - 4;
					if (!fits_simm16((int64_t)cont_pos(cont[e]) - (int64_t)(br_at + 4))) {
						long_leaf[e] = 1;
						changed = true;
					}
				}
			}
			if (!structured && (ah_flags[h] & 1) && !long_cond[e] && cb[e].sdir != 0) {
				const uint32_t br_at = pos[e] + be + (cb[e].sdir == 1 ? 0 : rev_cond[e] ? RC :
								      T[JT_CS_BR] - T[JT_CS]);
				const uint32_t tk = xl.entries[e].target;
				if (!fits_simm16((int64_t)pos[tk] - (int64_t)(br_at + 4))) {
					long_cond[e] = 1;
					changed = true;
				}
			}
			if (needs_branch(e) && !long_br[e]) {
				const uint32_t br_at = pos[e] + block_size(e, &pre, &be) - 4;
				if (!fits_simm16((int64_t)pos[succ(e)] - (int64_t)(br_at + 4))) {
					long_br[e] = 1;
					changed = true;
				}
			}
		}
		if (!changed)
			break;
	}
	if (total > (uint32_t)AH_JIT_AREA_BYTES) {
		*err = "compiled program exceeds the code area";
		return E2BIG;
	}
	for (uint32_t e = 0; e < n; e++)
		if (!placed[e] && e == xl.start) {
			*err = "internal error: start entry not placed";
			return EINVAL;
		}

	// emit
	std::vector<unsigned char> &img = *img_out;
	img.assign(asm_image(mode), asm_image(mode) + asm_image_len(mode));
	const size_t area = I.cb + T[JT_AREA];
	const unsigned char *src = asm_image(mode) + I.cb;
	// handler body h at area offset `at`; returns the bytes copied
	auto copy_body = [&](size_t at, uint32_t h) -> uint32_t {
		memcpy(&img[area + at], src + I.body_off[h], I.body_len[h]);
		return I.body_len[h];
	};
	auto code_off = [&](uint32_t e) { return T[JT_AREA] + pos[e]; }; // from .Lcb
	auto put32 = [&](size_t at, uint32_t v) { memcpy(&img[area + at], &v, 4); };
	auto copy_t = [&](size_t at, int a, uint32_t len) {
		memcpy(&img[area + at], src + T[a], len);
	};
	auto patch_simm16 = [&](size_t at, uint32_t target) {
		uint32_t w;
		memcpy(&w, &img[area + at], 4);
		const int32_t d = ((int32_t)target - (int32_t)(at + 4)) / 4;
		w = (w & 0xffff0000u) | ((uint32_t)d & 0xffffu);
		memcpy(&img[area + at], &w, 4);
	};
	for (uint32_t e : order) {
		const dp_entry &o = low[e];
		const uint32_t h = (uint32_t)o.handler;
		size_t at = pos[e];
		// (a long jump: s_add_u32 s60, s4, off; s_addc_u32 s61, s5, 0; s_setpc_b64 s[60:61])
		auto long_jump = [&](size_t a, uint32_t target_pos) {
			put32(a, 0x80000000u | (60u << 16) | (255u << 8) | 4u);
			put32(a + 4, T[JT_AREA] + target_pos);
			put32(a + 8, 0x80000000u | (0x04u << 23) | (61u << 16) | (128u << 8) | 5u);
			put32(a + 12, 0xbe800000u | (0x1du << 8) | 60u);
		};
		auto sopp = [&](size_t a, uint32_t op, uint32_t target_pos) { // s_branch / s_cbranch_*
			const int32_t d = ((int32_t)target_pos - (int32_t)(a + 4)) / 4;
			put32(a, 0xbf800000u | (op << 16) | ((uint32_t)d & 0xffffu));
		};
		const uint32_t OP_BRANCH = 0x02, OP_SCC0 = 0x04, OP_EXECZ = 0x08, OP_EXECNZ = 0x09;
		if (structured && join_of[e] >= 0) {
			const uint32_t sk = AH_S_JOIN + 2 * (uint32_t)jdepth[join_of[e]];
			put32(at, 0xbe800000u | (126u << 16) | (0x01u << 8) | sk); // s_mov_b64 exec, s[Tk]
			at += 4;
			if (!long_join[e]) {
				sopp(at, OP_EXECZ, cont_pos(cont[e]));
				at += 4;
			} else {
				put32(at, 0xbf800000u | (OP_EXECNZ << 16) | (LJ / 4));
				long_jump(at + 4, cont_pos(cont[e]));
				at += 4 + LJ;
			}
		}
		if (!cb[e].prologue.empty()) {
			memcpy(&img[area + at], cb[e].prologue.data(), cb[e].prologue.size());
			at += cb[e].prologue.size();
		}
		if (!cb[e].hoist.empty()) {
			memcpy(&img[area + at], cb[e].hoist.data(), cb[e].hoist.size());
			at += cb[e].hoist.size();
		}
		for (int r = 0; r < 6; r++) {
			if (!(pre_mask[e] & (1u << r)))
				continue;
			uint32_t v = sval_of(e, r);
			if (r == 2) { // s12: code offset of the next block (LOOKUPGEN resumes there)
				const uint32_t nx = xl.entries[e].next;
				v = nx < n && placed[nx] ? code_off(nx) : 0;
			}
			uint32_t ic;
			if (r != 2 && inline_code(v, &ic)) { // s_mov_b32 s(10+r), <inline constant>
				put32(at, 0xbe800000u | ((uint32_t)(10 + r) << 16) | ic);
				at += 4;
				continue;
			}
			copy_t(at, JT_MOV_S10 + r, 8);
			put32(at + 4, v);
			at += 8;
		}
		if (cb[e].fast && cb[e].splice_h >= 0) {
			// the fast body, the interpreter's handler body as its slow path, the rest
			const cc_block &c = cb[e];
			const uint32_t sh = (uint32_t)c.splice_h, sl = splice_len(e);
			std::vector<uint8_t> b(c.body);
			for (uint32_t at_br : c.splice_br) {
				if (at_br == ~0u)
					continue;
				int32_t rel = (int16_t)(b[at_br] | (b[at_br + 1] << 8));
				rel += (int32_t)(sl / 4);
				if (rel > 32767)
					return EINVAL; // (splice_len keeps a body far below this)
				b[at_br] = (uint8_t)rel;
				b[at_br + 1] = (uint8_t)(rel >> 8);
			}
			memcpy(&img[area + at], b.data(), c.splice_at);
			at += c.splice_at;
			for (int r = 0; r < 2; r++) { // s_mov_b32 s(10 + r), literal
				put32(at, 0xbe8000ffu | ((uint32_t)(10 + r) << 16));
				put32(at + 4, c.splice_sval[r]);
				at += 8;
			}
			at += copy_body(at, sh);
			put32(at, 0xbf8cc07fu); // s_waitcnt lgkmcnt(0)
			at += 4;
			memcpy(&img[area + at], b.data() + c.splice_at, b.size() - c.splice_at);
			at += b.size() - c.splice_at;
		} else if (cb[e].fast) {
			if (!cb[e].body.empty())
				memcpy(&img[area + at], cb[e].body.data(), cb[e].body.size());
			at += cb[e].body.size();
		} else {
			at += copy_body(at, h);
			if (ah_flags[h] & 2) {
				copy_t(at, JT_WAIT, 4);
				at += 4;
			}
		}
		if (structured && (ah_flags[h] & 1) && cb[e].sdir == 0) {
			// decided at compile time, never taken: the taken block's join finds no lane
			const uint32_t sk = AH_S_JOIN + 2 * (uint32_t)jdepth[e];
			put32(at, 0xbe800000u | (sk << 16) | (0x01u << 8) | 128u); // s_mov_b64 s[Tk], 0
			at += 4;
		} else if (structured && (ah_flags[h] & 1)) {
			// s_and_b64 s[Tk], vcc, exec; s_andn2_b64 exec, exec, vcc; s_cbranch_execz join
			const uint32_t sk = AH_S_JOIN + 2 * (uint32_t)jdepth[e];
			put32(at, 0x80000000u | (0x0du << 23) | (sk << 16) | (126u << 8) | 106u);
			put32(at + 4, 0x80000000u | (0x13u << 23) | (126u << 16) | (106u << 8) | 126u);
			at += 8;
			const uint32_t tk = xl.entries[e].target;
			if (!long_cond[e]) {
				sopp(at, OP_EXECZ, pos[tk]);
				at += 4;
			} else {
				put32(at, 0xbf800000u | (OP_EXECNZ << 16) | (LJ / 4));
				long_jump(at + 4, pos[tk]);
				at += 4 + LJ;
			}
		} else if ((ah_flags[h] & 1) && cb[e].sdir == 1) { // statically taken by every lane
			const uint32_t tk = xl.entries[e].target;
			if (!long_cond[e]) {
				copy_t(at, JT_BR, 4);
				patch_simm16(at, pos[tk]);
				at += 4;
			} else {
				copy_t(at, JT_JL, jl_len);
				put32(at + 4, code_off(tk));
				at += jl_len;
			}
		} else if ((ah_flags[h] & 1) && cb[e].sdir < 0 && rev_cond[e]) {
			// s_and_b64 s[48:49], vcc, exec          (lanes that loop)
			// s_andn2_b64 s[18:19], exec, vcc        (lanes that leave; SCC = any)
			// s_cbranch_scc0 .Lloop
			// s_mov_b64 exec, s[18:19]
			// v_mov_b32 v41, <code offset of the fall-through block>   (park them there)
			// s_mov_b64 exec, s[48:49]
			// s_cbranch_execnz .Lloop
			// (long jump to .Lr_schedule)
			// .Lloop: s_branch <taken block> (or a long jump)
			const uint32_t tk = xl.entries[e].target, nx = xl.entries[e].next;
			const size_t loop_at = at + RC;
			// (both branches go to the taken block itself when it is in reach, not through .Lloop)
			auto to_loop = [&](size_t a) -> uint32_t {
				return !long_cond[e] && fits_simm16((int64_t)pos[tk] - (int64_t)(a + 4)) ? pos[tk]
													 : (uint32_t)loop_at;
			};
			put32(at, 0x80000000u | (0x0du << 23) | (48u << 16) | (126u << 8) | 106u);
			put32(at + 4, 0x80000000u | (0x13u << 23) | (18u << 16) | (106u << 8) | 126u);
			sopp(at + 8, OP_SCC0, to_loop(at + 8));
			put32(at + 12, 0xbe800000u | (126u << 16) | (0x01u << 8) | 18u);
			put32(at + 16, 0x7e000000u | (41u << 17) | (0x01u << 9) | 255u);
			put32(at + 20, code_off(nx));
			put32(at + 24, 0xbe800000u | (126u << 16) | (0x01u << 8) | 48u);
			sopp(at + 28, OP_EXECNZ, to_loop(at + 28));
			put32(at + 32, 0x80000000u | (60u << 16) | (255u << 8) | 4u);
			put32(at + 36, T[JT_SCHED]);
			put32(at + 40, 0x80000000u | (0x04u << 23) | (61u << 16) | (128u << 8) | 5u);
			put32(at + 44, 0xbe800000u | (0x1du << 8) | 60u);
			at = loop_at;
			if (!long_cond[e]) {
				sopp(at, OP_BRANCH, pos[tk]);
				at += 4;
			} else {
				long_jump(at, pos[tk]);
				at += LJ;
			}
		} else if ((ah_flags[h] & 1) && cb[e].sdir < 0) {
			const uint32_t tk = xl.entries[e].target;
			if (!long_cond[e]) {
				copy_t(at, JT_CS, cs_len);
				patch_simm16(at + (T[JT_CS_BR] - T[JT_CS]), pos[tk]);
				put32(at + (T[JT_CS_VT] - T[JT_CS]) + 4, code_off(tk));
				at += cs_len;
			} else {
				copy_t(at, JT_CL, cl_len);
				put32(at + (T[JT_CL_LIT] - T[JT_CL]) + 4, code_off(tk));
				put32(at + (T[JT_CL_VT] - T[JT_CL]) + 4, code_off(tk));
				at += cl_len;
			}
		}
		if (needs_branch(e)) {
			const uint32_t sx = succ(e);
			if (!long_br[e]) {
				copy_t(at, JT_BR, 4);
				patch_simm16(at, pos[sx]);
				at += 4;
			} else {
				copy_t(at, JT_JL, jl_len);
				put32(at + 4, code_off(sx));
				at += jl_len;
			}
		}
		if (leaf_jumps(e)) {
			if (!long_leaf[e]) {
				sopp(at, OP_BRANCH, cont_pos(cont[e]));
				at += 4;
			} else {
				long_jump(at, cont_pos(cont[e]));
				at += LJ;
			}
		}
		uint32_t pre, be;
		if (at != pos[e] + block_size(e, &pre, &be)) {
			*err = "internal error: compiled block size mismatch";
			return EINVAL;
		}
	}
	if (structured) { // group end: every path has exited
		const size_t a = end_pos;
		put32(a, 0x80000000u | (60u << 16) | (255u << 8) | 4u);
		put32(a + 4, T[JT_GDONE]);
		put32(a + 8, 0x80000000u | (0x04u << 23) | (61u << 16) | (128u << 8) | 5u);
		put32(a + 12, 0xbe800000u | (0x1du << 8) | 60u);
	}
	if (code)
		code->assign(img.begin() + area, img.begin() + area + total);
	return 0;
}

// Build and load the compiled program for `mode`; on success *mod_out / *fn_out hold the
// module and its kernel.
int
asm_jit_build(int device, const dprog_host &xl, int mode, const std::vector<dp_map> &table,
	      void **mod_out, void **fn_out, void **fn_wide_out, uint32_t *stack_stride,
	      std::string *err)
{
	std::vector<unsigned char> img;
	int e = asm_jit_emit(xl, mode, table, &img, nullptr, stack_stride, err);
	if (e)
		return e;
	if (hipSetDevice(device) != hipSuccess)
		return EIO;
	hipModule_t mod = nullptr;
	if (hipModuleLoadData(&mod, img.data()) != hipSuccess) {
		*err = "loading the compiled program failed";
		return EIO;
	}
	hipFunction_t fn = nullptr;
	if (hipModuleGetFunction(&fn, mod, mode == 1 ? "ebpf_jit_s64" : "ebpf_jit_gen") != hipSuccess) {
		hipModuleUnload(mod);
		*err = "compiled program kernel missing";
		return EIO;
	}
	// the staged image's wide kernel (16 result slots for write phasing), where it has one
	hipFunction_t fw = nullptr;
	if (fn_wide_out && mode == 1 && AH_NVGPR_STAGED_WIDE &&
	    hipModuleGetFunction(&fw, mod, "ebpf_jit_s64w") != hipSuccess)
		fw = nullptr;
	*mod_out = mod;
	*fn_out = fn;
	if (fn_wide_out)
		*fn_wide_out = fw;
	return 0;
}

void
asm_jit_release(void *mod)
{
	if (mod)
		hipModuleUnload(static_cast<hipModule_t>(mod));
}
