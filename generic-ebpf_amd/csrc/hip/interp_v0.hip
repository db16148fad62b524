// interp_v0.hip — portable-HIP baseline of the batch interpreter (variant 1).
//
// One lane = one packet; the wave walks the translated device program (dprog.h) in lockstep:
// every step it picks the smallest entry index among its live lanes (a wave-uniform value, so
// the entry is fetched with scalar loads) and runs that entry for the lanes sitting on it.
// Replaces the caller's per-packet loop around ebpf_prog_run (ebpf_interpreter.c:23-372) with
// identical per-packet results.
//
// This variant keeps the eBPF register file in LDS (R[reg][lane], conflict-free for a
// wave-uniform register index) and does byte-wise, region-checked memory access.  It is the
// correctness baseline the hand-written gfx950 assembly interpreter (variant 0, asm/) is
// checked and timed against.
#include <hip/hip_runtime.h>

#include "../dprog.h"
#include "../jhash.h"

namespace {

constexpr int kWG = 256;
constexpr int kStack = 512;
constexpr int kHistBins = 257;

enum {
	F_NONE = 0, F_BAD_OPCODE = 1, F_DIV_ZERO = 2, F_MEM = 3, F_SLOT = 4, F_HELPER = 5,
	F_HELPER_UNSUPPORTED = 6, F_BAD_REG = 7, F_LOOP = 8, F_MAP_WRITE = 9, F_BAD_MAP = 10,
	F_WRITES = 11
};

// A logged write of the packet (dp_launch.vflags DP_VF_WCAP: counted; the one past
// DP_WRITES_MAX faults EBPF_FAULT_WRITES before it happens)
__device__ inline bool
over_cap(const dp_launch &L, uint32_t &writes)
{
	return (L.vflags & DP_VF_WCAP) && ++writes > DP_WRITES_MAX;
}

__device__ inline uint32_t
wave_min(uint32_t v)
{
	for (int o = 32; o > 0; o >>= 1)
		v = min(v, (uint32_t)__shfl_xor((int)v, o));
	return v;
}

struct regions {
	uint64_t pkt_lo, pkt_len, stk_lo;
};

// 0 = ok, else fault code.  Ranges: [pkt_lo, pkt_lo+len), [stk_lo, stk_lo+512), map mirrors'
// values (*map = the map's table index when the access lies there, else -1).
__device__ inline int
check(const regions &rg, const dp_launch &L, uint64_t a, uint32_t size, bool write, int *map = nullptr)
{
	if (map)
		*map = -1;
	if (rg.pkt_len >= size && a - rg.pkt_lo <= rg.pkt_len - size)
		return F_NONE;
	if (a - rg.stk_lo <= (uint64_t)(kStack - size))
		return F_NONE;
	for (uint32_t m = 0; m < L.nmaps; m++) {
		const dp_map &mp = L.maps[m];
		bool in;
		if (mp.flags & DP_MAP_HASH) { // only the value of an occupied-or-not slot
			const uint32_t lg = dp_hash_stride_log2(mp.flags);
			const uint64_t off = a - mp.dev_base;
			const uint64_t vo = dp_hash_value_off(dp_hash_key_size(mp.flags));
			const uint64_t so = off & ((1ull << lg) - 1);
			in = off < ((uint64_t)mp.max_entries << lg) && so >= vo && so - vo + size <= mp.value_size;
		} else {
			const uint64_t bytes = (uint64_t)mp.value_size * mp.max_entries;
			in = bytes >= size && a - mp.dev_base <= bytes - size;
		}
		if (in) {
			if (map)
				*map = (int)m;
			return F_NONE; // (stores too: ebpf_interpreter.c:343-366 writes the value in place)
		}
	}
	return F_MEM;
}

// The packet's own stores into map values (dp_launch.vflags bit 0): whole 8-byte words of the
// mirror as the packet sees them (dprog.h DP_OVL_*), newest last — in the lane's own DP_OVL_MAX
// entries, or in its slice of dp_launch.ovl_spill (a loop-free program that reads back more)
struct overlay {
	uint32_t n = 0;
	uint32_t cap = DP_OVL_MAX;
	uint64_t *addr;
	uint64_t *data;
	uint64_t own_addr[DP_OVL_MAX];
	uint64_t own_data[DP_OVL_MAX];
};

// `size` bytes at a: the mirror's (the batch-start values) with the packet's own stores over them
__device__ inline uint64_t
load_ovl(const overlay &o, uint64_t a, uint32_t size)
{
	uint64_t v = 0;
	for (uint32_t i = 0; i < size; i++) {
		const uint64_t b = a + i, w = b & ~7ull;
		uint8_t x = *reinterpret_cast<const uint8_t *>(b);
		for (uint32_t k = 0; k < o.n; k++)
			if (o.addr[k] == w)
				x = (uint8_t)(o.data[k] >> (8 * (b & 7)));
		v |= (uint64_t)x << (8 * i);
	}
	return v;
}

// Remember a store of `size` bytes of v at a; false, with nothing changed, when its words do not
// fit (only a program with loops that reads its counters back fills the overlay)
__device__ inline bool
ovl_store(overlay &o, uint64_t a, uint32_t size, uint64_t v)
{
	uint32_t fresh = 0;
	for (uint64_t w = a & ~7ull; w <= ((a + size - 1) & ~7ull); w += 8) {
		uint32_t k = 0;
		while (k < o.n && o.addr[k] != w)
			k++;
		fresh += k == o.n;
	}
	if (o.n + fresh > o.cap)
		return false;
	for (uint32_t i = 0; i < size; i++) {
		const uint64_t b = a + i, w = b & ~7ull;
		uint32_t k = 0;
		while (k < o.n && o.addr[k] != w)
			k++;
		if (k == o.n) {
			if (o.n == o.cap)
				return false;
			o.addr[k] = w;
			o.data[k] = *reinterpret_cast<const uint64_t *>(w); // (mirrors are padded to 8)
			o.n++;
		}
		const uint32_t sh = 8 * (uint32_t)(b & 7);
		o.data[k] = (o.data[k] & ~(0xffull << sh)) | ((uint64_t)(uint8_t)(v >> (8 * i)) << sh);
	}
	return true;
}

__device__ inline uint64_t
load_bytes(uint64_t a, uint32_t size)
{
	const uint8_t *p = reinterpret_cast<const uint8_t *>(a);
	uint64_t v = 0;
	for (uint32_t i = 0; i < size; i++)
		v |= (uint64_t)p[i] << (8 * i);
	return v;
}

__device__ inline void
store_bytes(uint64_t a, uint32_t size, uint64_t v)
{
	uint8_t *p = reinterpret_cast<uint8_t *>(a);
	for (uint32_t i = 0; i < size; i++)
		p[i] = (uint8_t)(v >> (8 * i));
}

__device__ inline bool
cond_taken(uint16_t op, uint64_t d, uint64_t s)
{
	switch (op & 0xf0) {
	case 0x10: return d == s;
	case 0x20: return d > s;
	case 0x30: return d >= s;
	case 0x40: return (d & s) != 0;
	case 0x50: return d != s;
	case 0x60: return (int64_t)d > (int64_t)s;
	case 0x70: return (int64_t)d >= (int64_t)s;
	case 0xa0: return d < s;
	case 0xb0: return d <= s;
	case 0xc0: return (int64_t)d < (int64_t)s;
	case 0xd0: return (int64_t)d <= (int64_t)s;
	}
	return false;
}

// hashtable_map_lookup_elem's search (ebpf_map_hashtable.c:285-301) over the device table:
// linear probing from jhash(key) to the key or an empty slot; the value's address or 0
__device__ inline uint64_t
hash_find(const dp_map &mp, const uint8_t *kp, uint32_t ks)
{
	const uint32_t hv = ebpf_jhash(kp, ks, 0);
	const uint32_t lg = dp_hash_stride_log2(mp.flags), mask = mp.max_entries - 1;
	for (uint32_t i = hv & mask;; i = (i + 1) & mask) {
		const uint8_t *slot = reinterpret_cast<const uint8_t *>(mp.dev_base + ((uint64_t)i << lg));
		const uint32_t *hdr = reinterpret_cast<const uint32_t *>(slot);
		if (hdr[0] == 0)
			return 0;
		if (hdr[1] != hv)
			continue;
		uint32_t b = 0;
		while (b < ks && slot[8 + b] == kp[b])
			b++;
		if (b == ks)
			return (uint64_t)(uintptr_t)(slot + dp_hash_value_off(ks));
	}
}

// A record in the batch's write log (dp_launch.upd_log): {u64 packet, u32 map << 20, u32 word},
// the rest for the caller; NULL when the log is full (the host sizes it: never)
__device__ inline uint8_t *
log_record(const dp_launch &L, uint64_t gid, uint32_t map, uint32_t word)
{
	if (L.upd_log == nullptr)
		return nullptr;
	const uint32_t slot = atomicAdd(reinterpret_cast<uint32_t *>(L.upd_log), 1u);
	if (slot >= L.upd_cap)
		return nullptr;
	uint8_t *rec = L.upd_log + 64 + (uint64_t)slot * L.upd_stride;
	*reinterpret_cast<uint64_t *>(rec) = L.pkt_base + gid;
	*reinterpret_cast<uint32_t *>(rec + 8) = map << 20;
	*reinterpret_cast<uint32_t *>(rec + 12) = word;
	return rec;
}

// A store of `size` bytes of v at a, inside the values of map mi (ebpf_gpu.h "Stores into map
// values"): `add` for a counter update adding `delta` (an addition when aligned to its width
// within the values, else a plain store of v).  UPD_ATOMIC maps take the addition into their
// delta area; the rest log a record for after the batch.  The packet's overlay remembers v.
// Returns 0 or a fault code.
__device__ inline int
value_store(const dp_launch &L, uint64_t gid, overlay &o, uint32_t &writes, int mi, uint64_t a,
	    uint32_t size, uint64_t v, bool add, uint64_t delta)
{
	const dp_map &mp = L.maps[mi];
	uint64_t off = a - mp.dev_base, voff = off;
	uint32_t slot = 0;
	if (mp.flags & DP_MAP_HASH) {
		const uint32_t lg = dp_hash_stride_log2(mp.flags);
		slot = (uint32_t)(off >> lg);
		voff = (off & ((1ull << lg) - 1)) - dp_hash_value_off(dp_hash_key_size(mp.flags));
	}
	add = add && voff % size == 0;
	const bool atomic = add && (mp.flags & DP_MAP_ATOMIC);
	if (!atomic && over_cap(L, writes)) // (every record counts; device atomics do not)
		return F_WRITES;
	// (a full overlay: only a program with loops that reads its counters back can fill it —
	// ebpf_gpu.h, 32 words — the write that needs one more faults WRITES before it happens)
	if ((L.vflags & 1) && !ovl_store(o, a, size, v))
		return F_WRITES;
	if (atomic) {
		uint8_t *d = reinterpret_cast<uint8_t *>(mp.dev_base) + dp_delta_off(mp.value_size, mp.max_entries) + off;
		if (size == 8)
			atomicAdd(reinterpret_cast<unsigned long long *>(d), (unsigned long long)delta);
		else
			atomicAdd(reinterpret_cast<uint32_t *>(d), (uint32_t)delta);
		return F_NONE;
	}
	uint8_t *rec = log_record(L, gid, (uint32_t)mi, (uint32_t)voff);
	if (rec == nullptr)
		return F_MEM;
	const uint64_t mask = size == 8 ? ~0ull : (1ull << (8 * size)) - 1;
	*reinterpret_cast<uint32_t *>(rec + 8) = ((uint32_t)mi << 20) | DP_REC_VALUE | (add ? DP_REC_ADD : 0u) | size;
	*reinterpret_cast<uint64_t *>(rec + 16) = (add ? delta : v) & mask;
	*reinterpret_cast<uint32_t *>(rec + 24) = slot;
	return F_NONE;
}

__global__ __launch_bounds__(kWG) void
ebpf_interp_v0(dp_launch L)
{
	__shared__ uint64_t R[11][kWG];
	__shared__ unsigned hist[kHistBins];
	const int tid = threadIdx.x;
	for (int b = tid; b < kHistBins; b += kWG)
		hist[b] = 0;
	__syncthreads();

	const uint64_t gid = (uint64_t)blockIdx.x * kWG + tid;
	const bool live = gid < L.count;
	uint8_t stack[kStack];
	regions rg;
	rg.pkt_lo = 0;
	rg.pkt_len = 0;
	if (live) {
		if (L.offsets) {
			// offsets[i], offsets[i + 1]; extents batches: offsets[2i], offsets[2i + 1].  An end
			// below its start or 4 GiB past it gives length 0 (every packet load faults MEM),
			// as in the assembly kernels
			const uint64_t k = (L.vflags & DP_VF_EXTENTS) ? 2 * gid : gid;
			const uint64_t lo = L.offsets[k], hi = L.offsets[k + 1];
			rg.pkt_lo = (uint64_t)L.data + (lo - L.off_base);
			rg.pkt_len = (hi >= lo && hi - lo < (1ull << 32)) ? hi - lo : 0;
		} else {
			rg.pkt_lo = (uint64_t)L.data + gid * L.stride;
			rg.pkt_len = L.stride;
		}
	}
	rg.stk_lo = (uint64_t)(uintptr_t)&stack[0];
	for (int r = 0; r < 11; r++)
		R[r][tid] = 0;
	R[1][tid] = rg.pkt_lo;
	R[10][tid] = rg.stk_lo + kStack;

	uint32_t T = L.start;
	bool active = live;
	int fault = F_NONE;
	uint64_t result = 0;
	uint32_t back = 0; // taken backward jumps (DK_LOOPCNT, standard semantics)
	overlay ovl;       // stores into map values the packet reads back (dp_launch.vflags)
	if (L.ovl_cap) {
		ovl.cap = L.ovl_cap;
		ovl.addr = reinterpret_cast<uint64_t *>(L.ovl_spill + (uint64_t)16 * L.ovl_cap * gid);
		ovl.data = ovl.addr + L.ovl_cap;
	} else {
		ovl.addr = ovl.own_addr;
		ovl.data = ovl.own_data;
	}
	uint32_t writes = 0; // logged writes (DP_VF_WCAP)

	for (;;) {
		const uint64_t am = __ballot(active);
		if (am == 0)
			break;
		const uint32_t t0 = (uint32_t)__shfl((int)T, __ffsll((long long)am) - 1);
		uint32_t t = t0;
		if (!__all(!active || T == t0))
			t = wave_min(active ? T : 0xffffffffu);
		t = __builtin_amdgcn_readfirstlane(t);
		if (!(active && T == t))
			continue;

		const dp_entry e = L.prog[t];
		const uint16_t k = e.kind;
		T = e.next;
		if (k == DK_FAULT) {
			fault = e.aux;
			active = false;
			continue;
		}
		const uint32_t cls = k & 7;
		if (k == 0x95) { // EXIT
			result = R[0][tid];
			active = false;
			continue;
		}
		if (k == DK_LOOPINIT) {
			back = 0;
			continue;
		}
		if (k == DK_OVLINIT) {
			ovl.n = 0;
			writes = 0;
			continue;
		}
		if (k == DK_LOOPCNT) {
			if (++back > DP_LOOP_BUDGET) {
				fault = F_LOOP;
				active = false;
			}
			continue;
		}
		if (k == DK_CALL_LOOKUP) {
			const uint64_t r1 = R[1][tid], r2 = R[2][tid];
			uint64_t res = 0;
			if (r1 != 0 && r2 != 0) {
				int mi = -1;
				for (uint32_t m = 0; m < L.nmaps; m++)
					if (L.maps[m].handle == r1) {
						mi = (int)m;
						break;
					}
				if (mi < 0) {
					fault = F_BAD_MAP;
					active = false;
					continue;
				}
				const dp_map &mp = L.maps[mi];
				const uint32_t ks = (mp.flags & DP_MAP_HASH) ? dp_hash_key_size(mp.flags) : 4;
				int f = check(rg, L, r2, ks, false);
				if (f) {
					fault = f;
					active = false;
					continue;
				}
				if (mp.flags & DP_MAP_HASH) {
					res = hash_find(mp, reinterpret_cast<const uint8_t *>(r2), ks);
				} else {
					uint32_t key = (uint32_t)load_bytes(r2, 4);
					if (key < mp.max_entries)
						res = mp.dev_base + (uint64_t)mp.value_size * key;
				}
			}
			R[0][tid] = res;
			continue;
		}
		if (k == DK_CALL_UPDATE) {
			// map_update_elem (ebpf_map.c:101-108 -> ebpf_map_array.c:185-211) with the device
			// batch's deferred write (map_writes.hip): the reference's return code, the write
			// logged for after the batch
			const uint64_t r2 = R[2][tid], r3 = R[3][tid], r4 = R[4][tid];
			uint64_t res = 22; // EINVAL: NULL key / value, flags > EBPF_EXIST
			if (r2 != 0 && r3 != 0 && r4 <= 2) {
				const dp_map &mp = L.maps[e.aux];
				if (mp.flags & DP_MAP_HASH) {
					// against the batch-start table (ebpf_map_hashtable.c:346-390): EEXIST /
					// ENOENT by the key's presence, EBUSY for a new key when the table was full;
					// a call that succeeds logs {flags << 8, key, value} for the host's replay
					const uint32_t ks = dp_hash_key_size(mp.flags);
					int f = check(rg, L, r2, ks, false);
					if (f) {
						fault = f;
						active = false;
						continue;
					}
					const uint8_t *kp = reinterpret_cast<const uint8_t *>(r2);
					const bool exists = hash_find(mp, kp, ks) != 0;
					const uint32_t *trailer = reinterpret_cast<const uint32_t *>(
					    mp.dev_base + dp_hash_trailer_off(mp.max_entries, mp.flags));
					res = exists && (r4 & 1) ? 17 : !exists && (r4 & 2) ? 2
					    : !exists && trailer[0] >= trailer[1] ? 16 : 0;
					if (res == 0) {
						if ((f = check(rg, L, r3, mp.value_size, false)) ||
						    (over_cap(L, writes) && (f = F_WRITES))) {
							fault = f;
							active = false;
							continue;
						}
						uint8_t *rec = log_record(L, gid, e.aux, (uint32_t)r4 << 8);
						if (!rec) {
							fault = F_MEM;
							active = false;
							continue;
						}
						const uint8_t *v = reinterpret_cast<const uint8_t *>(r3);
						for (uint32_t b = 0; b < ks; b++)
							rec[16 + b] = kp[b];
						for (uint32_t b = 0; b < mp.value_size; b++)
							rec[16 + dp_hash_key_bytes(ks) + b] = v[b];
					}
					R[0][tid] = res;
					continue;
				}
				if (r4 & 1) {
					res = 17; // EEXIST (EBPF_NOEXIST)
				} else {
					int f = check(rg, L, r2, 4, false);
					const uint32_t key = f ? 0 : (uint32_t)load_bytes(r2, 4);
					if (!f && key < mp.max_entries)
						f = check(rg, L, r3, mp.value_size, false);
					if (f) {
						fault = f;
						active = false;
						continue;
					}
					if (key < mp.max_entries) {
						if (over_cap(L, writes)) {
							fault = F_WRITES;
							active = false;
							continue;
						}
						uint8_t *rec = log_record(L, gid, e.aux, key);
						if (!rec) {
							fault = F_MEM; // (the host sizes the log: never)
							active = false;
							continue;
						}
						const uint8_t *v = reinterpret_cast<const uint8_t *>(r3);
						for (uint32_t b = 0; b < mp.value_size; b++)
							rec[16 + b] = v[b];
						res = 0;
					}
				}
			}
			R[0][tid] = res;
			continue;
		}
		if (k == DK_CALL_HDELETE) {
			// map_delete_elem on a hashtable (ebpf_map.c:126-132 -> ebpf_map_hashtable.c:
			// 475-502): EINVAL for a NULL key, else 0 with {1, key} logged for the host's replay
			const uint64_t r2 = R[2][tid];
			uint64_t res = 22;
			if (r2 != 0) {
				const dp_map &mp = L.maps[e.aux];
				const uint32_t ks = dp_hash_key_size(mp.flags);
				int f = check(rg, L, r2, ks, false);
				if (!f && over_cap(L, writes))
					f = F_WRITES;
				uint8_t *rec = f ? nullptr : log_record(L, gid, e.aux, 1);
				if (f || !rec) {
					fault = f ? f : F_MEM;
					active = false;
					continue;
				}
				const uint8_t *kp = reinterpret_cast<const uint8_t *>(r2);
				for (uint32_t b = 0; b < ks; b++)
					rec[16 + b] = kp[b];
				res = 0;
			}
			R[0][tid] = res;
			continue;
		}
		if (k >= DK_MOV64R && k <= DK_MOD32Z) { // standard-eBPF operations
			const uint64_t d = R[e.dst][tid], s = R[e.src][tid];
			const uint32_t d32 = (uint32_t)d, s32 = (uint32_t)s;
			uint64_t r;
			switch (k) {
			case DK_MOV64R: r = s; break;
			case DK_NEG64: r = 0 - d; break;
			case DK_NEG32: r = (uint32_t)(0u - d32); break;
			case DK_ARSH64I: r = (uint64_t)((int64_t)d >> (e.imm & 63)); break;
			case DK_ARSH64R: r = (uint64_t)((int64_t)d >> (s & 63)); break;
			case DK_ARSH32I: r = (uint32_t)((int32_t)d32 >> (e.imm & 31)); break;
			case DK_ARSH32R: r = (uint32_t)((int32_t)d32 >> (s32 & 31)); break;
			case DK_DIV64Z: r = s ? d / s : 0; break;
			case DK_MOD64Z: r = s ? d % s : d; break;
			case DK_DIV32Z: r = s32 ? d32 / s32 : 0; break;
			default: r = s32 ? d32 % s32 : d32; break;
			}
			R[e.dst][tid] = r;
			continue;
		}
		if (cls == DP_CLS_JMP32) { // standard eBPF: compares of the low 32 bits
			const uint32_t d = (uint32_t)R[e.dst][tid];
			const uint32_t s = (k & 0x08) ? (uint32_t)R[e.src][tid] : (uint32_t)e.imm;
			const bool sg = (k & 0xf0) == 0x60 || (k & 0xf0) == 0x70 || (k & 0xf0) == 0xc0 ||
					(k & 0xf0) == 0xd0;
			const uint64_t dx = sg ? (uint64_t)(int64_t)(int32_t)d : d;
			const uint64_t sx = sg ? (uint64_t)(int64_t)(int32_t)s : s;
			if (cond_taken(k, dx, sx))
				T = e.target;
			continue;
		}
		if (cls == 0x5) { // conditional jumps (JA and CALL/EXIT handled above / folded)
			const uint64_t d = R[e.dst][tid];
			const uint64_t s = (k & 0x08) ? R[e.src][tid] : e.imm;
			if (cond_taken(k, d, s))
				T = e.target;
			continue;
		}
		if (k < 0x100 && cls == 0x1) { // LDX
			const uint32_t size = (k & 0x18) == 0x00 ? 4 : (k & 0x18) == 0x08 ? 2 : (k & 0x18) == 0x10 ? 1 : 8;
			const uint64_t a = R[e.src][tid] + (uint64_t)(int64_t)e.off;
			int mi;
			int f = check(rg, L, a, size, false, &mi);
			if (f) {
				fault = f;
				active = false;
				continue;
			}
			R[e.dst][tid] = mi >= 0 && ovl.n ? load_ovl(ovl, a, size) : load_bytes(a, size);
			continue;
		}
		if (k == DK_CNT_STORE || k == DK_XADD || cls == 0x2 || cls == 0x3) {
			// ST / STX; the STX of a counter update; XADD (standard semantics)
			const uint32_t size = k >= 0x100 ? (e.aux & 0xff)
					      : (k & 0x18) == 0x00 ? 4 : (k & 0x18) == 0x08 ? 2 : (k & 0x18) == 0x10 ? 1 : 8;
			const uint64_t a = R[e.dst][tid] + (uint64_t)(int64_t)e.off;
			int mi;
			int f = check(rg, L, a, size, true, &mi);
			if (f) {
				fault = f;
				active = false;
				continue;
			}
			const uint64_t mask = size == 8 ? ~0ull : (1ull << (8 * size)) - 1;
			uint64_t v = (k < 0x100 && cls == 0x2) ? e.imm : R[e.src][tid], delta = 0, old = 0;
			const bool add = k == DK_CNT_STORE || k == DK_XADD;
			if (add) {
				old = mi >= 0 && ovl.n ? load_ovl(ovl, a, size) : load_bytes(a, size);
				delta = k == DK_XADD ? v : v - old; // (a counter update: what the ADD / SUB added)
				if (k == DK_XADD)
					v = old + v;
			}
			if (mi >= 0)
				f = value_store(L, gid, ovl, writes, mi, a, size, v, add, delta & mask);
			else
				store_bytes(a, size, v);
			if (f) {
				fault = f;
				active = false;
				continue;
			}
			if (k == DK_XADD && (e.aux & 0x100)) // BPF_FETCH: src = the old value
				R[e.src][tid] = old & mask;
			continue;
		}
		if (k == 0x18) { // LDDW
			R[e.dst][tid] = e.imm;
			continue;
		}
		// ALU / ALU64
		const uint64_t d = R[e.dst][tid];
		const uint64_t s = (k & 0x08) ? R[e.src][tid] : e.imm;
		uint64_t r;
		if (cls == 0x4) {
			const uint32_t d32 = (uint32_t)d, s32 = (uint32_t)s;
			switch (k & 0xf0) {
			case 0x00: r = (uint32_t)(d32 + s32); break;
			case 0x10: r = (uint32_t)(d32 - s32); break;
			case 0x20: r = (uint32_t)(d32 * s32); break;
			case 0x30:
				if (!s32) { fault = F_DIV_ZERO; active = false; continue; }
				r = d32 / s32;
				break;
			case 0x40: r = d32 | s32; break;
			case 0x50: r = d32 & s32; break;
			case 0x60: r = (uint32_t)(d32 << (s32 & 31)); break;
			case 0x70: r = d32 >> (s32 & 31); break;
			case 0x80: r = (uint32_t)(0u - (uint32_t)e.imm); break; // NEG ignores dst
			case 0x90:
				if (!s32) { fault = F_DIV_ZERO; active = false; continue; }
				r = d32 % s32;
				break;
			case 0xa0: r = d32 ^ s32; break;
			case 0xb0: r = s32; break;
			case 0xc0: r = d32 >> (s32 & 31); break; // logical
			default: { // 0xd0: LE / BE
				const int64_t w = (int64_t)e.imm;
				r = d;
				if (k == 0xd4) {
					if (w == 16) r = (uint16_t)d;
					else if (w == 32) r = (uint32_t)d;
				} else {
					if (w == 16) r = __builtin_bswap16((uint16_t)d);
					else if (w == 32) r = __builtin_bswap32((uint32_t)d);
					else if (w == 64) r = __builtin_bswap64(d);
				}
			}
			}
		} else {
			switch (k & 0xf0) {
			case 0x00: r = d + s; break;
			case 0x10: r = d - s; break;
			case 0x20: r = d * s; break;
			case 0x30:
				if (!s) { fault = F_DIV_ZERO; active = false; continue; }
				r = d / s;
				break;
			case 0x40: r = d | s; break;
			case 0x50: r = d & s; break;
			case 0x60: r = d << (s & 63); break;
			case 0x70: r = d >> (s & 63); break;
			case 0x80: r = d - e.imm; break; // NEG64 = dst - imm
			case 0x90:
				if (!s) { fault = F_DIV_ZERO; active = false; continue; }
				r = d % s;
				break;
			case 0xa0: r = d ^ s; break;
			case 0xb0: r = d + s; break; // MOV64 adds
			default: r = d >> (s & 63); break; // 0xc0 ARSH64, logical
			}
		}
		R[e.dst][tid] = r;
	}

	if (live) {
		L.ret[gid] = fault ? 0 : result;
		if (L.faults)
			L.faults[gid] = (uint8_t)fault;
		if (fault && L.upd_faulted) { // its logged map writes do not land
			const uint32_t b = (uint32_t)(L.pkt_base + gid);
			atomicOr(&L.upd_faulted[b >> 5], 1u << (b & 31));
		}
		if (L.hist)
			atomicAdd(&hist[fault ? 256 : (result < 255 ? (unsigned)result : 255u)], 1u);
	}
	if (L.hist) {
		__syncthreads();
		for (int b = tid; b < kHistBins; b += kWG)
			if (hist[b])
				atomicAdd(&L.hist[b], (unsigned long long)hist[b]);
	}
}

} // namespace

namespace {

} // namespace

hipError_t
launch_interp_v0(const dp_launch &L, hipStream_t stream)
{
	if (L.count == 0)
		return hipSuccess;
	// (a spilled overlay: in chunks of the packets its buffer holds, launched in stream order)
	const uint64_t chunk = L.ovl_cap ? L.ovl_chunk : L.count;
	for (uint64_t c0 = 0; c0 < L.count; c0 += chunk) {
		dp_launch C = L;
		C.count = L.count - c0 < chunk ? L.count - c0 : chunk;
		if (L.offsets)
			C.offsets = L.offsets + ((L.vflags & DP_VF_EXTENTS) ? 2 * c0 : c0);
		else
			C.data = L.data + c0 * L.stride;
		C.ret = L.ret + c0;
		if (L.faults)
			C.faults = L.faults + c0;
		C.pkt_base = L.pkt_base + c0;
		const uint64_t blocks = (C.count + kWG - 1) / kWG;
		hipLaunchKernelGGL(ebpf_interp_v0, dim3((unsigned)blocks), dim3(kWG), 0, stream, C);
		hipError_t e = hipGetLastError();
		if (e != hipSuccess)
			return e;
	}
	return hipSuccess;
}
