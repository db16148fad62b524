// dprog.h — the device program: the reference's bytecode unrolled into its executed states.
//
// The reference interpreter walks slots with a cumulative counter (ebpf_interpreter.c:39
// "inst = inst + pc++"), so what executes next depends on the pair (slot i, pc p), not on the
// slot alone.  The translator (translate.cpp) enumerates every (i, p) state reachable from
// (0, 1) and emits one dp_entry per state, with explicit successor indices.  The device kernels
// then never compute slot arithmetic: they follow `next` / `target`.  JA states are folded into
// their successors (a JA has no effect besides the state change), DIV/MOD by a zero immediate,
// invalid opcodes, bad registers, leaving the program and self-re-entering jumps become FAULT
// entries, and each CALL is resolved against the env's helper table at translation time.
//
// Shared by host C++ and HIP device code: plain C layout, 32 bytes per entry.
#pragma once
#include <stdint.h>
#include <stddef.h>

enum dp_kind : uint16_t {
	// 0x00..0xff: the eBPF opcode itself (ALU, ALU64, LDX, ST, STX, LDDW, cond jumps, EXIT)
	DK_FAULT = 0x100,       // terminal: aux = ebpf_fault code
	DK_CALL_LOOKUP = 0x101, // r0 = map_lookup_elem(r1, r2)  (ebpf_map.c:77-84)
	// standard-eBPF semantics (EBPF_SEM_STANDARD) where they differ from the reference's;
	// MOV64_IMM becomes an LDDW entry (dst = sext(imm)), and JMP32 entries keep their opcode
	// (class 0x06)
	DK_MOV64R = 0x102,  // dst = src
	DK_NEG64 = 0x103,   // dst = -dst
	DK_NEG32 = 0x104,   // dst = u32(-dst)
	DK_ARSH64I = 0x105, // dst = (s64)dst >> imm   (imm already masked to 63)
	DK_ARSH64R = 0x106, // dst = (s64)dst >> (src & 63)
	DK_ARSH32I = 0x107, // dst = u32((s32)dst >> imm)
	DK_ARSH32R = 0x108, // dst = u32((s32)dst >> (src & 31))
	DK_DIV64Z = 0x109,  // dst = src ? dst / src : 0
	DK_MOD64Z = 0x10a,  // dst = src ? dst % src : dst
	DK_DIV32Z = 0x10b,  // 32-bit forms, results zero-extended
	DK_MOD32Z = 0x10c,
	// map-writing helpers (device-batch semantics, ebpf_gpu.h "Map writes in a device batch");
	// the map is a translation-time constant: aux = its index in the dp_map table
	DK_CALL_UPDATE = 0x10d, // r0 = map_update_elem(map, r2, r3, r4) (ebpf_map.c:101-108)
	// Loops (standard semantics only; the reference's state graph is a tree): every taken
	// backward jump (a jump whose target is at or before its own slot) passes a LOOPCNT entry
	// that counts it for the lane; the (DP_LOOP_BUDGET + 1)-th faults EBPF_FAULT_LOOP.  The
	// program starts at a LOOPINIT entry (the lane's count = 0).  The count lives in the first
	// 4 bytes of the lane's stack slice, below the frame the program can address.
	DK_LOOPINIT = 0x10e,
	DK_LOOPCNT = 0x10f,
	// r0 = map_delete_elem(map, r2) on a hashtable map known at translation time (aux = its
	// table index): 0, the delete logged for after the batch (ebpf_map.c:130-136 ->
	// ebpf_map_hashtable.c:475-502); a NULL key is EINVAL
	DK_CALL_HDELETE = 0x110,
	// Stores into map values with the device batch's counter semantics (ebpf_gpu.h "Stores into
	// map values"): the STX of a counter update — the translator found LDX{W,DW} X = [P + off];
	// ADD/SUB X; STX [P + off] = X on one path — stores X like the STX (dst = P, src = X, off;
	// aux = 4 or 8 bytes) and, into a map value, adds X minus the value it re-reads there
	// (the packet's own view: nothing stored in between) instead of overwriting it.  aux bit 9:
	// the update's addend is an immediate, in imm (what the ADD / SUB adds)
	DK_CNT_STORE = 0x111,
	// XADD (standard semantics, BPF_STX | BPF_XADD): *(u32 / u64 *)(dst + off) += src; aux = 4
	// or 8 bytes, | 0x100 when imm was BPF_FETCH (src = the old value)
	DK_XADD = 0x112,
	// A program that reads its own stores into map values, or whose writes are capped, starts
	// here: the lane's overlay is emptied and its write count zeroed (DP_OVL_COUNT, DP_WCOUNT = 0)
	DK_OVLINIT = 0x113,
};
#define DP_VF_EXTENTS 4u // dp_launch.vflags: offsets are (start, end) pairs
// dp_launch.vflags: the assembly interpreter's staged kernel keeps each group's packets in the
// wave's LDS packet buffer until the group ends (keep mode: LDXPKTV reads them there)
#define DP_VF_KEEP 8u
// dp_launch.vflags: count each packet's logged writes and fault the one past DP_WRITES_MAX
#define DP_VF_WCAP 16u
#define DP_LOOP_BUDGET (1u << 20) // taken backward jumps a lane may make (standard semantics)
#define DP_CLS_JMP32 6

struct dp_entry {
	uint64_t handler; // asm interpreter: absolute handler address (patched per device)
	uint64_t imm;     // pre-extended immediate: sext(imm) for ALU64/JMP, u32(imm) for ALU32,
	                  // the full 64-bit value for LDDW
	uint32_t next;    // successor when the instruction falls through / jump not taken
	uint32_t target;  // successor when a conditional jump is taken
	uint16_t kind;    // dp_kind or opcode
	uint8_t dst, src;
	int16_t off;
	uint16_t aux;     // DK_FAULT: fault code
};
static_assert(sizeof(dp_entry) == 32, "dp_entry is 32 bytes");

// One map visible to device programs (resolved LDDW handle → device mirror).
//
// Array maps: the mirror is the value array (max_entries * value_size bytes), flags = 0.
// Hashtable maps (flags & DP_MAP_HASH): the mirror is a read-only open-addressing snapshot of
// the host table, rebuilt on upload: max_entries holds the slot count (a power of two, at least
// four times the map's max_entries, so every probe sequence reaches an empty slot), flags holds the
// key size and log2 of the slot stride.  Slot layout (stride a power of two):
//   u32 used (1) | u32 jhash(key) | key, zero-padded to dp_hash_key_bytes | value[value_size]
// A key hashes to slot jhash(key, key_size, 0) & (slots - 1), then linear probing.  Programs
// may read [value, value + value_size) through a lookup result; anything else in the table
// faults like any stray address.
struct dp_map {
	uint64_t handle;      // the value programs load with LDDW: the host struct ebpf_map*
	uint64_t dev_base;    // device address of the mirror
	uint32_t value_size;
	uint32_t max_entries; // hashtable: slot count
	uint32_t lds_off;     // assembly interpreter: LDS byte address of the map's copy, or ~0u
	uint32_t flags;       // DP_MAP_HASH | log2(stride) << 16 | key_size (hashtable), else 0
};
#define DP_MAP_HASH 0x80000000u
// Array maps the program changes only by counter updates, all aligned and of one width (the
// translator proves it): those land as device atomics into the map's delta area, right after its
// values in the mirror (dp_delta_off), added into the mirror after the batch.  Bit 28: 8-byte
// counters (else 4-byte).
#define DP_MAP_ATOMIC 0x40000000u
#define DP_MAP_ATOMIC64 0x10000000u
// ... whose counter updates the assembly kernels first sum per workgroup in an LDS table (at the
// LDS address in flags bits 0..15, zeroed at kernel start), added into the delta area when the
// workgroup ends: one global atomic per touched word and workgroup instead of one per update
#define DP_MAP_LDSDELTA 0x20000000u
#define DP_HASH_MAX_KEY 65535u // (the key size field of dp_map.flags)
#if defined(__HIPCC__)
#define DP_FN __host__ __device__ static inline
#else
#define DP_FN static inline
#endif
DP_FN uint32_t dp_hash_key_size(uint32_t flags) { return flags & 0xffffu; }
DP_FN uint32_t dp_hash_stride_log2(uint32_t flags) { return (flags >> 16) & 0x1fu; }
DP_FN uint32_t dp_hash_key_bytes(uint32_t key_size) { return (key_size + 7u) & ~7u; }
// offset of the value in a slot
DP_FN uint32_t dp_hash_value_off(uint32_t key_size) { return 8u + dp_hash_key_bytes(key_size); }
static_assert(sizeof(dp_map) == 32, "dp_map is 32 bytes");
// An array mirror's bytes are padded to 64 (loads of whole 8-byte words stay inside it), then the
// delta area of a DP_MAP_ATOMIC map (as many bytes again)
DP_FN uint64_t dp_delta_off(uint32_t value_size, uint32_t max_entries)
{
	return ((uint64_t)value_size * max_entries + 63u) & ~(uint64_t)63u;
}
// A hashtable's device table is followed by a 16-byte trailer: u32 live entries of the table the
// mirror was built from, u32 the map's max_entries (a device batch's map_update_elem of a new
// key is EBUSY when the batch-start table is full, ebpf_map_hashtable.c:371-375)
DP_FN uint64_t dp_hash_trailer_off(uint32_t slots, uint32_t flags)
{
	return (uint64_t)slots << dp_hash_stride_log2(flags);
}

// Kernel arguments (passed by value).
struct dp_launch {
	const dp_entry *prog;
	const dp_map *maps;
	uint8_t *data;
	const uint64_t *offsets; // NULL → fixed stride; else packet i = data + offsets[i] - off_base
	uint64_t off_base;
	uint64_t *ret;
	uint8_t *faults;         // may be NULL
	unsigned long long *hist; // EBPF_HIST_BINS counters, may be NULL
	uint64_t count;
	uint32_t stride;
	uint32_t start;          // entry index of the initial state (0, 1)
	uint32_t nmaps;
	uint32_t nentries;
	// assembly interpreter only:
	uint32_t stack_stride;    // LDS bytes per lane stack slice (S' in asm_runtime.cpp)
	uint32_t lds_stack_base;  // LDS byte offset of the first stack slice (after the histogram)
	uint32_t total_waves;     // persistent grid: waves in the launch (group stride); bits
	                          // 28..29: log2 of the superblock size (staged kernels)
	uint32_t lds_pkt_base;    // staged kernel: LDS byte offset of the per-wave packet buffers
	uint32_t *hist_rows;      // assembly kernels: the launch's private verdict partials
	                          // (DP_HIST_* layout below; hist points at it too, so faults count
	                          // into replica 0's bin 256); NULL = per-bin atomics into hist
	unsigned long long *hist_user; // the caller's histogram: the last workgroup stores (flags
	                          // bit 0) or adds the reduced partials there
	uint32_t hist_flags;      // bit 0: store instead of add (EBPF_BATCH_HIST_OVERWRITE)
	uint32_t nwg;             // workgroups in this launch (the ticket's arrival count)
	// map writes (DK_CALL_UPDATE): the batch's log, u32 record count at +0, records from +64:
	// {u64 packet index, u32 entry | map << 20, u32 key, value[value_size]}, upd_stride apart
	uint8_t *upd_log;
	uint32_t upd_cap;         // records the log holds
	uint32_t upd_stride;
	uint64_t pkt_base;        // index of this launch's first packet in its batch
	uint8_t *reserved0;       // (unused; keeps the offsets the assembly kernels load)
	uint32_t reserved1;
	uint32_t reserved2;
	// map writes: one bit per packet of the batch (index pkt_base + i, cleared by the host before
	// the batch), set when the packet faults; the apply step skips a faulted packet's logged
	// writes (a packet that faults leaves no write behind).  NULL for programs without map writes
	uint32_t *upd_faulted;
	const void *reserved3[2]; // (unused; keep vflags at the offset the assembly kernels load)
	uint32_t reserved4[3];
	// stores into map values (ebpf_gpu.h "Stores into map values"): bit 0 = the program reads
	// its own stores (an overlay of the words it stored, per lane: DP_OVL_* below); bit 1 = it
	// has value-store sites; bit 2 (DP_VF_EXTENTS) = `offsets` holds (start, end) pairs
	// (EBPF_BATCH_EXTENTS); bits 8..15 = the overlay's entries per lane
	uint32_t vflags;
	// staged kernels with result bursts: write phasing (gen_interp.py store_phased).  A wave keeps
	// its finished groups' results in registers and writes them while the GPU's constant clock
	// (s_memrealtime) is in a write window — (t mod 2^bits 16..20) < bits 0..15 — or when its
	// slots are full, so that result writes and packet reads reach HBM in separate phases.
	// 0 = off: results written once per superblock
	uint32_t wphase;
	// a loop-free program that reads back more stores into map values than DP_OVL_MAX words hold
	// (the portable HIP interpreter only): every lane's overlay in global memory, ovl_cap
	// {address, word} entries per lane at ovl_spill + 16 * ovl_cap * (lane's index in the launch);
	// 0 = the lane's own DP_OVL_MAX entries.  The launch runs in chunks of ovl_chunk packets
	// (what the buffer holds), in stream order
	uint32_t ovl_cap;
	uint32_t ovl_chunk;
	uint32_t reserved5;
	uint8_t *ovl_spill;
};
static_assert(sizeof(dp_launch) == 232, "dp_launch layout is shared with the assembly kernels");
static_assert(offsetof(dp_launch, vflags) == 0xcc, "gen_interp.py VFLAGS_OFF");
static_assert(offsetof(dp_launch, wphase) == 0xd0, "gen_interp.py WPHASE_OFF");

// The lane's LDS stack slice, below the frame the program addresses: the loop count (+0), the
// overlay's entry count (+4), an 8-byte scratch a store into a map value is redirected to (+8),
// the packet's logged writes (+16, dp_launch.vflags DP_VF_WCAP) and the overlay entries (+24:
// {u64 word address, u64 word as the packet sees it}, 16 B each).  Programs with value stores or
// capped writes keep at least the first 24 bytes.
#define DP_OVL_COUNT 4u
#define DP_OVL_SCRATCH 8u
#define DP_WCOUNT 16u
#define DP_OVL_ENTRIES 24u
#define DP_OVL_MAX 32u // overlay entries per lane kept on chip (more: dp_launch.ovl_spill)
#define DP_OVL_SPILL_MAX 4096u // ... spilled entries per lane at most (more: EOPNOTSUPP)
// Logged writes a packet may make in a device batch (ebpf_gpu.h "Map writes in a device batch":
// successful map_update_elem / map_delete_elem calls and stores into map values other than
// aligned counter updates); the next one faults EBPF_FAULT_WRITES.  Checked on the device only
// where a path can exceed it (programs with loops, dp_launch.vflags DP_VF_WCAP); 2 x this many
// overlay words hold every store it allows (DP_OVL_MAX)
#define DP_WRITES_MAX 16u

// Value-store records in the batch's write log: {u64 packet, u32 map << 20 | DP_REC_VALUE |
// kind << 16 | size, u32 byte offset (array: in the map's values; hashtable: in the value),
// u64 data (the stored bytes, or a counter's addend), u32 hashtable slot}
#define DP_REC_VALUE 0x80000u
#define DP_REC_ADD 0x10000u
#define DP_REC_VALUE_BYTES 32u

// Verdict partials of one assembly-kernel launch (gen_interp.py .Lfinish): 8 replicas of
// EBPF_HIST_BINS u64 (workgroup w adds to replica w & 7), then 9 u32 arrival tickets on 64-B
// lines of their own (one per replica, then the top one).  All zero between launches: the last
// workgroup swaps every word back to 0.
#define DP_HIST_REPLICAS 8u
#define DP_HIST_REPLICA_BYTES (257u * 8u)
#define DP_HIST_TICKET_OFF (DP_HIST_REPLICAS * DP_HIST_REPLICA_BYTES)
#define DP_HIST_PARTIAL_BYTES (DP_HIST_TICKET_OFF + 64u * (DP_HIST_REPLICAS + 1u))
