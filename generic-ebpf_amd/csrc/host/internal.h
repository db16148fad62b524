// internal.h — object model of the engine's libebpf.so (host side).
//
// Mirrors the reference's object core:
//   struct ebpf_env  ↔ sys/dev/ebpf/ebpf_env.h   (config + live-object refcount)
//   struct ebpf_obj  ↔ sys/dev/ebpf/ebpf_obj.h:35-40 (env ref, refcount, type, dtor; first member)
//   struct ebpf_prog ↔ sys/dev/ebpf/ebpf_prog.h:23-30
//   struct ebpf_map  ↔ sys/dev/ebpf/ebpf_map.h:23-32
// plus the per-device state the GPU backend keeps (translated program, map mirrors).
#pragma once

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "ebpf.h"
#include "ebpf_gpu.h"
#include "ebpf_vm_isa.h"
#include "../dprog.h"
#include "map_writes.h"

#define EBPF_EXPORT extern "C" __attribute__((visibility("default")))

enum ebpf_obj_type_id : uint32_t { EBPF_OBJ_TYPE_PROG = 0, EBPF_OBJ_TYPE_MAP = 1 };

struct ebpf_env {
	std::atomic<uint32_t> ref{0};   // live objects (ebpf_env.c:31 starts at 0)
	const struct ebpf_config *ec = nullptr;
	std::mutex lock;
	std::set<struct ebpf_map *> maps; // live maps: resolves LDDW handles to map objects
};

struct ebpf_obj {
	struct ebpf_env *eo_ee;
	std::atomic<uint32_t> eo_ref;
	uint32_t eo_type;
	void (*eo_dtor)(struct ebpf_obj *);
};

// Per-device mirror of one map's storage.
struct map_mirror {
	void *dev = nullptr;
	uint64_t version = ~0ull; // host version last uploaded
	uint16_t cpu = 0;         // percpu maps: the CPU whose copy was uploaded
	// host staging copy of the last upload (hashtable: the device table); a new upload makes a
	// new one, so a batch that captured it keeps the table its packets read
	std::shared_ptr<const std::vector<uint8_t>> image;
	// Cross-stream order of the mirror's users on its device (gpu_runtime.cpp mirror_read /
	// mirror_write_*): a write (an upload, or a batch's map writes landing) waits for every
	// launch that read the mirror on another stream since the previous write, and a launch on a
	// stream waits for the last write made on another stream.
	void *wr_ev = nullptr;         // hipEvent_t recorded after the last write
	std::vector<void *> synced;    // streams ordered after that write
	std::vector<void *> readers;   // streams whose launches read the mirror since that write
};

// The device mirror of a map (maps.cpp).  Array maps mirror their value array, hashtables a
// read-only open-addressing table (dprog.h dp_map).  Percpu maps mirror the copy of the CPU the
// batch is submitted from: a device batch behaves like the caller's own loop over
// ebpf_prog_run on its current CPU.  `bytes == 0` means no device form (hashtable keys over
// DP_HASH_MAX_KEY, tables over 64 GiB).
struct map_device_layout {
	size_t bytes = 0;
	uint32_t slots = 0; // dp_map.max_entries
	uint32_t flags = 0; // dp_map.flags
};
map_device_layout map_device_layout_of(const struct ebpf_map *em);
// Hashtable: fill `out` (layout.bytes) with the current table (percpu: `cpu`'s values), under
// the map's lock.
void map_device_image(struct ebpf_map *em, std::vector<uint8_t> &out, uint16_t cpu);
// Array / percpu array: the value array to mirror (percpu: `cpu`'s copy).
const uint8_t *map_array_image(struct ebpf_map *em, uint16_t cpu);
// The CPU the calling thread runs on, as the percpu maps index it (ebpf_linux_user.c:83-112).
uint16_t map_current_cpu();

struct ebpf_map {
	struct ebpf_obj eo; // must stay first (callers cast to struct ebpf_obj *)
	const struct ebpf_map_type *emt;
	uint32_t key_size;
	uint32_t value_size;
	uint32_t map_flags;
	uint32_t max_entries;
	bool percpu;
	void *data;                       // map-type private data
	std::atomic<uint64_t> version{0}; // bumped on every host-side write
	std::mutex mirror_lock;
	std::vector<map_mirror> mirrors;  // indexed by device
	// held by a launch from its mirror sync to its last enqueue, so that the reads and writes it
	// registers (map_mirror.readers / wr_ev) match the order its work reaches the streams
	std::mutex order_lock;
	// a device batch wrote the map (map_update_elem): that device's mirror is newer than the
	// host copy until map_pull_device_writes copies it back (after wb_event, a hipEvent_t)
	std::atomic<int> dev_dirty{-1};
	void *wb_event = nullptr;
	// array-map storage (for device mirroring); null for other map types
	uint8_t *array_storage() const;
	bool is_hashtable() const; // hashtable or percpu hashtable
};

// Assembly-interpreter LDS layout (per workgroup): verdict histogram [0, kHistLds), LDS-resident
// array-map copies [kMapLdsBase, + map_lds_bytes), staged kernel only: 4 per-wave 4-KB packet
// buffers, then the 256 per-lane stack slices.
constexpr uint32_t kHistLds = 1024; // bins 0..255 (bin 256 is counted in global memory)
constexpr uint32_t kMapLdsBase = kHistLds;
constexpr uint32_t kMapLdsBudget = 8192;
constexpr uint32_t kPktLdsPerWG = 4 * 4096;
// staged kernels, compiled programs: workgroups per CU for streaming programs (write phasing on
// long launches) and for programs that probe hashtables (gpu_runtime.cpp; the others: as many as
// LDS and VGPRs allow)
constexpr uint32_t kStreamWorkgroups = 4;
constexpr uint32_t kProbeWorkgroups = 5;

// The assembly interpreter's code objects (build/asm_image.cpp): mode 1 = staged 64-B kernels,
// mode 0 = general kernels.  Image 3 is mode 1 for the interpreter itself (variant 2): one
// result group per burst, 64 VGPRs and s0..s73, so 8 workgroups per CU are resident instead of 6
// (gen_interp.py NSGPR_INTERP).
constexpr int kModes = 2;
constexpr int kInterpStagedImage = 3;
extern __attribute__((visibility("hidden"))) const unsigned char ebpf_asm_hsaco_m1[], ebpf_asm_hsaco_m0[],
    ebpf_asm_hsaco_m3[];
extern __attribute__((visibility("hidden"))) const size_t ebpf_asm_hsaco_m1_len, ebpf_asm_hsaco_m0_len,
    ebpf_asm_hsaco_m3_len;
inline const unsigned char *asm_image(int mode)
{
	return mode == 1 ? ebpf_asm_hsaco_m1 : mode == 3 ? ebpf_asm_hsaco_m3 : ebpf_asm_hsaco_m0;
}
inline size_t asm_image_len(int mode)
{
	return mode == 1 ? ebpf_asm_hsaco_m1_len : mode == 3 ? ebpf_asm_hsaco_m3_len
		: ebpf_asm_hsaco_m0_len;
}

// Per (program, device): entries for each interpreter variant and the map table.
struct dprog_device {
	int device = -1;
	dp_entry *d_entries = nullptr;   // variant 1 (portable HIP): translated entries as is
	dp_map *d_maps = nullptr;
	std::vector<dp_map> table;
	uint32_t nentries = 0;
	uint32_t nmaps = 0;
	uint32_t map_lds_bytes = 0;      // LDS bytes taken by LDS-resident map copies (asm kernels)
	dp_entry *d_asm[kModes] = {};            // variant 2: lowered + linked, per mode
	uint32_t asm_stride[kModes] = {};        // LDS stack bytes per lane, per mode
	int asm_err[kModes] = {};
	void *jit_mod[kModes] = {};              // variant 0: compiled program module, per mode
	void *jit_fn[kModes] = {};               // its kernel
	void *jit_fn_wide = nullptr;             // mode 1: the same code with 16 result slots
	uint32_t jit_stride[kModes] = {};
	int jit_err[kModes] = {};                // E2BIG etc.: run the interpreter instead
	double build_ms[kModes] = {};            // compile (variant 0) or lower + link time, per mode
	void *d_upd = nullptr;                   // map writes: upd_map per table map (map_writes.h)
	std::vector<struct upd_map> upd_host;    // ... and its host copy
	uint64_t win_words = 0;                  // winner words the apply step needs
	uint32_t upd_stride = 0;                 // log record bytes
	int last_exec = -1;                      // ebpf_dexec_info.exec of the last launch
	int last_layout = -1;                    // its mode
};

// Whether a batch of the program writes maps (a log, or counter updates into delta areas).
struct dprog_host;
bool prog_writes_maps(const dprog_host &xl);

// Abstract value of a register (pointer provenance), computed by translate.cpp's dataflow pass
// over the state tree.  Used to specialise device handlers: packet loads at known offsets come
// from registers, stack accesses at known offsets from LDS, map lookups resolve statically.
enum av_kind : uint8_t {
	AV_UNKNOWN = 0,
	AV_CONST,       // off = the 64-bit value
	AV_CTX,         // packet start (r1 at entry) + off
	AV_STACK,       // stack top (r10 at entry) + off
	AV_MAPVAL,      // value of map #map (dp_map table index) + off, never NULL
	AV_MAPVAL_NULL, // as AV_MAPVAL, or NULL (a lookup result not yet NULL-checked)
	AV_CTXV,        // packet start + an offset not known at translation time (a cursor advanced
	                // in a loop, merged paths, advanced by an AV_SCALAR): a packet pointer, never
	                // the stack or a map value
	AV_SCALAR,      // a number not derived from any pointer: packet bytes, constants and ALU on
	                // them (a TLV length).  (Stack and map-value loads may return spilled
	                // pointers: they stay AV_UNKNOWN.)
};
struct av {
	uint8_t kind = AV_UNKNOWN;
	int16_t map = -1;
	int64_t off = 0;
	bool operator==(const av &o) const { return kind == o.kind && map == o.map && off == o.off; }
	bool operator!=(const av &o) const { return !(*this == o); }
};
struct dp_annot {
	av in[EBPF_REG_MAX]; // register state before the entry executes
	bool reached = false;
};

struct dprog_host {
	std::vector<dp_entry> entries;
	std::vector<dp_annot> annot;
	uint32_t start = 0;
	std::vector<struct ebpf_map *> maps; // referenced array maps, in dp_map table order
	bool writes_memory = false;          // any reachable ST/STX through a non-r10 base
	bool asm_needs_general = false;      // a store may touch the packet: no staged mode
	bool asm_gstage = false;             // general kernels stage packet headers (asm_program_gstage)
	bool asm_pktv = false;               // packet loads at run-time offsets (LDXPKTV), no packet stores
	bool asm_hdrlds = false;             // ... and keep them in LDS for run-time-offset loads
	                                     // (asm_program_hdrlds)
	uint32_t max_stack = 0;
	double translate_ms = 0;             // host time of translate_program
	// Map writes of a device batch (ebpf_gpu.h): the write log holds max_updates records per
	// packet — the most update / delete calls and logged stores into map values on one path
	// (0: no log).  Every written map is in exactly one of:
	std::vector<uint16_t> upd_maps;      // arrays whose records land on the device (winner words)
	std::vector<uint16_t> vstore_maps;   // ... of them, those a store into a map value may reach
	                                     // (one winner word per byte; the others: one per key)
	std::vector<uint16_t> hupd_maps;     // maps whose records replay on the host in order
	                                     // (hashtables; arrays mixing counter updates and stores)
	std::vector<uint16_t> atomic_maps;   // arrays changed only by aligned counter updates of one
	                                     // width: device atomics into the delta area (DP_MAP_ATOMIC)
	std::vector<uint8_t> atomic_width;   // ... their counter bytes (4 or 8), in that order
	uint32_t max_updates = 0;
	bool has_loops = false;              // standard semantics: backward jumps (LOOPCNT entries)
	uint32_t vstore_sites = 0;           // stores into map values / counter updates / XADD (reached)
	bool vstore_overlay = false;         // a load may read what the packet stored into a map value
	uint32_t ovl_entries = 0;            // ... overlay words per lane (2 per store on a path)
	bool write_cap = false;              // a path may log more than DP_WRITES_MAX writes (loops):
	                                     // the device counts them per packet (DP_VF_WCAP)
	bool reads_counters = false;         // loops, and a live counter-idiom register or XADD with
	                                     // BPF_FETCH on the slot graph (translate.cpp
	                                     // slot_reads_counters): the overlay holds the packet's
	                                     // view, DP_OVL_MAX words, the next faults WRITES
	int error = 0;
	std::string error_msg;
};

struct ebpf_prog {
	struct ebpf_obj eo; // must stay first
	const struct ebpf_prog_type *ept;
	uint32_t ndep_maps;
	uint32_t prog_len;
	struct ebpf_inst *prog;
	struct ebpf_map *dep_maps[EBPF_PROG_MAX_ATTACHED_MAPS];
	std::atomic<int> semantics{EBPF_SEM_REFERENCE}; // ebpf_prog_set_semantics
	// GPU backend state
	std::mutex dlock;
	std::unique_ptr<dprog_host> xlated;            // translation (device independent)
	std::vector<std::unique_ptr<dprog_device>> dev; // per device
};

// env / obj helpers (ebpf_env.c, ebpf_obj.c)
void env_acquire(struct ebpf_env *ee);
void env_release(struct ebpf_env *ee);
void obj_init(struct ebpf_env *ee, struct ebpf_obj *eo);

// translate.cpp
int translate_program(struct ebpf_prog *ep, dprog_host &out);

// gpu_runtime.cpp
void set_last_error(const std::string &msg);
// Translate the program (once; thread-safe).  0, or the translation's error.
int prog_ensure_translated(struct ebpf_prog *ep);
// the calling thread's device for the host-buffer entry points (ebpf_gpu_set_device)
int current_device();
// Copy a device batch's map writes back into the host copy (no-op unless em->dev_dirty).
// Returns 0, or EIO when the copy failed (the map then stays marked dirty).
int map_pull_device_writes(struct ebpf_map *em);
// A batch on `device` wrote the map (its writes land on `stream`, a hipStream_t).
void map_mark_device_write(struct ebpf_map *em, int device, void *stream);
void prog_release_device_state(struct ebpf_prog *ep);
void map_release_device_state(struct ebpf_map *em);

// The calling thread's current HIP device, restored when the scope ends: a C library must not
// change it (every exported entry point that selects a device holds one).
struct device_guard {
	int prev = -1;
	device_guard();
	~device_guard();
	device_guard(const device_guard &) = delete;
	device_guard &operator=(const device_guard &) = delete;
};
