// gpu_runtime.cpp — the GPU backend behind ebpf_gpu.h.
//
// Replaces the caller-side packet loop around ebpf_prog_run (hot loop #1) with
// device launches.  Per (program, device) it keeps the translated program (translate.cpp) and
// a table of the array maps the program references; per (map, device) a mirror of the map's
// storage that is refreshed before a launch whenever the host copy changed (host writes bump
// ebpf_map::version).  Launches are asynchronous on the caller's stream; nothing here ever
// executes eBPF on the CPU — without a GPU the entry points return ENODEV.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <thread>

#include "hist_ops.h"
#include "internal.h"
#include "map_writes.h"

hipError_t launch_interp_v0(const dp_launch &L, hipStream_t stream); // interp_v0.hip
// asm_runtime.cpp
hipError_t launch_interp_asm(const dp_launch &L, hipStream_t stream, int device, int mode,
			     uint32_t map_lds_bytes, void *fn, void *fn_wide, uint32_t stream_cap,
			     hipEvent_t ev_start, hipEvent_t ev_stop, unsigned long long *user_hist,
			     bool hist_overwrite);
int asm_available(int device);
uint32_t asm_max_workgroups(int device);
bool asm_lds_fits(int mode, uint32_t map_lds_bytes, uint32_t stack_stride);
bool asm_program_needs_general(const dprog_host &xl);
bool asm_program_gstage(const dprog_host &xl);
bool asm_program_hdrlds(const dprog_host &xl);
bool asm_hdrlds_fits(uint32_t map_lds_bytes, uint32_t stack_stride);
int asm_build_entries(int device, const dprog_host &xl, int mode, const std::vector<dp_map> &table,
		      dp_entry **d_out, uint32_t *stack_stride, std::string *err);
// asm_jit.cpp
int asm_jit_build(int device, const dprog_host &xl, int mode, const std::vector<dp_map> &table,
		  void **mod_out, void **fn_out, void **fn_wide_out, uint32_t *stack_stride, std::string *err);
void asm_jit_release(void *mod);
int asm_jit_emit(const dprog_host &xl, int mode, const std::vector<dp_map> &table,
		 std::vector<unsigned char> *img_out, std::vector<unsigned char> *code,
		 uint32_t *stack_stride, std::string *err);


namespace {

// Small array maps are copied into LDS by the assembly kernels at kernel start (value loads
// through a lookup result then read LDS).  Budget: kMapLdsBudget bytes per program.
uint32_t
plan_map_lds(const struct ebpf_map *em, uint32_t *used)
{
	if (em->is_hashtable())
		return ~0u;
	const uint64_t bytes = (uint64_t)em->value_size * em->max_entries;
	if (bytes == 0 || bytes % 4 != 0 || *used + bytes > kMapLdsBudget)
		return ~0u;
	const uint32_t off = kMapLdsBase + *used;
	*used += (uint32_t)((bytes + 15) & ~15ull);
	return off;
}

// The dp_map record of one map (dev_base filled in by the caller).
dp_map
map_record(const struct ebpf_map *em, uint32_t *lds_used)
{
	const map_device_layout l = map_device_layout_of(em);
	dp_map m;
	memset(&m, 0, sizeof(m));
	m.handle = (uint64_t)(uintptr_t)em;
	m.value_size = em->value_size;
	m.max_entries = l.slots;
	m.lds_off = plan_map_lds(em, lds_used);
	m.flags = l.flags;
	return m;
}

// Verdict-partial buffers of the assembly kernels (dprog.h DP_HIST_*), one per STREAM and
// device: launches on one stream run in order and each kernel leaves its buffer zero, so a
// stream reuses its own buffer with no event and no wait.  Streams are told apart by
// hipStreamGetId where the HIP runtime has it (ROCm >= 7.1: a stream handle can be recycled
// while work from its previous life is still in flight, an id is never reused), else by handle.
// At most kRowsMax streams per device own a buffer; past that the least recently used stream's
// buffer moves to the new stream, which first waits (on the GPU) for everything the old stream
// has submitted — or, if that stream no longer exists, the device drains.
struct rows_slot {
	void *p = nullptr;
	unsigned long long sid = 0; // owning stream's id
	hipStream_t stream = nullptr;
	uint64_t last = 0;          // order of the last use
	// map-writing programs (map_writes.hip): the stream's write log and winner words, grown on
	// demand (the kernels leave the log's counter and every winner word zero)
	void *log = nullptr;
	size_t log_bytes = 0;
	void *win = nullptr;
	size_t win_bytes = 0;
	// a batch's log was handed out and its apply step has not been enqueued since: its offer
	// kernel may have left winner words set, so the next batch clears them first
	bool win_pending = false;
	// the portable interpreter's spilled overlays (dp_launch.ovl_spill), grown on demand
	void *ovl = nullptr;
	size_t ovl_bytes = 0;
	// ebpf_prog_run_batch_multi_dev, when this stream leads its device: one histogram row per
	// shard on the device (any contents: every launch overwrites its row), and fork/join events
	void *mh = nullptr;
	size_t mh_bytes = 0;
	std::vector<hipEvent_t> ev;
	bool per_thread = false; // hipStreamPerThread: `stream` names a different stream per thread
};
// A batch's hold on its stream slot's winner words (upd_acquire -> upd_settled)
struct upd_owner {
	rows_slot *slot = nullptr;
	unsigned long long sid = 0;
};
std::mutex g_rows_lock;
std::vector<std::vector<rows_slot>> g_rows; // per device (capacity kRowsMax: slots never move)
uint64_t g_rows_tick = 0;
constexpr size_t kRowsMax = 64;

// The stream's slot (under g_rows_lock), created or taken over as described above.
int
slot_for(int device, hipStream_t stream, rows_slot **out)
{
	// (resolved at run time: torch bundles a HIP runtime older than the one this is built on)
	using get_id_fn = hipError_t (*)(hipStream_t, unsigned long long *);
	static const get_id_fn get_id =
	    reinterpret_cast<get_id_fn>(dlsym(RTLD_DEFAULT, "hipStreamGetId"));
	unsigned long long sid = (unsigned long long)(uintptr_t)stream;
	// hipStreamPerThread is one handle for one stream PER THREAD: two threads launching on it
	// run unordered, so each thread's stream gets its own slot (keyed by the thread)
	const bool per_thread = stream == hipStreamPerThread;
	if (per_thread)
		sid = (1ull << 63) | (unsigned long long)std::hash<std::thread::id>()(std::this_thread::get_id());
	else if (get_id && get_id(stream, &sid) != hipSuccess)
		return EIO;
	if ((int)g_rows.size() <= device)
		g_rows.resize(device + 1);
	std::vector<rows_slot> &pool = g_rows[device];
	rows_slot *lru = nullptr;
	for (rows_slot &r : pool) {
		if (r.sid == sid) {
			r.stream = stream;
			r.last = ++g_rows_tick;
			*out = &r;
			return 0;
		}
		if (!lru || r.last < lru->last)
			lru = &r;
	}
	if (pool.size() < kRowsMax) {
		pool.reserve(kRowsMax);
		rows_slot r;
		if (hipMalloc(&r.p, DP_HIST_PARTIAL_BYTES) != hipSuccess)
			return ENOMEM;
		if (hipMemsetAsync(r.p, 0, DP_HIST_PARTIAL_BYTES, stream) != hipSuccess) {
			hipFree(r.p);
			return ENOMEM;
		}
		r.sid = sid;
		r.stream = stream;
		r.per_thread = per_thread;
		r.last = ++g_rows_tick;
		pool.push_back(r);
		*out = &pool.back();
		return 0;
	}
	hipError_t e;
	if (lru->per_thread) {
		// (the handle names the calling thread's stream, not the owner's: drain the device)
		e = hipDeviceSynchronize();
	} else {
		hipEvent_t ev;
		if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
			return ENOMEM;
		e = hipEventRecord(ev, lru->stream);
		e = (e == hipSuccess) ? hipStreamWaitEvent(stream, ev, 0) : hipDeviceSynchronize();
		hipEventDestroy(ev);
	}
	if (e != hipSuccess)
		return EIO;
	lru->sid = sid;
	lru->stream = stream;
	lru->per_thread = per_thread;
	lru->last = ++g_rows_tick;
	*out = lru;
	return 0;
}

int
rows_acquire(int device, hipStream_t stream, void **out)
{
	std::lock_guard<std::mutex> g(g_rows_lock);
	rows_slot *r;
	int err = slot_for(device, stream, &r);
	if (!err)
		*out = r->p;
	return err;
}

int grow_zeroed(void **p, size_t *have, size_t need);

// The stream's spilled-overlay buffer of at least `bytes`
int
ovl_acquire(int device, hipStream_t stream, size_t bytes, uint8_t **out)
{
	std::lock_guard<std::mutex> g(g_rows_lock);
	rows_slot *r;
	int err = slot_for(device, stream, &r);
	if (!err)
		err = grow_zeroed(&r->ovl, &r->ovl_bytes, bytes);
	if (!err)
		*out = static_cast<uint8_t *>(r->ovl);
	return err;
}

// grow a zero-initialised buffer (synchronous: hipFree waits for the device, and so does the
// zeroing — hipMemset of device memory may return before it is done, and the launches that use
// the buffer run on streams that do not wait for the null stream: a 1-GiB spilled-overlay buffer
// was still being zeroed under the first kernel that wrote it)
int
grow_zeroed(void **p, size_t *have, size_t need)
{
	if (*have >= need)
		return 0;
	if (*p)
		hipFree(*p);
	*p = nullptr;
	*have = 0;
	if (hipMalloc(p, need) != hipSuccess)
		return ENOMEM;
	if (hipMemset(*p, 0, need) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
		hipFree(*p);
		*p = nullptr;
		return ENOMEM;
	}
	*have = need;
	return 0;
}

// The stream's map-write log (>= log_bytes) and winner words (>= win_bytes).
int
upd_acquire(int device, hipStream_t stream, size_t log_bytes, size_t win_bytes, uint8_t **log,
	    unsigned long long **win, upd_owner *owner)
{
	std::lock_guard<std::mutex> g(g_rows_lock);
	rows_slot *r;
	int err = slot_for(device, stream, &r);
	if (!err)
		err = grow_zeroed(&r->log, &r->log_bytes, log_bytes);
	if (!err)
		err = grow_zeroed(&r->win, &r->win_bytes, win_bytes);
	if (err)
		return err;
	if (r->win_pending) { // (the previous batch on this stream stopped before its apply step)
		if (hipMemsetAsync(r->win, 0, r->win_bytes, stream) != hipSuccess)
			return EIO;
	}
	r->win_pending = true;
	*log = static_cast<uint8_t *>(r->log);
	*win = static_cast<unsigned long long *>(r->win);
	owner->slot = r;
	owner->sid = r->sid;
	return 0;
}

// The batch's apply step is enqueued: the winner words will be zero again after it (unless the
// slot went to another stream meanwhile: that stream's flag is its own)
void
upd_settled(const upd_owner &o)
{
	std::lock_guard<std::mutex> g(g_rows_lock);
	if (o.slot && o.slot->sid == o.sid)
		o.slot->win_pending = false;
}

// The leading stream's multi-device scratch: `rows` histogram rows and `nev` events.
int
multi_acquire(int device, hipStream_t stream, uint32_t rows, size_t nev, unsigned long long **mh,
	      hipEvent_t **ev)
{
	std::lock_guard<std::mutex> g(g_rows_lock);
	rows_slot *r;
	int err = slot_for(device, stream, &r);
	if (!err)
		err = grow_zeroed(&r->mh, &r->mh_bytes, (size_t)rows * EBPF_HIST_BINS * 8);
	while (!err && r->ev.size() < nev) {
		hipEvent_t e;
		if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
			return ENOMEM;
		r->ev.push_back(e);
	}
	if (err)
		return err;
	*mh = static_cast<unsigned long long *>(r->mh);
	*ev = r->ev.data();
	return 0;
}

thread_local std::string t_err;
thread_local int t_dev = 0;
thread_local hipEvent_t t_time_ev[2] = {nullptr, nullptr}; // ebpf_gpu_time_next_launch
std::atomic<int> g_variant{0};

int
fail(int err, const std::string &msg)
{
	t_err = msg;
	return err;
}

int
hip_fail(hipError_t e, const char *what)
{
	return fail(e == hipErrorOutOfMemory ? ENOMEM : EIO,
		    std::string(what) + ": " + hipGetErrorString(e));
}

int
device_count()
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

// Which interpreter runs: 0 = the gfx950 assembly interpreter (default; an error if its code
// object cannot be loaded — never a silent fallback), 1 = the portable HIP baseline.
int
effective_variant(int)
{
	return g_variant.load();
}

int
ensure_translated(struct ebpf_prog *ep)
{
	if (ep->xlated)
		return ep->xlated->error;
	auto x = std::make_unique<dprog_host>();
	const auto t0 = std::chrono::steady_clock::now();
	int err = translate_program(ep, *x);
	x->translate_ms =
	    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	if (err && x->error == 0)
		x->error = err;
	if (!x->error) {
		x->asm_needs_general = asm_program_needs_general(*x);
		x->asm_gstage = asm_program_gstage(*x);
		x->asm_pktv = asm_program_hdrlds(*x);
		x->asm_hdrlds = x->asm_pktv && getenv("EBPF_NOHDRLDS") == nullptr;
	}
	ep->xlated = std::move(x);
	if (ep->xlated->error)
		return fail(ep->xlated->error, ep->xlated->error_msg);
	return 0;
}

int
ensure_translated_locked(struct ebpf_prog *ep)
{
	std::lock_guard<std::mutex> g(ep->dlock);
	return ensure_translated(ep);
}

bool
in_list(const std::vector<uint16_t> &v, size_t t)
{
	return std::find(v.begin(), v.end(), (uint16_t)t) != v.end();
}

int
ensure_map_mirror(struct ebpf_map *em, int device, void **dev)
{
	std::lock_guard<std::mutex> g(em->mirror_lock);
	if ((int)em->mirrors.size() <= device)
		em->mirrors.resize(device + 1);
	map_mirror &m = em->mirrors[device];
	if (m.dev == nullptr) {
		// an array: its values padded to 64 bytes, then the delta area of counter updates
		// (dprog.h dp_delta_off), both zero until the first upload
		const size_t bytes = em->is_hashtable() ? map_device_layout_of(em).bytes
							: 2 * dp_delta_off(em->value_size, em->max_entries);
		hipError_t e = hipMalloc(&m.dev, bytes);
		if (e == hipSuccess && !em->is_hashtable())
			e = hipMemset(m.dev, 0, bytes);
		if (e == hipSuccess) // (done before any stream uses it: grow_zeroed)
			e = hipDeviceSynchronize();
		if (e != hipSuccess)
			return hip_fail(e, "hipMalloc(map mirror)");
		m.version = ~0ull;
	}
	*dev = m.dev;
	return 0;
}

// Cross-stream order of one mirror's users (internal.h map_mirror; callers hold mirror_lock).
// Nothing is enqueued while every user of the mirror is on one stream.
bool
has_stream(const std::vector<void *> &v, hipStream_t s)
{
	return std::find(v.begin(), v.end(), static_cast<void *>(s)) != v.end();
}

// A launch on `s` is about to read the mirror: after the last write made on another stream.
void
mirror_read(map_mirror &m, hipStream_t s)
{
	if (m.wr_ev && !has_stream(m.synced, s)) {
		hipStreamWaitEvent(s, static_cast<hipEvent_t>(m.wr_ev), 0);
		m.synced.push_back(s);
	}
	if (!has_stream(m.readers, s))
		m.readers.push_back(s);
}

// A write of the mirror is about to be enqueued on `w`: after every launch that read it on
// another stream since the last write (an event recorded on that stream now covers all of
// them), and after the last write itself.
void
mirror_write_begin(map_mirror &m, hipStream_t w)
{
	for (void *r : m.readers) {
		if (r == static_cast<void *>(w))
			continue;
		hipEvent_t ev;
		if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
			hipStreamSynchronize(static_cast<hipStream_t>(r)); // (no event: wait on the host)
			continue;
		}
		hipEventRecord(ev, static_cast<hipStream_t>(r));
		hipStreamWaitEvent(w, ev, 0);
		hipEventDestroy(ev); // (released once it completes)
	}
	if (m.wr_ev && !has_stream(m.synced, w))
		hipStreamWaitEvent(w, static_cast<hipEvent_t>(m.wr_ev), 0);
}

// ... and it is enqueued: later users on other streams wait for it.
void
mirror_write_end(map_mirror &m, hipStream_t w)
{
	if (m.wr_ev == nullptr) {
		hipEvent_t ev;
		if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
			hipStreamSynchronize(w);
			m.synced.clear();
			m.readers.clear();
			return;
		}
		m.wr_ev = ev;
	}
	hipEventRecord(static_cast<hipEvent_t>(m.wr_ev), w);
	m.synced.assign(1, static_cast<void *>(w));
	m.readers.clear();
}

int
sync_map_mirrors(struct ebpf_prog *ep, int device, hipStream_t stream)
{
	const uint16_t cpu = map_current_cpu();
	for (struct ebpf_map *em : ep->xlated->maps) {
		const uint16_t c = em->percpu ? cpu : 0;
		// a batch wrote the map on another device, or on this one for another CPU's copy of a
		// percpu map (which is about to be replaced by this CPU's): its writes reach the host
		// copy first
		const int dd = em->dev_dirty.load(std::memory_order_acquire);
		if (dd >= 0) {
			bool pull = dd != device;
			if (!pull) {
				std::lock_guard<std::mutex> g(em->mirror_lock);
				pull = em->mirrors[device].cpu != c;
			}
			if (pull && map_pull_device_writes(em) != 0)
				return fail(EIO, "copying a device batch's map writes back failed");
		}
		std::lock_guard<std::mutex> g(em->mirror_lock);
		map_mirror &m = em->mirrors[device];
		uint64_t v = em->version.load();
		if (m.version != v || m.cpu != c) {
			hipError_t e;
			mirror_write_begin(m, stream);
			if (em->is_hashtable()) {
				// a fresh snapshot of the table; the staging copy must outlive the transfer
				auto img = std::make_shared<std::vector<uint8_t>>();
				map_device_image(em, *img, c);
				m.image = img;
				e = hipMemcpyAsync(m.dev, img->data(), img->size(), hipMemcpyHostToDevice, stream);
				if (e == hipSuccess)
					e = hipStreamSynchronize(stream);
			} else {
				// from a snapshot: the upload may wait on the stream for other streams'
				// readers (mirror_write_begin) while the host writes the map again.  The
				// previous upload from the snapshot has finished once the last write has
				// (every write of the mirror is ordered after the one before it).
				if (m.wr_ev)
					hipEventSynchronize(static_cast<hipEvent_t>(m.wr_ev));
				const size_t bytes = (size_t)em->value_size * em->max_entries;
				const uint8_t *src = map_array_image(em, c);
				auto img = std::make_shared<std::vector<uint8_t>>(src, src + bytes);
				m.image = img;
				e = hipMemcpyAsync(m.dev, img->data(), bytes, hipMemcpyHostToDevice, stream);
			}
			if (e != hipSuccess)
				return hip_fail(e, "hipMemcpyAsync(map mirror)");
			mirror_write_end(m, stream);
			m.version = v;
			m.cpu = c;
		}
		mirror_read(m, stream); // (the launch that follows reads it)
	}
	return 0;
}

// The maps' order locks, taken in address order for the span of one launch (internal.h
// ebpf_map.order_lock).
struct launch_order {
	std::vector<std::unique_lock<std::mutex>> held;
	explicit launch_order(const std::vector<struct ebpf_map *> &maps)
	{
		std::vector<struct ebpf_map *> v(maps);
		std::sort(v.begin(), v.end());
		for (struct ebpf_map *m : v)
			held.emplace_back(m->order_lock);
	}
};

int
prepare(struct ebpf_prog *ep, int device, dprog_device **out)
{
	if (device < 0 || device >= device_count())
		return fail(ENODEV, "no such GPU device");
	std::lock_guard<std::mutex> g(ep->dlock);
	int err = ensure_translated(ep);
	if (err)
		return err;
	if ((int)ep->dev.size() <= device)
		ep->dev.resize(device + 1);
	auto &dp = ep->dev[device];
	if (dp) {
		*out = dp.get();
		return 0;
	}
	hipError_t e = hipSetDevice(device);
	if (e != hipSuccess)
		return hip_fail(e, "hipSetDevice");
	auto nd = std::make_unique<dprog_device>();
	nd->device = device;
	const std::vector<dp_entry> &entries = ep->xlated->entries;
	e = hipMalloc(&nd->d_entries, entries.size() * sizeof(dp_entry));
	if (e != hipSuccess)
		return hip_fail(e, "hipMalloc(program)");
	e = hipMemcpy(nd->d_entries, entries.data(), entries.size() * sizeof(dp_entry),
		      hipMemcpyHostToDevice);
	if (e != hipSuccess)
		return hip_fail(e, "hipMemcpy(program)");
	nd->nentries = (uint32_t)entries.size();
	for (struct ebpf_map *em : ep->xlated->maps) {
		void *mdev = nullptr;
		err = ensure_map_mirror(em, device, &mdev);
		if (err)
			return err;
		dp_map m = map_record(em, &nd->map_lds_bytes);
		m.dev_base = (uint64_t)(uintptr_t)mdev;
		nd->table.push_back(m);
	}
	// arrays changed only by counter updates: device atomics into their delta areas
	for (size_t k = 0; k < ep->xlated->atomic_maps.size(); k++) {
		dp_map &m = nd->table[ep->xlated->atomic_maps[k]];
		m.flags |= DP_MAP_ATOMIC | (ep->xlated->atomic_width[k] == 8 ? DP_MAP_ATOMIC64 : 0u);
		// an LDS-resident map: its workgroup-local sums too (DP_MAP_LDSDELTA), if they fit
		const uint32_t bytes = m.value_size * m.max_entries;
		const uint32_t at = (nd->map_lds_bytes + 7) & ~7u;
		if (m.lds_off != ~0u && at + bytes <= kMapLdsBudget && kMapLdsBase + at < 0x10000u) {
			m.flags |= DP_MAP_LDSDELTA | (kMapLdsBase + at);
			nd->map_lds_bytes = at + ((bytes + 15) & ~15u);
		}
	}
	if (!nd->table.empty()) {
		e = hipMalloc(&nd->d_maps, nd->table.size() * sizeof(dp_map));
		if (e != hipSuccess)
			return hip_fail(e, "hipMalloc(map table)");
		e = hipMemcpy(nd->d_maps, nd->table.data(), nd->table.size() * sizeof(dp_map),
			      hipMemcpyHostToDevice);
		if (e != hipSuccess)
			return hip_fail(e, "hipMemcpy(map table)");
	}
	nd->nmaps = (uint32_t)nd->table.size();
	if (prog_writes_maps(*ep->xlated)) {
		// map writes: the apply step's view of the table (map_writes.h), winner words for every
		// byte of every map whose records land on the device, the log record size
		// (update records: {u64 packet, u32 map << 20, u32 key, value}; hashtable update records
		// {u64 packet, u32 map << 20, u32 op, key, value}, the key and the value each padded to
		// 8 bytes; value-store records DP_REC_VALUE_BYTES)
		const dprog_host &xl = *ep->xlated;
		std::vector<upd_map> um(nd->table.size());
		uint32_t rmax = 8;
		for (size_t t = 0; t < nd->table.size(); t++) {
			um[t].dev_base = nd->table[t].dev_base;
			um[t].value_size = nd->table[t].value_size;
			um[t].max_entries = nd->table[t].max_entries;
			um[t].win_off = nd->win_words;
			um[t].cls = UPD_NONE;
			um[t].gran = nd->table[t].value_size;
			if (in_list(xl.upd_maps, t)) {
				um[t].cls = UPD_DEVICE;
				// byte winners only where a store into a value may land; a map written only by
				// map_update_elem (whole values) needs one word per key
				if (in_list(xl.vstore_maps, t))
					um[t].gran = 1;
				nd->win_words += (uint64_t)nd->table[t].value_size * nd->table[t].max_entries /
						 um[t].gran;
				rmax = std::max(rmax, (nd->table[t].value_size + 7) & ~7u);
			}
			if (in_list(xl.hupd_maps, t)) {
				um[t].cls = UPD_HOST;
				if (nd->table[t].flags & DP_MAP_HASH)
					rmax = std::max(rmax, dp_hash_key_bytes(dp_hash_key_size(nd->table[t].flags)) +
								  ((nd->table[t].value_size + 7) & ~7u));
				else
					rmax = std::max(rmax, (nd->table[t].value_size + 7) & ~7u);
			}
			for (size_t k = 0; k < xl.atomic_maps.size(); k++)
				if (xl.atomic_maps[k] == t) {
					um[t].cls = UPD_ATOMIC;
					um[t].width = xl.atomic_width[k];
				}
		}
		if (xl.vstore_sites)
			rmax = std::max(rmax, DP_REC_VALUE_BYTES - 16);
		nd->upd_stride = 16 + rmax;
		nd->upd_host = um;
		if ((e = hipMalloc(&nd->d_upd, um.size() * sizeof(upd_map))) != hipSuccess ||
		    (e = hipMemcpy(nd->d_upd, um.data(), um.size() * sizeof(upd_map),
				   hipMemcpyHostToDevice)) != hipSuccess)
			return hip_fail(e, "map-write table");
	}
	dp = std::move(nd);
	*out = dp.get();
	return 0;
}

// Compiled program for `mode`, built on first use.  Returns 0 with dp->jit_fn[mode] set, or
// the build error (E2BIG: too large for the code area — the caller runs the interpreter).
int
jit_entries(struct ebpf_prog *ep, dprog_device *dp, int mode)
{
	std::lock_guard<std::mutex> g(ep->dlock);
	if (dp->jit_fn[mode])
		return 0;
	if (dp->jit_err[mode])
		return dp->jit_err[mode];
	std::string msg;
	const auto t0 = std::chrono::steady_clock::now();
	int err = asm_jit_build(dp->device, *ep->xlated, mode, dp->table, &dp->jit_mod[mode],
				&dp->jit_fn[mode], mode == 1 ? &dp->jit_fn_wide : nullptr,
				&dp->jit_stride[mode], &msg);
	dp->build_ms[mode] =
	    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	if (err) {
		dp->jit_err[mode] = err;
		return fail(err, msg);
	}
	return 0;
}

// Lowered assembly entries for `mode`, built on first use.
int
asm_entries(struct ebpf_prog *ep, dprog_device *dp, int mode)
{
	std::lock_guard<std::mutex> g(ep->dlock);
	if (dp->d_asm[mode])
		return 0;
	if (dp->asm_err[mode])
		return dp->asm_err[mode];
	std::string msg;
	const auto t0 = std::chrono::steady_clock::now();
	int err = asm_build_entries(dp->device, *ep->xlated, mode, dp->table, &dp->d_asm[mode],
				    &dp->asm_stride[mode], &msg);
	dp->build_ms[mode] =
	    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	if (err) {
		dp->asm_err[mode] = err;
		return fail(err, msg);
	}
	return 0;
}

// A device batch's map writes (map_writes.hip): the log its launches share, and where in the
// batch a launch starts.  The caller that passes a plan applies the log itself after the last
// launch (the host-buffer path: every chunk of one batch reads the maps as they were at its start).
struct upd_plan {
	uint8_t *log = nullptr;
	unsigned long long *win = nullptr;
	uint32_t cap = 0;
	uint64_t pkt_base = 0;
	uint32_t *faulted = nullptr; // one bit per packet of the batch (after the records)
	size_t faulted_bytes = 0;
	upd_owner owner;             // the stream slot whose winner words it uses (upd_acquire)
	// per table map, the device table its launches read (hashtables whose values the batch
	// stores into: a record names a slot, and this is the slot's key whatever is uploaded later)
	std::vector<std::shared_ptr<const std::vector<uint8_t>>> tables;
};

// Log capacity for `count` packets of a map-writing program (records, and bytes: the records,
// then the faulted-packet bitmap at *bitmap_off, *bitmap_bytes long).
int
upd_size(const struct ebpf_prog *ep, const dprog_device *dp, uint64_t count, uint32_t *cap,
	 size_t *bytes, size_t *bitmap_off, size_t *bitmap_bytes)
{
	const uint64_t rec = count * ep->xlated->max_updates;
	if (rec > UINT32_MAX)
		return fail(E2BIG, "map-writing program: more than 2^32 writes in one batch");
	*cap = (uint32_t)rec;
	*bitmap_off = (64 + rec * dp->upd_stride + 255) & ~(size_t)255;
	*bitmap_bytes = ((count + 31) / 32) * 4;
	*bytes = *bitmap_off + *bitmap_bytes;
	return 0;
}

// The log (and its bitmap) for `count` packets on `stream`.
int
upd_plan_for(struct ebpf_prog *ep, dprog_device *dp, uint64_t count, hipStream_t stream, upd_plan *P)
{
	size_t bytes, boff, bbytes;
	int err = upd_size(ep, dp, count, &P->cap, &bytes, &boff, &bbytes);
	if (!err)
		err = upd_acquire(dp->device, stream, bytes, dp->win_words * 8, &P->log, &P->win,
				  &P->owner);
	if (err)
		return fail(err, "map-write log");
	P->faulted = reinterpret_cast<uint32_t *>(P->log + boff);
	P->faulted_bytes = bbytes;
	// (the buffer is reused at other sizes: whatever lies where the bitmap now starts is stale).
	// The log's counter is zero after every apply step; it is zeroed here too, so that a batch
	// whose launch failed before its apply leaves nothing behind.  The winner words are zeroed
	// when allocated and only the apply step writes them (its first kernel offers, its second
	// re-arms every word that received an offer); a batch that stopped before its apply step was
	// enqueued leaves the stream's flag set, and upd_acquire clears them then
	hipError_t e = hipMemsetAsync(P->faulted, 0, bbytes, stream);
	if (e == hipSuccess)
		e = hipMemsetAsync(P->log, 0, 4, stream);
	return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync(map-write log)");
}

// After the batch: the logged writes land in the mirrors (packet order), and the written maps
// remember that this device's mirror is newer than their host copy.
int
upd_apply(struct ebpf_prog *ep, dprog_device *dp, const upd_plan &P, hipStream_t stream)
{
	std::vector<uint16_t> dev = ep->xlated->upd_maps;
	dev.insert(dev.end(), ep->xlated->atomic_maps.begin(), ep->xlated->atomic_maps.end());
	for (uint16_t t : dev) { // (the writes land after other streams' readers)
		struct ebpf_map *em = ep->xlated->maps[t];
		std::lock_guard<std::mutex> g(em->mirror_lock);
		mirror_write_begin(em->mirrors[dp->device], stream);
	}
	hipError_t e = launch_map_writes(P.log, P.cap, dp->upd_stride,
					 static_cast<const upd_map *>(dp->d_upd), dp->upd_host.data(),
					 (uint32_t)dp->upd_host.size(), P.win, P.faulted, stream);
	if (e != hipSuccess)
		return hip_fail(e, "map writes");
	upd_settled(P.owner);
	for (uint16_t t : dev)
		map_mark_device_write(ep->xlated->maps[t], dp->device, static_cast<void *>(stream));
	return 0;
}


// A shard's write log brought to the host (a batch whose shards ran on several devices: the
// logs are merged there, in global packet order).  Records as on the device (map_writes.h);
// `first` = the global index of the shard's packet 0.
struct host_log {
	std::vector<uint8_t> rec;
	uint32_t count = 0;
	uint32_t stride = 0;
	std::vector<uint32_t> faulted;
	uint64_t first = 0;
	int device = -1;
	std::vector<std::shared_ptr<const std::vector<uint8_t>>> tables; // upd_plan.tables
};

// Copy the plan's log (its records and faulted-packet bitmap) to the host.  Synchronous.
int
upd_fetch(const dprog_device *dp, const upd_plan &P, hipStream_t stream, uint64_t first, host_log *out)
{
	hipError_t e = hipStreamSynchronize(stream);
	uint32_t n = 0;
	if (e == hipSuccess && P.cap)
		e = hipMemcpy(&n, P.log, 4, hipMemcpyDeviceToHost);
	out->count = std::min(n, P.cap);
	out->stride = dp->upd_stride;
	out->first = first;
	out->device = dp->device;
	out->tables = P.tables;
	out->rec.resize((size_t)out->count * out->stride);
	out->faulted.resize(P.faulted_bytes / 4);
	if (e == hipSuccess && out->count)
		e = hipMemcpy(out->rec.data(), P.log + 64, out->rec.size(), hipMemcpyDeviceToHost);
	if (e == hipSuccess && P.faulted_bytes)
		e = hipMemcpy(out->faulted.data(), P.faulted, P.faulted_bytes, hipMemcpyDeviceToHost);
	// (the log's counter is re-armed by the apply step, or by the next batch's upd_plan_for)
	return e == hipSuccess ? 0 : hip_fail(e, "map-write log copy");
}

// A counter update, a store, or an update / delete call, applied to the host copy of a map.
void
apply_value(uint8_t *at, uint32_t size, bool add, const uint8_t *data)
{
	if (!add) {
		memcpy(at, data, size);
		return;
	}
	uint64_t v = 0, d = 0;
	memcpy(&v, at, size);
	memcpy(&d, data, size);
	v += d;
	memcpy(at, &v, size);
}

// The logs of a batch applied on the host, every record of a packet that did not fault (a
// counter update's record even then: ebpf_gpu.h) in (global packet, call) order:
//   - records of hupd_maps (hashtables; arrays mixing counter updates and stores), always:
//     hashtable update / delete calls replayed through the map's own update / delete (the
//     program side of ebpf_map_hashtable.c:346-431 / :475-502, percpu: the submitting CPU's
//     value), a replayed call that fails against the table as it then is (EEXIST, ENOENT, EBUSY)
//     leaving it unchanged; stores and counter updates into a hashtable value applied to the
//     element with the slot's key (the device table's image) if it still exists; array stores
//     and counter updates applied to the host copy;
//   - records of upd_maps (`arrays`: a batch whose shards ran on several devices) too, so the
//     last write of a byte wins — the device apply step's rule (map_writes.hip); every device
//     mirror of the maps changed here is then stale.
int
upd_apply_host(struct ebpf_prog *ep, const std::vector<host_log> &logs, bool arrays)
{
	const dprog_host &xl = *ep->xlated;
	struct ref {
		uint64_t order;
		const uint8_t *r;
		const host_log *h;
	};
	std::vector<ref> all;
	for (const host_log &h : logs)
		for (uint32_t i = 0; i < h.count; i++) {
			const uint8_t *r = h.rec.data() + (size_t)i * h.stride;
			uint64_t pkt;
			uint32_t em;
			memcpy(&pkt, r, 8);
			memcpy(&em, r + 8, 4);
			if ((em >> 20) >= xl.maps.size())
				return fail(EIO, "map-write log: a record names no map of the program");
			const bool add = (em & DP_REC_VALUE) && (em & DP_REC_ADD);
			if (!add && pkt / 32 < h.faulted.size() && ((h.faulted[pkt / 32] >> (pkt % 32)) & 1))
				continue; // the packet faulted: none of its writes land (counter updates do)
			if (in_list(xl.hupd_maps, em >> 20) || (arrays && in_list(xl.upd_maps, em >> 20)))
				all.push_back(ref{h.first + pkt, r, &h});
		}
	// Within a packet the records are already in call order: a lane takes its log slots one call
	// after the other and every log is gathered in slot order.  (The entry index is no order: a
	// run-time-map compare chain's copies, and merge points under standard semantics, are
	// numbered after entries that a path reaches later.)  So sort by packet only, stably.
	std::stable_sort(all.begin(), all.end(), [](const ref &a, const ref &b) { return a.order < b.order; });
	const uint16_t cpu = map_current_cpu();
	std::vector<uint16_t> host_arrays; // the array maps whose host copy changes here
	for (size_t t = 0; t < xl.maps.size(); t++)
		if (!xl.maps[t]->is_hashtable() &&
		    (in_list(xl.hupd_maps, t) || (arrays && in_list(xl.upd_maps, t))))
			host_arrays.push_back((uint16_t)t);
	for (uint16_t t : host_arrays)
		if (map_pull_device_writes(xl.maps[t]) != 0)
			return fail(EIO, "copying a device batch's map writes back failed");
	for (const ref &x : all) {
		uint32_t em, word;
		memcpy(&em, x.r + 8, 4);
		memcpy(&word, x.r + 12, 4);
		struct ebpf_map *m = xl.maps[em >> 20];
		if (em & DP_REC_VALUE) {
			const uint32_t size = em & 0xf;
			const bool add = (em & DP_REC_ADD) != 0;
			if (m->is_hashtable()) {
				// the slot's key in the table the batch's launch read (upd_plan.tables), not in
				// whatever a later upload left in the mirror
				uint32_t slot;
				memcpy(&slot, x.r + 24, 4);
				const map_device_layout l = map_device_layout_of(m);
				const uint16_t t = (uint16_t)(em >> 20);
				if (t >= x.h->tables.size() || !x.h->tables[t] || slot >= l.slots)
					continue;
				const std::vector<uint8_t> &img = *x.h->tables[t];
				const size_t so = (size_t)slot << dp_hash_stride_log2(l.flags);
				if (so + 8 + m->key_size > img.size())
					continue;
				uint8_t *v = static_cast<uint8_t *>(
				    m->emt->ops.lookup_elem(m, const_cast<uint8_t *>(img.data() + so + 8)));
				if (v != nullptr && word + size <= m->value_size) // (deleted before: nothing)
					apply_value(v + word, size, add, x.r + 16);
				continue;
			}
			if ((uint64_t)word + size > (uint64_t)m->value_size * m->max_entries)
				continue;
			uint8_t *img = const_cast<uint8_t *>(map_array_image(m, m->percpu ? cpu : 0));
			apply_value(img + word, size, add, x.r + 16);
			continue;
		}
		if (m->is_hashtable()) {
			void *key = const_cast<uint8_t *>(x.r + 16);
			void *value = const_cast<uint8_t *>(x.r + 16 + dp_hash_key_bytes(m->key_size));
			if ((word & 0xff) == 1)
				m->emt->ops.delete_elem(m, key);
			else
				m->emt->ops.update_elem(m, key, value, (word >> 8) & 0xff);
			continue;
		}
		if (word >= m->max_entries)
			continue; // (never: the routine checked it)
		uint8_t *img = const_cast<uint8_t *>(map_array_image(m, m->percpu ? cpu : 0));
		memcpy(img + (size_t)m->value_size * word, x.r + 16, m->value_size);
	}
	for (uint16_t t : host_arrays)
		xl.maps[t]->version.fetch_add(1);
	return 0;
}

// A batch sharded over several devices: the counter updates of its UPD_ATOMIC maps, summed in
// each device's delta area (one area per device, however many shards ran there), go into the
// host copy — after every shard is done — and the areas are zeroed.  The device mirrors are then
// stale.
int
delta_merge_host(struct ebpf_prog *ep, int ndev, const int *devices)
{
	const dprog_host &xl = *ep->xlated;
	if (xl.atomic_maps.empty())
		return 0;
	const uint16_t cpu = map_current_cpu();
	for (size_t k = 0; k < xl.atomic_maps.size(); k++) {
		struct ebpf_map *m = xl.maps[xl.atomic_maps[k]];
		if (map_pull_device_writes(m) != 0)
			return fail(EIO, "copying a device batch's map writes back failed");
		const uint32_t w = xl.atomic_width[k];
		const size_t bytes = (size_t)m->value_size * m->max_entries;
		uint8_t *img = const_cast<uint8_t *>(map_array_image(m, m->percpu ? cpu : 0));
		std::vector<uint8_t> d(bytes);
		for (int q = 0; q < ndev; q++) {
			bool seen = false;
			for (int q2 = 0; q2 < q; q2++)
				seen = seen || devices[q2] == devices[q];
			if (seen)
				continue;
			void *mdev = nullptr;
			{
				std::lock_guard<std::mutex> g(m->mirror_lock);
				if (devices[q] < (int)m->mirrors.size())
					mdev = m->mirrors[devices[q]].dev;
			}
			if (mdev == nullptr)
				continue;
			device_guard g2;
			hipError_t e = hipSetDevice(devices[q]);
			uint8_t *da = static_cast<uint8_t *>(mdev) + dp_delta_off(m->value_size, m->max_entries);
			if (e == hipSuccess)
				e = hipMemcpy(d.data(), da, bytes, hipMemcpyDeviceToHost);
			if (e == hipSuccess)
				e = hipMemset(da, 0, bytes);
			if (e == hipSuccess) // (done before the next launch's atomics: grow_zeroed)
				e = hipDeviceSynchronize();
			if (e != hipSuccess)
				return hip_fail(e, "counter updates copy");
			for (size_t o = 0; o < bytes; o += w)
				apply_value(img + o, w, true, d.data() + o);
		}
		m->version.fetch_add(1);
	}
	return 0;
}

// The end of a map-writing batch on one device: records of upd_maps and the counter updates of
// atomic_maps applied on the device (upd_apply), records of hupd_maps copied to the host and
// replayed there (synchronous).
int
upd_finish(struct ebpf_prog *ep, dprog_device *dp, const upd_plan &P, hipStream_t stream)
{
	const bool host = !ep->xlated->hupd_maps.empty();
	std::vector<host_log> logs(host ? 1 : 0);
	int err;
	if (host && (err = upd_fetch(dp, P, stream, 0, &logs[0])))
		return err;
	if (!ep->xlated->upd_maps.empty() || !ep->xlated->atomic_maps.empty()) {
		if ((err = upd_apply(ep, dp, P, stream)))
			return err;
	} else {
		upd_settled(P.owner); // (no offer kernel ran: the winner words are untouched)
	}
	return host ? upd_apply_host(ep, logs, false) : 0;
}

int
launch(struct ebpf_prog *ep, dprog_device *dp, const dp_launch &L0, hipStream_t stream,
       hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr, bool hist_overwrite = false,
       upd_plan *plan = nullptr)
{
	dp_launch L = L0;
	L.maps = dp->d_maps;
	L.nmaps = dp->nmaps;
	L.nentries = dp->nentries;
	L.start = ep->xlated->start;
	L.vflags = (ep->xlated->vstore_overlay ? 1u : 0u) | (ep->xlated->vstore_sites ? 2u : 0u) |
		   (std::min<uint32_t>(ep->xlated->ovl_entries, 255u) << 8) | (L0.vflags & DP_VF_EXTENTS) |
		   (ep->xlated->write_cap ? DP_VF_WCAP : 0u);
	launch_order order(ep->xlated->maps);
	int err = sync_map_mirrors(ep, dp->device, stream);
	if (err)
		return err;
	hipError_t e;
	upd_plan own;
	if (prog_writes_maps(*ep->xlated)) {
		if (plan == nullptr && (err = upd_plan_for(ep, dp, L0.count, stream, &own)))
			return err; // (this launch is the whole batch: its own log, applied below)
		upd_plan &P = plan ? *plan : own;
		if (ep->xlated->vstore_sites) // (the slot -> key map of the tables this launch reads)
			for (uint16_t t : ep->xlated->hupd_maps) {
				struct ebpf_map *em = ep->xlated->maps[t];
				if (!em->is_hashtable())
					continue;
				std::lock_guard<std::mutex> g(em->mirror_lock);
				if (P.tables.size() <= t)
					P.tables.resize(t + 1);
				P.tables[t] = em->mirrors[dp->device].image;
			}
		L.upd_log = P.log;
		L.upd_cap = P.cap;
		L.upd_stride = dp->upd_stride;
		L.pkt_base = P.pkt_base;
		L.upd_faulted = P.faulted;
	}
	const int variant = effective_variant(dp->device);
	const int mode = (L.offsets == nullptr && L.stride == 64 && !ep->xlated->asm_needs_general) ? 1 : 0;
	// the assembly kernels keep 256 lanes' stack slices in LDS: a program whose slice (stack
	// depth, loop count, value-store overlay) leaves them no room runs on the portable HIP
	// interpreter instead (its stack is per-thread memory)
	bool asm_fits = true;
	if (variant == 0 || variant == 2) {
		const bool compile = variant == 0;
		uint32_t stride;
		if (compile && (err = jit_entries(ep, dp, mode)) == 0) {
			stride = dp->jit_stride[mode];
		} else {
			if (compile && err != E2BIG)
				return err;
			if ((err = asm_entries(ep, dp, mode)))
				return err;
			stride = dp->asm_stride[mode];
		}
		asm_fits = asm_lds_fits(mode, dp->map_lds_bytes, stride);
	}
	// an overlay larger than the lanes keep on chip: the portable interpreter, spilled
	const bool spill = ep->xlated->vstore_overlay && ep->xlated->ovl_entries > DP_OVL_MAX;
	if (spill)
		asm_fits = false;
	if ((variant == 0 || variant == 2) && asm_fits) {
		// variant 0: the compiled program; a program too large for the code area runs on the
		// assembly interpreter instead (still the device path).  Programs with loops compile
		// too: the code generator keeps facts and liveness only across single-predecessor
		// edges, and a loop head (an entry point, >= 2 predecessors) starts from nothing known
		void *fn = nullptr;
		const bool compile = variant == 0;
		if (compile && dp->jit_fn[mode]) {
			L.prog = nullptr;
			L.stack_stride = dp->jit_stride[mode];
			fn = dp->jit_fn[mode];
		} else {
			L.prog = dp->d_asm[mode];
			L.stack_stride = dp->asm_stride[mode];
		}
		dp->last_exec = fn ? EBPF_EXEC_COMPILED : EBPF_EXEC_INTERPRETER;
		dp->last_layout = mode;
		// the staged kernels' keep mode (compiled and interpreted programs): a program that
		// loads its packet at run-time offsets reads them from the wave's LDS packet buffer
		// (gen_interp.py h_ldx_pktv), so the next group's DMA waits for the group's end
		if (mode == 1 && ep->xlated->asm_pktv && getenv("EBPF_NOKEEP") == nullptr)
			L.vflags |= DP_VF_KEEP;
		// general kernels: header staging (bit 31), and the headers kept in LDS too (bit 30;
		// when the 16 KB of packet buffers cost no resident workgroup: the VGPRs allow 6 per CU)
		const bool hdrlds = ep->xlated->asm_hdrlds && asm_hdrlds_fits(dp->map_lds_bytes, L.stack_stride);
		L.lds_pkt_base = mode != 0 ? 0 : hdrlds ? 0xc0000000u
						 : ep->xlated->asm_gstage ? 0x80000000u : 0;
		unsigned long long *user_hist = L.hist;
		if (L.hist) {
			void *part = nullptr;
			if ((err = rows_acquire(dp->device, stream, &part)))
				return fail(err, "no verdict-partial buffer");
			// faults (bin 256) count into replica 0 of the partials; the kernel's last
			// workgroup moves everything into the caller's histogram (user_hist)
			L.hist_rows = static_cast<uint32_t *>(part);
			L.hist = static_cast<unsigned long long *>(part);
		}
		// workgroups per CU on the staged kernels (asm_runtime.cpp, occupancy): compiled programs
		// that only stream packets run 4 (and are the ones write phasing serves); one that probes
		// hashtables runs 5 (C4H 1.49 -> 1.46 ms against 6, 1.53 at 4, profiles/r05/c4h_occ/).
		// The interpreter (fn == NULL) is bound by its scalar dispatch and wants every wave: C4
		// 1.86 -> 1.42 ms at 6 instead of 4 (profiles/r02/v2occ).  A compiled program with loops
		// runs 5, as a probing one does (C3L 0.2238 -> 0.2160 ms against 6, 0.241 at 4, three
		// runs each, profiles/r06/c3l_occ/; round 4's code had gained from 4 to 6)
		bool hash = false;
		for (const dp_map &m : dp->table)
			hash = hash || (m.flags & DP_MAP_HASH) != 0;
		uint32_t wg_cap = 0;
		if (mode == 1 && fn)
			wg_cap = (hash || ep->xlated->has_loops) ? kProbeWorkgroups : kStreamWorkgroups;
		e = launch_interp_asm(L, stream, dp->device, mode, dp->map_lds_bytes, fn,
				      fn ? dp->jit_fn_wide : nullptr, wg_cap, ev_start, ev_stop, user_hist,
				      hist_overwrite);
	} else {
		L.prog = dp->d_entries;
		dp->last_exec = EBPF_EXEC_HIP;
		dp->last_layout = 0;
		if (hist_overwrite && L.hist &&
		    (e = hipMemsetAsync(L.hist, 0, EBPF_HIST_BINS * sizeof(uint64_t), stream)) !=
			hipSuccess)
			return hip_fail(e, "hipMemsetAsync(hist)");
		if (spill) { // (chunks whose overlays fit 1 GiB)
			const uint64_t per = 16ull * ep->xlated->ovl_entries;
			uint64_t chunk = std::max<uint64_t>(256, ((1ull << 30) / per) & ~255ull);
			chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(L.count, 1));
			uint8_t *buf = nullptr;
			if ((err = ovl_acquire(dp->device, stream, chunk * per, &buf)))
				return fail(err, "spilled overlay");
			L.ovl_cap = ep->xlated->ovl_entries;
			L.ovl_chunk = (uint32_t)chunk;
			L.ovl_spill = buf;
		}
		if (ev_start)
			hipEventRecord(ev_start, stream);
		e = launch_interp_v0(L, stream); // (one kernel per chunk: the histogram is added in-kernel)
		if (ev_stop)
			hipEventRecord(ev_stop, stream);
	}
	if (e != hipSuccess)
		return hip_fail(e, "kernel launch");
	if (prog_writes_maps(*ep->xlated) && plan == nullptr)
		return upd_finish(ep, dp, own, stream);
	return 0;
}

int
validate_batch(const struct ebpf_pkt_batch *b, uint32_t allowed_flags = 0)
{
	if (b == nullptr || (b->data == nullptr && b->count != 0))
		return fail(EINVAL, "batch or batch->data is NULL");
	if (b->flags & ~(allowed_flags | EBPF_BATCH_EXTENTS))
		return fail(EINVAL, "batch->flags: unknown bits");
	if ((b->flags & EBPF_BATCH_EXTENTS) && b->offsets == nullptr && b->count != 0)
		return fail(EINVAL, "extents batch without offsets");
	if (b->offsets == nullptr && b->stride == 0 && b->count != 0)
		return fail(EINVAL, "fixed-stride batch with stride 0");
	return 0;
}

// Staging buffers of the host-buffer entry points: per device, a pool of sets (two streams, two
// chunk buffers, a histogram), one set per call in flight on that device, reused across calls.
struct staging {
	int device = -1;
	hipStream_t stream[2] = {nullptr, nullptr};
	hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
	hipEvent_t ev_plan = nullptr; // map-writing programs: the log's set-up on stream 0 (stream 1 waits)
	void *d_data[2] = {nullptr, nullptr};
	size_t data_cap[2] = {0, 0};
	void *d_small[2] = {nullptr, nullptr}; // ret | faults | offsets, per chunk
	size_t small_cap[2] = {0, 0};
	unsigned long long *d_hist = nullptr;
};
std::mutex g_stage_lock;
std::vector<std::vector<staging *>> g_stage_free; // per device

int
staging_acquire(int device, staging **out)
{
	{
		std::lock_guard<std::mutex> g(g_stage_lock);
		if ((int)g_stage_free.size() <= device)
			g_stage_free.resize(device + 1);
		if (!g_stage_free[device].empty()) {
			*out = g_stage_free[device].back();
			g_stage_free[device].pop_back();
			return 0;
		}
	}
	auto S = std::make_unique<staging>();
	S->device = device;
	hipError_t e = hipSetDevice(device);
	for (int i = 0; i < 2 && e == hipSuccess; i++)
		e = hipStreamCreateWithFlags(&S->stream[i], hipStreamNonBlocking);
	for (int i = 0; i < 4 && e == hipSuccess; i++)
		e = hipEventCreate(&S->ev[i]);
	if (e == hipSuccess)
		e = hipEventCreateWithFlags(&S->ev_plan, hipEventDisableTiming);
	if (e == hipSuccess)
		e = hipMalloc(&S->d_hist, EBPF_HIST_BINS * sizeof(unsigned long long));
	if (e != hipSuccess)
		return hip_fail(e, "staging set-up"); // (a set that failed half way is not pooled)
	*out = S.release();
	return 0;
}

void
staging_release(staging *S)
{
	std::lock_guard<std::mutex> g(g_stage_lock);
	g_stage_free[S->device].push_back(S);
}

int
stage_alloc(void **p, size_t *cap, size_t need)
{
	if (*cap >= need)
		return 0;
	if (*p)
		hipFree(*p);
	*p = nullptr;
	*cap = 0;
	hipError_t e = hipMalloc(p, need);
	if (e != hipSuccess)
		return hip_fail(e, "hipMalloc(staging)");
	*cap = need;
	return 0;
}

} // namespace

int
prog_ensure_translated(struct ebpf_prog *ep)
{
	return ensure_translated_locked(ep);
}

void
set_last_error(const std::string &msg)
{
	t_err = msg;
}

device_guard::device_guard()
{
	if (hipGetDevice(&prev) != hipSuccess)
		prev = -1;
}

device_guard::~device_guard()
{
	int now = -1;
	if (prev >= 0 && (hipGetDevice(&now) != hipSuccess || now != prev))
		hipSetDevice(prev);
}

void
prog_release_device_state(struct ebpf_prog *ep)
{
	device_guard dg;
	for (auto &dp : ep->dev) {
		if (!dp)
			continue;
		if (hipSetDevice(dp->device) == hipSuccess) {
			if (dp->d_entries)
				hipFree(dp->d_entries);
			if (dp->d_maps)
				hipFree(dp->d_maps);
			if (dp->d_upd)
				hipFree(dp->d_upd);
			for (auto *a : dp->d_asm)
				if (a)
					hipFree(a);
			for (auto *m : dp->jit_mod)
				asm_jit_release(m);
		}
	}
	ep->dev.clear();
}

void
map_release_device_state(struct ebpf_map *em)
{
	device_guard dg;
	if (em->wb_event) {
		hipEventSynchronize(static_cast<hipEvent_t>(em->wb_event));
		hipEventDestroy(static_cast<hipEvent_t>(em->wb_event));
		em->wb_event = nullptr;
	}
	for (size_t d = 0; d < em->mirrors.size(); d++) {
		if (hipSetDevice((int)d) != hipSuccess)
			continue;
		if (em->mirrors[d].wr_ev)
			hipEventDestroy(static_cast<hipEvent_t>(em->mirrors[d].wr_ev));
		if (em->mirrors[d].dev)
			hipFree(em->mirrors[d].dev);
	}
	em->mirrors.clear();
}

// The device's mirror now holds the batch's writes: it is the newest copy.  The version moves on
// so that other devices re-upload (after pulling these writes, sync_map_mirrors) while this
// device keeps its mirror.
void
map_mark_device_write(struct ebpf_map *em, int device, void *stream)
{
	std::lock_guard<std::mutex> g(em->mirror_lock);
	if (em->wb_event == nullptr) {
		hipEvent_t ev;
		if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
			return;
		em->wb_event = ev;
	} else if (em->dev_dirty.load() == device) {
		// another stream may have written the mirror and not finished: the event recorded below
		// must cover that apply too (the pull waits for every writer, not only the last)
		hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(em->wb_event), 0);
	}
	hipEventRecord(static_cast<hipEvent_t>(em->wb_event), static_cast<hipStream_t>(stream));
	const uint64_t v = em->version.fetch_add(1) + 1;
	if ((int)em->mirrors.size() > device) {
		em->mirrors[device].version = v;
		mirror_write_end(em->mirrors[device], static_cast<hipStream_t>(stream));
	}
	em->dev_dirty.store(device, std::memory_order_release);
}

int
map_pull_device_writes(struct ebpf_map *em)
{
	if (em->dev_dirty.load(std::memory_order_acquire) < 0)
		return 0;
	std::lock_guard<std::mutex> g(em->mirror_lock);
	const int d = em->dev_dirty.load(std::memory_order_acquire);
	if (d < 0 || d >= (int)em->mirrors.size())
		return 0;
	const map_mirror &m = em->mirrors[d];
	hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(em->wb_event));
	// array / percpu array: the mirror is the (submitting CPU's) value array
	uint8_t *dst = const_cast<uint8_t *>(map_array_image(em, em->percpu ? m.cpu : 0));
	if (e == hipSuccess && dst && m.dev)
		e = hipMemcpy(dst, m.dev, (size_t)em->value_size * em->max_entries, hipMemcpyDeviceToHost);
	if (e != hipSuccess) {
		set_last_error(std::string("map write-back: ") + hipGetErrorString(e));
		return EIO; // (still dirty: a later call tries again)
	}
	em->dev_dirty.store(-1, std::memory_order_release);
	return 0;
}

EBPF_EXPORT int
ebpf_gpu_device_count(void)
{
	return device_count();
}

EBPF_EXPORT int
ebpf_dev_init(int ndev)
{
	const int n = device_count();
	if (n <= 0)
		return fail(ENODEV, "no GPU visible");
	if (ndev <= 0)
		ndev = n;
	if (ndev > n)
		return fail(ENODEV, "ebpf_dev_init: more devices asked for than visible");
	device_guard dg;
	for (int d = 0; d < ndev; d++)
		if (!asm_available(d))
			return fail(EIO, "device " + std::to_string(d) + ": the kernels' code object did not load");
	return 0;
}

EBPF_EXPORT int
ebpf_gpu_set_device(int device)
{
	if (device < 0 || device >= device_count())
		return fail(ENODEV, "no such GPU device");
	t_dev = device;
	return 0;
}

int
current_device()
{
	return t_dev;
}

EBPF_EXPORT int
ebpf_gpu_time_next_launch(void *start_event, void *stop_event)
{
	if ((start_event == nullptr) != (stop_event == nullptr))
		return fail(EINVAL, "start_event and stop_event must both be set or both be NULL");
	t_time_ev[0] = static_cast<hipEvent_t>(start_event);
	t_time_ev[1] = static_cast<hipEvent_t>(stop_event);
	return 0;
}

EBPF_EXPORT int
ebpf_gpu_set_variant(int variant)
{
	if (variant < 0 || variant > 2)
		return fail(EINVAL, "variant must be 0 (compiled), 1 (portable HIP) or 2 (interpreter)");
	g_variant.store(variant);
	return 0;
}

EBPF_EXPORT const char *
ebpf_gpu_last_error(void)
{
	return t_err.c_str();
}

EBPF_EXPORT int
ebpf_prog_prepare_device(struct ebpf_prog *ep, int device)
{
	if (ep == nullptr)
		return fail(EINVAL, "prog is NULL");
	device_guard dg;
	dprog_device *dp;
	return prepare(ep, device, &dp);
}

EBPF_EXPORT int
ebpf_prog_set_semantics(struct ebpf_prog *ep, int semantics)
{
	if (ep == nullptr || (semantics != EBPF_SEM_REFERENCE && semantics != EBPF_SEM_STANDARD))
		return fail(EINVAL, "bad argument");
	std::lock_guard<std::mutex> g(ep->dlock);
	if (ep->xlated && ep->semantics.load() != semantics)
		return fail(EBUSY, "the program was already translated with other semantics");
	ep->semantics.store(semantics);
	return 0;
}

EBPF_EXPORT int
ebpf_prog_device_info(struct ebpf_prog *ep, struct ebpf_dprog_info *info)
{
	if (ep == nullptr || info == nullptr)
		return fail(EINVAL, "NULL argument");
	std::lock_guard<std::mutex> g(ep->dlock);
	int err = ensure_translated(ep);
	if (err)
		return err;
	info->nslots = ep->prog_len / 8;
	info->nentries = (uint32_t)ep->xlated->entries.size();
	info->nmaps = (uint32_t)ep->xlated->maps.size();
	info->max_stack = ep->xlated->max_stack;
	return 0;
}

EBPF_EXPORT int
ebpf_prog_device_exec(struct ebpf_prog *ep, int device, struct ebpf_dexec_info *info)
{
	if (ep == nullptr || info == nullptr)
		return fail(EINVAL, "NULL argument");
	std::lock_guard<std::mutex> g(ep->dlock);
	memset(info, 0, sizeof(*info));
	info->exec = -1;
	info->layout = -1;
	if (ep->xlated)
		info->translate_ms = ep->xlated->translate_ms;
	if (device < 0 || device >= (int)ep->dev.size() || !ep->dev[device])
		return 0;
	const dprog_device &dp = *ep->dev[device];
	info->exec = dp.last_exec;
	info->layout = dp.last_layout;
	if (dp.last_layout >= 0 && dp.last_exec != EBPF_EXEC_HIP)
		info->build_ms = dp.build_ms[dp.last_layout];
	return 0;
}

EBPF_EXPORT int
ebpf_prog_device_code(struct ebpf_prog *ep, int layout, void *buf, size_t *len)
{
	if (ep == nullptr || len == nullptr || layout < 0 || layout > 1)
		return fail(EINVAL, "bad argument");
	std::lock_guard<std::mutex> g(ep->dlock);
	int err = ensure_translated(ep);
	if (err)
		return err;
	// host-side map table: device bases are unknown without a device (0 here; the real table
	// differs only in those immediates)
	std::vector<dp_map> table;
	uint32_t used = 0;
	for (struct ebpf_map *em : ep->xlated->maps)
		table.push_back(map_record(em, &used));
	std::vector<unsigned char> img, code;
	uint32_t stride = 0;
	std::string msg;
	err = asm_jit_emit(*ep->xlated, layout, table, &img, &code, &stride, &msg);
	if (err)
		return fail(err, msg);
	const size_t cap = *len;
	*len = code.size();
	if (buf == nullptr || cap < code.size())
		return buf == nullptr ? 0 : fail(ENOSPC, "buffer too small");
	memcpy(buf, code.data(), code.size());
	return 0;
}

namespace {

// One device-resident batch (ebpf_prog_run_batch_dev); with `keep` (a shard of a multi-device
// batch of a map-writing program) its writes stay in their log, described by *keep (keep->cap
// stays 0 for a program without writes), for the host-side merge instead of being applied on
// the device.
int
batch_dev(struct ebpf_prog *ep, int device, const struct ebpf_pkt_batch *batch, uint64_t *ret_dev,
	  uint8_t *faults_dev, uint64_t *hist_dev, void *stream, upd_plan *keep)
{
	// the measurement hook is consumed by this call, whatever it returns
	hipEvent_t ev_start = t_time_ev[0], ev_stop = t_time_ev[1];
	t_time_ev[0] = t_time_ev[1] = nullptr;
	if (ep == nullptr || ret_dev == nullptr)
		return fail(EINVAL, "prog or ret is NULL");
	int err = validate_batch(batch, EBPF_BATCH_HIST_OVERWRITE);
	if (err)
		return err;
	const bool overwrite = (batch->flags & EBPF_BATCH_HIST_OVERWRITE) != 0;
	device_guard dg;
	dprog_device *dp;
	err = prepare(ep, device, &dp);
	if (err)
		return err;
	if (batch->count == 0) {
		if (ev_start) { // no kernel: an empty interval
			hipEventRecord(ev_start, static_cast<hipStream_t>(stream));
			hipEventRecord(ev_stop, static_cast<hipStream_t>(stream));
		}
		if (overwrite && hist_dev) {
			hipError_t e = hipMemsetAsync(hist_dev, 0, EBPF_HIST_BINS * sizeof(uint64_t),
						      static_cast<hipStream_t>(stream));
			if (e != hipSuccess)
				return hip_fail(e, "hipMemsetAsync(hist)");
		}
		return 0;
	}
	hipError_t e = hipSetDevice(device);
	if (e != hipSuccess)
		return hip_fail(e, "hipSetDevice");
	dp_launch L;
	memset(&L, 0, sizeof(L));
	L.data = (uint8_t *)batch->data;
	L.offsets = batch->offsets;
	L.off_base = 0;
	L.vflags = (batch->flags & EBPF_BATCH_EXTENTS) ? DP_VF_EXTENTS : 0;
	L.ret = ret_dev;
	L.faults = faults_dev;
	L.hist = reinterpret_cast<unsigned long long *>(hist_dev);
	L.count = batch->count;
	L.stride = batch->stride;
	hipStream_t st = static_cast<hipStream_t>(stream);
	if (keep && prog_writes_maps(*ep->xlated)) {
		if ((err = sync_map_mirrors(ep, device, st)) ||
		    (err = upd_plan_for(ep, dp, batch->count, st, keep)))
			return err;
		return launch(ep, dp, L, st, ev_start, ev_stop, overwrite, keep);
	}
	return launch(ep, dp, L, st, ev_start, ev_stop, overwrite);
}

} // namespace

EBPF_EXPORT int
ebpf_prog_run_batch_dev(struct ebpf_prog *ep, int device, const struct ebpf_pkt_batch *batch,
			uint64_t *ret_dev, uint8_t *faults_dev, uint64_t *hist_dev, void *stream)
{
	return batch_dev(ep, device, batch, ret_dev, faults_dev, hist_dev, stream, nullptr);
}

namespace {

// Packets [lo, hi) of a host-buffer batch on `device` with staging set S: chunked,
// double-buffered H2D -> kernel -> D2H on S's two streams.  Results go to ret[lo..hi) (and
// faults[lo..hi)); the shard's verdict histogram is left in S.d_hist (zeroed first) and the
// interpreter kernels' device time is added to *kernel_ms.  Synchronous.
int
run_host_shard(struct ebpf_prog *ep, dprog_device *dp, staging &S,
	       const struct ebpf_pkt_batch *batch, uint64_t lo, uint64_t hi, uint64_t *ret,
	       uint8_t *faults, double *kernel_ms, host_log *log_out = nullptr)
{
	hipError_t e = hipSetDevice(S.device);
	if (e != hipSuccess)
		return hip_fail(e, "hipSetDevice");
	const bool copy_back = ep->xlated->writes_memory;
	// Chunked, double-buffered: chunk k's H2D overlaps chunk k-1's kernel and D2H.
	const uint64_t chunk = batch->offsets ? (1ull << 20) : (1ull << 22);
	const bool ext = (batch->flags & EBPF_BATCH_EXTENTS) != 0;
	if ((e = hipMemsetAsync(S.d_hist, 0, EBPF_HIST_BINS * sizeof(unsigned long long),
				S.stream[0])) != hipSuccess ||
	    (e = hipStreamSynchronize(S.stream[0])) != hipSuccess)
		return hip_fail(e, "hipMemsetAsync(hist)");
	int err;
	// a map-writing program: one log for the whole shard, applied after its last chunk (every
	// chunk reads the maps as they were when the batch started)
	upd_plan plan;
	if (prog_writes_maps(*ep->xlated)) {
		// the log is set up on stream 0; the odd chunks run on stream 1 and log into it too
		if ((err = upd_plan_for(ep, dp, hi - lo, S.stream[0], &plan)))
			return err;
		if ((e = hipEventRecord(S.ev_plan, S.stream[0])) != hipSuccess ||
		    (e = hipStreamWaitEvent(S.stream[1], S.ev_plan, 0)) != hipSuccess)
			return hip_fail(e, "map-write log set-up");
	}
	bool timed[2] = {false, false};
	// on any error: drain both streams (buffers stay valid for the copies in flight)
	auto drain = [&](int rc) {
		hipStreamSynchronize(S.stream[0]);
		hipStreamSynchronize(S.stream[1]);
		return rc;
	};
	auto collect = [&](int b) -> hipError_t {
		if (!timed[b])
			return hipSuccess;
		float ms = 0;
		hipError_t te = hipEventElapsedTime(&ms, S.ev[2 * b], S.ev[2 * b + 1]);
		*kernel_ms += ms;
		timed[b] = false;
		return te;
	};
	for (uint64_t c0 = lo, k = 0; c0 < hi; c0 += chunk, k++) {
		const int b = (int)(k & 1);
		hipStream_t st = S.stream[b];
		const uint64_t cn = (hi - c0 < chunk) ? hi - c0 : chunk;
		uint64_t byte0, byte1;
		if (ext) { // the bytes the chunk's packets span (in any order, gaps included)
			byte0 = UINT64_MAX;
			byte1 = 0;
			for (uint64_t i = c0; i < c0 + cn; i++) {
				byte0 = std::min(byte0, batch->offsets[2 * i]);
				byte1 = std::max(byte1, batch->offsets[2 * i + 1]);
			}
			if (byte1 < byte0)
				byte0 = byte1;
		} else if (batch->offsets) {
			byte0 = batch->offsets[c0];
			byte1 = batch->offsets[c0 + cn];
		} else {
			byte0 = c0 * batch->stride;
			byte1 = (c0 + cn) * batch->stride;
		}
		// buffers of chunk k-2 are free again
		if ((e = hipStreamSynchronize(st)) != hipSuccess || (e = collect(b)) != hipSuccess)
			return drain(hip_fail(e, "batch chunk"));
		if ((err = stage_alloc(&S.d_data[b], &S.data_cap[b], byte1 - byte0 + 16)))
			return drain(err);
		const uint64_t noffs = ext ? 2 * cn : cn + 1;
		const size_t small = cn * 9 + (batch->offsets ? noffs * 8 : 0) + 64;
		if ((err = stage_alloc(&S.d_small[b], &S.small_cap[b], small)))
			return drain(err);
		uint8_t *sm = static_cast<uint8_t *>(S.d_small[b]);
		uint64_t *d_ret = reinterpret_cast<uint64_t *>(sm);
		uint64_t *d_offs = batch->offsets ? reinterpret_cast<uint64_t *>(sm + cn * 8) : nullptr;
		uint8_t *d_faults = sm + cn * 8 + (batch->offsets ? noffs * 8 : 0);
		const uint8_t *src = static_cast<const uint8_t *>(batch->data) + byte0;
		if ((e = hipMemcpyAsync(S.d_data[b], src, byte1 - byte0, hipMemcpyHostToDevice, st)) !=
		    hipSuccess)
			return drain(hip_fail(e, "hipMemcpyAsync(packets H2D)"));
		if (d_offs && (e = hipMemcpyAsync(d_offs, batch->offsets + (ext ? 2 * c0 : c0), noffs * 8,
						  hipMemcpyHostToDevice, st)) != hipSuccess)
			return drain(hip_fail(e, "hipMemcpyAsync(offsets H2D)"));
		dp_launch L;
		memset(&L, 0, sizeof(L));
		L.data = static_cast<uint8_t *>(S.d_data[b]);
		L.offsets = d_offs;
		L.off_base = byte0;
		L.vflags = ext ? DP_VF_EXTENTS : 0;
		L.ret = d_ret;
		L.faults = d_faults;
		L.hist = S.d_hist;
		L.count = cn;
		L.stride = batch->stride;
		if ((e = hipEventRecord(S.ev[2 * b], st)) != hipSuccess)
			return drain(hip_fail(e, "hipEventRecord"));
		plan.pkt_base = c0 - lo; // (the shard's own packet index: its bitmap starts at lo)
		if ((err = launch(ep, dp, L, st, nullptr, nullptr, false, &plan)))
			return drain(err);
		if ((e = hipEventRecord(S.ev[2 * b + 1], st)) != hipSuccess)
			return drain(hip_fail(e, "hipEventRecord"));
		timed[b] = true;
		if ((e = hipMemcpyAsync(ret + c0, d_ret, cn * 8, hipMemcpyDeviceToHost, st)) != hipSuccess)
			return drain(hip_fail(e, "hipMemcpyAsync(results D2H)"));
		if (faults && (e = hipMemcpyAsync(faults + c0, d_faults, cn, hipMemcpyDeviceToHost, st)) !=
				  hipSuccess)
			return drain(hip_fail(e, "hipMemcpyAsync(faults D2H)"));
		if (copy_back && (e = hipMemcpyAsync(const_cast<uint8_t *>(src), S.d_data[b],
						     byte1 - byte0, hipMemcpyDeviceToHost, st)) !=
				     hipSuccess)
			return drain(hip_fail(e, "hipMemcpyAsync(packets D2H)"));
	}
	for (int i = 0; i < 2; i++) {
		if ((e = hipStreamSynchronize(S.stream[i])) != hipSuccess || (e = collect(i)) != hipSuccess)
			return drain(hip_fail(e, "batch"));
	}
	if (prog_writes_maps(*ep->xlated) && hi > lo) {
		if (log_out) { // (several shards: the caller merges the logs; no offer kernel runs)
			if ((err = upd_fetch(dp, plan, S.stream[0], lo, log_out)) == 0)
				upd_settled(plan.owner);
			return err;
		}
		if ((err = upd_finish(ep, dp, plan, S.stream[0])))
			return drain(err);
		if ((e = hipStreamSynchronize(S.stream[0])) != hipSuccess)
			return hip_fail(e, "map writes");
	}
	return 0;
}

int
fill_stats(struct ebpf_batch_stats *stats, uint64_t n, const unsigned long long *h, double kernel_ms,
	   std::chrono::steady_clock::time_point t0)
{
	stats->packets = n;
	stats->faulted = h[256];
	for (int i = 0; i < EBPF_HIST_BINS; i++)
		stats->hist[i] = h[i];
	stats->kernel_ms = kernel_ms;
	stats->total_ms =
	    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	return 0;
}

int
check_devices(int ndev, const int *devices, bool distinct)
{
	if (ndev < 1 || devices == nullptr)
		return fail(EINVAL, "ndev < 1 or devices is NULL");
	const int have = device_count();
	for (int d = 0; d < ndev; d++) {
		if (devices[d] < 0 || devices[d] >= have)
			return fail(ENODEV, "no such GPU device");
		for (int d2 = 0; distinct && d2 < d; d2++)
			if (devices[d2] == devices[d])
				return fail(EINVAL, "a device appears twice in the list");
	}
	return 0;
}

} // namespace (host-buffer helpers)

int rccl_hist_allreduce(int ndev, const int *devices, uint64_t *const *hist, hipStream_t *streams,
			std::string *msg);

namespace {
std::mutex g_multi_lock; // ebpf_prog_run_batch_multi_dev's enqueue (its scratch is per stream)
}

EBPF_EXPORT int
ebpf_prog_run_batch(struct ebpf_prog *ep, const struct ebpf_pkt_batch *batch, uint64_t *ret,
		    uint8_t *faults, struct ebpf_batch_stats *stats)
{
	if (ep == nullptr || ret == nullptr)
		return fail(EINVAL, "prog or ret is NULL");
	int err = validate_batch(batch);
	if (err)
		return err;
	auto t0 = std::chrono::steady_clock::now();
	const int device = t_dev;
	device_guard dg;
	dprog_device *dp;
	if ((err = prepare(ep, device, &dp)))
		return err;
	staging *S;
	if ((err = staging_acquire(device, &S)))
		return err;
	double kernel_ms = 0;
	err = run_host_shard(ep, dp, *S, batch, 0, batch->count, ret, faults, &kernel_ms);
	unsigned long long h[EBPF_HIST_BINS];
	hipError_t e;
	if (!err && stats &&
	    (e = hipMemcpy(h, S->d_hist, sizeof(h), hipMemcpyDeviceToHost)) != hipSuccess)
		err = hip_fail(e, "hipMemcpy(hist)");
	staging_release(S);
	if (!err && stats)
		fill_stats(stats, batch->count, h, kernel_ms, t0);
	return err;
}

EBPF_EXPORT int
ebpf_prog_run_batch_multi(struct ebpf_prog *ep, int ndev, const int *devices,
			  const struct ebpf_pkt_batch *batch, uint64_t *ret, uint8_t *faults,
			  struct ebpf_batch_stats *stats)
{
	if (ep == nullptr || ret == nullptr)
		return fail(EINVAL, "prog or ret is NULL");
	int err = validate_batch(batch);
	if (err || (err = check_devices(ndev, devices, false)))
		return err;
	auto t0 = std::chrono::steady_clock::now();
	device_guard dg;
	// a map-writing program: each shard's writes stay in its log, merged and applied on the host
	// in global packet order after every shard is done
	const bool merge = ndev > 1 && ensure_translated_locked(ep) == 0 && prog_writes_maps(*ep->xlated);
	std::vector<host_log> logs(merge ? ndev : 0);
	std::vector<dprog_device *> dps(ndev);
	std::vector<staging *> S(ndev, nullptr);
	for (int d = 0; d < ndev && !err; d++)
		if (!(err = prepare(ep, devices[d], &dps[d])))
			err = staging_acquire(devices[d], &S[d]);
	std::vector<int> rc(ndev, 0);
	std::vector<std::string> msg(ndev);
	std::vector<double> kms(ndev, 0.0);
	std::vector<unsigned long long> h((size_t)ndev * EBPF_HIST_BINS, 0);
	if (!err) {
		// one host thread per shard: contiguous shards [d*n/N, (d+1)*n/N) (shard.shard_bounds)
		std::vector<std::thread> th;
		const uint64_t n = batch->count, base = n / ndev, extra = n % ndev;
		for (int d = 0; d < ndev; d++) {
			const uint64_t lo = d * base + std::min<uint64_t>(d, extra);
			const uint64_t hi = lo + base + ((uint64_t)d < extra ? 1 : 0);
			th.emplace_back([&, d, lo, hi] {
				rc[d] = run_host_shard(ep, dps[d], *S[d], batch, lo, hi, ret, faults, &kms[d],
						       merge ? &logs[d] : nullptr);
				hipError_t e;
				if (!rc[d] && (e = hipMemcpy(&h[(size_t)d * EBPF_HIST_BINS], S[d]->d_hist,
							     EBPF_HIST_BINS * 8, hipMemcpyDeviceToHost)) !=
						  hipSuccess)
					rc[d] = hip_fail(e, "hipMemcpy(hist)");
				msg[d] = t_err;
			});
		}
		for (auto &t : th)
			t.join();
		for (int d = 0; d < ndev && !err; d++)
			if ((err = rc[d]))
				fail(err, msg[d]);
	}
	for (staging *s : S)
		if (s)
			staging_release(s);
	if (!err && merge && !(err = delta_merge_host(ep, ndev, devices)))
		err = upd_apply_host(ep, logs, true);
	if (err || !stats)
		return err;
	// the results came back over PCIe anyway: the per-shard histograms are summed here
	unsigned long long sum[EBPF_HIST_BINS] = {0};
	double kmax = 0;
	for (int d = 0; d < ndev; d++) {
		for (int i = 0; i < EBPF_HIST_BINS; i++)
			sum[i] += h[(size_t)d * EBPF_HIST_BINS + i];
		kmax = std::max(kmax, kms[d]);
	}
	return fill_stats(stats, batch->count, sum, kmax, t0);
}

EBPF_EXPORT int
ebpf_prog_run_batch_multi_dev(struct ebpf_prog *ep, int ndev, const int *devices,
			      const struct ebpf_pkt_batch *shards, uint64_t *const *ret_dev,
			      uint8_t *const *faults_dev, uint64_t *const *hist_dev,
			      void *const *streams)
{
	if (ep == nullptr || shards == nullptr || ret_dev == nullptr)
		return fail(EINVAL, "prog, shards or ret_dev is NULL");
	int err = check_devices(ndev, devices, false);
	if (err)
		return err;
	for (int d = 0; d < ndev; d++)
		if ((err = validate_batch(&shards[d], EBPF_BATCH_HIST_OVERWRITE)))
			return err;
	device_guard dg;
	std::vector<hipStream_t> st(ndev);
	for (int d = 0; d < ndev; d++)
		st[d] = streams ? static_cast<hipStream_t>(streams[d]) : nullptr;
	// A map-writing program on several shards: the batch is the shards in list order; each
	// shard's writes stay in its log, copied to the host after its launch (synchronous), and
	// the merged logs are applied there in global packet order when every shard is done.
	const bool merge = ndev > 1 && ensure_translated_locked(ep) == 0 && prog_writes_maps(*ep->xlated);
	std::vector<host_log> logs(merge ? ndev : 0);
	auto run_shard = [&](int d, const struct ebpf_pkt_batch *b, uint64_t *hist) -> int {
		if (!merge)
			return batch_dev(ep, devices[d], b, ret_dev[d], faults_dev ? faults_dev[d] : nullptr,
					 hist, st[d], nullptr);
		uint64_t first = 0;
		for (int q = 0; q < d; q++)
			first += shards[q].count;
		upd_plan plan;
		int rc = batch_dev(ep, devices[d], b, ret_dev[d], faults_dev ? faults_dev[d] : nullptr, hist,
				   st[d], &plan);
		if (rc == 0 && plan.log) {
			device_guard g2;
			hipSetDevice(devices[d]);
			rc = upd_fetch(ep->dev[devices[d]].get(), plan, st[d], first, &logs[d]);
			if (rc == 0) // (merged on the host: no offer kernel runs)
				upd_settled(plan.owner);
		}
		return rc;
	};
	if (hist_dev == nullptr) { // no collective: independent launches
		for (int d = 0; d < ndev; d++)
			if ((err = run_shard(d, &shards[d], nullptr)))
				return err;
		if (!merge)
			return 0;
		return (err = delta_merge_host(ep, ndev, devices)) ? err : upd_apply_host(ep, logs, true);
	}
	// The histogram: every shard's launch SETS its row of the scratch of its device's leading
	// stream (the first shard on that device); the rows of one device are summed into row 0,
	// row 0 is summed across devices (RCCL), and only then stored into (EBPF_BATCH_HIST_OVERWRITE)
	// or added to each caller histogram.  The caller's buffers never take part in the collective.
	std::lock_guard<std::mutex> serial(g_multi_lock); // (one call's enqueue at a time: the scratch)
	struct group {
		int device;
		std::vector<int> shard; // shard[0] leads
		unsigned long long *mh = nullptr;
		hipEvent_t *ev = nullptr;
	};
	std::vector<group> G;
	for (int d = 0; d < ndev; d++) {
		auto it = std::find_if(G.begin(), G.end(), [&](const group &g) { return g.device == devices[d]; });
		if (it == G.end()) {
			G.push_back(group{devices[d], {}});
			it = G.end() - 1;
		}
		it->shard.push_back(d);
	}
	hipError_t e;
	for (group &g : G) {
		const hipStream_t lead = st[g.shard[0]];
		if ((e = hipSetDevice(g.device)) != hipSuccess)
			return hip_fail(e, "hipSetDevice");
		// events: [0] fork (lead -> the others), [1 + j] join of shard j, [1 + k] the result
		const size_t k = g.shard.size();
		if ((err = multi_acquire(g.device, lead, (uint32_t)k, k + 2, &g.mh, &g.ev)))
			return fail(err, "multi-device histogram scratch");
		if (k > 1 && (e = hipEventRecord(g.ev[0], lead)) != hipSuccess)
			return hip_fail(e, "hipEventRecord");
		for (size_t j = 0; j < k; j++) {
			const int d = g.shard[j];
			if (j > 0 && st[d] != lead && (e = hipStreamWaitEvent(st[d], g.ev[0], 0)) != hipSuccess)
				return hip_fail(e, "hipStreamWaitEvent");
			struct ebpf_pkt_batch b = shards[d];
			b.flags |= EBPF_BATCH_HIST_OVERWRITE;
			if ((err = run_shard(d, &b, reinterpret_cast<uint64_t *>(g.mh + j * EBPF_HIST_BINS))))
				return err;
			if (j > 0 && st[d] != lead &&
			    ((e = hipEventRecord(g.ev[1 + j], st[d])) != hipSuccess ||
			     (e = hipStreamWaitEvent(lead, g.ev[1 + j], 0)) != hipSuccess))
				return hip_fail(e, "shard join");
		}
		if ((e = hipSetDevice(g.device)) != hipSuccess ||
		    (e = launch_hist_sum_rows(g.mh, (uint32_t)k, lead)) != hipSuccess)
			return hip_fail(e, "histogram rows");
	}
	const char *force = getenv("EBPF_FORCE_RCCL"); // (tests: the collective on one GPU)
	if (G.size() > 1 || (force && *force == '1')) {
		std::vector<int> dv;
		std::vector<uint64_t *> hv;
		std::vector<hipStream_t> sv;
		for (const group &g : G) {
			dv.push_back(g.device);
			hv.push_back(reinterpret_cast<uint64_t *>(g.mh));
			sv.push_back(st[g.shard[0]]);
		}
		std::string msg;
		if ((err = rccl_hist_allreduce((int)G.size(), dv.data(), hv.data(), sv.data(), &msg)))
			return fail(err, msg);
	}
	for (group &g : G) {
		const hipStream_t lead = st[g.shard[0]];
		const size_t k = g.shard.size();
		if ((e = hipSetDevice(g.device)) != hipSuccess)
			return hip_fail(e, "hipSetDevice");
		for (size_t j = 0; j < k; j++) {
			const int d = g.shard[j];
			const bool ow = (shards[d].flags & EBPF_BATCH_HIST_OVERWRITE) != 0;
			if ((e = launch_hist_store(reinterpret_cast<unsigned long long *>(hist_dev[d]), g.mh, ow,
						   lead)) != hipSuccess)
				return hip_fail(e, "histogram store");
		}
		// the other shards' streams see their histogram (and the scratch is free) after this
		if (k > 1 && (e = hipEventRecord(g.ev[1 + k], lead)) != hipSuccess)
			return hip_fail(e, "hipEventRecord");
		for (size_t j = 1; j < k; j++) {
			const int d = g.shard[j];
			if (st[d] != lead && (e = hipStreamWaitEvent(st[d], g.ev[1 + k], 0)) != hipSuccess)
				return hip_fail(e, "hipStreamWaitEvent");
		}
	}
	if (!merge)
		return 0;
	return (err = delta_merge_host(ep, ndev, devices)) ? err : upd_apply_host(ep, logs, true);
}
