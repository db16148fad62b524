/*
 * ebpf_gpu.h — batch execution of one loaded eBPF program over many packets on MI355X.
 *
 * This is the engine's C-ABI extension to the reference API (sys/sys/ebpf.h).  The reference
 * has no batch entry point: callers loop over packets and call ebpf_prog_run(ctx, ep) once per
 * packet (sys/dev/ebpf/ebpf_interpreter.c:23; hot loop #1 in SURVEY.md §3(C)).  Each function
 * below replaces that caller loop:
 *
 *   ebpf_prog_run_batch      ↔ for (i..n) ret[i] = ebpf_prog_run(pkt_i, ep);   host buffers
 *   ebpf_prog_run_batch_dev  ↔ the same loop over device-resident packets (the measured path)
 *
 * Per packet the result is bit-identical to ebpf_prog_run on the same bytes (reference
 * semantics, including its quirks: cumulative pc stepping, MOV64 = add, NEG, logical ARSH —
 * ebpf_interpreter.c:39,89-91,110-115,182-184,197-208).  Where the reference has no defined
 * behaviour (it crashes, aborts, hangs or reads stray memory) the device stops that packet
 * and records an ebpf_fault code instead; ret[i] is then 0.
 *
 * Plain pointers and sizes only; no torch or HIP types in any signature (a HIP stream is
 * passed as void*).
 */
#ifndef EBPF_AMD_EBPF_GPU_H
#define EBPF_AMD_EBPF_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ebpf_prog;
struct ebpf_map;

/* Map writes in a device batch.  The reference runs packets one at a time, so a program's
 * map_update_elem (ebpf_map.c:101-108 -> ebpf_map_array.c:185-211) is seen by the next packet.
 * A device batch runs its packets at once; its defined semantics are those of the caller's
 * loop with the writes held back until the loop ends:
 *   - every packet reads the maps as they were when the batch started (its own writes too);
 *   - map_update_elem returns the reference's code: EINVAL for a NULL key or value or flags >
 *     EBPF_EXIST, EEXIST for EBPF_NOEXIST (an array's keys all exist), EINVAL for a key >=
 *     max_entries, else 0;
 *   - after the batch the writes land in packet order, a packet's own in call order: the last
 *     write of a key wins; a packet that faults (any code, even after its writes) leaves no
 *     write behind;
 *   - map_delete_elem on an array map returns EINVAL (ebpf_map_array.c:246-250);
 *   - on a hashtable map, map_update_elem returns the reference's code against the batch-start
 *     table: EINVAL as above, EEXIST (EBPF_NOEXIST, the key present) / ENOENT (EBPF_EXIST, the
 *     key absent) (ebpf_map_hashtable.c:87-100), EBUSY for a new key when the table was full
 *     (:371-377), else 0; map_delete_elem returns 0 (:475-502; EINVAL for a NULL key).  The key
 *     is read (region-checked) before the flags are judged, the value only by a call returning
 *     0.  The calls that returned 0 are replayed on the host table after the batch, in the same
 *     packet / call order, through the map's own update / delete (percpu: the submitting CPU's
 *     value): the table is the one the reference would hold after those calls in that order; a
 *     replayed call that fails against the table as it then is (EEXIST, ENOENT, EBUSY) leaves it
 *     unchanged.  A batch with hashtable writes synchronises with the host before it returns;
 *   - the map may be known only at run time (r1 computed or loaded): the helper then checks r1
 *     against the maps of the program; r1 NULL (or a NULL key / value, or flags > EBPF_EXIST)
 *     is EINVAL as in ebpf_map.c:101-108 / :130-136, a pointer that is no map of them faults
 *     EBPF_FAULT_BAD_MAP (the reference dereferences it);
 *   - a loop-free program makes every write its path reaches, however many, as the reference
 *     does (the log is sized by the program's longest path).  A program with loops (standard
 *     semantics: a backward jump reachable from slot 0 on the slot graph — not JA -1, which
 *     spins into EBPF_FAULT_LOOP, nor a jump before slot 0, EBPF_FAULT_SLOT; decided from the
 *     bytecode) has no per-path bound, so there a packet may make 16 logged
 *     writes: map_update_elem calls that return 0, every hashtable map_delete_elem (whether the
 *     key exists is known only at the replay), stores into map values, and counter updates
 *     into a hashtable's values (records replayed after the batch); counter updates into an
 *     array aligned to their width (below) are not counted (device atomics).  The 17th faults
 *     the packet with EBPF_FAULT_WRITES (a fault: its writes do not land, its counter updates
 *     do);
 *   - a writing program sharded over several devices (ebpf_prog_run_batch_multi*): the batch is
 *     the shards in order, every shard reads the batch-start maps, and the shards' writes are
 *     merged on the host in that global packet order after the last shard — the same result as
 *     one batch on one device (ebpf_prog_run_batch_multi_dev then synchronises its streams).
 * The written values live in the device's mirror of the map until the host API touches the map
 * (lookup / update / delete / get_next_key, or a helper call from ebpf_prog_run), which copies
 * them back first.  ebpf_prog_run itself keeps the reference's immediate writes.
 *
 * Stores into map values.  The reference hands the program a pointer into the map's storage
 * (array_map_lookup_elem, ebpf_map_array.c:115-124; a hashtable element's value,
 * ebpf_map_hashtable.c:285-301) and ST / STX write through it in place
 * (ebpf_interpreter.c:343-366).  In a device batch:
 *   - a packet's loads (LDX, and the load of a counter update or XADD below) see its own
 *     earlier stores into map values; other packets of the batch see the batch-start maps.
 *     Helper calls read keys and values as the batch started.  (A loop-free path may store and
 *     read back up to 2,048 times; past 16 such stores the batch runs on the portable
 *     interpreter, the packets' views in device memory.  Loops: below);
 *   - after the batch the stores land in packet order, a packet's own in program order, byte by
 *     byte: the last store of each byte wins (together with map_update_elem's whole values);
 *   - counter updates land as additions: three consecutive instructions (JA aside)
 *     LDX{W,DW} X = [P + off] (X != P); ADD or SUB to X of an immediate or of a register other
 *     than X (64-bit; 32-bit too for W; under the reference's semantics MOV64, which adds);
 *     STX [P + off] = X of the same width — and, under standard semantics, XADD
 *     (BPF_STX | BPF_XADD, W / DW; imm 0, or 1 = BPF_FETCH: src receives the old value) — add
 *     (stored - loaded) mod 2^width when the address is aligned to the width within the map's
 *     values (arrays: from the first value; hashtables: from the value's start), else land as
 *     plain stores.  Additions commute, so a map that only counter updates touch in a batch ends
 *     as the reference's sequential run leaves it (per-packet counters, byte counts);
 *   - a packet that faults leaves no write behind except its counter updates, which are atomic
 *     operations: they take effect when executed;
 *   - EBPF_FAULT_MAP_WRITE is left for a store into a map value the translation did not provide
 *     for (a packet-relative pointer that lands in a map);
 *   - in a program with loops (standard semantics) a counter update must go to a hashtable
 *     (a logged write, counted as above) or to an array that only aligned counter updates of
 *     one width change (the batch functions return EOPNOTSUPP for an array that mixes them with
 *     other writes).  The packet may read its counters back through an XADD with BPF_FETCH or
 *     through the idiom's register (live after the STX: the program "reads its counters back",
 *     decided from its bytecode on the slot graph — a reachable such XADD or idiom, a CALL
 *     reading its helper's arguments (lookup, delete r1-r2; update r1-r4), EXIT r0); it then
 *     sees the batch-start value plus its own additions,
 *     kept in 32 8-byte words of map values per packet: a store, counter update or XADD that
 *     needs a word beyond them faults EBPF_FAULT_WRITES before it happens (a word already held
 *     is free: one counter updated on every trip takes one).  The map still lands as additions.
 *     A read-back of another form (a later plain load of a counter's word) returns EOPNOTSUPP
 *     when the program also updates array counters (device atomics, not counted, so nothing
 *     else bounds that view); with hashtable counters alone it is allowed.  Plain stores,
 *     hashtable counter updates and map_update_elem / map_delete_elem in loops are limited
 *     only by the 16 logged writes per packet.
 * How it runs: arrays changed only by aligned counter updates of one width take device atomics
 * into a delta area next to their mirror (added into the values after the batch); other arrays'
 * stores land on the device (per-byte winners); hashtables, and arrays that mix counter updates
 * with stores, replay the batch's records on the host in order. */

/* Per-packet fault codes (0 = the program reached EXIT). */
enum ebpf_fault {
	EBPF_FAULT_NONE = 0,
	EBPF_FAULT_BAD_OPCODE = 1,   /* opcode outside the dispatch table (ebpf_interpreter.c:367-369: abort) */
	EBPF_FAULT_DIV_ZERO = 2,     /* DIV/MOD by 0 (reference: SIGFPE) */
	EBPF_FAULT_MEM = 3,          /* load/store outside this packet, its stack or a map value */
	EBPF_FAULT_SLOT = 4,         /* stepping left the program (reference reads past the buffer) */
	EBPF_FAULT_HELPER = 5,       /* CALL id outside [0,64) or an unset helper slot (:283) */
	EBPF_FAULT_HELPER_UNSUPPORTED = 6, /* helper with no device implementation */
	EBPF_FAULT_BAD_REG = 7,      /* dst/src register nibble >= 11 (reference overflows reg[]) */
	EBPF_FAULT_LOOP = 8,         /* a jump that re-enters its own state: the reference never returns;
	                                standard semantics: the loop budget is spent (see below) */
	EBPF_FAULT_MAP_WRITE = 9,    /* store into a map value through a pointer the translation did
	                                not see reach a map ("Stores into map values" above) */
	EBPF_FAULT_BAD_MAP = 10,     /* map helper called with r1 not a map of this program's env */
	EBPF_FAULT_WRITES = 11,      /* the packet's 17th logged map write in a device batch ("Map
	                                writes in a device batch" above) */
	EBPF_FAULT_MAX
};

/* Batch descriptor.  Fixed-stride mode (offsets == NULL): packet i occupies
 * [data + i*stride, data + (i+1)*stride).  Offsets mode: packet i occupies
 * [data + offsets[i], data + offsets[i+1]) — offsets has count+1 entries.  Extents mode
 * (flags & EBPF_BATCH_EXTENTS): packet i occupies [data + offsets[2i], data + offsets[2i+1]) —
 * offsets has 2*count entries, start <= end, packets in any order, with gaps between them or
 * overlapping (a capture's records in place: ebpf_pcap_extents).  A program that stores into
 * overlapping packets leaves their common bytes unspecified. */
struct ebpf_pkt_batch {
	const void *data;
	const uint64_t *offsets;
	uint64_t count;
	uint32_t stride;
	uint32_t flags; /* EBPF_BATCH_* */
};

/* ebpf_prog_run_batch_dev: hist_dev receives this batch's counts instead of having them added,
 * so the caller need not zero it before each launch. */
#define EBPF_BATCH_HIST_OVERWRITE 0x1u
/* Every batch entry point: offsets holds (start, end) pairs (extents mode above). */
#define EBPF_BATCH_EXTENTS 0x2u

/* Verdict histogram: bin min(r0, 255) for packets that reached EXIT, bin 256 = faulted. */
#define EBPF_HIST_BINS 257

/* Per-call summary for the host-buffer entry point. */
struct ebpf_batch_stats {
	uint64_t packets;
	uint64_t faulted;
	uint64_t hist[EBPF_HIST_BINS];
	double kernel_ms;     /* device time of the interpreter launches */
	double total_ms;      /* wall time including H2D/D2H */
};

/* A packet capture as a batch (the path starts in host memory: a NIC ring or a pcap buffer).
 * `capture` holds a classic libpcap file (magic 0xa1b2c3d4 / 0xa1b23c4d, either byte order):
 * packet i of the batch is record i's captured bytes, in offsets form, ready for
 * ebpf_prog_run_batch.  The library allocates batch->data and batch->offsets (pinned host memory
 * when `pinned` and a GPU is present, else pageable); release both with ebpf_pcap_batch_free.
 * The capture buffer stays the caller's and is not referenced afterwards.
 * A record whose captured length exceeds the header's snaplen becomes its first snaplen bytes
 * (libpcap's reader does the same), counted in info->truncated.
 * Returns 0, EINVAL (not a classic pcap capture, or a record header or record that runs past
 * the end of `capture`; ebpf_gpu_last_error says which), ENOMEM.  Host only: no GPU needed. */
struct ebpf_pcap_info {
	uint32_t linktype;     /* the capture's link-layer type (1 = Ethernet) */
	uint32_t snaplen;
	uint32_t nanosecond;   /* 1: nanosecond timestamps (magic 0xa1b23c4d) */
	uint32_t byte_swapped; /* 1: written in the other byte order */
	uint64_t truncated;    /* records whose captured length is below the original length */
	uint64_t bytes;        /* captured bytes of all records (batch->offsets[count]) */
};
int ebpf_pcap_batch(const void *capture, size_t len, int pinned, struct ebpf_pkt_batch *batch,
		    struct ebpf_pcap_info *info);
/* The same capture as an extents-mode batch over the capture itself: batch->data = capture (no
 * copy; it must stay valid while the batch is used), batch->offsets = the library's (start, end)
 * pair of every record's captured bytes (snaplen-truncated as above), flags =
 * EBPF_BATCH_EXTENTS.  Only the offsets are allocated (pinned on request); release them with
 * ebpf_pcap_batch_free, which leaves an extents batch's data alone.  Same errors. */
int ebpf_pcap_extents(const void *capture, size_t len, int pinned, struct ebpf_pkt_batch *batch,
		      struct ebpf_pcap_info *info);
void ebpf_pcap_batch_free(struct ebpf_pkt_batch *batch);

/* Number of visible GPUs (0 on a host without one). Never fails. */
int ebpf_gpu_device_count(void);

/* Initialise the device backend on GPUs 0..ndev-1 (ndev <= 0: every visible GPU): load the
 * kernels' code object on each, which the first batch on a device would otherwise do.  Optional.
 * Returns 0, ENODEV (no GPU, or ndev above the visible count), EIO (a code object did not
 * load on a device; ebpf_gpu_last_error says which).  (ebpf_dev_init) */
int ebpf_dev_init(int ndev);

/* Translate + upload the program (and its maps) to `device`.  Called implicitly by the run
 * functions; explicit calls move the one-time cost out of a timed region.
 * Returns 0, ENODEV (no GPU / no device code object), E2BIG (program state graph too large),
 * ENOMEM. */
int ebpf_prog_prepare_device(struct ebpf_prog *ep, int device);

/* Host buffers in, host buffers out; runs on the current device (ebpf_gpu_set_device).
 * ret: count u64 (required).  faults: count u8 (optional).  stats: optional.
 * Returns 0 or an errno; packet faults are NOT call errors. */
int ebpf_prog_run_batch(struct ebpf_prog *ep, const struct ebpf_pkt_batch *batch,
			uint64_t *ret, uint8_t *faults, struct ebpf_batch_stats *stats);

/* ebpf_prog_run_batch without blocking the caller: the job is queued for the worker pool of the
 * calling thread's current device (two persistent threads per device, a FIFO of at most 64
 * queued jobs) and the call returns at once, so a NIC-ring or capture consumer can fill its next
 * segment meanwhile; ebpf_batch_wait blocks until ret/faults hold the results, returns the
 * batch's error code (ebpf_prog_run_batch's) and releases the job (wait once per job).  The
 * program, the batch's buffers, ret and faults must stay valid until the wait; several jobs may
 * be in flight.
 * Returns 0, EINVAL (NULL argument), ENODEV (no GPU), ENOMEM, EAGAIN (the device's queue is
 * full — wait for an earlier job — or no worker thread could be started). */
struct ebpf_batch_job;
int ebpf_prog_run_batch_async(struct ebpf_prog *ep, const struct ebpf_pkt_batch *batch,
			      uint64_t *ret, uint8_t *faults, struct ebpf_batch_job **job);
int ebpf_batch_wait(struct ebpf_batch_job *job, struct ebpf_batch_stats *stats);

/* Device-resident batch: every pointer (batch->data, batch->offsets, ret_dev, faults_dev,
 * hist_dev) is device memory on `device`.  Enqueued on `stream` (hipStream_t, NULL = default
 * stream) and returns without synchronising.  faults_dev / hist_dev may be NULL; hist_dev is
 * EBPF_HIST_BINS u64 counters that the kernel ADDS to (zero it yourself), or, with
 * EBPF_BATCH_HIST_OVERWRITE in batch->flags, sets to this batch's counts. */
int ebpf_prog_run_batch_dev(struct ebpf_prog *ep, int device, const struct ebpf_pkt_batch *batch,
			    uint64_t *ret_dev, uint8_t *faults_dev, uint64_t *hist_dev,
			    void *stream);

/* One batch sharded over several GPUs of this process (packets are independent,
 * maps are read-only during a batch, so the batch splits into contiguous shards
 * [d*n/N, (d+1)*n/N) with no data exchange; bytecode and map mirrors are replicated per device).
 *
 * ebpf_prog_run_batch_multi: host buffers, as ebpf_prog_run_batch; one host thread per device
 *   runs its shard's chunked H2D -> kernel -> D2H pipeline.  `devices` may repeat a device (two
 *   shards then share it).  stats->hist is the sum of the shards' histograms, stats->kernel_ms
 *   the slowest shard's device time.
 * ebpf_prog_run_batch_multi_dev: device-resident, asynchronous: shards[d], ret_dev[d],
 *   faults_dev[d] (optional), hist_dev[d] (optional) live on devices[d] and each launch is
 *   enqueued on streams[d] (NULL array = default streams).  `devices` may repeat a device.  With
 *   hist_dev, the batch's histogram — the SUM over all shards — is added to each hist_dev[d], or
 *   stored into it when shards[d].flags has EBPF_BATCH_HIST_OVERWRITE, as ebpf_prog_run_batch_dev
 *   does for one shard.  The sum is formed in library-owned scratch (the shards of one device
 *   summed on the first one's stream, then one RCCL all-reduce (uint64, sum) over the distinct
 *   devices: the path's only collective); streams[d] sees hist_dev[d] complete in stream order.
 *   Returns ENOSYS if several distinct devices are given and RCCL (librccl.so.1) cannot be
 *   loaded.
 * Neither changes the calling thread's current HIP device (no entry point of this header does).
 * Both return 0 or an errno (ENODEV: a device index out of range; EINVAL: bad arguments). */
int ebpf_prog_run_batch_multi(struct ebpf_prog *ep, int ndev, const int *devices,
			      const struct ebpf_pkt_batch *batch, uint64_t *ret, uint8_t *faults,
			      struct ebpf_batch_stats *stats);
int ebpf_prog_run_batch_multi_dev(struct ebpf_prog *ep, int ndev, const int *devices,
				  const struct ebpf_pkt_batch *shards, uint64_t *const *ret_dev,
				  uint8_t *const *faults_dev, uint64_t *const *hist_dev,
				  void *const *streams);

/* Select the device used by ebpf_prog_run_batch for the calling thread. */
int ebpf_gpu_set_device(int device);

/* Device path used by subsequent launches (all bit-identical):
 *   0 = default: the program compiled to gfx950 code (copy-and-patch of the assembly
 *       interpreter's handlers); a program too large for the code area runs on the assembly
 *       interpreter.  Launches fail with ENOSYS if the code object cannot be loaded.
 *   1 = the portable HIP interpreter (correctness baseline).
 *   2 = the hand-written gfx950 assembly interpreter. */
int ebpf_gpu_set_variant(int variant);

/* Measurement hook (extension): the calling thread's next ebpf_prog_run_batch_dev records
 * `start_event` at the start of the launch's kernel and `stop_event` at its end, on the launch
 * stream, so that hipEventElapsedTime gives the kernel's own duration (a launch is one kernel:
 * the verdict histogram is reduced inside it).  Both are hipEvent_t of the HIP runtime the
 * library runs on; NULL, NULL cancels.  Returns 0, or EINVAL if only one is NULL. */
int ebpf_gpu_time_next_launch(void *start_event, void *stop_event);

/* Instruction semantics of a program (extension: the reference has only the first).
 *   EBPF_SEM_REFERENCE (default): the reference interpreter's, quirks included
 *       (ebpf_interpreter.c:23-372: cumulative stepping, MOV64 adds, NEG ignores dst, NEG64 is
 *       dst - imm, logical ARSH, DIV/MOD by zero faults).
 *   EBPF_SEM_STANDARD: standard eBPF as compilers emit it: sequential pc (a jump goes to
 *       pc + 1 + off), MOV64 moves (imm sign-extended), NEG/NEG64 negate dst, arithmetic ARSH,
 *       DIV by zero gives 0 and MOD by zero leaves dst (32-bit ops: truncated), and the JMP32
 *       class (opcode class 0x06, compares of the low 32 bits).  Loops: in a device batch a
 *       packet may take 2^20 backward jumps (taken jumps whose target is at or before their own
 *       slot); the next one stops it with EBPF_FAULT_LOOP.  Map writes inside loops: see "Map
 *       writes in a device batch" and "Stores into map values" above (16 logged writes per
 *       packet; counter updates as additions).  ebpf_prog_run runs any program unbounded.
 * Applies to ebpf_prog_run and to device batches.  Returns 0, EINVAL (bad argument) or EBUSY
 * (the program was already translated for a device). */
#define EBPF_SEM_REFERENCE 0
#define EBPF_SEM_STANDARD 1
int ebpf_prog_set_semantics(struct ebpf_prog *ep, int semantics);

/* Information about the translated device program. */
struct ebpf_dprog_info {
	uint32_t nslots;       /* prog_len / 8 */
	uint32_t nentries;     /* executed-state entries after translation */
	uint32_t nmaps;        /* array maps resolved from LDDW immediates */
	uint32_t max_stack;    /* deepest statically known stack access (bytes below r10) */
};
int ebpf_prog_device_info(struct ebpf_prog *ep, struct ebpf_dprog_info *info);

/* What ran, and what it cost to get there (extension; measurement and diagnostics). */
#define EBPF_EXEC_COMPILED 0     /* the program compiled to gfx950 code (variant 0) */
#define EBPF_EXEC_HIP 1          /* the portable HIP interpreter (variant 1) */
#define EBPF_EXEC_INTERPRETER 2  /* the gfx950 assembly interpreter (variant 2, or variant 0 on a
                                    program too large for the code area) */
struct ebpf_dexec_info {
	int32_t exec;          /* EBPF_EXEC_* of the last launch on `device`; -1 = none yet */
	int32_t layout;        /* its kernel: 1 = staged fixed 64-B packets, 0 = general; -1 =
	                          none */
	double translate_ms;   /* host time of the state-tree translation (once per program) */
	double build_ms;       /* compile (COMPILED) or lower + link (INTERPRETER) time for that
	                          kernel on that device, paid at its first launch; 0 for HIP */
};
int ebpf_prog_device_exec(struct ebpf_prog *ep, int device, struct ebpf_dexec_info *info);

/* Diagnostics: the program as compiled for variant 0, raw gfx950 instruction bytes, for packet
 * `layout` 1 (fixed 64-B packets) or 0 (any stride / offsets); others EINVAL.  Host only (no
 * GPU needed; map base addresses are then 0).  *len: in = size of buf, out = bytes of code.  buf == NULL just
 * sizes.  Returns 0, ENOSPC (buf too small), E2BIG (program too large to compile). */
int ebpf_prog_device_code(struct ebpf_prog *ep, int layout, void *buf, size_t *len);

/* Human-readable description of the last error on this thread ("" if none). */
const char *ebpf_gpu_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* EBPF_AMD_EBPF_GPU_H */
