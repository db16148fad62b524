// map_writes.h — shared by the host runtime and map_writes.hip (the apply step of map writes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One map of a map-writing program, as the apply kernels see it.  Hashtable records
// (is_hash) are replayed on the host after the batch (gpu_runtime.cpp upd_apply_host): the
// kernels leave them alone.
struct upd_map {
	uint64_t dev_base;    // the device mirror
	uint32_t value_size;
	uint32_t max_entries;
	uint64_t win_off;     // first winner word of this map (one u64 per key)
	uint32_t is_hash;
	uint32_t pad;
};

// Apply the log's records to the mirrors (last write per key, packet order) but those of the
// packets whose bit is set in `faulted` (the host clears it before the batch), and re-arm the
// log's counter; `win` holds sum(max_entries) zeroed u64 and is left zero.
hipError_t launch_map_writes(const uint8_t *log, uint32_t cap, uint32_t stride, const upd_map *maps,
			     unsigned long long *win, const uint32_t *faulted, hipStream_t stream);
