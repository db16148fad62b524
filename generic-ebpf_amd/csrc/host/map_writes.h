// map_writes.h — shared by the host runtime and map_writes.hip (the apply step of map writes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One map of a map-writing program, as the apply kernels see it (dprog_host upd_maps /
// hupd_maps / atomic_maps).  Only UPD_DEVICE maps' records land here; the records of UPD_HOST
// maps (hashtables, arrays mixing counter updates and stores) are replayed on the host after the
// batch (gpu_runtime.cpp upd_apply_host), and UPD_ATOMIC maps log nothing (their counter updates
// went into the delta area during the batch).
enum { UPD_NONE = 0, UPD_DEVICE = 1, UPD_HOST = 2, UPD_ATOMIC = 3 };
struct upd_map {
	uint64_t dev_base;    // the device mirror
	uint32_t value_size;
	uint32_t max_entries;
	uint64_t win_off;     // first winner word of this map
	uint32_t gran;        // value bytes per winner word: 1 when stores into its values may reach
	                      // the map (byte winners), else value_size (whole-value updates: per key)
	uint32_t pad;
	uint32_t cls;         // UPD_*
	uint32_t width;       // UPD_ATOMIC: counter bytes (4 or 8)
};

// Apply the log's records to the mirrors of UPD_DEVICE maps — byte by byte, the last write in
// (packet, call) order wins — but those of the packets whose bit is set in `faulted` (the host
// clears it before the batch), and re-arm the log's counter; `win` holds the winner words
// (zeroed, and left zero).  Then add every UPD_ATOMIC map's delta area into its values (and zero
// it).  `nmaps` entries in `maps`.
hipError_t launch_map_writes(const uint8_t *log, uint32_t cap, uint32_t stride, const upd_map *maps,
			     const upd_map *maps_host, uint32_t nmaps, unsigned long long *win,
			     const uint32_t *faulted, hipStream_t stream);
