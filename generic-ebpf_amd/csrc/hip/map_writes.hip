// map_writes.hip — the write side of a device batch (ebpf_gpu.h "Map writes in a device batch",
// "Stores into map values").
//
// During the batch every packet reads the maps as they were when it started (plus, through its
// overlay, its own stores into map values); each map_update_elem that succeeds and each store
// into a map value appends a record to the batch's log (dprog.h dp_launch.upd_log):
//   update:      {u64 packet, u32 map << 20, u32 key, value[value_size]}
//   value store: {u64 packet, u32 map << 20 | DP_REC_VALUE | kind | size, u32 offset, u64 data, ..}
// After the batch the writes land in the array mirrors in packet order — within a packet in call
// order (a lane takes its log slots call by call) — byte by byte, so the last write of a byte wins,
// as if the packets had run one after the other (ebpf_map_array.c:173-183 memcpy,
// ebpf_interpreter.c:343-366 stores).  Two passes over the log: every record offers its order for
// each byte it writes (atomicMax), then the record holding a byte's maximum copies that byte and
// re-arms its winner word; the log's counter is re-armed by the host (memset).  A map that
// stores into its values never reach has one winner word per key instead of per byte (its
// records all write whole values: upd_map.gran).  Counter updates
// of UPD_ATOMIC maps were added into the map's delta area during the batch: a third kernel adds
// that area into the values and zeroes it.
#include <hip/hip_runtime.h>

#include "../dprog.h"
#include "host/map_writes.h"

namespace {

// A record's order: (packet, log slot).  A lane takes its log slots one call after the other,
// so within a packet the slot index is the call order (the state-tree entry index is not: a
// run-time-map compare chain's copies and standard-semantics merge points are numbered after
// entries that a path reaches later).
__device__ inline uint64_t
rec_order(const uint8_t *r, uint32_t slot)
{
	const uint64_t pkt = *reinterpret_cast<const uint64_t *>(r);
	return ((pkt << 32) | slot) + 1; // 0 = no write
}

// The bytes [*lo, *lo + *n) of the map's values a record writes (false: none here).
__device__ inline bool
rec_span(const uint8_t *r, const upd_map &m, uint64_t *lo, uint32_t *n)
{
	const uint32_t w = *reinterpret_cast<const uint32_t *>(r + 8);
	const uint32_t x = *reinterpret_cast<const uint32_t *>(r + 12);
	if (w & DP_REC_VALUE) {
		*lo = x;
		*n = w & 0xf;
		return (w & DP_REC_ADD) == 0 && *lo + *n <= (uint64_t)m.value_size * m.max_entries;
	}
	if (x >= m.max_entries)
		return false;
	*lo = (uint64_t)x * m.value_size;
	*n = m.value_size;
	return true;
}

__global__ void __launch_bounds__(256)
upd_offer(const uint8_t *__restrict__ log, uint32_t cap, uint32_t stride,
	  const upd_map *__restrict__ maps, unsigned long long *__restrict__ win,
	  const uint32_t *__restrict__ faulted)
{
	const uint32_t n = min(*reinterpret_cast<const uint32_t *>(log), cap);
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint8_t *r = log + 64 + (uint64_t)i * stride;
		const uint32_t pkt = *reinterpret_cast<const uint32_t *>(r);
		if (faulted && ((faulted[pkt >> 5] >> (pkt & 31)) & 1u))
			continue; // the packet faulted after this write: no write of it lands
		const upd_map &m = maps[*reinterpret_cast<const uint32_t *>(r + 8) >> 20];
		uint64_t lo;
		uint32_t nb;
		if (m.cls != UPD_DEVICE || !rec_span(r, m, &lo, &nb))
			continue; // (replayed on the host, or an atomic map's)
		const unsigned long long o = rec_order(r, i);
		for (uint32_t b = 0; b < nb; b += m.gran)
			atomicMax(&win[m.win_off + (lo + b) / m.gran], o);
	}
}

__global__ void __launch_bounds__(256)
upd_apply(const uint8_t *__restrict__ log, uint32_t cap, uint32_t stride,
	  const upd_map *__restrict__ maps, unsigned long long *__restrict__ win)
{
	const uint32_t n = min(*reinterpret_cast<const uint32_t *>(log), cap);
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint8_t *r = log + 64 + (uint64_t)i * stride;
		const upd_map &m = maps[*reinterpret_cast<const uint32_t *>(r + 8) >> 20];
		uint64_t lo;
		uint32_t nb;
		if (m.cls != UPD_DEVICE || !rec_span(r, m, &lo, &nb))
			continue;
		const unsigned long long o = rec_order(r, i);
		uint8_t *dst = reinterpret_cast<uint8_t *>(m.dev_base) + lo;
		for (uint32_t b = 0; b < nb; b += m.gran) {
			unsigned long long *w = &win[m.win_off + (lo + b) / m.gran];
			if (*w != o)
				continue;
			for (uint32_t c = 0; c < m.gran; c++)
				dst[b + c] = r[16 + b + c];
			*w = 0; // the winner re-arms its word (a later check by a loser sees 0 != its order)
		}
	}
}

// values[i] += delta[i], delta[i] = 0: the counter updates of a UPD_ATOMIC map
template <typename T>
__global__ void __launch_bounds__(256)
delta_apply(T *__restrict__ vals, T *__restrict__ delta, uint64_t words)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const T d = delta[i];
		if (d) {
			vals[i] += d;
			delta[i] = 0;
		}
	}
}

} // namespace

hipError_t
launch_map_writes(const uint8_t *log, uint32_t cap, uint32_t stride, const upd_map *maps,
		  const upd_map *maps_host, uint32_t nmaps, unsigned long long *win,
		  const uint32_t *faulted, hipStream_t stream)
{
	bool device = false;
	for (uint32_t t = 0; t < nmaps; t++)
		device = device || maps_host[t].cls == UPD_DEVICE;
	if (cap && device) {
		const uint32_t blocks = std::min<uint32_t>((cap + 255) / 256, 2048);
		hipLaunchKernelGGL(upd_offer, dim3(blocks), dim3(256), 0, stream, log, cap, stride, maps,
				   win, faulted);
		hipLaunchKernelGGL(upd_apply, dim3(blocks), dim3(256), 0, stream, log, cap, stride, maps,
				   win);
	}
	for (uint32_t t = 0; t < nmaps; t++) {
		const upd_map &m = maps_host[t];
		if (m.cls != UPD_ATOMIC)
			continue;
		const uint64_t bytes = (uint64_t)m.value_size * m.max_entries, words = bytes / m.width;
		uint8_t *v = reinterpret_cast<uint8_t *>(m.dev_base);
		uint8_t *d = v + dp_delta_off(m.value_size, m.max_entries);
		const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + 255) / 256, 2048);
		if (m.width == 8)
			hipLaunchKernelGGL(delta_apply<unsigned long long>, dim3(blocks), dim3(256), 0, stream,
					   reinterpret_cast<unsigned long long *>(v),
					   reinterpret_cast<unsigned long long *>(d), words);
		else
			hipLaunchKernelGGL(delta_apply<uint32_t>, dim3(blocks), dim3(256), 0, stream,
					   reinterpret_cast<uint32_t *>(v), reinterpret_cast<uint32_t *>(d), words);
	}
	hipError_t e = hipGetLastError();
	if (e != hipSuccess || cap == 0)
		return e;
	return hipMemsetAsync(const_cast<uint8_t *>(log), 0, 4, stream);
}
