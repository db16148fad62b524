// map_writes.hip — the write side of a device batch (ebpf_gpu.h "Map writes in a device batch").
//
// During the batch every packet reads the maps as they were when it started; each
// map_update_elem that succeeds appends a record to the batch's log (dprog.h dp_launch.upd_log:
// {u64 packet, u32 entry | map << 20, u32 key, value}).  After the batch the writes land in the
// array-map mirrors in packet order — within a packet in call order (a lane takes its log
// slots call by call) — so the last write of a key wins, as if the packets had run one after the
// other (ebpf_map_array.c:173-183 memcpy).  Two passes over the log: every record offers its
// order for its key (atomicMax), then the record holding the maximum copies its value and
// re-arms the key's winner word; the log's counter is re-armed by the host (memset).
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
		const uint32_t mi = *reinterpret_cast<const uint32_t *>(r + 8) >> 20;
		const uint32_t key = *reinterpret_cast<const uint32_t *>(r + 12);
		if (maps[mi].is_hash)
			continue; // (replayed on the host)
		atomicMax(&win[maps[mi].win_off + key], (unsigned long long)rec_order(r, i));
	}
}

__global__ void __launch_bounds__(256)
upd_apply(const uint8_t *__restrict__ log, uint32_t cap, uint32_t stride,
	  const upd_map *__restrict__ maps, unsigned long long *__restrict__ win)
{
	const uint32_t n = min(*reinterpret_cast<const uint32_t *>(log), cap);
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint8_t *r = log + 64 + (uint64_t)i * stride;
		const uint32_t mi = *reinterpret_cast<const uint32_t *>(r + 8) >> 20;
		const uint32_t key = *reinterpret_cast<const uint32_t *>(r + 12);
		if (maps[mi].is_hash)
			continue;
		unsigned long long *w = &win[maps[mi].win_off + key];
		if (*w != (unsigned long long)rec_order(r, i))
			continue;
		const upd_map &m = maps[mi];
		uint8_t *dst = reinterpret_cast<uint8_t *>(m.dev_base) + (uint64_t)m.value_size * key;
		for (uint32_t b = 0; b < m.value_size; b++)
			dst[b] = r[16 + b];
		*w = 0; // the winner re-arms its key (a later check by a loser sees 0 != its order)
	}
}

} // namespace

hipError_t
launch_map_writes(const uint8_t *log, uint32_t cap, uint32_t stride, const upd_map *maps,
		  unsigned long long *win, const uint32_t *faulted, hipStream_t stream)
{
	if (cap == 0)
		return hipSuccess;
	const uint32_t blocks = std::min<uint32_t>((cap + 255) / 256, 2048);
	hipLaunchKernelGGL(upd_offer, dim3(blocks), dim3(256), 0, stream, log, cap, stride, maps, win,
			   faulted);
	hipLaunchKernelGGL(upd_apply, dim3(blocks), dim3(256), 0, stream, log, cap, stride, maps, win);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess)
		return e;
	return hipMemsetAsync(const_cast<uint8_t *>(log), 0, 4, stream);
}
