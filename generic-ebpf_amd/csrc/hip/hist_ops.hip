// hist_ops.hip — verdict-histogram arithmetic of the multi-device batch
// (ebpf_prog_run_batch_multi_dev).
//
// Every shard's launch sets its own row of a library-owned scratch (EBPF_HIST_BINS u64 per
// shard); the rows of the shards that share a device are summed into row 0, row 0 is summed
// across devices by one RCCL all-reduce, and the total is then stored into (or added to) each
// caller histogram.  The caller's histograms are never the collective's buffer, so counts that
// add mode accumulated in them before the call are not multiplied by the device count.
#include <hip/hip_runtime.h>

#include "../dprog.h"
#include "ebpf_gpu.h"
#include "host/hist_ops.h"

namespace {

__global__ void __launch_bounds__(256)
hist_sum_rows(unsigned long long *__restrict__ rows, uint32_t k)
{
	for (uint32_t i = threadIdx.x; i < EBPF_HIST_BINS; i += blockDim.x) {
		unsigned long long s = rows[i];
		for (uint32_t r = 1; r < k; r++)
			s += rows[(size_t)r * EBPF_HIST_BINS + i];
		rows[i] = s;
	}
}

__global__ void __launch_bounds__(256)
hist_store(unsigned long long *__restrict__ dst, const unsigned long long *__restrict__ src,
	   uint32_t overwrite)
{
	for (uint32_t i = threadIdx.x; i < EBPF_HIST_BINS; i += blockDim.x)
		dst[i] = overwrite ? src[i] : dst[i] + src[i];
}

} // namespace

hipError_t
launch_hist_sum_rows(unsigned long long *rows, uint32_t k, hipStream_t stream)
{
	if (k <= 1)
		return hipSuccess;
	hipLaunchKernelGGL(hist_sum_rows, dim3(1), dim3(256), 0, stream, rows, k);
	return hipGetLastError();
}

hipError_t
launch_hist_store(unsigned long long *dst, const unsigned long long *src, bool overwrite,
		  hipStream_t stream)
{
	hipLaunchKernelGGL(hist_store, dim3(1), dim3(256), 0, stream, dst, src, overwrite ? 1u : 0u);
	return hipGetLastError();
}
