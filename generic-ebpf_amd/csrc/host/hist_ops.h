// hist_ops.h — shared by the host runtime and hist_ops.hip (multi-device histogram arithmetic).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// rows[0..EBPF_HIST_BINS) += rows[r*EBPF_HIST_BINS ..] for r in [1, k).
hipError_t launch_hist_sum_rows(unsigned long long *rows, uint32_t k, hipStream_t stream);
// dst = src (overwrite) or dst += src, EBPF_HIST_BINS u64.
hipError_t launch_hist_store(unsigned long long *dst, const unsigned long long *src, bool overwrite,
			     hipStream_t stream);
