// bucket.hip — length classes of a batch, for the length-bucketed launches of mixed-size batches
// (gpu_runtime.cpp launch_bucketed; gen_interp.py "Length-bucketed launches").
//
// A batch in offsets form (packet i = data + offsets[i] - off_base, offsets[i+1] - offsets[i]
// bytes) is split into classes by packet length and alignment; perm lists the packet indices
// class after class, in packet order inside each class (a stable counting sort), so that each
// class's launch runs 64 (or G) packets of similar size per wave — the same divergent paths and,
// in the span-staged classes, one LDS slot size.  Class 0 is everything the span-staged kernels
// do not take: packets of at most lim[0] bytes (their headers are staged in registers already),
// longer than the last limit, or not 16-byte aligned (the span DMA reads aligned 16-B blocks).
// Class k >= 1: lim[k-1] < length <= lim[k], 16-B aligned.
//
// Path-sorted launches (gpu_runtime.cpp launch_pathsorted) sort by a byte per packet instead: the
// fault code the classifying run left (code_base + q at cut point q: class q + 1; anything else:
// class 0).
//
// Two kernels over contiguous tiles of the batch: bucket_count (per tile and class counts), then
// bucket_scatter (each tile's base per class from the counts before it; ranks in packet order by
// wave ballots), which also writes the class table cls[k] = {start, count} the launches read.
#include <hip/hip_runtime.h>

#include "host/bucket.h"

namespace {

constexpr int kThreads = 256;

__device__ inline uint32_t
klass(const bucket_args &a, uint64_t i)
{
	if (a.code) {
		const uint32_t c = (uint32_t)a.code[i] - a.code_base; // (below code_base: wraps, class 0)
		return c + 1 < a.nclass ? c + 1 : 0;
	}
	const uint64_t o0 = a.offsets[i], o1 = a.offsets[i + 1];
	const uint64_t len = o1 - o0; // (a decreasing offset is a huge length: class 0)
	const uint64_t addr = (uint64_t)(uintptr_t)a.data + (o0 - a.off_base);
	if (addr & 15)
		return 0;
	for (uint32_t k = 1; k < a.nclass; k++)
		if (len > a.lim[k - 1] && len <= a.lim[k])
			return k;
	return 0;
}

__global__ void __launch_bounds__(kThreads)
bucket_count(bucket_args a)
{
	__shared__ uint32_t cnt[kBucketMaxClass];
	if (threadIdx.x < kBucketMaxClass)
		cnt[threadIdx.x] = 0;
	__syncthreads();
	const uint64_t lo = (uint64_t)blockIdx.x * a.tile;
	const uint64_t hi = lo + a.tile < a.count ? lo + a.tile : a.count;
	for (uint64_t i = lo + threadIdx.x; i < hi; i += kThreads)
		atomicAdd(&cnt[klass(a, i)], 1u);
	__syncthreads();
	if (threadIdx.x < kBucketMaxClass)
		a.blk_cnt[(size_t)blockIdx.x * kBucketMaxClass + threadIdx.x] = cnt[threadIdx.x];
}

__global__ void __launch_bounds__(kThreads)
bucket_scatter(bucket_args a)
{
	__shared__ uint32_t red[kThreads / 64][2 * kBucketMaxClass];
	__shared__ uint32_t base[kBucketMaxClass];
	__shared__ uint32_t wcnt[kThreads / 64][kBucketMaxClass];
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	// per class: the whole batch's count and the count of the tiles before this one
	uint32_t tot[kBucketMaxClass] = {}, before[kBucketMaxClass] = {};
	for (uint32_t b = threadIdx.x; b < gridDim.x; b += kThreads)
		for (uint32_t k = 0; k < kBucketMaxClass; k++) {
			const uint32_t c = a.blk_cnt[(size_t)b * kBucketMaxClass + k];
			tot[k] += c;
			before[k] += b < blockIdx.x ? c : 0u;
		}
	for (uint32_t k = 0; k < kBucketMaxClass; k++) {
		for (int o = 32; o > 0; o >>= 1) {
			tot[k] += __shfl_down(tot[k], o);
			before[k] += __shfl_down(before[k], o);
		}
		if (lane == 0) {
			red[wave][k] = tot[k];
			red[wave][kBucketMaxClass + k] = before[k];
		}
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t start = 0;
		for (uint32_t k = 0; k < kBucketMaxClass; k++) {
			uint32_t t = 0, bf = 0;
			for (uint32_t w = 0; w < kThreads / 64; w++) {
				t += red[w][k];
				bf += red[w][kBucketMaxClass + k];
			}
			base[k] = start + bf;
			if (blockIdx.x == 0) {
				a.cls[2 * k] = start;
				a.cls[2 * k + 1] = t;
			}
			start += t;
		}
		if (blockIdx.x == 0) { // (the whole batch as one slot range: path-sorted launches)
			a.cls[2 * kBucketMaxClass] = 0;
			a.cls[2 * kBucketMaxClass + 1] = (uint32_t)a.count;
		}
	}
	__syncthreads();
	const uint64_t lo = (uint64_t)blockIdx.x * a.tile;
	const uint64_t hi = lo + a.tile < a.count ? lo + a.tile : a.count;
	for (uint64_t r = lo; r < hi; r += kThreads) {
		const uint64_t i = r + threadIdx.x;
		const bool live = i < hi;
		const uint32_t k = live ? klass(a, i) : kBucketMaxClass;
		uint32_t rank = 0;
		for (uint32_t c = 0; c < kBucketMaxClass; c++) {
			const uint64_t m = __ballot(k == c);
			if (k == c)
				rank = __popcll(m & ((1ull << lane) - 1ull));
			if (lane == 0)
				wcnt[wave][c] = (uint32_t)__popcll(m);
		}
		__syncthreads();
		if (live) {
			uint32_t off = base[k];
			for (uint32_t w = 0; w < wave; w++)
				off += wcnt[w][k];
			a.perm[off + rank] = (uint32_t)i;
		}
		__syncthreads();
		if (threadIdx.x < kBucketMaxClass) {
			uint32_t t = 0;
			for (uint32_t w = 0; w < kThreads / 64; w++)
				t += wcnt[w][threadIdx.x];
			base[threadIdx.x] += t;
		}
		__syncthreads();
	}
}

} // namespace

uint32_t
bucket_tiles(uint64_t count, uint32_t *tile)
{
	// about 4 tiles of 256 packets per CU-sized block, at most kBucketMaxTiles tiles
	uint64_t t = (count + kBucketMaxTiles - 1) / kBucketMaxTiles;
	t = (t + kThreads - 1) / kThreads * kThreads;
	if (t < 4096)
		t = 4096;
	*tile = (uint32_t)t;
	return (uint32_t)((count + t - 1) / t);
}

hipError_t
launch_bucket(const bucket_args &a, uint32_t tiles, hipStream_t stream)
{
	hipLaunchKernelGGL(bucket_count, dim3(tiles), dim3(kThreads), 0, stream, a);
	hipLaunchKernelGGL(bucket_scatter, dim3(tiles), dim3(kThreads), 0, stream, a);
	return hipGetLastError();
}
