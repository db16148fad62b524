// bucket.h — shared by the host runtime and bucket.hip (length classes of a mixed-size batch, or
// the path classes of a path-sorted launch).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr uint32_t kBucketMaxClass = 16;
constexpr uint32_t kBucketMaxTiles = 1024;

struct bucket_args {
	const uint64_t *offsets; // count + 1 entries
	uint64_t off_base;
	const uint8_t *data;
	uint64_t count;          // < 2^32
	uint32_t lim[kBucketMaxClass]; // class k >= 1: lim[k-1] < length <= lim[k] (16-B aligned)
	uint32_t nclass;
	uint32_t tile;           // packets per tile (bucket_tiles)
	uint32_t *blk_cnt;       // tiles x kBucketMaxClass
	uint32_t *perm;          // count packet indices, class after class
	uint32_t *cls;           // kBucketMaxClass x {start, count}, then {0, count} (the whole batch)
	// path classes instead of length classes (code != NULL): packet i is in class
	// code[i] - code_base + 1 when that is in [1, nclass), else class 0
	const uint8_t *code;
	uint32_t code_base;
};

// Tiles of the two bucketing kernels for `count` packets (*tile packets each).
uint32_t bucket_tiles(uint64_t count, uint32_t *tile);
// Both kernels, in order, on `stream`.
hipError_t launch_bucket(const bucket_args &a, uint32_t tiles, hipStream_t stream);
