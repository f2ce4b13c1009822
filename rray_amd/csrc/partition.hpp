// partition.hpp — the multi-GPU row partition and the gather layout, shared by the device kernels
// (multi.cpp unshuffle_kernel), the host ABI (rr_part_rows, rr_unshuffle_host) and therefore by every
// caller that rehearses the N > 1 path without a GPU (bench.py --dry-run, tests/test_dist_gloo.py).
//
// Part p of nparts owns the output rows {y : (y / block) % nparts == p} (interleaved blocks balance the
// sky / floor cost), rendered into a tile in increasing y.  The gather (ncclGather, root 0)
// lays the tiles back to back, each padded to the largest part's row count (part 0's).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rr {

// rows of part `part` (closed form of counting its blocks)
__host__ __device__ inline int64_t part_rows_count(int64_t height, int32_t part, int32_t nparts, int32_t block) {
    const int64_t cycle = (int64_t)block * nparts;
    const int64_t full = height / cycle;
    int64_t rest = height - full * cycle - (int64_t)part * block;
    rest = rest < 0 ? 0 : (rest > block ? (int64_t)block : rest);
    return full * block + rest;
}

// padded rows per tile in the gathered buffer: part 0 holds the most rows
__host__ __device__ inline int64_t gather_tile_rows(int64_t height, int32_t nparts, int32_t block) {
    return part_rows_count(height, 0, nparts, block);
}

// output row y -> its row in the gathered buffer: tile p = (y / block) % nparts, local row
// j = (y / (block * nparts)) * block + y % block of that tile
__host__ __device__ inline int64_t gathered_row_of(int64_t y, int32_t nparts, int32_t block, int64_t tile_rows) {
    const int64_t p = (y / block) % nparts;
    const int64_t j = (y / ((int64_t)block * nparts)) * block + y % block;
    return p * tile_rows + j;
}

// tile row j of part `part` -> its output row (the inverse of gathered_row_of within one tile)
__host__ __device__ inline int64_t frame_row_of(int64_t j, int32_t part, int32_t nparts, int32_t block) {
    return ((j / block) * nparts + part) * (int64_t)block + j % block;
}

// The runs of part `part`'s tile: f(first tile row, first output row, rows) for each interleave block it owns,
// in tile order.  Sender and receiver of the frame transfer enumerate the same runs, so their point-to-point
// operations pair up in order (multi.cpp); rr_unshuffle_host copies the same runs on the CPU.
template <class F>
inline void for_each_part_run(int64_t height, int32_t part, int32_t nparts, int32_t block, F&& f) {
    const int64_t rows = part_rows_count(height, part, nparts, block);
    for (int64_t j = 0; j < rows; j += block)
        f(j, frame_row_of(j, part, nparts, block), rows - j < block ? rows - j : (int64_t)block);
}

}  // namespace rr
