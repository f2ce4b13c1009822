// partition.hpp — the multi-GPU row partition and the staging layout, shared by the device kernels
// (multi.cpp place_tile_kernel), the host ABI (rr_part_rows, rr_unshuffle_host) and therefore by every
// caller that rehearses the N > 1 path without a GPU (bench.py --dry-run, tests/test_dist_gloo.py).
//
// Part p of nparts owns the output rows {y : (y / block) % nparts == p} (interleaved blocks balance the
// sky / floor cost), rendered into a tile in increasing y.  The transfer (one ncclSend per
// part, one ncclRecv per part on rank 0, multi.cpp) lays the tiles back to back in a staging buffer of
// `height` rows, unpadded: part p's tile starts at stage row stage_row_offset(p).
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

// first stage row of part `part`'s tile: the rows of parts 0 .. part-1 (each owns `full` whole blocks, and the
// remainder of the last cycle goes block by block to the parts in order, so parts below `part` hold
// min(rest, part * block) of it)
__host__ __device__ inline int64_t stage_row_offset(int64_t height, int32_t part, int32_t nparts, int32_t block) {
    const int64_t cycle = (int64_t)block * nparts;
    const int64_t full = height / cycle, rest = height - full * cycle, lead = (int64_t)part * block;
    return (int64_t)part * full * block + (rest < lead ? rest : lead);
}

// output row y -> its row in the staging buffer: tile p = (y / block) % nparts, local row
// j = (y / (block * nparts)) * block + y % block of that tile, at stage_row_offset(p) + j
__host__ __device__ inline int64_t stage_row_of(int64_t y, int64_t height, int32_t nparts, int32_t block) {
    const int32_t p = (int32_t)((y / block) % nparts);
    const int64_t j = (y / ((int64_t)block * nparts)) * block + y % block;
    return stage_row_offset(height, p, nparts, block) + j;
}

// tile row j of part `part` -> its output row (the inverse of stage_row_of within one tile)
__host__ __device__ inline int64_t frame_row_of(int64_t j, int32_t part, int32_t nparts, int32_t block) {
    return ((j / block) * nparts + part) * (int64_t)block + j % block;
}

// The runs of part `part`'s tile: f(first tile row, first output row, rows) for each interleave block it owns,
// in tile order — the rows place_tile_kernel moves from the staging buffer into the frame (multi.cpp);
// rr_unshuffle_host copies the same runs on the CPU.
template <class F>
inline void for_each_part_run(int64_t height, int32_t part, int32_t nparts, int32_t block, F&& f) {
    const int64_t rows = part_rows_count(height, part, nparts, block);
    for (int64_t j = 0; j < rows; j += block)
        f(j, frame_row_of(j, part, nparts, block), rows - j < block ? rows - j : (int64_t)block);
}

}  // namespace rr
