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

// Cost-balanced contiguous bands (the multi-device default, multi.cpp): bounds[0] = 0 <= ... <= bounds[nparts] =
// height such that part p's cost — the sum of row_cost over its rows, plus root_extra for part 0 (rank 0's transfer
// work, which runs beside its render) — is as even as `align` allows.  Each inner bound is the row where the
// cumulative cost (root_extra counted first) crosses p / nparts of the total, interpolated within the row and rounded
// to the nearest multiple of align, kept monotone.  Host only.
inline void balance_bands(const double* row_cost, int64_t height, int32_t nparts, double root_extra, int32_t align,
                          int64_t* bounds) {
    const auto cost = [&](int64_t y) { return row_cost[y] > 0.0 ? row_cost[y] : 0.0; };  // NaN and negatives count 0
    const double extra = root_extra > 0.0 ? root_extra : 0.0;
    double total = extra;
    for (int64_t y = 0; y < height; ++y) total += cost(y);
    bounds[0] = 0;
    int64_t y = 0;
    double acc = extra;  // cost of rows [0, y) plus the root's extra
    for (int32_t p = 1; p < nparts; ++p) {
        const double target = total * (double)p / (double)nparts;
        while (y < height && acc + cost(y) <= target) acc += cost(y++);
        // the crossing lies in row y: the fraction of it that completes the target
        double at = (double)y;
        if (y < height && cost(y) > 0.0) at += (target - acc) / cost(y);
        int64_t b = (int64_t)(at / align + 0.5) * align;
        if (b > height) b = height;
        if (b < bounds[p - 1]) b = bounds[p - 1];
        bounds[p] = b;
    }
    bounds[nparts] = height;
}

}  // namespace rr
