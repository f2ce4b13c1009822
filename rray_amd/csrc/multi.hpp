// multi.hpp — multi-device contexts (rray.h: rr_create_multi / rr_create_rank): one frame split in
// interleaved row blocks across devices, the f64 tiles gathered to global rank 0 with one RCCL
// gather over xGMI, un-interleaved there into frame order.  The reference renders one frame across
// all of its workers (camera.rs:107-121, rayon par_bridge); this spreads the same frame over GPUs.
#pragma once
#include <stdint.h>

#include "../../include/rray/rray.h"

struct rr_group;

namespace rr {

// Per local device the group owns two ordinary single-device contexts (frames alternate between them,
// DESIGN.md §5).  Global ranks rank0 .. rank0 + nlocal - 1 live in this process.
int group_create_local(int n, const int* device_ids, rr_group** out);
int group_create_rank(int device, int nranks, int rank, const uint8_t* unique_id, rr_group** out);
// nparts virtual ranks on one device (rr_create_virtual): the same tiles, buffers, streams, staging buffer and
// placement kernels as a real group, with each ncclSend / ncclRecv pair done by a device-local copy into rank 0's
// staging buffer (partition.hpp stage_row_offset)
int group_create_virtual(int device, int nparts, rr_group** out);
void group_destroy(rr_group* g);
int group_upload(rr_group* g, const rr_scene_desc* d);
int group_render_gather(rr_group* g, const rr_camera* cam, const rr_render_opts* o, void* d_frame, void* stream);
int group_render(rr_group* g, const rr_camera* cam, const rr_render_opts* o, double* out_canvas, double* out_avg,
                 rr_stats* stats);
int group_last_stats(rr_group* g, rr_stats* s);
rr_ctx* group_local(rr_group* g, int l);  // local device context l (0 = the lowest global rank here)
// rr_kernel_profile / rr_kernel_times for local part 0, over both of its render contexts
int group_kernel_profile(rr_group* g, int enable);
int group_kernel_times(rr_group* g, double* ms, uint64_t* launches, int32_t n);
int group_info(const rr_group* g, int32_t* nranks, int32_t* rank0, int32_t* nlocal);
// the band bounds (rr_group_bands / rr_group_set_bands)
int group_bands(rr_group* g, int64_t* bounds, int32_t n);
int group_set_bands(rr_group* g, const int64_t* bounds, int32_t n);
// api.cpp: every argument check of rr_render_device, without enqueueing anything
int render_validate(rr_ctx* c, const rr_camera* cam, const rr_render_opts* o);

}  // namespace rr
