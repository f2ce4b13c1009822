// multi.cpp — multi-device render contexts: cost-balanced row bands received straight into rank 0's frame (the
// default, ABI 10), or row-interleaved tiles through a staging buffer placed into frame order on rank 0
// (RR_PART_INTERLEAVE).
//
// Camera::render (camera.rs:107-121) spreads one frame over every rayon worker; here one frame is spread over GPUs.
// Bands (default): global rank r renders the output rows [bands[r], bands[r + 1]) as an f64 AA-averaged tile in its
// own HBM; the bounds balance the parts' render time (calibrate_bands, once per layout).  Inside one RCCL group per
// frame every other rank sends its tile to rank 0 in one ncclSend (over xGMI), which rank 0 receives straight into
// the frame's rows (one ncclRecv per part), and rank 0 copies its own tile there: no staging buffer, no placement.
// Interleaved (RR_PART_INTERLEAVE): rank r renders the output rows {y : (y / block) % nranks == r}; every rank sends
// its whole tile to rank 0, which receives each part's tile — its own included, as a send to itself — back to back
// into a staging buffer of `height` rows (part p at partition.hpp stage_row_offset(p)); one copy kernel per part then
// places the tile's runs into their frame rows (frame_row_of).  Either way two tile buffers alternate so that
// rendering frame k+1 overlaps the transfer of frame k (a render waits only for the transfer that last read its
// buffer), and each part alternates between two render contexts (scene copy + workspace) on two render streams.
//
// Three shapes of the same group: rr_create_multi (this process drives n devices, ncclCommInitAll,
// ncclGroupStart/End around every device's operations), rr_create_rank (one process per GPU, ncclCommInitRank
// from an id made by rr_rccl_unique_id on rank 0 and shared by the host) and rr_create_virtual (every part on one
// device, no communicator): a virtual group runs the same tiles, bands, offsets and placement kernels, with a
// device-local copy of each tile into its frame rows (interleaved: its stage rows) standing in for the send /
// receive pair.
#include "multi.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "device_guard.hpp"
#include "kernels.hpp"
#include "partition.hpp"
#include "trace.hpp"

void rr_set_error(const char* msg);  // api.cpp

namespace {

int gfail(int code, const std::string& msg) {
    rr_set_error(msg.c_str());
    return code;
}
#define GHIP(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return gfail(RR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define GNCCL(expr)                                                                             \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess) return gfail(RR_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

struct DevMem {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(want, 256));
        if (e == hipSuccess) bytes = std::max<size_t>(want, 256);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// A tile's rows in the staging buffer -> their frame rows (partition.hpp frame_row_of), on the root after the
// transfer.  One thread per double; both sides are contiguous along a row.
__global__ void __launch_bounds__(256) place_tile_kernel(const double* __restrict__ tile, double* __restrict__ out,
                                                         int64_t row_len, int64_t rows, int32_t part, int32_t nparts,
                                                         int32_t block) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= row_len * rows) return;
    const int64_t j = i / row_len, x = i - j * row_len;
    out[rr::frame_row_of(j, part, nparts, block) * row_len + x] = tile[i];
}

hipError_t launch_place_tile(const double* tile, double* out, int64_t W, int64_t rows, int32_t part, int32_t nparts,
                             int32_t block, hipStream_t st) {
    const int64_t n = W * 3 * rows;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(place_tile_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, tile, out, W * 3, rows,
                       part, nparts, block);
    return hipGetLastError();
}

}  // namespace

struct rr_group {
    int nranks = 1, rank0 = 0;
    std::vector<int> devices;
    std::vector<rr_ctx*> subs[2];         // per local part: frame k renders on subs[k % 2] / render_st[k % 2]
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> render_st[2], comm_st;
    std::vector<hipEvent_t> ev_rendered[2], ev_gathered[2];
    bool virt = false;                    // rr_create_virtual: every part on one device, send/recv = local copies
    int fail_after = -1;                  // fault injection for the drain tests (RRAY_TEST_FAIL_AFTER_PART): the call
                                          // fails once this local part's render is enqueued
    hipEvent_t ev_caller = nullptr;       // root: the caller's stream position at the gather call
    std::vector<DevMem> tile[2];          // per local part: its tile (rows of the part, in tile order)
    DevMem frame;                         // root: assembled frame for the blocking rr_render
    DevMem stage;                         // root: every part's tile back to back (part p at stage_row_offset(p))
    // band partition (the default): rank p renders output rows [bands[p], bands[p + 1]); calibrated on the first band
    // frame of a layout (calibrate_bands) or imposed by rr_group_set_bands
    std::vector<int64_t> bands;
    int64_t band_w = -1, band_h = -1;     // the layout the bands were made for
    int32_t band_aa = -1;
    DevMem dbounds;                       // rank processes: the bounds' device copy for the broadcast
    int64_t k = 0;                        // frames issued (buffer and render context = k % 2)
    int nlocal() const { return (int)devices.size(); }
    int last() const { return k > 0 ? (int)((k - 1) & 1) : 0; }  // the set that rendered the latest frame
    bool root_here() const { return rank0 == 0; }
    // the stream that transfers part l's tile (and releases its buffer): its own comm stream, or for a
    // virtual group the root's, where the copies into the frame run
    hipStream_t gather_stream(int l) const { return virt ? comm_st[0] : comm_st[l]; }
};

namespace rr {

static int group_setup(rr_group* g) {
    const int n = (int)g->devices.size();
    if (const char* f = std::getenv("RRAY_TEST_FAIL_AFTER_PART")) g->fail_after = std::atoi(f);
    g->comm_st.assign(n, nullptr);
    for (int b = 0; b < 2; ++b) {
        g->subs[b].assign(n, nullptr);
        g->render_st[b].assign(n, nullptr);
        g->ev_rendered[b].assign(n, nullptr);
        g->ev_gathered[b].assign(n, nullptr);
        g->tile[b].resize(n);
    }
    for (int l = 0; l < n; ++l) {
        for (int b = 0; b < 2; ++b) {
            int rc = rr_create(g->devices[l], &g->subs[b][l]);
            if (rc != RR_OK) return rc;
        }
        GHIP(hipSetDevice(g->devices[l]));
        for (int b = 0; b < 2; ++b) GHIP(hipStreamCreateWithFlags(&g->render_st[b][l], hipStreamNonBlocking));
        GHIP(hipStreamCreateWithFlags(&g->comm_st[l], hipStreamNonBlocking));
        for (int b = 0; b < 2; ++b) {
            GHIP(hipEventCreateWithFlags(&g->ev_rendered[b][l], hipEventDisableTiming));
            GHIP(hipEventCreateWithFlags(&g->ev_gathered[b][l], hipEventDisableTiming));
        }
    }
    if (g->root_here()) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipEventCreateWithFlags(&g->ev_caller, hipEventDisableTiming));
    }
    return RR_OK;
}

int group_create_local(int n, const int* ids, rr_group** out) {
    DeviceGuard device_guard;
    if (!out || n < 1 || !ids) return gfail(RR_E_ARG, "rr_create_multi: need n >= 1 device ids");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return gfail(RR_E_HIP, "no HIP device available");
    for (int i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= count) return gfail(RR_E_ARG, "device index out of range");
        for (int j = 0; j < i; ++j)
            if (ids[j] == ids[i]) return gfail(RR_E_ARG, "rr_create_multi: device ids must be distinct");
    }
    rr_group* g = new rr_group();
    g->nranks = n;
    g->rank0 = 0;
    g->devices.assign(ids, ids + n);
    int rc = group_setup(g);
    if (rc == RR_OK) {
        g->comms.assign(n, nullptr);
        ncclResult_t r = ncclCommInitAll(g->comms.data(), n, ids);
        if (r != ncclSuccess) {
            g->comms.clear();
            rc = gfail(RR_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
    }
    if (rc != RR_OK) {
        std::string msg = rr_last_error();
        group_destroy(g);
        return gfail(rc, msg);
    }
    *out = g;
    return RR_OK;
}

int group_create_rank(int device, int nranks, int rank, const uint8_t* unique_id, rr_group** out) {
    DeviceGuard device_guard;
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || !unique_id)
        return gfail(RR_E_ARG, "rr_create_rank: need 0 <= rank < nranks and an RCCL unique id");
    *out = nullptr;
    rr_group* g = new rr_group();
    g->nranks = nranks;
    g->rank0 = rank;
    g->devices.assign(1, device);
    int rc = group_setup(g);
    if (rc == RR_OK) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        g->comms.assign(1, nullptr);
        (void)hipSetDevice(device);
        ncclResult_t r = ncclCommInitRank(&g->comms[0], nranks, id, rank);
        if (r != ncclSuccess) {
            g->comms.clear();
            rc = gfail(RR_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
    }
    if (rc != RR_OK) {
        std::string msg = rr_last_error();
        group_destroy(g);
        return gfail(rc, msg);
    }
    *out = g;
    return RR_OK;
}

int group_create_virtual(int device, int nparts, rr_group** out) {
    DeviceGuard device_guard;
    if (!out || nparts < 1) return gfail(RR_E_ARG, "rr_create_virtual: need nparts >= 1");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return gfail(RR_E_HIP, "no HIP device available");
    if (device < 0 || device >= count) return gfail(RR_E_ARG, "device index out of range");
    rr_group* g = new rr_group();
    g->nranks = nparts;
    g->rank0 = 0;
    g->virt = true;
    g->devices.assign(nparts, device);  // one context (scene copy, workspace, streams) per part
    int rc = group_setup(g);
    if (rc != RR_OK) {
        std::string msg = rr_last_error();
        group_destroy(g);
        return gfail(rc, msg);
    }
    *out = g;
    return RR_OK;
}

// Waits for a stream to drain.  A stream that is still busy after 30 s is named on stderr (once) before the wait
// goes on: work still enqueued at teardown means an earlier call returned without draining it, or a kernel
// that does not end — either way the name says which part and stream, where a bare hang would not (DESIGN.md §5,
// the round-4 teardown hang).
static void drain_stream(hipStream_t st, const char* what, size_t part, int set) {
    if (!st) return;
    const auto t0 = std::chrono::steady_clock::now();
    bool told = false;
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) {  // done, or failed (then nothing more completes on it)
            if (e != hipSuccess) trace("drain: %s stream of part %zu (set %d): %s", what, part, set, hipGetErrorString(e));
            return;
        }
        if (!told && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
            std::fprintf(stderr, "rray: group teardown: %s stream of part %zu (set %d) still busy after 30 s\n", what,
                         part, set);
            trace("drain: %s stream of part %zu (set %d) still busy after 30 s", what, part, set);
            told = true;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// Every stream of the group drained: the render streams of both sets and the transfer streams.
static void group_drain(rr_group* g) {
    for (size_t l = 0; l < g->devices.size(); ++l) {
        (void)hipSetDevice(g->devices[l]);
        for (int b = 0; b < 2; ++b)
            if (l < g->render_st[b].size()) drain_stream(g->render_st[b][l], "render", l, b);
        if (l < g->comm_st.size()) drain_stream(g->comm_st[l], "transfer", l, -1);
    }
}

void group_destroy(rr_group* g) {
    DeviceGuard device_guard;
    if (!g) return;
    trace("group_destroy %p: %d parts, %lld frames; drain", (void*)g, g->nlocal(), (long long)g->k);
    group_drain(g);
    trace("group_destroy %p: drained", (void*)g);
    for (ncclComm_t c : g->comms)
        if (c) (void)ncclCommDestroy(c);
    // the parts' render contexts first, then the group's streams: a context waits only on its own event (rr_ctx::ev_out,
    // recorded after each call's work) and never touches a stream after its call returns, but destroying the contexts
    // while the streams still exist keeps the teardown order obviously safe (the round-4 hang)
    for (int b = 0; b < 2; ++b)
        for (size_t l = 0; l < g->subs[b].size(); ++l)
            if (g->subs[b][l]) {
                trace("group_destroy %p: context of part %zu set %d", (void*)g, l, b);
                rr_destroy(g->subs[b][l]);
                g->subs[b][l] = nullptr;
            }
    trace("group_destroy %p: contexts destroyed", (void*)g);
    for (size_t l = 0; l < g->devices.size(); ++l) {
        (void)hipSetDevice(g->devices[l]);
        for (int b = 0; b < 2; ++b) {
            if (l < g->tile[b].size()) g->tile[b][l].release();
            if (l < g->ev_rendered[b].size() && g->ev_rendered[b][l]) (void)hipEventDestroy(g->ev_rendered[b][l]);
            if (l < g->ev_gathered[b].size() && g->ev_gathered[b][l]) (void)hipEventDestroy(g->ev_gathered[b][l]);
        }
        for (int b = 0; b < 2; ++b)
            if (l < g->render_st[b].size() && g->render_st[b][l]) (void)hipStreamDestroy(g->render_st[b][l]);
        if (l < g->comm_st.size() && g->comm_st[l]) (void)hipStreamDestroy(g->comm_st[l]);
        if (l == 0) g->dbounds.release();
        if (l == 0 && g->root_here()) {
            g->frame.release();
            g->stage.release();
            if (g->ev_caller) (void)hipEventDestroy(g->ev_caller);
        }
    }
    trace("group_destroy %p: done", (void*)g);
    delete g;
}

int group_upload(rr_group* g, const rr_scene_desc* d) {
    DeviceGuard device_guard;
    for (int l = 0; l < g->nlocal(); ++l) {  // the scene is replicated to every device (<= a few MB), per render context
        GHIP(hipSetDevice(g->devices[l]));
        for (int b = 0; b < 2; ++b) GHIP(hipStreamSynchronize(g->render_st[b][l]));
        GHIP(hipStreamSynchronize(g->comm_st[l]));
        for (int b = 0; b < 2; ++b) {
            int rc = rr_scene_upload(g->subs[b][l], d);
            if (rc != RR_OK) return rc;
        }
    }
    return RR_OK;
}

// Enqueues one frame: every local part's render into its tile buffer of set b, the transfer into the staging
// buffer (RCCL send / receive pairs, or a virtual group's device copies) and, on the root, the placement kernels
// into `frame`.  `enqueued` turns true with the first enqueued operation: the caller drains the group when this
// returns an error after that point, so no work outlives a failed call.
static int enqueue_frame(rr_group* g, const rr_camera* cam, const std::vector<rr_render_opts>& opts, double* frame,
                         hipStream_t caller, int64_t W, int64_t H, int32_t block, int b, bool& enqueued) {
    const int n = g->nlocal();
    const int64_t row = W * 3;
    for (int l = 0; l < n; ++l) {
        GHIP(hipSetDevice(g->devices[l]));
        // the transfer that last read this buffer (two frames ago) must be done before it is overwritten; the
        // render context and stream of set b are free once that frame's render is (same stream)
        GHIP(hipStreamWaitEvent(g->render_st[b][l], g->ev_gathered[b][l], 0));
        enqueued = true;
        int rc = rr_render_device(g->subs[b][l], cam, &opts[l], nullptr, g->tile[b][l].p, g->render_st[b][l]);
        if (rc != RR_OK) return rc;
        if (l == g->fail_after) return gfail(RR_E_HIP, "injected failure after part " + std::to_string(l) + "'s render");
        GHIP(hipEventRecord(g->ev_rendered[b][l], g->render_st[b][l]));
        GHIP(hipStreamWaitEvent(g->gather_stream(l), g->ev_rendered[b][l], 0));
    }
    double* stage = g->root_here() ? static_cast<double*>(g->stage.p) : nullptr;
    if (g->virt) {
        // the send / receive pairs of a real group, as device-local copies: part l's tile into its stage rows, on
        // the root's transfer stream (where the receives run)
        GHIP(hipSetDevice(g->devices[0]));
        for (int l = 0; l < n; ++l) {
            const int64_t rows = part_rows_count(H, l, g->nranks, block);
            if (rows > 0)
                GHIP(hipMemcpyAsync(stage + stage_row_offset(H, l, g->nranks, block) * row, g->tile[b][l].p,
                                    (size_t)(rows * row) * sizeof(double), hipMemcpyDeviceToDevice, g->comm_st[0]));
        }
    } else {
        // one RCCL group per frame: each local part sends its whole tile to rank 0 in one ncclSend, and rank 0
        // receives every part's tile (its own from itself) into its stage rows.  One operation per part: the round-4
        // first cut posted one send / receive per 8-row run (270 per C3 frame on rank 0), and the per-operation cost
        // made the one-rank group's frame 1.49 ms slower than the single render (7.83 vs 6.34 ms).  The group is
        // always closed, also when posting an operation fails.
        ncclResult_t r = ncclGroupStart();
        if (r == ncclSuccess) {
            for (int l = 0; l < n && r == ncclSuccess; ++l) {
                const int64_t rows = part_rows_count(H, g->rank0 + l, g->nranks, block);
                if (rows > 0)
                    r = ncclSend(g->tile[b][l].p, (size_t)(rows * row), ncclFloat64, 0, g->comms[l], g->comm_st[l]);
                if (!(g->root_here() && l == 0)) continue;
                for (int32_t p = 0; p < g->nranks && r == ncclSuccess; ++p) {
                    const int64_t pr = part_rows_count(H, p, g->nranks, block);
                    if (pr > 0)
                        r = ncclRecv(stage + stage_row_offset(H, p, g->nranks, block) * row, (size_t)(pr * row),
                                     ncclFloat64, p, g->comms[0], g->comm_st[0]);
                }
            }
            const ncclResult_t e = ncclGroupEnd();
            if (r == ncclSuccess) r = e;
        }
        if (r != ncclSuccess) return gfail(RR_E_HIP, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    }
    if (g->root_here()) {
        GHIP(hipSetDevice(g->devices[0]));
        // d_frame is written in the caller's stream order: only the placement waits for it (the receives into the
        // private stage do not, so peers' sends never wait on unrelated caller work)
        if (caller) GHIP(hipStreamWaitEvent(g->comm_st[0], g->ev_caller, 0));
        for (int32_t p = 0; p < g->nranks; ++p)
            GHIP(launch_place_tile(stage + stage_row_offset(H, p, g->nranks, block) * row, frame, W,
                                   part_rows_count(H, p, g->nranks, block), p, g->nranks, block, g->comm_st[0]));
    }
    for (int l = 0; l < n; ++l) {  // a virtual group's tiles are all read on comm_st[0]
        GHIP(hipSetDevice(g->devices[l]));
        GHIP(hipEventRecord(g->ev_gathered[b][l], g->gather_stream(l)));
    }
    if (g->root_here() && caller) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipStreamWaitEvent(caller, g->ev_gathered[b][0], 0));
    }
    return RR_OK;
}

// Cost-balanced bands for this layout.  Rank 0 measures the frame's cost per row on its own device: the frame as 16
// bands of equal height (multiples of 8 rows), each rendered three times on one context and the third render timed
// with events (the first renders of a layout build its camera bundles and run in a guessed wave order; a part renders
// its band over and over), which gives a per-row profile; rr_balance_bands cuts it into N bands, with rank 0's own
// transfer work added to its band (a device copy of the frame, timed: rank 0 writes the other parts' incoming rows and
// copies its own, beside its render).  Two refinements then time each of the N bands the same way and rescale the
// profile inside it to the measured time before cutting again: 16 equal bands are not additive (a band's time is not
// the sum of its rows' shares: launch tails, and the cost order of a small launch), the N bands are what the parts
// will render.  A process group gets the bounds from rank 0 by one ncclBroadcast — the only collective besides the
// frames' transfers, once per layout.  Every rank calls this for the same frame (the layout is an argument every rank
// passes alike).
static int calibrate_bands(rr_group* g, const rr_camera* cam, const rr_render_opts* o, int64_t W, int64_t H) {
    const int N = g->nranks;
    const int64_t row = W * 3;
    std::vector<int64_t> b(N + 1, 0);
    group_drain(g);  // a layout change: nothing of the previous frames may still use the buffers below
    if (g->root_here()) {
        GHIP(hipSetDevice(g->devices[0]));
        rr_ctx* c = g->subs[0][0];
        hipStream_t st = g->render_st[0][0];
        GHIP(g->stage.ensure((size_t)H * (size_t)row * sizeof(double)));
        GHIP(g->frame.ensure((size_t)H * (size_t)row * sizeof(double)));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        GHIP(hipEventCreate(&e0));
        GHIP(hipEventCreate(&e1));
        // rows [y0, y1): three renders, the third timed
        const auto time_band = [&](int64_t y0, int64_t y1, float& ms) -> int {
            rr_render_opts so = *o;
            so.part = 0;
            so.nparts = 1;
            so.row_begin = (int32_t)y0;
            so.row_end = (int32_t)y1;
            so.flags = RR_OUT_AVG | RR_NO_FRAME_TIMING;
            double* out = static_cast<double*>(g->stage.p) + y0 * row;
            for (int k = 0; k < 3; ++k) {
                if (k == 2) GHIP(hipEventRecord(e0, st));
                int rc = rr_render_device(c, cam, &so, nullptr, out, st);
                if (rc != RR_OK) return rc;
            }
            GHIP(hipEventRecord(e1, st));
            GHIP(hipEventSynchronize(e1));
            GHIP(hipEventElapsedTime(&ms, e0, e1));
            return RR_OK;
        };
        int rc = RR_OK;
        std::vector<double> cost(H, 0.0);
        const int64_t nb = std::min<int64_t>(16, (H + 7) / 8);
        const int64_t hb = ((H + nb - 1) / nb + 7) / 8 * 8;
        for (int64_t y0 = 0; y0 < H && rc == RR_OK; y0 += hb) {
            const int64_t y1 = std::min<int64_t>(H, y0 + hb);
            float ms = 0.0f;
            rc = time_band(y0, y1, ms);
            for (int64_t y = y0; y < y1; ++y) cost[y] = (double)ms / (double)(y1 - y0);
        }
        double extra = 0.0;
        if (rc == RR_OK && N > 1) {
            float copy_ms = 0.0f;
            GHIP(hipEventRecord(e0, st));
            GHIP(hipMemcpyAsync(g->frame.p, g->stage.p, (size_t)H * (size_t)row * sizeof(double), hipMemcpyDeviceToDevice,
                                st));
            GHIP(hipEventRecord(e1, st));
            GHIP(hipEventSynchronize(e1));
            GHIP(hipEventElapsedTime(&copy_ms, e0, e1));
            // a copy reads and writes every byte: the incoming (N - 1) / N of the frame is written once, the own band
            // (about 1 / N of it) read and written
            extra = (double)copy_ms * (0.5 * (double)(N - 1) / N + 1.0 / N);
        }
        if (rc == RR_OK) balance_bands(cost.data(), H, N, extra, 8, b.data());
        for (int it = 0; it < 2 && rc == RR_OK && N > 1; ++it) {
            for (int p = 0; p < N && rc == RR_OK; ++p) {
                if (b[p + 1] <= b[p]) continue;
                float ms = 0.0f;
                rc = time_band(b[p], b[p + 1], ms);
                double sum = 0.0;
                for (int64_t y = b[p]; y < b[p + 1]; ++y) sum += cost[y];
                if (rc == RR_OK && sum > 0.0)
                    for (int64_t y = b[p]; y < b[p + 1]; ++y) cost[y] *= (double)ms / sum;
            }
            if (rc == RR_OK) balance_bands(cost.data(), H, N, extra, 8, b.data());
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (rc != RR_OK) return rc;
        trace("calibrate_bands %p: %lld x %lld, %d parts, band 0 = %lld rows, extra %.4f ms", (void*)g, (long long)W,
              (long long)H, N, (long long)b[1], extra);
    }
    if (!g->virt && g->nlocal() < N) {  // one process per GPU: rank 0's bounds to every rank
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(g->dbounds.ensure((size_t)(N + 1) * sizeof(int64_t)));
        if (g->root_here())
            GHIP(hipMemcpy(g->dbounds.p, b.data(), (size_t)(N + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
        GNCCL(ncclBroadcast(g->dbounds.p, g->dbounds.p, (size_t)(N + 1), ncclInt64, 0, g->comms[0], g->comm_st[0]));
        GHIP(hipStreamSynchronize(g->comm_st[0]));
        GHIP(hipMemcpy(b.data(), g->dbounds.p, (size_t)(N + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    }
    g->bands = b;
    g->band_w = W;
    g->band_h = H;
    g->band_aa = o->aa;
    return RR_OK;
}

// One band frame: every local part renders its band into its tile buffer; rank 0 receives the other parts' tiles
// straight into their frame rows (one ncclRecv per part) and copies its own there; a virtual group copies every
// tile into its rows on the root's transfer stream in place of the send / receive pairs.  `enqueued` as enqueue_frame.
static int enqueue_frame_bands(rr_group* g, const rr_camera* cam, const std::vector<rr_render_opts>& opts, double* frame,
                               hipStream_t caller, int64_t W, int b, bool& enqueued) {
    const int n = g->nlocal();
    const int64_t row = W * 3;
    const auto rows_of = [&](int p) { return g->bands[p + 1] - g->bands[p]; };
    for (int l = 0; l < n; ++l) {
        GHIP(hipSetDevice(g->devices[l]));
        GHIP(hipStreamWaitEvent(g->render_st[b][l], g->ev_gathered[b][l], 0));
        enqueued = true;
        if (rows_of(g->rank0 + l) > 0) {
            int rc = rr_render_device(g->subs[b][l], cam, &opts[l], nullptr, g->tile[b][l].p, g->render_st[b][l]);
            if (rc != RR_OK) return rc;
        }
        if (l == g->fail_after) return gfail(RR_E_HIP, "injected failure after part " + std::to_string(l) + "'s render");
        GHIP(hipEventRecord(g->ev_rendered[b][l], g->render_st[b][l]));
        GHIP(hipStreamWaitEvent(g->gather_stream(l), g->ev_rendered[b][l], 0));
    }
    if (g->root_here()) {
        GHIP(hipSetDevice(g->devices[0]));
        // the frame is written in the caller's stream order: the copies and receives into it wait for the caller
        if (caller) GHIP(hipStreamWaitEvent(g->comm_st[0], g->ev_caller, 0));
    }
    if (g->virt) {
        GHIP(hipSetDevice(g->devices[0]));
        for (int l = 0; l < n; ++l)
            if (rows_of(l) > 0)
                GHIP(hipMemcpyAsync(frame + g->bands[l] * row, g->tile[b][l].p, (size_t)(rows_of(l) * row) * sizeof(double),
                                    hipMemcpyDeviceToDevice, g->comm_st[0]));
    } else {
        if (g->root_here() && rows_of(0) > 0) {
            GHIP(hipSetDevice(g->devices[0]));
            GHIP(hipMemcpyAsync(frame, g->tile[b][0].p, (size_t)(rows_of(0) * row) * sizeof(double), hipMemcpyDeviceToDevice,
                                g->comm_st[0]));
        }
        ncclResult_t r = ncclGroupStart();
        if (r == ncclSuccess) {
            for (int l = 0; l < n && r == ncclSuccess; ++l) {
                const int p = g->rank0 + l;
                if (p != 0 && rows_of(p) > 0)
                    r = ncclSend(g->tile[b][l].p, (size_t)(rows_of(p) * row), ncclFloat64, 0, g->comms[l], g->comm_st[l]);
                if (!(g->root_here() && l == 0)) continue;
                for (int32_t q = 1; q < g->nranks && r == ncclSuccess; ++q)
                    if (rows_of(q) > 0)
                        r = ncclRecv(frame + g->bands[q] * row, (size_t)(rows_of(q) * row), ncclFloat64, q, g->comms[0],
                                     g->comm_st[0]);
            }
            const ncclResult_t e = ncclGroupEnd();
            if (r == ncclSuccess) r = e;
        }
        if (r != ncclSuccess) return gfail(RR_E_HIP, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    }
    for (int l = 0; l < n; ++l) {  // a virtual group's tiles are all read on comm_st[0]
        GHIP(hipSetDevice(g->devices[l]));
        GHIP(hipEventRecord(g->ev_gathered[b][l], g->gather_stream(l)));
    }
    if (g->root_here() && caller) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipStreamWaitEvent(caller, g->ev_gathered[b][0], 0));
    }
    return RR_OK;
}

int group_bands(rr_group* g, int64_t* bounds, int32_t n) {
    if (g->bands.empty()) return 0;
    if (n < g->nranks + 1) return gfail(RR_E_ARG, "rr_group_bands: need nranks + 1 values");
    std::copy(g->bands.begin(), g->bands.end(), bounds);
    return g->nranks + 1;
}

int group_set_bands(rr_group* g, const int64_t* bounds, int32_t n) {
    if (n != g->nranks + 1) return gfail(RR_E_ARG, "rr_group_set_bands: need nranks + 1 bounds");
    if (bounds[0] != 0) return gfail(RR_E_ARG, "rr_group_set_bands: bounds[0] must be 0");
    for (int32_t p = 0; p < g->nranks; ++p)
        if (bounds[p + 1] < bounds[p]) return gfail(RR_E_ARG, "rr_group_set_bands: bounds must not decrease");
    group_drain(g);
    g->bands.assign(bounds, bounds + n);
    g->band_h = bounds[n - 1];
    g->band_w = 0;  // any width and aa of that height (checked per frame)
    g->band_aa = 0;
    return RR_OK;
}

int group_render_gather(rr_group* g, const rr_camera* cam, const rr_render_opts* o, void* d_frame, void* stream) {
    DeviceGuard device_guard;
    if (!cam || !o) return gfail(RR_E_ARG, "null camera/options");
    if (o->nparts != 1 || o->part != 0 || o->row_begin != 0 || o->row_end != 0)
        return gfail(RR_E_ARG, "a multi-device context splits the whole frame itself: pass part 0 of 1, no band");
    if (o->flags & (RR_OUT_CANVAS | RR_OUT_AVG_F32))
        return gfail(RR_E_ARG, "multi-device contexts produce the f64 AA-averaged image only (RR_OUT_AVG)");
    if (o->aa < 1 || cam->hsize <= 0 || cam->vsize <= 0 || cam->hsize % o->aa || cam->vsize % o->aa)
        return gfail(RR_E_ARG, "camera size must be a positive multiple of aa");
    if (g->root_here() && !d_frame) return gfail(RR_E_ARG, "rank 0 needs a device frame buffer");
    const int32_t block = o->block_rows > 0 ? o->block_rows : 8;
    const int64_t W = cam->hsize / o->aa, H = cam->vsize / o->aa, row = W * 3;
    const int b = (int)(g->k & 1);
    const int n = g->nlocal();
    const bool interleave = (o->flags & RR_PART_INTERLEAVE) != 0;
    if (!interleave && (g->bands.empty() || g->band_h != H ||
                        (g->band_w != 0 && (g->band_w != W || g->band_aa != o->aa)))) {
        int rc = calibrate_bands(g, cam, o, W, H);
        if (rc != RR_OK) return rc;
    }
    // every part's options and buffers are checked / allocated before any work is enqueued: a failure
    // here returns before this rank joins the collective, never between its render and its transfer
    std::vector<rr_render_opts> opts(n, *o);
    for (int l = 0; l < n; ++l) {
        rr_render_opts& so = opts[l];
        const int p = g->rank0 + l;
        int64_t rows;
        if (interleave) {
            so.part = p;
            so.nparts = g->nranks;
            so.block_rows = block;
            rows = part_rows_count(H, so.part, g->nranks, block);
        } else {  // the band [bands[p], bands[p + 1])
            so.part = 0;
            so.nparts = 1;
            so.block_rows = block;
            so.row_begin = (int32_t)g->bands[p];
            so.row_end = (int32_t)g->bands[p + 1];
            rows = g->bands[p + 1] - g->bands[p];
        }
        so.flags = RR_OUT_AVG | (o->flags & RR_NO_FRAME_TIMING);
        if (rows > 0) {
            int rc = render_validate(g->subs[b][l], cam, &so);
            if (rc != RR_OK) return rc;
        }
        GHIP(hipSetDevice(g->devices[l]));
        GHIP(g->tile[b][l].ensure((size_t)rows * (size_t)row * sizeof(double)));
    }
    if (g->root_here() && interleave) {  // the staging buffer (the whole frame's rows), before any work is enqueued
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(g->stage.ensure((size_t)H * (size_t)row * sizeof(double)));
    }
    hipStream_t caller = g->root_here() ? (hipStream_t)stream : nullptr;
    if (caller) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipEventRecord(g->ev_caller, caller));
    }
    bool enqueued = false;
    trace("group_render_gather %p: frame %lld, %d parts, %lld x %lld, block %d", (void*)g, (long long)g->k, n,
          (long long)W, (long long)H, block);
    const int rc = interleave ? enqueue_frame(g, cam, opts, static_cast<double*>(d_frame), caller, W, H, block, b, enqueued)
                              : enqueue_frame_bands(g, cam, opts, static_cast<double*>(d_frame), caller, W, b, enqueued);
    if (rc != RR_OK) {
        trace("group_render_gather %p: error %d after %s: %s", (void*)g, rc, enqueued ? "enqueuing" : "no work",
              rr_last_error());
        if (enqueued) {  // drain what this call enqueued before reporting: nothing of a failed frame stays in flight
            const std::string msg = rr_last_error();
            group_drain(g);
            rr_set_error(msg.c_str());
        }
        return rc;
    }
    trace("group_render_gather %p: frame %lld enqueued", (void*)g, (long long)g->k);
    ++g->k;
    return RR_OK;
}

int group_render(rr_group* g, const rr_camera* cam, const rr_render_opts* o, double* out_canvas, double* out_avg,
                 rr_stats* stats) {
    DeviceGuard device_guard;
    if (!cam || !o) return gfail(RR_E_ARG, "null camera/options");
    if ((o->flags & RR_OUT_CANVAS) && out_canvas)
        return gfail(RR_E_ARG, "multi-device contexts produce the f64 AA-averaged image only (RR_OUT_AVG)");
    if (o->aa < 1 || cam->hsize <= 0 || cam->vsize <= 0 || cam->hsize % o->aa || cam->vsize % o->aa)
        return gfail(RR_E_ARG, "camera size must be a positive multiple of aa");
    const int64_t W = cam->hsize / o->aa, H = cam->vsize / o->aa;
    if (g->root_here()) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(g->frame.ensure((size_t)W * H * 3 * sizeof(double)));
    }
    rr_render_opts so = *o;
    so.flags = RR_OUT_AVG | (o->flags & RR_PART_INTERLEAVE);
    int rc = group_render_gather(g, cam, &so, g->root_here() ? g->frame.p : nullptr, nullptr);
    if (rc != RR_OK) return rc;
    trace("group_render %p: synchronise", (void*)g);
    for (int l = 0; l < g->nlocal(); ++l) {  // every stream synchronised: a failure here leaves nothing in flight either
        GHIP(hipSetDevice(g->devices[l]));
        for (int b = 0; b < 2; ++b) {
            const hipError_t e = hipStreamSynchronize(g->render_st[b][l]);
            if (e != hipSuccess) {
                group_drain(g);
                return gfail(RR_E_HIP, std::string("hipStreamSynchronize(render): ") + hipGetErrorString(e));
            }
        }
        const hipError_t e = hipStreamSynchronize(g->comm_st[l]);
        if (e != hipSuccess) {
            group_drain(g);
            return gfail(RR_E_HIP, std::string("hipStreamSynchronize(transfer): ") + hipGetErrorString(e));
        }
    }
    if (g->root_here() && out_avg && (o->flags & RR_OUT_AVG)) {
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipMemcpy(out_avg, g->frame.p, (size_t)W * H * 3 * sizeof(double), hipMemcpyDeviceToHost));
    }
    trace("group_render %p: synchronised", (void*)g);
    rr_stats local;
    rc = group_last_stats(g, stats ? stats : &local);
    if (rc != RR_OK) return rc;
    const uint64_t nan = (stats ? stats : &local)->nan_rays;
    if (nan)
        return gfail(RR_E_NAN, std::to_string(nan) + " ray(s) met a NaN intersection t in a list of >= 2 entries "
                                                     "(the reference panics in sort_by, scene.rs:104)");
    return RR_OK;
}

int group_last_stats(rr_group* g, rr_stats* s) {
    if (!s) return gfail(RR_E_ARG, "null stats");
    std::memset(s, 0, sizeof(*s));
    for (rr_ctx* c : g->subs[g->last()]) {  // the latest frame's contexts, summed over this process's devices
        rr_stats t;
        int rc = rr_last_stats(c, &t);
        if (rc != RR_OK) return rc;
        s->rays += t.rays;
        s->shadow_rays += t.shadow_rays;
        s->shade_events += t.shade_events;
        s->n1n2_scans += t.n1n2_scans;
        s->group_tests += t.group_tests;
        s->group_hits += t.group_hits;
        s->samples += t.samples;
        s->prim_tests += t.prim_tests;
        s->kernel_ms = std::max(s->kernel_ms, t.kernel_ms);
        s->nan_rays += t.nan_rays;
        for (int k = 0; k < 3; ++k) {
            s->exact_flops[k] += t.exact_flops[k];
            s->wave_visits[k] += t.wave_visits[k];
        }
    }
    return RR_OK;
}

rr_ctx* group_local(rr_group* g, int l) { return (l >= 0 && l < g->nlocal()) ? g->subs[0][l] : nullptr; }

// per-launch kernel timing on local part 0: both render contexts (their launches alternate by frame)
int group_kernel_profile(rr_group* g, int enable) {
    for (int b = 0; b < 2; ++b) {
        int rc = rr_kernel_profile(g->subs[b][0], enable);
        if (rc != RR_OK) return rc;
    }
    return RR_OK;
}
int group_kernel_times(rr_group* g, double* ms, uint64_t* launches, int32_t n) {
    std::vector<double> m2(n > 0 ? n : 0, 0.0);
    std::vector<uint64_t> l2(n > 0 ? n : 0, 0);
    int rc = rr_kernel_times(g->subs[0][0], ms, launches, n);
    if (rc < 0) return rc;
    rc = rr_kernel_times(g->subs[1][0], m2.data(), l2.data(), n);
    if (rc < 0) return rc;
    for (int k = 0; k < n && k < rc; ++k) {
        if (ms) ms[k] += m2[k];
        if (launches) launches[k] += l2[k];
    }
    return rc;
}

int group_info(const rr_group* g, int32_t* nranks, int32_t* rank0, int32_t* nlocal) {
    if (nranks) *nranks = g->nranks;
    if (rank0) *rank0 = g->rank0;
    if (nlocal) *nlocal = (int32_t)g->nlocal();
    return RR_OK;
}

}  // namespace rr

extern "C" int rr_rccl_unique_id(uint8_t* out, int32_t n) {
    if (!out || n < (int32_t)sizeof(ncclUniqueId)) return gfail(RR_E_ARG, "rr_rccl_unique_id: need RR_RCCL_ID_BYTES bytes");
    ncclUniqueId id;
    GNCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return RR_OK;
}
