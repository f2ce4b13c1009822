/*
 * rray.h — C ABI of the MI355X (gfx950) render path for davelpz/rray.
 *
 * Drop-in boundary for the reference's per-pixel render loop:
 *   Camera::render(&self, &Scene) -> Canvas        src/raytracer/camera.rs:107-121
 *     -> Scene::color_at / intersect / shade_hit / is_shadowed / reflected_color /
 *        refracted_color                           src/raytracer/scene.rs:97-336
 *     -> Object::intersect (+ local_intersect)     src/raytracer/object.rs:45-48
 * and its YAML/CLI front-end
 *   render_scene_from_file(path, w, h, png, aa)    src/raytracer/scene_builder_yaml.rs:429-436
 *
 * Everything is extern "C" with plain pointers and sizes so a Rust host binds it with
 * an `extern "C"` block.  Return codes: 0 = OK, < 0 = error
 * (the reference's panics, scene_builder_yaml.rs / db.rs, become codes); the message is
 * available from rr_last_error().  Never aborts or throws across the ABI.
 *
 * There is no CPU fallback: every render entry point runs the HIP kernels and fails with
 * RR_E_HIP when no gfx950 device is usable.
 */
#ifndef RRAY_RRAY_H
#define RRAY_RRAY_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RR_ABI_VERSION 10

/* error codes */
#define RR_OK 0
#define RR_E_ARG (-1)        /* invalid argument / inconsistent descriptor */
#define RR_E_HIP (-2)        /* HIP runtime error (no device, launch failure, ...) */
#define RR_E_SCENE (-3)      /* scene the reference would panic on (scene_builder_yaml.rs) */
#define RR_E_NONAFFINE (-4)  /* inverse transform with row 3 != (0,0,0,1) */
#define RR_E_LIMIT (-5)      /* exceeds a compiled limit (depth, pattern nesting) */
#define RR_E_IO (-6)         /* file missing / unreadable / unwritable */
#define RR_E_NAN (-7)        /* NaN intersection t in a list of >= 2 entries: the reference panics in
                                Vec::sort_by(partial_cmp().unwrap()) (scene.rs:104, group.rs:88, csg.rs:231).
                                rr_render / rr_color_at return it after writing their outputs; for
                                rr_render_device see rr_stats.nan_rays. */

/* object kinds — Sphere, Plane, Group, Triangle, SmoothTriangle, Cube, Cylinder, Cone, Csg, Torus
 * (src/raytracer/object/) */
enum { RR_SPHERE = 0, RR_PLANE = 1, RR_GROUP = 2, RR_TRIANGLE = 3, RR_SMOOTH_TRIANGLE = 4,
       RR_CUBE = 5, RR_CYLINDER = 6, RR_CONE = 7, RR_CSG = 8, RR_TORUS = 9 };
/* CSG operations — CsgOperation (csg.rs:13-17) */
enum { RR_CSG_UNION = 0, RR_CSG_INTERSECTION = 1, RR_CSG_DIFFERENCE = 2 };
/* pattern kinds — PatternType (src/raytracer/material/pattern.rs:10-21), in-scope subset */
enum { RR_PAT_TEST = 0, RR_PAT_SOLID = 1, RR_PAT_STRIPE = 2, RR_PAT_GRADIENT = 3,
       RR_PAT_RING = 4, RR_PAT_CHECKER = 5, RR_PAT_BLEND = 6, RR_PAT_PERTURBED = 7, RR_PAT_NOISE = 8,
       RR_PAT_TEXTURE = 9 /* pat_a = texture index */ };
/* light kinds — LightType (src/raytracer/light.rs:10-14) */
enum { RR_LIGHT_POINT = 0, RR_LIGHT_AREA = 1 };

#define RR_MAX_DEPTH 8          /* max `remaining` (render uses 5, camera.rs:113) */
#define RR_MAX_GROUP_DEPTH 6    /* nested group levels */
#define RR_MAX_AREA_LEVEL 1024  /* area light `level` (level^2 jittered samples per shading event; the
                                   reference takes any usize, scene_builder_yaml.rs:137).  Bound by the
                                   kernels' cell arithmetic: (col + u) / level is the proven shared-divisor
                                   quotient (tests/test_division.py, every level 1..1024) and the cell index
                                   s < level^2 <= 2^20 fits the jitter key's 20-bit field.  The YAML front-end
                                   and rr_scene_upload both refuse larger levels (RR_E_LIMIT / RR_E_SCENE). */
#define RR_MAX_PATTERN_DEPTH 8  /* nested pattern levels */
#define RR_MAX_CSG_ENTRIES 32   /* intersections one CSG subtree can produce for one ray */
#define RR_MAX_OCTAVES 64       /* octave_perlin octaves (noise.rs:11-29) */

/*
 * The scene exactly as the reference's object registry holds it (object/db.rs:11-13 +
 * Scene{light, ids}, scene.rs:24-27).  All arrays are caller-owned and copied by
 * rr_scene_upload.  Object ids index every per-object array.
 */
typedef struct {
    int32_t n_objects;
    const int32_t* kind;         /* RR_SPHERE.. per object */
    const int32_t* parent;       /* parent group id or -1 (Object::get_parent_id) */
    const double* transform;     /* n_objects x 16, row-major (Matrix.data, matrix.rs:20-25) */
    const double* inverse;       /* optional n_objects x 16; NULL: computed like matrix.rs:389-412 */
    const int32_t* material;     /* material index per object (ignored for groups) */
    const double* tri;           /* n_objects x 18: p1,p2,p3,n1,n2,n3 (triangles; NULL if none) */
    const int32_t* child_start;  /* per object: offset into children[] (groups) */
    const int32_t* child_count;  /* per object: number of children (Group.child_ids order) */
    const int32_t* children;
    int32_t n_top;               /* Scene.ids (tie-break order of the stable sort) */
    const int32_t* top;

    int32_t n_materials;         /* Material (material.rs:35-44) */
    const double* mat;           /* n_materials x 7: ambient, diffuse, specular, shininess,
                                    reflective, transparency, refractive_index */
    const int32_t* mat_pattern;  /* root pattern per material */

    int32_t n_patterns;          /* Pattern tree nodes (pattern.rs:23-27) */
    const int32_t* pat_kind;
    const int32_t* pat_a;        /* child pattern ids (-1 if none) */
    const int32_t* pat_b;
    const double* pat_color;     /* n_patterns x 3 (Solid) */
    const double* pat_scale;     /* n_patterns (Blend) */
    const double* pat_transform; /* n_patterns x 16 */

    int32_t n_lights;            /* Light (light.rs:17-21) */
    const int32_t* light_kind;
    const double* light;         /* n_lights x 15: position, intensity, corner, u, v */
    const int32_t* light_level;  /* area light sample level (light.rs:13) */

    /* ABI 3 */
    const double* shape;         /* optional n_objects x 3: minimum, maximum, closed (cylinder.rs:29-37,
                                    cone.rs:30-38); NULL: -inf, +inf, open.  Torus (ABI 4):
                                    shape[0] = minor_radius (torus.rs:23-31; major radius 1) */
    const int32_t* csg_op;       /* optional per object: RR_CSG_* (CSG objects; their two children,
                                    left then right, are the group child lists) */
    /* ABI 4: Perturbed / Noise patterns (pattern.rs:16-19); pat_scale is their scale, pat_a the
       perturbed pattern, pat_a / pat_b the noise's two sub-patterns */
    const int32_t* pat_octaves;      /* optional per pattern (`usize`, <= RR_MAX_OCTAVES); NULL: 1 */
    const double* pat_persistence;   /* optional per pattern; NULL: 1.0 */
    /* ABI 4: image textures (texture.rs:6-11, Texture::new decodes + to_rgba8) */
    int32_t n_textures;
    const int32_t* tex_size;         /* n_textures x 2: width, height (>= 1 each) */
    const uint8_t* texels;           /* RGBA8 rows top to bottom, textures back to back */
} rr_scene_desc;

/* Camera (camera.rs:18-27): hsize/vsize are the SUPERSAMPLED sizes (W*aa, H*aa). */
typedef struct {
    int64_t hsize, vsize;
    double field_of_view, pixel_size, half_width, half_height;
    double transform[16];
} rr_camera;

/* render options */
typedef struct {
    int32_t aa;            /* anti-aliasing level; camera sizes are W*aa x H*aa */
    int32_t max_depth;     /* reflect/refract recursion budget (5 in camera.rs:113) */
    uint64_t seed;         /* area-light jitter seed (replaces thread_rng, light.rs:57-59) */
    int32_t jitter_mode;   /* 0 = counter hash jitter, 1 = cell centre */
    int32_t part, nparts;  /* row sharding: output rows y with (y/block_rows)%nparts == part */
    int32_t block_rows;    /* rows per interleaved block (default 8) */
    int32_t flags;         /* RR_OUT_* */
    /* ABI 10: a contiguous band of output rows [row_begin, row_end) instead of an interleaved part (part 0 of 1
       only; row_begin == row_end == 0: no band, and any other pair with row_end <= row_begin is refused).  Rows, pixels and the area-light jitter are the full frame's, so a band equals
       those rows of the whole frame bit for bit. */
    int32_t row_begin, row_end;
} rr_render_opts;
#define RR_OUT_CANVAS 1    /* write the supersampled canvas (Canvas.pixels layout) */
#define RR_OUT_AVG 2       /* write the AA-averaged image (canvas.rs:76-96, before `as u8`) */
#define RR_OUT_AVG_F32 4   /* rr_render_device only: the AA-averaged image rounded to float (3 floats per
                              pixel; the average itself is computed in f64) — compact tiles for gathers */
#define RR_NO_FRAME_TIMING 8 /* rr_render_device only: no HIP event pair around the frame (each event
                                record costs the stream a few microseconds); rr_stats.kernel_ms is 0 */
#define RR_PART_INTERLEAVE 16 /* ABI 10, multi-device contexts: interleaved row tiles, a staging buffer and placement
                                 kernels on rank 0 (the ABI 9 transfer) instead of cost-balanced bands */

typedef struct {
    uint64_t rays;          /* closest-hit rays (primary + reflected + refracted) */
    uint64_t shadow_rays;   /* is_shadowed rays */
    uint64_t shade_events;  /* shade_hit calls */
    uint64_t n1n2_scans;    /* prepare_computations container walks (transparent hits) */
    uint64_t group_tests, group_hits;
    uint64_t samples;       /* pixel x AA samples rendered */
    uint64_t prim_tests;    /* exact f64 leaf tests executed (lane-level, after culling) */
    double kernel_ms;       /* render + AA kernels, HIP events (0 with RR_NO_FRAME_TIMING) */
    uint64_t exact_flops[3];  /* f64 flops of those tests (SURVEY §8d model) per walk: trace, shadow, n1n2 */
    uint64_t wave_visits[3];  /* wave-level node visits (exact test issued for a 64-lane wave), same order */
    /* ABI 6: rays whose intersection list (as far as the walk computed it) held a NaN t among >= 2
       entries — where the reference panics; > 0 makes rr_render return RR_E_NAN */
    uint64_t nan_rays;
} rr_stats;

typedef struct rr_ctx rr_ctx;
typedef struct rr_scene rr_scene;

/* ---- library ---- */
int32_t rr_abi_version(void);
const char* rr_last_error(void);            /* thread-local message of the last failure */
int rr_device_count(int* out);

/* ---- context: one device, one stream (not thread-safe; one render at a time) ---- */
int rr_create(int device, rr_ctx** out);
void rr_destroy(rr_ctx* ctx);
/* flattens (DFS order, 3x4 inverses, group AABBs) and uploads to HBM (scene.rs, group.rs);
 * a multi-device context replicates the scene to every device */
int rr_scene_upload(rr_ctx* ctx, const rr_scene_desc* desc);

/* ---- multi-device contexts (ABI 5): one frame across several GPUs (camera.rs:107-121 spreads one
 * frame over every rayon worker).  ABI 10 default: global rank r renders a contiguous band of output rows
 * [bounds[r], bounds[r+1]) as an f64 AA-averaged tile; the bands are balanced by cost on the first frame of a
 * layout (rank 0 renders that frame once as 64 timed bands, rr_balance_bands, and broadcasts the bounds to every
 * rank: one ncclBroadcast per layout), and rank 0's band is kept lighter by its own transfer work.  One RCCL group
 * per frame (over xGMI): every other rank sends its tile to rank 0 in one ncclSend, which rank 0 receives straight
 * into the frame's rows; rank 0 copies its own tile there.  No staging buffer, no placement kernel.
 * With RR_PART_INTERLEAVE (the ABI 9 transfer): rank r renders the output rows {y : (y/block_rows) % N == r};
 * every rank sends its whole tile to rank 0 in one ncclSend, and rank 0 receives every part's tile (its own from
 * itself) back to back into a staging buffer of `height` rows, one ncclRecv per part (part p at row
 * rr_stage_row_offset); one copy kernel per part then places the tile's rows into their frame rows.  The context
 * owns a render and a transfer stream per device and the RCCL communicator.  rr_render (blocking; out_avg filled on rank 0 only) and
 * rr_render_gather_device (asynchronous) take part 0 of 1: the context does the split.  Only the
 * f64 averaged image is produced (no RR_OUT_CANVAS / RR_OUT_AVG_F32).  rr_color_at / rr_is_shadowed /
 * rr_kernel_times act on the context's first local device; rr_last_stats sums its local devices. */
#define RR_RCCL_ID_BYTES 128
/* this process drives n devices (ncclCommInitAll); images are bit-identical to one device's */
int rr_create_multi(int n_devices, const int* device_ids, rr_ctx** out);
/* one process per GPU: rank 0 makes an id with rr_rccl_unique_id, the host shares it (any channel),
 * every rank calls rr_create_rank with it (ncclCommInitRank; collective) */
int rr_rccl_unique_id(uint8_t* out, int32_t n_bytes);
int rr_create_rank(int device, int nranks, int rank, const uint8_t* unique_id, rr_ctx** out);
/* nranks in the group, this context's first global rank, devices this context drives (1/0/1 for rr_create) */
int rr_context_info(const rr_ctx* ctx, int32_t* nranks, int32_t* rank, int32_t* ndevices);
/* ABI 7: nparts VIRTUAL ranks on one device — the N > 1 path of a real group (per-part contexts and
 * streams, tiles, double buffering, the staging buffer at the same per-part offsets and the same placement
 * kernels) with only the ncclSend / ncclRecv pairs replaced by device-local copies of each tile into the
 * staging buffer.  For exercising / testing the multi-GPU frame assembly on one GPU; images are
 * bit-identical to one part's. */
int rr_create_virtual(int device, int nparts, rr_ctx** out);
/* ABI 10: band bounds from per-row costs: bounds[0] = 0 <= bounds[1] <= ... <= bounds[nparts] = height, every inner
 * bound a multiple of `align`, such that part p's cost sum(row_cost[bounds[p] .. bounds[p+1]-1]) (plus root_extra
 * for part 0, the same unit) is as even as the alignment allows.  Host only.  Returns RR_OK. */
int rr_balance_bands(const double* row_cost, int64_t height, int32_t nparts, double root_extra, int32_t align,
                     int64_t* bounds);
/* ABI 10: the band bounds of a multi-device context (nranks + 1 values; n >= nranks + 1) once its first band frame
 * has calibrated them, and rr_group_set_bands to impose bounds (every rank the same; skips the calibration until the
 * frame layout changes).  rr_group_bands returns the number of bounds written (0: not calibrated yet). */
int rr_group_bands(rr_ctx* ctx, int64_t* bounds, int32_t n);
int rr_group_set_bands(rr_ctx* ctx, const int64_t* bounds, int32_t n);
/* ABI 9: first row of part `part`'s tile in the staging buffer (the rows of parts 0 .. part-1; partition.hpp
 * stage_row_offset).  part == nparts gives height. */
int64_t rr_stage_row_offset(int64_t height, int32_t part, int32_t nparts, int32_t block_rows);
/* ABI 9 (was ABI 7 with padded tiles): the frame from tiles a caller transferred itself (e.g. torch.distributed
 * send / recv; the same layout and run arithmetic as the device transfer): staged = the nparts tiles back to back,
 * unpadded, part p's rows (increasing y) at row rr_stage_row_offset(height, p, nparts, block_rows), height rows of
 * width*3 doubles in all -> frame = height rows in frame order.  No device needed (CPU rehearsals of the N > 1 path
 * use it).  The buffers are not checked: both must hold height * width * 3 doubles (rray_amd.unshuffle checks its
 * array's shape before the call). */
int rr_unshuffle_host(const double* staged, double* frame, int64_t width, int64_t height, int32_t nparts,
                      int32_t block_rows);
/* ABI 8: build provenance — the sha256 prefix of the product sources this library was built from
 * (rray_amd/build.py source_digest(): rray_amd/csrc/*, this header, the build script).  Static string. */
const char* rr_build_digest(void);
/* Whole frame -> d_frame (W*H*3 doubles on rank 0's device; ignored on other ranks), enqueued after
 * the work already on `hip_stream` (NULL: no ordering with the caller) and completed in its order;
 * not synchronised.  Collective: every rank calls it for every frame.  Tiles are double-buffered, so
 * frame k+1 renders while frame k is being gathered.  On a single-device context it is
 * rr_render_device(d_avg = d_frame). */
int rr_render_gather_device(rr_ctx* ctx, const rr_camera* cam, const rr_render_opts* opts, void* d_frame,
                            void* hip_stream);

/* Camera::new (camera.rs:41-63) */
int rr_camera_new(int64_t hsize, int64_t vsize, double field_of_view, const double transform[16], rr_camera* out);

/* Camera::render (camera.rs:107-121).  Host buffers:
 *   out_canvas: hsize*vsize_part*3 doubles (RR_OUT_CANVAS) — identical layout to Canvas.pixels;
 *   out_avg:    W*rows_part*3 doubles (RR_OUT_AVG).
 * Rows are this part's rows in increasing order (see rr_part_rows).  Blocking. */
int rr_render(rr_ctx* ctx, const rr_camera* cam, const rr_render_opts* opts, double* out_canvas, double* out_avg,
              rr_stats* stats);
/* Same, into DEVICE buffers on the context's device, enqueued on `hip_stream` (NULL: ctx stream)
 * and NOT synchronised — for collectives that consume the tile straight from HBM.  d_avg holds
 * doubles, or floats with RR_OUT_AVG_F32. */
int rr_render_device(rr_ctx* ctx, const rr_camera* cam, const rr_render_opts* opts, void* d_canvas, void* d_avg,
                     void* hip_stream);
/* AA-averaged rows owned by `part` of `nparts` (interleaved blocks of block_rows output rows). */
int64_t rr_part_rows(int64_t height, int32_t part, int32_t nparts, int32_t block_rows, int64_t* rows_out);
/* Per-kernel HIP-event timing on the context's stream.  rr_kernel_profile(ctx, 1) resets and enables
 * it; rr_kernel_times fills accumulated milliseconds and launch counts per kernel in the order
 * trace, n1n2, shade, shadow, finish, combine, aa, trace_shade, chain, deep (returns the number of kernels,
 * 10; the shadow walks and the light sum run inside shade, so shadow and finish stay 0; scenes without
 * transparent materials run trace and shade as one trace_shade kernel, and those whose materials reflect run
 * every reflection chain in one chain kernel — deep only with RRAY_DEEP=1). */
int rr_kernel_profile(rr_ctx* ctx, int enable);
int rr_kernel_times(rr_ctx* ctx, double* ms, uint64_t* launches, int32_t n);
/* stats of the last rr_render/rr_render_device on this context (synchronises) */
int rr_last_stats(rr_ctx* ctx, rr_stats* stats);

/* Scene::color_at (scene.rs:128-136) for a batch of rays (rr_color_at), and
 * Scene::is_shadowed (scene.rs:234-245) for a batch of point/light pairs.  Host buffers. */
int rr_color_at(rr_ctx* ctx, int64_t n, const double* origins, const double* directions, int32_t remaining,
                uint64_t seed, int32_t jitter_mode, double* out_rgb);
int rr_is_shadowed(rr_ctx* ctx, int64_t n, const double* points, const double* light_positions, int32_t* out);

/* Host-only inspection of the flattening (no device needed): per-object inverse transforms as the
 * kernels use them (4x4, row 3 == 0,0,0,1), group bounding boxes (group.rs:128-149; zeros for
 * non-groups) and each object's index in the flattened depth-first order (-1: not in the tree).
 * Any output pointer may be NULL. */
int rr_scene_inspect(const rr_scene_desc* desc, double* inverses, double* group_aabbs, int32_t* node_of_object);

/* ---- front-end: scene_builder_yaml.rs / load_obj.rs / canvas.rs / main.rs ---- */
/* render_scene_from_str up to camera.render: parse YAML (first document), build the scene.
 * obj_root: directory relative OBJ paths are resolved against (NULL: current directory). */
int rr_scene_from_yaml(const char* yaml_text, const char* obj_root, int64_t width, int64_t height, int32_t aa,
                       rr_scene** out_scene, rr_camera* out_camera);
const rr_scene_desc* rr_scene_desc_of(const rr_scene* scene);
void rr_scene_free(rr_scene* scene);
/* canvas.rs:76-105 + write_to_file: AA-averaged f64 image -> RGBA8 (`as u8`) -> PNG */
int rr_quantize(const double* avg, int64_t n_pixels, uint8_t* rgba);
int rr_write_png(const char* path, const uint8_t* rgba, int64_t width, int64_t height);
/* render_scene_from_file (scene_builder_yaml.rs:429-436) on `device` */
int rr_render_scene_from_file(const char* path, int64_t width, int64_t height, const char* png_file, int32_t aa,
                              int device);
/* the same on n devices of this process (rr_create_multi) */
int rr_render_scene_from_file_devices(const char* path, int64_t width, int64_t height, const char* png_file,
                                      int32_t aa, int n_devices, const int* device_ids);

#ifdef __cplusplus
}
#endif
#endif /* RRAY_RRAY_H */
