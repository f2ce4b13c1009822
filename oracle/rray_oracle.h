/*
 * rray_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the davelpz/rray render path (reference snapshot 2024-08-07,
 * Rust crate at /root/reference).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library; the product
 * (rray_amd/, include/rray/rray.h) never links, calls or falls back to it.
 *
 * It follows the reference's own structure op-for-op: a per-scene object
 * registry (object/db.rs), per-object inverse transforms applied to the ray
 * (object.rs:45-48), full intersection lists + stable sort (scene.rs:97-106),
 * recursive color_at / shade_hit / reflected / refracted colour
 * (scene.rs:128-336), the n1/n2 container walk (intersection.rs:50-95),
 * Phong lighting (light.rs:98-140) and pattern trees (pattern.rs:145-215).
 * Built with -ffp-contract=off so no multiply-add is fused (rustc never fuses).
 *
 * Deviation (documented in DESIGN.md): the area-light jitter of light.rs:57-59
 * uses rand::thread_rng (non-deterministic); here it is a counter-based hash
 * shared bit-for-bit with the HIP kernel (orc_jitter below).
 */
#ifndef RRAY_ORACLE_H
#define RRAY_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_world orc_world;

/* pattern kinds (pattern.rs:10-21) */
enum { ORC_PAT_TEST = 0, ORC_PAT_SOLID = 1, ORC_PAT_STRIPE = 2, ORC_PAT_GRADIENT = 3,
       ORC_PAT_RING = 4, ORC_PAT_CHECKER = 5, ORC_PAT_BLEND = 6, ORC_PAT_PERTURBED = 7, ORC_PAT_NOISE = 8,
       ORC_PAT_TEXTURE = 9 /* a = texture id */ };
/* object kinds */
enum { ORC_SPHERE = 0, ORC_PLANE = 1, ORC_GROUP = 2, ORC_TRIANGLE = 3, ORC_SMOOTH_TRIANGLE = 4,
       ORC_CUBE = 5, ORC_CYLINDER = 6, ORC_CONE = 7, ORC_CSG = 8,
       ORC_TORUS = 9 /* minor radius = shape param `minimum` */ };
/* CSG operations (csg.rs:13-17) */
enum { ORC_CSG_UNION = 0, ORC_CSG_INTERSECTION = 1, ORC_CSG_DIFFERENCE = 2 };

typedef struct {
    uint64_t rays;          /* Scene::intersect calls (primary + secondary + shadow) */
    uint64_t shadow_rays;   /* of which from is_shadowed */
    uint64_t sphere_tests, plane_tests, tri_tests, group_tests, group_hits;
    uint64_t cube_tests, cyl_tests, cone_tests, csg_tests;
    uint64_t shade_events;  /* shade_hit calls */
    uint64_t nan_sorts;     /* sort comparisons that would panic in the reference */
    uint64_t torus_tests;
} orc_stats;

/* ---- matrices (matrix.rs) — 4x4 row-major double[16] ---- */
void   orc_mat_identity(double out[16]);
void   orc_mat_translate(double x, double y, double z, double out[16]);
void   orc_mat_scale(double x, double y, double z, double out[16]);
void   orc_mat_rotate(int axis /*0=x,1=y,2=z*/, double radians, double out[16]);
void   orc_mat_shear(double xy, double xz, double yx, double yz, double zx, double zy, double out[16]);
void   orc_mat_multiply(const double a[16], const double b[16], double out[16]);
void   orc_mat_inverse(const double a[16], double out[16]);
double orc_mat_determinant(const double a[16]);
void   orc_mat_view_transform(const double from[3], const double to[3], const double up[3], double out[16]);
void   orc_mat_multiply_tuple(const double m[16], const double t[4], double out[4]);

/* ---- world construction ---- */
orc_world* orc_world_new(void);
void orc_world_free(orc_world* w);
int  orc_add_object(orc_world* w, int kind, int parent /* -1: scene top level */);
int  orc_add_triangle(orc_world* w, int parent, const double p1[3], const double p2[3], const double p3[3]);
int  orc_add_smooth_triangle(orc_world* w, int parent, const double p1[3], const double p2[3], const double p3[3],
                             const double n1[3], const double n2[3], const double n3[3]);
/* load_obj.rs:124-139 + tobj 4.0.2 semantics; returns the group id or <0 on error */
int  orc_load_obj(orc_world* w, const char* path, int parent, const double mat7[7], int pattern);
void orc_set_transform(orc_world* w, int id, const double m[16]);
/* cylinder / cone: minimum, maximum, closed (cylinder.rs:29-37, cone.rs:30-38) */
void orc_set_shape_params(orc_world* w, int id, double minimum, double maximum, int closed);
/* CSG: operation; its left and right are the first and second object added with it as parent */
void orc_set_csg_op(orc_world* w, int id, int op);
/* csg.rs:67-80 intersection_allowed; csg.rs:82-101 filter_intersections over (t, obj) */
int  orc_csg_allowed(int op, int lhit, int inl, int inr);
void orc_get_shape_params(orc_world* w, int id, double out[3]);
int  orc_get_csg_op(orc_world* w, int id);
int  orc_csg_filter(orc_world* w, int csg, int n, const double* t, const int* obj, int* keep_index);
/* mat7 = ambient, diffuse, specular, shininess, reflective, transparency, refractive_index */
void orc_set_material(orc_world* w, int id, const double mat7[7], int pattern /* -1 = default white solid */);
int  orc_pattern_new(orc_world* w, int kind, const double color[3], int a, int b, double scale, const double m[16]);
/* perturbed / noise: octaves and persistence (pattern.rs:104-118; scale is the pattern's scale) */
void orc_pattern_set_noise(orc_world* w, int pattern, int64_t octaves, double persistence);
/* noise.rs: fastnoise-lite 1.1.1 Perlin (seed 1337, frequency 0.01f) and octave_perlin */
double orc_noise_3d(double x, double y, double z);
double orc_octave_perlin(double x, double y, double z, int64_t octaves, double persistence);
int  orc_add_point_light(orc_world* w, const double pos[3], const double color[3]);
int  orc_add_area_light(orc_world* w, const double corner[3], const double u[3], const double v[3],
                        const double color[3], int level);
void orc_remove_light(orc_world* w, int index);
int  orc_num_children(orc_world* w, int id);
int  orc_num_objects(orc_world* w);
int  orc_num_patterns(orc_world* w);
/* kind, a, b -> ints[3]; scale, persistence -> dbl[2]; octaves -> *octaves */
void orc_pattern_info(orc_world* w, int id, int32_t ints[3], double dbl[2], int64_t* octaves);
void orc_get_inverse(orc_world* w, int id, double out[16]);

/* ---- queries mirroring the reference's unit-test entry points ---- */
int  orc_intersect(orc_world* w, const double o[3], const double d[3], int max, double* t, int* obj, double* u, double* v);
int  orc_local_intersect(orc_world* w, int id, const double o[4], const double d[4], int max, double* t, int* obj, double* u, double* v);
void orc_color_at(orc_world* w, const double o[3], const double d[3], int remaining, double out[3]);
/* xs given explicitly (t,obj,u,v); hit = index into xs.  what: 0 shade_hit, 1 reflected, 2 refracted */
void orc_shade(orc_world* w, const double o[3], const double d[3], int n, const double* t, const int* obj,
               const double* u, const double* v, int hit, int remaining, int what, double out[3]);
/* comps: t, point[4], eyev[4], normalv[4], inside, over[4], under[4], reflectv[4], n1, n2, schlick (27 doubles) */
void orc_prepare_computations(orc_world* w, const double o[3], const double d[3], int n, const double* t, const int* obj,
                              const double* u, const double* v, int hit, double out[27]);
int  orc_is_shadowed(orc_world* w, const double p[3], const double light_pos[3]);
void orc_lighting(orc_world* w, int obj, int light, const double point[3], const double eyev[3], const double normalv[3],
                  double in_shadow, double out[3]);
void orc_pattern_at(orc_world* w, int pattern, const double p[3], double out[3]);
/* texture.rs: RGBA8 rows top to bottom (image crate RgbaImage); returns the texture id */
int  orc_add_texture(orc_world* w, int width, int height, const uint8_t* rgba);
void orc_texture_color(orc_world* w, int tex, double u, double v, uint8_t out[4]);
/* Object::uv_mapping of object `obj` at an object-space point */
void orc_uv_mapping(orc_world* w, int obj, const double p[3], double out[2]);
/* roots 0.0.8 find_roots_quartic(a4, a3, a2, a1, a0): returns the number of roots (0-4), ascending */
int  orc_find_roots_quartic(double a4, double a3, double a2, double a1, double a0, double out[4]);
int  orc_find_roots_cubic(double a3, double a2, double a1, double a0, double out[4]);
int  orc_find_roots_quadratic(double a2, double a1, double a0, double out[4]);
void orc_normal_at(orc_world* w, int obj, const double p[3], double u, double v, double out[4]);
void orc_world_to_object(orc_world* w, int obj, const double p[3], double out[4]);
void orc_normal_to_world(orc_world* w, int obj, const double n[3], double out[4]);
void orc_group_aabb(orc_world* w, int id, double out[6]);

/* ---- camera + render (camera.rs, canvas.rs) ---- */
typedef struct {
    int64_t hsize, vsize;
    double field_of_view, pixel_size, half_width, half_height;
    double transform[16];
} orc_camera;
void orc_camera_new(int64_t hsize, int64_t vsize, double fov, const double transform[16], orc_camera* out);
void orc_ray_for_pixel(const orc_camera* c, int64_t px, int64_t py, double o[4], double d[4]);
/* Renders rows [row0, row0+nrows) of the (hsize x vsize) supersampled canvas, rows with
 * (y / band) % band_stride == band_phase only (band_stride=1: every row).
 * canvas: hsize*vsize*3 doubles (only rendered rows written).  Returns 0 or <0 (reference panic). */
int  orc_render(orc_world* w, const orc_camera* c, int max_depth, uint64_t seed, int jitter_mode, int threads,
                int band, int band_stride, int band_phase, double* canvas, orc_stats* stats);
/* canvas.rs:76-105 AA box average (before u8 quantisation): out = (hsize/aa)*(vsize/aa)*3 */
void orc_aa_average(const double* canvas, int64_t hsize, int64_t vsize, int aa, double* out);
/* (v*255.0) as u8 — Rust saturating cast */
void orc_quantize(const double* avg, int64_t n_pixels, uint8_t* rgba);

/* counter-based area-light jitter shared with the HIP kernel */
double orc_jitter(uint64_t seed, uint64_t sample, uint32_t path, uint32_t light, uint32_t s, uint32_t which);
void   orc_set_context(orc_world* w, uint64_t seed, int jitter_mode, uint64_t sample);
void   orc_set_pow_mode(orc_world* w, int mode);  /* diagnostic: 1 = correctly rounded integer powers */
void   orc_get_stats(orc_world* w, orc_stats* out);

#ifdef __cplusplus
}
#endif
#endif
