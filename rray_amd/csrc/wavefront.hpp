// wavefront.hpp — per-level ray queues of the wavefront render (host + device view).
//
// Scene::color_at recursion (scene.rs:128-336) is evaluated level by level: level d holds every
// pending color_at(ray, max_depth - d).  Each level runs trace -> [n1/n2 walk] -> shade (which
// includes the shadow walks and the light sum); children (reflected / refracted rays) are appended
// to level d+1 with a parent link.  Events without children deliver their value at once (canvas or
// the parent's slot); events with children are listed as pending and a bottom-up combine pass
// finishes them, reproducing shade_hit's summation exactly (scene.rs:172-177).
#pragma once
#include <stdint.h>

namespace rr {

// a pending color_at(ray, rem) at level >= 1 (level 0 rays come from the camera or the caller)
struct alignas(16) Event {
    double o[3], d[3];
    uint32_t sample;  // local sample index (this part / batch-relative + base)
    uint32_t path;    // recursion path code: root 1, reflected child 2p, refracted child 2p+1
    int32_t parent;   // event index at level - 1
    int32_t slot;     // 0 = reflected child, 1 = refracted child
};
static_assert(sizeof(Event) == 64, "Event layout");

struct alignas(16) HitRec {  // closest hit of an event (first t >= 0 of the sorted xs)
    double t, u, v;
    int32_t node;  // -1: miss
    int32_t k;     // local entry index (sphere t1 = 0, t2 = 1)
};

// shade_hit's pending sum of an event with children.  Split so that scenes without transparency
// (C3's reflection chains) move 64 B per pending event instead of 112: the refraction half lives
// in a parallel CombExt array that exists only when some material is transparent.
struct alignas(64) CombRec {
    double surf[3];
    double refl_res[3];  // color_at(reflect ray) * reflective, or 0
    double refl;
    int32_t parent;      // event index at level - 1 (-1 at level 0)
    int32_t flags;       // CF_*
};
struct CombExt {
    double refr_res[3];  // color_at(refract ray) * transparency, or 0
    double transp, R;
};
static_assert(sizeof(CombRec) == 64, "CombRec layout");
// Scenes without transparency (the FUSED kernels): an event has at most one child, its reflection,
// so no combine pass runs — the chain's leaf folds every ancestor's record on its way up.
struct alignas(16) ChainRec {
    double surf[3];
    double refl;      // the material's reflective
    int32_t parent;   // event index at level - 1 (-1 at level 0)
    int32_t pad[3];
};
static_assert(sizeof(ChainRec) == 48 && sizeof(ChainRec) <= sizeof(CombRec), "ChainRec layout");
enum { CF_HIT = 1, CF_REFRACT_CHILD = 2 };
// A reflection chain leaving its camera wave at depth RR_DEEP_FROM for the deep launch (render_levels.inc
// chain_kernel): the pending reflected ray, the chain's records of depths 0 .. RR_DEEP_FROM - 1 (shade_hit's
// surface sum and the material's reflective), and the camera sample's output index.
constexpr int RR_DEEP_FROM = 2;
// deep-queue segments: camera blocks b with equal b >> RR_DEEP_SHIFT append to one segment (neighbouring tiles,
// so a deep wave's rays come from one stretch of the frame), capacity (256 << RR_DEEP_SHIFT) entries
constexpr int RR_DEEP_SHIFT = 5;
struct alignas(16) DeepRec {
    double o[3], d[3];
    double rec[RR_DEEP_FROM][4];
    uint32_t ls;
    uint32_t pad[3];
};
static_assert(sizeof(DeepRec) == 128, "DeepRec layout");

// per-level device counters.  Fused levels (no transparency) queue their children in RR_NSEG segments
// (block b appends to segment b % RR_NSEG with one atomic per wave, no workgroup barrier; the next
// level's block b reads segment b % RR_NSEG — blocks are dealt to the XCDs round-robin, so a segment's
// producer and consumer run on the same XCD); LC_SEG0 + s counts segment s of the level.
constexpr int RR_NSEG = 1024;
enum { LC_CHILDREN = 0, LC_PENDING, LC_N1N2, LC_SEG0, LC_COUNT = LC_SEG0 + RR_NSEG };

}  // namespace rr
