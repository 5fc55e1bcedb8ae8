// rt_device.h — data layout shared by the host flattener and the gfx950
// kernel (plain structs, no HIP types, so g++ can include it too).
//
// HBM layout:
//   RtNode   64 B  one child record: the 7-DOP slabs of a non-empty octree
//                  node + where its contents are. The children of an
//                  internal node occupy `cnt` consecutive records starting at
//                  `ref`, in child-index order (empty children are dropped;
//                  they can never be hit by a non-NaN ray).
//                  Record 0 is the root.
//   tri4     48 B  per triangle, in leaf order: {a.xyz, prim}, {e1.xyz, 0},
//                  {e2.xyz, 0} with e1 = b - a, e2 = c - a computed exactly
//                  as Triangle::intersect does (triangle.h:21-22).
//   RtMat    32 B  SimpleMaterial {emission.rgb, metalness, diffuse.rgb, roughness}.
//   env      16 B  per texel RGBA (alpha 0), plus f32 luminance and CDF.
#pragma once

#include <stdint.h>

#include "rt_fp.h"

struct alignas(16) float4_ {
    float x, y, z, w;
};
RT_HD void rt_pin(float4_ v)  // (rt_fp.h rt_pin, per component)
{
    rt_pin(v.x);
    rt_pin(v.y);
    rt_pin(v.z);
    rt_pin(v.w);
}

#define RT_LEAF_BIT 0x80000000u

struct alignas(16) RtNode {
    float dn[7];
    float df[7];
    uint32_t ref;  // internal: first child record; leaf: first triangle (leaf order)
    uint32_t cnt;  // internal: number of child records (1..8); leaf: RT_LEAF_BIT | triangle count
};
static_assert(sizeof(RtNode) == 64, "RtNode must be 64 B");

// Search BVH (binary, SAH) over the same triangles, used to find the closest
// Moller-Trumbore hit fast; the octree then verifies it (rt_fast.h). 64 B:
// the two child boxes (conservatively padded) and, per child, an inner node
// index (count 0), a leaf's first entry in bvh_tri4 (count > 0) or nothing
// (count -1).
struct alignas(16) BvhNode {
    float lmin[3], lmax[3], rmin[3], rmax[3];
    int32_t left, right, lcount, rcount;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 B");

// 4-wide search BVH collapsed from the binary one (rt_scene.cpp
// collapse_bvh4): 128 B = one L2 line; child boxes stored per axis so a
// node is 8 float4 loads and four slab tests in lock-step. Child c: inner
// node index (cnt 0), leaf's first entry in bvh_tri4 (cnt 1..4) or nothing
// (cnt -1, box empty).
// Search-BVH node: four 32-B child records {lo.xyz, hi.xyz, ref, cnt}, so one
// lane can load one child with two 16-B loads (rt_fast.h quad walks).
// cnt: -1 empty slot, 0 inner node (ref = node index), > 0 leaf of cnt
// triangles starting at bvh_tri4 record 3 * ref.
struct Bvh4Child {
    float lo[3], hi[3];
    int32_t ref, cnt;
};
struct alignas(128) Bvh4Node {
    Bvh4Child ch[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node must be 128 B");
// 16-wide search BVH (rt_scene.cpp build_bvh16, walked by 16-lane rows: rt_row.h): node
// i is records [16 i, 16 i + 16) of Bvh4Child, 512 B, one record per lane of a row, and
// holds two levels of 4-wide node i: its leaf children and the children of its inner
// children (an inner record's ref is a 4-wide node index, which is also its 16-wide node).
// Same boxes, same leaves (<= 4 triangles), so the same hits; same item numbering, so a
// walk may switch between quads and rows at any trip.
#define RT_BVH16_W 16

struct alignas(16) RtMat {
    float er, eg, eb, metalness;
    float dr, dg, db, roughness;
};

struct RtSceneView {
    const RtNode* nodes;
    const float4_* tri4;
    const int32_t* prim2k;
    const int32_t* mat_idx;
    const int32_t* matk;  // leaf-order triangle k -> mat_idx[prim of k] (device: one load instead of two)
    const RtMat* mats;
    const int32_t* emissive;
    const float4_* spheres;  // 2 records each: {c.xyz, r}, {prim bits, 0, 0, 0}
    const float4_* env;
    const float* env_lum;
    const float* cdf;
    const float* cdf_row;     // [eh]  cdf of each row's last texel
    const float* cdf_coarse;  // [eh][cdf_cw]  cdf[y*ew + 32j + 31]
    const float* cdf_fence;   // [1 + eh][272] fence tables (rt_trace.h cdf_search_fence), or null
    int32_t n_emissive, n_spheres, ew, eh;
    int32_t n_tris, chain_monotone, cdf_cw;  // chain_monotone: see rt_fast.h chain_ok
    float cdf_total;  // cdf[ew * eh - 1] (render_kernel.cpp:572, :619), a parameter instead of a load
    int32_t n_mats;   // entries of mats
    int32_t brute;  // 1: INTERSECT_SCENE is the brute-force loop (USE_BVH 0, render_kernel.cpp:453-483)
    // search BVH + octree back-links for the verification walk
    const Bvh4Node* bvh4;      // [0] = root
    const Bvh4Child* bvh16;    // 16-wide form, RT_BVH16_W records per node, node 0 = root
    const float4_* bvh4s;      // oriented slab of each 4-wide child ([node * 4 + c]; rt_fast.h slab_ok)
    const float4_* bvh16s;     // the same, in bvh16's record order ([node * RT_BVH16_W + j])
    const float4_* bvh_tri4;   // 3 records per triangle in BVH leaf order: {a.xyz, k}, {e1, leaf record}, {e2}
    const int32_t* parent;     // octree record -> parent record (-1 for the root)
    const int32_t* leaf_of;    // leaf-order triangle k -> its octree leaf record
    int32_t tri_mat;  // 1: tri4[3k + 1].w holds the material index of leaf-order triangle k (device copy)
    // near box (rt_fast.h far_origin): a query whose origin lies outside it is answered by the exact
    // octree walk; the scene's box widened by RT_NEAR_SCALE x its largest extent (rt_view_near)
    float near_lo[3], near_hi[3];
};

struct RtCamera {
    float m[16];
    float fov_dist;
};

// Per-render counters (stats build). Closest-hit queries: rays traced,
// child-volume tests, triangle tests, leaf visits, tie-order slow paths;
// shading: material fetches, env texel fetches, CDF probes; occlusion
// (any-hit) queries: rays, volume tests, triangle tests, leaf visits.
enum {
    RT_STAT_RAYS = 0,
    RT_STAT_VOL,
    RT_STAT_TRI,
    RT_STAT_LEAF,
    RT_STAT_MAT,
    RT_STAT_ENV,
    RT_STAT_CDF,
    RT_STAT_HEAP_SLOW,
    RT_STAT_ANY_RAYS,
    RT_STAT_ANY_VOL,
    RT_STAT_ANY_TRI,
    RT_STAT_ANY_LEAF,
    RT_STAT_VERIFY,    // octree slab tests of the verification walks
    RT_STAT_FALLBACK,  // queries answered by the exact octree walk
    RT_STAT_QUAD_VISITS,  // k_trace: inner-node visits of the quad walks (one per quad trip)
    RT_STAT_WAVE_SLOTS,   // k_trace: per 16-query chunk, 16 x its longest walk's visits (SIMT slots)
    RT_STAT_REFILLS,      // k_trace stream: refill rounds of the waves
    RT_STAT_DRAIN_SLOTS,  // k_trace stream: the WAVE_SLOTS spent after the wave's stream ran out
    RT_STAT_DRAIN_VISITS, // ... and the QUAD_VISITS among them
    RT_STAT_STEPS,        // path steps (rt_wave.h path_step calls that were not waiting on a parked walk)
    RT_STAT_COUNT
};
