// rt_fast.h — exact scene queries through a fast search structure.
//
// The reference answers every query with its octree walk (bvh.h:127-209),
// whose cost per ray has a heavy tail (rays grazing the tessellated surface
// test thousands of volumes before the early exit can fire). Its *answer*,
// though, is pinned down by a few facts we can check cheaply:
//
//  (1) A hit can only come from a triangle whose Moller-Trumbore test
//      (tri_test, the reference's arithmetic) returns true. A binary SAH BVH
//      with conservatively padded boxes finds all such triangles in any
//      window [0, T] — so "no M-T hit at all" means "the reference finds no
//      hit", exactly.
//  (2) Occlusion (the reference uses INTERSECT_SCENE only as a boolean there)
//      is "some M-T-hit triangle lies in a leaf all of whose octree
//      ancestors pass their slab tests" — pruning only starts after a hit.
//      So: BVH any-hit, then the exact slab tests along the candidate's
//      octree ancestor chain.
//  (3) Closest hit: let k* be the closest M-T hit (t*), t2 a lower bound on
//      every other triangle's hit distance. The reference returns (t*, k*)
//      if k*'s leaf is reachable (all ancestor slab tests pass) and no
//      ancestor A can be pruned by the early exit before k* is found:
//      pruning A needs `closest < t_near(A)` with `closest` >= t2 until k*
//      is visited, so t2 >= t_near(A) for every ancestor rules it out; and
//      no other triangle ties t*. Every such fact is checked here with the
//      reference's own float arithmetic; a query that fails a check is
//      re-answered by the exact octree walk (rt_traverse.h) — rare.
#pragma once

#include "rt_traverse.h"

namespace rtk {

// Ray constants for the padded-box slab test (any sound test works here:
// the boxes are padded; this one just must not miss them).
struct RayB {
    float inv[3], oi[3];
};

RT_HD RayB rayb_setup(V3 o, V3 d)
{
    RayB r;
    const float dd[3] = {d.x, d.y, d.z}, oo[3] = {o.x, o.y, o.z};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float di = __builtin_fabsf(dd[i]) < 1e-20f ? rt_copysignf(1e-20f, dd[i]) : dd[i];
        r.inv[i] = 1.0f / di;
        r.oi[i] = -oo[i] * r.inv[i];
    }
    return r;
}

// Entry distance of a box if the ray passes through it within [0, tmax].
RT_HD bool box_hit(const float* mn, const float* mx, const RayB& r, float tmax, float& tnear)
{
    float t0 = -__builtin_inff(), t1 = tmax;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float a = mn[i] * r.inv[i] + r.oi[i], b = mx[i] * r.inv[i] + r.oi[i];
        t0 = __builtin_fmaxf(t0, __builtin_fminf(a, b));
        t1 = __builtin_fminf(t1, __builtin_fmaxf(a, b));
    }
    tnear = t0;
    return t0 <= t1 && t1 >= 0.0f;
}

struct BvhNodeR {
    float lmin[3], lmax[3], rmin[3], rmax[3];
    int32_t left, right, lcount, rcount;
};
RT_HD BvhNodeR load_bvh(const BvhNode* nodes, int i)
{
    const float4_* p = (const float4_*)(nodes + i);
    const float4_ a = p[0], b = p[1], c = p[2], d = p[3];
    BvhNodeR n;
    n.lmin[0] = a.x, n.lmin[1] = a.y, n.lmin[2] = a.z, n.lmax[0] = a.w;
    n.lmax[1] = b.x, n.lmax[2] = b.y, n.rmin[0] = b.z, n.rmin[1] = b.w;
    n.rmin[2] = c.x, n.rmax[0] = c.y, n.rmax[1] = c.z, n.rmax[2] = c.w;
    n.left = (int32_t)rt_asuint(d.x), n.right = (int32_t)rt_asuint(d.y);
    n.lcount = (int32_t)rt_asuint(d.z), n.rcount = (int32_t)rt_asuint(d.w);
    return n;
}

// Relative width of the window past t* in which other hits are collected.
#define RT_T2_WINDOW 1.0e-3f

struct FastHit {
    float t, t2;  // closest M-T hit (-1: none), smallest other hit seen (window-bounded)
    int k;        // leaf-order triangle of t
    int leaf;     // its octree leaf record
    bool tie;     // another triangle hit at exactly t
    bool ovf;     // the bounded stack overflowed: answer unknown
};

RT_HD void fast_leaf(const RtSceneView& S, int first, int count, V3 o, V3 d, FastHit& h, Stats* st)
{
    for (int j = 0; j < count; j++) {
        const int i = first + j;
        float t;
        if (tri_test(S.bvh_tri4, i, o, d, t)) {
            if (t < h.t) {
                h.t2 = h.t;
                h.t = t;
                h.k = (int)rt_asuint(S.bvh_tri4[3 * i].w);
                h.leaf = (int)rt_asuint(S.bvh_tri4[3 * i + 1].w);
                h.tie = false;
            } else if (t == h.t) {
                h.tie = true;
                h.t2 = t;
            } else if (t < h.t2) {
                h.t2 = t;
            }
        }
    }
    if (st) st->c[RT_STAT_TRI] += count;
}

// All M-T hits within [0, t*(1 + RT_T2_WINDOW)]: closest, tie flag, second.
// STK: rec(i) / set_rec(i, v) over CAP entries.
template <class STK>
RT_HD void fast_closest(const RtSceneView& S, V3 o, V3 d, STK& stk, FastHit& h, Stats* st)
{
    h.t = __builtin_inff();
    h.t2 = __builtin_inff();
    h.k = -1;
    h.tie = false;
    h.ovf = false;
    if (st) st->c[RT_STAT_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) {
        h.t = -1.0f;
        return;
    }
    const RayB rb = rayb_setup(o, d);
    int sp = 0;
    int cur = 0;
    for (;;) {
        const BvhNodeR n = load_bvh(S.bvh, cur);
        if (st) st->c[RT_STAT_VOL] += 2;
        const float tmax = h.t + h.t * RT_T2_WINDOW;
        float tl, tr;
        const bool hl = n.lcount >= 0 && box_hit(n.lmin, n.lmax, rb, tmax, tl);
        const bool hr = n.rcount >= 0 && box_hit(n.rmin, n.rmax, rb, tmax, tr);
        int next = -1, far_ = -1;
        if (hl && n.lcount > 0) fast_leaf(S, n.left, n.lcount, o, d, h, st);
        if (hr && n.rcount > 0) fast_leaf(S, n.right, n.rcount, o, d, h, st);
        const bool il = hl && n.lcount == 0, ir = hr && n.rcount == 0;
        if (il && ir) {
            const bool lfirst = tl <= tr;
            next = lfirst ? n.left : n.right;
            far_ = lfirst ? n.right : n.left;
        } else if (il) {
            next = n.left;
        } else if (ir) {
            next = n.right;
        }
        if (far_ >= 0) {
            if (sp == STK::CAP) {
                h.ovf = true;
                return;
            }
            stk.set_rec(sp++, (uint32_t)far_);
        }
        if (next >= 0) {
            cur = next;
            continue;
        }
        // pop, skipping subtrees the window has closed behind (their boxes are re-tested anyway)
        if (sp == 0) break;
        cur = (int)stk.rec(--sp);
    }
    if (h.k < 0) h.t = -1.0f;
}

// Exact slab tests along an octree leaf's ancestor chain (root included).
// need_t2: also require t2 >= t_near for every non-root record.
//
// Shortcut (exact): an internal volume is the min / max of its children's
// planes (bvh.h:55-65, compute_volume), so along a chain every plane of an
// ancestor is at least as far out as the leaf's. Each slab quotient is a
// monotone function of its plane value for a fixed ray (a float subtraction,
// then a product with a fixed reciprocal, then a rounding), so an ancestor's
// computed interval contains the leaf's in every plane: if the leaf passes,
// every ancestor passes with t_near(A) <= t_near(leaf). The host checks the
// plane nesting for the whole tree (chain_monotone); otherwise the full
// chain is walked.
RT_HD bool chain_ok(const RtSceneView& S, const RayK& K, int rec, bool need_t2, float t2, Stats* st)
{
    for (;;) {
        float tn;
        if (st) st->c[RT_STAT_VERIFY]++;
        if (!slab_test(load_node(S.nodes, (uint32_t)rec), K, tn)) return false;
        const int p = S.parent[rec];
        if (p < 0) return true;
        if (need_t2 && !(t2 >= tn)) return false;
        if (S.chain_monotone) return true;
        rec = p;
    }
}

// Closest-hit query answered through the BVH and verified against the
// octree. Returns false when the answer must come from the exact walk.
template <class STK>
RT_HD bool fast_query_closest(const RtSceneView& S, V3 o, V3 d, STK& stk, float& t_out, int& k_out, Stats* st)
{
    FastHit h;
    fast_closest(S, o, d, stk, h, st);
    if (h.ovf) return false;
    if (h.k < 0) {  // no M-T hit anywhere: the reference finds none either
        t_out = -1.0f;
        k_out = -1;
        return true;
    }
    if (h.tie) return false;
    RayK K;
    ray_setup(o, d, K);
    const float t2 = __builtin_fminf(h.t2, h.t + h.t * RT_T2_WINDOW);
    if (!chain_ok(S, K, h.leaf, true, t2, st)) return false;
    t_out = h.t;
    k_out = h.k;
    return true;
}

// Occlusion query (exact; needs no fallback): is there an M-T-hit triangle
// whose octree leaf the reference's walk reaches?
template <class STK>
RT_HD int fast_query_any(const RtSceneView& S, V3 o, V3 d, STK& stk, Stats* st)
{
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) return 0;
    const RayB rb = rayb_setup(o, d);
    RayK K;
    bool kset = false;
    int sp = 0;
    int cur = 0;
    for (;;) {
        const BvhNodeR n = load_bvh(S.bvh, cur);
        if (st) st->c[RT_STAT_ANY_VOL] += 2;
        float tl, tr;
        const bool hl = n.lcount >= 0 && box_hit(n.lmin, n.lmax, rb, __builtin_inff(), tl);
        const bool hr = n.rcount >= 0 && box_hit(n.rmin, n.rmax, rb, __builtin_inff(), tr);
        for (int side = 0; side < 2; side++) {
            const bool hit = side ? hr : hl;
            const int cnt = side ? n.rcount : n.lcount;
            if (!hit || cnt == 0) continue;
            const int first = side ? n.right : n.left;
            if (st) st->c[RT_STAT_ANY_TRI] += cnt;
            for (int j = 0; j < cnt; j++) {
                float t;
                if (tri_test(S.bvh_tri4, first + j, o, d, t)) {
                    if (!kset) {
                        ray_setup(o, d, K);
                        kset = true;
                    }
                    if (chain_ok(S, K, (int)rt_asuint(S.bvh_tri4[3 * (first + j) + 1].w), false, 0.0f, st)) return 1;
                }
            }
        }
        const bool il = hl && n.lcount == 0, ir = hr && n.rcount == 0;
        int next = -1;
        if (il && ir) {
            const bool lfirst = tl <= tr;
            next = lfirst ? n.left : n.right;
            if (sp == STK::CAP) return -1;
            stk.set_rec(sp++, (uint32_t)(lfirst ? n.right : n.left));
        } else if (il) {
            next = n.left;
        } else if (ir) {
            next = n.right;
        }
        if (next >= 0) {
            cur = next;
            continue;
        }
        if (sp == 0) return 0;
        cur = (int)stk.rec(--sp);
    }
}

// Plain-array node-index stack (host build).
template <int N>
struct IdxStack {
    static constexpr int CAP = N;
    uint32_t r[N];
    RT_HD uint32_t rec(int i) const { return r[i]; }
    RT_HD void set_rec(int i, uint32_t v) { r[i] = v; }
};

}  // namespace rtk
