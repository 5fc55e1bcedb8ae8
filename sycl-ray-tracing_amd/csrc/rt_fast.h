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
#ifndef RT_BOX_FMA
#define RT_BOX_FMA 1  // device box test with fused multiply-adds (cfg2: 824-833 vs 819-825 Msamples/s, 3 A/B pairs)
#endif
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
#if defined(__HIP_DEVICE_COMPILE__) && RT_BOX_FMA
        // (one rounding instead of two: the padding covers either; entry distances only
        // order the visits, the answer is the verified closest hit either way)
        const float a = __builtin_fmaf(mn[i], r.inv[i], r.oi[i]), b = __builtin_fmaf(mx[i], r.inv[i], r.oi[i]);
#else
        const float a = mn[i] * r.inv[i] + r.oi[i], b = mx[i] * r.inv[i] + r.oi[i];
#endif
        t0 = __builtin_fmaxf(t0, __builtin_fminf(a, b));
        t1 = __builtin_fminf(t1, __builtin_fmaxf(a, b));
    }
    tnear = t0;
    return t0 <= t1 && t1 >= 0.0f;
}

// Entry and exit distances of a box (box_hit's arithmetic) for the slab test below.
RT_HD bool box_hit2(const float* mn, const float* mx, const RayB& r, float tmax, float& tnear, float& tfar)
{
    float t0 = -__builtin_inff(), t1 = tmax;
#pragma unroll
    for (int i = 0; i < 3; i++) {
#if defined(__HIP_DEVICE_COMPILE__) && RT_BOX_FMA
        const float a = __builtin_fmaf(mn[i], r.inv[i], r.oi[i]), b = __builtin_fmaf(mx[i], r.inv[i], r.oi[i]);
#else
        const float a = mn[i] * r.inv[i] + r.oi[i], b = mx[i] * r.inv[i] + r.oi[i];
#endif
        t0 = __builtin_fmaxf(t0, __builtin_fminf(a, b));
        t1 = __builtin_fminf(t1, __builtin_fmaxf(a, b));
    }
    tnear = t0;
    tfar = t1;
    return t0 <= t1 && t1 >= 0.0f;
}

// f16 bits -> f32 (the slab normals: finite, |x| <= 1)
RT_HD float rt_half(uint32_t h)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
#else
    const uint32_t e = (h >> 10) & 31u, m = h & 1023u;
    const float mag = e == 0 ? (float)m * 0x1p-24f : (float)(1024u + m) * __builtin_ldexpf(1.0f, (int)e - 25);
    return (h & 0x8000u) ? -mag : mag;
#endif
}

// Oriented slab of a search-BVH child (rt_scene.cpp build_slabs): s = {normal x | y << 16 and
// z as f16 bits, lo, hi}. The ray's segment [max(t0, 0), t1] inside the child's box can only
// reach a triangle of the child if it meets {lo <= n.x <= hi}; false when the whole segment
// lies on one side. Conservative: the host's margin covers this f32 arithmetic for a ray
// whose origin lies in the near box (far_origin below; DESIGN.md §4 "Far origins and grazing
// hits"), the only rays the search BVH answers; a child without a slab has n = 0, lo = -inf, hi = +inf
// (and a NaN from inf * 0 only drops that endpoint: fmin / fmax).
#ifndef RT_SLABS
#define RT_SLABS 1
#endif
RT_HD bool slab_ok(const float4_& s, V3 o, V3 d, float t0, float t1)
{
    const uint32_t w = rt_asuint(s.x);
    const float nx = rt_half(w & 0xffffu), ny = rt_half(w >> 16), nz = rt_half(rt_asuint(s.y) & 0xffffu);
#if defined(__HIP_DEVICE_COMPILE__)
    const float no = __builtin_fmaf(nz, o.z, __builtin_fmaf(ny, o.y, nx * o.x));
    const float nd = __builtin_fmaf(nz, d.z, __builtin_fmaf(ny, d.y, nx * d.x));
    const float p0 = __builtin_fmaf(__builtin_fmaxf(t0, 0.0f), nd, no), p1 = __builtin_fmaf(t1, nd, no);
#else
    const float no = nx * o.x + ny * o.y + nz * o.z, nd = nx * d.x + ny * d.y + nz * d.z;
    const float p0 = no + __builtin_fmaxf(t0, 0.0f) * nd, p1 = no + t1 * nd;
#endif
    return !(__builtin_fmaxf(p0, p1) < s.z || __builtin_fminf(p0, p1) > s.w);
}

struct Bvh4R {
    float lo[3][4], hi[3][4];
    int32_t ref[4], cnt[4];
};
// Child c of a node is records 2c ({lo.xyz, hi.x}) and 2c + 1 ({hi.yz, ref, cnt}).
RT_HD Bvh4R bvh4_unpack(const float4_* q)
{
    Bvh4R n;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float4_ a = q[2 * c], b = q[2 * c + 1];
        n.lo[0][c] = a.x, n.lo[1][c] = a.y, n.lo[2][c] = a.z;
        n.hi[0][c] = a.w, n.hi[1][c] = b.x, n.hi[2][c] = b.y;
        n.ref[c] = (int32_t)rt_asuint(b.z);
        n.cnt[c] = (int32_t)rt_asuint(b.w);
    }
    return n;
}
RT_HD Bvh4R load_bvh4(const Bvh4Node* nodes, int i)
{
    const float4_* p = (const float4_*)(nodes + i);
    float4_ q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = p[j];
    return bvh4_unpack(q);
}

// The four child boxes of a node: entry distance and "passes within [0, tmax]".
// (and their oriented slabs, slab_ok, when the scene has them: node's records S.bvh4s[4 node + c])
RT_HD void box4(const RtSceneView& S, int node, const Bvh4R& n, const RayB& r, V3 o, V3 d, float tmax, float* tn,
                bool* hit)
{
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float mn[3] = {n.lo[0][c], n.lo[1][c], n.lo[2][c]}, mx[3] = {n.hi[0][c], n.hi[1][c], n.hi[2][c]};
        float tf;
        hit[c] = n.cnt[c] >= 0 && box_hit2(mn, mx, r, tmax, tn[c], tf);
        if (RT_SLABS && hit[c] && S.bvh4s) hit[c] = slab_ok(S.bvh4s[4 * (size_t)node + c], o, d, tn[c], tf);
    }
}

// A leaf's triangle records (count <= 4, contiguous in bvh_tri4), all
// loaded before any is tested: one memory round trip per leaf.
struct LeafTris {
    float4_ a[4], e1[4], e2[4];
};
RT_HD void load_leaf(const RtSceneView& S, int first, int count, LeafTris& L)
{
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int i = first + (j < count ? j : count - 1);
        L.a[j] = S.bvh_tri4[3 * i];
        L.e1[j] = S.bvh_tri4[3 * i + 1];
        L.e2[j] = S.bvh_tri4[3 * i + 2];
    }
}

// Sorts four (key, value) pairs by key, ascending (5 compare-exchanges).
RT_HD void sort4(float* k, int* v)
{
    auto cx = [&](int i, int j) {
        if (k[j] < k[i]) {
            const float tk = k[i];
            k[i] = k[j];
            k[j] = tk;
            const int tv = v[i];
            v[i] = v[j];
            v[j] = tv;
        }
    };
    cx(0, 1);
    cx(2, 3);
    cx(0, 2);
    cx(1, 3);
    cx(1, 2);
}

// Relative width of the window past t* in which other hits are collected.
#ifndef RT_T2_WINDOW
#define RT_T2_WINDOW 1.0e-5f  // (cfg2 r02: 1e-3 / 1e-4 / 1e-5 -> closest box tests 3.571 / 3.544 / 3.540 G, fallbacks 375 each; 828-832 / 833 / 833-836 Msamples/s)
#endif

// Search-BVH walk: 1 = one item (node or leaf) per trip (fast_closest_u /
// fast_any_u), 0 = one node per trip with its leaf children inline.
#ifndef RT_FAST_WALK_C
#define RT_FAST_WALK_C 0
#endif
#ifndef RT_FAST_WALK_A
#define RT_FAST_WALK_A 1
#endif

struct FastHit {
    float t, t2;  // closest M-T hit (-1: none), smallest other hit distance above t seen (window-bounded)
    int k;        // leaf-order triangle of t (among triangles tied at t in one octree leaf: the first in its list)
    int leaf;     // its octree leaf record
    bool tie;     // another triangle hit at exactly t in another octree leaf (brute force: anywhere)
    bool ovf;     // the bounded stack overflowed: answer unknown
    int prim;     // brute-force mode: original index of t's triangle, the lowest among the ties
};

// One M-T hit (t, leaf-order k, octree leaf, original index prim) into h: closest, second
// distance, ties. Triangles tied at t inside ONE octree leaf are settled here: the reference
// visits that leaf once and takes the first of them in its list (strict `<`, bvh.h:150-161),
// i.e. the lowest leaf-order k (flatten_octree writes each leaf's list in order); ties across
// leaves depend on its heap order, so they flag `tie` (the exact walk answers). In brute-force
// mode (USE_BVH 0) a tie goes to the lowest original index, as the reference's loop does.
RT_HD void fast_take(FastHit& h, float t, int k, int leaf, int prim, bool brute)
{
    if (t < h.t) {
        h.t2 = h.t;
        h.t = t;
        h.k = k;
        h.leaf = leaf;
        h.prim = prim;
        h.tie = false;
    } else if (t == h.t) {
        if (brute) {
            h.tie = true;
            if (prim < h.prim) {
                h.k = k;
                h.leaf = leaf;
                h.prim = prim;
            }
        } else if (leaf == h.leaf) {
            if (k < h.k) {
                h.k = k;
                h.prim = prim;
            }
        } else {
            h.tie = true;
        }
    } else if (t < h.t2) {
        h.t2 = t;
    }
}

RT_HD void fast_leaf(const RtSceneView& S, int first, int count, V3 o, V3 d, FastHit& h, Stats* st)
{
    LeafTris L;
    load_leaf(S, first, count, L);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (j >= count) break;
        float t;
        if (tri_test_v(ld3(L.a[j]), ld3(L.e1[j]), ld3(L.e2[j]), o, d, t))
            fast_take(h, t, (int)rt_asuint(L.a[j].w), (int)rt_asuint(L.e1[j].w), (int)rt_asuint(L.e2[j].w), S.brute != 0);
    }
    if (st) st->c[RT_STAT_TRI] += count;
}

// All M-T hits within [0, t*(1 + RT_T2_WINDOW)]: closest, tie flag, second.
// The result does not depend on the visiting order (every box holding a hit
// in the final window is entered: the window only shrinks, to the final
// one), so the walk is free to go nearest-first and to drop stack entries
// the window has closed behind.
// STK: CAP entries, rec(i) / key(i) / set(i, rec, key).
template <class STK>
RT_HD void fast_closest(const RtSceneView& S, V3 o, V3 d, STK& stk, FastHit& h, Stats* st)
{
    h.t = __builtin_inff();
    h.t2 = __builtin_inff();
    h.k = -1;
    h.prim = 0x7fffffff;
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
        const Bvh4R n = load_bvh4(S.bvh4, cur);
        if (st) st->c[RT_STAT_VOL] += 4;
        float tn[4];
        bool hit[4];
        box4(S, cur, n, rb, o, d, h.t + h.t * RT_T2_WINDOW, tn, hit);
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (hit[c] && n.cnt[c] > 0) fast_leaf(S, n.ref[c], n.cnt[c], o, d, h, st);
        const float tmax = h.t + h.t * RT_T2_WINDOW;  // (the leaves may have narrowed it)
        float k[4];
        int v[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const bool open = hit[c] && n.cnt[c] == 0 && tn[c] <= tmax;
            k[c] = open ? tn[c] : __builtin_inff();
            v[c] = open ? n.ref[c] : -1;
        }
        sort4(k, v);
        // far children on the stack (nearest of them on top), nearest next
#pragma unroll
        for (int j = 3; j >= 1; j--)
            if (v[j] >= 0) {
                if (sp == STK::CAP) {
                    h.ovf = true;
                    return;
                }
                stk.set(sp++, (uint32_t)v[j], k[j]);
            }
        if (v[0] >= 0) {
            cur = v[0];
            continue;
        }
        // pop, dropping entries the window has closed behind
        cur = -1;
        while (sp > 0) {
            --sp;
            if (stk.key(sp) <= tmax) {
                cur = (int)stk.rec(sp);
                break;
            }
        }
        if (cur < 0) break;
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

// ---------------------------------------------------------------------------
// One-item-per-trip walks. Inner nodes and leaves are both stack items; each
// trip of the loop loads one item with the same load instructions (an inner
// node's 8 records or a leaf's 3 * count triangle records, from either array)
// and then runs the box tests or the triangle tests on it. A wave whose lanes
// mix nodes and leaves pays one memory round trip per trip instead of one per
// leaf child of the node (fast_closest above tests a node's leaf children in
// four divergent branches, each with its own round trip).
// Item encoding: node index i >= 0; leaf ~((first << 2) | (count - 1)) < 0.
RT_HD int leaf_item(int first, int count) { return ~((first << 2) | (count - 1)); }

struct ItemRecs {
    float4_ q[12];
};
RT_HD void load_item(const RtSceneView& S, int item, ItemRecs& R)
{
    const bool leaf = item < 0;
    const int v = ~item;
    const float4_* p = leaf ? S.bvh_tri4 + 3 * (v >> 2) : (const float4_*)(S.bvh4 + item);
    const int nrec = leaf ? 3 * ((v & 3) + 1) : 8;
#pragma unroll
    for (int j = 0; j < 12; j++)
        if (j < nrec) R.q[j] = p[j];
}
RT_HD Bvh4R node_of(const ItemRecs& R)
{
    return bvh4_unpack(R.q);
}

// fast_closest, one item per trip (same result: the set of hits in the final
// window does not depend on the visiting order).
template <class STK>
RT_HD void fast_closest_u(const RtSceneView& S, V3 o, V3 d, STK& stk, FastHit& h, Stats* st)
{
    h.t = __builtin_inff();
    h.t2 = __builtin_inff();
    h.k = -1;
    h.prim = 0x7fffffff;
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
        ItemRecs R;
        load_item(S, cur, R);
        if (cur >= 0) {
            const Bvh4R n = node_of(R);
            if (st) st->c[RT_STAT_VOL] += 4;
            float tn[4];
            bool hit[4];
            const float tmax = h.t + h.t * RT_T2_WINDOW;
            box4(S, cur, n, rb, o, d, tmax, tn, hit);
            float k[4];
            int v[4];
            bool ok[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                ok[c] = hit[c] && tn[c] <= tmax;
                k[c] = ok[c] ? tn[c] : __builtin_inff();
                v[c] = n.cnt[c] > 0 ? leaf_item(n.ref[c], n.cnt[c]) : n.ref[c];
            }
            // sort the valid children by entry distance (invalid keys are +inf)
            int ix[4] = {0, 1, 2, 3};
            float kk[4] = {k[0], k[1], k[2], k[3]};
            sort4(kk, ix);
            int nv = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) nv += ok[c] ? 1 : 0;
            // far children on the stack (nearest of them on top), nearest next
            bool over = false;
#pragma unroll
            for (int j = 3; j >= 1; j--)
                if (j < nv) {
                    if (sp == STK::CAP)
                        over = true;
                    else
                        stk.set(sp++, (uint32_t)v[ix[j]], kk[j]);
                }
            if (over) {
                h.ovf = true;
                return;
            }
            if (nv > 0) {
                cur = v[ix[0]];
                continue;
            }
        } else {
            const int cnt = ((~cur) & 3) + 1;
            if (st) st->c[RT_STAT_TRI] += cnt;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (j >= cnt) break;
                float t;
                if (tri_test_v(ld3(R.q[3 * j]), ld3(R.q[3 * j + 1]), ld3(R.q[3 * j + 2]), o, d, t))
                    fast_take(h, t, (int)rt_asuint(R.q[3 * j].w), (int)rt_asuint(R.q[3 * j + 1].w),
                              (int)rt_asuint(R.q[3 * j + 2].w), S.brute != 0);
            }
        }
        // pop, dropping entries the window has closed behind
        const float tmax = h.t + h.t * RT_T2_WINDOW;
        cur = 0x7fffffff;
        while (sp > 0) {
            --sp;
            if (stk.key(sp) <= tmax) {
                cur = (int)stk.rec(sp);
                break;
            }
        }
        if (cur == 0x7fffffff) break;
    }
    if (h.k < 0) h.t = -1.0f;
}

// fast_query_any, one item per trip.
template <class STK>
RT_HD int fast_any_u(const RtSceneView& S, V3 o, V3 d, STK& stk, Stats* st)
{
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) return 0;
    const RayB rb = rayb_setup(o, d);
    RayK K;
    bool kset = false;
    int sp = 0;
    int cur = 0;
    for (;;) {
        ItemRecs R;
        load_item(S, cur, R);
        bool have = false;
        if (cur >= 0) {
            const Bvh4R n = node_of(R);
            if (st) st->c[RT_STAT_ANY_VOL] += 4;
            float tn[4];
            bool hit[4];
            box4(S, cur, n, rb, o, d, __builtin_inff(), tn, hit);
            bool over = false;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                if (!hit[c]) continue;
                const int it = n.cnt[c] > 0 ? leaf_item(n.ref[c], n.cnt[c]) : n.ref[c];
                if (!have) {
                    cur = it;
                    have = true;
                } else if (sp == STK::CAP) {
                    over = true;
                } else {
                    stk.set(sp++, (uint32_t)it, 0.0f);
                }
            }
            if (over) return -1;
        } else {
            const int cnt = ((~cur) & 3) + 1;
            if (st) st->c[RT_STAT_ANY_TRI] += cnt;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (j >= cnt) break;
                float t;
                if (tri_test_v(ld3(R.q[3 * j]), ld3(R.q[3 * j + 1]), ld3(R.q[3 * j + 2]), o, d, t)) {
                    if (S.brute) return 1;  // USE_BVH 0: any triangle hit occludes
                    if (!kset) {
                        ray_setup(o, d, K);
                        kset = true;
                    }
                    if (chain_ok(S, K, (int)rt_asuint(R.q[3 * j + 1].w), false, 0.0f, st)) return 1;
                }
            }
        }
        if (have) continue;
        if (sp == 0) return 0;
        cur = (int)stk.rec(--sp);
    }
}

// ---------------------------------------------------------------------------
// Where the search BVH's answer cannot be trusted ("Far origins and grazing
// hits"). Moller-Trumbore (triangle.h:24-44) computes s = o - a and then u = f (s.h),
// v = f (d.q), t = f (e2.q): the rounding of the dot products is ~eps |s| |d| |e| while
// det = e1.(d x e2) = |d| |e1 x e2| cos(theta) can be as small as 1e-7 (its only guard). The
// u + v <= 1 and u <= 1 tests (and t) then carry an error of ~eps |s| / (sin(alpha) cos(theta)) in
// space: the reference accepts rays that pass outside the triangle by that much. The search
// BVH's boxes are padded by 1e-4 of their coordinates' magnitude (rt_scene.cpp pad_box), which
// covers it only while |s| and the grazing factor stay moderate. Two cases go to the exact walk:
//  * far_origin: the ray starts outside the near box (the scene's box widened by RT_NEAR_SCALE x
//    its largest extent): |s| is unbounded there (profiles/r06_far_probe.json);
//  * fuzzy_hit (RT_FUZZ_CHECK builds; off in the product): the found hit's own Moller-Trumbore
//    fuzz eps |s| |d| |e1| |e2| / |det| exceeds RT_FUZZ_TAU x its box pad. A neighbour the walk
//    did not enter (its fuzz beyond its pad) is usually a grazing triangle of the same surface,
//    and the found hit then shares that conditioning. Measured (profiles/r06_far_origin.json):
//    it removes most of the near grazing misses of the probe but costs cfg2 4 % at tau 1 (2 %
//    the leaf-test arithmetic, 1.5 % the extra exact walks of grazing rays), so it stays off.
#ifndef RT_FUZZ_CHECK
#define RT_FUZZ_CHECK 0
#endif
#ifndef RT_FUZZ_TAU
#define RT_FUZZ_TAU 1.0f
#endif
RT_HD bool far_origin(const RtSceneView& S, V3 o)
{
    return o.x < S.near_lo[0] || o.x > S.near_hi[0] || o.y < S.near_lo[1] || o.y > S.near_hi[1] ||
           o.z < S.near_lo[2] || o.z > S.near_hi[2];
}
// Is the Moller-Trumbore answer for leaf-order triangle k (records a, e1, e2) fuzzier than
// RT_FUZZ_TAU x the pad of its box? (squares: no division, no square root)
RT_HD bool fuzzy_tri(float4_ ra, float4_ r1, float4_ r2, V3 o, V3 d)
{
    const V3 a = ld3(ra), e1 = ld3(r1), e2 = ld3(r2);
    const float det = dot(e1, cross(d, e2));
    const V3 s = sub(o, a);
    auto amax = [](V3 v) { return __builtin_fmaxf(__builtin_fabsf(v.x), __builtin_fmaxf(__builtin_fabsf(v.y), __builtin_fabsf(v.z))); };
#ifdef RT_FUZZ_LITE
    const float m = __builtin_fmaxf(1.0f, amax(a));  // (<= the box's magnitude: flags a little more)
#else
    const float m = __builtin_fmaxf(__builtin_fmaxf(1.0f, amax(a)), __builtin_fmaxf(amax(add(a, e1)), amax(add(a, e2))));
#endif
    constexpr float c = 5.9604645e-8f / (1e-4f * RT_FUZZ_TAU);  // eps / (pad per unit magnitude x tau)
    const float lhs = (c * c) * dot(s, s) * dot(d, d) * dot(e1, e1) * dot(e2, e2);
    return !(lhs <= (m * m) * (det * det));  // (a NaN goes to the exact walk too)
}
// (device walks: quad_tri marks a fuzzy hit's octree leaf record with this bit; records < 2^30)
#define RT_FZ_BIT 0x40000000
RT_HD bool fuzzy_hit(const RtSceneView& S, int k, V3 o, V3 d)
{
    const float4_* r = S.tri4 + 3 * (size_t)k;
    return fuzzy_tri(r[0], r[1], r[2], o, d);
}


// Closest-hit query answered through the BVH and verified against the
// octree. Returns false when the answer must come from the exact walk.
template <class STK, int WALK = RT_FAST_WALK_C>
RT_HD bool fast_query_closest(const RtSceneView& S, V3 o, V3 d, STK& stk, float& t_out, int& k_out, Stats* st)
{
    if (far_origin(S, o)) return false;
    FastHit h;
    if (WALK == 1)
        fast_closest_u(S, o, d, stk, h, st);
    else
        fast_closest(S, o, d, stk, h, st);
    if (h.ovf) return false;
    if (h.k < 0) {  // no M-T hit anywhere: the reference finds none either
        t_out = -1.0f;
        k_out = -1;
        return true;
    }
    if (RT_FUZZ_CHECK && fuzzy_hit(S, h.k, o, d)) return false;
    if (S.brute) {  // USE_BVH 0: the closest M-T hit, lowest index on ties; no octree
        t_out = h.t;
        k_out = h.k;
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
// whose octree leaf the reference's walk reaches? 1 / 0; -1 when the
// bounded stack overflowed (answer unknown).
template <class STK, int WALK = RT_FAST_WALK_A>
RT_HD int fast_query_any(const RtSceneView& S, V3 o, V3 d, STK& stk, Stats* st)
{
    if (far_origin(S, o)) return -1;
    if (WALK == 1) return fast_any_u(S, o, d, stk, st);
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) return 0;
    const RayB rb = rayb_setup(o, d);
    RayK K;
    bool kset = false;
    int sp = 0;
    int cur = 0;
    for (;;) {
        const Bvh4R n = load_bvh4(S.bvh4, cur);
        if (st) st->c[RT_STAT_ANY_VOL] += 4;
        float tn[4];
        bool hit[4];
        box4(S, cur, n, rb, o, d, __builtin_inff(), tn, hit);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (!hit[c] || n.cnt[c] <= 0) continue;
            const int cnt = n.cnt[c];
            if (st) st->c[RT_STAT_ANY_TRI] += cnt;
            LeafTris L;
            load_leaf(S, n.ref[c], cnt, L);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (j >= cnt) break;
                float t;
                if (tri_test_v(ld3(L.a[j]), ld3(L.e1[j]), ld3(L.e2[j]), o, d, t)) {
                    if (S.brute) return 1;  // USE_BVH 0: any triangle hit occludes
                    if (!kset) {
                        ray_setup(o, d, K);
                        kset = true;
                    }
                    if (chain_ok(S, K, (int)rt_asuint(L.e1[j].w), false, 0.0f, st)) return 1;
                }
            }
        }
        cur = -1;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (!hit[c] || n.cnt[c] != 0) continue;
            if (cur < 0) {
                cur = n.ref[c];
            } else {
                if (sp == STK::CAP) return -1;
                stk.set(sp++, (uint32_t)n.ref[c], 0.0f);
            }
        }
        if (cur >= 0) continue;
        if (sp == 0) return 0;
        cur = (int)stk.rec(--sp);
    }
}

// Plain-array node stack with keys (host build).
template <int N>
struct IdxStack {
    static constexpr int CAP = N;
    uint32_t r[N];
    float k[N];
    RT_HD uint32_t rec(int i) const { return r[i]; }
    RT_HD float key(int i) const { return k[i]; }
    RT_HD void set(int i, uint32_t v, float kv) { r[i] = v, k[i] = kv; }
};

}  // namespace rtk
