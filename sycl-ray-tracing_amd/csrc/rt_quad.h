// rt_quad.h — search-BVH queries walked by a quad of lanes (gfx950 only).
//
// The one-lane walks of rt_fast.h execute, for every trip of the wave, the
// box tests of a node and (unrolled) the Moller-Trumbore tests of all of its
// leaf children: whenever any of the 64 lanes needs a branch the whole wave
// pays for it, so a node visit costs ~2000 wave instructions (~3-4 us per
// visit measured on an idle MI355X, tools/chunk_trace.py). A query's latency
// sets how fast a pixel's 64 x (bounces + 1) dependent steps can go, which
// bounds the frame when few pixels are left (and at 8 GPUs, always).
//
// Here four consecutive lanes (a quad) walk one query together:
//  * inner node: lane j loads child j (two 16-B loads of its 32-B record,
//    rt_device.h Bvh4Child) and runs one box test; the quad ranks the hits
//    by entry distance through DPP quad permutes, the nearest becomes the
//    next item and the others are pushed (each lane writes its own entry);
//  * leaf: lane j runs the reference's Moller-Trumbore test on triangle j;
//    the quad reduces (closest, second, tie) with DPP.
// Every trip is one memory round trip and ~1/10 of the instructions. The
// answer is the one rt_fast.h defines (same window, same tie / second-hit
// bookkeeping, same verification), so the query falls back to the exact
// octree walk in exactly the same cases.
//
// Contract: all four lanes of a quad call these functions together with the
// same ray, in quad-uniform control flow (DPP reads the other lanes).
#pragma once

#include "rt_fast.h"

namespace rtk {

#define RT_QX1 0xB1  // quad_perm [1,0,3,2]: lane j ^ 1
#define RT_QX2 0x4E  // quad_perm [2,3,0,1]: lane j ^ 2
#define RT_QX3 0x1B  // quad_perm [3,2,1,0]: lane j ^ 3

template <int CTRL>
__device__ __forceinline__ int qdpp(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float qdppf(float v)
{
    return __int_as_float(qdpp<CTRL>(__float_as_int(v)));
}
// Is lane sub ^ x below lane sub?
__device__ __forceinline__ bool s_lower(int sub, int x) { return (sub ^ x) < sub; }
// OR over the quad (used to broadcast the value of the one lane that holds it, others 0)
__device__ __forceinline__ int qor(int v)
{
    v |= qdpp<RT_QX1>(v);
    return v | qdpp<RT_QX2>(v);
}
__device__ __forceinline__ int qsum(int v)
{
    v += qdpp<RT_QX1>(v);
    return v + qdpp<RT_QX2>(v);
}

// Per-quad stack in LDS: entry i of quad q at [i * QPB + q].
template <int N, int QPB>
struct QuadStack {
    static constexpr int CAP = N;
    uint32_t* r;  // base + q
    float* k;
    __device__ __forceinline__ uint32_t rec(int i) const { return r[i * QPB]; }
    __device__ __forceinline__ float key(int i) const { return k[i * QPB]; }
    __device__ __forceinline__ void set(int i, uint32_t rv, float kv)
    {
        r[i * QPB] = rv;
        k[i * QPB] = kv;
    }
    __device__ __forceinline__ void set_rec(int i, uint32_t rv) { r[i * QPB] = rv; }
};

// LDS-staged top of the search BVH: the first RT_TOP_NODES nodes (breadth-first,
// rt_scene.cpp bvh4_top_first), copied once per block; every walk starts there,
// so its first trips read LDS instead of L2.
// Measured on cfg2 (r02): 0 / 21 / 32 / 64 nodes: 676 / 676 / 675 / 666 Msamples/s (the
// top levels stay L2-resident anyway), so it is off by default.
#ifndef RT_TOP_NODES
#define RT_TOP_NODES 0
#endif
__device__ __forceinline__ float4_* top_nodes()
{
    __shared__ float4_ s_top[RT_TOP_NODES > 0 ? RT_TOP_NODES * 8 : 1];
    return s_top;
}
// Copies the top nodes (whole block; ends with a barrier) and returns the count staged.
__device__ __forceinline__ int top_nodes_stage(const RtSceneView& S)
{
    const int n = min(S.bvh4_ntop, RT_TOP_NODES);
    float4_* t = top_nodes();
    const float4_* g = (const float4_*)S.bvh4;
    for (int i = (int)threadIdx.x; i < 8 * n; i += (int)blockDim.x) t[i] = g[i];
    __syncthreads();
    return n;
}
// Lane sub's 32-B child record of inner node `node` (LDS when staged).
__device__ __forceinline__ void child_record(const RtSceneView& S, int node, int sub, float4_& a, float4_& b)
{
    if (RT_TOP_NODES > 0 && node < S.bvh4_top) {
        const float4_* q = top_nodes() + 8 * node + 2 * sub;
        a = q[0];
        b = q[1];
    } else {
        const float4_* p = (const float4_*)(S.bvh4 + node) + 2 * sub;
        a = p[0];
        b = p[1];
    }
}

// Lane `sub`'s child of inner node `node`: box test within [0, tmax].
struct QChild {
    int item;  // node index or leaf item (rt_fast.h leaf_item)
    bool ok;
    float tn;
};
__device__ __forceinline__ QChild quad_child(const RtSceneView& S, int node, int sub, const RayB& rb, float tmax)
{
    float4_ a, b;
    child_record(S, node, sub, a, b);
    rt_pin(a);
    rt_pin(b);
    const int ref = (int)rt_asuint(b.z), cnt = (int)rt_asuint(b.w);
    const float mn[3] = {a.x, a.y, a.z}, mx[3] = {a.w, b.x, b.y};
    QChild c;
    c.ok = cnt >= 0 && box_hit(mn, mx, rb, tmax, c.tn) && c.tn <= tmax;
    c.item = cnt > 0 ? leaf_item(ref, cnt) : ref;
    return c;
}

// Lane `sub`'s triangle of a leaf item: Moller-Trumbore (the reference's
// arithmetic). Returns t (+inf when the lane has no triangle or no hit).
__device__ __forceinline__ float quad_tri(const RtSceneView& S, int item, int sub, V3 o, V3 d, int& k, int& leaf,
                                          int& prim)
{
    const int v = ~item;
    const int first = v >> 2, cnt = (v & 3) + 1;
    float tv = __builtin_inff();
    k = -1;
    leaf = -1;
    prim = 0x7fffffff;
    if (sub < cnt) {
        const float4_* p = S.bvh_tri4 + 3 * (first + sub);
        const float4_ a = p[0], e1 = p[1], e2 = p[2];
        rt_pin(a);
        rt_pin(e1);
        rt_pin(e2);
        float t;
        if (tri_test_v(ld3(a), ld3(e1), ld3(e2), o, d, t)) {
            tv = t;
            k = (int)rt_asuint(a.w);
            leaf = (int)rt_asuint(e1.w);
            prim = (int)rt_asuint(e2.w);
        }
    }
    return tv;
}

// fast_closest (rt_fast.h) walked by a quad. h is quad-uniform on return.
template <class QSTK>
__device__ void quad_closest(const RtSceneView& S, V3 o, V3 d, QSTK& stk, int sub, FastHit& h, Stats* st)
{
    h.t = __builtin_inff();
    h.t2 = __builtin_inff();
    h.k = -1;
    h.leaf = -1;
    h.prim = 0x7fffffff;
    h.tie = false;
    h.ovf = false;
    if (st && sub == 0) st->c[RT_STAT_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) {
        h.t = -1.0f;
        return;
    }
    const RayB rb = rayb_setup(o, d);
    int sp = 0;
    int cur = 0;
    for (;;) {
        if (cur >= 0) {
            if (st && sub == 0) st->c[RT_STAT_VOL] += 4;
            const float tmax = h.t + h.t * RT_T2_WINDOW;
            const QChild c = quad_child(S, cur, sub, rb, tmax);
            const float key = c.ok ? c.tn : __builtin_inff();
            // rank by (key, lane): the nearest hit child has rank 0
            const float k1 = qdppf<RT_QX1>(key), k2 = qdppf<RT_QX2>(key), k3 = qdppf<RT_QX3>(key);
            const int s1 = sub ^ 1, s2 = sub ^ 2, s3 = sub ^ 3;
            const int rank = (k1 < key || (k1 == key && s1 < sub) ? 1 : 0) + (k2 < key || (k2 == key && s2 < sub) ? 1 : 0) +
                             (k3 < key || (k3 == key && s3 < sub) ? 1 : 0);
            const int nv = qsum(c.ok ? 1 : 0);
            if (sp + nv - 1 > QSTK::CAP) {
                h.ovf = true;
                return;
            }
            // far children on the stack, nearest of them on top (rank 1 at sp + nv - 2)
            if (c.ok && rank > 0) stk.set(sp + nv - 1 - rank, (uint32_t)c.item, key);
            if (nv > 0) {
                sp += nv - 1;
                cur = qor(c.ok && rank == 0 ? c.item : 0);
                continue;
            }
        } else {
            if (st && sub == 0) st->c[RT_STAT_TRI] += ((~cur) & 3) + 1;
            int k, leaf, prim;
            const float tv = quad_tri(S, cur, sub, o, d, k, leaf, prim);
            // quad (smallest, second smallest) of the lanes' hit distances
            float m1 = tv, m2 = __builtin_inff();
            {
                const float o1 = qdppf<RT_QX1>(m1), o2 = qdppf<RT_QX1>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            {
                const float o1 = qdppf<RT_QX2>(m1), o2 = qdppf<RT_QX2>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            // the lane holding m1 with the lowest original index (brute-force mode: the reference's
            // loop keeps the lowest index of a tie; octree mode: any tie falls back anyway)
            int pm = tv == m1 ? prim : 0x7fffffff;
            pm = min(pm, qdpp<RT_QX1>(pm));
            pm = min(pm, qdpp<RT_QX2>(pm));
            const bool mine = tv == m1 && prim == pm;
            if (m1 < h.t) {
                h.t2 = __builtin_fminf(h.t, m2);
                h.t = m1;
                h.k = qor(mine ? k : 0);
                h.leaf = qor(mine ? leaf : 0);
                h.prim = pm;
                h.tie = m2 == m1;
            } else if (m1 == h.t && m1 < __builtin_inff()) {
                h.tie = true;
                h.t2 = m1;
                if (pm < h.prim) {
                    h.k = qor(mine ? k : 0);
                    h.leaf = qor(mine ? leaf : 0);
                    h.prim = pm;
                }
            } else {
                h.t2 = __builtin_fminf(h.t2, m1);
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

// chain_ok (rt_fast.h) by a quad: lane j evaluates slab planes j and j + 4
// (the last lane only plane 3) with ray_setup's and slab_test's arithmetic,
// and the quad combines the running max / min. The reference's max / min
// (`(a < b) ? b : a`) never let a NaN quotient into the accumulator, which
// starts at -inf / +inf, so the combination order does not change the result
// (a +-0 can differ in sign, and only ever meets comparisons). rec is
// quad-uniform; the answer is returned to every lane.
__device__ __forceinline__ bool quad_chain_ok(const RtSceneView& S, V3 o, V3 d, int rec, bool need_t2, float t2,
                                              int sub, Stats* st)
{
    const float s3 = rt_sqrtf(3.0f) / 3;
    // the 7 plane normals of bvh.cpp:8-16 (ray_setup), selected without a private array
    auto normal = [&](int p) {
        if (p < 3) return v3(p == 0 ? 1.0f : 0.0f, p == 1 ? 1.0f : 0.0f, p == 2 ? 1.0f : 0.0f);
        return v3(p == 4 || p == 5 ? -s3 : s3, p == 5 || p == 6 ? -s3 : s3, s3);
    };
    const int p0 = sub, p1 = sub + 4;  // p1 == 7: none
    const V3 n0 = normal(p0), n1 = normal(p1 < 7 ? p1 : 0);
    const float num0 = dot(n0, o), num1 = dot(n1, o);
    const double r0 = 1.0 / (double)dot(n0, d), r1 = 1.0 / (double)dot(n1, d);
    for (;;) {
        if (st && sub == 0) st->c[RT_STAT_VERIFY]++;
        const float* nd = (const float*)(S.nodes + rec);  // RtNode: dn[7], df[7], ref, cnt
        const float dn0 = nd[p0], df0 = nd[7 + p0], dn1 = nd[p1 < 7 ? p1 : 0], df1 = nd[7 + (p1 < 7 ? p1 : 0)];
        const int par = S.parent[rec];
        rt_pin(dn0);
        rt_pin(df0);
        rt_pin(dn1);
        rt_pin(df1);
        rt_pin(par);
        float tn = -__builtin_inff(), tf = __builtin_inff();
        {
            const bool neg = r0 < 0.0;
            float a = slab_div((neg ? df0 : dn0) - num0, r0), b = slab_div((neg ? dn0 : df0) - num0, r0);
            if (__builtin_isinf(r0)) a = -__builtin_inff(), b = __builtin_inff();
            tn = rt_max(tn, a);
            tf = rt_min(tf, b);
        }
        if (p1 < 7) {
            const bool neg = r1 < 0.0;
            float a = slab_div((neg ? df1 : dn1) - num1, r1), b = slab_div((neg ? dn1 : df1) - num1, r1);
            if (__builtin_isinf(r1)) a = -__builtin_inff(), b = __builtin_inff();
            tn = rt_max(tn, a);
            tf = rt_min(tf, b);
        }
        tn = rt_max(tn, qdppf<RT_QX1>(tn));
        tn = rt_max(tn, qdppf<RT_QX2>(tn));
        tf = rt_min(tf, qdppf<RT_QX1>(tf));
        tf = rt_min(tf, qdppf<RT_QX2>(tf));
        if (tf < tn) return false;
        if (par < 0) return true;
        if (need_t2 && !(t2 >= tn)) return false;
        if (S.chain_monotone) return true;
        rec = par;
    }
}

// fast_query_closest by a quad: true with (t, k) when answered, false when
// the exact walk must answer (same cases as the one-lane walk).
template <class QSTK>
__device__ bool quad_query_closest(const RtSceneView& S, V3 o, V3 d, QSTK& stk, int sub, float& t_out, int& k_out,
                                   Stats* st)
{
    FastHit h;
    quad_closest(S, o, d, stk, sub, h, st);
    if (h.ovf) return false;
    if (h.k < 0) {
        t_out = -1.0f;
        k_out = -1;
        return true;
    }
    if (S.brute) {  // USE_BVH 0: the closest M-T hit, lowest index on ties; no octree
        t_out = h.t;
        k_out = h.k;
        return true;
    }
    if (h.tie) return false;
    const float t2 = __builtin_fminf(h.t2, h.t + h.t * RT_T2_WINDOW);
    if (!quad_chain_ok(S, o, d, h.leaf, true, t2, sub, st)) return false;
    t_out = h.t;
    k_out = h.k;
    return true;
}

// fast_query_any by a quad: 1 / 0, -1 when the bounded stack overflowed.
template <class QSTK>
__device__ int quad_query_any(const RtSceneView& S, V3 o, V3 d, QSTK& stk, int sub, Stats* st)
{
    if (st && sub == 0) st->c[RT_STAT_ANY_RAYS]++;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) return 0;
    const RayB rb = rayb_setup(o, d);
    int sp = 0;
    int cur = 0;
    for (;;) {
        bool have = false;
        if (cur >= 0) {
            if (st && sub == 0) st->c[RT_STAT_ANY_VOL] += 4;
            const QChild c = quad_child(S, cur, sub, rb, __builtin_inff());
            const int okb = c.ok ? 1 : 0;
            // exclusive prefix of the ok lanes: the first one is next, the rest are pushed
            const int o1 = qdpp<RT_QX1>(okb), o2 = qdpp<RT_QX2>(okb), o3 = qdpp<RT_QX3>(okb);
            const int pre = (s_lower(sub, 1) ? o1 : 0) + (s_lower(sub, 2) ? o2 : 0) + (s_lower(sub, 3) ? o3 : 0);
            const int nv = okb + o1 + o2 + o3;
            if (sp + nv - 1 > QSTK::CAP) return -1;
            if (c.ok && pre > 0) stk.set(sp + pre - 1, (uint32_t)c.item, 0.0f);
            if (nv > 0) {
                sp += nv - 1;
                cur = qor(c.ok && pre == 0 ? c.item : 0);
                have = true;
            }
        } else {
            if (st && sub == 0) st->c[RT_STAT_ANY_TRI] += ((~cur) & 3) + 1;
            int k, leaf, prim;
            const float tv = quad_tri(S, cur, sub, o, d, k, leaf, prim);
            const int hitb = tv < __builtin_inff() ? 1 : 0;
            if (S.brute) {
                if (qor(hitb)) return 1;  // USE_BVH 0: any triangle hit occludes
            } else {
                // each hit lane's octree leaf in turn, checked by the whole quad
                const int h1 = qdpp<RT_QX1>(hitb), h2 = qdpp<RT_QX2>(hitb), h3 = qdpp<RT_QX3>(hitb);
                const int l1 = qdpp<RT_QX1>(leaf), l2 = qdpp<RT_QX2>(leaf), l3 = qdpp<RT_QX3>(leaf);
#pragma unroll
                for (int j = 0; j < 4; j++) {  // quad lane j (same order in every lane)
                    const int x = j ^ sub;     // its distance in the xor pattern from this lane
                    const int hj = x == 0 ? hitb : x == 1 ? h1 : x == 2 ? h2 : h3;
                    if (!hj) continue;
                    const int lj = x == 0 ? leaf : x == 1 ? l1 : x == 2 ? l2 : l3;
                    if (quad_chain_ok(S, o, d, lj, false, 0.0f, sub, st)) return 1;
                }
            }
        }
        if (have) continue;
        if (sp == 0) return 0;
        cur = (int)stk.rec(--sp);
    }
}

// The whole-walk loops above, cut at trip boundaries and specialized by kind
// (ANY: quad_query_any's visit order and answer; else quad_closest's), so that
// k_trace can start a quad on its next query the moment its walk ends. One call
// is one trip: the same loads, tests and stack moves as one iteration of those
// loops, so the visits and answers are theirs.
struct QState {
    V3 o, d;
    RayB rb;
    FastHit h;
    int sp, cur;
    int bot;  // occlusion walks shared with other quads (k_trace drain): entries below bot were taken
    int calls;  // quad_visit calls so far (k_trace: the heavy-class prediction)
};

// false: the answer is already known (a NaN ray: no hit), no trip needed.
template <bool ANY>
__device__ __forceinline__ bool qstate_begin(QState& q, V3 o, V3 d, int sub, Stats* st)
{
    if (st && sub == 0) st->c[ANY ? RT_STAT_ANY_RAYS : RT_STAT_RAYS]++;
    q.o = o;
    q.d = d;
    q.h.t = __builtin_inff();
    q.h.t2 = __builtin_inff();
    q.h.k = ANY ? 0 : -1;
    q.h.leaf = -1;
    q.h.prim = 0x7fffffff;
    q.h.tie = false;
    q.h.ovf = false;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) {
        q.h.t = -1.0f;
        return false;
    }
    q.rb = rayb_setup(o, d);
    q.sp = 0;
    q.cur = 0;
    q.bot = 0;
    return true;
}

// One trip. 0: go on; 1: the walk is over (ANY: q.h.k = 1 occluded / 0 not; else the
// closest-hit record in q.h, to quad_closest_answer); -1: the bounded stack overflowed.
#ifndef RT_VISIT_DESCEND
#define RT_VISIT_DESCEND 2  // inner-node trips a quad_visit call may take in a row before returning
                            // (cfg2, refill 8: 1 / 2 / 4 -> 680 / 725 / 706 Msamples/s)
#endif
#ifndef RT_CLOSEST_PAIR
#define RT_CLOSEST_PAIR 0  // closest-hit walks: an inner trip also takes the stack top's node when it is in the window
                           // (measured: quad visits -8 %, box tests +11 %, fallbacks 375 -> 468, cfg2 710-722 vs 849-855)
#endif
#ifndef RT_ANY_WIDE
#define RT_ANY_WIDE 2  // nodes per occlusion trip with RT_ANY_PAIR (2: the current one and the stack top;
                       // 3 measured 821-824 vs 848-853 Msamples/s on cfg2)
#endif
#ifndef RT_ANY_PAIR
#define RT_ANY_PAIR 1  // occlusion walks: an inner trip also takes the stack top's node (8 boxes per round trip;
                       // cfg2 850-858 vs 834-835 Msamples/s, quad visits -6 %, cfg4 8-way shard 411 -> 402 ms)
#endif
// Lane sub's children of two inner nodes (a, and b when pair), both records loaded
// before either is tested: one memory round trip; box tests within [0, tmax].
__device__ __forceinline__ void quad_child2(const RtSceneView& S, int a, int b, bool pair, int sub, const RayB& rb,
                                            float tmax, QChild& ca, QChild& cb)
{
    float4_ a0, a1, b0 = float4_{0.0f, 0.0f, 0.0f, 0.0f}, b1 = b0;
    child_record(S, a, sub, a0, a1);
    if (pair) child_record(S, b, sub, b0, b1);
    rt_pin(a0);
    rt_pin(a1);
    rt_pin(b0);
    rt_pin(b1);
    {
        const int ref = (int)rt_asuint(a1.z), cnt = (int)rt_asuint(a1.w);
        const float mn[3] = {a0.x, a0.y, a0.z}, mx[3] = {a0.w, a1.x, a1.y};
        ca.ok = cnt >= 0 && box_hit(mn, mx, rb, tmax, ca.tn) && ca.tn <= tmax;
        ca.item = cnt > 0 ? leaf_item(ref, cnt) : ref;
    }
    {
        const int ref = (int)rt_asuint(b1.z), cnt = (int)rt_asuint(b1.w);
        const float mn[3] = {b0.x, b0.y, b0.z}, mx[3] = {b0.w, b1.x, b1.y};
        cb.ok = pair && cnt >= 0 && box_hit(mn, mx, rb, tmax, cb.tn) && cb.tn <= tmax;
        cb.item = cnt > 0 ? leaf_item(ref, cnt) : ref;
    }
}

template <bool ANY, int DESC = RT_VISIT_DESCEND, class QSTK>
__device__ __forceinline__ int quad_visit(const RtSceneView& S, QState& q, QSTK& stk, int sub, Stats* st)
{
    FastHit& h = q.h;
#pragma unroll 1
    for (int dd = 0; dd < DESC && q.cur >= 0; dd++) {
        if (ANY && RT_ANY_PAIR) {
            // the stack top (RT_ANY_WIDE 3: the top two) inner nodes are walked in the same
            // trip (the occlusion answer does not depend on the visit order)
            constexpr int NW = RT_ANY_WIDE;
            int nd[NW];
            nd[0] = q.cur;
            int m = 1;
#pragma unroll
            for (int j = 1; j < NW; j++) {
                nd[j] = -1;
                if (m == j && q.sp > q.bot) {
                    const int t = (int)stk.rec(q.sp - 1);
                    if (t >= 0) {
                        nd[j] = t;
                        q.sp--;
                        m++;
                    }
                }
            }
            if (st && sub == 0) st->c[RT_STAT_ANY_VOL] += 4 * m;
            float4_ r0[NW], r1[NW];
#pragma unroll
            for (int j = 0; j < NW; j++) {
                r0[j] = r1[j] = float4_{0.0f, 0.0f, 0.0f, 0.0f};
                if (j < m) child_record(S, nd[j], sub, r0[j], r1[j]);
            }
#pragma unroll
            for (int j = 0; j < NW; j++) {
                rt_pin(r0[j]);
                rt_pin(r1[j]);
            }
            int base = 0, first = 0;
            bool any_first = false;
#pragma unroll
            for (int j = 0; j < NW; j++) {
                const int ref = (int)rt_asuint(r1[j].z), cnt = (int)rt_asuint(r1[j].w);
                const float mn[3] = {r0[j].x, r0[j].y, r0[j].z}, mx[3] = {r0[j].w, r1[j].x, r1[j].y};
                float tn;
                const bool ok = j < m && cnt >= 0 && box_hit(mn, mx, q.rb, __builtin_inff(), tn);
                const int item = cnt > 0 ? leaf_item(ref, cnt) : ref;
                const int o = ok ? 1 : 0;
                const int o1 = qdpp<RT_QX1>(o), o2 = qdpp<RT_QX2>(o), o3 = qdpp<RT_QX3>(o);
                const int pre = base + (s_lower(sub, 1) ? o1 : 0) + (s_lower(sub, 2) ? o2 : 0) + (s_lower(sub, 3) ? o3 : 0);
                // hit k of the 4 * NW slots (node 0's children, then node 1's, ...) goes to
                // stack position sp + k - 1; hit 0 is next
                if (ok && pre > 0) {
                    if (q.sp + pre - 1 < QSTK::CAP) stk.set_rec(q.sp + pre - 1, (uint32_t)item);
                }
                if (ok && pre == 0) {
                    first = item;
                    any_first = true;
                }
                base += o + o1 + o2 + o3;
            }
            const int nv = base;
            if (q.sp + nv - 1 > QSTK::CAP) return -1;
            if (nv > 0) {
                q.sp += nv - 1;
                q.cur = qor(any_first ? first : 0);
                continue;
            }
            q.cur = 0x7ffffffe;
            break;
        }
        if (!ANY && RT_CLOSEST_PAIR) {
            // the stack top (the nearest pending box), when it is an inner node within the
            // window, is walked in the same trip; the 8 children are ranked together
            const float tmax = h.t + h.t * RT_T2_WINDOW;
            int b = -1;
            if (q.sp > 0) {
                const int t = (int)stk.rec(q.sp - 1);
                if (t >= 0 && stk.key(q.sp - 1) <= tmax) b = t;
            }
            const bool pair = b >= 0;
            if (pair) q.sp--;
            if (st && sub == 0) st->c[RT_STAT_VOL] += pair ? 8 : 4;
            QChild ca, cb;
            quad_child2(S, q.cur, b, pair, sub, q.rb, tmax, ca, cb);
            const float ka = ca.ok ? ca.tn : __builtin_inff(), kb = cb.ok ? cb.tn : __builtin_inff();
            const float a1 = qdppf<RT_QX1>(ka), a2 = qdppf<RT_QX2>(ka), a3 = qdppf<RT_QX3>(ka);
            const float b1 = qdppf<RT_QX1>(kb), b2 = qdppf<RT_QX2>(kb), b3 = qdppf<RT_QX3>(kb);
            const int s1 = sub ^ 1, s2 = sub ^ 2, s3 = sub ^ 3;
            // slots: A's children sub 0-3, then B's 4-7; ties go to the lower slot
            const int ra = (a1 < ka || (a1 == ka && s1 < sub) ? 1 : 0) + (a2 < ka || (a2 == ka && s2 < sub) ? 1 : 0) +
                           (a3 < ka || (a3 == ka && s3 < sub) ? 1 : 0) + (kb < ka ? 1 : 0) + (b1 < ka ? 1 : 0) +
                           (b2 < ka ? 1 : 0) + (b3 < ka ? 1 : 0);
            const int rb = (b1 < kb || (b1 == kb && s1 < sub) ? 1 : 0) + (b2 < kb || (b2 == kb && s2 < sub) ? 1 : 0) +
                           (b3 < kb || (b3 == kb && s3 < sub) ? 1 : 0) + (ka <= kb ? 1 : 0) + (a1 <= kb ? 1 : 0) +
                           (a2 <= kb ? 1 : 0) + (a3 <= kb ? 1 : 0);
            const int nv = qsum((ca.ok ? 1 : 0) + (cb.ok ? 1 : 0));
            if (q.sp + nv - 1 > QSTK::CAP) return -1;
            if (ca.ok && ra > 0) stk.set(q.sp + nv - 1 - ra, (uint32_t)ca.item, ka);
            if (cb.ok && rb > 0) stk.set(q.sp + nv - 1 - rb, (uint32_t)cb.item, kb);
            if (nv > 0) {
                q.sp += nv - 1;
                q.cur = qor(ca.ok && ra == 0 ? ca.item : cb.ok && rb == 0 ? cb.item : 0);
                continue;
            }
            q.cur = 0x7ffffffe;
            break;
        }
        if (st && sub == 0) st->c[ANY ? RT_STAT_ANY_VOL : RT_STAT_VOL] += 4;
        const float tmax = ANY ? __builtin_inff() : h.t + h.t * RT_T2_WINDOW;
        const QChild c = quad_child(S, q.cur, sub, q.rb, tmax);
        if (ANY) {
            const int okb = c.ok ? 1 : 0;
            const int o1 = qdpp<RT_QX1>(okb), o2 = qdpp<RT_QX2>(okb), o3 = qdpp<RT_QX3>(okb);
            const int pre = (s_lower(sub, 1) ? o1 : 0) + (s_lower(sub, 2) ? o2 : 0) + (s_lower(sub, 3) ? o3 : 0);
            const int nv = okb + o1 + o2 + o3;
            if (q.sp + nv - 1 > QSTK::CAP) return -1;
            if (c.ok && pre > 0) stk.set_rec(q.sp + pre - 1, (uint32_t)c.item);  // (an occlusion walk never reads keys)
            if (nv > 0) {
                q.sp += nv - 1;
                q.cur = qor(c.ok && pre == 0 ? c.item : 0);
                continue;
            }
        } else {
            const float key = c.ok ? c.tn : __builtin_inff();
            const float k1 = qdppf<RT_QX1>(key), k2 = qdppf<RT_QX2>(key), k3 = qdppf<RT_QX3>(key);
            const int s1 = sub ^ 1, s2 = sub ^ 2, s3 = sub ^ 3;
            const int rank = (k1 < key || (k1 == key && s1 < sub) ? 1 : 0) + (k2 < key || (k2 == key && s2 < sub) ? 1 : 0) +
                             (k3 < key || (k3 == key && s3 < sub) ? 1 : 0);
            const int nv = qsum(c.ok ? 1 : 0);
            if (q.sp + nv - 1 > QSTK::CAP) return -1;
            if (c.ok && rank > 0) stk.set(q.sp + nv - 1 - rank, (uint32_t)c.item, key);
            if (nv > 0) {
                q.sp += nv - 1;
                q.cur = qor(c.ok && rank == 0 ? c.item : 0);
                continue;
            }
        }
        // no child hit: pop (below)
        q.cur = 0x7ffffffe;
        break;
    }
    if (q.cur >= 0 && q.cur != 0x7ffffffe) return 0;  // (descended DESC times; still inner)
    if (q.cur < 0) {
        if (st && sub == 0) st->c[ANY ? RT_STAT_ANY_TRI : RT_STAT_TRI] += ((~q.cur) & 3) + 1;
        int k, leaf, prim;
        const float tv = quad_tri(S, q.cur, sub, q.o, q.d, k, leaf, prim);
        if (ANY) {
            const int hitb = tv < __builtin_inff() ? 1 : 0;
            if (S.brute) {
                if (qor(hitb)) {
                    h.k = 1;
                    return 1;
                }
            } else {
                const int h1 = qdpp<RT_QX1>(hitb), h2 = qdpp<RT_QX2>(hitb), h3 = qdpp<RT_QX3>(hitb);
                const int l1 = qdpp<RT_QX1>(leaf), l2 = qdpp<RT_QX2>(leaf), l3 = qdpp<RT_QX3>(leaf);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int x = j ^ sub;
                    const int hj = x == 0 ? hitb : x == 1 ? h1 : x == 2 ? h2 : h3;
                    if (!hj) continue;
                    const int lj = x == 0 ? leaf : x == 1 ? l1 : x == 2 ? l2 : l3;
                    if (quad_chain_ok(S, q.o, q.d, lj, false, 0.0f, sub, st)) {
                        h.k = 1;
                        return 1;
                    }
                }
            }
        } else {
            float m1 = tv, m2 = __builtin_inff();
            {
                const float o1 = qdppf<RT_QX1>(m1), o2 = qdppf<RT_QX1>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            {
                const float o1 = qdppf<RT_QX2>(m1), o2 = qdppf<RT_QX2>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            int pm = tv == m1 ? prim : 0x7fffffff;
            pm = min(pm, qdpp<RT_QX1>(pm));
            pm = min(pm, qdpp<RT_QX2>(pm));
            const bool mine = tv == m1 && prim == pm;
            if (m1 < h.t) {
                h.t2 = __builtin_fminf(h.t, m2);
                h.t = m1;
                h.k = qor(mine ? k : 0);
                h.leaf = qor(mine ? leaf : 0);
                h.prim = pm;
                h.tie = m2 == m1;
            } else if (m1 == h.t && m1 < __builtin_inff()) {
                h.tie = true;
                h.t2 = m1;
                if (pm < h.prim) {
                    h.k = qor(mine ? k : 0);
                    h.leaf = qor(mine ? leaf : 0);
                    h.prim = pm;
                }
            } else {
                h.t2 = __builtin_fminf(h.t2, m1);
            }
        }
    }
    if (ANY) {
        if (q.sp <= q.bot) return 1;  // (h.k = 0: no occluder in this quad's part of the walk)
        q.cur = (int)stk.rec(--q.sp);
        return 0;
    }
    const float tmax = h.t + h.t * RT_T2_WINDOW;
    int nxt = 0x7fffffff;
    while (q.sp > 0) {
        --q.sp;
        if (stk.key(q.sp) <= tmax) {
            nxt = (int)stk.rec(q.sp);
            break;
        }
    }
    q.cur = nxt;
    return nxt == 0x7fffffff ? 1 : 0;
}

// quad_query_closest's answer from a finished walk: true with (t, k), false when the
// exact walk must answer.
__device__ __forceinline__ bool quad_closest_answer(const RtSceneView& S, const QState& q, int sub, float& t_out,
                                                    int& k_out, Stats* st)
{
    const FastHit& h = q.h;
    if (h.k < 0) {
        t_out = -1.0f;
        k_out = -1;
        return true;
    }
    if (S.brute) {
        t_out = h.t;
        k_out = h.k;
        return true;
    }
    if (h.tie) return false;
    const float t2 = __builtin_fminf(h.t2, h.t + h.t * RT_T2_WINDOW);
    if (!quad_chain_ok(S, q.o, q.d, h.leaf, true, t2, sub, st)) return false;
    t_out = h.t;
    k_out = h.k;
    return true;
}

// A quad walk as a state machine, one node or leaf visit per qwalk_step, so
// that a wave can refill a quad with its next query the moment the quad's
// walk ends instead of waiting for the wave's slowest walk (k_trace), and so
// that closest and occlusion walks share one loop (k_tail). anyq false:
// quad_query_closest's answer; anyq true: quad_query_any's. The occlusion
// answer does not depend on the visit order (any hit whose octree chain
// holds), so both kinds descend nearest-first; an occlusion walk keeps no
// window (tmax inf). Every field is quad-uniform.
struct QWalk {
    V3 o, d;
    RayB rb;
    FastHit h;
    int sp, cur;
    bool anyq;
    float t;  // answer: closest t (-1: no hit) ...
    int k;    // ... and leaf-order triangle (-1: none); occlusion: 1 / 0
};

// Starts a walk. Returns 0 (walk with qwalk_step) or 1 when the answer is
// already known (a NaN ray: no hit).
__device__ __forceinline__ int qwalk_begin(QWalk& w, V3 o, V3 d, bool anyq, int sub, Stats* st)
{
    if (st && sub == 0) st->c[anyq ? RT_STAT_ANY_RAYS : RT_STAT_RAYS]++;
    w.o = o;
    w.d = d;
    w.anyq = anyq;
    w.t = -1.0f;
    w.k = anyq ? 0 : -1;
    if (rt_isnan(d.x) || rt_isnan(d.y) || rt_isnan(d.z) || rt_isnan(o.x) || rt_isnan(o.y) || rt_isnan(o.z)) return 1;
    w.h.t = __builtin_inff();
    w.h.t2 = __builtin_inff();
    w.h.k = -1;
    w.h.leaf = -1;
    w.h.prim = 0x7fffffff;
    w.h.tie = false;
    w.rb = rayb_setup(o, d);
    w.sp = 0;
    w.cur = 0;
    return 0;
}

// The memory of one visit, loaded before it is used (qwalk_issue), so that a
// caller can put other loads in flight beside it: inner node, lane sub's 32-B
// child record (x0, x1); leaf, lane sub's 48-B triangle (x0, x1, x2).
struct QVisit {
    float4_ x0, x1, x2;
};
__device__ __forceinline__ void qwalk_issue(const QWalk& w, const RtSceneView& S, int sub, QVisit& v)
{
    if (w.cur >= 0) {
        child_record(S, w.cur, sub, v.x0, v.x1);
        rt_pin(v.x0);
        rt_pin(v.x1);
    } else {
        const int it = ~w.cur;
        if (sub <= (it & 3)) {
            const float4_* p = S.bvh_tri4 + 3 * ((it >> 2) + sub);
            v.x0 = p[0];
            v.x1 = p[1];
            v.x2 = p[2];
            rt_pin(v.x0);
            rt_pin(v.x1);
            rt_pin(v.x2);
        }
    }
}

// One visit on the loaded records. Returns 0 while the walk goes on, 1 with
// the answer in (t, k), -1 when the exact walk must answer (stack overflow, a
// tie, a failed chain).
template <class QSTK>
__device__ int qwalk_consume(QWalk& w, const RtSceneView& S, QSTK& stk, int sub, const QVisit& v, Stats* st)
{
    const bool anyq = w.anyq;
    FastHit& h = w.h;
    if (w.cur >= 0) {
        if (st && sub == 0) st->c[anyq ? RT_STAT_ANY_VOL : RT_STAT_VOL] += 4;
        const float tmax = anyq ? __builtin_inff() : h.t + h.t * RT_T2_WINDOW;
        QChild c;
        {  // (quad_child on the loaded record)
            const int ref = (int)rt_asuint(v.x1.z), cnt = (int)rt_asuint(v.x1.w);
            const float mn[3] = {v.x0.x, v.x0.y, v.x0.z}, mx[3] = {v.x0.w, v.x1.x, v.x1.y};
            c.ok = cnt >= 0 && box_hit(mn, mx, w.rb, tmax, c.tn) && c.tn <= tmax;
            c.item = cnt > 0 ? leaf_item(ref, cnt) : ref;
        }
        const float key = c.ok ? c.tn : __builtin_inff();
        // closest: rank by (key, lane), the nearest hit child has rank 0; occlusion (order-free
        // answer): the ok lanes in lane order, as quad_query_any (nearest-first measured slower)
        int rank;
        if (anyq) {
            const int okb = c.ok ? 1 : 0;
            const int o1 = qdpp<RT_QX1>(okb), o2 = qdpp<RT_QX2>(okb), o3 = qdpp<RT_QX3>(okb);
            const int pre = (s_lower(sub, 1) ? o1 : 0) + (s_lower(sub, 2) ? o2 : 0) + (s_lower(sub, 3) ? o3 : 0);
            const int nok = okb + o1 + o2 + o3;
            rank = pre == 0 ? 0 : nok - pre;  // first ok lane next; the others pushed, the second on top
        } else {
            const float k1 = qdppf<RT_QX1>(key), k2 = qdppf<RT_QX2>(key), k3 = qdppf<RT_QX3>(key);
            const int s1 = sub ^ 1, s2 = sub ^ 2, s3 = sub ^ 3;
            rank = (k1 < key || (k1 == key && s1 < sub) ? 1 : 0) + (k2 < key || (k2 == key && s2 < sub) ? 1 : 0) +
                   (k3 < key || (k3 == key && s3 < sub) ? 1 : 0);
        }
        const int nv = qsum(c.ok ? 1 : 0);
        if (w.sp + nv - 1 > QSTK::CAP) return -1;
        // far children on the stack, the next of them on top
        if (c.ok && rank > 0) stk.set(w.sp + nv - 1 - rank, (uint32_t)c.item, key);
        if (nv > 0) {
            w.sp += nv - 1;
            w.cur = qor(c.ok && rank == 0 ? c.item : 0);
            return 0;
        }
    } else {
        if (st && sub == 0) st->c[anyq ? RT_STAT_ANY_TRI : RT_STAT_TRI] += ((~w.cur) & 3) + 1;
        int k = -1, leaf = -1, prim = 0x7fffffff;
        float tv = __builtin_inff();
        {  // (quad_tri on the loaded record)
            float t;
            if (sub <= ((~w.cur) & 3) && tri_test_v(ld3(v.x0), ld3(v.x1), ld3(v.x2), w.o, w.d, t)) {
                tv = t;
                k = (int)rt_asuint(v.x0.w);
                leaf = (int)rt_asuint(v.x1.w);
                prim = (int)rt_asuint(v.x2.w);
            }
        }
        if (anyq) {
            const int hitb = tv < __builtin_inff() ? 1 : 0;
            if (S.brute) {
                if (qor(hitb)) {  // USE_BVH 0: any triangle hit occludes
                    w.k = 1;
                    return 1;
                }
            } else {
                // each hit lane's octree leaf in turn, checked by the whole quad
                const int h1 = qdpp<RT_QX1>(hitb), h2 = qdpp<RT_QX2>(hitb), h3 = qdpp<RT_QX3>(hitb);
                const int l1 = qdpp<RT_QX1>(leaf), l2 = qdpp<RT_QX2>(leaf), l3 = qdpp<RT_QX3>(leaf);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int x = j ^ sub;
                    const int hj = x == 0 ? hitb : x == 1 ? h1 : x == 2 ? h2 : h3;
                    if (!hj) continue;
                    const int lj = x == 0 ? leaf : x == 1 ? l1 : x == 2 ? l2 : l3;
                    if (quad_chain_ok(S, w.o, w.d, lj, false, 0.0f, sub, st)) {
                        w.k = 1;
                        return 1;
                    }
                }
            }
        } else {
            // quad (smallest, second smallest) of the lanes' hit distances
            float m1 = tv, m2 = __builtin_inff();
            {
                const float o1 = qdppf<RT_QX1>(m1), o2 = qdppf<RT_QX1>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            {
                const float o1 = qdppf<RT_QX2>(m1), o2 = qdppf<RT_QX2>(m2);
                const float n1 = __builtin_fminf(m1, o1), n2 = __builtin_fminf(__builtin_fmaxf(m1, o1), __builtin_fminf(m2, o2));
                m1 = n1, m2 = n2;
            }
            // the lane holding m1 with the lowest original index
            int pm = tv == m1 ? prim : 0x7fffffff;
            pm = min(pm, qdpp<RT_QX1>(pm));
            pm = min(pm, qdpp<RT_QX2>(pm));
            const bool mine = tv == m1 && prim == pm;
            if (m1 < h.t) {
                h.t2 = __builtin_fminf(h.t, m2);
                h.t = m1;
                h.k = qor(mine ? k : 0);
                h.leaf = qor(mine ? leaf : 0);
                h.prim = pm;
                h.tie = m2 == m1;
            } else if (m1 == h.t && m1 < __builtin_inff()) {
                h.tie = true;
                h.t2 = m1;
                if (pm < h.prim) {
                    h.k = qor(mine ? k : 0);
                    h.leaf = qor(mine ? leaf : 0);
                    h.prim = pm;
                }
            } else {
                h.t2 = __builtin_fminf(h.t2, m1);
            }
        }
    }
    // pop, dropping entries the window has closed behind
    const float tmax = anyq ? __builtin_inff() : h.t + h.t * RT_T2_WINDOW;
    int nxt = 0x7fffffff;
    while (w.sp > 0) {
        --w.sp;
        if (stk.key(w.sp) <= tmax) {
            nxt = (int)stk.rec(w.sp);
            break;
        }
    }
    w.cur = nxt;
    if (nxt != 0x7fffffff) return 0;
    // the walk is over
    if (anyq || h.k < 0) return 1;  // (t, k) = (-1, -1) / occlusion 0
    if (!S.brute) {                  // USE_BVH 0: the closest M-T hit, lowest index on ties; no octree
        if (h.tie) return -1;
        const float t2 = __builtin_fminf(h.t2, h.t + h.t * RT_T2_WINDOW);
        if (!quad_chain_ok(S, w.o, w.d, h.leaf, true, t2, sub, st)) return -1;
    }
    w.t = h.t;
    w.k = h.k;
    return 1;
}

template <class QSTK>
__device__ __forceinline__ int qwalk_step(QWalk& w, const RtSceneView& S, QSTK& stk, int sub, Stats* st)
{
    QVisit v;
    qwalk_issue(w, S, sub, v);
    return qwalk_consume(w, S, stk, sub, v, st);
}

// A whole walk (k_tail: a wave's closest and occlusion queries in one loop).
// Returns 1 with (t, k) or the occlusion answer in k, -1: exact walk.
template <class QSTK>
__device__ int quad_query_mixed(const RtSceneView& S, V3 o, V3 d, QSTK& stk, int sub, bool anyq, QWalk& w, Stats* st)
{
    int r = qwalk_begin(w, o, d, anyq, sub, st);
    while (r == 0) r = qwalk_step(w, S, stk, sub, st);
    return r;
}

}  // namespace rtk
