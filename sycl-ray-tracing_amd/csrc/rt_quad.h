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

// Lane sub's 32-B child record of inner node `node`. (Staging the top of the search
// BVH in LDS per block measured slower at every depth tried, r02: the top levels stay
// L2-resident)
__device__ __forceinline__ void child_record(const RtSceneView& S, int node, int sub, float4_& a, float4_& b)
{
    const float4_* p = (const float4_*)(S.bvh4 + node) + 2 * sub;
    a = p[0];
    b = p[1];
}

// Oriented slabs (rt_fast.h slab_ok) in the quad walks: each lane also loads its child's
// 16-B slab record in the same round trip.
#ifndef RT_SLAB_QUAD
#define RT_SLAB_QUAD RT_SLABS
#endif

// Lane `sub`'s child of inner node `node`: box (and slab) test within [0, tmax].
struct QChild {
    int item;  // node index or leaf item (rt_fast.h leaf_item)
    bool ok;
    float tn;
};
__device__ __forceinline__ QChild quad_child(const RtSceneView& S, int node, int sub, const RayB& rb, float tmax, V3 o,
                                             V3 d)
{
    float4_ a, b;
    child_record(S, node, sub, a, b);
#if RT_SLAB_QUAD
    const float4_ sl = S.bvh4s[4 * (size_t)node + sub];
    rt_pin(sl);
#endif
    rt_pin(a);
    rt_pin(b);
    const int ref = (int)rt_asuint(b.z), cnt = (int)rt_asuint(b.w);
    const float mn[3] = {a.x, a.y, a.z}, mx[3] = {a.w, b.x, b.y};
    QChild c;
    float tf;
    c.ok = cnt >= 0 && box_hit2(mn, mx, rb, tmax, c.tn, tf) && c.tn <= tmax;
#if RT_SLAB_QUAD
    c.ok = c.ok && slab_ok(sl, o, d, c.tn, tf);
#else
    (void)o, (void)d;
#endif
    c.item = cnt > 0 ? leaf_item(ref, cnt) : ref;
    return c;
}

// Lane `sub`'s triangle of a leaf item: Moller-Trumbore (the reference's
// arithmetic). Returns t (+inf when the lane has no triangle or no hit).
// MARK (closest-hit walks): a hit fuzzier than its box pad marks its leaf (below).
template <bool MARK>
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
            // (RT_FUZZ_CHECK builds: a hit fuzzier than its box pad marks its leaf, and the
            // walk's answer then goes to the exact walk, quad_closest_answer; the mark travels
            // with the leaf through the reductions, and a same-leaf tie of marked and unmarked
            // hits counts as mixed)
            leaf = (int)rt_asuint(e1.w) | (RT_FUZZ_CHECK && MARK && fuzzy_tri(a, e1, e2, o, d) ? RT_FZ_BIT : 0);
            prim = (int)rt_asuint(e2.w);
        }
    }
    return tv;
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

// A quad's walk, one trip per quad_visit call and specialized by kind (ANY: an
// occlusion walk, whose answer does not depend on the visit order; else the
// closest-hit walk of rt_fast.h fast_closest, nearest child first, with its window
// and second-hit bookkeeping), so that k_trace can start a quad on its next query
// the moment its walk ends. The answer is rt_fast.h's, so a query falls back to the
// exact octree walk in exactly the same cases.
struct QState {
    V3 o, d;
    RayB rb;
    FastHit h;
    int sp, cur;
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
    return true;
}

// One trip. 0: go on; 1: the walk is over (ANY: q.h.k = 1 occluded / 0 not; else the
// closest-hit record in q.h, to quad_closest_answer); -1: the bounded stack overflowed.
#ifndef RT_VISIT_DESCEND
#define RT_VISIT_DESCEND 2  // inner-node trips a quad_visit call may take in a row before returning
                            // (cfg2, refill 8: 1 / 2 / 4 -> 680 / 725 / 706 Msamples/s)
#endif
// Occlusion walks take the stack top's inner node in the same trip as the current one
// (8 child boxes per memory round trip): cfg2 850-858 vs 834-835 Msamples/s, quad visits
// -6 %, cfg4 8-way shard 411 -> 402 ms (r02). Three nodes per trip (821-824) and the
// same pairing for closest-hit walks (710-722: the looser nearest-first order cost 25 %
// more exact-walk fallbacks) were slower (profiles/r02_k_trace_variants.jsonl).
// PAIR = false (stats renders only, rt_set_stats(ctx, 2)): occlusion walks take one node per
// trip, so their box-test counters are the necessary ones (answers do not depend on the order).
#ifndef RT_POP_PAIRED
#define RT_POP_PAIRED 1
#endif
template <bool ANY, int DESC = RT_VISIT_DESCEND, bool PAIR = true, class QSTK>
__device__ __forceinline__ int quad_visit(const RtSceneView& S, QState& q, QSTK& stk, int sub, Stats* st)
{
    FastHit& h = q.h;
#pragma unroll 1
    for (int dd = 0; dd < DESC && q.cur >= 0; dd++) {
        if (ANY) {
            // the current node and the stack top's inner node in one trip
            constexpr int NW = PAIR ? 2 : 1;
            int nd[NW];
            nd[0] = q.cur;
            int m = 1;
#pragma unroll
            for (int j = 1; j < NW; j++) {
                nd[j] = -1;
                if (m == j && q.sp > 0) {
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
#if RT_SLAB_QUAD
            float4_ sl[NW];
#endif
#pragma unroll
            for (int j = 0; j < NW; j++) {
                r0[j] = r1[j] = float4_{0.0f, 0.0f, 0.0f, 0.0f};
#if RT_SLAB_QUAD
                sl[j] = float4_{0.0f, 0.0f, -__builtin_inff(), __builtin_inff()};
                if (j < m) sl[j] = S.bvh4s[4 * (size_t)nd[j] + sub];
#endif
                if (j < m) child_record(S, nd[j], sub, r0[j], r1[j]);
            }
#pragma unroll
            for (int j = 0; j < NW; j++) {
                rt_pin(r0[j]);
                rt_pin(r1[j]);
#if RT_SLAB_QUAD
                rt_pin(sl[j]);
#endif
            }
            int base = 0, first = 0;
            bool any_first = false;
#pragma unroll
            for (int j = 0; j < NW; j++) {
                const int ref = (int)rt_asuint(r1[j].z), cnt = (int)rt_asuint(r1[j].w);
                const float mn[3] = {r0[j].x, r0[j].y, r0[j].z}, mx[3] = {r0[j].w, r1[j].x, r1[j].y};
                float tn, tf;
#if RT_SLAB_QUAD
                const bool ok = j < m && cnt >= 0 && box_hit2(mn, mx, q.rb, __builtin_inff(), tn, tf) &&
                                slab_ok(sl[j], q.o, q.d, tn, tf);
#else
                const bool ok = j < m && cnt >= 0 && box_hit2(mn, mx, q.rb, __builtin_inff(), tn, tf);
#endif
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
        if (st && sub == 0) st->c[RT_STAT_VOL] += 4;
        const float tmax = h.t + h.t * RT_T2_WINDOW;
        const QChild c = quad_child(S, q.cur, sub, q.rb, tmax, q.o, q.d);
        const float key = c.ok ? c.tn : __builtin_inff();
        // rank by (key, lane): the nearest hit child has rank 0
        const float k1 = qdppf<RT_QX1>(key), k2 = qdppf<RT_QX2>(key), k3 = qdppf<RT_QX3>(key);
        const int s1 = sub ^ 1, s2 = sub ^ 2, s3 = sub ^ 3;
        const int rank = (k1 < key || (k1 == key && s1 < sub) ? 1 : 0) + (k2 < key || (k2 == key && s2 < sub) ? 1 : 0) +
                         (k3 < key || (k3 == key && s3 < sub) ? 1 : 0);
        const int nv = qsum(c.ok ? 1 : 0);
        if (q.sp + nv - 1 > QSTK::CAP) return -1;
        // far children on the stack, nearest of them on top (rank 1 at sp + nv - 2)
        if (c.ok && rank > 0) stk.set(q.sp + nv - 1 - rank, (uint32_t)c.item, key);
        if (nv > 0) {
            q.sp += nv - 1;
            q.cur = qor(c.ok && rank == 0 ? c.item : 0);
            continue;
        }
        // no child hit: pop (below)
        q.cur = 0x7ffffffe;
        break;
    }
    if (q.cur >= 0 && q.cur != 0x7ffffffe) return 0;  // (descended DESC times; still inner)
    if (q.cur < 0) {
        if (st && sub == 0) st->c[ANY ? RT_STAT_ANY_TRI : RT_STAT_TRI] += ((~q.cur) & 3) + 1;
        int k, leaf, prim;
        const float tv = quad_tri<!ANY>(S, q.cur, sub, q.o, q.d, k, leaf, prim);
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
            // rt_fast.h fast_take over the quad's four hits: m1 the closest, m2 the next distance
            // above it, the winner among the lanes at m1 (brute force: lowest original index;
            // else lowest leaf-order k, the first in its octree leaf's list), and whether the
            // lanes at m1 span more than one octree leaf (a tie only the exact walk settles)
            float m1 = __builtin_fminf(tv, qdppf<RT_QX1>(tv));
            m1 = __builtin_fminf(m1, qdppf<RT_QX2>(m1));
            float m2 = tv > m1 ? tv : __builtin_inff();
            m2 = __builtin_fminf(m2, qdppf<RT_QX1>(m2));
            m2 = __builtin_fminf(m2, qdppf<RT_QX2>(m2));
            int key = tv == m1 ? (S.brute ? prim : k) : 0x7fffffff;
            key = min(key, qdpp<RT_QX1>(key));
            key = min(key, qdpp<RT_QX2>(key));
            const bool mine = tv == m1 && (S.brute ? prim : k) == key;
            const int wk = qor(mine ? k : 0), wl = qor(mine ? leaf : 0), wp = qor(mine ? prim : 0);
            const bool mixed = qor(tv == m1 && m1 < __builtin_inff() && leaf != wl ? 1 : 0) != 0;
            if (m1 < h.t) {
                h.t2 = __builtin_fminf(h.t, m2);
                h.t = m1;
                h.k = wk;
                h.leaf = wl;
                h.prim = wp;
                h.tie = mixed;
            } else if (m1 == h.t && m1 < __builtin_inff()) {
                h.t2 = __builtin_fminf(h.t2, m2);
                if (S.brute) {
                    h.tie = true;
                    if (wp < h.prim) h.k = wk, h.leaf = wl, h.prim = wp;
                } else if (!mixed && wl == h.leaf) {
                    if (wk < h.k) h.k = wk, h.prim = wp;
                } else {
                    h.tie = true;
                }
            } else {
                h.t2 = __builtin_fminf(h.t2, m1);
            }
        }
    }
    if (ANY) {
        if (q.sp == 0) return 1;  // (h.k = 0: no occluder)
        q.cur = (int)stk.rec(--q.sp);
        return 0;
    }
    const float tmax = h.t + h.t * RT_T2_WINDOW;
    int nxt = 0x7fffffff;
    while (q.sp > 0) {
#if RT_POP_PAIRED >= 2  // two entries per LDS round trip: the pops past a closed window run in pairs
        if (q.sp >= 2) {
            const float k1 = stk.key(q.sp - 1), k2 = stk.key(q.sp - 2);
            const int r1 = (int)stk.rec(q.sp - 1), r2 = (int)stk.rec(q.sp - 2);
            rt_pin(r1);
            rt_pin(r2);
            if (k1 <= tmax) {
                q.sp -= 1;
                nxt = r1;
                break;
            }
            q.sp -= 2;
            if (k2 <= tmax) {
                nxt = r2;
                break;
            }
            continue;
        }
#endif
        --q.sp;
#if RT_POP_PAIRED  // the entry's key and item read together: one LDS round trip per pop, not two
        const float kk = stk.key(q.sp);
        const int rr = (int)stk.rec(q.sp);
        rt_pin(rr);  // (else the compiler sinks the item's read past the loop: two round trips)
        if (kk <= tmax) {
            nxt = rr;
            break;
        }
#else
        if (stk.key(q.sp) <= tmax) {
            nxt = (int)stk.rec(q.sp);
            break;
        }
#endif
    }
    q.cur = nxt;
    return nxt == 0x7fffffff ? 1 : 0;
}

// The closest-hit answer of a finished walk: true with (t, k), false when the exact
// octree walk must answer (a tie, or the verification fails: rt_fast.h).
__device__ __forceinline__ bool quad_closest_answer(const RtSceneView& S, const QState& q, int sub, float& t_out,
                                                    int& k_out, Stats* st)
{
    const FastHit& h = q.h;
    if (h.k < 0) {
        t_out = -1.0f;
        k_out = -1;
        return true;
    }
    // the found hit fuzzier than its box pad (rt_fast.h fuzzy_tri, marked by quad_tri)
    if (RT_FUZZ_CHECK && (h.leaf & RT_FZ_BIT)) return false;
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

}  // namespace rtk
