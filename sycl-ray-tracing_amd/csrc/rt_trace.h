// rt_trace.h — scene queries and shading primitives of the path tracer that
// runs on gfx950 (and, compiled for the host, in the hostsim test build).
//
// Restates the functions source/render_kernel.cpp's ray_trace_pixel calls,
// with the reference's exact float/double evaluation order. Differences are
// purely structural:
//  * BVH: the recursive priority-queue octree traversal (bvh.h:127-209) is
//    re-expressed as an explicit-stack walk over RtNode child blocks that
//    visits nodes in the identical order (libstdc++ heap tie order included)
//    and applies the identical early-exit rule; see trace_closest().
//    Occlusion-only queries use trace_any() (same reachable set, first hit).
//  * libm: rt_libm.h (glibc-bit-exact).
// The bounce loop itself lives in rt_wave.h (wavefront form).
#pragma once

#include "rt_device.h"
#include "rt_fp.h"
#include "rt_libm.h"

namespace rtk {

// ---------------------------------------------------------------- vectors
struct V3 {
    float x, y, z;
};
RT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
RT_HD V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD V3 neg(V3 v) { return v3(-v.x, -v.y, -v.z); }
RT_HD V3 mul(float k, V3 v) { return v3(k * v.x, k * v.y, k * v.z); }
RT_HD float dot(V3 u, V3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
RT_HD float length(V3 v) { return rt_sqrtf(dot(v, v)); }
RT_HD V3 normalize(V3 v)
{
    float kk = 1.0f / length(v);
    return mul(kk, v);
}
RT_HD V3 cross(V3 u, V3 v)
{
    return v3((u.y * v.z) - (u.z * v.y), (u.z * v.x) - (u.x * v.z), (u.x * v.y) - (u.y * v.x));
}

struct Col {
    float r, g, b;
};
RT_HD Col col(float v) { return Col{v, v, v}; }
RT_HD Col cadd(Col a, Col b) { return Col{a.r + b.r, a.g + b.g, a.b + b.b}; }
RT_HD Col csub(Col a, Col b) { return Col{a.r + (-b.r), a.g + (-b.g), a.b + (-b.b)}; }
RT_HD Col cmul(Col a, Col b) { return Col{a.r * b.r, a.g * b.g, a.b * b.b}; }
RT_HD Col cscale(Col c, float k) { return Col{c.r * k, c.g * k, c.b * k}; }
RT_HD Col cdiv(Col c, float k)  // color.h:459-463 (multiply by the reciprocal)
{
    float kk = 1 / k;
    return cscale(c, kk);
}

// --------------------------------------------------------------------- rng
struct Rng {  // xorshift.h:10-31
    uint32_t a;
    RT_HD float next()
    {
        uint32_t x = a;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        a = x;
        return rt_min((float)x / 4294967296.0f, 1.0f - 1.0e-6f);
    }
};

// -------------------------------------------------------------------- scene
struct Hit {
    float t;   // -1: none
    int k;     // leaf-order triangle index, or -2 - sphere index
    int prim;  // primitive id (triangle id or sphere prim)
    int mi;    // material index when the triangle record carries it (RtSceneView::tri_mat), else -1
    V3 p, n;
};

RT_HD V3 ld3(const float4_& f) { return v3(f.x, f.y, f.z); }

// ------------------------------------------------------------- traversal
#define RT_STACK_CAP 232  // >= 7 * 32 + 1: worst case for an octree of depth 32

struct StackEnt {
    uint32_t rec;   // record index | FIRST | LAST flags
    float tnear;
    int32_t snap;   // leaves visited when the previous sibling was popped
};
#define RT_ENT_FIRST 0x80000000u
#define RT_ENT_LAST 0x40000000u
#define RT_ENT_MASK 0x3fffffffu

struct Stats {
    unsigned long long c[RT_STAT_COUNT];
};

// Per-ray slab constants: den = n.d, num = n.o for the 7 plane normals
// (bvh.h:133-137) and rinv = 1/(double)den. The slab quotient
// (d - num) / den is evaluated as (float)((double)(d - num) * rinv): with
// rinv within 2^-53 of 1/den and one more rounding in the product, the
// double result is within ~2^-52 (relative) of the exact quotient, while
// the exact quotient of two floats is never closer than 2^-49 (relative)
// to a float rounding boundary, so the final rounding to float gives the
// correctly rounded IEEE f32 quotient — the reference's `/` — for every
// finite operand (tests: test_gpu_parity.py::test_gpu_slab_division_exact).
// On gfx950 that is 3 instructions instead of the ~10 of an IEEE f32 divide.
struct RayK {
    float num[7];
    double rinv[7];  // 1/den: +-inf exactly when den == 0, negative exactly when den < 0
};

RT_HD float slab_div(float a, double rinv) { return (float)((double)a * rinv); }

RT_HD bool ray_setup(V3 o, V3 d, RayK& k)
{
    const float s = rt_sqrtf(3.0f) / 3;
    const V3 N[7] = {v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1), v3(s, s, s), v3(-s, s, s), v3(-s, -s, s), v3(s, -s, s)};
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const float den = dot(N[i], d);
        k.num[i] = dot(N[i], o);
        k.rinv[i] = 1.0 / (double)den;
        bad = bad || rt_isnan(den) || rt_isnan(k.num[i]);
    }
    // A NaN component makes every slab test pass and every triangle test
    // fail (NaN compares false), so such a ray can never hit.
    return !bad;
}

// A node record in registers: loaded with four 16-B loads up front (one
// memory round trip instead of one per plane).
struct uint2_ {
    uint32_t x, y;
};
// (ref, cnt) of a record: the last 8 bytes, one load.
RT_HD uint2_ load_link(const RtNode* nodes, uint32_t i)
{
    const uint2_* p = (const uint2_*)(nodes + i) + 7;
    return *p;
}

struct NodeR {
    float dn[7], df[7];
    uint32_t ref, cnt;
};
RT_HD NodeR load_node(const RtNode* nodes, uint32_t i)
{
    const float4_* p = (const float4_*)(nodes + i);
    const float4_ a = p[0], b = p[1], c = p[2], d = p[3];
    NodeR n;
    n.dn[0] = a.x, n.dn[1] = a.y, n.dn[2] = a.z, n.dn[3] = a.w;
    n.dn[4] = b.x, n.dn[5] = b.y, n.dn[6] = b.z, n.df[0] = b.w;
    n.df[1] = c.x, n.df[2] = c.y, n.df[3] = c.z, n.df[4] = c.w;
    n.df[5] = d.x, n.df[6] = d.y;
    n.ref = rt_asuint(d.z);
    n.cnt = rt_asuint(d.w);
    return n;
}

// BoundingVolume::intersect (bounding_volume.h:101-126), branch-free:
//  * a plane with denom == 0 is skipped by the reference; here it yields
//    (-inf, +inf), the identity of the max / min that follow;
//  * `if (denom < 0) swap(near, far)` is applied to the operands instead of
//    the quotients (same two quotients, same arithmetic);
//  * the early `t_far < t_near` exit cannot change the outcome (prefix
//    max/min are monotone), so all planes are evaluated.
RT_HD bool slab_test(const NodeR& nd, const RayK& k, float& tnear)
{
    float tn = -__builtin_inff(), tf = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const double r = k.rinv[i];
        const bool neg = r < 0.0;
        float a = slab_div((neg ? nd.df[i] : nd.dn[i]) - k.num[i], r);
        float b = slab_div((neg ? nd.dn[i] : nd.df[i]) - k.num[i], r);
        if (__builtin_isinf(r)) {  // den == 0: the reference skips the plane
            a = -__builtin_inff();
            b = __builtin_inff();
        }
        tn = rt_max(tn, a);
        tf = rt_min(tf, b);
    }
    tnear = tn;
    return !(tf < tn);
}
RT_HD bool slab_test(const RtNode& nd, const RayK& k, float& tnear)
{
    NodeR r;
    for (int i = 0; i < 7; i++) r.dn[i] = nd.dn[i], r.df[i] = nd.df[i];
    return slab_test(r, k, tnear);
}

// Triangle::intersect (triangle.h:16-60) on the pre-subtracted record.
RT_HD bool tri_test_v(V3 a, V3 e1, V3 e2, V3 o, V3 d, float& t_out)
{
    const float EPS = 0.0000001f;
    V3 h = cross(d, e2);
    float det = dot(e1, h);
    if (det > -EPS && det < EPS) return false;
    float f = 1.0f / det;
    V3 s = sub(o, a);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    V3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot(e2, q);
    if (t > EPS) {
        t_out = t;
        return true;
    }
    return false;
}
RT_HD bool tri_test(const float4_* tri4, int k, V3 o, V3 d, float& t_out)
{
    return tri_test_v(ld3(tri4[3 * k]), ld3(tri4[3 * k + 1]), ld3(tri4[3 * k + 2]), o, d, t_out);
}

// RenderKernel::intersect_scene, the brute-force triangle loop (USE_BVH 0,
// render_kernel.cpp:453-471): every triangle in buffer order, the closest kept
// with a strict `<`, so the lowest index wins a tie. Returns the leaf-order
// index k (-1: none) and t (-1: none); the sphere loop follows (rt_wave.h).
RT_HD void brute_closest(const RtSceneView& S, V3 o, V3 d, float& best_t, int& best_k)
{
    best_t = -1.0f;
    best_k = -1;
    for (int i = 0; i < S.n_tris; i++) {
        const int k = S.prim2k[i];
        float t;
        if (tri_test(S.tri4, k, o, d, t))
            if (t < best_t || best_t == -1.0f) {
                best_t = t;
                best_k = k;
            }
    }
}
RT_HD bool brute_any(const RtSceneView& S, V3 o, V3 d)  // INTERSECT_SCENE as a boolean
{
    for (int i = 0; i < S.n_tris; i++) {
        float t;
        if (tri_test(S.tri4, i, o, d, t) && t > 0.0f) return true;
    }
    return false;
}

// ------------------------------------------------ libstdc++ heap emulation
// std::priority_queue<QueueElement, vector, greater> (bvh.h:170-199): pushes
// in child order, pops the minimum t_near. Equal keys pop in the order
// libstdc++'s push_heap / __adjust_heap produce (bits/stl_heap.h); emulated
// here exactly so equal-t hits resolve like the reference.
RT_HD void heap_sift_up(float* k, int* v, int hole, float key, int val)
{
    int parent = (hole - 1) / 2;
    while (hole > 0 && k[parent] > key) {
        k[hole] = k[parent];
        v[hole] = v[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    k[hole] = key;
    v[hole] = val;
}
RT_HD void heap_pop(float* k, int* v, int len)  // std::pop_heap on [0, len)
{
    if (len <= 1) return;
    const int L = len - 1;
    const float key = k[L];
    const int val = v[L];
    k[L] = k[0];
    v[L] = v[0];
    int hole = 0, second = 0;
    while (second < (L - 1) / 2) {
        second = 2 * (second + 1);
        if (k[second] > k[second - 1]) second--;
        k[hole] = k[second];
        v[hole] = v[second];
        hole = second;
    }
    if ((L & 1) == 0 && second == (L - 2) / 2) {
        second = 2 * (second + 1);
        k[hole] = k[second - 1];
        v[hole] = v[second - 1];
        hole = second - 1;
    }
    heap_sift_up(k, v, hole, key, val);
}
// Order m (key, id) pairs given in push order into pop order.
RT_HD void heap_order(float* key, int* id, int m, float* okey, int* oid)
{
    float hk[8];
    int hv[8];
    for (int i = 0; i < m; i++) heap_sift_up(hk, hv, i, key[i], id[i]);
    for (int n = m; n > 0; n--) {
        okey[m - n] = hk[0];
        oid[m - n] = hv[0];
        heap_pop(hk, hv, n);
    }
}

RT_HD void leaf_test(const RtSceneView& S, uint32_t ref, uint32_t cnt, V3 o, V3 d, float& best_t, int& best_k,
                     Stats* st)
{
    const int n = (int)(cnt & ~RT_LEAF_BIT);
    const int k0 = (int)ref;
    for (int j = 0; j < n; j++) {
        float t;
        if (tri_test(S.tri4, k0 + j, o, d, t))
            if (t < best_t || best_t == -1) {
                best_t = t;
                best_k = k0 + j;
            }
    }
    if (st) {
        st->c[RT_STAT_TRI] += n;
        st->c[RT_STAT_LEAF] += 1;
    }
}

// Closest hit over the octree: BVH::intersect (bvh.cpp:62-65, bvh.h:127-209).
// Returns best_t (-1 if none) and the leaf-order triangle index.
RT_HD void trace_closest(const RtSceneView& S, V3 o, V3 d, StackEnt* stack, float& best_t, int& best_k, Stats* st)
{
    best_t = -1.0f;
    best_k = -1;
    RayK K;
    if (st) st->c[RT_STAT_RAYS]++;
    if (!ray_setup(o, d, K)) return;

    const RtNode root = S.nodes[0];
    float tn;
    if (st) st->c[RT_STAT_VOL]++;
    if (!slab_test(root, K, tn)) return;
    if (root.cnt & RT_LEAF_BIT) {
        leaf_test(S, root.ref, root.cnt, o, d, best_t, best_k, st);
        return;
    }
    int sp = 0;
    int leaves = 0;
    uint32_t rec = 0;
    RtNode nd = root;
    for (;;) {
        // ---- visit `nd` (internal): test its children, order, push
        {
            const int base = (int)nd.ref;
            const int nc = (int)nd.cnt;
            float hk[8];
            int hi[8];
            int m = 0;
            bool tie = false;
            for (int c = 0; c < nc; c++) {
                const RtNode ch = S.nodes[base + c];
                float t;
                if (slab_test(ch, K, t)) {
                    for (int j = 0; j < m; j++) tie |= (hk[j] == t);
                    hk[m] = t;
                    hi[m] = base + c;
                    m++;
                }
            }
            if (st) st->c[RT_STAT_VOL] += nc;
            if (m > 0) {
                float ok[8];
                int oi[8];
                if (tie) {
                    heap_order(hk, hi, m, ok, oi);
                    if (st) st->c[RT_STAT_HEAP_SLOW]++;
                } else {
                    // distinct keys: pop order is ascending t_near
                    for (int i = 0; i < m; i++) {
                        int r = 0;
                        for (int j = 0; j < m; j++) r += hk[j] < hk[i];
                        ok[r] = hk[i];
                        oi[r] = hi[i];
                    }
                }
                // push farthest first so the nearest is on top
                for (int i = m - 1; i >= 0; i--) {
                    uint32_t f = (uint32_t)oi[i];
                    if (i == 0) f |= RT_ENT_FIRST;
                    if (i == m - 1) f |= RT_ENT_LAST;
                    stack[sp].rec = f;
                    stack[sp].tnear = ok[i];
                    stack[sp].snap = 0;
                    sp++;
                }
            }
        }
        // ---- pop the next node to visit
        for (;;) {
            if (sp == 0) return;
            const StackEnt e = stack[--sp];
            if (!(e.rec & RT_ENT_FIRST)) {
                // the previous sibling returned true iff it visited a leaf
                // and a hit exists
                const bool prev_true = best_t > 0.0f && leaves > e.snap;
                const float closest = rt_min(100000000.0f, best_t);
                if (prev_true && closest < e.tnear) {
                    // early exit of the parent: drop e and its remaining siblings
                    if (!(e.rec & RT_ENT_LAST))
                        while (!(stack[--sp].rec & RT_ENT_LAST)) {
                        }
                    continue;
                }
            }
            if (!(e.rec & RT_ENT_LAST)) stack[sp - 1].snap = leaves;
            rec = e.rec & RT_ENT_MASK;
            nd = S.nodes[rec];
            if (nd.cnt & RT_LEAF_BIT) {
                leaf_test(S, nd.ref, nd.cnt, o, d, best_t, best_k, st);
                leaves++;
                continue;
            }
            break;  // internal: expand it
        }
    }
}

// ------------------------------------------- short-stack closest-hit walk
// The same traversal as trace_closest() with a bounded stack of 8-byte
// entries (record | FIRST | LAST, t_near) that the gfx950 kernel keeps in
// LDS. Two changes of representation, no change of order or result:
//  * "the previous sibling returned true" needs "a leaf was visited since
//    that sibling was popped": one bit per stack group level in `lmask`,
//    cleared when a non-last entry of the level is popped, set (all levels)
//    on every leaf visit — instead of a leaf-count snapshot per entry;
//  * equal-key children are ordered by running std::push_heap / pop_heap in
//    place over their stack slots: pop_heap leaves the popped element at the
//    end of the range, so after m pops slot sp+m-1 holds the first popped
//    (nearest) child — exactly the push layout (nearest on top).
// Returns false if the stack would overflow (the caller re-traces the ray
// with trace_closest()); best_t / best_k are then meaningless.
template <class STK>
RT_HD void stk_sift_up(STK& s, int base, int hole, float key, uint32_t val)
{
    int parent = (hole - 1) / 2;
    while (hole > 0 && s.key(base + parent) > key) {
        s.set(base + hole, s.rec(base + parent), s.key(base + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    s.set(base + hole, val, key);
}

template <class STK>
RT_HD void stk_pop_heap(STK& s, int base, int len)  // std::pop_heap on [base, base+len)
{
    if (len <= 1) return;
    const int L = len - 1;
    const float key = s.key(base + L);
    const uint32_t val = s.rec(base + L);
    s.set(base + L, s.rec(base), s.key(base));
    int hole = 0, second = 0;
    while (second < (L - 1) / 2) {
        second = 2 * (second + 1);
        if (s.key(base + second) > s.key(base + second - 1)) second--;
        s.set(base + hole, s.rec(base + second), s.key(base + second));
        hole = second;
    }
    if ((L & 1) == 0 && second == (L - 2) / 2) {
        second = 2 * (second + 1);
        s.set(base + hole, s.rec(base + second - 1), s.key(base + second - 1));
        hole = second - 1;
    }
    stk_sift_up(s, base, hole, key, val);
}

template <class STK>
RT_HD bool trace_closest_short(const RtSceneView& S, V3 o, V3 d, STK& stk, float& best_t, int& best_k, Stats* st)
{
    best_t = -1.0f;
    best_k = -1;
    RayK K;
    if (st) st->c[RT_STAT_RAYS]++;
    if (!ray_setup(o, d, K)) return true;
    const RtNode root = S.nodes[0];
    float tn;
    if (st) st->c[RT_STAT_VOL]++;
    if (!slab_test(root, K, tn)) return true;
    if (root.cnt & RT_LEAF_BIT) {
        leaf_test(S, root.ref, root.cnt, o, d, best_t, best_k, st);
        return true;
    }
    int sp = 0, groups = 0;
    uint32_t lmask = 0;
    uint32_t base = root.ref, nc = root.cnt;
    for (;;) {
        // ---- expand an internal node: test its children, order, push
        {
            float hk[8];
            uint32_t hi[8];
            int m = 0;
            bool tie = false;
            for (uint32_t c = 0; c < nc; c++) {
                const NodeR ch = load_node(S.nodes, base + c);
                float t;
                if (slab_test(ch, K, t)) {
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        tie |= (j < m) && hk[j] == t;
                        if (j == m) {
                            hk[j] = t;
                            hi[j] = base + c;
                        }
                    }
                    m++;
                }
            }
            if (st) st->c[RT_STAT_VOL] += nc;
            if (m > 0) {
                if (sp + m > STK::CAP) return false;
                if (!tie) {
                    // distinct keys: pop order is ascending t_near; slot of rank r is sp+m-1-r
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        if (i < m) {
                            int r = 0;
#pragma unroll
                            for (int j = 0; j < 8; j++) r += (j < m) && hk[j] < hk[i];
                            stk.set(sp + m - 1 - r, hi[i], hk[i]);
                        }
                    }
                } else {
                    if (st) st->c[RT_STAT_HEAP_SLOW]++;
#pragma unroll
                    for (int i = 0; i < 8; i++)
                        if (i < m) stk_sift_up(stk, sp, i, hk[i], hi[i]);
                    for (int len = m; len > 1; len--) stk_pop_heap(stk, sp, len);
                }
                stk.set_rec(sp + m - 1, stk.rec(sp + m - 1) | RT_ENT_FIRST);
                stk.set_rec(sp, stk.rec(sp) | RT_ENT_LAST);
                sp += m;
                groups++;
            }
        }
        // ---- pop the next node to visit
        for (;;) {
            if (sp == 0) return true;
            --sp;
            const uint32_t er = stk.rec(sp);
            const uint32_t lvl = (uint32_t)(groups - 1);
            if (!(er & RT_ENT_FIRST)) {
                const bool prev_true = best_t > 0.0f && ((lmask >> lvl) & 1u);
                const float closest = rt_min(100000000.0f, best_t);
                if (prev_true && closest < stk.key(sp)) {
                    // early exit of the parent: drop this entry and its remaining siblings
                    if (!(er & RT_ENT_LAST))
                        while (!(stk.rec(--sp) & RT_ENT_LAST)) {
                        }
                    groups--;
                    continue;
                }
            }
            if (er & RT_ENT_LAST)
                groups--;
            else
                lmask &= ~(1u << lvl);
            const uint2_ link = load_link(S.nodes, er & RT_ENT_MASK);
            if (link.y & RT_LEAF_BIT) {
                leaf_test(S, link.x, link.y, o, d, best_t, best_k, st);
                lmask = ~0u;
                continue;
            }
            base = link.x;
            nc = link.y;
            break;
        }
    }
}

// Plain-array stack for the host build and the scratch fallback.
template <int N>
struct ArrayStack {
    static constexpr int CAP = N;
    uint32_t r[N];
    float k[N];
    RT_HD uint32_t rec(int i) const { return r[i]; }
    RT_HD float key(int i) const { return k[i]; }
    RT_HD void set(int i, uint32_t rv, float kv) { r[i] = rv, k[i] = kv; }
    RT_HD void set_rec(int i, uint32_t rv) { r[i] = rv; }
};

// Occlusion query: does the reference's traversal find ANY triangle hit?
// Pruning in BVH::intersect is by slab tests (independent of the hit state)
// and by the early exit, which only fires once a hit exists; so the
// reference finds a hit iff some leaf reachable through passing slab tests
// holds a triangle the ray hits. This walk visits that same reachable set
// in child order (no sorting) and stops at the first hit.
RT_HD bool trace_any(const RtSceneView& S, V3 o, V3 d, uint32_t* stack, Stats* st)
{
    RayK K;
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (!ray_setup(o, d, K)) return false;
    float tn;
    if (st) st->c[RT_STAT_ANY_VOL]++;
    if (!slab_test(S.nodes[0], K, tn)) return false;
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const RtNode nd = S.nodes[stack[--sp]];
        if (nd.cnt & RT_LEAF_BIT) {
            const int n = (int)(nd.cnt & ~RT_LEAF_BIT);
            if (st) {
                st->c[RT_STAT_ANY_TRI] += n;
                st->c[RT_STAT_ANY_LEAF] += 1;
            }
            for (int j = 0; j < n; j++) {
                float t;
                if (tri_test(S.tri4, (int)nd.ref + j, o, d, t)) return true;
            }
            continue;
        }
        const int base = (int)nd.ref, nc = (int)nd.cnt;
        if (st) st->c[RT_STAT_ANY_VOL] += nc;
        for (int c = nc - 1; c >= 0; c--) {
            if (slab_test(S.nodes[base + c], K, tn)) stack[sp++] = (uint32_t)(base + c);
        }
    }
    return false;
}

// trace_any() with a bounded stack: 1 hit, 0 no hit, -1 overflow (the
// caller re-runs trace_any() with an unbounded stack).
template <class STK>
RT_HD int trace_any_short(const RtSceneView& S, V3 o, V3 d, STK& stk, Stats* st)
{
    RayK K;
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (!ray_setup(o, d, K)) return 0;
    float tn;
    if (st) st->c[RT_STAT_ANY_VOL]++;
    if (!slab_test(S.nodes[0], K, tn)) return 0;
    int sp = 0;
    stk.set_rec(sp++, 0);
    while (sp > 0) {
        const uint2_ link = load_link(S.nodes, stk.rec(--sp));
        if (link.y & RT_LEAF_BIT) {
            const int n = (int)(link.y & ~RT_LEAF_BIT);
            if (st) {
                st->c[RT_STAT_ANY_TRI] += n;
                st->c[RT_STAT_ANY_LEAF] += 1;
            }
            for (int j = 0; j < n; j++) {
                float t;
                if (tri_test(S.tri4, (int)link.x + j, o, d, t)) return 1;
            }
            continue;
        }
        const int base = (int)link.x, nc = (int)link.y;
        if (st) st->c[RT_STAT_ANY_VOL] += nc;
        for (int c = nc - 1; c >= 0; c--) {
            if (slab_test(load_node(S.nodes, (uint32_t)(base + c)), K, tn)) {
                if (sp == STK::CAP) return -1;
                stk.set_rec(sp++, (uint32_t)(base + c));
            }
        }
    }
    return 0;
}

// Sphere::intersect (sphere.h:11-52)
RT_HD bool sphere_test(const float4_* sp, int i, V3 o, V3 d, Hit& h)
{
    const float4_ s0 = sp[2 * i];
    const V3 c = ld3(s0);
    V3 L = sub(o, c);
    float b = 2.0f * dot(d, L);
    float cc = dot(L, L) - s0.w * s0.w;
    float delta = b * b - 4.0f * 1.0f * cc;
    if (delta < 0.0f) return false;
    float t = -1.0f;
    if (delta == 0.0f)
        t = -b / 2.0f;
    else {
        float sq = rt_sqrtf(delta);
        float t1 = (-b - sq) / 2.0f, t2 = (-b + sq) / 2.0f;
        if (t1 < t2) {
            t = t1;
            if (t < 0.0f) t = t2;
        }
    }
    if (t < 0.0f) return false;
    h.t = t;
    h.p = add(o, mul(t, d));
    h.n = normalize(sub(h.p, c));
    h.prim = rt_asuint(sp[2 * i + 1].x);
    h.k = -2 - i;
    return true;
}

// ----------------------------------------------------------------- shading
struct Mat {
    Col emission, diffuse;
    float metalness, roughness;
};
// A material record: from the LDS copy when the shading kernel staged the table
// (lds_shade_init, n_mats <= RT_MAT_LDS), else from memory.
#define RT_MAT_LDS 64
#if defined(__HIPCC__)
__shared__ RtMat rt_mat_lds[RT_MAT_LDS];
#endif
RT_HD RtMat mat_rec(const RtSceneView& S, int i)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (S.n_mats <= RT_MAT_LDS) return rt_mat_lds[i];
#endif
    return S.mats[i];
}
RT_HD Mat load_mat(const RtSceneView& S, int prim)
{
    const RtMat m = mat_rec(S, S.mat_idx[prim]);
    return Mat{Col{m.er, m.eg, m.eb}, Col{m.dr, m.dg, m.db}, m.metalness, m.roughness};
}
// The material of a hit: for a triangle (leaf-order k >= 0) through matk[k],
// the same entry as mat_idx[prim] (built at upload), without the dependent load.
RT_HD Mat load_mat_hit(const RtSceneView& S, int k, int prim)
{
    const RtMat m = mat_rec(S, (k >= 0 && S.matk) ? S.matk[k] : S.mat_idx[prim]);
    return Mat{Col{m.er, m.eg, m.eb}, Col{m.dr, m.dg, m.db}, m.metalness, m.roughness};
}
// The material of a hit record (its material index already read with the triangle when
// the device records carry it: one dependent load fewer).
RT_HD Mat load_mat_of(const RtSceneView& S, const Hit& h)
{
    if (h.mi < 0) return load_mat_hit(S, h.k, h.prim);
    const RtMat m = mat_rec(S, h.mi);
    return Mat{Col{m.er, m.eg, m.eb}, Col{m.dr, m.dg, m.db}, m.metalness, m.roughness};
}

RT_HD V3 rotate_around_normal(V3 n, V3 l)  // render_kernel.cpp:5-22
{
    float sign = rt_copysignf(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float b = n.x * n.y * a;
    V3 b1 = v3(1.0f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    V3 b2 = v3(b, sign + n.y * n.y * a, -n.y);
    return add(add(mul(l.x, b1), mul(l.y, b2)), mul(l.z, n));
}

RT_HD Col fresnel_schlick(Col F0, float NoV)  // :218-221
{
    return cadd(F0, cscale(csub(col(1.0f), F0), rt_powf((1.0f - NoV), 5.0f)));
}
RT_HD float ggx_d(float alpha, float NoH)  // :223-233 (double division)
{
    NoH = rt_min(NoH, 0.999999f);
    float alpha2 = alpha * alpha;
    float NoH2 = NoH * NoH;
    float b = (NoH2 * (alpha2 - 1.0f) + 1.0f);
    return (float)((double)alpha2 * 0.31830988618379067154 / (double)(b * b));
}
RT_HD float g1(float k, float d) { return d / (d * (1.0f - k) + k); }
RT_HD float smith(float r2, float NoV, float NoL)
{
    float k = r2 / 2.0f;
    return g1(k, NoL) * g1(k, NoV);
}
#define RT_PI_F 3.14159265358979323846f

RT_HD float ct_pdf(const Mat& m, V3 V, V3 L, V3 N)  // :247-258
{
    V3 H = normalize(add(V, L));
    float alpha = m.roughness * m.roughness;
    float VoH = rt_max(0.0f, dot(V, H));
    float NoH = rt_max(0.0f, dot(N, H));
    float D = ggx_d(alpha, NoH);
    return D * NoH / (4.0f * VoH);
}

RT_HD Col ct_lobe(const Mat& m, float NoV, float NoL, float NoH, float VoH, float alpha, float* D_out)
{
    Col F0 = cadd(col(0.04f * (1.0f - m.metalness)), cscale(m.diffuse, m.metalness));
    Col F = fresnel_schlick(F0, VoH);
    float D = ggx_d(alpha, NoH);
    float G = smith(alpha, NoV, NoL);
    Col kD = col(1.0f - m.metalness);
    kD = cmul(kD, csub(col(1.0f), F));
    Col diffuse = cdiv(cmul(kD, m.diffuse), RT_PI_F);
    Col spec = cdiv(cscale(cscale(F, D), G), 4.0f * NoV * NoL);
    if (D_out) *D_out = D;
    return cadd(diffuse, spec);
}

RT_HD Col ct_brdf(const Mat& m, V3 L, V3 V, V3 N)  // :260-301
{
    V3 H = normalize(add(V, L));
    float NoV = rt_max(0.0f, dot(N, V));
    float NoL = rt_max(0.0f, dot(N, L));
    float NoH = rt_max(0.0f, dot(N, H));
    float VoH = rt_max(0.0f, dot(H, V));
    if (NoV > 0.0f && NoL > 0.0f && NoH > 0.0f) return ct_lobe(m, NoV, NoL, NoH, VoH, m.roughness * m.roughness, nullptr);
    return col(0.0f);
}

// cook_torrance_brdf_importance_sample (:392-451). out_dir is left untouched
// when the sampled microfacet normal is below the surface.
RT_HD Col ct_sample(const Mat& m, V3 V, V3 N, V3& out_dir, float& pdf, Rng& rng)
{
    pdf = 0.0f;
    const float alpha = m.roughness * m.roughness;
    float r1 = rng.next();
    float r2 = rng.next();
    float phi = 2.0f * RT_PI_F * r1;
    float theta = rt_acosf((1.0f - r2) / (r2 * (alpha * alpha - 1.0f) + 1.0f));
    float sin_theta, cos_theta, sin_phi, cos_phi;
    rt_sincosf(theta, sin_theta, cos_theta);
    rt_sincosf(phi, sin_phi, cos_phi);
    V3 local = v3(cos_phi * sin_theta, sin_phi * sin_theta, cos_theta);
    V3 mn = rotate_around_normal(N, local);
    if (dot(mn, N) < 0.0f) return col(0.0f);
    V3 L = normalize(sub(mul(2.0f * dot(mn, V), mn), V));
    out_dir = L;
    float NoV = rt_max(0.0f, dot(N, V));
    float NoL = rt_max(0.0f, dot(N, L));
    float NoH = rt_max(0.0f, dot(N, mn));
    float VoH = rt_max(0.0f, dot(mn, V));
    if (NoV > 0.0f && NoL > 0.0f && NoH > 0.0f) {
        float D;
        Col out = ct_lobe(m, NoV, NoL, NoH, VoH, alpha, &D);
        pdf = D * NoH / (4.0f * VoH);
        return out;
    }
    return col(0.0f);
}

RT_HD float power_heuristic(float a, float b)
{
    float a2 = a * a;
    return a2 / (a2 + b * b);
}

RT_HD Col env_texel(const RtSceneView& S, int x, int y, Stats* st)
{
    if (st) st->c[RT_STAT_ENV]++;
    const float4_ e = S.env[y * S.ew + x];
    return Col{e.x, e.y, e.z};
}

RT_HD Col env_from_dir(const RtSceneView& S, V3 d, Stats* st)  // :520-530
{
    float u = 0.5f + rt_atan2f(d.z, d.x) / (2.0f * RT_PI_F);
    float v = 0.5f + rt_asinf(d.y) / RT_PI_F;
    int x = rt_maxi(rt_mini(rt_f2i(u * (float)S.ew), S.ew - 1), 0);
    int y = rt_maxi(rt_mini(rt_f2i(v * (float)S.eh), S.eh - 1), 0);
    return env_texel(S, x, y, st);
}

// Counting form of the reference's search. Its loop (lower = 0, upper =
// m; while lower < upper: mid = (lower + upper) / 2; value < a[mid] ? upper
// = mid : lower = mid + 1) never reads a[m] and, on a sequence where the
// predicate !(value < a[i]) is a prefix (a non-decreasing sequence without
// NaN, checked on the host — rt_scene.cpp env_cdf_fences), returns the length
// of that prefix within [0, m): #{i < m : !(value < a[i])}. A NaN value makes
// every predicate true and returns m, as the loop does. The count is read
// off three levels of 16 fences, one 64-B load each: block ends at 256 (t[0..16)),
// block ends at 16 (t[16..272)), then the 16 entries themselves.
// One level of fence_count: the 16 entries of block b at lv + c / b (one 64-B load).
RT_HD int fence_level(const float* lv, int c, int b, int m, float value)
{
    const float4_* p = (const float4_*)(lv + c / b);
    const float4_ q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    const float k[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                         q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    int n = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) n += (c + b * (j + 1) - 1 < m && !(value < k[j])) ? 1 : 0;
    return c + n * b;
}

RT_HD int fence_count(const float* a, const float* t, int m, float value)
{
    int c = fence_level(t, 0, 256, m, value);
    c = fence_level(t + 16, c, 16, m, value);
    return fence_level(a, c, 1, m, value);
}

// The row search's fence table and row ends staged in LDS by the shading kernels
// (lds_cdf_init: k_step, k_tail), so three of the search's six dependent loads are LDS
// reads. RT_CDF_LDS 0: every level from global memory.
#ifndef RT_CDF_LDS
#define RT_CDF_LDS 1
#endif
#define RT_CDF_LDS_ROWS 1024
#if defined(__HIPCC__) && RT_CDF_LDS
__shared__ float4_ rt_cdf_lds[(272 + RT_CDF_LDS_ROWS) / 4];  // fence table 0 (272), then cdf_row
#endif
#if defined(__HIPCC__)
// The shading kernels' LDS copies (k_step, k_tail; whole block, ends with a barrier).
__device__ __forceinline__ void lds_shade_init(const RtSceneView& S)
{
#if RT_CDF_LDS
    if (S.cdf_fence && S.eh <= RT_CDF_LDS_ROWS) {
        float* t = (float*)rt_cdf_lds;
        for (int i = (int)threadIdx.x; i < 272 + S.eh; i += (int)blockDim.x)
            t[i] = i < 272 ? S.cdf_fence[i] : S.cdf_row[i - 272];
    }
#endif
    if (S.n_mats <= RT_MAT_LDS)
        for (int i = (int)threadIdx.x; i < S.n_mats; i += (int)blockDim.x) rt_mat_lds[i] = S.mats[i];
    __syncthreads();
}
#endif

RT_HD void cdf_search(const RtSceneView& S, float value, int& x, int& y, Stats* st)  // :532-567
{
    if (S.cdf_fence) {
#if defined(__HIP_DEVICE_COMPILE__) && RT_CDF_LDS
        if (S.eh <= RT_CDF_LDS_ROWS) {
            const float* t = (const float*)rt_cdf_lds;
            y = fence_count(t + 272, t, S.eh - 1, value);
        } else
#endif
        y = fence_count(S.cdf_row, S.cdf_fence, S.eh - 1, value);
        x = fence_count(S.cdf + (size_t)y * S.ew, S.cdf_fence + (size_t)(1 + y) * 272, S.ew - 1, value);
        if (st) st->c[RT_STAT_CDF] += 6;  // six 64-B fence loads
        return;
    }
    int lower = 0, upper = S.eh - 1;
    const int xi = S.ew - 1;
    int probes = 0;
    (void)xi;
    // Same probes and comparisons as the reference; the values come from
    // exact copies laid out for locality: cdf_row[y] = cdf[y*ew + ew-1]
    // (the row search reads one 4-KB array) and cdf_coarse[y][j] =
    // cdf[y*ew + 32j + 31] (for a power-of-two width the first column probes
    // all land there, the rest inside one 128-B line).
    while (lower < upper) {
        int yi = (lower + upper) / 2;
        probes++;
        if (value < S.cdf_row[yi])
            upper = yi;
        else
            lower = yi + 1;
    }
    y = rt_maxi(rt_mini(lower, S.eh), 0);
    lower = 0;
    upper = S.ew - 1;
    const float* row = S.cdf + (size_t)y * S.ew;
    const float* crow = S.cdf_coarse + (size_t)y * S.cdf_cw;
    while (lower < upper) {
        int xm = (lower + upper) / 2;
        probes++;
        const float c = ((xm & 31) == 31 && (xm >> 5) < S.cdf_cw) ? crow[xm >> 5] : row[xm];
        if (value < c)
            upper = xm;
        else
            lower = xm + 1;
    }
    x = rt_maxi(rt_mini(lower, S.ew), 0);
    if (st) st->c[RT_STAT_CDF] += probes;
}

}  // namespace rtk
