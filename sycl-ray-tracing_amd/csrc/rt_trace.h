// rt_trace.h — the per-pixel path tracer that runs on gfx950 (and, compiled
// for the host, in the hostsim test build).
//
// Restates source/render_kernel.cpp (ray_trace_pixel and everything it calls)
// with the reference's exact float/double evaluation order. Differences are
// purely structural:
//  * BVH: the recursive priority-queue octree traversal (bvh.h:127-209) is
//    re-expressed as an explicit-stack walk over RtNode child blocks that
//    visits nodes in the identical order (libstdc++ heap tie order included)
//    and applies the identical early-exit rule; see trace_closest().
//  * libm: rt_libm.h (glibc-bit-exact).
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
    V3 p, n;
};

RT_HD V3 ld3(const float4_& f) { return v3(f.x, f.y, f.z); }

// plane normals (bvh.cpp:8-16)
#define RT_S3 0.577350269f
RT_HD void ray_planes(V3 o, V3 d, float* den, float* num)
{
    const float s = rt_sqrtf(3.0f) / 3;
    const V3 N[7] = {v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1), v3(s, s, s), v3(-s, s, s), v3(-s, -s, s), v3(s, -s, s)};
#pragma unroll
    for (int i = 0; i < 7; i++) {
        den[i] = dot(N[i], d);
        num[i] = dot(N[i], o);
    }
}

// BoundingVolume::intersect (bounding_volume.h:101-126). The early
// `t_far < t_near` exit inside the loop cannot change the outcome (prefix
// max/min are monotone), so the slab loop runs to completion.
RT_HD bool slab_test(const RtNode& nd, const float* den, const float* num, float& tnear)
{
    float tn = -__builtin_inff(), tf = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const float d = den[i];
        if (d == 0.0f) continue;
        float a = (nd.dn[i] - num[i]) / d;
        float b = (nd.df[i] - num[i]) / d;
        if (d < 0.0f) {
            float t = a;
            a = b;
            b = t;
        }
        tn = rt_max(tn, a);
        tf = rt_min(tf, b);
    }
    tnear = tn;
    return !(tf < tn);
}

// Triangle::intersect (triangle.h:16-60) on the pre-subtracted record.
RT_HD bool tri_test(const float4_* tri4, int k, V3 o, V3 d, float& t_out)
{
    const V3 a = ld3(tri4[3 * k]), e1 = ld3(tri4[3 * k + 1]), e2 = ld3(tri4[3 * k + 2]);
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

RT_HD void leaf_test(const RtSceneView& S, const RtNode& nd, V3 o, V3 d, float& best_t, int& best_k, Stats* st)
{
    const int n = (int)(nd.cnt & ~RT_LEAF_BIT);
    const int k0 = (int)nd.ref;
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
    float den[7], num[7];
    ray_planes(o, d, den, num);
    if (st) st->c[RT_STAT_RAYS]++;
    // A NaN component makes every slab test pass and every triangle test
    // fail (NaN compares false), so such a ray can never hit: skip the walk.
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 7; i++) bad = bad || rt_isnan(den[i]) || rt_isnan(num[i]);
    if (bad) return;

    const RtNode root = S.nodes[0];
    float tn;
    if (st) st->c[RT_STAT_VOL]++;
    if (!slab_test(root, den, num, tn)) return;
    if (root.cnt & RT_LEAF_BIT) {
        leaf_test(S, root, o, d, best_t, best_k, st);
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
                if (slab_test(ch, den, num, t)) {
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
                leaf_test(S, nd, o, d, best_t, best_k, st);
                leaves++;
                continue;
            }
            break;  // internal: expand it
        }
    }
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

// INTERSECT_SCENE = intersect_scene_bvh (render_kernel.cpp:485-502)
RT_HD bool intersect_scene(const RtSceneView& S, V3 o, V3 d, StackEnt* stack, Hit& h, Stats* st)
{
    float t;
    int k;
    trace_closest(S, o, d, stack, t, k, st);
    h.t = t;
    h.k = k;
    h.prim = -1;
    if (k >= 0) {
        // HitInfo fields of the winning Triangle::intersect (triangle.h:46-56)
        const V3 e1 = ld3(S.tri4[3 * k + 1]), e2 = ld3(S.tri4[3 * k + 2]);
        h.p = add(o, mul(t, d));
        h.n = normalize(cross(e1, e2));
        h.prim = (int)rt_asuint(S.tri4[3 * k].w);
    }
    for (int i = 0; i < S.n_spheres; i++) {
        Hit sh;
        if (sphere_test(S.spheres, i, o, d, sh))
            if (sh.t < h.t || h.t == -1.0f) h = sh;
    }
    return h.t > 0.0f;
}

// ----------------------------------------------------------------- shading
struct Mat {
    Col emission, diffuse;
    float metalness, roughness;
};
RT_HD Mat load_mat(const RtSceneView& S, int prim)
{
    const RtMat m = S.mats[S.mat_idx[prim]];
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
    float sin_theta = rt_sinf(theta);
    V3 local = v3(rt_cosf(phi) * sin_theta, rt_sinf(phi) * sin_theta, rt_cosf(theta));
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

RT_HD void cdf_search(const RtSceneView& S, float value, int& x, int& y, Stats* st)  // :532-567
{
    int lower = 0, upper = S.eh - 1;
    const int xi = S.ew - 1;
    int probes = 0;
    while (lower < upper) {
        int yi = (lower + upper) / 2;
        probes++;
        if (value < S.cdf[yi * S.ew + xi])
            upper = yi;
        else
            lower = yi + 1;
    }
    y = rt_maxi(rt_mini(lower, S.eh), 0);
    lower = 0;
    upper = S.ew - 1;
    while (lower < upper) {
        int xm = (lower + upper) / 2;
        probes++;
        if (value < S.cdf[y * S.ew + xm])
            upper = xm;
        else
            lower = xm + 1;
    }
    x = rt_maxi(rt_mini(lower, S.ew), 0);
    if (st) st->c[RT_STAT_CDF] += probes;
}

struct Ctx {
    RtSceneView S;
    RtCamera cam;
    int W, H, spp, bounces;
};

RT_HD bool occluded(const Ctx& C, V3 o, V3 d, StackEnt* stack, Stats* st)
{
    Hit h;
    return intersect_scene(C.S, o, d, stack, h, st);
}

RT_HD Col sample_env(const Ctx& C, V3 rd, const Hit& h, const Mat& m, Rng& rng, StackEnt* stack, Stats* st)
{
    const RtSceneView& S = C.S;
    const float total = S.cdf[S.ew * S.eh - 1];
    int x, y;
    cdf_search(S, rng.next() * total, x, y, st);
    float u = (float)x / (float)S.ew, v = (float)y / (float)S.eh;
    float phi = (float)((double)(u * 2.0f) * 3.14159265358979323846);
    float theta = (float)((double)v * 3.14159265358979323846);
    Col env_sample = col(0.0f);
    float st_ = rt_sinf(theta), ct_ = rt_cosf(theta);
    V3 dir = v3(-st_ * rt_cosf(phi), -ct_, -st_ * rt_sinf(phi));
    float cosine = dot(h.n, dir);
    if (cosine > 0.0f) {
        if (!occluded(C, add(h.p, mul(1.0e-4f, h.n)), dir, stack, st)) {
            float pdf = S.env_lum[y * S.ew + x] / total;
            pdf = (float)((double)((pdf * (float)S.ew) * (float)S.eh) /
                          (2.0 * 3.14159265358979323846 * 3.14159265358979323846 * (double)st_));
            Col rad = env_texel(S, x, y, st);
            Col brdf = ct_brdf(m, dir, neg(rd), h.n);
            float bp = ct_pdf(m, neg(rd), dir, h.n);
            float mis = power_heuristic(pdf, bp);
            env_sample = cdiv(cmul(cscale(cscale(brdf, cosine), mis), rad), pdf);
        }
    }
    float bsp;
    V3 bdir = v3(0.0f, 0.0f, 0.0f);
    Col bis = ct_sample(m, neg(rd), h.n, bdir, bsp, rng);
    cosine = rt_max(dot(h.n, bdir), 0.0f);
    Col brdf_sample = col(0.0f);
    if (bsp != 0.0f && cosine > 0.0f) {
        if (!occluded(C, add(h.p, mul(1.0e-5f, h.n)), bdir, stack, st)) {
            Col sky = env_from_dir(S, bdir, st);
            float th = rt_acosf(bdir.z);
            float sth = rt_sinf(th);
            float epdf = (0.3086f * sky.r + 0.6094f * sky.g + 0.0820f * sky.b) / S.cdf[S.ew * S.eh - 1];
            epdf *= (float)(S.ew * S.eh);
            epdf = (float)((double)epdf / (2.0 * 3.14159265358979323846 * 3.14159265358979323846 * (double)sth));
            float mis = power_heuristic(bsp, epdf);
            brdf_sample = cdiv(cmul(cscale(cscale(sky, mis), cosine), bis), bsp);
        }
    }
    return cadd(brdf_sample, env_sample);
}

RT_HD Col sample_lights(const Ctx& C, V3 rd, const Hit& h, const Mat& m, Rng& rng, StackEnt* stack, Stats* st)
{
    const RtSceneView& S = C.S;
    Col light = col(0.0f);
    if (S.n_emissive > 0) {
        // sample_random_point_on_lights (:715-742)
        int li = rt_f2i(rng.next() * (float)S.n_emissive);
        li = S.emissive[li];
        const int lk = S.prim2k[li];
        const V3 A = ld3(S.tri4[3 * lk]), AB = ld3(S.tri4[3 * lk + 1]), AC = ld3(S.tri4[3 * lk + 2]);
        float r1 = rng.next();
        float r2 = rng.next();
        float sr1 = rt_sqrtf(r1);
        float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
        V3 P = add(add(A, mul(u, AB)), mul(v, AC));
        V3 nrm = cross(AB, AC);
        float ln = length(nrm);
        V3 lnorm = mul(1 / ln, nrm);
        float area = ln * 0.5f;
        float nb = (float)S.n_emissive;
        float lpdf = 1.0f / (nb * area);

        V3 so = add(h.p, mul(1.0e-4f, h.n));
        V3 sd = sub(P, so);
        float dist = length(sd);
        V3 sdn = normalize(sd);
        float dl = rt_max(dot(lnorm, neg(sdn)), 0.0f);
        if (dl > 0.0f) {
            Hit sh;  // evaluate_shadow_ray (:744-759)
            bool in_shadow = false;
            if (intersect_scene(S, so, sdn, stack, sh, st)) in_shadow = sh.t + 1.0e-4f < dist;
            if (!in_shadow) {
                if (st) st->c[RT_STAT_MAT]++;
                const Mat em = load_mat(S, li);
                lpdf *= dist * dist;
                lpdf /= dl;
                Col brdf = ct_brdf(m, sdn, neg(rd), h.n);
                float cp = ct_pdf(m, neg(rd), sdn, h.n);
                if (cp != 0.0f) {
                    float mis = power_heuristic(lpdf, cp);
                    float cosine = dot(h.n, sdn);
                    light = cdiv(cscale(cmul(cscale(em.emission, cosine), brdf), mis), lpdf);
                }
            }
        }
    }
    Col bmis = col(0.0f);
    V3 sdir = v3(0.0f, 0.0f, 0.0f);
    float dpdf;
    Col brdf = ct_sample(m, neg(rd), h.n, sdir, dpdf, rng);
    if (!(brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f)) {
        Hit nh;
        if (intersect_scene(S, add(h.p, mul(1.0e-5f, h.n)), sdir, stack, nh, st)) {
            float ca = rt_max(dot(nh.n, neg(sdir)), 0.0f);
            if (ca > 0.0f) {
                if (st) st->c[RT_STAT_MAT]++;
                const Mat mm = load_mat(S, nh.prim);
                const Col e = mm.emission;
                if (e.r > 0 || e.g > 0 || e.b > 0) {
                    float d2 = nh.t * nh.t;
                    // Triangle::area (triangle.cpp:8-11) of the hit triangle
                    // (an emissive *sphere* hit reads past the triangle buffer in the
                    // reference — undefined behaviour; we use area 0 there)
                    const int kk = nh.k >= 0 ? nh.k : (nh.prim >= 0 && nh.prim < S.n_tris ? S.prim2k[nh.prim] : -1);
                    float la = kk < 0 ? 0.0f : length(cross(ld3(S.tri4[3 * kk + 1]), ld3(S.tri4[3 * kk + 2]))) / 2;
                    float lp = d2 / (la * ca);
                    float mis = power_heuristic(dpdf, lp);
                    float cosine = dot(h.n, sdir);
                    bmis = cdiv(cscale(cmul(cscale(brdf, cosine), e), mis), dpdf);
                }
            }
        }
    }
    return cadd(light, bmis);
}

RT_HD V3 xform_point(const RtCamera& c, V3 p)  // mat.cpp:94-111
{
    const float* m = c.m;
    float xt = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yt = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zt = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wt = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    float w = 1.f / wt;
    if (wt == 1.f) return v3(xt, yt, zt);
    return v3(xt * w, yt * w, zt * w);
}

// RenderKernel::ray_trace_pixel (render_kernel.cpp:75-181): returns the
// HDR pixel colour `final_color` (before it is added to the framebuffer).
RT_HD Col trace_pixel(const Ctx& C, int x, int y, StackEnt* stack, Stats* st)
{
    const RtSceneView& S = C.S;
    Rng rng{(uint32_t)(31 + x * y * C.spp)};
    for (int i = 0; i < 10; i++) rng.next();
    Col fin = col(0.0f);
    const V3 o = xform_point(C.cam, v3(0.0f, 0.0f, 0.0f));
    for (int s = 0; s < C.spp; s++) {
        float xj = ((float)x + 0.5f) + rng.next() - 1.0f;
        float yj = ((float)y + 0.5f) + rng.next() - 1.0f;
        // get_camera_ray (:56-73)
        float xn = xj / (float)C.W * 2.0f - 1.0f;
        xn *= (float)C.W / (float)C.H;
        float yn = yj / (float)C.H * 2.0f - 1.0f;
        V3 pd = xform_point(C.cam, v3(xn, yn, C.cam.fov_dist));
        V3 ro = o, rd = normalize(sub(pd, o));
        Col thr = col(1.0f), sc = col(0.0f);
        int state = 0;  // 0 BOUNCE, 1 MISSED
        for (int bounce = 0; bounce < C.bounces; bounce++) {
            if (state == 0) {
                Hit h;
                if (intersect_scene(S, ro, rd, stack, h, st)) {
                    if (st) st->c[RT_STAT_MAT]++;
                    const Mat m = load_mat(S, h.prim);
                    Col lr = sample_lights(C, rd, h, m, rng, stack, st);
                    Col er = sample_env(C, rd, h, m, rng, stack, st);
                    float bpdf;
                    V3 dir = v3(0.0f, 0.0f, 0.0f);
                    Col brdf = ct_sample(m, neg(rd), h.n, dir, bpdf, rng);
                    if (bounce == 0) sc = cadd(sc, m.emission);
                    sc = cadd(sc, cmul(cadd(lr, er), thr));
                    if ((brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f) || bpdf < 1.0e-8f || rt_isinf(bpdf))
                        break;
                    thr = cmul(thr, cdiv(cscale(brdf, rt_max(0.0f, dot(dir, h.n))), bpdf));
                    ro = add(h.p, mul(1.0e-4f, h.n));
                    rd = dir;
                } else
                    state = 1;
            } else {
                if (bounce == 1) sc = cadd(sc, cmul(env_from_dir(S, rd, st), thr));
                break;
            }
        }
        fin = cadd(fin, sc);
    }
    const float k = (float)C.spp;
    fin.r /= k;
    fin.g /= k;
    fin.b /= k;
    return fin;
}

// framebuffer update + exposure / gamma tone-map (:167-180), in place.
RT_HD void tonemap_into(float* px, Col fin)
{
    px[0] += fin.r;
    px[1] += fin.g;
    px[2] += fin.b;
    const float a = px[3] + 0.0f;
    px[3] = 1.0f + (-((-a) * 1.5f));
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float e = rt_expf((-px[c]) * 1.5f);
        float tm = 1.0f + (-e);
        px[c] = rt_powf(tm, 1.0f / 2.2f);
    }
}

}  // namespace rtk
