// rt_octet.h — the exact octree walks (rt_traverse.h) run by 8 lanes per query
// (gfx950 only; k_step's exact roles).
//
// A query the search-BVH walk cannot settle (a tie, a failed verification, a
// stack overflow: ~1e-6 of them) is answered by the reference's own octree walk,
// whose cost is a chain of dependent loads: rt_traverse.h takes one child volume
// or one triangle per step, so a node of 8 children is 8 round trips plus the
// pop's link load. A k_step launch that holds such a walk lasts as long as it
// (cfg4 8-way shard, one lane: sparse k_step 37-53 us without a fallback,
// 144-192 us with one, profiles/r04l_iter1.json), and every path of the lane
// waits for that launch.
//
// Here the 8 lanes of an octet load and test a node's children (or 8 triangles
// of a leaf) at once; everything that orders the walk — the push order, the
// distinct-key ranks, the libstdc++ heap emulation for equal keys, the
// FIRST / LAST group flags, the early-exit pop — is rt_traverse.h's code, run by
// all 8 lanes alike on octet-uniform state, so the visit order, the answer and
// the tie order are exactly trace_closest()'s / trace_any()'s. The stack is a
// 32-entry ring per octet in LDS over the leader lane's global spill area (as
// SpillStack), and each ring entry also keeps the child's (ref, cnt), read with
// its box, so a pop needs no link load: one round trip per node.
//
// Contract: the 8 lanes of an octet (lanes 8k .. 8k+7 of the wave) call these
// functions together with the same T (octet-uniform control flow).
#pragma once

#include "rt_traverse.h"
#include "rt_row.h"

namespace rtk {

#define RT_OCT_CAP 32                // ring entries per octet (4 LDS words each)
#define RT_OCT_NOLINK 0xffffffffu    // ring entry without its node's (ref, cnt): load the link

// An octet's stack window: entry i at slot i & (CAP - 1); below `lo` in the spill area.
struct OctRing {
    static constexpr int CAP = RT_OCT_CAP, MASK = RT_OCT_CAP - 1;
    uint32_t* r;   // record | FIRST | LAST
    float* k;      // t_near
    uint32_t* lr;  // the node's ref
    uint32_t* lc;  // the node's cnt (RT_OCT_NOLINK: unknown)
    __device__ __forceinline__ uint32_t rec(int i) const { return r[i & MASK]; }
    __device__ __forceinline__ float key(int i) const { return k[i & MASK]; }
    __device__ __forceinline__ void set(int i, uint32_t rv, float kv)
    {
        r[i & MASK] = rv;
        k[i & MASK] = kv;
    }
    __device__ __forceinline__ void set_rec(int i, uint32_t rv) { r[i & MASK] = rv; }
};

// The octet's ring in a block's LDS (4 * RT_OCT_CAP words per octet, 32 octets per block of 256).
__device__ __forceinline__ OctRing oct_ring(uint32_t* lds)
{
    uint32_t* g = lds + (threadIdx.x >> 3) * (4 * RT_OCT_CAP);
    return OctRing{g, (float*)(g + RT_OCT_CAP), g + 2 * RT_OCT_CAP, g + 3 * RT_OCT_CAP};
}

__device__ __forceinline__ unsigned oct_bits(unsigned long long b) { return (unsigned)(b >> (__lane_id() & 56)) & 0xFFu; }
__device__ __forceinline__ int oct_lane0() { return (int)(__lane_id() & 56); }

struct TravG {
    V3 o, d;
    RayK K;
    float best_t;
    int best_k;
    int sp, lo, groups;
    uint32_t lmask;
    int mode;
    uint32_t base, n;
    int steps;
    bool hit;  // (occlusion)
};

__device__ __forceinline__ void octg_enter(TravG& T, uint32_t ref, uint32_t cnt)
{
    T.base = ref;
    T.n = cnt & ~RT_LEAF_BIT;
    T.mode = (cnt & RT_LEAF_BIT) ? TM_LEAF : TM_EXPAND;
}

__device__ __forceinline__ bool octg_setup(const RtSceneView& S, TravG& T, V3 o, V3 d, Stats* st, bool any, int sub)
{
    T.o = o;
    T.d = d;
    T.best_t = -1.0f;
    T.best_k = -1;
    T.sp = T.lo = T.groups = 0;
    T.lmask = 0;
    T.steps = 0;
    T.hit = false;
    T.mode = TM_DONE;
    if (st && sub == 0) st->c[any ? RT_STAT_ANY_RAYS : RT_STAT_RAYS]++;
    if (S.brute) {  // USE_BVH 0 (test configurations): the loop answers at once
        if (any)
            T.hit = brute_any(S, o, d);
        else
            brute_closest(S, o, d, T.best_t, T.best_k);
        return false;
    }
    if (!ray_setup(o, d, T.K)) return false;
    float tn;
    if (st && sub == 0) st->c[any ? RT_STAT_ANY_VOL : RT_STAT_VOL]++;
    const NodeR root = load_node(S.nodes, 0);
    if (!slab_test(root, T.K, tn)) return false;
    octg_enter(T, root.ref, root.cnt);
    return true;
}

// The node's children (lane j: child j) or one 8-triangle chunk of a leaf, loaded and tested.
struct OctProbe {
    bool h;
    float t;
    uint32_t ref, cnt;
};
__device__ __forceinline__ OctProbe oct_children(const RtSceneView& S, const TravG& T, int sub)
{
    OctProbe p{false, 0.0f, 0u, RT_OCT_NOLINK};
    if ((uint32_t)sub < T.n) {
        const NodeR ch = load_node(S.nodes, T.base + (uint32_t)sub);
        p.h = slab_test(ch, T.K, p.t);
        p.ref = ch.ref;
        p.cnt = ch.cnt;
    }
    return p;
}

// A ring entry's node: from the ring when it holds the link, else the node record's link.
__device__ __forceinline__ void oct_link(const RtSceneView& S, const OctRing& w, int i, bool inwin, uint32_t er,
                                         uint32_t& ref, uint32_t& cnt)
{
    cnt = inwin ? w.lc[i & OctRing::MASK] : RT_OCT_NOLINK;
    ref = inwin ? w.lr[i & OctRing::MASK] : 0u;
    if (cnt == RT_OCT_NOLINK) {
        const uint2_ link = load_link(S.nodes, er & RT_ENT_MASK);
        ref = link.x;
        cnt = link.y;
    }
}

// ---------------------------------------------------------------- closest hit
// travc_pop, on the ring.
__device__ __forceinline__ void octc_pop(const RtSceneView& S, TravG& T, const OctRing& w, const uint32_t* spr,
                                         const float* spk)
{
    for (;;) {
        if (T.sp == 0) {
            T.mode = TM_DONE;
            return;
        }
        const int i = --T.sp;
        const bool inwin = i >= T.lo;
        const uint32_t er = inwin ? w.rec(i) : spr[i];
        const float ek = (er & RT_ENT_FIRST) ? 0.0f : (inwin ? w.key(i) : spk[i]);
        uint32_t ref, cnt;
        if (T.sp < T.lo) T.lo = T.sp;
        const uint32_t lvl = (uint32_t)(T.groups - 1);
        if (!(er & RT_ENT_FIRST)) {
            const bool prev_true = T.best_t > 0.0f && ((T.lmask >> lvl) & 1u);
            const float closest = rt_min(100000000.0f, T.best_t);
            if (prev_true && closest < ek) {
                // early exit of the parent: drop this entry and its remaining siblings
                if (!(er & RT_ENT_LAST))
                    for (;;) {
                        const int j = --T.sp;
                        if ((j >= T.lo ? w.rec(j) : spr[j]) & RT_ENT_LAST) break;
                    }
                if (T.sp < T.lo) T.lo = T.sp;
                T.groups--;
                continue;
            }
        }
        if (er & RT_ENT_LAST)
            T.groups--;
        else
            T.lmask &= ~(1u << lvl);
        oct_link(S, w, i, inwin, er, ref, cnt);
        octg_enter(T, ref, cnt);
        return;
    }
}

// One node (all its children, or all triangles of a leaf), then the pops to the next node
// (travc_step's work for the node, in its order).
__device__ __forceinline__ void octc_node(const RtSceneView& S, TravG& T, OctRing& w, uint32_t* spr, float* spk,
                                          int sub, Stats* st)
{
    const int g0 = oct_lane0();
    if (T.mode == TM_LEAF) {
        if (st && sub == 0) {
            st->c[RT_STAT_TRI] += T.n;
            st->c[RT_STAT_LEAF]++;
        }
        for (uint32_t c0 = 0; c0 < T.n; c0 += 8) {
            float t = 0.0f;
            const bool h = c0 + (uint32_t)sub < T.n && tri_test(S.tri4, (int)(T.base + c0 + (uint32_t)sub), T.o, T.d, t);
            const unsigned hm = oct_bits(__ballot(h));
            // triangle order, strict '<' (leaf_test)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float tj = __shfl(t, g0 + j);
                if (((hm >> j) & 1u) && (tj < T.best_t || T.best_t == -1)) {
                    T.best_t = tj;
                    T.best_k = (int)(T.base + c0 + (uint32_t)j);
                }
            }
        }
        T.steps += (int)T.n;
        T.lmask = ~0u;  // a leaf was visited: every stack level sees it
        octc_pop(S, T, w, spr, spk);
        return;
    }
    const OctProbe p = oct_children(S, T, sub);
    if (st && sub == 0) st->c[RT_STAT_VOL] += T.n;
    T.steps += (int)T.n;
    const unsigned hm = oct_bits(__ballot(p.h));
    if (hm) {
        // the hits in child order (travc_step's hk / hi, and its running tie test)
        float hk[8];
        uint32_t hi[8];
        int m = 0;
        bool tie = false;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float tj = __shfl(p.t, g0 + j);
            if ((hm >> j) & 1u) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    tie |= (i < m) && hk[i] == tj;
                    if (i == m) {
                        hk[i] = tj;
                        hi[i] = T.base + (uint32_t)j;
                    }
                }
                m++;
            }
        }
        while (T.sp + m - T.lo > OctRing::CAP) {  // make room: spill the window's bottom
            spr[T.lo] = w.rec(T.lo);
            spk[T.lo] = w.key(T.lo);
            T.lo++;
        }
        if (!tie) {
            // distinct keys: pop order is ascending t_near; rank r goes to slot sp+m-1-r
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (i < m) {
                    int r = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) r += (j < m) && hk[j] < hk[i];
                    w.set(T.sp + m - 1 - r, hi[i], hk[i]);
                }
            }
        } else {
            if (st && sub == 0) st->c[RT_STAT_HEAP_SLOW]++;
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < m) stk_sift_up(w, T.sp, i, hk[i], hi[i]);
            for (int len = m; len > 1; len--) stk_pop_heap(w, T.sp, len);
        }
        w.set_rec(T.sp + m - 1, w.rec(T.sp + m - 1) | RT_ENT_FIRST);
        w.set_rec(T.sp, w.rec(T.sp) | RT_ENT_LAST);
        // each entry's node link, from the lane that loaded its record
        for (int i = 0; i < m; i++) {
            const int s = T.sp + i;
            const uint32_t c = (w.rec(s) & RT_ENT_MASK) - T.base;
            const uint32_t lr = __shfl(p.ref, g0 + (int)(c & 7u)), lc = __shfl(p.cnt, g0 + (int)(c & 7u));
            w.lr[s & OctRing::MASK] = lr;
            w.lc[s & OctRing::MASK] = c < T.n ? lc : RT_OCT_NOLINK;
        }
        T.sp += m;
        T.groups++;
    }
    octc_pop(S, T, w, spr, spk);
}

__device__ __forceinline__ bool octc_parkable(const TravG& T) { return T.mode != TM_DONE && T.lo == 0 && T.sp <= RT_PARK_STACK; }

// travc_park's record (the octet's leader writes it).
__device__ __forceinline__ void octc_park(const TravG& T, const OctRing& w, uint32_t target, ParkC* P, int sub)
{
    if (sub != 0) return;
    P->o[0] = T.o.x, P->o[1] = T.o.y, P->o[2] = T.o.z;
    P->d[0] = T.d.x, P->d[1] = T.d.y, P->d[2] = T.d.z;
    P->best_t = T.best_t;
    P->best_k = T.best_k;
    P->sp = T.sp;
    P->groups = T.groups;
    P->mode = T.mode;
    P->lmask = T.lmask;
    P->base = T.base;
    P->n = T.n;
    P->target = target;
    P->pad = 0;
    for (int i = 0; i < RT_PARK_STACK; i++) {
        P->r[i] = i < T.sp ? w.rec(i) : 0u;
        P->k[i] = i < T.sp ? w.key(i) : 0.0f;
    }
}

__device__ __forceinline__ uint32_t octc_resume(const RtSceneView& S, const ParkC* P, TravG& T, OctRing& w, int sub)
{
    T.o = v3(P->o[0], P->o[1], P->o[2]);
    T.d = v3(P->d[0], P->d[1], P->d[2]);
    ray_setup(T.o, T.d, T.K);
    T.best_t = P->best_t;
    T.best_k = P->best_k;
    T.sp = P->sp;
    T.lo = 0;
    T.groups = P->groups;
    T.lmask = P->lmask;
    T.mode = P->mode;
    T.base = P->base;
    T.n = P->n;
    T.steps = 0;
    T.hit = false;
    for (int i = sub; i < T.sp; i += 8) {  // lane j: entries j, j + 8
        const uint32_t r = P->r[i];
        const uint2_ link = load_link(S.nodes, r & RT_ENT_MASK);
        w.set(i, r, P->k[i]);
        w.lr[i] = link.x;
        w.lc[i] = link.y;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return P->target;
}

// ------------------------------------------------------------------ occlusion
// trace_any's reachable set (trava_step's order: children pushed in reverse, child 0
// popped first); stops at the first hit.
__device__ __forceinline__ void octa_pop(const RtSceneView& S, TravG& T, const OctRing& w, const uint32_t* spr)
{
    if (T.sp == 0) {
        T.mode = TM_DONE;
        return;
    }
    const int i = --T.sp;
    const bool inwin = i >= T.lo;
    const uint32_t er = inwin ? w.rec(i) : spr[i];
    if (T.sp < T.lo) T.lo = T.sp;
    uint32_t ref, cnt;
    oct_link(S, w, i, inwin, er, ref, cnt);
    octg_enter(T, ref, cnt);
}

__device__ __forceinline__ void octa_node(const RtSceneView& S, TravG& T, OctRing& w, uint32_t* spr, int sub,
                                          Stats* st)
{
    const int g0 = oct_lane0();
    if (T.mode == TM_LEAF) {
        for (uint32_t c0 = 0; c0 < T.n; c0 += 8) {
            float t;
            const bool h = c0 + (uint32_t)sub < T.n && tri_test(S.tri4, (int)(T.base + c0 + (uint32_t)sub), T.o, T.d, t);
            const unsigned hm = oct_bits(__ballot(h));
            if (st && sub == 0) st->c[RT_STAT_ANY_TRI] += hm ? __ffs(hm) : min(8u, T.n - c0);
            if (hm) {
                T.hit = true;
                T.mode = TM_DONE;
                return;
            }
        }
        if (st && sub == 0) st->c[RT_STAT_ANY_LEAF]++;
        T.steps += (int)T.n;
        octa_pop(S, T, w, spr);
        return;
    }
    const OctProbe p = oct_children(S, T, sub);
    if (st && sub == 0) st->c[RT_STAT_ANY_VOL] += T.n;
    T.steps += (int)T.n;
    const unsigned hm = oct_bits(__ballot(p.h));
    // children in reverse, so that child 0 is popped first
    for (int c = (int)T.n - 1; c >= 0; c--) {
        if (!((hm >> c) & 1u)) continue;
        if (T.sp - T.lo == OctRing::CAP) {
            spr[T.lo] = w.rec(T.lo);
            T.lo++;
        }
        w.set_rec(T.sp, T.base + (uint32_t)c);
        w.lr[T.sp & OctRing::MASK] = __shfl(p.ref, g0 + c);
        w.lc[T.sp & OctRing::MASK] = __shfl(p.cnt, g0 + c);
        T.sp++;
    }
    octa_pop(S, T, w, spr);
}

__device__ __forceinline__ bool octa_parkable(const TravG& T) { return T.mode != TM_DONE && T.lo == 0 && T.sp <= RT_PARK_STACK; }

__device__ __forceinline__ void octa_park(const TravG& T, const OctRing& w, uint32_t target, ParkA* P, int sub)
{
    if (sub != 0) return;
    P->o[0] = T.o.x, P->o[1] = T.o.y, P->o[2] = T.o.z;
    P->d[0] = T.d.x, P->d[1] = T.d.y, P->d[2] = T.d.z;
    P->sp = T.sp;
    P->mode = T.mode;
    P->base = T.base;
    P->n = T.n;
    P->target = target;
    P->pad = 0;
    for (int i = 0; i < RT_PARK_STACK; i++) P->r[i] = i < T.sp ? w.rec(i) : 0u;
}

__device__ __forceinline__ uint32_t octa_resume(const RtSceneView& S, const ParkA* P, TravG& T, OctRing& w, int sub)
{
    T.o = v3(P->o[0], P->o[1], P->o[2]);
    T.d = v3(P->d[0], P->d[1], P->d[2]);
    ray_setup(T.o, T.d, T.K);
    T.sp = P->sp;
    T.lo = 0;
    T.mode = P->mode;
    T.base = P->base;
    T.n = P->n;
    T.steps = 0;
    T.hit = false;
    for (int i = sub; i < T.sp; i += 8) {
        const uint32_t r = P->r[i];
        const uint2_ link = load_link(S.nodes, r & RT_ENT_MASK);
        w.set_rec(i, r);
        w.lr[i] = link.x;
        w.lc[i] = link.y;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return P->target;
}

}  // namespace rtk
