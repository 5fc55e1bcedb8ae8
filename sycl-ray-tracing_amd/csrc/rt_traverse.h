// rt_traverse.h — resumable, step-at-a-time forms of the octree walks
// (trace_closest / trace_any in rt_trace.h), run by the gfx950 trace kernels
// and by the hostsim build.
//
// Why: the work per ray of the reference's traversal has an extreme tail
// (dragon stand-in: 85 % of closest-hit rays need < 16 child-volume tests,
// 0.1 % need 8k-28k — rays grazing the tessellated surface, which must test
// every volume they pierce before a hit allows the early exit). A lock-step
// "one ray per lane until done" loop makes every wave, and every wavefront
// iteration, wait for its slowest ray. Here a ray advances by one unit of
// work per call (one child-volume test or one triangle test, plus the stack
// pops that follow it), so a lane whose ray finishes takes the next ray at
// once, and a ray that has used its step budget is parked (its state saved to
// memory) and resumed by the next launch while its path waits.
//
// The order of node visits, the early-exit rule and the tie order are those
// of trace_closest() exactly (see trace_closest_short() for the two changes
// of representation: per-level leaf mask, in-place heap); only the control
// flow is cut into steps. The stack is a window of its CAP top entries (LDS
// on the device) over a per-lane spill area, so there is no depth limit.
#pragma once

#include "rt_trace.h"

namespace rtk {

enum TravMode : int { TM_EXPAND = 0, TM_LEAF = 1, TM_DONE = 2 };

// A stack whose top CAP entries live in the fast window FAST (slot i & (CAP-1));
// entries below `lo` live only in the spill area.
template <class FAST>
struct SpillStack {
    FAST f;
    uint32_t* spill_r;  // RT_STACK_CAP entries for this lane
    float* spill_k;     // (unused by the occlusion walk)
    static constexpr int CAP = FAST::CAP;
    static constexpr int MASK = CAP - 1;
    static_assert(CAP >= 8 && (CAP & MASK) == 0, "the window is a ring: CAP must be a power of two >= 8");
    RT_HD uint32_t rec(int i, int lo) const { return i >= lo ? f.rec(i & MASK) : spill_r[i]; }
    RT_HD float key(int i, int lo) const { return i >= lo ? f.key(i & MASK) : spill_k[i]; }
};

// Index-shifting view of the window for the heap routines (all of the group
// being pushed, [sp, sp+m), is inside the window by construction).
template <class FAST>
struct WinView {
    FAST& f;
    int off;
    RT_HD uint32_t rec(int i) const { return f.rec((off + i) & (FAST::CAP - 1)); }
    RT_HD float key(int i) const { return f.key((off + i) & (FAST::CAP - 1)); }
    RT_HD void set(int i, uint32_t r, float k) { f.set((off + i) & (FAST::CAP - 1), r, k); }
    RT_HD void set_rec(int i, uint32_t r) { f.set_rec((off + i) & (FAST::CAP - 1), r); }
};

// ------------------------------------------------------------ closest hit
struct TravC {
    V3 o, d;
    RayK K;
    float best_t;
    int best_k;
    int sp, lo, groups;
    uint32_t lmask;
    int mode;
    uint32_t base, n, c;  // EXPAND: children [base, base+n); LEAF: triangles [base, base+n); next c
    int m;
    bool tie;
    float hk[8];
    uint32_t hi[8];
    int steps;
};

RT_HD void travc_enter(TravC& T, uint32_t ref, uint32_t cnt)
{
    T.base = ref;
    T.c = 0;
    if (cnt & RT_LEAF_BIT) {
        T.n = cnt & ~RT_LEAF_BIT;
        T.mode = TM_LEAF;
    } else {
        T.n = cnt;
        T.m = 0;
        T.tie = false;
        T.mode = TM_EXPAND;
    }
}

// Pops to the next node to work on (trace_closest_short's pop loop).
template <class FAST>
RT_HD void travc_pop(const RtSceneView& S, TravC& T, SpillStack<FAST>& stk)
{
    for (;;) {
        if (T.sp == 0) {
            T.mode = TM_DONE;
            return;
        }
        --T.sp;
        const uint32_t er = stk.rec(T.sp, T.lo);  // (read before the window shrinks below it)
        const float ek = (er & RT_ENT_FIRST) ? 0.0f : stk.key(T.sp, T.lo);
        if (T.sp < T.lo) T.lo = T.sp;
        const uint32_t lvl = (uint32_t)(T.groups - 1);
        if (!(er & RT_ENT_FIRST)) {
            const bool prev_true = T.best_t > 0.0f && ((T.lmask >> lvl) & 1u);
            const float closest = rt_min(100000000.0f, T.best_t);
            if (prev_true && closest < ek) {
                // early exit of the parent: drop this entry and its remaining siblings
                if (!(er & RT_ENT_LAST))
                    while (!(stk.rec(--T.sp, T.lo) & RT_ENT_LAST)) {
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
        const uint2_ link = load_link(S.nodes, er & RT_ENT_MASK);
        travc_enter(T, link.x, link.y);
        return;
    }
}

// Starts a query (ray constants, root volume). False: already finished.
RT_HD bool travc_begin(const RtSceneView& S, TravC& T, V3 o, V3 d, Stats* st)
{
    T.o = o;
    T.d = d;
    T.best_t = -1.0f;
    T.best_k = -1;
    T.sp = T.lo = T.groups = 0;
    T.lmask = 0;
    T.steps = 0;
    T.mode = TM_DONE;
    if (st) st->c[RT_STAT_RAYS]++;
    if (S.brute) {  // USE_BVH 0: the loop answers at once
        brute_closest(S, o, d, T.best_t, T.best_k);
        return false;
    }
    if (!ray_setup(o, d, T.K)) return false;
    float tn;
    if (st) st->c[RT_STAT_VOL]++;
    const NodeR root = load_node(S.nodes, 0);
    if (!slab_test(root, T.K, tn)) return false;
    travc_enter(T, root.ref, root.cnt);
    return true;
}

// One unit of work: a triangle test (LEAF) or a child-volume test (EXPAND),
// then the push / pops that complete the node. True while work remains.
template <class FAST>
RT_HD bool travc_step(const RtSceneView& S, TravC& T, SpillStack<FAST>& stk, Stats* st)
{
    T.steps++;
    if (T.mode == TM_LEAF) {
        const int k = (int)(T.base + T.c);
        float t;
        if (tri_test(S.tri4, k, T.o, T.d, t))
            if (t < T.best_t || T.best_t == -1) {
                T.best_t = t;
                T.best_k = k;
            }
        if (st) st->c[RT_STAT_TRI]++;
        if (++T.c < T.n) return true;
        if (st) st->c[RT_STAT_LEAF]++;
        T.lmask = ~0u;  // a leaf was visited: every stack level sees it
        travc_pop(S, T, stk);
        return T.mode != TM_DONE;
    }
    {
        const uint32_t rec = T.base + T.c;
        const NodeR ch = load_node(S.nodes, rec);
        float t;
        if (st) st->c[RT_STAT_VOL]++;
        if (slab_test(ch, T.K, t)) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                T.tie |= (j < T.m) && T.hk[j] == t;
                if (j == T.m) {
                    T.hk[j] = t;
                    T.hi[j] = rec;
                }
            }
            T.m++;
        }
    }
    if (++T.c < T.n) return true;
    const int m = T.m;
    if (m > 0) {
        while (T.sp + m - T.lo > SpillStack<FAST>::CAP) {  // make room: spill the window's bottom
            stk.spill_r[T.lo] = stk.f.rec(T.lo & SpillStack<FAST>::MASK);
            stk.spill_k[T.lo] = stk.f.key(T.lo & SpillStack<FAST>::MASK);
            T.lo++;
        }
        WinView<FAST> w{stk.f, T.sp};
        if (!T.tie) {
            // distinct keys: pop order is ascending t_near; rank r goes to slot m-1-r
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (i < m) {
                    int r = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) r += (j < m) && T.hk[j] < T.hk[i];
                    w.set(m - 1 - r, T.hi[i], T.hk[i]);
                }
            }
        } else {
            if (st) st->c[RT_STAT_HEAP_SLOW]++;
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < m) stk_sift_up(w, 0, i, T.hk[i], T.hi[i]);
            for (int len = m; len > 1; len--) stk_pop_heap(w, 0, len);
        }
        w.set_rec(m - 1, w.rec(m - 1) | RT_ENT_FIRST);
        w.set_rec(0, w.rec(0) | RT_ENT_LAST);
        T.sp += m;
        T.groups++;
    }
    travc_pop(S, T, stk);
    return T.mode != TM_DONE;
}

// Parked closest-hit query: taken only at a node boundary (c == 0) with
// nothing spilled, so the window holds the whole stack.
#define RT_PARK_STACK 16
struct ParkC {
    float o[3], d[3];
    float best_t;
    int32_t best_k;
    int32_t sp, groups, mode;
    uint32_t lmask, base, n, target, pad;
    uint32_t r[RT_PARK_STACK];
    float k[RT_PARK_STACK];
};

RT_HD bool travc_parkable(const TravC& T) { return T.mode != TM_DONE && T.c == 0 && T.lo == 0 && T.sp <= RT_PARK_STACK; }

template <class FAST>
RT_HD void travc_park(const TravC& T, const SpillStack<FAST>& stk, uint32_t target, ParkC* P)
{
    ParkC q;
    q.o[0] = T.o.x, q.o[1] = T.o.y, q.o[2] = T.o.z;
    q.d[0] = T.d.x, q.d[1] = T.d.y, q.d[2] = T.d.z;
    q.best_t = T.best_t;
    q.best_k = T.best_k;
    q.sp = T.sp;
    q.groups = T.groups;
    q.mode = T.mode;
    q.lmask = T.lmask;
    q.base = T.base;
    q.n = T.n;
    q.target = target;
    q.pad = 0;
    for (int i = 0; i < RT_PARK_STACK; i++) {
        q.r[i] = i < T.sp ? stk.f.rec(i & SpillStack<FAST>::MASK) : 0u;
        q.k[i] = i < T.sp ? stk.f.key(i & SpillStack<FAST>::MASK) : 0.0f;
    }
    *P = q;
}

template <class FAST>
RT_HD uint32_t travc_resume(const ParkC* P, TravC& T, SpillStack<FAST>& stk)
{
    const ParkC q = *P;
    T.o = v3(q.o[0], q.o[1], q.o[2]);
    T.d = v3(q.d[0], q.d[1], q.d[2]);
    ray_setup(T.o, T.d, T.K);
    T.best_t = q.best_t;
    T.best_k = q.best_k;
    T.sp = q.sp;
    T.lo = 0;
    T.groups = q.groups;
    T.lmask = q.lmask;
    T.mode = q.mode;
    T.base = q.base;
    T.n = q.n;
    T.c = 0;
    T.m = 0;
    T.tie = false;
    T.steps = 0;
    for (int i = 0; i < q.sp; i++) stk.f.set(i & SpillStack<FAST>::MASK, q.r[i], q.k[i]);
    return q.target;
}

// -------------------------------------------------------------- occlusion
// trace_any() cut into steps (same reachable set; stops at the first hit).
struct TravA {
    V3 o, d;
    RayK K;
    int sp, lo, mode;
    uint32_t base, n, c;
    int steps;
    bool hit;
};

RT_HD void trava_enter(TravA& T, uint32_t ref, uint32_t cnt)
{
    T.base = ref;
    T.c = 0;
    T.n = cnt & ~RT_LEAF_BIT;
    T.mode = (cnt & RT_LEAF_BIT) ? TM_LEAF : TM_EXPAND;
}

template <class FAST>
RT_HD void trava_pop(const RtSceneView& S, TravA& T, SpillStack<FAST>& stk)
{
    if (T.sp == 0) {
        T.mode = TM_DONE;
        return;
    }
    --T.sp;
    const uint32_t rec = stk.rec(T.sp, T.lo);
    if (T.sp < T.lo) T.lo = T.sp;
    const uint2_ link = load_link(S.nodes, rec);
    trava_enter(T, link.x, link.y);
}

RT_HD bool trava_begin(const RtSceneView& S, TravA& T, V3 o, V3 d, Stats* st)
{
    T.o = o;
    T.d = d;
    T.sp = T.lo = 0;
    T.steps = 0;
    T.hit = false;
    T.mode = TM_DONE;
    if (st) st->c[RT_STAT_ANY_RAYS]++;
    if (S.brute) {  // USE_BVH 0
        T.hit = brute_any(S, o, d);
        return false;
    }
    if (!ray_setup(o, d, T.K)) return false;
    float tn;
    if (st) st->c[RT_STAT_ANY_VOL]++;
    const NodeR root = load_node(S.nodes, 0);
    if (!slab_test(root, T.K, tn)) return false;
    trava_enter(T, root.ref, root.cnt);
    return true;
}

template <class FAST>
RT_HD bool trava_step(const RtSceneView& S, TravA& T, SpillStack<FAST>& stk, Stats* st)
{
    T.steps++;
    if (T.mode == TM_LEAF) {
        float t;
        if (st) st->c[RT_STAT_ANY_TRI]++;
        if (tri_test(S.tri4, (int)(T.base + T.c), T.o, T.d, t)) {
            T.hit = true;
            T.mode = TM_DONE;
            return false;
        }
        if (++T.c < T.n) return true;
        if (st) st->c[RT_STAT_ANY_LEAF]++;
        trava_pop(S, T, stk);
        return T.mode != TM_DONE;
    }
    {
        // children in reverse, so that child 0 is popped first (trace_any's order)
        const uint32_t rec = T.base + (T.n - 1 - T.c);
        float tn;
        if (st) st->c[RT_STAT_ANY_VOL]++;
        if (slab_test(load_node(S.nodes, rec), T.K, tn)) {
            if (T.sp - T.lo == SpillStack<FAST>::CAP) {
                stk.spill_r[T.lo] = stk.f.rec(T.lo & SpillStack<FAST>::MASK);
                T.lo++;
            }
            stk.f.set_rec(T.sp & SpillStack<FAST>::MASK, rec);
            T.sp++;
        }
    }
    if (++T.c < T.n) return true;
    trava_pop(S, T, stk);
    return T.mode != TM_DONE;
}

struct ParkA {
    float o[3], d[3];
    int32_t sp, mode;
    uint32_t base, n, target, pad;
    uint32_t r[RT_PARK_STACK];
};

RT_HD bool trava_parkable(const TravA& T) { return T.mode != TM_DONE && T.c == 0 && T.lo == 0 && T.sp <= RT_PARK_STACK; }

template <class FAST>
RT_HD void trava_park(const TravA& T, const SpillStack<FAST>& stk, uint32_t target, ParkA* P)
{
    ParkA q;
    q.o[0] = T.o.x, q.o[1] = T.o.y, q.o[2] = T.o.z;
    q.d[0] = T.d.x, q.d[1] = T.d.y, q.d[2] = T.d.z;
    q.sp = T.sp;
    q.mode = T.mode;
    q.base = T.base;
    q.n = T.n;
    q.target = target;
    q.pad = 0;
    for (int i = 0; i < RT_PARK_STACK; i++) q.r[i] = i < T.sp ? stk.f.rec(i & SpillStack<FAST>::MASK) : 0u;
    *P = q;
}

template <class FAST>
RT_HD uint32_t trava_resume(const ParkA* P, TravA& T, SpillStack<FAST>& stk)
{
    const ParkA q = *P;
    T.o = v3(q.o[0], q.o[1], q.o[2]);
    T.d = v3(q.d[0], q.d[1], q.d[2]);
    ray_setup(T.o, T.d, T.K);
    T.sp = q.sp;
    T.lo = 0;
    T.mode = q.mode;
    T.base = q.base;
    T.n = q.n;
    T.c = 0;
    T.steps = 0;
    T.hit = false;
    for (int i = 0; i < q.sp; i++) stk.f.set_rec(i & SpillStack<FAST>::MASK, q.r[i]);
    return q.target;
}

}  // namespace rtk
