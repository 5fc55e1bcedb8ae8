// rt_row.h — search-BVH queries walked by a row of 16 lanes over the 16-wide
// form of the search BVH (gfx950 only).
//
// Where the walks are latency-bound — a sparse k_trace launch ends with its
// longest walk, and a k_tail round waits for the slowest query of its wave —
// a query's latency is its number of dependent memory round trips. A quad
// (rt_quad.h) takes one trip per 4-wide node; a row of 16 lanes takes one trip
// per 16-wide node (rt_device.h Bvh16: two 4-wide levels), so a walk descends
// in half the trips:
//  * inner node: lane j loads record j of the node (32 B, the row reads 512
//    contiguous bytes) and tests its box; the hits are ranked by entry distance
//    (15 DPP row rotations: each lane counts the (key, lane) pairs below its
//    own), the nearest is next and lane j pushes its own entry;
//  * leaves: the leaf and up to three more leaves right below it on the stack
//    (what a one-leaf walk would pop next) are tested together, four lanes
//    per leaf, one triangle per lane; the row reduces (closest, second, tie)
//    with DPP.
// The answer is rt_fast.h's (every box holding a hit in the final window is
// entered; the window only shrinks), so a query falls back to the exact octree
// walk in exactly the cases the quad walk does. Occlusion walks (ANY) need no
// order: the first hit is next, the others are pushed.
//
// Contract: the 16 lanes of a row call these functions together, in
// row-uniform control flow (DPP reads the other lanes of the row).
#pragma once

#include "rt_quad.h"

namespace rtk {

// Oriented slabs (rt_fast.h slab_ok) in the row walks: each lane also loads its record's
// 16-B slab in the same round trip.
#ifndef RT_SLAB_ROW
#define RT_SLAB_ROW RT_SLABS
#endif

#define RT_DPP_ROW_MIRROR 0x140       // lane i <- lane 15 - i of its row
#define RT_DPP_ROW_HALF_MIRROR 0x141  // lane i <- lane 7 - i of its half row
#define RT_DPP_ROW_ROR(k) (0x120 + (k))  // lane i <- lane (i - k) mod 16 of its row

template <int CTRL>
__device__ __forceinline__ int rdpp(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float rdppf(float v)
{
    return __int_as_float(rdpp<CTRL>(__float_as_int(v)));
}
// Over the 16 lanes of the row, every lane gets the result (quads, then half rows, then rows).
__device__ __forceinline__ int row_or(int v)
{
    v |= qdpp<RT_QX1>(v);
    v |= qdpp<RT_QX2>(v);
    v |= rdpp<RT_DPP_ROW_HALF_MIRROR>(v);
    return v | rdpp<RT_DPP_ROW_MIRROR>(v);
}
__device__ __forceinline__ int row_min(int v)
{
    v = min(v, qdpp<RT_QX1>(v));
    v = min(v, qdpp<RT_QX2>(v));
    v = min(v, rdpp<RT_DPP_ROW_HALF_MIRROR>(v));
    return min(v, rdpp<RT_DPP_ROW_MIRROR>(v));
}
// minimum over the row's 16 lanes (every lane gets it)
__device__ __forceinline__ float row_minf(float v)
{
    v = __builtin_fminf(v, qdppf<RT_QX1>(v));
    v = __builtin_fminf(v, qdppf<RT_QX2>(v));
    v = __builtin_fminf(v, rdppf<RT_DPP_ROW_HALF_MIRROR>(v));
    return __builtin_fminf(v, rdppf<RT_DPP_ROW_MIRROR>(v));
}
// Rank of (key, lane) among the row's 16 pairs: a permutation of 0..15 (the lane
// each rotation reads from is taken from the rotation itself, not assumed).
template <int K>
__device__ __forceinline__ int row_rank_from(float key, int sub)
{
    const float o = rdppf<RT_DPP_ROW_ROR(K)>(key);
    const int os = rdpp<RT_DPP_ROW_ROR(K)>(sub);
    const int c = (o < key || (o == key && os < sub)) ? 1 : 0;
    if constexpr (K < 15)
        return c + row_rank_from<K + 1>(key, sub);
    else
        return c;
}
__device__ __forceinline__ int row_rank(float key, int sub) { return row_rank_from<1>(key, sub); }

// This lane's bits of the row in a wave ballot.
__device__ __forceinline__ unsigned row_bits(unsigned long long b) { return (unsigned)(b >> (__lane_id() & 48)) & 0xFFFFu; }

// One trip (and up to DESC inner-node trips in a row before returning), the row form of
// quad_visit: 0 go on, 1 the walk is over (ANY: q.h.k = 1 occluded / 0 not; else the
// closest-hit record in q.h, to quad_closest_answer), -1 the bounded stack overflowed.
// sub = lane within the row (0..15); q.cur is a 16-wide node index or a leaf item.
template <bool ANY, int DESC, class RSTK>
__device__ __forceinline__ int row_visit(const RtSceneView& S, QState& q, RSTK& stk, int sub, Stats* st)
{
    FastHit& h = q.h;
#pragma unroll 1
    for (int dd = 0; dd < DESC && q.cur >= 0; dd++) {
        const float4_* p = (const float4_*)(S.bvh16 + (size_t)q.cur * RT_BVH16_W + sub);
        const float4_ a = p[0], b = p[1];
#if RT_SLAB_ROW
        const float4_ sl = S.bvh16s[(size_t)q.cur * RT_BVH16_W + sub];
        rt_pin(sl);
#endif
        rt_pin(a);
        rt_pin(b);
        const int ref = (int)rt_asuint(b.z), cnt = (int)rt_asuint(b.w);
        const float mn[3] = {a.x, a.y, a.z}, mx[3] = {a.w, b.x, b.y};
        const float tmax = ANY ? __builtin_inff() : h.t + h.t * RT_T2_WINDOW;
        float tn, tf;
#if RT_SLAB_ROW
        const bool ok = cnt >= 0 && box_hit2(mn, mx, q.rb, tmax, tn, tf) && (ANY || tn <= tmax) && slab_ok(sl, q.o, q.d, tn, tf);
#else
        const bool ok = cnt >= 0 && box_hit2(mn, mx, q.rb, tmax, tn, tf) && (ANY || tn <= tmax);
#endif
        const int item = cnt > 0 ? leaf_item(ref, cnt) : ref;
        const unsigned m = row_bits(__ballot(ok));
        const int nv = __popc(m);
        if (st) {  // (st is row-uniform: the whole row takes the ballot)
            const int nb = __popc(row_bits(__ballot(cnt >= 0)));
            if (sub == 0) st->c[ANY ? RT_STAT_ANY_VOL : RT_STAT_VOL] += nb;
        }
        if (q.sp + nv - 1 > RSTK::CAP) return -1;
        int first;
        if (ANY) {
            // hit i of the row (lane order) goes to stack position sp + i - 1; hit 0 is next
            const int pre = __popc(m & ((1u << sub) - 1u));
            if (ok && pre > 0) stk.set_rec(q.sp + pre - 1, (uint32_t)item);
            first = ok && pre == 0;
        } else {
            // far hits on the stack, nearest of them on top (rank 1 at sp + nv - 2); a hit's
            // key is finite and below every miss's +inf, so the hits hold ranks 0 .. nv - 1
            const float key = ok ? __builtin_fminf(tn, 3.0e38f) : __builtin_inff();
            const int rank = row_rank(key, sub);
            if (ok && rank > 0) stk.set(q.sp + nv - 1 - rank, (uint32_t)item, key);
            first = ok && rank == 0;
        }
        if (nv > 0) {
            q.sp += nv - 1;
            q.cur = row_or(first ? item : 0);
            continue;
        }
        q.cur = 0x7ffffffe;  // no child hit: pop (below)
        break;
    }
    if (q.cur >= 0 && q.cur != 0x7ffffffe) return 0;  // (descended DESC times; still inner)
    if (q.cur < 0) {
        // this leaf and up to three leaves right below it on the stack: four lanes each
        int l0 = q.cur, l1 = 0, l2 = 0, l3 = 0, nl = 1;
        const float tw = h.t + h.t * RT_T2_WINDOW;
#pragma unroll
        for (int g = 1; g < 4; g++) {
            if (nl != g || q.sp == 0) break;
            const int t = (int)stk.rec(q.sp - 1);
#if RT_POP_PAIRED
            const float tk = ANY ? 0.0f : stk.key(q.sp - 1);  // (read with the item: one LDS round trip)
            if (!ANY) rt_pin(tk);
            if (t >= 0 || (!ANY && !(tk <= tw))) break;  // an inner node, or closed by the window
#else
            if (t >= 0 || (!ANY && !(stk.key(q.sp - 1) <= tw))) break;  // an inner node, or closed by the window
#endif
            q.sp--;
            nl++;
            (g == 1 ? l1 : g == 2 ? l2 : l3) = t;
        }
        if (st && sub == 0) {
            int nt = ((~l0) & 3) + 1;
            if (nl > 1) nt += ((~l1) & 3) + 1;
            if (nl > 2) nt += ((~l2) & 3) + 1;
            if (nl > 3) nt += ((~l3) & 3) + 1;
            st->c[ANY ? RT_STAT_ANY_TRI : RT_STAT_TRI] += nt;
        }
        const int g = sub >> 2;
        const int mine_leaf = g == 0 ? l0 : g == 1 ? l1 : g == 2 ? l2 : l3;
        int k = -1, leaf = -1, prim = 0x7fffffff;
        float tv = __builtin_inff();
        if (g < nl) tv = quad_tri<!ANY>(S, mine_leaf, sub & 3, q.o, q.d, k, leaf, prim);
        if (ANY) {
            unsigned hm = row_bits(__ballot(tv < __builtin_inff()));
            if (S.brute) {
                if (hm) {
                    h.k = 1;
                    return 1;
                }
            } else {
                while (hm) {  // row-uniform: each hit's octree chain, checked by every quad of the row
                    const int j = __ffs(hm) - 1;
                    hm &= hm - 1u;
                    const int lj = __shfl(leaf, (int)(__lane_id() & 48) + j);
                    if (quad_chain_ok(S, q.o, q.d, lj, false, 0.0f, sub & 3, sub == 0 ? st : nullptr)) {
                        h.k = 1;
                        return 1;
                    }
                }
            }
        } else {
            // rt_quad.h's leaf reduction over the row's sixteen hits (rt_fast.h fast_take)
            const float m1 = row_minf(tv);
            const float m2 = row_minf(tv > m1 ? tv : __builtin_inff());
            const int key = row_min(tv == m1 ? (S.brute ? prim : k) : 0x7fffffff);
            const bool mine = tv == m1 && (S.brute ? prim : k) == key;
            const int wk = row_or(mine ? k : 0), wl = row_or(mine ? leaf : 0), wp = row_or(mine ? prim : 0);
            const bool mixed = row_or(tv == m1 && m1 < __builtin_inff() && leaf != wl ? 1 : 0) != 0;
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

}  // namespace rtk
