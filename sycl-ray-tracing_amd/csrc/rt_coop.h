// rt_coop.h — one search-BVH query walked by all four rows of a wave (gfx950 only).
//
// Where a wave has a single walk left — a tail round whose other queries are
// answered (k_tail), or the last walk of a k_trace wave whose stream is out — the
// round or the launch waits for that walk alone while 48 of its 64 lanes idle.
// Here the four rows of the wave walk it together over the 16-wide BVH (rt_row.h):
// each row holds an item of its own (a node it descends into, or up to four
// leaves), and the items left over are on one shared stack that an idle row pops
// from. A trip of the wave tests up to four 16-wide nodes (64 boxes) or sixteen
// leaves in one memory round trip.
//
// The answer is rt_fast.h's, as for the row walk: a stack entry is dropped only
// when its entry distance is outside the current window, the window only shrinks,
// so every box that holds a hit inside the final window is entered. Boxes a
// one-row walk would have dropped later may be entered too; their hits lie
// outside the final window, where they change neither the closest hit (t, its
// lowest-prim triangle) nor the tie flag, and the second-hit bound the
// verification reads is clamped to the window (quad_closest_answer). The hit
// record is folded in as a set (closest, second, tie, lowest prim at the
// closest), so the rows' order of merging does not matter. Occlusion walks need
// no order at all.
//
// Contract: all 64 lanes of the wave call coop_walk together with the same q (its
// fields wave-uniform); the stack is one row's (STK), shared by the rows.
#pragma once

#include "rt_row.h"

namespace rtk {

#define RT_COOP_IDLE 0x7fffffff  // a row without an item

// The wave walks q to its end. 1: over (ANY: q.h.k = 1 occluded / 0 not; else the
// closest-hit record in q.h, to quad_closest_answer); -1: the shared stack overflowed.
// calls: trips taken (added to q.calls by the caller if it wants them).
template <bool ANY, class STK>
__device__ int coop_walk(const RtSceneView& S, QState& q, STK& stk, Stats* st, int& trips)
{
    const int lane = (int)__lane_id(), row = lane >> 4, sub = lane & 15;
    FastHit& h = q.h;
    int cur = row == 0 ? q.cur : RT_COOP_IDLE;  // this row's item (row-uniform)
    trips = 0;
    for (;;) {
        // ---- every row without an item takes one from the stack (row order); a row at a
        // leaf also takes up to three leaves right below it (row_visit's leaf batch)
        const float tw = ANY ? __builtin_inff() : h.t + h.t * RT_T2_WINDOW;
        int l0 = 0, l1 = 0, l2 = 0, l3 = 0, nl = 0;
        bool any_item = false;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int rc = __builtin_amdgcn_readlane(cur, 16 * r);
            if (rc == RT_COOP_IDLE) {
                while (q.sp > 0) {
                    --q.sp;
                    if (ANY || stk.key(q.sp) <= tw) {
                        rc = (int)stk.rec(q.sp);
                        break;
                    }
                }
            }
            int b1 = 0, b2 = 0, b3 = 0, bn = 0;
            if (rc != RT_COOP_IDLE && rc < 0) {
                bn = 1;
#pragma unroll
                for (int g = 1; g < 4; g++) {
                    if (bn != g || q.sp == 0) break;
                    const int t = (int)stk.rec(q.sp - 1);
                    if (t >= 0 || (!ANY && !(stk.key(q.sp - 1) <= tw))) break;  // an inner node, or closed by the window
                    q.sp--;
                    bn++;
                    (g == 1 ? b1 : g == 2 ? b2 : b3) = t;
                }
            }
            any_item = any_item || rc != RT_COOP_IDLE;
            if (row == r) {
                cur = rc;
                l0 = rc, l1 = b1, l2 = b2, l3 = b3, nl = bn;
            }
        }
        if (!any_item) return 1;  // (ANY: h.k = 0, no occluder; else q.h is the answer)
        trips++;
        const bool inner = cur != RT_COOP_IDLE && cur >= 0;
        // ---- inner rows: the 16 children of the row's node (row_visit's inner trip)
        bool ok = false;
        float tn = __builtin_inff();
        int item = 0, nb = 0;
        if (inner) {
            const float4_* p = (const float4_*)(S.bvh16 + (size_t)cur * RT_BVH16_W + sub);
            const float4_ a = p[0], b = p[1];
            rt_pin(a);
            rt_pin(b);
            const int ref = (int)rt_asuint(b.z), cnt = (int)rt_asuint(b.w);
            const float mn[3] = {a.x, a.y, a.z}, mx[3] = {a.w, b.x, b.y};
            ok = cnt >= 0 && box_hit(mn, mx, q.rb, tw, tn) && (ANY || tn <= tw);
            item = cnt > 0 ? leaf_item(ref, cnt) : ref;
            nb = cnt >= 0 ? 1 : 0;
        }
        const unsigned m = row_bits(__ballot(ok));
        const int nv = __popc(m);
        if (st) {
            const int rb = __popc(row_bits(__ballot(nb != 0)));
            if (inner && sub == 0) st->c[ANY ? RT_STAT_ANY_VOL : RT_STAT_VOL] += rb;
        }
        bool push_me;
        int slot_in_row;  // (push_me) position in the row's block of pushes, 0 = bottom
        int first;
        if (ANY) {
            // hit i of the row (lane order) is pushed at position i - 1; hit 0 is next
            const int pre = __popc(m & ((1u << sub) - 1u));
            push_me = ok && pre > 0;
            slot_in_row = pre - 1;
            first = ok && pre == 0;
        } else {
            // far hits pushed, nearest of them on top; a hit's key is finite and below a miss's
            const float key = ok ? __builtin_fminf(tn, 3.0e38f) : __builtin_inff();
            const int rank = row_rank(key, sub);
            push_me = ok && rank > 0;
            slot_in_row = nv - 1 - rank;
            first = ok && rank == 0;
            tn = key;
        }
        const int nxt = row_or(first ? item : 0);
        // ---- leaf rows: up to four leaves, four lanes each (row_visit's leaf trip)
        const int g = sub >> 2;
        const int mine_leaf = g == 0 ? l0 : g == 1 ? l1 : g == 2 ? l2 : l3;
        int k = -1, leaf = -1, prim = 0x7fffffff;
        float tv = __builtin_inff();
        if (g < nl) tv = quad_tri(S, mine_leaf, sub & 3, q.o, q.d, k, leaf, prim);
        if (st && nl > 0 && sub == 0) {
            int nt = ((~l0) & 3) + 1;
            if (nl > 1) nt += ((~l1) & 3) + 1;
            if (nl > 2) nt += ((~l2) & 3) + 1;
            if (nl > 3) nt += ((~l3) & 3) + 1;
            st->c[ANY ? RT_STAT_ANY_TRI : RT_STAT_TRI] += nt;
        }
        // ---- pushes to the shared stack: row blocks in row order
        const unsigned long long bp = __ballot(push_me);
        int total = 0, below = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c = __popcll((bp >> (16 * r)) & 0xFFFFull);
            if (r < row) below += c;
            total += c;
        }
        if (q.sp + total > STK::CAP) return -1;
        if (push_me) {
            if (ANY)
                stk.set_rec(q.sp + below + slot_in_row, (uint32_t)item);
            else
                stk.set(q.sp + below + slot_in_row, (uint32_t)item, tn);
        }
        q.sp += total;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (other rows pop these entries)
        __builtin_amdgcn_wave_barrier();
        if (inner) cur = nv > 0 ? nxt : RT_COOP_IDLE;
        else cur = RT_COOP_IDLE;  // (a leaf row, or an idle one)
        // ---- the leaf rows' results, folded into the walk's record
        if (ANY) {
            bool found = false;
            unsigned hm = row_bits(__ballot(tv < __builtin_inff()));
            if (S.brute) {
                found = hm != 0;
            } else {
                while (hm) {  // row-uniform: each hit's octree chain, checked by every quad of the row
                    const int j = __ffs(hm) - 1;
                    hm &= hm - 1u;
                    const int lj = __shfl(leaf, (lane & 48) + j);
                    if (quad_chain_ok(S, q.o, q.d, lj, false, 0.0f, sub & 3, sub == 0 ? st : nullptr)) {
                        found = true;
                        break;
                    }
                }
            }
            if (__ballot(found)) {
                h.k = 1;
                return 1;
            }
        } else {
            float m1 = tv, m2 = __builtin_inff();
            row_merge2<RT_QX1>(m1, m2);
            row_merge2<RT_QX2>(m1, m2);
            row_merge2<RT_DPP_ROW_HALF_MIRROR>(m1, m2);
            row_merge2<RT_DPP_ROW_MIRROR>(m1, m2);
            const int pm = row_min(tv == m1 ? prim : 0x7fffffff);
            const bool mine = tv == m1 && prim == pm;
            const int kk = row_or(mine ? k : 0), lf = row_or(mine ? leaf : 0);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m1), 16 * r));
                if (!(r1 < __builtin_inff())) continue;  // (no hit in row r's leaves)
                const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m2), 16 * r));
                const int rp = __builtin_amdgcn_readlane(pm, 16 * r);
                const int rk = __builtin_amdgcn_readlane(kk, 16 * r), rl = __builtin_amdgcn_readlane(lf, 16 * r);
                if (r1 < h.t) {
                    h.t2 = __builtin_fminf(h.t, r2);
                    h.t = r1;
                    h.k = rk;
                    h.leaf = rl;
                    h.prim = rp;
                    h.tie = r2 == r1;
                } else if (r1 == h.t) {
                    h.tie = true;
                    h.t2 = r1;
                    if (rp < h.prim) {
                        h.k = rk;
                        h.leaf = rl;
                        h.prim = rp;
                    }
                } else {
                    h.t2 = __builtin_fminf(h.t2, r1);
                }
            }
        }
    }
}

}  // namespace rtk
