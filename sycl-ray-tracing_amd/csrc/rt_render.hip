// rt_render.hip — gfx950 backend of librt_hip.so: device buffers, the
// wavefront render kernels and their launches.
//
// A render (run_wave) is a loop of iterations over the in-flight path slots
// (one slot per pixel of the launch), split into up to 3 independent lanes on
// their own streams:
//   k_trace  every closest-hit and occlusion query of the iteration, walked
//            by quads of lanes over the search BVH with octree verification
//            (rt_quad.h), as a per-wave stream with quad refill; queries it
//            cannot settle go to the fallback lists
//   k_step   its first blocks walk the fallbacks (and resume parked walks)
//            with the exact octree walk (rt_traverse.h); the rest resolve the
//            last bounce, shade the new hit (RNG draws, sampling) or end the
//            sample / start the next one, and append the emitted rays to five
//            per-kind queues (64-way sharded, wave-aggregated atomics)
//   k_tail   once few paths are left: all of them in one launch, each wave
//            stepping its own paths and tracing their rays with its quads
// Queue sizes live in device memory; the host only launches and, every 8
// iterations, reads the live-slot count.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include <dlfcn.h>
#include <chrono>
#include <mutex>
#include <thread>

#include <rccl/rccl.h>

#include "rt_context.h"
#include "rt_wave.h"
#include "rt_quad.h"
#include "rt_row.h"
#include "rt_octet.h"

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return rt_fail(ctx, RT_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));     \
    } while (0)

namespace {

#define RT_MAX_TIMED_ITERS 16384
#define RT_MAX_LANES 4  // wavefront lanes (streams) per render (run_wave)
#define RT_FAST_K 768         // fast lane: paths handed over (run_wave)
#define RT_FAST_SPP 2.25      // ... from iteration RT_FAST_SPP x spp on
#define RT_FAST_MAX_SPP 4096  // ... in renders of at most this many samples per pixel
#define RT_LANES4_MAX 1572864  // auto lanes: 4 at most this many slots per launch, else 3
#ifndef RT_STEP_OCC
#define RT_STEP_OCC 3  // k_step waves per SIMD
#endif
#ifndef RT_STEP_FILL
// k_step: blocks per CU at most, one grid-fill at its occupancy (one slot per thread below
// that; above, each wave strides over 64-slot chunks). cfg2 over 4 A/B rounds on 2 boxes:
// 8 / 4 / 3 / 2 -> 128.8-129.3 / 128.5-128.9 / 128.0-128.4 / 127.3-128.4 ms
// (profiles/r06_step_fill_ab.json)
#define RT_STEP_FILL RT_STEP_OCC
#endif
#ifndef RT_TAIL_ROWS
#define RT_TAIL_ROWS 1  // k_tail walks with rows (rt_row.h)
#endif

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// counters[] layout (int32). Iteration i (p = i & 1) runs k_trace(i) then
// k_step(i); every set is zeroed by a launch between its last reader and its
// next writer, so no reset launch is needed:
//   Q[p]      queue sizes     filled by k_step(i-1) / k_init, read by k_trace(i); k_trace(i) zeroes Q[p^1]
//   ACT[p]    live count      filled by k_step(i-1) / k_init, read by k_step(i);  k_trace(i) zeroes ACT[p^1]
//   FB[p]     fallback lists  filled by k_trace(i) (queries the quad walk could not settle), walked
//                             exactly by k_step(i); k_step(i) zeroes FB[p^1] for k_trace(i + 1)
//   PARK[p]   parked walks    filled by k_step(i), resumed by k_step(i + 1); k_trace(i) zeroes PARK[p]
//   DONE[p]   finished walks  slots, filled by k_step(i); k_trace(i + 1) releases them (r_park -= 1)
//                             and k_step(i + 1) zeroes DONE[p]. The release waits for a kernel
//                             boundary so the walk's results are visible before the path steps.
//   TK        exact-walk work tickets of k_step(i); k_trace(i) zeroes them
//
// Q and ACT are sharded: the appends of a 64-item input chunk go to one of
// RT_QSHARDS shards (append_emit), each a segment of W.seg_cap entries with
// its own counter on its own 128-B line. One counter per queue took every
// wave's atomic: ~630 us per 2 M appends on 6 counters against ~25 us
// sharded 64 ways (tools/micro/atomics.hip on the MI355X).
enum {
    C_FBC0 = 0,
    C_FBC1,
    C_FBA0,
    C_FBA1,
    C_PARKC0,
    C_PARKC1,
    C_PARKA0,
    C_PARKA1,
    C_TK_EXACT_C,
    C_TK_EXACT_A,
    C_TK_TAIL,       // k_tail: next live-list entry to take
    C_DONE0,
    C_DONE1,
    C_SHARDED = 64,  // sharded counters from here (qc_at / ac_at)
};
#define RT_QSHARDS 64
#define RT_HSHARDS 8   // heavy-class shards per kind (input shard sh -> heavy shard sh % 8)
#define RT_CSTRIDE 32  // ints from one sharded counter to the next (one 128-B line each)
#define C_HEAVY (C_SHARDED + (2 * rtk::RK_COUNT + 2) * RT_QSHARDS * RT_CSTRIDE)
#define C_COUNT (C_HEAVY + 2 * rtk::RK_COUNT * RT_HSHARDS * RT_CSTRIDE)
#define C_ZERO (C_SHARDED - 1)  // never written: the count of a padding segment
__host__ __device__ __forceinline__ int qc_at(int par, int kind, int shard)
{
    return C_SHARDED + ((par * rtk::RK_COUNT + kind) * RT_QSHARDS + shard) * RT_CSTRIDE;
}
__host__ __device__ __forceinline__ int ac_at(int par, int shard)
{
    return C_SHARDED + ((2 * rtk::RK_COUNT + par) * RT_QSHARDS + shard) * RT_CSTRIDE;
}
__host__ __device__ __forceinline__ int hc_at(int par, int kind, int shard)
{
    return C_HEAVY + ((par * rtk::RK_COUNT + kind) * RT_HSHARDS + shard) * RT_CSTRIDE;
}

// Queue segments in k_trace's stream order. Each role's heavy class comes first, so the
// walks predicted long (their path's previous query of the kind took >= W.heavy_calls
// trips) start at the head of every wave's stream instead of setting its drain:
//   [closest kinds' heavy shards][closest kinds' shards][occlusion kinds' heavy][occlusion kinds']
// then zero-count padding to a multiple of 64 (shard_prefix).
#define RT_NCK 4  // closest kinds: CONT, LSH, BL, CAM
#define RT_SEG_CH (RT_NCK * RT_HSHARDS)
#define RT_SEG_AH (RT_SEG_CH + RT_NCK * RT_QSHARDS)
#define RT_SEG_A (RT_SEG_AH + (rtk::RK_COUNT - RT_NCK) * RT_HSHARDS)
#define RT_SEG_END (RT_SEG_A + (rtk::RK_COUNT - RT_NCK) * RT_QSHARDS)
#define RT_NSEG ((RT_SEG_END + 63) / 64 * 64)
struct SegId {
    int kind, shard;
    bool heavy;
};
__host__ __device__ __forceinline__ SegId seg_id(int j)
{
    SegId s;
    if (j < RT_SEG_CH) {
        s.heavy = true, s.kind = j / RT_HSHARDS, s.shard = j % RT_HSHARDS;
    } else if (j < RT_SEG_AH) {
        s.heavy = false, s.kind = (j - RT_SEG_CH) / RT_QSHARDS, s.shard = (j - RT_SEG_CH) % RT_QSHARDS;
    } else if (j < RT_SEG_A) {
        s.heavy = true, s.kind = RT_NCK + (j - RT_SEG_AH) / RT_HSHARDS, s.shard = (j - RT_SEG_AH) % RT_HSHARDS;
    } else {
        s.heavy = false, s.kind = RT_NCK + (j - RT_SEG_A) / RT_QSHARDS, s.shard = (j - RT_SEG_A) % RT_QSHARDS;
    }
    return s;
}
__host__ __device__ __forceinline__ int seg_counter(int par, int j)
{
    if (j >= RT_SEG_END) return C_ZERO;
    const SegId s = seg_id(j);
    return s.heavy ? hc_at(par, s.kind, s.shard) : qc_at(par, s.kind, s.shard);
}

struct Backend {
    int device = 0;
    int index = 0;    // position in the context's device list (0: the root)
    hipStream_t own = nullptr;  // device-side work not on a caller's stream (multi-device shards, pixel lists)
    DevBuf nodes, tri4, prim2k, mat_idx, mats, emissive, spheres, env, env_lum, cdf;
    DevBuf bvh4, bvh16, bvh4s, bvh16s, bvh_tri4, parent, leaf_of, cdf_row, cdf_coarse, cdf_fence, matk;
    DevBuf stats;     // 2 x RT_STAT_COUNT u64: all kernels, then the tail kernel's share
    DevBuf handovers; // u64: queries k_trace handed to the exact walk, every render since the last reset
    DevBuf iterq;     // stats renders: per-iteration {queries, live slots} (RT_ITER_LOG)
    DevBuf wlog;      // stats renders with a walk log: count (256 B), then 3 float4 per record
    DevBuf wave[RT_MAX_LANES];      // per lane: path state, pending records, results, queues, lists
    DevBuf counters[RT_MAX_LANES];  // per lane: C_COUNT int32
    // fast lane (rt_test_schedule fast_k): per lane its handed-over list + ticket, counters,
    // samples-done histogram and spill area; the lanes' views for the one tail kernel over them
    DevBuf fast[RT_MAX_LANES], fcnt[RT_MAX_LANES], fhist[RT_MAX_LANES], fspill[RT_MAX_LANES], fviews;
    int32_t* h_hist[RT_MAX_LANES] = {};
    rtk::WaveView* h_fviews = nullptr;  // pinned
    hipEvent_t fev[RT_MAX_LANES] = {}, fev_done = nullptr;
    hipEvent_t hev[RT_MAX_LANES] = {};  // fast lane: each lane's samples-done histogram readback
    bool fev_done_recorded = false;
    hipEvent_t ftev[2] = {};  // (timed renders: around the fast lane's kernel)
    hipStream_t fs = nullptr;  // the fast lane's stream with 4 lanes (fewer: the first idle lane stream)
    DevBuf xy;        // pixel list (rt_render_pixels)
    DevBuf fb;        // host-fb staging
    int32_t* h_act[RT_MAX_LANES] = {};     // per lane, pinned: live-slot counters (sharded) + 8 fallback counters
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_done = nullptr;  // end of the last run_wave (all lanes joined): the next render waits for it
    bool done_recorded = false;
    hipStream_t ls[RT_MAX_LANES] = {};      // lanes 1.. streams (lane 0 runs on the caller's)
    hipEvent_t ev_fork = nullptr, ev_join[RT_MAX_LANES] = {}, ev_lane[RT_MAX_LANES] = {};
    int lanes = 0;                          // RT_LANES; 0: auto, 4 lanes for launches of at most RT_LANES4_MAX
                                            // slots, else 3 (cfg2 1-4 lanes: 452 / 499 / 519 / 509 Msamples/s, r01;
                                            // r03: 3 / 4 lanes cfg2 147.5 / 148.6 ms, cfg4 8-way shard 398 / 386 ms,
                                            // 6 / 8 lanes 230-710 ms: more streams than the 4 hardware queues)
    RtSceneView view{};
    int bl_rays = 1, any_rays = 1;
    int last_iters = 0;
    int tail_iter = -1;     // iteration whose step launch was the tail kernel (-1: none)
    int budget = 1024;  // steps per query per launch before it parks (RT_STEP_BUDGET)
    // optional per-kernel timing: events around each launch of each class
    bool timing = false;
    hipEvent_t tev[RT_MAX_LANES][3][RT_MAX_TIMED_ITERS] = {};
    double kms[3] = {0, 0, 0};      // k_trace, k_step, k_tail
    long klaunch[3] = {0, 0, 0};
};

int ensure(rt_context* c, DevBuf& b, size_t bytes)
{
    if (b.bytes >= bytes && b.p) return RT_OK;
    if (b.p) HIPCHK(c, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    if (bytes == 0) return RT_OK;
    HIPCHK(c, hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    return RT_OK;
}

template <class T>
int upload(rt_context* c, DevBuf& b, const std::vector<T>& v)
{
    const size_t bytes = v.size() * sizeof(T);
    if (int r = ensure(c, b, bytes > 0 ? bytes : 16)) return r;
    if (bytes) HIPCHK(c, hipMemcpy(b.p, v.data(), bytes, hipMemcpyHostToDevice));
    return RT_OK;
}


// ------------------------------------------------------------ wave helpers
#ifndef RT_DEBUG_FB
#define RT_DEBUG_FB 0  // study builds: count k_trace's exact-walk hand-overs and the octet walks'
                       // parks of the timed renders, printed on stderr after each run_wave
#endif
#if RT_DEBUG_FB
__device__ unsigned long long rt_dbg_fb[8];  // k_trace closest fallbacks, octet parks, occlusion fallbacks, overflows, ties, chain fails, from rows, -
#define RT_DBG(i) atomicAdd(&rt_dbg_fb[i], 1ull)
#else
#define RT_DBG(i) ((void)0)
#endif
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-aggregated append: every lane of the wave must call this converged.
// Returns this lane's slot in the queue whose size lives at *counter.
__device__ __forceinline__ int wave_append(int32_t* counter, bool want)
{
    const unsigned long long b = __ballot(want);
    if (b == 0) return -1;
    const int leader = __ffsll((long long)b) - 1;
    int base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, __popcll(b));
    base = __shfl(base, leader);
    const unsigned long long lt = (lane_id() == 0) ? 0ull : (b & (~0ull >> (64 - lane_id())));
    return want ? base + __popcll(lt) : -1;
}

// Per-lane traversal stack in LDS: entry i of thread t at [i * 256 + t]
// (a wave at equal depth touches 64 consecutive words: no bank conflicts).
template <int N>
struct LdsStack {
    static constexpr int CAP = N;
    uint32_t* r;
    float* k;
    __device__ __forceinline__ uint32_t rec(int i) const { return r[i * 256]; }
    __device__ __forceinline__ float key(int i) const { return k[i * 256]; }
    __device__ __forceinline__ void set(int i, uint32_t rv, float kv)
    {
        r[i * 256] = rv;
        k[i * 256] = kv;
    }
    __device__ __forceinline__ void set_rec(int i, uint32_t rv) { r[i * 256] = rv; }
};

// Static wave-strided work assignment: wave w of the grid takes items
// [w*64, w*64+64), then strides by the grid's wave count. (A shared atomic
// ticket per 64 items serialized ~4k atomics on one address per launch:
// ~45 us even for an empty queue.)
__device__ __forceinline__ int wave_gid() { return (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); }
__device__ __forceinline__ int wave_count() { return (int)((gridDim.x * blockDim.x) >> 6); }

template <bool STATS>
__device__ __forceinline__ void flush_stats(const rtk::Stats& st, unsigned long long* out)
{
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++)
            if (st.c[i]) atomicAdd(&out[i], st.c[i]);
}

// ------------------------------------------------------------------ kernels
// Queue record base of (kind, heavy class, shard): a normal shard holds seg_cap records, a
// heavy shard RT_QSHARDS / RT_HSHARDS seg_caps (it takes the input shards sh with sh % RT_HSHARDS = its index).
__host__ __device__ __forceinline__ size_t qbase(bool heavy, int shard, size_t seg_cap)
{
    return heavy ? ((size_t)RT_QSHARDS + (size_t)shard * (RT_QSHARDS / RT_HSHARDS)) * seg_cap : (size_t)shard * seg_cap;
}

// Appends what the wave's lanes emitted to the queues and the live list of
// parity pout, in the shard of the 64-item input chunk `base` (whole wave).
// Shards take contiguous runs of the n_in inputs' chunks, so a queue read in
// order follows its input order (pixel order, through the compactions).
template <class E>
__device__ __forceinline__ void append_emit(const rtk::WaveView& W, int pout, int base, int n_in, int p, const E& e)
{
    const int cps = ((n_in + 63) / 64 + RT_QSHARDS - 1) / RT_QSHARDS;  // chunks per shard
    const int sh = min(RT_QSHARDS - 1, (base >> 6) / cps);
    const size_t seg = (size_t)sh * W.seg_cap;
    const unsigned long long lt = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
    if (W.r_heavy) {  // heavy class on: the rays of a path flagged heavy go to its kind's heavy shard
        const int hs = sh % RT_HSHARDS;
        unsigned long long b[2 * rtk::RK_COUNT + 1];
#pragma unroll
        for (int k = 0; k < rtk::RK_COUNT; k++) {
            const bool m = (e.mask >> k) & 1u;
            b[k] = __ballot(m && !e.heavy);
            b[rtk::RK_COUNT + k] = __ballot(m && e.heavy);
        }
        b[2 * rtk::RK_COUNT] = __ballot(e.active);
        int r[2 * rtk::RK_COUNT + 1];
        if (lane_id() == 0) {
#pragma unroll
            for (int k = 0; k <= 2 * rtk::RK_COUNT; k++) {
                const int c = k < rtk::RK_COUNT ? qc_at(pout, k, sh)
                              : k < 2 * rtk::RK_COUNT ? hc_at(pout, k - rtk::RK_COUNT, hs)
                                                      : ac_at(pout, sh);
                r[k] = b[k] ? atomicAdd(W.counters + c, __popcll(b[k])) : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < rtk::RK_COUNT; k++) {
            const int ih = __shfl(r[rtk::RK_COUNT + k], 0) + __popcll(b[rtk::RK_COUNT + k] & lt);
            const int i = __shfl(r[k], 0) + __popcll(b[k] & lt);
            if ((e.mask >> k) & 1u) W.q[k][e.heavy ? qbase(true, hs, W.seg_cap) + ih : qbase(false, sh, W.seg_cap) + i] = e.rec(k, p);
        }
        const int a = __shfl(r[2 * rtk::RK_COUNT], 0) + __popcll(b[2 * rtk::RK_COUNT] & lt);
        if (e.active) W.act_out[seg + a] = p;
        return;
    }
    // the six reservations (five queues, the live list) issued back to back by lane 0
    // and waited for once, then the stores: one atomic round trip, not six in a row
    unsigned long long b[rtk::RK_COUNT + 1];
#pragma unroll
    for (int k = 0; k < rtk::RK_COUNT; k++) b[k] = __ballot((e.mask >> k) & 1u);
    b[rtk::RK_COUNT] = __ballot(e.active);
    int r[rtk::RK_COUNT + 1];
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k <= rtk::RK_COUNT; k++)
            r[k] = b[k] ? atomicAdd(W.counters + (k < rtk::RK_COUNT ? qc_at(pout, k, sh) : ac_at(pout, sh)),
                                    __popcll(b[k]))
                        : 0;
    }
#pragma unroll
    for (int k = 0; k < rtk::RK_COUNT; k++) {
        const int i = __shfl(r[k], 0) + __popcll(b[k] & lt);
        if ((e.mask >> k) & 1u) W.q[k][qbase(false, sh, W.seg_cap) + i] = e.rec(k, p);
    }
    const int a = __shfl(r[rtk::RK_COUNT], 0) + __popcll(b[rtk::RK_COUNT] & lt);
    if (e.active) W.act_out[seg + a] = p;
}


// Exclusive prefix sums of the sharded counters at cnt[at(j)], j < m (m a
// multiple of 64), into pre[0..m] (LDS); every thread of the block calls.
template <class AT>
__device__ __forceinline__ void shard_prefix(const int32_t* cnt, int m, AT at, int* pre)
{
    const int nw = (int)(blockDim.x >> 6), w = (int)(threadIdx.x >> 6);
    for (int g = w; g < m / 64; g += nw) {  // one wave per 64 counters: inclusive scan
        int v = cnt[at(g * 64 + lane_id())];
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(v, o);
            if (lane_id() >= o) v += u;
        }
        pre[g * 64 + lane_id() + 1] = v;
    }
    __syncthreads();
    // chain the groups: entry (g, lane) adds the totals of groups < g (read before any write)
    int add[8];
    const int ng = m / 64;
    for (int g = w; g < ng && g < 8 * nw; g += nw) {
        int off = 0;
        for (int h = 0; h < g; h++) off += pre[h * 64 + 64];
        add[g / nw] = off;
    }
    __syncthreads();
    for (int g = w; g < ng && g < 8 * nw; g += nw) pre[g * 64 + lane_id() + 1] += add[g / nw];
    if (threadIdx.x == 0) pre[0] = 0;
    __syncthreads();
}

// Segment j of a prefix table pre[0..m] holding global index g (pre[j] <= g < pre[j+1]).
__device__ __forceinline__ int shard_find(const int* pre, int m, int g)
{
    int lo = 0, hi = m - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= g)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

// The same search with M (a compile-time table size) as an 8-way search: each round reads 7
// entries at once (independent LDS reads, one round trip) and advances by the count at or below
// g (the table is non-decreasing), so 448 entries take 3 dependent round trips instead of 9 and
// 64 take 2 instead of 6. k_trace's refill (on ~4 of 5 wave trips, the whole wave waiting) and
// every k_step / k_tail chunk start search these tables.
#ifndef RT_FIND8
#define RT_FIND8 1
#endif
template <int M>
__device__ __forceinline__ int shard_find8(const int* pre, int g)
{
#if RT_FIND8
    constexpr int TOP = M > 512 ? 512 : M > 64 ? 64 : M > 8 ? 8 : 1;
    static_assert(M <= 4096, "three or four 8-way rounds");
    int lo = 0;
#pragma unroll
    for (int step = TOP; step >= 1; step >>= 3) {
        int c = 0;
#pragma unroll
        for (int k = 1; k < 8; k++) {
            const int j = lo + step * k;
            c += (j < M && pre[j] <= g) ? 1 : 0;
        }
        lo += step * c;
    }
    return lo;
#else
    return shard_find(pre, M, g);
#endif
}

// Where stream position g's queue record lives (segment table pre[0..RT_NSEG]) and its kind.
__device__ __forceinline__ const rtk::RayRec* queue_item_ptr(const rtk::WaveView& W, const int* pre, int g, int& kind)
{
    const int j = shard_find8<RT_NSEG>(pre, g);
    const SegId s = seg_id(j);
    kind = s.kind;
    rtk::RayRec* qk = W.q[0];
#pragma unroll
    for (int k2 = 1; k2 < rtk::RK_COUNT; k2++) qk = s.kind == k2 ? W.q[k2] : qk;
    return qk + qbase(s.heavy, s.shard, W.seg_cap) + (g - pre[j]);
}

// Queue item of stream position g (segment table pre[0..RT_NSEG], k_trace): the ray and its kind.
__device__ __forceinline__ rtk::RayRec queue_item_at(const rtk::WaveView& W, const int* pre, int g, int& kind)
{
    // (the queue base by selects: W.q[kind] with a lane-varying kind would be a load; heavy
    // shard h: after the kind's RT_QSHARDS segments, RT_QSHARDS / RT_HSHARDS seg_caps each)
    return *queue_item_ptr(W, pre, g, kind);
}

// k_trace's look-ahead (RT_TRACE_PREFETCH): right after a refill, the wave's next 16 stream
// positions are copied into its LDS buffer by direct-to-LDS loads (lane 2i + h: half h of
// record i, 16 B; the hardware puts lane L's 16 B at buf + 16 L), their kinds alongside; the next
// refill takes its records from there (a refill needs at most 16 positions, all from the
// cursor on, which the buffer starts at), so the refill no longer waits on the queue's memory.
#ifndef RT_TRACE_PREFETCH
#define RT_TRACE_PREFETCH 1
#endif
struct QPrefetch {
    float4_* buf;  // the wave's 64 x 16 B (records 0..15 in the first 512 B)
    int* kind;     // the wave's 16 kinds (-1: past the end of the stream)
};
__device__ __forceinline__ void queue_prefetch(const rtk::WaveView& W, const int* pre, const QPrefetch& pf, int first, int cursor,
                                               int wg, int wn, int total)
{
    const int lane = lane_id(), i = lane >> 1;
    const int j = cursor + i;
    const int idx = (wg + (j >> 4) * wn) * 16 + (j & 15);
    const bool ok = lane < 32 && idx < total;
    int kind = -1;
    if (ok) {
        const rtk::RayRec* rp = queue_item_ptr(W, pre, first + idx, kind);
        __builtin_amdgcn_global_load_lds((const void*)((const float4_*)rp + (lane & 1)),
                                         (__attribute__((address_space(3))) void*)pf.buf, 16, 0, 0);
    }
    if (lane < 32 && (lane & 1) == 0) pf.kind[i] = ok ? kind : -1;
}

// Path init: every slot seeds its RNG and emits its first camera ray (into Q[0], ACT[0]).
__global__ __launch_bounds__(256) void k_init(rtk::WaveView W)
{
    rtlibm::lds_tables_init();  // (a pixel of a 0-bounce render is tone-mapped here)
    const int p = blockIdx.x * blockDim.x + threadIdx.x;  // grid covers whole waves
    rtk::Emit e;
    e.mask = 0;
    e.active = false;
    e.heavy = false;
    if (p < W.n_slots) rtk::path_init(W, p, e);
    append_emit(W, 0, p & ~63, W.n_slots, p, e);
}

// After a lane's last step: the tone-map of every pixel of the lane (rt_wave.h tonemap_pixel).
__global__ __launch_bounds__(256) void k_tonemap(rtk::WaveView W)
{
    rtlibm::lds_tables_init();
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < W.n_slots) rtk::tonemap_pixel(W, p);
}

// ------------------------------------------------------------- query kernel
// Every closest-hit and occlusion query of the iteration, plus the exact
// octree walks of the queries the previous iteration could not settle, in
// one launch: the blocks are split into four roles computed alike by every
// block from the counters.
//  * exact roles (blocks first, so their long dependent walks start early
//    and hide under the bulk): the previous launch's fallback lists and
//    parked walks, through the resumable octree walk (rt_traverse.h).
//    Persistent waves; idle lanes refill once RT_REFILL of them are idle; a
//    walk that has taken W.budget steps parks at its next node boundary and
//    continues in the next launch.
//  * fast roles (the rest, split in proportion to the two queues): one query
//    per lane through the search BVH (rt_fast.h), node-index stack in LDS. A
//    query whose answer needs the exact walk (or whose stack would overflow)
//    goes to the fallback list for the next launch, and its slot's r_park
//    count keeps k_step off the path until the walk has finished.
#ifndef RT_STEP_EMIT_LDS
#define RT_STEP_EMIT_LDS 1  // k_step's and k_tail's emitted rays wait in LDS (rt_wave.h EmitLds), not in VGPRs
#endif
#define RT_LDS_WORDS 16         // LDS words per lane of k_trace (16 KB per block of 256)
#define RT_LDS_CAP_FAST 16      // search-BVH stack: node + key in LDS ...
#define RT_SPILL_FAST RT_FAST_SPILL  // ... then in the lane's global spill area
#define RT_LDS_CAP_CLOSEST 8    // exact walks: key + record (windows are powers of two)
#define RT_LDS_CAP_ANY 16
#define RT_REFILL 16
#define RT_QSTACK 32            // quad walks (rt_quad.h): stack entries per quad (item + key, 64 quads per block)
#define RT_RSTACK 64            // row walks (rt_row.h): stack entries per row (item + key, 16 rows per block)
#ifndef RT_TRACE_REFILL
#define RT_TRACE_REFILL 4       // k_trace: idle quads of a wave that trigger a refill from its query stream
                                // (r02, cfg2: 4 / 8 -> 726 / 723 vs 678 Msamples/s with static 16-query chunks)
#endif
#ifndef RT_HEAVY_CALLS
#define RT_HEAVY_CALLS 6        // heavy class (seg_id): quad_visit calls of a walk that flag its path (0: off).
                                // cfg2 (r02): off / 3 / 6 / 10 / 16 -> 737 / 744 / 744-748 / 740 / 735 Msamples/s;
                                // 1-lane k_trace 124.1 -> 117.2 ms, drain slots 838 M -> 737 M
                                // (a dynamic, per-XCD-ticketed tail of the stream, 10-40 %: 684-691, rejected)
#endif
#ifndef RT_TRACE_OCC
#define RT_TRACE_OCC 6          // k_trace waves per SIMD (8 fits the quad walks in 64 VGPRs but measured
                                // 512 vs 539 Msamples/s: more trace waves crowd the other lanes k_step)
#endif

// Search-BVH stack of a fast query: entries [0, N) in LDS (entry i of
// thread t at [i * 256 + t]: a wave at equal depth touches 64 consecutive
// words), the rest in the lane's global spill area (deep stacks are rare).
template <int N, int M>
struct FastStack {
    static constexpr int CAP = N + M;
    uint32_t* r;
    float* k;
    uint32_t* gr;
    float* gk;
    __device__ __forceinline__ uint32_t rec(int i) const { return i < N ? r[i * 256] : gr[i - N]; }
    __device__ __forceinline__ float key(int i) const { return i < N ? k[i * 256] : gk[i - N]; }
    __device__ __forceinline__ void set(int i, uint32_t rv, float kv)
    {
        if (i < N) {
            r[i * 256] = rv;
            k[i * 256] = kv;
        } else {
            gr[i - N] = rv;
            gk[i - N] = kv;
        }
    }
};

// Does this query skip the search-BVH walk for the exact octree walk? Its origin lies outside
// the near box (rt_fast.h far_origin), or the force_fallback stressor's ray hash selects it.
__device__ __forceinline__ bool forced_fallback(const rtk::WaveView& W, const float4_& o, const float4_& d)
{
    return (W.far_check && rtk::far_origin(W.S, rtk::v3of(o))) || rtk::forced_fallback(W.force_fb, o, d);
}

// Blocks [0, n0) take role 0, the rest role 1, in proportion to the work.
__device__ __forceinline__ int split_blocks(int nb, int w0, int w1)
{
    if (w0 + w1 == 0) return 0;
    int n0 = (int)((long)nb * w0 / ((long)w0 + w1));
    if (w0 > 0 && n0 == 0) n0 = 1;
    if (w1 > 0 && n0 == nb) n0 = nb - 1;
    return n0;
}

// A finished exact walk: its slot goes to DONE[par]; k_trace(i + 1) releases it.
__device__ __forceinline__ void walk_done(const rtk::WaveView& W, int par, uint32_t target)
{
    const int j = atomicAdd(W.counters + C_DONE0 + par, 1);
    W.done[par][j] = (int32_t)(target >> 3);
}

#ifndef RT_EXACT_OCTET
#define RT_EXACT_OCTET 1  // k_step's exact walks: 8 lanes per query (rt_octet.h); 0: one lane per query
#endif
#if RT_EXACT_OCTET
// Exact octree walks of k_step(i) (par = i & 1), one octet of lanes per query (rt_octet.h):
// the walks parked by k_step(i - 1) (PARK[par ^ 1], the first n_res tickets), then the
// fallbacks of k_trace(i) (FB[par]). ANY selects the occlusion walk.
template <bool ANY>
__device__ void exact_octets(const rtk::WaveView& W, int par, uint32_t* lds, int lane, int n_res, int total,
                             rtk::Stats* st)
{
    rtk::OctRing w = rtk::oct_ring(lds);
    const int sub = lane_id() & 7;
    uint32_t* spr = W.spill_r + (size_t)(lane & ~7) * RT_STACK_CAP;  // the leader lane's spill area
    float* spk = W.spill_k + (size_t)(lane & ~7) * RT_STACK_CAP;
    const rtk::RayRec* fb = ANY ? W.fb_a[par] : W.fb_c[par];
    int32_t* ticket = W.counters + (ANY ? C_TK_EXACT_A : C_TK_EXACT_C);
    int32_t* parked = W.counters + (ANY ? C_PARKA0 : C_PARKC0) + par;
    rtk::TravG T;
    bool has = false, drained = false;  // (octet-uniform)
    uint32_t target = 0;
    auto done = [&]() {
        if (sub == 0) {
            if (ANY)
                rtk::finish_any(W, target, T.hit);  // (false, or the brute-force answer)
            else
                rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
            walk_done(W, par, target);
        }
    };
    for (;;) {
        const unsigned long long bneed = __ballot(!has && sub == 0);
        const int nneed = __popcll(bneed);
        if (!drained && (nneed >= RT_REFILL / 8 || nneed == 8)) {
            int base = 0;
            if (lane_id() == 0) base = atomicAdd(ticket, nneed);
            base = __shfl(base, 0);
            if (base + nneed >= total) drained = true;
            if (!has) {
                const int idx = base + __popcll(bneed & ((1ull << rtk::oct_lane0()) - 1ull));
                if (idx < n_res) {
                    target = ANY ? rtk::octa_resume(W.S, &W.park_a[par ^ 1][idx], T, w, sub)
                                 : rtk::octc_resume(W.S, &W.park_c[par ^ 1][idx], T, w, sub);
                    has = true;
                } else if (idx < total) {
                    const rtk::RayRec r = fb[idx - n_res];
                    target = (rt_asuint(r.o.w) << 3) | rt_asuint(r.d.w);
                    if (st && sub == 0) st->c[RT_STAT_FALLBACK]++;
                    has = rtk::octg_setup(W.S, T, rtk::v3of(r.o), rtk::v3of(r.d), st, ANY, sub);
                    if (!has) done();
                }
            }
        }
        if (!__any(has)) {
            if (drained) break;
            continue;
        }
        if (has) {
            if (ANY)
                rtk::octa_node(W.S, T, w, spr, sub, st);
            else
                rtk::octc_node(W.S, T, w, spr, spk, sub, st);
            if (T.mode == rtk::TM_DONE) {
                done();
                has = false;
            } else if (T.steps >= W.budget && (ANY ? rtk::octa_parkable(T) : rtk::octc_parkable(T))) {
                int ps = 0;
                if (sub == 0) ps = atomicAdd(parked, 1);
                if (sub == 0) RT_DBG(1);
                ps = __shfl(ps, rtk::oct_lane0());
                if (ps < W.park_cap) {
                    if (ANY)
                        rtk::octa_park(T, w, target, &W.park_a[par][ps], sub);
                    else
                        rtk::octc_park(T, w, target, &W.park_c[par][ps], sub);
                    has = false;
                } else {
                    T.steps = 0;  // park pool full: keep going
                }
            }
        }
    }
}
#else
// Exact octree walks of k_step(i) (par = i & 1): the walks parked by k_step(i - 1)
// (PARK[par ^ 1], the first n_res tickets), then the fallbacks of k_trace(i) (FB[par]).
__device__ void exact_closest(const rtk::WaveView& W, int par, uint32_t* lds, int lane, int n_res, int total,
                              rtk::Stats* st)
{
    using FAST = LdsStack<RT_LDS_CAP_CLOSEST>;
    rtk::SpillStack<FAST> stk{FAST{lds + threadIdx.x, (float*)lds + RT_LDS_CAP_CLOSEST * 256 + threadIdx.x},
                              W.spill_r + (size_t)lane * RT_STACK_CAP, W.spill_k + (size_t)lane * RT_STACK_CAP};
    const rtk::RayRec* fb = W.fb_c[par];
    rtk::TravC T;
    bool has = false, drained = false;
    uint32_t target = 0;
    for (;;) {
        const bool need = !has;
        const unsigned long long bneed = __ballot(need);
        const int nneed = __popcll(bneed);
        if (!drained && (nneed >= RT_REFILL || nneed == 64)) {
            int base = 0;
            if (lane_id() == 0) base = atomicAdd(W.counters + C_TK_EXACT_C, nneed);
            base = __shfl(base, 0);
            if (base + nneed >= total) drained = true;
            if (need) {
                const int idx = base + __popcll(bneed & ((1ull << lane_id()) - 1ull));
                if (idx < n_res) {
                    target = rtk::travc_resume(&W.park_c[par ^ 1][idx], T, stk);
                    has = true;
                } else if (idx < total) {
                    const rtk::RayRec r = fb[idx - n_res];
                    target = (rt_asuint(r.o.w) << 3) | rt_asuint(r.d.w);
                    if (st) st->c[RT_STAT_FALLBACK]++;
                    has = rtk::travc_begin(W.S, T, rtk::v3of(r.o), rtk::v3of(r.d), st);
                    if (!has) {
                        rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
                        walk_done(W, par, target);
                    }
                }
            }
        }
        if (!__any(has)) {
            if (drained) break;
            continue;
        }
        if (has) {
            if (!rtk::travc_step(W.S, T, stk, st)) {
                rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
                walk_done(W, par, target);
                has = false;
            } else if (T.steps >= W.budget && rtk::travc_parkable(T)) {
                const int ps = atomicAdd(W.counters + C_PARKC0 + par, 1);
                if (ps < W.park_cap) {
                    rtk::travc_park(T, stk, target, &W.park_c[par][ps]);
                    has = false;
                } else {
                    T.steps = 0;  // park pool full: keep going
                }
            }
        }
    }
}

__device__ void exact_any(const rtk::WaveView& W, int par, uint32_t* lds, int lane, int n_res, int total,
                          rtk::Stats* st)
{
    using FAST = LdsStack<RT_LDS_CAP_ANY>;
    rtk::SpillStack<FAST> stk{FAST{lds + threadIdx.x, nullptr}, W.spill_r + (size_t)lane * RT_STACK_CAP, nullptr};
    const rtk::RayRec* fb = W.fb_a[par];
    rtk::TravA T;
    bool has = false, drained = false;
    uint32_t target = 0;
    for (;;) {
        const bool need = !has;
        const unsigned long long bneed = __ballot(need);
        const int nneed = __popcll(bneed);
        if (!drained && (nneed >= RT_REFILL || nneed == 64)) {
            int base = 0;
            if (lane_id() == 0) base = atomicAdd(W.counters + C_TK_EXACT_A, nneed);
            base = __shfl(base, 0);
            if (base + nneed >= total) drained = true;
            if (need) {
                const int idx = base + __popcll(bneed & ((1ull << lane_id()) - 1ull));
                if (idx < n_res) {
                    target = rtk::trava_resume(&W.park_a[par ^ 1][idx], T, stk);
                    has = true;
                } else if (idx < total) {
                    const rtk::RayRec r = fb[idx - n_res];
                    target = (rt_asuint(r.o.w) << 3) | rt_asuint(r.d.w);
                    if (st) st->c[RT_STAT_FALLBACK]++;
                    has = rtk::trava_begin(W.S, T, rtk::v3of(r.o), rtk::v3of(r.d), st);
                    if (!has) {
                        rtk::finish_any(W, target, T.hit);  // (false, or the brute-force answer)
                        walk_done(W, par, target);
                    }
                }
            }
        }
        if (!__any(has)) {
            if (drained) break;
            continue;
        }
        if (has) {
            if (!rtk::trava_step(W.S, T, stk, st)) {
                rtk::finish_any(W, target, T.hit);
                walk_done(W, par, target);
                has = false;
            } else if (T.steps >= W.budget && rtk::trava_parkable(T)) {
                const int ps = atomicAdd(W.counters + C_PARKA0 + par, 1);
                if (ps < W.park_cap) {
                    rtk::trava_park(T, stk, target, &W.park_a[par][ps]);
                    has = false;
                } else {
                    T.steps = 0;
                }
            }
        }
    }
}

#endif

// Path step of iteration i (par = i & 1): resolve, shade, next sample, for
// every live path not waiting on an exact walk; the first blocks instead run
// the exact octree walks of this iteration's fallbacks and of the walks parked
// last iteration (they need the registers this kernel has anyway; k_trace
// stays small enough for 8 waves per SIMD).
template <bool STATS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_OCC, 8))) void k_step(rtk::WaveView W, int par, unsigned long long* stats)
{
    // (the exact roles' stacks; in the path-step blocks, the emitted rays: rt_wave.h EmitLds)
    __shared__ uint32_t s_lds[(RT_STEP_EMIT_LDS ? 6 * rtk::RK_COUNT : RT_LDS_WORDS) * 256];
    static_assert(6 * rtk::RK_COUNT >= RT_LDS_WORDS, "the exact roles' stacks fit the emit columns");
    __shared__ int s_pre[RT_QSHARDS + 1];
    rtlibm::lds_tables_init();
    rtk::lds_shade_init(W.S);  // (the env-map row search and a small material table from LDS)
    int32_t* cnt = W.counters;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // for k_trace(i + 1); DONE[par ^ 1] was released by k_trace(i)
        cnt[C_FBC0 + (par ^ 1)] = cnt[C_FBA0 + (par ^ 1)] = 0;
        cnt[C_DONE0 + (par ^ 1)] = 0;
        // (k_trace(i)'s hand-overs to the exact walk, summed for rt_device_exact_handovers: a
        // health figure, ~1e-6 of the queries; a search-BVH walk that went wrong shows here)
        const int nf = cnt[C_FBC0 + par] + cnt[C_FBA0 + par];
        if (W.handovers && nf > 0) atomicAdd(W.handovers, (unsigned long long)nf);
    }
    rtk::Stats st;
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++) st.c[i] = 0;
    rtk::Stats* ps = STATS ? &st : nullptr;
    // exact roles: 32 walks per block to start with (8 octets per wave), at most half of the
    // spill lanes and a quarter of the grid each
    const int nrc = min(cnt[C_PARKC0 + (par ^ 1)], W.park_cap), nra = min(cnt[C_PARKA0 + (par ^ 1)], W.park_cap);
    const int ec = nrc + cnt[C_FBC0 + par], ea = nra + cnt[C_FBA0 + par];
    // (the host launches >= 3 blocks, so both exact roles and the path step each get one:
    // with gridDim 3, half = 1; above, the exact roles take at most half of the grid)
    const int half = min(W.spill_lanes / 512, max(1, (int)gridDim.x / 4));
    constexpr int WPB = RT_EXACT_OCTET ? 32 : 64;  // walks per block at once (octets / lanes)
    const int nbe_c = min(half, (ec + WPB - 1) / WPB), nbe_a = min(half, (ea + WPB - 1) / WPB);
    const int b = (int)blockIdx.x;
    if (b < nbe_c) {
#if RT_EXACT_OCTET
        exact_octets<false>(W, par, s_lds, b * 256 + (int)threadIdx.x, nrc, ec, ps);
#else
        exact_closest(W, par, s_lds, b * 256 + (int)threadIdx.x, nrc, ec, ps);
#endif
        flush_stats<STATS>(st, stats);
        return;
    }
    if (b < nbe_c + nbe_a) {
#if RT_EXACT_OCTET
        exact_octets<true>(W, par, s_lds, (W.spill_lanes / 512 + b - nbe_c) * 256 + (int)threadIdx.x, nra, ea, ps);
#else
        exact_any(W, par, s_lds, (W.spill_lanes / 512 + b - nbe_c) * 256 + (int)threadIdx.x, nra, ea, ps);
#endif
        flush_stats<STATS>(st, stats);
        return;
    }
    shard_prefix(cnt, RT_QSHARDS, [&](int j) { return ac_at(par, j); }, s_pre);
    const int n = s_pre[RT_QSHARDS];
    if (STATS && W.iterq && b == nbe_c + nbe_a && threadIdx.x == 0 && W.iter < RT_MAX_TIMED_ITERS)
        W.iterq[2 * W.iter + 1] = n;
    const int nbs = (int)gridDim.x - (nbe_c + nbe_a);
    const int wg = (b - nbe_c - nbe_a) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
    const int wn = nbs * (int)(blockDim.x >> 6);
    for (int base = wg * 64; base < n; base += wn * 64) {
        const int idx = base + lane_id();
#if RT_STEP_EMIT_LDS
        rtk::EmitLds<256> e;
        e.s = reinterpret_cast<float*>(s_lds) + threadIdx.x;
#else
        rtk::Emit e;
#endif
        e.mask = 0;
        e.active = false;
        e.heavy = false;
        int p = -1;
        if (idx < n) {
            const int sh = shard_find8<RT_QSHARDS>(s_pre, idx);
            p = W.act_in[(size_t)sh * W.seg_cap + (idx - s_pre[sh])];
            rtk::path_step(W, p, e, ps);
        }
        append_emit(W, par ^ 1, base, n, p, e);
    }
    flush_stats<STATS>(st, stats);
}

// The fast lane's hand-over (run_wave), between a lane's k_trace and k_step: the live paths of
// iteration par's list with at most W.fast_thr samples done and no parked query, up to
// W.fast_cap of them, move to W.fast_list (their wait counts become -1: k_step drops them from
// the lane's live list, rt_wave.h path_step; the fast lane's tail kernel clears the mark).
__global__ __launch_bounds__(256) void k_hand(rtk::WaveView W, int par)
{
    __shared__ int s_pre[RT_QSHARDS + 1];
    shard_prefix(W.counters, RT_QSHARDS, [&](int j) { return ac_at(par, j); }, s_pre);
    const int n = s_pre[RT_QSHARDS];
    for (int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x); idx < n; idx += (int)(gridDim.x * blockDim.x)) {
        const int sh = shard_find8<RT_QSHARDS>(s_pre, idx);
        const int p = W.act_in[(size_t)sh * W.seg_cap + (idx - s_pre[sh])];
        if ((int)rt_asuint(W.p_thr[p].w) > W.fast_thr || W.r_park[p] != 0) continue;
        const int j = atomicAdd(W.fast_ticket, 1);
        if (j >= W.fast_cap) continue;
        W.fast_list[j] = p;
        W.r_park[p] = -1;
    }
}

// Samples done by the live paths of iteration par's list (the fast lane's selection, run_wave).
__global__ __launch_bounds__(256) void k_hist(rtk::WaveView W, int par, int32_t* __restrict__ hist)
{
    __shared__ int s_pre[RT_QSHARDS + 1];
    shard_prefix(W.counters, RT_QSHARDS, [&](int j) { return ac_at(par, j); }, s_pre);
    const int n = s_pre[RT_QSHARDS];
    for (int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x); idx < n; idx += (int)(gridDim.x * blockDim.x)) {
        const int sh = shard_find8<RT_QSHARDS>(s_pre, idx);
        const int p = W.act_in[(size_t)sh * W.seg_cap + (idx - s_pre[sh])];
        atomicAdd(hist + min((int)rt_asuint(W.p_thr[p].w), W.spp), 1);
    }
}

// Stats renders with a walk log (rt_test_walk_log, include/rt_hip.h): one record per walk of at
// least W.wlog_min quad_visit calls. where: 0 k_trace quads, 1 a k_trace drain's rows, 2 k_tail.
__device__ __noinline__ void walk_log(const rtk::WaveView& W, rtk::V3 o, rtk::V3 d, uint32_t target, int calls, float t,
                                      int k, int where)
{
    if (W.wlog_every < 0 && t != -2.0f) return;  // (only the walks left to the exact walk)
    if (W.wlog_every > 1 && ((target * 2654435761u) ^ ((uint32_t)W.iter * 40503u)) % (uint32_t)W.wlog_every != 0u) return;
    const int i = atomicAdd(W.wlog_n, 1);
    if (i >= W.wlog_cap) return;
    float4_* r = W.wlog + 3 * (size_t)i;
    r[0] = float4_{o.x, o.y, o.z, rt_asfloat((target & 7u) | ((uint32_t)where << 8))};
    r[1] = float4_{d.x, d.y, d.z, rt_asfloat((uint32_t)calls)};
    r[2] = float4_{t, rt_asfloat((uint32_t)k), rt_asfloat((uint32_t)W.iter), rt_asfloat(target >> 3)};
}

// A row's stack held in its wave's quad stacks (k_trace's drain, trace_stream): row k of a
// wave uses the words of the wave's quads 4k .. 4k+3, entry e at depth e >> 2 of quad
// 4k + (e & 3), so converting the wave's walks to rows needs no other LDS.
struct RowInQuadStack {
    static constexpr int CAP = 4 * RT_QSTACK;
    uint32_t* r;  // the word of quad 4k, depth 0
    float* k;
    __device__ __forceinline__ uint32_t rec(int i) const { return r[(i >> 2) * 64 + (i & 3)]; }
    __device__ __forceinline__ float key(int i) const { return k[(i >> 2) * 64 + (i & 3)]; }
    __device__ __forceinline__ void set(int i, uint32_t rv, float kv)
    {
        r[(i >> 2) * 64 + (i & 3)] = rv;
        k[(i >> 2) * 64 + (i & 3)] = kv;
    }
    __device__ __forceinline__ void set_rec(int i, uint32_t rv) { r[(i >> 2) * 64 + (i & 3)] = rv; }
};

#if RT_DRAIN_STRONG_FENCE  // (study build: the hand-off's ordering made explicit)
#define RT_DRAIN_FENCE()                                       \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); \
        __builtin_amdgcn_s_waitcnt(0);                         \
        __builtin_amdgcn_wave_barrier();                       \
    } while (0)
#else
#define RT_DRAIN_FENCE()                                       \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                       \
    } while (0)
#endif
#ifndef RT_DRAIN_ROWS
#define RT_DRAIN_ROWS 3  // k_trace: once a wave's stream is out and at most this many quads still walk,
                         // their walks continue as rows (rt_row.h); 0 = off. cfg4 8-way shard, one
                         // MI355X (profiles/r04i_drain_probe.json, r04j_probe.json): off / 4 / 3 / 2 / 1 ->
                         // 370-373 / 362.6-362.9 / 359.9-361.4 / 360.5-363.6 / 366.5-367.3 ms, cfg2 148.0 /
                         // 145.3-145.9 / 145.1-145.4 / 145.6-146.0 / 147.1-147.6 ms
#endif

// k_trace's fast roles with per-quad refill (RT_TRACE_REFILL > 0): see k_trace.
// G = lanes per query: 4 (quads over the 4-wide BVH, rt_quad.h) or 16 (rows over the 16-wide
// BVH, rt_row.h). With quads, the drain (the wave's stream out, its last long walks running
// while the other quads idle) continues those walks as rows: same items, same stack entries
// (the 16-wide BVH is numbered like the 4-wide one), half the trips per remaining level.
template <bool ANY, bool STATS, bool PAIR, int G, class QSTK>
__device__ __forceinline__ void trace_stream(const rtk::WaveView& W, const RtSceneView& S, QSTK& stk, const int* s_pre,
                                             int first, int total, int wg, int wn, int32_t* fbn, rtk::RayRec* fbl,
                                             rtk::Stats* ps, const QPrefetch& pf)
{
    static_assert(G == 4 || G == 16, "quads or rows");
    constexpr unsigned long long ALL_IDLE = G == 4 ? 0x1111111111111111ull : 0x0001000100010001ull;
    constexpr int REFILL = G == 4 ? RT_TRACE_REFILL : 1;  // idle groups that trigger a refill
    const int lane = lane_id(), qd = lane / G;
    int sub = lane & (G - 1);
    int cursor = 0;                     // the wave's next stream position (uniform)
    bool exhausted = wg * 16 >= total;  // (uniform)
    bool active = false;
    uint32_t target = 0;
    rtk::QState q;  // (its ray is the query's: a fallback record is rebuilt from q.o, q.d and target)
#if RT_TRACE_PREFETCH
    if (!exhausted) queue_prefetch(W, s_pre, pf, first, cursor, wg, wn, total);
#endif
    // a walk's end: its answer, or the exact walk's list; gs = lanes of the group walking it
    auto finish = [&](int res, int gs) {
        // a long walk: the path's next rays go to the heavy class (head of the next streams)
        // (q.calls counts quad_visit calls; a row call covers two 4-wide levels and counts 2)
        if (W.r_heavy && sub == 0 && q.calls >= W.heavy_calls) W.r_heavy[target >> 3] = 1;
        if (STATS && W.iterq && sub == 0 && W.iter < RT_MAX_TIMED_ITERS) {
            // (RT_ITER_LOG: the launch's longest walk in quad_visit calls per role, and
            // how many walks took more than 8)
            int32_t* q2 = W.iterq + 2 * RT_MAX_TIMED_ITERS + 4 * W.iter;
            atomicMax(q2 + (ANY ? 1 : 0), q.calls);
            if (q.calls > 8) atomicAdd(q2 + 2, 1);
        }
        float t = 0.0f;
        int k = 0;
        int why = res < 0 ? 3 : 0;  // (walk log: why the exact walk answers: 1 tie, 2 chain check, 3 stack overflow)
        // (rows: each quad of the row verifies alike; one counts)
        if (res > 0 && !ANY && !rtk::quad_closest_answer(S, q, sub & 3, t, k, gs == 4 || sub == 0 ? ps : nullptr)) {
            res = -1;
            why = q.h.tie ? 1 : 2;
        }
        if (STATS && W.wlog && sub == 0 && q.calls >= W.wlog_min)
            walk_log(W, q.o, q.d, target, q.calls, res <= 0 ? -2.0f : ANY ? (float)(q.h.k == 1) : t, res <= 0 ? why : k,
                     gs == 4 ? 0 : 1);
        if (sub == 0) {
            if (res > 0) {
                if (ANY)
                    rtk::finish_any(W, target, q.h.k == 1);
                else
                    rtk::finish_closest(W, target, q.o, q.d, t, k);
            } else {  // the exact walk answers it (k_step(i)); the queue record again (o.w: slot)
                fbl[atomicAdd(fbn, 1)] = rtk::RayRec{rtk::f4(q.o, rt_asfloat(target >> 3)),
                                                     rtk::f4(q.d, rt_asfloat(target & 7u))};
                RT_DBG(ANY ? 2 : 0);
                RT_DBG(why == 3 ? 3 : why == 1 ? 4 : 5);
                if (gs == 16) RT_DBG(6);
                atomicAdd(&W.r_park[target >> 3], 1);
                if (STATS && W.iterq && W.iter < RT_MAX_TIMED_ITERS)
                    atomicAdd(W.iterq + 2 * RT_MAX_TIMED_ITERS + 4 * W.iter + 3, 1);  // (RT_ITER_LOG: fallbacks)
            }
        }
    };
    for (;;) {
        const unsigned long long bidle = __ballot(!active && sub == 0);
        if (!exhausted && (__popcll(bidle) >= REFILL || bidle == ALL_IDLE)) {
            if (!active) {
                const int j = cursor + __popcll(bidle & ((1ull << (qd * G)) - 1ull));  // this group's stream position
                const int idx = (wg + (j >> 4) * wn) * 16 + (j & 15);
                if (idx < total) {
#if RT_TRACE_PREFETCH
                    const int slot = j - cursor;  // (0..15: the buffer starts at the cursor)
                    // (the compiler does not order LDS reads after direct-to-LDS loads: wait for
                    // the vector-memory counter here, vmcnt(0), before reading the buffer)
                    __builtin_amdgcn_s_waitcnt(0x0F70);
                    rtk::RayRec r;
                    r.o = pf.buf[2 * slot];
                    r.d = pf.buf[2 * slot + 1];
                    const int kind = pf.kind[slot];
#else
                    int kind;
                    rtk::RayRec r = queue_item_at(W, s_pre, first + idx, kind);
#endif
                    target = (rt_asuint(r.o.w) << 3) | (uint32_t)kind;
                    if (forced_fallback(W, r.o, r.d)) {
                        if (sub == 0) {
                            r.d.w = rt_asfloat(target & 7u);
                            fbl[atomicAdd(fbn, 1)] = r;
                            atomicAdd(&W.r_park[target >> 3], 1);
                        }
                    } else if (rtk::qstate_begin<ANY>(q, rtk::v3of(r.o), rtk::v3of(r.d), sub, ps)) {
                        active = true;
                        q.calls = 0;
                    } else if (sub == 0) {  // (a NaN ray: no hit)
                        if (ANY)
                            rtk::finish_any(W, target, false);
                        else
                            rtk::finish_closest(W, target, q.o, q.d, -1.0f, -1);
                    }
                }
            }
            cursor += __popcll(bidle);
            exhausted = (wg + (cursor >> 4) * wn) * 16 >= total;
#if RT_TRACE_PREFETCH
            // (every lane has read its record: the buffer is free for the next 16 positions)
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (!exhausted) queue_prefetch(W, s_pre, pf, first, cursor, wg, wn, total);
#endif
            if (STATS && lane == 0) ps->c[RT_STAT_REFILLS]++;
        }
        const unsigned long long bact = __ballot(active && sub == 0);
        if (!bact) {
            if (exhausted) break;
            continue;
        }
        if (G == 4 && W.drain_rows > 0 && exhausted && __popcll(bact) <= W.drain_rows) break;  // to rows (below)
        if (STATS) {  // SIMT slots of this trip: 16 quads, the active ones used
            if (active && sub == 0) ps->c[exhausted ? RT_STAT_DRAIN_VISITS : RT_STAT_QUAD_VISITS]++;
            if (lane == 0) ps->c[exhausted ? RT_STAT_DRAIN_SLOTS : RT_STAT_WAVE_SLOTS] += 64 / G;
        }
        if (active) {
            int res;
            if constexpr (G == 4)
                res = rtk::quad_visit<ANY, RT_VISIT_DESCEND, PAIR>(S, q, stk, sub, ps);
            else
                res = rtk::row_visit<ANY, RT_VISIT_DESCEND>(S, q, stk, sub, ps);
            q.calls += G == 4 ? 1 : 2;
            if (res != 0) {
                active = false;
                finish(res, G);
            }
        }
    }
    if constexpr (G == 4) {
        // The drain as rows: the k-th walking quad of the wave (lane order) continues on row k.
        const unsigned long long bact = __ballot(active && sub == 0);
        if (!bact) return;
        const int row = lane >> 4;
        unsigned long long m = bact;
        for (int i = 0; i < row; i++) m &= m - 1ull;
#ifndef RT_DRAIN_SRC_LANE
#define RT_DRAIN_SRC_LANE 0  // (study: which lane of the walking quad hands its state to the row)
#endif
        const int src = (m ? __ffsll((long long)m) - 1 : 0) + RT_DRAIN_SRC_LANE;  // the walking quad's lane
        const bool ract = m != 0;
        // its state (quad-uniform) to the row's lanes
        auto pf = [&](float v) { return __shfl(v, src); };
        auto pi = [&](int v) { return __shfl(v, src); };
        q.o = rtk::v3(pf(q.o.x), pf(q.o.y), pf(q.o.z));
        q.d = rtk::v3(pf(q.d.x), pf(q.d.y), pf(q.d.z));
        for (int i = 0; i < 3; i++) q.rb.inv[i] = pf(q.rb.inv[i]), q.rb.oi[i] = pf(q.rb.oi[i]);
        q.h.t = pf(q.h.t), q.h.t2 = pf(q.h.t2), q.h.k = pi(q.h.k), q.h.leaf = pi(q.h.leaf), q.h.prim = pi(q.h.prim);
        q.h.tie = pi(q.h.tie ? 1 : 0) != 0, q.h.ovf = pi(q.h.ovf ? 1 : 0) != 0;
        q.sp = pi(q.sp), q.cur = pi(q.cur), q.calls = pi(q.calls);
        target = (uint32_t)pi((int)target);
        // its stack (<= RT_QSTACK entries), through registers: read everything, then write
        sub = lane & 15;
        const int wq = (int)(threadIdx.x >> 6) * 16;  // the wave's first quad in the block
        uint32_t* qr = stk.r - (threadIdx.x >> 2) + wq;  // word of the wave's quad 0, depth 0
        float* qk = stk.k - (threadIdx.x >> 2) + wq;
        const int sq = src >> 2;
        uint32_t r0 = 0, r1 = 0;
        float k0 = 0.0f, k1 = 0.0f;
        if (ract && sub < q.sp) r0 = qr[sub * 64 + sq], k0 = qk[sub * 64 + sq];
        if (ract && sub + 16 < q.sp) r1 = qr[(sub + 16) * 64 + sq], k1 = qk[(sub + 16) * 64 + sq];
        RT_DRAIN_FENCE();
        RowInQuadStack rs{qr + 4 * row, qk + 4 * row};
        if (ract && sub < q.sp) rs.set(sub, r0, k0);
        if (ract && sub + 16 < q.sp) rs.set(sub + 16, r1, k1);
        RT_DRAIN_FENCE();
        active = ract;
#if RT_DRAIN_RESTART == 1  // (study build: the row walk restarts at the root, the quad's stack dropped)
        q.sp = 0;
        if (q.cur != 0x7fffffff) q.cur = 0;
#elif RT_DRAIN_RESTART == 2  // (study build: a new walk of the same ray, nothing of the quad's kept)
        if (ract) rtk::qstate_begin<ANY>(q, q.o, q.d, sub, nullptr);
#elif RT_DRAIN_RESTART == 3  // (study build: the ray's box-test form recomputed from o and d)
        q.rb = rtk::rayb_setup(q.o, q.d);
#elif RT_DRAIN_RESTART == 4  // (study build: the walk's hit record reset; the walk goes on from its stack)
        q.h.t = __builtin_inff(), q.h.t2 = __builtin_inff(), q.h.k = ANY ? 0 : -1, q.h.leaf = -1;
        q.h.prim = 0x7fffffff, q.h.tie = false, q.h.ovf = false;
        q.sp = 0;
        if (q.cur != 0x7fffffff) q.cur = 0;
#endif
        while (__any(active)) {
            if (STATS) {
                if (active && sub == 0) ps->c[RT_STAT_DRAIN_VISITS]++;
                if (lane == 0) ps->c[RT_STAT_DRAIN_SLOTS] += 4;
            }
            if (active) {
                const int res = rtk::row_visit<ANY, RT_VISIT_DESCEND>(S, q, rs, sub, ps);
                q.calls += 2;
                if (res != 0) {
                    active = false;
                    finish(res, 16);
                }
            }
        }
    }
}

template <bool STATS, bool PAIR = true, int G = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TRACE_OCC, 8))) void k_trace(rtk::WaveView W, int par, unsigned long long* stats)
{
    __shared__ uint32_t s_lds[RT_LDS_WORDS * 256];
    __shared__ int s_pre[RT_NSEG + 1];
    __shared__ float4_ s_qbuf[RT_TRACE_PREFETCH ? 4 : 1][64];  // per wave: the next 16 stream records (queue_prefetch)
    __shared__ int s_qkind[RT_TRACE_PREFETCH ? 4 : 1][16];
    const QPrefetch pf{s_qbuf[RT_TRACE_PREFETCH ? threadIdx.x >> 6 : 0], s_qkind[RT_TRACE_PREFETCH ? threadIdx.x >> 6 : 0]};
    int32_t* cnt = W.counters;
    if (blockIdx.x == 0) {  // filled by k_step(i) next
        for (int j = threadIdx.x; j < (rtk::RK_COUNT + 1) * RT_QSHARDS; j += blockDim.x)
            cnt[j < rtk::RK_COUNT * RT_QSHARDS ? qc_at(par ^ 1, j / RT_QSHARDS, j % RT_QSHARDS)
                                                : ac_at(par ^ 1, j - rtk::RK_COUNT * RT_QSHARDS)] = 0;
        for (int j = threadIdx.x; j < rtk::RK_COUNT * RT_HSHARDS; j += blockDim.x)
            cnt[hc_at(par ^ 1, j / RT_HSHARDS, j % RT_HSHARDS)] = 0;
        if (threadIdx.x == 0) {
            cnt[C_PARKC0 + par] = cnt[C_PARKA0 + par] = 0;
            cnt[C_TK_EXACT_C] = cnt[C_TK_EXACT_A] = 0;
        }
    }
    // release the paths whose exact walks k_step(i - 1) finished
    {
        const int nd = cnt[C_DONE0 + (par ^ 1)];
        for (int j = (int)(blockIdx.x * blockDim.x + threadIdx.x); j < nd; j += (int)(gridDim.x * blockDim.x))
            atomicSub(&W.r_park[W.done[par ^ 1][j]], 1);
    }
    rtk::Stats st;
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++) st.c[i] = 0;
    rtk::Stats* ps = STATS ? &st : nullptr;
    const int b = (int)blockIdx.x;

    const RtSceneView S = W.S;
    // fast roles: a quad of lanes per query (rt_quad.h), or a row of 16 (rt_row.h)
    // queue segments in stream order (seg_id: each role's heavy class first): prefix table in LDS
    shard_prefix(cnt, RT_NSEG, [&](int j) { return seg_counter(par, j); }, s_pre);
    // without occlusion walks (analytic spheres) every kind is a closest-hit query
    const int c0 = 0, a0 = s_pre[RT_SEG_AH];
    const int nc = (W.any_rays ? a0 : s_pre[RT_SEG_END]) - c0;
    const int na = W.any_rays ? s_pre[RT_SEG_END] - a0 : 0;
    if (STATS && W.iterq && b == 0 && threadIdx.x == 0 && W.iter < RT_MAX_TIMED_ITERS) W.iterq[2 * W.iter] = nc + na;
    const int fb0 = 0, nbf = (int)gridDim.x;
    const int nbc = split_blocks(nbf, nc, na);
    const bool closest = b - fb0 < nbc;
    const int rb = closest ? b - fb0 : b - fb0 - nbc;                       // block index within the role
    const int rnb = closest ? nbc : nbf - nbc;                              // blocks of the role
    const int wg = rb * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);  // wave index within the role
    const int wn = rnb * (int)(blockDim.x >> 6);
    const int total = closest ? nc : na;
    int32_t* fbn = cnt + (closest ? C_FBC0 : C_FBA0) + par;  // walked exactly by k_step(i)
    rtk::RayRec* fbl = closest ? W.fb_c[par] : W.fb_a[par];
    // The wave's queries are a stream (its 16-query chunks base = wg*16 + c*wn*16 in turn):
    // each quad walks one, one trip per loop (rt_quad.h quad_visit), and as soon as
    // RT_TRACE_REFILL quads are idle they all take the next queries, so a long walk holds
    // up its own quad, not the wave's next 15 queries.
    if constexpr (G == 4) {
        rtk::QuadStack<RT_QSTACK, 64> stk{s_lds + (threadIdx.x >> 2), (float*)s_lds + RT_QSTACK * 64 + (threadIdx.x >> 2)};
        if (closest)
            trace_stream<false, STATS, PAIR, 4>(W, S, stk, s_pre, c0, total, wg, wn, fbn, fbl, ps, pf);
        else
            trace_stream<true, STATS, PAIR, 4>(W, S, stk, s_pre, a0, total, wg, wn, fbn, fbl, ps, pf);
    } else {
        static_assert(2 * RT_RSTACK * 16 <= RT_LDS_WORDS * 256, "row stacks fit k_trace's LDS");
        rtk::QuadStack<RT_RSTACK, 16> stk{s_lds + (threadIdx.x >> 4), (float*)s_lds + RT_RSTACK * 16 + (threadIdx.x >> 4)};
        if (closest)
            trace_stream<false, STATS, PAIR, 16>(W, S, stk, s_pre, c0, total, wg, wn, fbn, fbl, ps, pf);
        else
            trace_stream<true, STATS, PAIR, 16>(W, S, stk, s_pre, a0, total, wg, wn, fbn, fbl, ps, pf);
    }
    flush_stats<STATS>(st, stats);
}

// ------------------------------------------------------------- tail kernel
// When few paths are left (the last pixels of a frame are the ones whose
// samples bounce the most), an iteration costs its slowest query plus its
// slowest step no matter how few paths it carries, and a pixel's 64 x
// (bounces + 1) steps are a chain: the frame end is set by that chain. The
// tail kernel takes the remaining paths in one launch and lets each wave run
// its own: up to W.tail_paths paths per wave (lanes 0..P-1), step them, trace
// the rays they emitted from an LDS list with quads, repeat; a wave whose path
// finishes takes the next one from the live list. No grid-wide step, no
// launches: each path runs at its own pace.
// Entry condition (run_wave): no query is parked or waiting for the exact
// walk, so every path is ready to step; a query the quad walk cannot answer
// is answered here by the exact walk, inline, by lane 0 of its quad.
#define RT_TAIL_MAXP 16  // paths per wave at most (RK_COUNT rays each per list)
#ifndef RT_TAIL_EMIT_LDS
#define RT_TAIL_EMIT_LDS RT_STEP_EMIT_LDS
#endif
#if RT_TAIL_EMIT_LDS
// k_tail: a path's emitted rays stay in the wave's LDS columns (EmitLds<RT_TAIL_MAXP>, lane j
// of the wave's paths in column j); the lists hold (j << 3 | kind) (l0: closest-hit kinds,
// l1: occlusion)
using TailEmit = rtk::EmitLds<RT_TAIL_MAXP>;
__device__ __forceinline__ void tail_lists(const TailEmit& e, int last_kind, uint8_t* l0, uint8_t* l1, int* nl)
{
    const int lane = lane_id();
    nl[0] = nl[1] = 0;
#pragma unroll
    for (int k = 0; k < rtk::RK_COUNT; k++) {
        const bool want = (e.mask >> k) & 1u;
        const unsigned long long b = __ballot(want);
        const int l = k <= last_kind ? 0 : 1;
        if (want) (l ? l1 : l0)[nl[l] + __popcll(b & ((1ull << lane) - 1ull))] = (uint8_t)((lane << 3) | k);
        nl[l] += __popcll(b);
    }
}
// k_tail's path step (lanes with my >= 0) and list append, out of line (its registers apart
// from the walk loop's; inlined, the tail loop spilled across every step: cfg2 811 -> 828
// Msamples/s, cfg4 8-way shard 436 -> 403 ms, r02): bit 0 the lane's path stays in
// flight, bits 1-10 / 11- the closest / occlusion list lengths.
__device__ __noinline__ int tail_step(const rtk::WaveView& W, int my, int last_kind, float* cols, uint8_t* l0, uint8_t* l1,
                                      rtk::Stats* ps)
{
    TailEmit e;
    e.s = cols + (lane_id() & (RT_TAIL_MAXP - 1));  // (lanes >= W.tail_paths never step)
    e.mask = 0;
    e.active = false;
    e.heavy = false;
    if (my >= 0) rtk::path_step(W, my, e, ps);
    int nl[2];
    tail_lists(e, last_kind, l0, l1, nl);
    return (e.active ? 1 : 0) | (nl[0] << 1) | (nl[1] << 11);
}
#else
// k_tail: a path's emitted rays -> the wave's LDS lists (l0: closest-hit kinds, l1: occlusion)
__device__ __forceinline__ void tail_lists(const rtk::Emit& e, int slot, int last_kind, rtk::RayRec* l0, rtk::RayRec* l1,
                                           int* nl)
{
    const int lane = lane_id();
    nl[0] = nl[1] = 0;
#pragma unroll
    for (int k = 0; k < rtk::RK_COUNT; k++) {
        const bool want = (e.mask >> k) & 1u;
        const unsigned long long b = __ballot(want);
        const int l = k <= last_kind ? 0 : 1;
        if (want) {
            const int pos = nl[l] + __popcll(b & ((1ull << lane) - 1ull));
            (l ? l1 : l0)[pos] = e.rec(k, slot, rt_asfloat(((uint32_t)slot << 3) | (uint32_t)k));
        }
        nl[l] += __popcll(b);
    }
}
// (as above, the rays in registers and the lists of whole records)
__device__ __noinline__ int tail_step(const rtk::WaveView& W, int my, int last_kind, rtk::RayRec* l0, rtk::RayRec* l1,
                                      rtk::Stats* ps)
{
    rtk::Emit e;
    e.mask = 0;
    e.active = false;
    e.heavy = false;
    if (my >= 0) rtk::path_step(W, my, e, ps);
    int nl[2];
    tail_lists(e, my, last_kind, l0, l1, nl);
    return (e.active ? 1 : 0) | (nl[0] << 1) | (nl[1] << 11);
}
#endif
// k_tail's inline exact walk (a query the quad walk cannot settle: ~1e-6 of them), kept
// out of line so that its registers do not add to the tail loop's: inlined, k_tail
// needed 468 VGPR spill slots at its 168-VGPR budget, out of line ~190.
template <class XS>
__device__ __noinline__ void tail_exact(const rtk::WaveView& W, int l, uint32_t target, rtk::V3 o, rtk::V3 d, XS& xs,
                                        rtk::Stats* ps)
{
    if (l == 0) {
        rtk::TravC T;
        if (rtk::travc_begin(W.S, T, o, d, ps))
            while (rtk::travc_step(W.S, T, xs, ps)) {
            }
        rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
    } else {
        rtk::TravA T;
        if (rtk::trava_begin(W.S, T, o, d, ps))
            while (rtk::trava_step(W.S, T, xs, ps)) {
            }
        rtk::finish_any(W, target, T.hit);  // (begin leaves the brute-force answer in T.hit)
    }
}
#ifndef RT_TAIL_DESCEND
#define RT_TAIL_DESCEND RT_VISIT_DESCEND  // inner-node trips per quad_visit call in k_tail
#endif
#ifndef RT_TAIL_OCC
#define RT_TAIL_OCC 3    // k_tail waves per SIMD (2: no spills but half the paths per launch; 3 measured faster)
#endif
// FAST: the fast lane's launch, one kernel over every lane's handed-over paths: blocks
// [fparts[l], fparts[l + 1]) step lane l's (fviews[l]: its fast list as shard 0 of its own
// counters, its own spill area).
template <bool STATS, bool PAIR, int G, bool FAST>
__device__ __forceinline__ void tail_body(const rtk::WaveView& W, int par, unsigned long long* stats, int blk)
{
#if RT_TAIL_EMIT_LDS
    __shared__ float s_em[4][6 * rtk::RK_COUNT * RT_TAIL_MAXP];        // per wave: its paths' rays (TailEmit columns)
    __shared__ uint8_t s_q[4][2][RT_TAIL_MAXP * rtk::RK_COUNT];        // per wave: closest list, occlusion list
    __shared__ int s_my[4][RT_TAIL_MAXP];                              // per wave: the slot of column j
#else
    __shared__ rtk::RayRec s_q[4][2][RT_TAIL_MAXP * rtk::RK_COUNT];  // per wave: closest list, occlusion list
#endif
    __shared__ uint32_t s_stk[2 * RT_QSTACK * 64];
    __shared__ int s_pre[RT_QSHARDS + 1];
    rtlibm::lds_tables_init();
    rtk::lds_shade_init(W.S);  // (the env-map row search and a small material table from LDS)
    int32_t* cnt = W.counters;
    shard_prefix(cnt, RT_QSHARDS, [&](int j) { return ac_at(par, j); }, s_pre);
    const int n = FAST ? min(s_pre[RT_QSHARDS], W.fast_cap) : s_pre[RT_QSHARDS];  // (fast lane: its list)
    const RtSceneView S = W.S;
    rtk::Stats st;
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++) st.c[i] = 0;
    rtk::Stats* ps = STATS ? &st : nullptr;
    // G lanes per query: quads (4-wide BVH) or rows (16-wide BVH, rt_row.h), each with its LDS stack
    static_assert(G == 4 || G == 16, "quads or rows");
    constexpr int SCAP = G == 4 ? RT_QSTACK : RT_RSTACK, GPB = 256 / G;
    static_assert(2 * SCAP * GPB <= 2 * RT_QSTACK * 64, "group stacks fit k_tail's LDS");
    const int wv = (int)(threadIdx.x >> 6), lane = lane_id(), sub = lane & (G - 1), qd = (int)(threadIdx.x / G);
    using STK = rtk::QuadStack<SCAP, GPB>;
    STK stk{s_stk + qd, (float*)s_stk + SCAP * GPB + qd};
    const size_t gl = (size_t)blk * blockDim.x + threadIdx.x;
    rtk::SpillStack<STK> xs{stk, W.spill_r + gl * RT_STACK_CAP, W.spill_k + gl * RT_STACK_CAP};
    const int P = W.tail_paths;
    const int last_kind = W.any_rays ? rtk::RK_CAM : rtk::RK_BENV;
    int my = -1;
    bool drained = false;
    int rounds = 0;  // (RT_ITER_LOG: the longest pool loop of the launch)
    long long tk_step = 0, tk_walk = 0;  // (RT_ITER_LOG: 100 MHz ticks in path_step / in the walks)
    long long tk_solo = 0;               // (RT_ITER_LOG: ... in walk trips with one group walking)
    int trips = 0, solo_trips = 0;
    const bool probe = STATS && W.iterq && W.iter + 1 < RT_MAX_TIMED_ITERS;
    for (;;) {
        // refill the wave's pool from the live list
        const bool need = lane < P && my < 0;
        const unsigned long long bneed = __ballot(need);
        if (bneed && !drained) {
            const int nneed = __popcll(bneed);
            int base = 0;
            if (lane == 0) base = atomicAdd(cnt + C_TK_TAIL, nneed);
            base = __shfl(base, 0);
            if (base + nneed >= n) drained = true;
            const int idx = base + __popcll(bneed & ((1ull << lane) - 1ull));
            if (need && idx < n) {
                const int sh = shard_find8<RT_QSHARDS>(s_pre, idx);
                my = W.act_in[(size_t)sh * W.seg_cap + (idx - s_pre[sh])];
                if (FAST) W.r_park[my] = 0;  // (k_hand's mark)
            }
        }
        if (!__any(my >= 0)) break;
        rounds++;
        // step; the emitted rays -> the wave's LDS lists
        const long long t0 = probe ? wall_clock64() : 0;
        int nl[2];
        {
#if RT_TAIL_EMIT_LDS
            if (lane < RT_TAIL_MAXP) s_my[wv][lane] = my;
            const int r = tail_step(W, my, last_kind, s_em[wv], s_q[wv][0], s_q[wv][1], ps);
#else
            const int r = tail_step(W, my, last_kind, s_q[wv][0], s_q[wv][1], ps);
#endif
            if (!(r & 1)) my = -1;
            nl[0] = (r >> 1) & 0x3ff;
            nl[1] = r >> 11;
        }
        long long t1 = 0;
        if (probe) {
            t1 = wall_clock64();
            tk_step += __shfl(t1, 0) - __shfl(t0, 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the lists are read by other lanes
        __builtin_amdgcn_wave_barrier();
        // trace: both lists in one index space, streamed over the wave's 16 quads (an idle
        // quad takes the next query at once), each quad walking its own kind a few trips
        // per call (rt_quad.h quad_visit): a step waits for its slowest query, not for
        // the slowest of every 16-query pass
        const int nq = nl[0] + nl[1];
        int next = 0;  // the next query of the lists (uniform)
        bool act = false;
        int l = 0;
        uint32_t target = 0;
        rtk::QState q;
        for (;;) {
            bool exact = false;
            const unsigned long long bidle = __ballot(!act && sub == 0);
            if (next < nq) {
                const int qi = next + __popcll(bidle & ((1ull << (lane & ~(G - 1))) - 1ull));  // this group's query
                if (!act && qi < nq) {
                    l = qi < nl[0] ? 0 : 1;
#if RT_TAIL_EMIT_LDS
                    const int ent = s_q[wv][l][l ? qi - nl[0] : qi], j = ent >> 3, kind = ent & 7;
                    TailEmit ce;
                    ce.s = s_em[wv] + j;
                    rtk::RayRec r;
                    r.o = rtk::f4(ce.o(kind), 0.0f);
                    r.d = rtk::f4(ce.d(kind), 0.0f);
                    target = ((uint32_t)s_my[wv][j] << 3) | (uint32_t)kind;
#else
                    const rtk::RayRec r = s_q[wv][l][l ? qi - nl[0] : qi];
                    target = rt_asuint(r.d.w);
#endif
                    q.o = rtk::v3of(r.o);
                    q.d = rtk::v3of(r.d);
                    if (forced_fallback(W, r.o, r.d)) {
                        exact = true;
                    } else {
                        act = l ? rtk::qstate_begin<true>(q, q.o, q.d, sub, ps) : rtk::qstate_begin<false>(q, q.o, q.d, sub, ps);
                        if (STATS) q.calls = 0;
                        if (!act && sub == 0) {  // (a NaN ray: no hit)
                            if (l == 0)
                                rtk::finish_closest(W, target, q.o, q.d, -1.0f, -1);
                            else
                                rtk::finish_any(W, target, false);
                        }
                    }
                }
                next = min(nq, next + __popcll(bidle));
            }
            long long ts = 0;
            bool solo = false;
            if (probe) {
                ts = wall_clock64();
                solo = __popcll(__ballot(act && sub == 0)) == 1;
            }
            if (act) {
                int res;
                if constexpr (G == 4)
                    res = l ? rtk::quad_visit<true, RT_TAIL_DESCEND, PAIR>(S, q, stk, sub, ps)
                            : rtk::quad_visit<false, RT_TAIL_DESCEND>(S, q, stk, sub, ps);
                else
                    res = l ? rtk::row_visit<true, RT_TAIL_DESCEND>(S, q, stk, sub, ps)
                            : rtk::row_visit<false, RT_TAIL_DESCEND>(S, q, stk, sub, ps);
                if (STATS) q.calls += G == 4 ? 1 : 2;
                if (res != 0) {
                    act = false;
                    float t = 0.0f;
                    int k = 0;
                    const bool ok = res > 0 && (l == 1 || rtk::quad_closest_answer(S, q, sub & 3, t, k,
                                                                                    G == 4 || sub == 0 ? ps : nullptr));
                    if (STATS && W.wlog && sub == 0 && q.calls >= W.wlog_min)
                        walk_log(W, q.o, q.d, target, q.calls, !ok ? -2.0f : l ? (float)(q.h.k == 1) : t, k, 2);
                    if (ok && sub == 0) {
                        if (l == 0)
                            rtk::finish_closest(W, target, q.o, q.d, t, k);
                        else
                            rtk::finish_any(W, target, q.h.k == 1);
                    }
                    exact = !ok;
                }
            }
            if (exact && sub == 0) {  // the exact octree walk, to completion
                if (STATS) st.c[RT_STAT_FALLBACK]++;
                xs.f = stk;
                tail_exact(W, l, target, q.o, q.d, xs, ps);
            }
            if (probe) {
                const long long te = wall_clock64();
                trips++;
                if (solo) {
                    solo_trips++;
                    tk_solo += __shfl(te, 0) - __shfl(ts, 0);
                }
            }
            if (next >= nq && !__any(act)) break;
        }
        if (probe) {
            const long long t2 = wall_clock64();
            tk_walk += __shfl(t2, 0) - __shfl(t1, 0);
        }
    }
    if (STATS && W.iterq && lane == 0 && W.iter < RT_MAX_TIMED_ITERS) atomicMax(W.iterq + 2 * W.iter + 1, rounds);
    if (probe && lane == 0) {
        atomicAdd(W.iterq + 2 * W.iter + 2, (int)(tk_step >> 4));
        atomicAdd(W.iterq + 2 * W.iter + 3, (int)(tk_walk >> 4));
        int32_t* q2 = W.iterq + 2 * RT_MAX_TIMED_ITERS + 4 * (W.iter + 1);  // (the tail row's last columns)
        atomicAdd(q2, (int)(tk_solo >> 4));
        atomicAdd(q2 + 1, trips);
        atomicAdd(q2 + 2, solo_trips);
    }
    flush_stats<STATS>(st, stats);
    flush_stats<STATS>(st, stats + RT_STAT_COUNT);  // (the tail kernel's share, for per-kernel byte counts)
}
template <bool STATS, bool PAIR = true, int G = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TAIL_OCC, RT_TAIL_OCC))) void k_tail(
    rtk::WaveView W, int par, unsigned long long* stats)
{
    tail_body<STATS, PAIR, G, false>(W, par, stats, (int)blockIdx.x);
}
template <bool STATS, bool PAIR = true, int G = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TAIL_OCC, RT_TAIL_OCC))) void k_tail_fast(
    const rtk::WaveView* __restrict__ fviews, int4 fparts, unsigned long long* stats)
{
    const int b = (int)blockIdx.x;
    const int fl = (b >= fparts.y) + (b >= fparts.z) + (b >= fparts.w);
    const int b0 = fl == 0 ? 0 : fl == 1 ? fparts.y : fl == 2 ? fparts.z : fparts.w;
    tail_body<STATS, PAIR, G, true>(fviews[fl], 0, stats, b - b0);
}

__global__ __launch_bounds__(256) void k_intersect(RtSceneView S, const float* __restrict__ rays, int32_t* __restrict__ out,
                                                   int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    rtk::StackEnt stack[RT_STACK_CAP];
    const float* r = rays + 6 * (size_t)i;
    const rtk::V3 o = rtk::v3(r[0], r[1], r[2]), d = rtk::v3(r[3], r[4], r[5]);
    float t;
    int k;
    rtk::query_closest(S, o, d, stack, t, k, nullptr);
    rtk::Hit h;
    const bool f = rtk::hit_from(S, o, d, t, k, h);
    int32_t* ot = out + 11 * (size_t)i;
    ot[0] = f ? 1 : 0;
    ot[1] = h.prim;
    ot[2] = (int32_t)rt_asuint(t);
    const bool any = t != -1.0f;
    ot[3] = any ? (int32_t)rt_asuint(h.p.x) : 0;
    ot[4] = any ? (int32_t)rt_asuint(h.p.y) : 0;
    ot[5] = any ? (int32_t)rt_asuint(h.p.z) : 0;
    ot[6] = any ? (int32_t)rt_asuint(h.n.x) : 0;
    ot[7] = any ? (int32_t)rt_asuint(h.n.y) : 0;
    ot[8] = any ? (int32_t)rt_asuint(h.n.z) : 0;
    ot[9] = (int32_t)rt_asuint(-1.0f);
    ot[10] = (int32_t)rt_asuint(-1.0f);
}

// Search-BVH query micro-benchmark (tools/query_bench.py): one query per
// lane, the k_trace stack layout. out_t = t (closest) or 0/1 (any), -2 when
// the query needs the exact walk.
template <bool ANY, int WALK>
__global__ __launch_bounds__(256, 4) void k_query(RtSceneView S, const float4_* __restrict__ rays,
                                                  float* __restrict__ out_t, int* __restrict__ out_k, int n,
                                                  uint32_t* spill_r, float* spill_k)
{
    __shared__ uint32_t s_lds[2 * RT_LDS_CAP_FAST * 256];
    const size_t gl = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    FastStack<RT_LDS_CAP_FAST, RT_SPILL_FAST> stk{s_lds + threadIdx.x, (float*)s_lds + RT_LDS_CAP_FAST * 256 + threadIdx.x,
                                                  spill_r + gl * RT_SPILL_FAST, spill_k + gl * RT_SPILL_FAST};
    const int stride = (int)(gridDim.x * blockDim.x);
    for (int i = (int)gl; i < n; i += stride) {
        const rtk::V3 o = rtk::v3of(rays[2 * i]), d = rtk::v3of(rays[2 * i + 1]);
        if (ANY) {
            const int a = rtk::fast_query_any<decltype(stk), WALK>(S, o, d, stk, nullptr);
            out_t[i] = a < 0 ? -2.0f : (float)a;
            out_k[i] = 0;
        } else {
            float t = 0;
            int k = 0;
            const bool ok = rtk::fast_query_closest<decltype(stk), WALK>(S, o, d, stk, t, k, nullptr);
            out_t[i] = ok ? t : -2.0f;
            out_k[i] = ok ? (k >= 0 ? (int)rt_asuint(S.tri4[3 * (size_t)k].w) : -1) : -2;  // (the original triangle index)
        }
    }
}

// The same through the product's quad walks (rt_quad.h quad_visit, k_trace's per-trip
// code and answer): four lanes per query.
template <bool ANY, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_query_quad(RtSceneView S, const float4_* __restrict__ rays,
                                                    float* __restrict__ out_t, int* __restrict__ out_k, int n)
{
    __shared__ uint32_t s_lds[2 * RT_QSTACK * 64];
    const int q = (int)(threadIdx.x >> 2), sub = (int)(threadIdx.x & 3);
    rtk::QuadStack<RT_QSTACK, 64> stk{s_lds + q, (float*)s_lds + RT_QSTACK * 64 + q};
    const int stride = (int)(gridDim.x * blockDim.x) >> 2;
    for (int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 2); i < n; i += stride) {
        rtk::QState qs;
        int res = 1;
        if (rtk::far_origin(S, rtk::v3of(rays[2 * i])))
            res = -1;  // (the exact walk's)
        else if (rtk::qstate_begin<ANY>(qs, rtk::v3of(rays[2 * i]), rtk::v3of(rays[2 * i + 1]), sub, nullptr))
            do {
                res = rtk::quad_visit<ANY>(S, qs, stk, sub, nullptr);
            } while (res == 0);
        float t = -1.0f;
        int k = -1;
        const bool ok = res > 0 && (ANY || rtk::quad_closest_answer(S, qs, sub, t, k, nullptr));
        if (sub == 0) {
            if (ANY) {
                out_t[i] = ok ? (float)(qs.h.k == 1 ? 1 : 0) : -2.0f;
                out_k[i] = 0;
            } else {
                out_t[i] = ok ? t : -2.0f;
                out_k[i] = ok ? (k >= 0 ? (int)rt_asuint(S.tri4[3 * (size_t)k].w) : -1) : -2;  // (the original triangle index)
            }
        }
    }
}

// The same through the row walks (rt_row.h row_visit over the 16-wide BVH): 16 lanes per query.
template <bool ANY>
__global__ __launch_bounds__(256) void k_query_row(RtSceneView S, const float4_* __restrict__ rays,
                                                   float* __restrict__ out_t, int* __restrict__ out_k, int n)
{
    __shared__ uint32_t s_lds[2 * RT_RSTACK * 16];
    const int r = (int)(threadIdx.x >> 4), sub = (int)(threadIdx.x & 15);
    rtk::QuadStack<RT_RSTACK, 16> stk{s_lds + r, (float*)s_lds + RT_RSTACK * 16 + r};
    const int stride = (int)(gridDim.x * blockDim.x) >> 4;
    for (int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4); i < n; i += stride) {
        rtk::QState qs;
        int res = 1;
        if (rtk::far_origin(S, rtk::v3of(rays[2 * i])))
            res = -1;  // (the exact walk's)
        else if (rtk::qstate_begin<ANY>(qs, rtk::v3of(rays[2 * i]), rtk::v3of(rays[2 * i + 1]), sub, nullptr))
            do {
                res = rtk::row_visit<ANY, RT_VISIT_DESCEND>(S, qs, stk, sub, nullptr);
            } while (res == 0);
        float t = -1.0f;
        int k = -1;
        const bool ok = res > 0 && (ANY || rtk::quad_closest_answer(S, qs, sub & 3, t, k, nullptr));
        if (sub == 0) {
            if (ANY) {
                out_t[i] = ok ? (float)(qs.h.k == 1 ? 1 : 0) : -2.0f;
                out_k[i] = 0;
            } else {
                out_t[i] = ok ? t : -2.0f;
                out_k[i] = ok ? (k >= 0 ? (int)rt_asuint(S.tri4[3 * (size_t)k].w) : -1) : -2;  // (the original triangle index)
            }
        }
    }
}

// numerics self-test kernel (tests/test_gpu_parity.py): out[i] = f(in[i])
__global__ void k_libm(int fn, const float* __restrict__ in, const float* __restrict__ in2, float* __restrict__ out, int n)
{
    rtlibm::lds_tables_init();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[i];
    float r;
    switch (fn) {
        case 0: r = rt_expf(x); break;
        case 1: r = rt_powf(x, in2[i]); break;
        case 2: r = rt_sinf(x); break;
        case 3: r = rt_cosf(x); break;
        case 4: r = rt_acosf(x); break;
        case 5: r = rt_asinf(x); break;
        case 6: r = rt_atan2f(x, in2[i]); break;
        case 7: r = rt_sqrtf(x); break;
        case 8: r = x / in2[i]; break;
        case 9: r = (float)((double)x * 0.31830988618379067154 / (double)in2[i]); break;
        default: r = rtk::slab_div(x, 1.0 / (double)in2[i]); break;  // the slab quotient
    }
    out[i] = r;
}

// ------------------------------------------------------------- wave memory
}  // namespace

// ------------------------------------------------------------------- hooks
namespace {
// A context drives one Backend per device. rt_create: one device, renders on the
// caller's stream. rt_create_multi: devices[0] is the root that holds the caller's
// framebuffer; a render shards its rows over the devices (render_multi).
struct Group {
    std::vector<Backend*> dev;     // dev[0]: the root
    bool multi = false;            // rt_create_multi over two or more devices
    bool loopback = false;         // (RT_MULTI_LOOPBACK test contexts) shards exchanged by device copies
    std::vector<ncclComm_t> comms; // ncclCommInitAll over the devices, in order (RCCL exchange)
    DevBuf stage;                  // root: N blocks of rows_max rows (scatter source / gather target)
    std::vector<DevBuf> shard;     // device d >= 1: its block
};

Group* grp(rt_context* c) { return (Group*)c->backend; }
Backend* be(rt_context* c) { return grp(c)->dev[0]; }

// RCCL, loaded on the first multi-device context: the library need not be present
// (or be the same build as a framework's own copy) for single-device use.
struct Rccl {
    void* h = nullptr;
    decltype(&ncclCommInitAll) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclScatter) scatter = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
};
std::mutex g_rccl_mu;
Rccl g_rccl;

const Rccl* rccl_load(std::string& err)
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.h) return &g_rccl;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        err = std::string("librt_hip: RCCL not found (librccl.so.1): ") + dlerror();
        return nullptr;
    }
    Rccl r;
    r.h = h;
    r.init = (decltype(r.init))dlsym(h, "ncclCommInitAll");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.scatter = (decltype(r.scatter))dlsym(h, "ncclScatter");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.errstr = (decltype(r.errstr))dlsym(h, "ncclGetErrorString");
    if (!r.init || !r.destroy || !r.scatter || !r.gather || !r.group_start || !r.group_end || !r.errstr) {
        err = "librt_hip: librccl.so.1 lacks ncclCommInitAll / ncclScatter / ncclGather";
        return nullptr;
    }
    g_rccl = r;
    return &g_rccl;
}

#define NCCLCHK(ctx, R, expr)                                                                    \
    do {                                                                                         \
        ncclResult_t e_ = (expr);                                                                \
        if (e_ != ncclSuccess) return rt_fail(ctx, RT_ERR_HIP, std::string(#expr ": ") + (R)->errstr(e_)); \
    } while (0)

int create_one(rt_context* c, int device, Backend** out)
{
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return rt_fail(c, RT_ERR_NODEV, "librt_hip: no HIP device available (this library has no CPU path)");
    if (device < 0 || device >= n) return rt_fail(c, RT_ERR_NODEV, "librt_hip: device index out of range");
    HIPCHK(c, hipSetDevice(device));
    Backend* b = new Backend();
    *out = b;
    b->device = device;
    HIPCHK(c, hipEventCreate(&b->ev0));
    HIPCHK(c, hipEventCreate(&b->ev1));
    for (int l = 0; l < RT_MAX_LANES; l++) {
        HIPCHK(c, hipHostMalloc((void**)&b->h_act[l], RT_QSHARDS * RT_CSTRIDE * 4 + 64, hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&b->ev_lane[l], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&b->ev_join[l], hipEventDisableTiming));
        if (l > 0) HIPCHK(c, hipStreamCreateWithFlags(&b->ls[l], hipStreamNonBlocking));
    }
    HIPCHK(c, hipStreamCreateWithFlags(&b->own, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming));
    return RT_OK;
}

void destroy_one(Backend* b)
{
    (void)hipSetDevice(b->device);
    (void)hipDeviceSynchronize();
    DevBuf* all[] = {&b->nodes, &b->tri4, &b->prim2k, &b->mat_idx, &b->mats, &b->emissive, &b->spheres, &b->env,
                     &b->env_lum, &b->cdf, &b->bvh4, &b->bvh16, &b->bvh4s, &b->bvh16s, &b->bvh_tri4, &b->parent, &b->leaf_of, &b->cdf_row, &b->cdf_coarse,
                     &b->cdf_fence, &b->matk, &b->stats, &b->xy, &b->fb, &b->iterq, &b->wlog, &b->fviews};
    for (DevBuf* d : all)
        if (d->p) (void)hipFree(d->p);
    for (int l = 0; l < RT_MAX_LANES; l++)
        for (DevBuf* d : {&b->wave[l], &b->counters[l], &b->fast[l], &b->fcnt[l], &b->fhist[l], &b->fspill[l]})
            if (d->p) (void)hipFree(d->p);
    for (int l = 0; l < RT_MAX_LANES; l++) {
        if (b->h_hist[l]) (void)hipHostFree(b->h_hist[l]);
        if (b->fev[l]) (void)hipEventDestroy(b->fev[l]);
        if (b->hev[l]) (void)hipEventDestroy(b->hev[l]);
    }
    if (b->h_fviews) (void)hipHostFree(b->h_fviews);
    if (b->fev_done) (void)hipEventDestroy(b->fev_done);
    if (b->fs) (void)hipStreamDestroy(b->fs);
    for (hipEvent_t e : b->ftev)
        if (e) (void)hipEventDestroy(e);
    for (int l = 0; l < RT_MAX_LANES; l++) {
        if (b->h_act[l]) (void)hipHostFree(b->h_act[l]);
        if (b->ev_lane[l]) (void)hipEventDestroy(b->ev_lane[l]);
        if (b->ev_join[l]) (void)hipEventDestroy(b->ev_join[l]);
        if (b->ls[l]) (void)hipStreamDestroy(b->ls[l]);
    }
    if (b->own) (void)hipStreamDestroy(b->own);
    if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
    if (b->ev_done) (void)hipEventDestroy(b->ev_done);
    for (auto& lane : b->tev)
        for (auto& row : lane)
            for (hipEvent_t ev : row)
                if (ev) (void)hipEventDestroy(ev);
    if (b->ev0) (void)hipEventDestroy(b->ev0);
    if (b->ev1) (void)hipEventDestroy(b->ev1);
    delete b;
}

// Scene, BVH and env of the context into one device's memory (replicated per device).
int upload_one(rt_context* c, Backend* b, const std::vector<int32_t>& matk, bool mats_only)
{
    HIPCHK(c, hipSetDevice(b->device));
    // the previous render may still run (rt_render_device returns at once, its kernels on
    // non-blocking streams that a null-stream copy does not wait for): it reads these tables
    if (b->done_recorded) HIPCHK(c, hipEventSynchronize(b->ev_done));
    int r = 0;
    if (mats_only) {  // rt_set_materials: the material table (and what depends on it) alone
        if ((r = upload(c, b->mats, c->mats))) return r;
        b->view.mats = (const RtMat*)b->mats.p;
        b->view.n_mats = (int)c->mats.size();
        b->bl_rays = rt_scene_has_emissive_prim(c) ? 1 : 0;
        return RT_OK;
    }
    // device triangle records carry the material index in e1.w (rt_wave.h hit_from)
    std::vector<float4_> tri4 = c->flat.tri4;
    for (size_t k = 0; k < matk.size(); k++) std::memcpy(&tri4[3 * k + 1].w, &matk[k], 4);
    if ((r = upload(c, b->nodes, c->flat.nodes)) || (r = upload(c, b->tri4, tri4)) ||
        (r = upload(c, b->prim2k, c->flat.prim2k)) || (r = upload(c, b->mat_idx, c->mat_idx)) ||
        (r = upload(c, b->mats, c->mats)) || (r = upload(c, b->emissive, c->emissive)) ||
        (r = upload(c, b->spheres, c->spheres)) || (r = upload(c, b->env, c->env)) ||
        (r = upload(c, b->env_lum, c->env_lum)) || (r = upload(c, b->cdf, c->cdf)) ||
        (r = upload(c, b->bvh4, c->flat.bvh4)) || (r = upload(c, b->bvh16, c->flat.bvh16)) ||
        (r = upload(c, b->bvh4s, c->flat.bvh4s)) || (r = upload(c, b->bvh16s, c->flat.bvh16s)) ||
        (r = upload(c, b->bvh_tri4, c->flat.bvh_tri4)) ||
        (r = upload(c, b->parent, c->flat.parent)) || (r = upload(c, b->leaf_of, c->flat.leaf_of)) ||
        (r = upload(c, b->cdf_row, c->cdf_row)) || (r = upload(c, b->cdf_coarse, c->cdf_coarse)) ||
        (r = upload(c, b->cdf_fence, c->cdf_fence)) || (r = upload(c, b->matk, matk)) ||
        (r = ensure(c, b->stats, 2 * RT_STAT_COUNT * sizeof(unsigned long long))))
        return r;
    for (int l = 0; l < RT_MAX_LANES; l++)
        if ((r = ensure(c, b->counters[l], C_COUNT * sizeof(int32_t)))) return r;
    RtSceneView v{};
    v.nodes = (const RtNode*)b->nodes.p;
    v.tri4 = (const float4_*)b->tri4.p;
    v.prim2k = (const int32_t*)b->prim2k.p;
    v.mat_idx = (const int32_t*)b->mat_idx.p;
    v.matk = (const int32_t*)b->matk.p;
    v.mats = (const RtMat*)b->mats.p;
    v.n_mats = (int)c->mats.size();
    v.emissive = (const int32_t*)b->emissive.p;
    v.spheres = (const float4_*)b->spheres.p;
    v.env = (const float4_*)b->env.p;
    v.env_lum = (const float*)b->env_lum.p;
    v.cdf = (const float*)b->cdf.p;
    v.cdf_row = (const float*)b->cdf_row.p;
    v.cdf_coarse = (const float*)b->cdf_coarse.p;
    v.cdf_fence = c->cdf_fence.empty() ? nullptr : (const float*)b->cdf_fence.p;
    v.cdf_cw = c->cdf_cw;
    v.cdf_total = c->cdf.empty() ? 0.0f : c->cdf.back();
    v.n_emissive = (int)c->emissive.size();
    v.n_spheres = (int)(c->spheres.size() / 2);
    v.ew = c->ew;
    v.eh = c->eh;
    v.n_tris = (int)(c->tris.size() / 9);
    v.chain_monotone = c->flat.chain_monotone ? 1 : 0;
    v.brute = c->brute ? 1 : 0;
    v.bvh4 = (const Bvh4Node*)b->bvh4.p;
    v.bvh16 = (const Bvh4Child*)b->bvh16.p;
    v.bvh4s = (const float4_*)b->bvh4s.p;
    v.bvh16s = (const float4_*)b->bvh16s.p;
    v.bvh_tri4 = (const float4_*)b->bvh_tri4.p;
    v.parent = (const int32_t*)b->parent.p;
    v.leaf_of = (const int32_t*)b->leaf_of.p;
    v.tri_mat = 1;
    rt_view_near(c, v);
    b->view = v;
    b->bl_rays = rt_scene_has_emissive_prim(c) ? 1 : 0;
    b->any_rays = v.n_spheres == 0 ? 1 : 0;
    return RT_OK;
}
}  // namespace

int rt_backend_create(rt_context* c)
{
    Group* g = new Group();
    c->backend = g;
    // (one listed device: a single-device context on it, unless a test asks for the driver
    // and a one-rank RCCL clique: rt_test_create_multi_rccl)
    g->multi = c->devices.size() > 1 || (c->force_multi && !c->devices.empty());
    g->loopback = g->multi && c->loopback;
    const std::vector<int> ids = g->multi ? c->devices : std::vector<int>{c->device};
    for (int d : ids) {
        Backend* b = nullptr;
        const int r = create_one(c, d, &b);
        if (b) {
            b->index = (int)g->dev.size();
            g->dev.push_back(b);
        }
        if (r) return r;
    }
    if (g->multi) g->shard.resize(ids.size());
    if (g->multi && !g->loopback) {
        std::string err;
        const Rccl* R = rccl_load(err);
        if (!R) return rt_fail(c, RT_ERR_NODEV, err);
        g->comms.resize(ids.size());
        NCCLCHK(c, R, R->init(g->comms.data(), (int)ids.size(), ids.data()));
    }
    return RT_OK;
}

void rt_backend_destroy(rt_context* c)
{
    Group* g = grp(c);
    if (!g) return;
    for (Backend* b : g->dev) destroy_one(b);
    if (!g->comms.empty()) {
        std::string err;
        if (const Rccl* R = rccl_load(err))
            for (ncclComm_t cm : g->comms)
                if (cm) (void)R->destroy(cm);
    }
    for (size_t d = 0; d < g->shard.size(); d++)
        if (g->shard[d].p) {
            (void)hipSetDevice(g->multi ? c->devices[d] : c->device);
            (void)hipFree(g->shard[d].p);
        }
    if (g->stage.p) {
        (void)hipSetDevice(g->multi ? c->devices[0] : c->device);
        (void)hipFree(g->stage.p);
    }
    delete g;
    c->backend = nullptr;
}

int rt_backend_upload(rt_context* c)
{
    Group* g = grp(c);
    const bool mats_only = c->mats_dirty_only && !c->dirty;
    // material index of each leaf-order triangle k: mat_idx[prim(k)] (rt_trace.h load_mat_hit)
    std::vector<int32_t> matk;
    if (!mats_only) {
        matk.resize(c->flat.tri4.size() / 3);
        for (size_t k = 0; k < matk.size(); k++) {
            int32_t prim;
            std::memcpy(&prim, &c->flat.tri4[3 * k].w, 4);
            matk[k] = c->mat_idx[prim];
        }
    }
    for (Backend* b : g->dev)
        if (int r = upload_one(c, b, matk, mats_only)) return r;
    return RT_OK;
}

namespace {
// One wavefront run over a subset of the launch's pixels (a "lane"): its own
// path slots, queues, counters and stream. run_wave drives RT_LANES lanes on
// as many streams (row j of the launch -> lane j % lanes) so that one lane's
// k_step and the tails of its launches overlap another lane's k_trace.
struct WaveLane {
    rtk::WaveView W{};
    int32_t* lists[2] = {nullptr, nullptr};
    int32_t* cnt = nullptr;
    int32_t* h = nullptr;  // pinned readback: ACT shard counts, then 8 FB / PARK counters
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    int n = 0, it = 0, tail_iter = -1;
    long live = 0;  // live paths at the last readback (an upper bound: paths only finish)
    bool done = false, tail_next = false;
    int await = 0;  // 0 none, 1 live count, 2 fallback counts (tail entry check)
    int fast_state = 0;  // fast lane: 0 waiting, 4 threshold read back (pending), 1 hand-over at the
                         // next k_step, 2 handed over, 3 none
    int fast_thr = 0, fast_n = 0;  // ... samples-done threshold, paths at most
    hipEvent_t (*tev)[RT_MAX_TIMED_ITERS] = nullptr;  // [3][RT_MAX_TIMED_ITERS]
};

// Runs the wavefront loop for n slots of `src` into fb (device, n float4).
int run_wave(rt_context* c, Backend* b, int w, int h, int spp, int bounces, const rtk::PixSrc& src, int n,
                    float4_* fb, hipStream_t s)
{
    if (n <= 0) return RT_OK;
    // every render of a context reuses its lanes' slots and counters: the previous render
    // (whose tail kernel may still run, on another stream) must finish first
    if (b->done_recorded) HIPCHK(c, hipStreamWaitEvent(s, b->ev_done, 0));
    int dev_cus = 256;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, b->device);
    const int threads = 256;
    // k_trace: wave-strided over 2 grid-fills; RT_TRACE_OCC blocks resident per CU (quad
    // walks: 6 waves/SIMD measured best, 423 vs 374 Msamples/s at 4 and 350 at 8)
    // k_trace grid-fills (RT_TRACE_FILLS): with per-wave query streams one fill is best, a wave's
    // stream is longer and its end (the last long walk) costs less; cfg2: 0.75 / 1 / 1.25 / 1.5 / 2 / 3
    // -> 739 / 730-740 / 731 / 724 / 708-710 / 692 Msamples/s
    const int trace_blocks = dev_cus * RT_TRACE_OCC;
    const RtSchedule& sc = c->sched;
    const RtDiag& dg = c->diag;
    const bool S = c->stats_enabled;
    const bool SEQ = S && c->stats_seq;  // (counter renders with unpaired occlusion walks: rt_set_stats(ctx, 2))
    unsigned long long* stats = (unsigned long long*)b->stats.p;
    if (S) HIPCHK(c, hipMemsetAsync(b->stats.p, 0, b->stats.bytes, s));
    const char* iter_log = dg.iter_log.empty() ? nullptr : dg.iter_log.c_str();  // per-iteration log of lane 0: counts (stats renders) / ms (timed)
    const bool wlog = S && dg.wlog_cap > 0 && b->index == 0;
    if (wlog) {
        if (int r = ensure(c, b->wlog, 256 + (size_t)dg.wlog_cap * 48)) return r;
        HIPCHK(c, hipMemsetAsync(b->wlog.p, 0, 256, s));
    }
    if (!b->handovers.p) {
        if (int r = ensure(c, b->handovers, 8)) return r;
        HIPCHK(c, hipMemsetAsync(b->handovers.p, 0, 8, s));
    }
    if (S && iter_log) {
        if (int r = ensure(c, b->iterq, RT_MAX_TIMED_ITERS * 24)) return r;
        HIPCHK(c, hipMemsetAsync(b->iterq.p, 0, RT_MAX_TIMED_ITERS * 24, s));
    }
    // lanes: rows interleave (row j of the launch -> lane j % lanes); pixel lists split in runs
    const int lanes_set = sc.lanes > 0 ? std::min(RT_MAX_LANES, sc.lanes) : b->lanes;
    const int fast_k = spp <= RT_FAST_MAX_SPP ? std::max(0, std::min(1 << 16, sc.fast_k >= 0 ? sc.fast_k : RT_FAST_K)) : 0;
    // (auto: 3 lanes with the fast lane, the fourth hardware queue its stream)
    int nl = lanes_set > 0 ? lanes_set : n <= RT_LANES4_MAX && fast_k == 0 ? 4 : 3;
    const int rows = src.xy ? 0 : n / src.W;
    while (nl > 1 && (n < nl * 65536 || (!src.xy && rows < nl))) nl--;
    WaveLane L[RT_MAX_LANES];
    const int force_fb = sc.force_fallback;  // (test stressor, rt_test_schedule)
    const int heavy_calls = sc.heavy_calls >= 0 ? sc.heavy_calls : RT_HEAVY_CALLS;
    // the next sample's camera ray traced ahead (rt_wave.h next_camera): 1; 0 off; 2 only where
    // the pixel's previous sample ended (cfg2 -1.5 ms, the cfg4 8-way shard unchanged, r04)
    const int spec_cam = sc.spec_cam >= 0 ? sc.spec_cam : 1;
    // The camera ray traced ahead costs a walk whenever the sample goes on. In k_tail a round
    // waits for its path's slowest query, often that camera walk: there it is off (cfg4 8-way
    // shard 352.3-354.6 -> 343.5 ms, cfg2 142.5-143.6 -> 141.3-141.6, profiles/r04q_cam.json).
    const int tail_spec_cam = sc.tail_spec_cam >= 0 ? sc.tail_spec_cam : 0;  // the tail kernel's mode (as spec_cam)
    // k_tail paths per wave: a round waits for the slowest walk of the wave's ~3 P queries, so
    // fewer paths per wave move each chain faster. With the entry held at the same live count
    // (r03, P x RT_TAIL_ENTER = 3.5): P = 5 / 3 / 2 / 1 -> cfg2 886-893 / 892-896 / 897-901 /
    // 887-890 Msamples/s, cfg4 8-way shard (slowest rank) 401 / - / 390 / 405 ms
    // row walks (rt_row.h, 16 lanes per query over the 16-wide BVH) where walks are latency-bound:
    // the tail kernel (tail_rows: its rounds wait for their slowest walk). cfg4 8-way shard, one
    // MI355X (profiles/r04c_row_probe.json, r04d_tail_probe.json): quads 380-382 ms; tail rows
    // 367-370; rows for whole k_trace launches below 32 K / 131 K paths 415 / 420-428 ms (removed).
    // (counter renders with unpaired occlusion walks, SEQ: every walk a quad walk, so that the box
    // tests counted are the ones a one-node-per-trip walk makes; a row trip tests 16)
    const int tail_rows = SEQ ? 0 : sc.tail_rows >= 0 ? (sc.tail_rows != 0) : RT_TAIL_ROWS;
    const int drain_rows = SEQ ? 0 : sc.drain_rows >= 0 ? sc.drain_rows : RT_DRAIN_ROWS;  // k_trace: a drain's walks continue as rows
    // (rows: one path per wave, its ~4 queries on the wave's 4 rows: shard 367 ms vs 2 / 3 paths
    // 373-378 / 373-375 at the same entry live count)
    const int tail_p = sc.tail_paths >= 0 ? std::min(RT_TAIL_MAXP, sc.tail_paths) : tail_rows ? 1 : 2;
    const int tail_blocks = dev_cus * RT_TAIL_OCC;  // one grid-fill of k_tail
    // a lane enters the tail kernel at 2x one grid-fill's pool (the waves refill from the live
    // list): with 2 paths per wave, RT_TAIL_ENTER = 1.4 / 1.75 / 2.2 / 2.8 -> cfg2 888-897 /
    // 891-898 / 893-897 / 874-879 Msamples/s (5 paths at 0.7: 888-892), cfg4 8-way shard
    // 393.5 / 389.6 / 393.1 / - ms (profiles/r03_tail_paths_ab.json)
    // (4 lanes, the auto count of launches of <= 1.5 M slots: 1.4 — cfg4 8-way shard, 4 rounds on
    // one MI355X: 2.0 / 1.5 / 1.25 / 1.0 -> 384-391 / 380-384 / 379-383 / 382-390 ms,
    // profiles/r03_tail_enter4.json)
    const double tail_enter = sc.tail_enter >= 0.0 ? sc.tail_enter : nl == 4 ? 1.4 : 2.0;
    // Fast lane: from iteration fast_spp x spp on, each lane's share of the fast_k live paths
    // with the fewest samples done (the pixels with the longest chains, tools/fastlane_model.py)
    // leaves the wavefront at the lane's next k_step; when every lane has handed its share over,
    // one tail kernel steps them all on a stream of their own (an idle lane's: 3 lanes + the fast
    // lane are the 4 hardware queues), at a tail round's pace beside the wavefront. cfg4 8-way
    // shard (rank 1) / cfg2, one MI355X, 3 rounds (profiles/r05_fast_lane.json): 4 lanes, none
    // 319.7-323.9 / 134.9-135.4 ms; 3 lanes + fast lane 768 paths at 2.0 / 2.25 x spp
    // 311.5-316.1 / 134.7-136.4 and 312.2-316.9 / 133.7-134.0; 1024 paths 308.1-317.6; 1536 and
    // more slower (r04's fast lane beside 4 lanes, a fifth stream: slower, r04x).
    const long fast_iter = (long)((sc.fast_spp >= 0.0 ? sc.fast_spp : RT_FAST_SPP) * spp);
    bool fast_launched = false, fast_ran = false;
    if (fast_k > 0 && nl == RT_MAX_LANES && !b->fs) HIPCHK(c, hipStreamCreateWithFlags(&b->fs, hipStreamNonBlocking));
    const hipStream_t fstream = fast_k > 0 ? (nl < RT_MAX_LANES ? b->ls[nl] : b->fs) : nullptr;
    const long tail_max = (long)(tail_enter * tail_blocks * 4 * tail_p / nl);
    if (nl > 1) {
        HIPCHK(c, hipEventRecord(b->ev_fork, s));
        for (int l = 1; l < nl; l++) HIPCHK(c, hipStreamWaitEvent(b->ls[l], b->ev_fork, 0));
    }
    for (int l = 0; l < nl; l++) {
        WaveLane& La = L[l];
        rtk::PixSrc ls = src;
        float4_* lfb = fb;
        int fb_rs = 1;
        if (nl == 1) {
            La.n = n;
        } else if (src.xy) {
            const int b0 = (int)((long)n * l / nl), b1 = (int)((long)n * (l + 1) / nl);
            La.n = b1 - b0;
            ls.xy = src.xy + 2 * (size_t)b0;
            lfb = fb + b0;
        } else {
            La.n = ((rows - l + nl - 1) / nl) * src.W;
            ls.off = src.off + l * src.stride;
            ls.stride = nl * src.stride;
            lfb = fb + (size_t)l * src.W;
            fb_rs = nl;
        }
        La.live = La.n;
        La.s = l == 0 ? s : b->ls[l];
        La.cnt = (int32_t*)b->counters[l].p;
        La.h = b->h_act[l];
        La.ev = b->ev_lane[l];
        La.tev = b->tev[l];
        rtk::WaveView& W = La.W;
        W.park_cap = 1 << 16;
        W.heavy_calls = heavy_calls;
        W.spec_cam = spec_cam;
        W.shards = RT_QSHARDS;
        W.seg_cap = 64 * (((La.n + 63) / 64 + RT_QSHARDS - 1) / RT_QSHARDS);  // (append_emit: chunks per shard)
        W.spill_lanes = dev_cus * 4 * threads;  // exact walks: up to dev_cus * 2 blocks per role
        W.fspill_lanes = 0;
        const size_t need = rtk::wave_carve(nullptr, (size_t)La.n, W);
        if (int r = ensure(c, b->wave[l], need)) return r;
        rtk::wave_carve((char*)b->wave[l].p, (size_t)La.n, W);
        W.S = b->view;
        rt_view_near(c, W.S);  // (rt_test_schedule may have changed it since the upload)
        W.cam = c->cam;
        W.src = ls;
        W.W = w;
        W.H = h;
        W.spp = spp;
        W.bounces = bounces;
        rtk::set_view_consts(W);
        W.n_slots = La.n;
        W.bl_rays = b->bl_rays;
        W.any_rays = b->any_rays;
        W.fb = lfb;
        W.fb_rs = fb_rs;
        W.budget = sc.step_budget > 0 ? sc.step_budget : b->budget;
        W.counters = La.cnt;
        W.tail_paths = tail_p;
        W.drain_rows = drain_rows;
        W.force_fb = force_fb;
        W.fast_cap = 0;
        La.fast_state = fast_k > 0 ? 0 : 3;
        La.fast_n = (int)((long)fast_k * (l + 1) / nl - (long)fast_k * l / nl);
        if (fast_k > 0) {  // the fast lane's buffers and events (first use)
            if (int r = ensure(c, b->fast[l], (size_t)(La.fast_n + 1) * 4)) return r;
            if (int r = ensure(c, b->fcnt[l], C_COUNT * sizeof(int32_t))) return r;
            if (int r = ensure(c, b->fhist[l], (RT_FAST_MAX_SPP + 1) * 4)) return r;
            if (int r = ensure(c, b->fspill[l], (size_t)((La.fast_n + 3) / 4) * threads * RT_STACK_CAP * 8)) return r;
            if (!b->h_hist[l]) HIPCHK(c, hipHostMalloc((void**)&b->h_hist[l], (RT_FAST_MAX_SPP + 1) * 4, hipHostMallocDefault));
            if (!b->fev[l]) HIPCHK(c, hipEventCreateWithFlags(&b->fev[l], hipEventDisableTiming));
            if (!b->hev[l]) HIPCHK(c, hipEventCreateWithFlags(&b->hev[l], hipEventDisableTiming));
            HIPCHK(c, hipMemsetAsync(b->fcnt[l].p, 0, C_COUNT * sizeof(int32_t), La.s));
        }
        W.iterq = (S && iter_log && l == 0) ? (int32_t*)b->iterq.p : nullptr;
        W.handovers = (unsigned long long*)b->handovers.p;
        if (wlog) {
            W.wlog_n = (int32_t*)b->wlog.p;
            W.wlog = (float4_*)((char*)b->wlog.p + 256);
            W.wlog_min = dg.wlog_min;
            W.wlog_cap = dg.wlog_cap;
            W.wlog_every = dg.wlog_every;
        }
        La.lists[0] = (int32_t*)W.act_in;
        La.lists[1] = W.act_out;
        HIPCHK(c, hipMemsetAsync(La.cnt, 0, C_COUNT * sizeof(int32_t), La.s));
        HIPCHK(c, hipMemsetAsync(W.r_park, 0, (size_t)La.n * 4, La.s));
        W.act_in = La.lists[1];
        W.act_out = La.lists[0];
        hipLaunchKernelGGL(k_init, dim3((La.n + threads - 1) / threads), dim3(threads), 0, La.s, W);
        HIPCHK(c, hipGetLastError());
    }
    if (dg.verbose)
        fprintf(stderr, "[rt] run_wave n=%d lanes=%d cus=%d trace_blocks=%d budget=%d\n", n, nl, dev_cus, trace_blocks,
                L[0].W.budget);

    // A sample takes at most bounces + 1 iterations without fallbacks; an
    // exact walk delays its path by at least one iteration. The bound only
    // guards against a runaway loop.
    const long max_iters = 64l * spp * ((long)bounces + 1) + 4096;
    const size_t act_bytes = RT_QSHARDS * RT_CSTRIDE * 4;
    // grids sized by the last known live count: k_step one slot per thread; k_trace up to
    // five queries per path, a quad each, over two grid-fills, never fewer blocks than the
    // exact-walk roles can claim (dev_cus * 4) plus room for the fast roles
    // (k_step: at least 3 blocks, one per exact-walk role and one for the path step, so a
    // small live count with fallbacks or parked walks pending still steps its paths)
    auto step_blocks_of = [&](const WaveLane& La) {
        return (int)std::max(3l, std::min((La.live + threads - 1) / threads, (long)dev_cus * RT_STEP_FILL));
    };
    auto trace_blocks_of = [&](const WaveLane& La) {
        const long want = (20 * La.live + 2 * threads - 1) / (2 * threads);
        return (int)std::min((long)trace_blocks, std::max(want, (long)dev_cus * 4 + 64));
    };
    auto launch_trace = [&](WaveLane& La) -> int {
        rtk::WaveView& W = La.W;
        const int par = La.it & 1;
        W.iter = La.it;
        W.act_in = La.lists[par];
        W.act_out = La.lists[par ^ 1];
        const bool T = b->timing && La.it < RT_MAX_TIMED_ITERS;
        if (T)
            for (int k = 0; k < 3; k++)
                if (!La.tev[k][La.it]) HIPCHK(c, hipEventCreate(&La.tev[k][La.it]));
        if (T) HIPCHK(c, hipEventRecord(La.tev[0][La.it], La.s));
        const dim3 g(trace_blocks_of(La));
        if (SEQ)
            hipLaunchKernelGGL((k_trace<true, false>), g, dim3(threads), 0, La.s, W, par, stats);
        else if (S)
            hipLaunchKernelGGL((k_trace<true, true>), g, dim3(threads), 0, La.s, W, par, stats);
        else
            hipLaunchKernelGGL((k_trace<false, true>), g, dim3(threads), 0, La.s, W, par, stats);
        if (T) HIPCHK(c, hipEventRecord(La.tev[1][La.it], La.s));
        HIPCHK(c, hipGetLastError());
        return RT_OK;
    };
    // the fast lane's tail kernel, once every lane has handed its share over (or has none)
    auto fast_launch = [&]() -> int {
        if (fast_k == 0 || fast_launched) return RT_OK;
        bool any = false;
        for (int l = 0; l < nl; l++) {
            if (L[l].fast_state < 2 || L[l].fast_state == 4) return RT_OK;  // (a lane still to hand over)
            any = any || L[l].fast_state == 2;
        }
        fast_launched = true;
        if (!any) return RT_OK;
        if (!b->h_fviews)
            HIPCHK(c, hipHostMalloc((void**)&b->h_fviews, sizeof(rtk::WaveView) * RT_MAX_LANES, hipHostMallocDefault));
        if (!b->fev_done) HIPCHK(c, hipEventCreateWithFlags(&b->fev_done, hipEventDisableTiming));
        if (b->fev_done_recorded) HIPCHK(c, hipEventSynchronize(b->fev_done));  // (the last render's copy of the views)
        if (int r = ensure(c, b->fviews, sizeof(rtk::WaveView) * RT_MAX_LANES)) return r;
        int start[RT_MAX_LANES + 1] = {}, tot = 0;
        for (int l = 0; l < RT_MAX_LANES; l++) {
            start[l] = tot;
            if (l >= nl || L[l].fast_state != 2) continue;
            rtk::WaveView FW = L[l].W;
            FW.act_in = (int32_t*)b->fast[l].p;
            FW.counters = (int32_t*)b->fcnt[l].p;
            FW.fast_cap = L[l].fast_n;
            FW.tail_paths = 1;  // (one path per wave, its queries on the wave's rows)
            const int blocks = (L[l].fast_n + 3) / 4;
            FW.spill_r = (uint32_t*)b->fspill[l].p;
            FW.spill_k = (float*)((uint32_t*)b->fspill[l].p + (size_t)blocks * threads * RT_STACK_CAP);
            FW.iterq = nullptr;
            FW.spec_cam = spec_cam ? tail_spec_cam : 0;
            b->h_fviews[l] = FW;
            tot += blocks;
            HIPCHK(c, hipStreamWaitEvent(fstream, b->fev[l], 0));
        }
        HIPCHK(c, hipMemcpyAsync(b->fviews.p, b->h_fviews, sizeof(rtk::WaveView) * RT_MAX_LANES, hipMemcpyHostToDevice,
                                 fstream));
        const rtk::WaveView* fv = (const rtk::WaveView*)b->fviews.p;
        if (b->timing) {
            for (hipEvent_t& e : b->ftev)
                if (!e) HIPCHK(c, hipEventCreate(&e));
            HIPCHK(c, hipEventRecord(b->ftev[0], fstream));
        }
        const int4 parts = make_int4(start[0], start[1], start[2], start[3]);
        if (SEQ)
            hipLaunchKernelGGL((k_tail_fast<true, false, 4>), dim3(tot), dim3(threads), 0, fstream, fv, parts, stats);
        else if (S)
            hipLaunchKernelGGL((k_tail_fast<true, true, 16>), dim3(tot), dim3(threads), 0, fstream, fv, parts, stats);
        else
            hipLaunchKernelGGL((k_tail_fast<false, true, 16>), dim3(tot), dim3(threads), 0, fstream, fv, parts, stats);
        HIPCHK(c, hipGetLastError());
        if (b->timing) HIPCHK(c, hipEventRecord(b->ftev[1], fstream));
        HIPCHK(c, hipEventRecord(b->fev_done, fstream));
        b->fev_done_recorded = fast_ran = true;
        return RT_OK;
    };
    // the fast lane's threshold: the samples-done count of the lane's fast_n-th slowest live
    // path, from the histogram k_hist read back (polled: the host thread serving every lane
    // never blocks on it; the hand-over happens at the first k_step after it has landed)
    auto fast_threshold = [&](WaveLane& La) -> int {
        const int l = (int)(&La - L);
        const hipError_t q = hipEventQuery(b->hev[l]);
        if (q == hipErrorNotReady) return RT_OK;
        HIPCHK(c, q);
        long acc = 0;
        int thr = spp;
        for (int k = 0; k <= spp; k++)
            if ((acc += b->h_hist[l][k]) >= La.fast_n) {
                thr = k;
                break;
            }
        La.fast_thr = thr;
        La.fast_state = 1;
        return RT_OK;
    };
    auto launch_step = [&](WaveLane& La) -> int {
        const int par = La.it & 1;
        const int l = (int)(&La - L);
        if (La.fast_state == 4)
            if (int r = fast_threshold(La)) return r;
        const bool hand = La.fast_state == 1;
        int32_t* fl = (int32_t*)b->fast[l].p;
        if (hand) {  // this step hands the lane's slowest paths to the fast lane
            HIPCHK(c, hipMemsetAsync(fl + La.fast_n, 0, 4, La.s));
            rtk::WaveView HW = La.W;
            HW.fast_list = fl;
            HW.fast_ticket = fl + La.fast_n;
            HW.fast_cap = La.fast_n;
            HW.fast_thr = La.fast_thr;
            hipLaunchKernelGGL(k_hand, dim3((unsigned)std::min(1024l, (La.live + threads - 1) / threads)), dim3(threads), 0,
                               La.s, HW, par);
            HIPCHK(c, hipGetLastError());
        }
        if (S)
            hipLaunchKernelGGL(k_step<true>, dim3(step_blocks_of(La)), dim3(threads), 0, La.s, La.W, par, stats);
        else
            hipLaunchKernelGGL(k_step<false>, dim3(step_blocks_of(La)), dim3(threads), 0, La.s, La.W, par, stats);
        if (hand) {  // (its list's length as shard 0 of the fast lane's counters)
            La.fast_state = 2;
            HIPCHK(c, hipMemcpyAsync((int32_t*)b->fcnt[l].p + ac_at(0, 0), fl + La.fast_n, 4, hipMemcpyDeviceToDevice, La.s));
            HIPCHK(c, hipEventRecord(b->fev[l], La.s));
            if (int r = fast_launch()) return r;
        }
        if (b->timing && La.it < RT_MAX_TIMED_ITERS) HIPCHK(c, hipEventRecord(La.tev[2][La.it], La.s));
        HIPCHK(c, hipGetLastError());
        La.it++;
        return RT_OK;
    };
    auto read_live = [&](WaveLane& La) -> int {  // ACT counts of the next iteration
        HIPCHK(c, hipMemcpyAsync(La.h, La.cnt + ac_at(La.it & 1, 0), act_bytes, hipMemcpyDeviceToHost, La.s));
        HIPCHK(c, hipEventRecord(La.ev, La.s));
        La.await = 1;
        return RT_OK;
    };
    // enqueue up to 8 iterations, then a readback
    auto issue = [&](WaveLane& La) -> int {
        for (int k = 0; k < 8 && La.it < max_iters; k++) {
            if (int r = launch_trace(La)) return r;
            if (La.tail_next) {  // does any query wait for the exact walk?
                HIPCHK(c, hipMemcpyAsync(La.h + act_bytes / 4, La.cnt, 8 * 4, hipMemcpyDeviceToHost, La.s));
                HIPCHK(c, hipEventRecord(La.ev, La.s));
                La.await = 2;
                return RT_OK;
            }
            if (int r = launch_step(La)) return r;
            if ((La.it & 7) == 0) break;
        }
        return read_live(La);
    };
    auto process = [&](WaveLane& La) -> int {
        HIPCHK(c, hipEventSynchronize(La.ev));
        const int kind = La.await;
        La.await = 0;
        if (kind == 2) {  // (a fallback pending: step, then the live count, checked again next iteration)
            const int par = La.it & 1;
            const int32_t* f = La.h + act_bytes / 4;
            if (f[C_FBC0 + par] == 0 && f[C_FBA0 + par] == 0 && f[C_PARKC0 + (par ^ 1)] == 0 &&
                f[C_PARKA0 + (par ^ 1)] == 0) {  // (k_trace(i) released DONE[par ^ 1])
                // few paths left and none waits: the tail kernel finishes them all
                HIPCHK(c, hipMemsetAsync(La.cnt + C_TK_TAIL, 0, 4, La.s));
                const dim3 g(tail_blocks);
                La.W.spec_cam = spec_cam ? tail_spec_cam : 0;  // (the lane's last launch)
                if (SEQ)
                    hipLaunchKernelGGL((k_tail<true, false, 4>), g, dim3(threads), 0, La.s, La.W, par, stats);
                else if (S)
                    hipLaunchKernelGGL((tail_rows ? k_tail<true, true, 16> : k_tail<true, true, 4>), g, dim3(threads), 0, La.s, La.W, par, stats);
                else
                    hipLaunchKernelGGL((tail_rows ? k_tail<false, true, 16> : k_tail<false, true, 4>), g, dim3(threads), 0, La.s, La.W, par, stats);
                if (b->timing && La.it < RT_MAX_TIMED_ITERS) HIPCHK(c, hipEventRecord(La.tev[2][La.it], La.s));
                HIPCHK(c, hipGetLastError());
                La.tail_iter = La.it;
                La.it++;
                La.done = true;
                return RT_OK;
            }
            if (int r = launch_step(La)) return r;
            return read_live(La);
        }
        long live = 0;
        for (int j = 0; j < RT_QSHARDS; j++) live += La.h[j * RT_CSTRIDE];
        La.live = live;
        La.done = live == 0;
        La.tail_next = !La.done && live <= tail_max;
        if ((La.fast_state == 0 || La.fast_state == 4) && (La.done || La.tail_next)) {  // (no hand-over from this lane)
            if (La.fast_state == 4) HIPCHK(c, hipEventSynchronize(b->hev[(int)(&La - L)]));  // (its readback is done with h_hist)
            La.fast_state = 3;
            if (int r = fast_launch()) return r;
        } else if (La.fast_state == 0 && La.it >= fast_iter) {
            // the samples-done histogram of the lane's live paths, read back asynchronously
            // (fast_threshold picks it up from a later k_step launch)
            const int l = (int)(&La - L);
            int32_t* hh = (int32_t*)b->fhist[l].p;
            HIPCHK(c, hipMemsetAsync(hh, 0, (size_t)(spp + 1) * 4, La.s));
            rtk::WaveView HW = La.W;
            HW.act_in = La.lists[La.it & 1];
            hipLaunchKernelGGL(k_hist, dim3((unsigned)std::min(1024l, (live + threads - 1) / threads)), dim3(threads), 0,
                               La.s, HW, La.it & 1, hh);
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipMemcpyAsync(b->h_hist[l], hh, (size_t)(spp + 1) * 4, hipMemcpyDeviceToHost, La.s));
            HIPCHK(c, hipEventRecord(b->hev[l], La.s));
            La.fast_state = 4;
        }
        return RT_OK;
    };
    for (int l = 0; l < nl; l++)
        if (int r = issue(L[l])) return r;
    // The host serves whichever lane's readback has completed (hipEventQuery), so a lane whose
    // batch is done is refilled at once instead of idling while the host blocks on another
    // lane's event (blocking in lane order left lanes idle 17-34 ms of a 367-ms cfg4 8-way
    // shard: profiles/r04e_tl.json; 379.5-380.2 -> 370.5-373.2 ms, cfg2 148.5-149.7 -> 148.0,
    // profiles/r04i_drain_probe.json).
    // (a thread that finds no lane done for a while sleeps between polls: in a multi-device
    // render every device thread polls like this, and the caller's host work shares the cores)
    auto idle_since = std::chrono::steady_clock::now();
    for (;;) {
        bool any = false, moved = false;
        for (int l = 0; l < nl; l++) {
            WaveLane& La = L[l];
            if (La.await) {
                any = true;
                const hipError_t q = hipEventQuery(La.ev);
                if (q == hipErrorNotReady) continue;
                HIPCHK(c, q);
                if (int r = process(La)) return r;
                moved = true;
            }
            if (!La.done && !La.await) {
                if (La.it >= max_iters) {
                    HIPCHK(c, hipStreamSynchronize(La.s));
                    return rt_fail(c, RT_ERR_STATE, "render: wavefront loop did not drain in " +
                                                            std::to_string(max_iters) + " iterations (step budget " +
                                                            std::to_string(b->budget) + ")");
                }
                if (int r = issue(La)) return r;
                any = moved = true;
            }
        }
        if (!any) break;
        if (moved) {
            idle_since = std::chrono::steady_clock::now();
        } else if (std::chrono::steady_clock::now() - idle_since > std::chrono::microseconds(200)) {
            std::this_thread::sleep_for(std::chrono::microseconds(10));
        } else {
            std::this_thread::yield();
        }
    }
    for (int l = 0; l < nl; l++) {  // each lane's pixels tone-mapped after its last step
        if (fast_ran)
            HIPCHK(c, hipStreamWaitEvent(L[l].s, b->fev_done, 0));  // (and the fast lane's)
        hipLaunchKernelGGL(k_tonemap, dim3((L[l].n + threads - 1) / threads), dim3(threads), 0, L[l].s, L[l].W);
        HIPCHK(c, hipGetLastError());
    }
    b->last_iters = 0;
    for (int l = 0; l < nl; l++) {
        b->last_iters = std::max(b->last_iters, L[l].it);
        if (l > 0) {
            HIPCHK(c, hipEventRecord(b->ev_join[l], b->ls[l]));
            HIPCHK(c, hipStreamWaitEvent(s, b->ev_join[l], 0));
        }
    }
    b->tail_iter = L[0].tail_iter;
    HIPCHK(c, hipEventRecord(b->ev_done, s));
    b->done_recorded = true;
    if (wlog) {  // (diagnostics: device 0's records of this render replace the last render's)
        int32_t nw = 0;
        HIPCHK(c, hipMemcpyAsync(&nw, b->wlog.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        RtDiag& d = c->diag;
        d.wlog_total = nw;
        d.wlog.assign((size_t)std::min(nw, d.wlog_cap) * RT_WLOG_FLOATS, 0.0f);
        if (!d.wlog.empty())
            HIPCHK(c, hipMemcpy(d.wlog.data(), (char*)b->wlog.p + 256, d.wlog.size() * 4, hipMemcpyDeviceToHost));
    }
    if (S && iter_log) {
        std::vector<int32_t> hq((size_t)6 * RT_MAX_TIMED_ITERS);
        HIPCHK(c, hipMemcpyAsync(hq.data(), b->iterq.p, hq.size() * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if (FILE* f = fopen((std::string(iter_log) + ".counts").c_str(), "w")) {
            const int32_t* h2 = hq.data() + 2 * RT_MAX_TIMED_ITERS;
            for (int i = 0; i <= L[0].it && i < RT_MAX_TIMED_ITERS; i++)
                fprintf(f, "%d %d %d %d %d %d %d\n", i, hq[2 * i], hq[2 * i + 1], h2[4 * i], h2[4 * i + 1], h2[4 * i + 2],
                        h2[4 * i + 3]);
            fclose(f);
        }
    }
    if (b->timing) {  // per-kernel-class time of this render (HIP events on the launch streams)
        HIPCHK(c, hipStreamSynchronize(s));
        FILE* lf = iter_log ? fopen((std::string(iter_log) + ".ms").c_str(), "w") : nullptr;
        for (int l = 0; l < nl; l++)
            for (int i = 0; i < L[l].it && i < RT_MAX_TIMED_ITERS; i++)
                for (int k = 0; k < 2; k++) {
                    float ms = 0;
                    HIPCHK(c, hipEventElapsedTime(&ms, L[l].tev[k][i], L[l].tev[k + 1][i]));
                    const int cls = (k == 1 && i == L[l].tail_iter) ? 2 : k;  // the tail kernel: class "other"
                    b->kms[cls] += ms;
                    b->klaunch[cls] += 1;
                    if (lf && l == 0) {
                        if (k == 0)
                            fprintf(lf, "%d %.4f", i, ms);
                        else
                            fprintf(lf, " %.4f\n", ms);
                    }
                }
        if (lf) fclose(lf);
        // RT_TIMELINE=file: every lane's launches on one clock (ms from lane 0's first
        // k_trace): lane, iteration, k_trace start, k_trace end = k_step start, k_step end,
        // 1 for the tail kernel (tools/timeline.py); the fast lane's kernel as lane `lanes`,
        // iteration 0, flag 2
        // (device index d > 0 of a multi-device context writes file.d: the device threads run concurrently)
        if (!dg.timeline.empty()) {
            const char* tl = dg.timeline.c_str();
            std::string rows;
            char line[128];
            for (int l = 0; l < nl; l++)
                for (int i = 0; i < L[l].it && i < RT_MAX_TIMED_ITERS; i++) {
                    float t[3];
                    for (int k = 0; k < 3; k++) HIPCHK(c, hipEventElapsedTime(&t[k], L[0].tev[0][0], L[l].tev[k][i]));
                    snprintf(line, sizeof line, "%d %d %.4f %.4f %.4f %d\n", l, i, t[0], t[1], t[2],
                             i == L[l].tail_iter ? 1 : 0);
                    rows += line;
                }
            if (fast_ran) {
                float t[2];
                for (int k = 0; k < 2; k++) HIPCHK(c, hipEventElapsedTime(&t[k], L[0].tev[0][0], b->ftev[k]));
                snprintf(line, sizeof line, "%d 0 %.4f %.4f %.4f 2\n", nl, t[0], t[1], t[1]);
                rows += line;
            }
            const std::string path = b->index > 0 ? std::string(tl) + "." + std::to_string(b->index) : std::string(tl);
            if (FILE* f = fopen(path.c_str(), "w")) {
                fwrite(rows.data(), 1, rows.size(), f);
                fclose(f);
            }
        }
    }
#if RT_DEBUG_FB
    {
        unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(c, hipStreamSynchronize(s));
        for (int l = 0; l < nl; l++) HIPCHK(c, hipStreamSynchronize(L[l].s));
        HIPCHK(c, hipMemcpyFromSymbol(v, HIP_SYMBOL(rt_dbg_fb), sizeof v));
        int its = 0;
        for (int l = 0; l < nl; l++) its = std::max(its, L[l].it);
        fprintf(stderr, "[rt dbg] n=%d iters=%d k_trace fallbacks closest=%llu any=%llu (overflow %llu tie %llu chain %llu; rows %llu) octet parks=%llu closest row drains=%llu\n",
                n, its, v[0], v[2], v[3], v[4], v[5], v[6], v[1], v[7]);
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(c, hipMemcpyToSymbol(HIP_SYMBOL(rt_dbg_fb), z, sizeof z));
    }
#endif
    return RT_OK;
}

int finish_stats(rt_context* c, Backend* b, hipStream_t s)
{
    if (!c->stats_enabled) return RT_OK;
    HIPCHK(c, hipMemcpyAsync(c->stats, b->stats.p, sizeof(c->stats), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return RT_OK;
}

// Rows of a multi-device render: request row j (image row off + j*stride) belongs to
// device j mod N. Device d's rows go to block d of the root's staging buffer (rows_max
// rows each; the tail of a short block is padding), ncclScatter sends block d to
// device d, every device renders its block with its own wavefront loop (one host
// thread per device: run_wave polls its lanes), and ncclGather brings the blocks back
// for the un-permute. Pack and un-permute are strided 2-D copies on the root.
int render_multi(rt_context* c, Group* g, int w, int h, int spp, int bounces, float4_* fb, int off, int stride,
                 hipStream_t s)
{
    const int N = (int)g->dev.size();
    std::string err;
    const Rccl* R = nullptr;
    if (!g->loopback && !(R = rccl_load(err))) return rt_fail(c, RT_ERR_NODEV, err);
    const int rows = (h - off + stride - 1) / stride;
    const int rows_max = (rows + N - 1) / N;
    const size_t blk = (size_t)rows_max * w;  // float4 per block
    auto rows_of = [&](int d) { return rows > d ? (rows - d + N - 1) / N : 0; };
    Backend* root = g->dev[0];
    for (int d = 1; d < N; d++) {
        HIPCHK(c, hipSetDevice(g->dev[d]->device));
        if (int r = ensure(c, g->shard[d], std::max<size_t>(blk, 1) * sizeof(float4_))) return r;
    }
    HIPCHK(c, hipSetDevice(root->device));
    if (int r = ensure(c, g->stage, std::max<size_t>(blk, 1) * N * sizeof(float4_))) return r;
    float4_* stage = (float4_*)g->stage.p;
    HIPCHK(c, hipEventRecord(root->ev0, s));
    const size_t pitch = (size_t)w * sizeof(float4_);
    for (int d = 0; d < N; d++)
        if (rows_of(d))
            HIPCHK(c, hipMemcpy2DAsync(stage + d * blk, pitch, fb + (size_t)d * w, N * pitch, pitch, rows_of(d),
                                       hipMemcpyDeviceToDevice, s));
    std::vector<hipStream_t> st(N);
    for (int d = 0; d < N; d++) st[d] = d == 0 ? s : g->dev[d]->own;
    const size_t cnt = blk * 4;  // floats per block
    if (g->loopback) {  // block d -> device d by a device copy on the root stream; the shard streams wait for it
        for (int d = 1; d < N; d++)
            HIPCHK(c, hipMemcpyAsync(g->shard[d].p, stage + d * blk, blk * sizeof(float4_), hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipEventRecord(root->ev_fork, s));
        for (int d = 1; d < N; d++) {
            HIPCHK(c, hipSetDevice(g->dev[d]->device));
            HIPCHK(c, hipStreamWaitEvent(st[d], root->ev_fork, 0));
        }
        HIPCHK(c, hipSetDevice(root->device));
    } else {
        NCCLCHK(c, R, R->group_start());
        for (int d = 0; d < N; d++)
            NCCLCHK(c, R, R->scatter(stage, d == 0 ? (void*)stage : g->shard[d].p, cnt, ncclFloat, 0, g->comms[d], st[d]));
        NCCLCHK(c, R, R->group_end());
    }
    // the wavefront loops, one host thread per device; errors are collected per device
    // and raised once after the join (rt_for_devices). run_wave resets the stats itself.
    if (int r = rt_for_devices(c, N, [&](int d) -> int {
            Backend* b = g->dev[d];
            HIPCHK(c, hipSetDevice(b->device));
            const rtk::PixSrc src{w, off + d * stride, N * stride, nullptr};
            float4_* dst = d == 0 ? stage : (float4_*)g->shard[d].p;
            return run_wave(c, b, w, h, spp, bounces, src, rows_of(d) * w, dst, st[d]);
        }))
        return r;
    HIPCHK(c, hipSetDevice(root->device));
    if (g->loopback) {  // each block back to the root after its device's loop; the root stream waits for all
        for (int d = 1; d < N; d++) {
            Backend* b = g->dev[d];
            HIPCHK(c, hipSetDevice(b->device));
            HIPCHK(c, hipMemcpyAsync(stage + d * blk, g->shard[d].p, blk * sizeof(float4_), hipMemcpyDeviceToDevice, st[d]));
            HIPCHK(c, hipEventRecord(b->ev_join[0], st[d]));
            HIPCHK(c, hipSetDevice(root->device));
            HIPCHK(c, hipStreamWaitEvent(s, b->ev_join[0], 0));
        }
    } else {
        NCCLCHK(c, R, R->group_start());
        for (int d = 0; d < N; d++)
            NCCLCHK(c, R, R->gather(d == 0 ? (const void*)stage : g->shard[d].p, stage, cnt, ncclFloat, 0, g->comms[d], st[d]));
        NCCLCHK(c, R, R->group_end());
    }
    for (int d = 0; d < N; d++)
        if (rows_of(d))
            HIPCHK(c, hipMemcpy2DAsync(fb + (size_t)d * w, N * pitch, stage + d * blk, pitch, pitch, rows_of(d),
                                       hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipEventRecord(root->ev1, s));
    if (c->stats_enabled) {  // counters summed over the devices
        unsigned long long sum[2 * RT_STAT_COUNT] = {};
        for (int d = 0; d < N; d++) {
            HIPCHK(c, hipSetDevice(g->dev[d]->device));
            HIPCHK(c, hipMemcpyAsync(c->stats, g->dev[d]->stats.p, sizeof(c->stats), hipMemcpyDeviceToHost, st[d]));
            HIPCHK(c, hipStreamSynchronize(st[d]));
            for (int i = 0; i < 2 * RT_STAT_COUNT; i++) sum[i] += c->stats[i];
        }
        std::memcpy(c->stats, sum, sizeof sum);
        HIPCHK(c, hipSetDevice(root->device));
    }
    root->last_iters = 0;
    for (Backend* b : g->dev) root->last_iters = std::max(root->last_iters, b->last_iters);
    return RT_OK;
}
}  // namespace

int rt_backend_render(rt_context* c, int w, int h, int spp, int bounces, float* host_fb, void* dev_fb, int row_offset,
                      int row_stride, void* stream)
{
    Group* g = grp(c);
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(b->device));
    hipStream_t s = (hipStream_t)stream;
    const int rows_local = (h - row_offset + row_stride - 1) / row_stride;
    const size_t npx = (size_t)rows_local * w;
    if (npx > 0x7fffffff / 8) return rt_fail(c, RT_ERR_ARG, "render: too many pixels for one launch");
    float4_* fb = (float4_*)dev_fb;
    if (host_fb) {
        if (int r = ensure(c, b->fb, npx * sizeof(float4_))) return r;
        fb = (float4_*)b->fb.p;
        HIPCHK(c, hipMemcpyAsync(fb, host_fb, npx * sizeof(float4_), hipMemcpyHostToDevice, s));
    }
    if (g->multi) {
        if (int r = render_multi(c, g, w, h, spp, bounces, fb, row_offset, row_stride, s)) return r;
    } else {
        rtk::PixSrc src{w, row_offset, row_stride, nullptr};
        HIPCHK(c, hipEventRecord(b->ev0, s));
        if (int r = run_wave(c, b, w, h, spp, bounces, src, (int)npx, fb, s)) return r;
        HIPCHK(c, hipEventRecord(b->ev1, s));
    }
    if (host_fb) {
        HIPCHK(c, hipMemcpyAsync(host_fb, fb, npx * sizeof(float4_), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, b->ev0, b->ev1));
        c->last_kernel_ms = ms;
    } else {
        c->last_kernel_ms = -1.0;  // read with rt_device_last_kernel_ms after the caller synchronizes
    }
    return g->multi ? RT_OK : finish_stats(c, b, s);
}

// The material sweep as replicas (rt_render_variants): variant v on device v mod N, one
// host thread per device (rt_for_devices), each device walking its variants in order on
// its own stream: the variant's table goes into the device's material buffer with a copy
// ordered after the previous variant's frame (same stream), then the wavefront loop.
// No exchange between devices.
int rt_backend_render_variants(rt_context* c, int w, int h, int spp, int bounces, int n_var,
                               const std::vector<RtMat>& tabs, int n_mats, int off, int stride, float* host_fb,
                               void* const* d_fbs)
{
    Group* g = grp(c);
    const int N = (int)g->dev.size();
    const int rows = (h - off + stride - 1) / stride;
    const size_t npx = (size_t)rows * w;
    if (npx > 0x7fffffff / 8) return rt_fail(c, RT_ERR_ARG, "render: too many pixels for one launch");
    std::vector<float> ms(N, 0.0f);
    // counters summed over every variant of every device (run_wave zeroes a device's per render)
    std::vector<std::vector<unsigned long long>> vsum(N, std::vector<unsigned long long>(2 * RT_STAT_COUNT, 0));
    const int r = rt_for_devices(c, N, [&](int d) -> int {
        Backend* b = g->dev[d];
        HIPCHK(c, hipSetDevice(b->device));
        hipStream_t s = b->own;
        if (b->done_recorded) HIPCHK(c, hipEventSynchronize(b->ev_done));  // (the table and buffers are reused)
        if (int e = ensure(c, b->mats, (size_t)n_mats * sizeof(RtMat))) return e;
        b->view.mats = (const RtMat*)b->mats.p;
        b->view.n_mats = n_mats;
        if (host_fb)
            if (int e = ensure(c, b->fb, npx * sizeof(float4_))) return e;
        HIPCHK(c, hipEventRecord(b->ev0, s));
        for (int v = d; v < n_var; v += N) {
            const RtMat* tab = tabs.data() + (size_t)v * n_mats;
            b->bl_rays = rt_table_has_emissive_prim(c, tab) ? 1 : 0;
            // (pageable source: the copy is staged before the call returns, and ordered on s
            // after the previous variant's frame, whose lanes joined back into s)
            HIPCHK(c, hipMemcpyAsync(b->mats.p, tab, (size_t)n_mats * sizeof(RtMat), hipMemcpyHostToDevice, s));
            float4_* fb = host_fb ? (float4_*)b->fb.p : (float4_*)d_fbs[v];
            if (host_fb)
                HIPCHK(c, hipMemcpyAsync(fb, host_fb + 4 * npx * v, npx * sizeof(float4_), hipMemcpyHostToDevice, s));
            const rtk::PixSrc src{w, off, stride, nullptr};
            if (int e = run_wave(c, b, w, h, spp, bounces, src, (int)npx, fb, s)) return e;
            if (host_fb)
                HIPCHK(c, hipMemcpyAsync(host_fb + 4 * npx * v, fb, npx * sizeof(float4_), hipMemcpyDeviceToHost, s));
            if (c->stats_enabled) {  // (diagnostic renders: this variant's counters, before the next zeroes them)
                unsigned long long one[2 * RT_STAT_COUNT];
                HIPCHK(c, hipMemcpyAsync(one, b->stats.p, sizeof one, hipMemcpyDeviceToHost, s));
                HIPCHK(c, hipStreamSynchronize(s));
                for (int i = 0; i < 2 * RT_STAT_COUNT; i++) vsum[d][i] += one[i];
            }
        }
        HIPCHK(c, hipEventRecord(b->ev1, s));
        HIPCHK(c, hipStreamSynchronize(s));
        HIPCHK(c, hipEventElapsedTime(&ms[d], b->ev0, b->ev1));
        return 0;
    });
    // the bound table comes back with the next render's upload (rt_render_variants marks it)
    for (Backend* b : g->dev) b->bl_rays = rt_scene_has_emissive_prim(c) ? 1 : 0;
    HIPCHK(c, hipSetDevice(be(c)->device));
    if (r) return r;
    c->last_kernel_ms = *std::max_element(ms.begin(), ms.end());
    if (c->stats_enabled)  // every variant of every device, summed
        for (int i = 0; i < 2 * RT_STAT_COUNT; i++) {
            c->stats[i] = 0;
            for (int d = 0; d < N; d++) c->stats[i] += vsum[d][i];
        }
    return RT_OK;
}

// One device's share of a pixel list (host buffers in and out).
static int render_pixels_one(rt_context* c, Backend* b, int w, int h, int spp, int bounces, const int* xy, int n,
                             float* rgba, float* ms_out)
{
    HIPCHK(c, hipSetDevice(b->device));
    if (n == 0) return RT_OK;
    const size_t bxy = (size_t)n * 8, brgba = (size_t)n * 16;
    if (int r = ensure(c, b->xy, bxy)) return r;
    if (int r = ensure(c, b->fb, brgba)) return r;
    hipStream_t s = b->own;
    HIPCHK(c, hipMemcpyAsync(b->xy.p, xy, bxy, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(b->fb.p, rgba, brgba, hipMemcpyHostToDevice, s));
    if (c->stats_enabled) HIPCHK(c, hipMemsetAsync(b->stats.p, 0, b->stats.bytes, s));
    rtk::PixSrc src{w, 0, 1, (const int32_t*)b->xy.p};
    HIPCHK(c, hipEventRecord(b->ev0, s));
    if (int r = run_wave(c, b, w, h, spp, bounces, src, n, (float4_*)b->fb.p, s)) return r;
    HIPCHK(c, hipEventRecord(b->ev1, s));
    HIPCHK(c, hipMemcpyAsync(rgba, b->fb.p, brgba, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    *ms_out = ms;
    return RT_OK;
}

int rt_backend_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    Group* g = grp(c);
    const int N = (int)g->dev.size();
    if (N == 1) {
        float ms = 0;
        if (int r = render_pixels_one(c, g->dev[0], w, h, spp, bounces, xy, n, rgba, &ms)) return r;
        c->last_kernel_ms = ms;
        return finish_stats(c, g->dev[0], g->dev[0]->own);
    }
    // pixel i -> device i mod N (pixels are independent); host-side split and merge
    std::vector<std::vector<int>> pxy(N);
    std::vector<std::vector<float>> prgba(N);
    for (int i = 0; i < n; i++) {
        pxy[i % N].push_back(xy[2 * i]);
        pxy[i % N].push_back(xy[2 * i + 1]);
        prgba[i % N].insert(prgba[i % N].end(), rgba + 4 * (size_t)i, rgba + 4 * (size_t)i + 4);
    }
    std::vector<int> rc(N, RT_OK);
    std::vector<float> ms(N, 0.0f);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < N; d++)
            th.emplace_back([&, d] {
                rc[d] = render_pixels_one(c, g->dev[d], w, h, spp, bounces, pxy[d].data(), (int)pxy[d].size() / 2,
                                          prgba[d].data(), &ms[d]);
            });
        for (auto& t : th) t.join();
    }
    for (int d = 0; d < N; d++)
        if (rc[d]) return rc[d];
    for (int i = 0; i < n; i++) std::memcpy(rgba + 4 * (size_t)i, &prgba[i % N][4 * (size_t)(i / N)], 16);
    c->last_kernel_ms = *std::max_element(ms.begin(), ms.end());
    if (c->stats_enabled) {
        unsigned long long sum[2 * RT_STAT_COUNT] = {};
        for (int d = 0; d < N; d++) {
            if (int r = finish_stats(c, g->dev[d], g->dev[d]->own)) return r;
            for (int i = 0; i < 2 * RT_STAT_COUNT; i++) sum[i] += c->stats[i];
        }
        std::memcpy(c->stats, sum, sizeof sum);
    }
    return RT_OK;
}

int rt_backend_intersect(rt_context* c, const float* rays, int n, void* out)
{
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(b->device));
    const size_t br = (size_t)n * 24, bo = (size_t)n * 44;
    if (int r = ensure(c, b->xy, br + bo)) return r;
    float* dr = (float*)b->xy.p;
    int32_t* dout = (int32_t*)((char*)b->xy.p + br);
    HIPCHK(c, hipMemcpy(dr, rays, br, hipMemcpyHostToDevice));
    const int threads = 256, blocks = (n + threads - 1) / threads;
    HIPCHK(c, hipEventRecord(b->ev0, 0));
    hipLaunchKernelGGL(k_intersect, dim3(blocks), dim3(threads), 0, 0, b->view, dr, dout, n);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(b->ev1, 0));
    HIPCHK(c, hipEventSynchronize(b->ev1));
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    c->last_kernel_ms = ms;
    HIPCHK(c, hipMemcpy(out, dout, bo, hipMemcpyDeviceToHost));
    return RT_OK;
}

// Device self-tests of the numerics (libm restatement, IEEE div/sqrt/f64).
extern "C" int rt_device_libm(int device, int fn, const float* in, const float* in2, float* out, int n)
{
    if (hipSetDevice(device) != hipSuccess) return RT_ERR_NODEV;
    float *d_in = nullptr, *d_in2 = nullptr, *d_out = nullptr;
    const size_t b = (size_t)n * 4;
    if (hipMalloc(&d_in, b) != hipSuccess || hipMalloc(&d_in2, b) != hipSuccess || hipMalloc(&d_out, b) != hipSuccess)
        return RT_ERR_HIP;
    (void)hipMemcpy(d_in, in, b, hipMemcpyHostToDevice);
    if (in2) (void)hipMemcpy(d_in2, in2, b, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_libm, dim3((n + 255) / 256), dim3(256), 0, 0, fn, d_in, d_in2, d_out, n);
    hipError_t e = hipMemcpy(out, d_out, b, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_in2);
    (void)hipFree(d_out);
    return e == hipSuccess ? RT_OK : RT_ERR_HIP;
}

// Search-BVH query micro-benchmark: rays[n][8] (origin xyz _, direction xyz _),
// mode bit 0 = any (else closest), bits 1.. = walk variant (0-1 one lane, 2-3 lane + spill,
// 4-5 quads, 6-7 quads at 8 waves/SIMD, 8-9 rows);
// reps timed launches (HIP events), mean ms per launch into *ms.
extern "C" int rt_device_queries(rt_context* c, int mode, const float* rays, int n, int reps, float* out_t,
                                 int* out_k, double* ms)
{
    if (!c || !c->backend || n <= 0 || reps < 1 || mode < 0 || mode > 9) return RT_ERR_ARG;
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(b->device));
    if (c->dirty) {
        if (int r = rt_backend_upload(c)) return r;
        c->dirty = false;
    }
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b->device);
    const int threads = 256, blocks = std::min((n + threads - 1) / threads, cus * 8);
    const int qblocks = std::min((4 * n + threads - 1) / threads, cus * 16);
    const int rblocks = std::min((16 * n + threads - 1) / threads, cus * 16);
    float4_* d_rays = nullptr;
    float* d_t = nullptr;
    int* d_k = nullptr;
    uint32_t* sr = nullptr;
    float* sk = nullptr;
    const size_t lanes = (size_t)blocks * threads;
    HIPCHK(c, hipMalloc(&d_rays, (size_t)n * 32));
    HIPCHK(c, hipMalloc(&d_t, (size_t)n * 4));
    HIPCHK(c, hipMalloc(&d_k, (size_t)n * 4));
    HIPCHK(c, hipMalloc(&sr, lanes * RT_SPILL_FAST * 4));
    HIPCHK(c, hipMalloc(&sk, lanes * RT_SPILL_FAST * 4));
    HIPCHK(c, hipMemcpy(d_rays, rays, (size_t)n * 32, hipMemcpyHostToDevice));
    auto launch = [&]() {
        switch (mode) {
            case 0: hipLaunchKernelGGL((k_query<false, 0>), dim3(blocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n, sr, sk); break;
            case 1: hipLaunchKernelGGL((k_query<true, 0>), dim3(blocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n, sr, sk); break;
            case 2: hipLaunchKernelGGL((k_query<false, 1>), dim3(blocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n, sr, sk); break;
            case 3: hipLaunchKernelGGL((k_query<true, 1>), dim3(blocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n, sr, sk); break;
            case 4: hipLaunchKernelGGL((k_query_quad<false, 1>), dim3(qblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
            case 5: hipLaunchKernelGGL((k_query_quad<true, 1>), dim3(qblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
            case 6: hipLaunchKernelGGL((k_query_quad<false, 8>), dim3(qblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
            case 7: hipLaunchKernelGGL((k_query_quad<true, 8>), dim3(qblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
            case 8: hipLaunchKernelGGL((k_query_row<false>), dim3(rblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
            default: hipLaunchKernelGGL((k_query_row<true>), dim3(rblocks), dim3(threads), 0, 0, b->view, d_rays, d_t, d_k, n); break;
        }
    };
    launch();  // warm-up
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(b->ev0, 0));
    for (int r = 0; r < reps; r++) launch();
    HIPCHK(c, hipEventRecord(b->ev1, 0));
    HIPCHK(c, hipEventSynchronize(b->ev1));
    float t = 0;
    HIPCHK(c, hipEventElapsedTime(&t, b->ev0, b->ev1));
    if (ms) *ms = t / reps;
    HIPCHK(c, hipMemcpy(out_t, d_t, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_k, d_k, (size_t)n * 4, hipMemcpyDeviceToHost));
    (void)hipFree(d_rays);
    (void)hipFree(d_t);
    (void)hipFree(d_k);
    (void)hipFree(sr);
    (void)hipFree(sk);
    return RT_OK;
}

// Time between the events around the last rt_render_device launch sequence
// (recorded on its stream); call after synchronizing that stream.
extern "C" double rt_device_last_kernel_ms(rt_context* c)
{
    if (!c || !c->backend) return -1.0;
    Backend* b = be(c);
    float ms = 0;
    if (hipEventSynchronize(b->ev1) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, b->ev0, b->ev1) != hipSuccess) return -1.0;
    c->last_kernel_ms = ms;
    return ms;
}

// Iterations the last wavefront render took.
extern "C" int rt_device_last_iterations(rt_context* c) { return c && c->backend ? be(c)->last_iters : -1; }

// Queries k_trace handed to the exact octree walk (ties, failed verifications, stack
// overflows, far origins, the force_fallback stressor) in every render on every device of
// the context since the last reset: the walks' health figure (~2e-6 per sample on cfg2).
// Waits for the devices.
extern "C" int rt_device_exact_handovers(rt_context* c, unsigned long long* out, int reset)
{
    if (!c || !c->backend || !out) return RT_ERR_ARG;
    unsigned long long sum = 0;
    for (Backend* b : grp(c)->dev) {
        HIPCHK(c, hipSetDevice(b->device));
        HIPCHK(c, hipDeviceSynchronize());
        if (!b->handovers.p) continue;
        unsigned long long v = 0;
        HIPCHK(c, hipMemcpy(&v, b->handovers.p, 8, hipMemcpyDeviceToHost));
        sum += v;
        if (reset) HIPCHK(c, hipMemset(b->handovers.p, 0, 8));
    }
    *out = sum;
    return RT_OK;
}

// Per-kernel-class timing (k_trace, k_step, k_tail) over the renders since it
// was enabled, summed over the context's devices: out_ms[3] total ms (HIP events
// around every launch on its lane's stream), out_launches[3].
extern "C" int rt_device_kernel_timing(rt_context* c, int enable, double* out_ms, long* out_launches)
{
    if (!c || !c->backend) return RT_ERR_ARG;
    Group* g = grp(c);
    for (int k = 0; k < 3; k++) {
        double ms = 0;
        long n = 0;
        for (Backend* b : g->dev) ms += b->kms[k], n += b->klaunch[k];
        if (out_ms) out_ms[k] = ms;
        if (out_launches) out_launches[k] = n;
    }
    if (enable >= 0)
        for (Backend* b : g->dev) {
            b->timing = enable != 0;
            for (int k = 0; k < 3; k++) b->kms[k] = 0, b->klaunch[k] = 0;
        }
    return RT_OK;
}

// Wavefront lanes (streams) per render on every device of the context (RT_LANES at
// creation; 1 serializes a render's launches, for per-launch kernel timing; 0: auto).
extern "C" int rt_device_set_lanes(rt_context* c, int lanes)
{
    if (!c || !c->backend || lanes < 0) return RT_ERR_ARG;
    for (Backend* b : grp(c)->dev) b->lanes = std::min(RT_MAX_LANES, lanes);
    return RT_OK;
}

#ifndef RT_BUILD_SRC
#define RT_BUILD_SRC "unknown"
#endif
#ifndef RT_BUILD_DEFS
#define RT_BUILD_DEFS ""
#endif
extern "C" const char* rt_build_id(void) { return "src=" RT_BUILD_SRC " defs=" RT_BUILD_DEFS " (gfx950)"; }
