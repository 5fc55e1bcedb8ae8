// rt_hostsim.cpp — CPU build of the *product* device code (rt_trace.h),
// linked into librt_hostsim.so for the CPU test suite only.
//
// It lets the container (no GPU) check that the kernel's algorithm — the
// explicit-stack octree walk, the heap-order emulation, the libm
// restatement — reproduces the oracle bit for bit before the same source is
// compiled for gfx950. It is NOT a fallback: the product library
// librt_hip.so has no CPU path and fails loudly without a device.
#include <omp.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_context.h"
#include "rt_wave.h"

// Stack window and step budget of the host build: smaller than the
// device's so that the CPU tests exercise spilling (dragon rays need up to
// 19 entries) and parking / resuming across iterations all the time.
#ifndef RT_HOSTSIM_SHORT_CAP
#define RT_HOSTSIM_SHORT_CAP 8
#endif
#ifndef RT_HOSTSIM_FAST_CAP
#define RT_HOSTSIM_FAST_CAP 32
#endif
#ifndef RT_HOSTSIM_BUDGET
#define RT_HOSTSIM_BUDGET 24
#endif

int rt_backend_create(rt_context*) { return RT_OK; }
void rt_backend_destroy(rt_context*) {}
int rt_backend_upload(rt_context*) { return RT_OK; }

// adds the per-thread counters into out (callers zero it once per render: a variant sweep sums)
static void merge_stats(unsigned long long* out, const std::vector<rtk::Stats>& s)
{
    for (const auto& t : s)
        for (int i = 0; i < RT_STAT_COUNT; i++) out[i] += t.c[i];
}

// The OpenMP team of one "device" thread of a multi-device render: the caller's thread
// count split over the N devices (each device thread runs its own parallel regions), and
// the caller's own setting restored afterwards (device 0 runs on the caller's thread).
struct OmpShare {
    int all, each;
    explicit OmpShare(int n) : all(omp_get_max_threads()), each(std::max(1, omp_get_max_threads() / std::max(1, n))) {}
    void enter() const { omp_set_num_threads(each); }
    ~OmpShare() { omp_set_num_threads(all); }
};

// The product's wavefront loop (rt_render.hip run_wave) on the host:
// same stage functions, same queues; appends are plain atomics.
template <class E>
static void host_append(const rtk::WaveView& W, int32_t* act_count, int p, const E& e)
{
    for (int k = 0; k < rtk::RK_COUNT; k++)
        if ((e.mask >> k) & 1u) W.q[k][__atomic_fetch_add(&W.counters[k], 1, __ATOMIC_RELAXED)] = e.rec(k, p);
    if (e.active) W.act_out[__atomic_fetch_add(act_count, 1, __ATOMIC_RELAXED)] = p;
}

static int run_wave_host(rt_context* c, int w, int h, int spp, int bounces, const rtk::PixSrc& src, int n,
                         float4_* fb, unsigned long long* stats_out, const RtMat* mats = nullptr)
{
    if (n <= 0) return RT_OK;
    rtk::WaveView W{};
    W.park_cap = 1 << 14;
    W.spec_cam = c->sched.spec_cam >= 0 ? c->sched.spec_cam : 1;  // (rt_test_schedule; the product's default)
    W.force_fb = c->sched.force_fallback;
    W.spill_lanes = 0;  // the host threads keep their own spill areas
    W.shards = 1;       // one segment per queue (plain atomics on the host)
    W.seg_cap = n;
    std::vector<char> arena(rtk::wave_carve(nullptr, (size_t)n, W));
    rtk::wave_carve(arena.data(), (size_t)n, W);
    W.S = rt_host_view(c);
    if (mats) W.S.mats = mats;  // (rt_render_variants: a variant's table, same size as the bound one)
    W.cam = c->cam;
    W.src = src;
    W.W = w;
    W.H = h;
    W.spp = spp;
    W.bounces = bounces;
    rtk::set_view_consts(W);
    W.n_slots = n;
    W.bl_rays = rt_table_has_emissive_prim(c, W.S.mats) ? 1 : 0;
    W.any_rays = W.S.n_spheres == 0 ? 1 : 0;
    W.fb = fb;
    W.budget = RT_HOSTSIM_BUDGET;
    int32_t counters[rtk::RK_COUNT] = {0};
    int32_t act[2] = {0, 0};
    int32_t parkc[2] = {0, 0}, parka[2] = {0, 0};
    W.counters = counters;
    std::memset(W.r_park, 0, (size_t)n * 4);
    int32_t* lists[2] = {(int32_t*)W.act_in, W.act_out};
    std::vector<rtk::Stats> st(omp_get_max_threads());
    for (auto& s : st) std::memset(&s, 0, sizeof s);

    W.act_out = lists[0];
#pragma omp parallel for schedule(static)
    for (int p = 0; p < n; p++) {
        rtk::Emit e;
        rtk::path_init(W, p, e);
        host_append(W, &act[0], p, e);
    }
    using FAST = rtk::ArrayStack<RT_HOSTSIM_SHORT_CAP>;
    const int last_kind = W.any_rays ? rtk::RK_CAM : rtk::RK_BENV;
    int32_t fbc[2] = {0, 0}, fba[2] = {0, 0};
    for (long it = 0;; it++) {
        const int par = (int)(it & 1);
        // k_trace, exact roles: the walks the last iteration left (parked
        // ones, then its fallback lists); each holds one r_park count of its slot
        const int nrc = std::min(parkc[par], W.park_cap), nra = std::min(parka[par], W.park_cap);
        const int nc = nrc + fbc[par], na = nra + fba[par];
#pragma omp parallel
        {
            std::vector<uint32_t> spr(RT_STACK_CAP);
            std::vector<float> spk(RT_STACK_CAP);
            rtk::SpillStack<FAST> stk{FAST{}, spr.data(), spk.data()};
            rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 16)
            for (int idx = 0; idx < nc; idx++) {
                rtk::TravC T;
                uint32_t target;
                bool has;
                if (idx < nrc) {
                    target = rtk::travc_resume(&W.park_c[par][idx], T, stk);
                    has = true;
                } else {
                    const rtk::RayRec r = W.fb_c[par][idx - nrc];
                    target = (rt_asuint(r.o.w) << 3) | rt_asuint(r.d.w);
                    if (ps) ps->c[RT_STAT_FALLBACK]++;
                    has = rtk::travc_begin(W.S, T, rtk::v3of(r.o), rtk::v3of(r.d), ps);
                    if (!has) {
                        rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
                        __atomic_fetch_sub(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                    }
                }
                while (has) {
                    if (!rtk::travc_step(W.S, T, stk, ps)) {
                        rtk::finish_closest(W, target, T.o, T.d, T.best_t, T.best_k);
                        __atomic_fetch_sub(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                        break;
                    }
                    if (T.steps >= W.budget && rtk::travc_parkable(T)) {
                        const int slot = __atomic_fetch_add(&parkc[par ^ 1], 1, __ATOMIC_RELAXED);
                        if (slot < W.park_cap) {
                            rtk::travc_park(T, stk, target, &W.park_c[par ^ 1][slot]);
                            break;
                        }
                        T.steps = 0;
                    }
                }
            }
#pragma omp for schedule(dynamic, 16)
            for (int idx = 0; idx < na; idx++) {
                rtk::TravA T;
                uint32_t target;
                bool has;
                if (idx < nra) {
                    target = rtk::trava_resume(&W.park_a[par][idx], T, stk);
                    has = true;
                } else {
                    const rtk::RayRec r = W.fb_a[par][idx - nra];
                    target = (rt_asuint(r.o.w) << 3) | rt_asuint(r.d.w);
                    if (ps) ps->c[RT_STAT_FALLBACK]++;
                    has = rtk::trava_begin(W.S, T, rtk::v3of(r.o), rtk::v3of(r.d), ps);
                    if (!has) {
                        rtk::finish_any(W, target, T.hit);  // (false, or the brute-force answer)
                        __atomic_fetch_sub(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                    }
                }
                while (has) {
                    if (!rtk::trava_step(W.S, T, stk, ps)) {
                        rtk::finish_any(W, target, T.hit);
                        __atomic_fetch_sub(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                        break;
                    }
                    if (T.steps >= W.budget && rtk::trava_parkable(T)) {
                        const int slot = __atomic_fetch_add(&parka[par ^ 1], 1, __ATOMIC_RELAXED);
                        if (slot < W.park_cap) {
                            rtk::trava_park(T, stk, target, &W.park_a[par ^ 1][slot]);
                            break;
                        }
                        T.steps = 0;
                    }
                }
            }
        }
        // k_trace, fast roles: this iteration's queries through the search
        // BVH; failures go to the fallback lists of the next iteration
        int nq = 0;
        for (int k = rtk::RK_CONT; k <= last_kind; k++) nq += counters[k];
        const int nqa = W.any_rays ? counters[rtk::RK_ESH] + counters[rtk::RK_BENV] : 0;
        int32_t* fbc_out = &fbc[par ^ 1];
        int32_t* fba_out = &fba[par ^ 1];
#pragma omp parallel
        {
            rtk::IdxStack<RT_HOSTSIM_FAST_CAP> fst;
            rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < nq; idx++) {
                uint32_t target;
                rtk::RayRec r = rtk::queue_item(W, counters, rtk::RK_CONT, last_kind, idx, target);
                float t;
                int k;
                if (!rtk::forced_fallback(W.force_fb, r.o, r.d) &&
                    rtk::fast_query_closest(W.S, rtk::v3of(r.o), rtk::v3of(r.d), fst, t, k, ps)) {
                    rtk::finish_closest(W, target, rtk::v3of(r.o), rtk::v3of(r.d), t, k);
                } else {
                    r.d.w = rt_asfloat(target & 7u);
                    W.fb_c[par ^ 1][__atomic_fetch_add(fbc_out, 1, __ATOMIC_RELAXED)] = r;
                    __atomic_fetch_add(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                }
            }
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < nqa; idx++) {
                uint32_t target;
                rtk::RayRec r = rtk::queue_item(W, counters, rtk::RK_ESH, rtk::RK_BENV, idx, target);
                const int a = rtk::forced_fallback(W.force_fb, r.o, r.d) ? -1
                              : rtk::fast_query_any(W.S, rtk::v3of(r.o), rtk::v3of(r.d), fst, ps);
                if (a >= 0) {
                    rtk::finish_any(W, target, a == 1);
                } else {
                    r.d.w = rt_asfloat(target & 7u);
                    W.fb_a[par ^ 1][__atomic_fetch_add(fba_out, 1, __ATOMIC_RELAXED)] = r;
                    __atomic_fetch_add(&W.r_park[target >> 3], 1, __ATOMIC_RELAXED);
                }
            }
        }
        // k_step
        for (int k = 0; k < rtk::RK_COUNT; k++) counters[k] = 0;
        parkc[par] = parka[par] = 0;
        fbc[par] = fba[par] = 0;
        act[par ^ 1] = 0;
        W.act_in = lists[par];
        W.act_out = lists[par ^ 1];
        const int n_in = act[par];
        if (n_in == 0) break;
#pragma omp parallel
        {
            rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < n_in; idx++) {
                const int p = W.act_in[idx];
                // (the step's rays in a column, as k_step keeps them in LDS: rt_wave.h EmitLds)
                float col[6 * rtk::RK_COUNT];
                rtk::EmitLds<1> e;
                e.s = col;
                rtk::path_step(W, p, e, ps);
                host_append(W, &act[par ^ 1], p, e);
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (int p = 0; p < n; p++) rtk::tonemap_pixel(W, p);
    merge_stats(stats_out, st);
    return RT_OK;
}

// A compacted shard (row j = image row off + j*stride). A multi-device context
// (rt_create_multi) splits it the way the gfx950 backend's render_multi does: row j to
// "device" j mod N, each device's rows packed into a block, rendered as the rows
// off + d*stride + k*N*stride, and un-permuted (here with host copies instead of
// ncclScatter / ncclGather).
static int render_shard(rt_context* c, int w, int h, int spp, int bounces, int off, int stride, int rows,
                        float4_* shard)
{
    const int N = c->devices.empty() ? 1 : (int)c->devices.size();
    if (N == 1) {
        rtk::PixSrc src{w, off, stride, nullptr};
        std::fill(c->stats, c->stats + RT_STAT_COUNT, 0ull);
        return run_wave_host(c, w, h, spp, bounces, src, rows * w, shard, c->stats);
    }
    // one host thread per "device", as render_multi (rt_for_devices: per-device error slots),
    // each with its share of the OpenMP threads (not a full team per device)
    std::vector<std::vector<unsigned long long>> dst(N, std::vector<unsigned long long>(RT_STAT_COUNT, 0));
    const OmpShare share(N);
    const int r = rt_for_devices(c, N, [&](int d) {
        share.enter();
        const int rows_d = rows > d ? (rows - d + N - 1) / N : 0;
        std::vector<float4_> blk((size_t)rows_d * w);
        for (int k = 0; k < rows_d; k++) std::memcpy(&blk[(size_t)k * w], shard + (size_t)(d + k * N) * w, 16 * (size_t)w);
        rtk::PixSrc src{w, off + d * stride, N * stride, nullptr};
        if (int e = run_wave_host(c, w, h, spp, bounces, src, rows_d * w, blk.data(), dst[d].data())) return e;
        for (int k = 0; k < rows_d; k++) std::memcpy(shard + (size_t)(d + k * N) * w, &blk[(size_t)k * w], 16 * (size_t)w);
        return 0;
    });
    if (r) return r;
    for (int i = 0; i < RT_STAT_COUNT; i++) {
        c->stats[i] = 0;
        for (int d = 0; d < N; d++) c->stats[i] += dst[d][i];
    }
    return RT_OK;
}

int rt_backend_render(rt_context* c, int w, int h, int spp, int bounces, float* host_fb, void* dev_fb, int row_offset,
                      int row_stride, void*)
{
    // host_fb: the full frame (rt_render). dev_fb: in this build a host
    // pointer to a compacted row shard, row j = image row row_offset +
    // j*row_stride (rt_render_device semantics, used by the gloo tests).
    const int rows_local = (h - row_offset + row_stride - 1) / row_stride;
    const double t0 = omp_get_wtime();
    int r;
    if (host_fb) {
        // the full frame holds all rows; the wavefront works on the shard's rows
        std::vector<float4_> shard((size_t)rows_local * w);
        for (int j = 0; j < rows_local; j++)
            std::memcpy(&shard[(size_t)j * w], host_fb + 4 * (size_t)(row_offset + j * row_stride) * w, 16 * (size_t)w);
        r = render_shard(c, w, h, spp, bounces, row_offset, row_stride, rows_local, shard.data());
        for (int j = 0; j < rows_local; j++)
            std::memcpy(host_fb + 4 * (size_t)(row_offset + j * row_stride) * w, &shard[(size_t)j * w], 16 * (size_t)w);
    } else {
        r = render_shard(c, w, h, spp, bounces, row_offset, row_stride, rows_local, (float4_*)dev_fb);
    }
    c->last_kernel_ms = (omp_get_wtime() - t0) * 1e3;
    return r;
}

// The material sweep as replicas: variant v on "device" v mod N (one host thread each,
// rt_for_devices), every device walking its variants in order (rt_render.hip's driver).
int rt_backend_render_variants(rt_context* c, int w, int h, int spp, int bounces, int n_var,
                               const std::vector<RtMat>& tabs, int n_mats, int off, int stride, float* host_fb,
                               void* const* d_fbs)
{
    const int N = c->devices.empty() ? 1 : (int)c->devices.size();
    const int rows = (h - off + stride - 1) / stride;
    const size_t npx = (size_t)rows * w;
    const double t0 = omp_get_wtime();
    std::vector<std::vector<unsigned long long>> dst(N, std::vector<unsigned long long>(RT_STAT_COUNT, 0));
    const OmpShare share(N);
    const int r = rt_for_devices(c, N, [&](int d) {
        share.enter();
        for (int v = d; v < n_var; v += N) {
            // (hostsim: the per-variant mats pointer must cover the context's material indices)
            std::vector<RtMat> tab(tabs.begin() + (size_t)v * n_mats, tabs.begin() + (size_t)(v + 1) * n_mats);
            float4_* fb = host_fb ? (float4_*)(host_fb + 4 * npx * v) : (float4_*)d_fbs[v];  // (host pointers here)
            rtk::PixSrc src{w, off, stride, nullptr};
            if (int e = run_wave_host(c, w, h, spp, bounces, src, (int)npx, fb, dst[d].data(), tab.data())) return e;
        }
        return 0;
    });
    c->last_kernel_ms = (omp_get_wtime() - t0) * 1e3;
    if (r) return r;
    for (int i = 0; i < RT_STAT_COUNT; i++) {
        c->stats[i] = 0;
        for (int d = 0; d < N; d++) c->stats[i] += dst[d][i];
    }
    return RT_OK;
}

int rt_backend_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    rtk::PixSrc src{w, 0, 1, xy};
    std::fill(c->stats, c->stats + RT_STAT_COUNT, 0ull);
    return run_wave_host(c, w, h, spp, bounces, src, n, (float4_*)rgba, c->stats);
}

int rt_backend_intersect(rt_context* c, const float* rays, int n, void* out)
{
    const RtSceneView S = rt_host_view(c);
    std::vector<rtk::Stats> st(omp_get_max_threads());
    for (auto& s : st) std::memset(&s, 0, sizeof s);
#pragma omp parallel
    {
        std::vector<rtk::StackEnt> stack(RT_STACK_CAP);
        rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < n; i++) {
            const float* r = rays + 6 * (size_t)i;
            const rtk::V3 ro = rtk::v3(r[0], r[1], r[2]), rd = rtk::v3(r[3], r[4], r[5]);
            float t;
            int k;
            rtk::query_closest(S, ro, rd, stack.data(), t, k, ps);
            rtk::Hit h;
            bool f = rtk::hit_from(S, ro, rd, t, k, h);
            int32_t* o = (int32_t*)out + 11 * (size_t)i;
            const float neg1 = -1.0f;
            o[0] = f ? 1 : 0;
            o[1] = h.prim;
            std::memcpy(o + 2, &h.t, 4);
            float pn[6] = {0, 0, 0, 0, 0, 0};
            if (h.t != -1.0f) {
                pn[0] = h.p.x, pn[1] = h.p.y, pn[2] = h.p.z;
                pn[3] = h.n.x, pn[4] = h.n.y, pn[5] = h.n.z;
            }
            std::memcpy(o + 3, pn, 24);
            std::memcpy(o + 9, &neg1, 4);
            std::memcpy(o + 10, &neg1, 4);
        }
    }
    std::fill(c->stats, c->stats + RT_STAT_COUNT, 0ull);
    merge_stats(c->stats, st);
    return RT_OK;
}

// The search-BVH closest-hit query the render's k_trace stage runs (rt_fast.h
// fast_query_closest, with its verification), for tests/test_hostsim.py: out_t = the
// answer's t (-1 no hit) or -2 when the exact octree walk must answer; out_k its
// triangle's original index (-1 none). rays[n][6] = origin, direction.
extern "C" int rt_hostsim_fast_queries(rt_context* c, const float* rays, int n, float* out_t, int* out_k)
{
    if (!c || n < 0 || (n > 0 && (!rays || !out_t || !out_k))) return RT_ERR_ARG;
    if (!c->have_bvh) return RT_ERR_STATE;
    const RtSceneView S = rt_host_view(c);
#pragma omp parallel
    {
        rtk::IdxStack<RT_HOSTSIM_FAST_CAP> fst;
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < n; i++) {
            const float* r = rays + 6 * (size_t)i;
            float t;
            int k;
            if (rtk::fast_query_closest(S, rtk::v3(r[0], r[1], r[2]), rtk::v3(r[3], r[4], r[5]), fst, t, k, nullptr)) {
                out_t[i] = t;
                out_k[i] = k < 0 ? -1 : (int)rt_asuint(S.tri4[3 * (size_t)k].w);
            } else {
                out_t[i] = -2.0f;
                out_k[i] = -2;
            }
        }
    }
    return RT_OK;
}

// Heap-order emulation self-check against std::priority_queue (exported for
// tests/test_hostsim.py): keys[m] in push order -> order[m] of pushed indices.
#include <queue>
extern "C" int rt_hostsim_heap_order(const float* keys, int m, int* order_emul, int* order_std)
{
    if (m < 1 || m > 8) return -1;
    float k[8], ok[8];
    int id[8], oi[8];
    for (int i = 0; i < m; i++) k[i] = keys[i], id[i] = i;
    rtk::heap_order(k, id, m, ok, oi);
    for (int i = 0; i < m; i++) order_emul[i] = oi[i];
    struct QE {
        int id;
        float t;
        bool operator>(const QE& o) const { return t > o.t; }
    };
    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
    for (int i = 0; i < m; i++) q.emplace(QE{i, keys[i]});
    for (int i = 0; i < m; i++) {
        order_std[i] = q.top().id;
        q.pop();
    }
    return 0;
}

#ifndef RT_BUILD_SRC
#define RT_BUILD_SRC "unknown"
#endif
#ifndef RT_BUILD_DEFS
#define RT_BUILD_DEFS ""
#endif
extern "C" const char* rt_build_id(void) { return "src=" RT_BUILD_SRC " defs=" RT_BUILD_DEFS " (hostsim)"; }
