// rt_hostsim.cpp — CPU build of the *product* device code (rt_trace.h),
// linked into librt_hostsim.so for the CPU test suite only.
//
// It lets the container (no GPU) check that the kernel's algorithm — the
// explicit-stack octree walk, the heap-order emulation, the libm
// restatement — reproduces the oracle bit for bit before the same source is
// compiled for gfx950. It is NOT a fallback: the product library
// librt_hip.so has no CPU path and fails loudly without a device.
#include <omp.h>

#include <cstring>
#include <vector>

#include "rt_context.h"
#include "rt_wave.h"

// Short-stack capacity of the host build: smaller than the device's so that
// the CPU tests take the overflow fallback often (dragon rays need up to 19).
#ifndef RT_HOSTSIM_SHORT_CAP
#define RT_HOSTSIM_SHORT_CAP 8
#endif

int rt_backend_create(rt_context*) { return RT_OK; }
void rt_backend_destroy(rt_context*) {}
int rt_backend_upload(rt_context*) { return RT_OK; }

static void merge_stats(rt_context* c, const std::vector<rtk::Stats>& s)
{
    for (int i = 0; i < RT_STAT_COUNT; i++) c->stats[i] = 0;
    for (const auto& t : s)
        for (int i = 0; i < RT_STAT_COUNT; i++) c->stats[i] += t.c[i];
}

// The product's wavefront loop (rt_render.hip run_wave) on the host:
// same stage functions, same queues; appends are plain atomics.
static void host_append(const rtk::WaveView& W, int32_t* act_count, int p, const rtk::Emit& e)
{
    for (int k = 0; k < rtk::RK_COUNT; k++)
        if ((e.mask >> k) & 1u) W.q[k][__atomic_fetch_add(&W.counters[k], 1, __ATOMIC_RELAXED)] = e.r[k];
    if (e.active) W.act_out[__atomic_fetch_add(act_count, 1, __ATOMIC_RELAXED)] = p;
}

static int run_wave_host(rt_context* c, int w, int h, int spp, int bounces, const rtk::PixSrc& src, int n,
                         float4_* fb)
{
    if (n <= 0) return RT_OK;
    rtk::WaveView W{};
    std::vector<char> arena(rtk::wave_carve(nullptr, (size_t)n, W));
    rtk::wave_carve(arena.data(), (size_t)n, W);
    W.S = rt_host_view(c);
    W.cam = c->cam;
    W.src = src;
    W.W = w;
    W.H = h;
    W.spp = spp;
    W.bounces = bounces;
    W.n_slots = n;
    W.bl_rays = rt_scene_has_emissive_prim(c) ? 1 : 0;
    W.any_rays = W.S.n_spheres == 0 ? 1 : 0;
    W.fb = fb;
    int32_t counters[rtk::RK_COUNT] = {0};
    int32_t act[2] = {0, 0};
    W.counters = counters;
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
    const long max_iters = (long)spp * ((long)bounces + 1) + 2;
    for (long it = 0; it < max_iters; it++) {
        const int cur = (int)(it & 1);
        const int nc = counters[rtk::RK_CONT] + counters[rtk::RK_LSH] + counters[rtk::RK_BL];
        const int na = counters[rtk::RK_ESH] + counters[rtk::RK_BENV];
#pragma omp parallel
        {
            std::vector<rtk::StackEnt> stack(RT_STACK_CAP);
            std::vector<uint32_t> astack(RT_STACK_CAP);
            rtk::ArrayStack<RT_HOSTSIM_SHORT_CAP> sstack;
            rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < nc; idx++) {
                int kind = rtk::RK_CONT, i = idx;
                if (i >= counters[rtk::RK_CONT]) {
                    i -= counters[rtk::RK_CONT];
                    kind = rtk::RK_LSH;
                    if (i >= counters[rtk::RK_LSH]) {
                        i -= counters[rtk::RK_LSH];
                        kind = rtk::RK_BL;
                    }
                }
                const rtk::RayRec r = W.q[kind][i];
                const int slot = (int)rt_asuint(r.o.w);
                float t;
                int k;
                // a small short stack so the tests exercise the overflow fallback
                if (!rtk::query_closest_short(W.S, rtk::v3of(r.o), rtk::v3of(r.d), sstack, t, k, ps))
                    rtk::query_closest(W.S, rtk::v3of(r.o), rtk::v3of(r.d), stack.data(), t, k, ps);
                if (kind == rtk::RK_CONT) {
                    W.r_cont_t[slot] = t;
                    W.r_cont_k[slot] = k;
                } else if (kind == rtk::RK_LSH) {
                    W.r_lsh_t[slot] = t;
                } else {
                    W.r_bl_t[slot] = t;
                    W.r_bl_k[slot] = k;
                }
            }
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < na; idx++) {
                const int n0 = counters[rtk::RK_ESH];
                const int kind = idx < n0 ? rtk::RK_ESH : rtk::RK_BENV;
                const rtk::RayRec r = W.q[kind][idx < n0 ? idx : idx - n0];
                const int slot = (int)rt_asuint(r.o.w);
                bool hit;
                if (W.any_rays) {
                    const int a = rtk::trace_any_short(W.S, rtk::v3of(r.o), rtk::v3of(r.d), sstack, ps);
                    hit = a >= 0 ? a == 1 : rtk::trace_any(W.S, rtk::v3of(r.o), rtk::v3of(r.d), astack.data(), ps);
                } else {
                    float t;
                    int k;
                    rtk::query_closest(W.S, rtk::v3of(r.o), rtk::v3of(r.d), stack.data(), t, k, ps);
                    hit = t > 0.0f;
                }
                (kind == rtk::RK_ESH ? W.r_esh : W.r_benv)[slot] = hit ? 1 : 0;
            }
        }
        for (int k = 0; k < rtk::RK_COUNT; k++) counters[k] = 0;
        act[cur ^ 1] = 0;
        W.act_in = lists[cur];
        W.act_out = lists[cur ^ 1];
        const int n_in = act[cur];
        if (n_in == 0) break;
#pragma omp parallel
        {
            rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 64)
            for (int idx = 0; idx < n_in; idx++) {
                const int p = W.act_in[idx];
                rtk::Emit e;
                rtk::path_step(W, p, e, ps);
                host_append(W, &act[cur ^ 1], p, e);
            }
        }
    }
    merge_stats(c, st);
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
    rtk::PixSrc src{w, row_offset, row_stride, nullptr};
    int r;
    if (host_fb) {
        // the full frame holds all rows; the wavefront works on the shard's rows
        std::vector<float4_> shard((size_t)rows_local * w);
        for (int j = 0; j < rows_local; j++)
            std::memcpy(&shard[(size_t)j * w], host_fb + 4 * (size_t)(row_offset + j * row_stride) * w, 16 * (size_t)w);
        r = run_wave_host(c, w, h, spp, bounces, src, rows_local * w, shard.data());
        for (int j = 0; j < rows_local; j++)
            std::memcpy(host_fb + 4 * (size_t)(row_offset + j * row_stride) * w, &shard[(size_t)j * w], 16 * (size_t)w);
    } else {
        r = run_wave_host(c, w, h, spp, bounces, src, rows_local * w, (float4_*)dev_fb);
    }
    c->last_kernel_ms = (omp_get_wtime() - t0) * 1e3;
    return r;
}

int rt_backend_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    rtk::PixSrc src{w, 0, 1, xy};
    return run_wave_host(c, w, h, spp, bounces, src, n, (float4_*)rgba);
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
    merge_stats(c, st);
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
