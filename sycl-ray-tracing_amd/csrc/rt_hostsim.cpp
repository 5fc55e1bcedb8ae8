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
#include "rt_trace.h"

int rt_backend_create(rt_context*) { return RT_OK; }
void rt_backend_destroy(rt_context*) {}
int rt_backend_upload(rt_context*) { return RT_OK; }

static void merge_stats(rt_context* c, const std::vector<rtk::Stats>& s)
{
    for (int i = 0; i < RT_STAT_COUNT; i++) c->stats[i] = 0;
    for (const auto& t : s)
        for (int i = 0; i < RT_STAT_COUNT; i++) c->stats[i] += t.c[i];
}

int rt_backend_render(rt_context* c, int w, int h, int spp, int bounces, float* host_fb, void* dev_fb, int row_offset,
                      int row_stride, void*)
{
    // host_fb: the full frame (rt_render). dev_fb: in this build a host
    // pointer to a compacted row shard, row j = image row row_offset +
    // j*row_stride (rt_render_device semantics, used by the gloo tests).
    float* out = host_fb ? host_fb : (float*)dev_fb;
    const bool shard = host_fb == nullptr;
    rtk::Ctx C{rt_host_view(c), c->cam, w, h, spp, bounces};
    std::vector<rtk::Stats> st(omp_get_max_threads());
    for (auto& s : st) std::memset(&s, 0, sizeof s);
    const int rows_local = (h - row_offset + row_stride - 1) / row_stride;
    const double t0 = omp_get_wtime();
#pragma omp parallel
    {
        std::vector<rtk::StackEnt> stack(RT_STACK_CAP);
        rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic)
        for (int j = 0; j < rows_local; j++) {
            const int y = row_offset + j * row_stride;
            for (int x = 0; x < w; x++) {
                rtk::Col f = rtk::trace_pixel(C, x, y, stack.data(), ps);
                rtk::tonemap_into(out + 4 * ((size_t)(shard ? j : y) * w + x), f);
            }
        }
    }
    c->last_kernel_ms = (omp_get_wtime() - t0) * 1e3;
    merge_stats(c, st);
    return RT_OK;
}

int rt_backend_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    rtk::Ctx C{rt_host_view(c), c->cam, w, h, spp, bounces};
    std::vector<rtk::Stats> st(omp_get_max_threads());
    for (auto& s : st) std::memset(&s, 0, sizeof s);
#pragma omp parallel
    {
        std::vector<rtk::StackEnt> stack(RT_STACK_CAP);
        rtk::Stats* ps = c->stats_enabled ? &st[omp_get_thread_num()] : nullptr;
#pragma omp for schedule(dynamic, 8)
        for (int i = 0; i < n; i++) {
            rtk::Col f = rtk::trace_pixel(C, xy[2 * i], xy[2 * i + 1], stack.data(), ps);
            rtk::tonemap_into(rgba + 4 * (size_t)i, f);
        }
    }
    merge_stats(c, st);
    return RT_OK;
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
            rtk::Hit h;
            bool f = rtk::intersect_scene(S, rtk::v3(r[0], r[1], r[2]), rtk::v3(r[3], r[4], r[5]), stack.data(), h, ps);
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
