// rt_context.h — the state behind an rt_context* (include/rt_hip.h).
//
// Host-side scene state is shared; the compute backend (rt_render.hip for
// gfx950, rt_hostsim.cpp for the CPU debugging build used by the CPU test
// suite) implements the rt_backend_* hooks.
#pragma once

#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_device.h"
#include "rt_scene.h"

// Schedule of the wavefront loop (rt_render.hip run_wave). The product runs the defaults
// (-1: the backend's own choice); rt_test_schedule (tests and measurement tools only,
// include/rt_hip.h) overrides them per context. No parameter changes a pixel: the GPU
// schedule tests render with each and compare the bits. Nothing here is read from the
// environment.
struct RtSchedule {
    int lanes = 0;             // wavefront lanes per render (0: auto, rt_device_set_lanes)
    int tail_paths = -1;       // k_tail paths per wave (0: no tail kernel)
    double tail_enter = -1.0;  // k_tail entry: live paths per lane, in grid-fills' pools
    int tail_rows = -1;        // k_tail walks by rows (1) or quads (0)
    int drain_rows = -1;       // k_trace: a drain's last walks continue as rows (0: off)
    int heavy_calls = -1;      // k_trace heavy class threshold in quad_visit calls (0: off)
    int spec_cam = -1;         // camera ray traced ahead: 0 never, 1 always, 2 where the last sample ended
    int tail_spec_cam = -1;    // the same in k_tail
    int force_fallback = 0;    // stressor: every k-th query (by a ray hash) skips to the exact walk
    int step_budget = -1;      // exact-walk steps per query per launch before it parks
    int fast_k = -1;           // fast lane: this many of the slowest paths to a tail kernel early (0: off)
    double fast_spp = -1.0;    // ... at the lanes' first readback from iteration fast_spp x spp on
    double near_scale = -1.0;  // near box: the scene's box widened by this x its largest extent (rt_view_near;
                               // study probes only: answers never depend on it, only which walk gives them)
};

// Diagnostics, read from the environment once when the context is created (rt_create*):
// RT_TIMELINE (per-launch timeline file), RT_ITER_LOG (per-iteration log prefix),
// RT_VERBOSE. They change no result and no schedule.
struct RtDiag {
    std::string timeline, iter_log;
    bool verbose = false;
    // walk log (rt_test_walk_log): stats renders record every search-BVH walk of at least
    // min_calls quad_visit calls (row trips count 2), up to cap records of RT_WLOG_FLOATS
    int wlog_min = 0, wlog_cap = 0, wlog_every = 1;
    std::vector<float> wlog;  // the last stats render's records
    long wlog_total = 0;      // walks that qualified (may exceed cap)
};

struct rt_context {
    int device = 0;
    RtSchedule sched;
    RtDiag diag;
    // rt_create_multi: the devices a render shards over (rows y -> device y mod N, RCCL
    // scatter / gather through devices[0]); empty for a single-device context (rt_create).
    // One entry: a single-device context on that ordinal (nothing to shard, no RCCL)
    std::vector<int> devices;
    bool loopback = false;        // devices may repeat: shards exchanged by device copies, not RCCL
    bool force_multi = false;     // (rt_test_create_multi_rccl) the multi-device driver and RCCL even for one device
    int fail_device = -1;         // rt_test_fail_device (tests only): that device fails its share
    std::string err;

    // RenderKernel constructor inputs (render_kernel.h:27-34)
    std::vector<float> tris;      // [N][9]
    std::vector<int32_t> mat_idx; // >= N entries (spheres append theirs)
    std::vector<RtMat> mats;
    std::vector<int32_t> emissive;
    std::vector<float4_> spheres; // 2 records per sphere
    bool have_scene = false;

    rt::Octree octree;
    rt::FlatBvh flat;
    bool have_bvh = false;

    std::vector<float4_> env;     // RGBA, alpha 0
    std::vector<float> env_lum, cdf;
    std::vector<float> cdf_row, cdf_coarse;  // exact copies of CDF entries (rt_trace.h cdf_search)
    std::vector<float> cdf_fence;            // fence tables of the counting search (empty: not eligible)
    int cdf_cw = 0;
    int ew = 0, eh = 0;
    bool have_env = false;

    RtCamera cam{};
    bool have_cam = false;

    bool brute = false;           // USE_BVH 0 (rt_set_intersect_mode)
    bool stats_enabled = false;
    bool stats_seq = false;       // rt_set_stats(ctx, 2): occlusion walks unpaired (gfx950), see rt_hip.h
    unsigned long long stats[2 * RT_STAT_COUNT] = {};  // all kernels, then the gfx950 tail kernel's share
    double last_kernel_ms = 0.0;

    bool dirty = true;            // host state changed since the last upload
    bool mats_dirty_only = false; // only the material table changed (rt_set_materials)
    void* backend = nullptr;
};

// ---- backend hooks
int rt_backend_create(rt_context* ctx);
void rt_backend_destroy(rt_context* ctx);
int rt_backend_upload(rt_context* ctx);
int rt_backend_render(rt_context* ctx, int w, int h, int spp, int bounces, float* host_fb, void* dev_fb, int row_offset,
                      int row_stride, void* stream);
// n_variants material tables (RtMat, n_mats each, back to back); variant v on device v mod N
int rt_backend_render_variants(rt_context* ctx, int w, int h, int spp, int bounces, int n_variants,
                               const std::vector<RtMat>& tables, int n_mats, int row_offset, int row_stride,
                               float* host_fb, void* const* d_fbs);
// rt_scene_has_emissive_prim for another material table over the context's material indices
bool rt_table_has_emissive_prim(const rt_context* ctx, const RtMat* table);
int rt_backend_render_pixels(rt_context* ctx, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba);
int rt_backend_intersect(rt_context* ctx, const float* rays, int n, void* out);

int rt_fail(rt_context* ctx, int code, const std::string& msg);
// RtDiag from the environment (rt_create*)
void rt_read_diag(rt_context* ctx);
// While set (per host thread), rt_fail writes its message to *sink instead of the
// context: the per-device threads of a multi-device render report into their own
// slots, and the caller raises the error once, after the join (rt_for_devices).
void rt_err_sink(std::string* sink);

// fn(d) for every device d of a multi-device render: d >= 1 on threads of their own,
// d = 0 on the caller's. Each device's errors go to its own slot; after the join the
// lowest failing device's code and message are raised on the context (one writer).
// c->fail_device (rt_test_fail_device, tests only) fails that device before its work starts.
template <class F>
int rt_for_devices(rt_context* c, int n, F fn)
{
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    const int inject = c->fail_device;
    auto one = [&](int d) {
        rt_err_sink(&msg[d]);
        rc[d] = d == inject ? rt_fail(c, RT_ERR_STATE, "injected failure (rt_test_fail_device)") : fn(d);
        rt_err_sink(nullptr);
    };
    {
        std::vector<std::thread> th;
        for (int d = 1; d < n; d++) th.emplace_back(one, d);
        one(0);
        for (auto& t : th) t.join();
    }
    for (int d = 0; d < n; d++)
        if (rc[d]) return rt_fail(c, rc[d], "device " + std::to_string(d) + ": " + msg[d]);
    return 0;
}
RtSceneView rt_host_view(const rt_context* ctx);  // host-memory view (hostsim)
// The view's near box (rt_fast.h far_origin): the octree root's axis planes (the scene's box)
// widened on every side by RT_NEAR_SCALE (or sched.near_scale) x the box's largest extent;
// unbounded for an empty scene.
#ifndef RT_NEAR_SCALE
#define RT_NEAR_SCALE 0.5
#endif
void rt_view_near(const rt_context* ctx, RtSceneView& v);
// Does any primitive (triangle or sphere) use a material with a positive
// emission component (the test at render_kernel.cpp:696)? If not, the
// BRDF->light query of sample_light_sources can never contribute.
bool rt_scene_has_emissive_prim(const rt_context* ctx);
