// rt_capi_host.cpp — the backend-independent half of the C ABI
// (include/rt_hip.h): argument checking, host scene preparation, host
// helpers. The compute half lives in rt_render.hip (gfx950).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "rt_context.h"

namespace {
std::mutex g_err_mu;
std::string g_err;
thread_local std::string* tl_sink = nullptr;  // rt_err_sink
void set_global_err(const std::string& m)
{
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = m;
}
}  // namespace

void rt_err_sink(std::string* sink) { tl_sink = sink; }

void rt_read_diag(rt_context* c)
{
    if (const char* e = std::getenv("RT_TIMELINE")) c->diag.timeline = e;
    if (const char* e = std::getenv("RT_ITER_LOG")) c->diag.iter_log = e;
    c->diag.verbose = std::getenv("RT_VERBOSE") != nullptr;
}

int rt_fail(rt_context* ctx, int code, const std::string& msg)
{
    if (tl_sink) {  // a device thread of a multi-device render: its own slot (rt_for_devices)
        *tl_sink = msg;
        return code;
    }
    if (ctx) {
        std::lock_guard<std::mutex> lk(g_err_mu);
        ctx->err = msg;
    }
    set_global_err(msg);
    return code;
}

RtSceneView rt_host_view(const rt_context* c)
{
    RtSceneView v{};
    v.nodes = c->flat.nodes.data();
    v.tri4 = c->flat.tri4.data();
    v.prim2k = c->flat.prim2k.data();
    v.mat_idx = c->mat_idx.data();
    v.mats = c->mats.data();
    v.n_mats = (int)c->mats.size();
    v.emissive = c->emissive.data();
    v.spheres = c->spheres.data();
    v.env = c->env.data();
    v.env_lum = c->env_lum.data();
    v.cdf = c->cdf.data();
    v.brute = c->brute ? 1 : 0;
    v.cdf_row = c->cdf_row.data();
    v.cdf_fence = c->cdf_fence.empty() ? nullptr : c->cdf_fence.data();
    v.cdf_coarse = c->cdf_coarse.data();
    v.cdf_cw = c->cdf_cw;
    v.cdf_total = c->cdf.empty() ? 0.0f : c->cdf.back();
    v.n_emissive = (int)c->emissive.size();
    v.n_spheres = (int)(c->spheres.size() / 2);
    v.ew = c->ew;
    v.eh = c->eh;
    v.n_tris = (int)(c->tris.size() / 9);
    v.chain_monotone = c->flat.chain_monotone ? 1 : 0;
    v.bvh4 = c->flat.bvh4.data();
    v.bvh16 = c->flat.bvh16.data();
    v.bvh4s = c->flat.bvh4s.data();
    v.bvh16s = c->flat.bvh16s.data();
    v.bvh_tri4 = c->flat.bvh_tri4.data();
    v.parent = c->flat.parent.data();
    v.leaf_of = c->flat.leaf_of.data();
    v.tri_mat = 0;
    rt_view_near(c, v);
    return v;
}

void rt_view_near(const rt_context* c, RtSceneView& v)
{
    const double scale = c->sched.near_scale >= 0.0 ? c->sched.near_scale : RT_NEAR_SCALE;
    // the scene's box: the octree root's axis planes (PLANE_NORMALS 0-2 are the axes: the
    // vertices' min / max) and every analytic sphere's box
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, ext = 0.0;
    if (!c->flat.nodes.empty())
        for (int i = 0; i < 3; i++) lo[i] = c->flat.nodes[0].dn[i], hi[i] = c->flat.nodes[0].df[i];
    for (size_t k = 0; k + 1 < c->spheres.size(); k += 2) {
        const float4_& sp = c->spheres[k];
        const double cc[3] = {sp.x, sp.y, sp.z}, r = std::fabs((double)sp.w);
        for (int i = 0; i < 3; i++) lo[i] = std::min(lo[i], cc[i] - r), hi[i] = std::max(hi[i], cc[i] + r);
    }
    bool have = true;
    for (int i = 0; i < 3; i++) {
        if (!(lo[i] <= hi[i]) || !std::isfinite(lo[i]) || !std::isfinite(hi[i])) have = false;
        else ext = std::max(ext, hi[i] - lo[i]);
    }
    for (int i = 0; i < 3; i++) {
        const double w = have ? scale * ext : 0.0;
        // rounded outwards; beyond float range (or no scene): unbounded
        v.near_lo[i] = have ? std::nextafter((float)(lo[i] - w), -INFINITY) : -INFINITY;
        v.near_hi[i] = have ? std::nextafter((float)(hi[i] + w), INFINITY) : INFINITY;
    }
}

bool rt_table_has_emissive_prim(const rt_context* c, const RtMat* table)
{
    for (int32_t mi : c->mat_idx) {
        const RtMat& m = table[mi];
        if (m.er > 0 || m.eg > 0 || m.eb > 0) return true;
    }
    return false;
}

bool rt_scene_has_emissive_prim(const rt_context* c) { return rt_table_has_emissive_prim(c, c->mats.data()); }

extern "C" {

int rt_version(void) { return 10000; }

const char* rt_last_error(const rt_context* ctx)
{
    if (ctx) return ctx->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    static thread_local std::string copy;
    copy = g_err;
    return copy.c_str();
}

int rt_create(int device, rt_context** out)
{
    if (!out) return rt_fail(nullptr, RT_ERR_ARG, "rt_create: out is NULL");
    *out = nullptr;
    rt_context* c = new rt_context();
    c->device = device;
    rt_read_diag(c);
    int r = rt_backend_create(c);
    if (r) {
        set_global_err(c->err);
        rt_backend_destroy(c);
        delete c;
        return r;
    }
    *out = c;
    return RT_OK;
}

}  // extern "C"

namespace {
// ids: non-negative and distinct (one rank per GPU in the RCCL clique); the range is
// checked against the devices present when the backend opens them (RT_ERR_NODEV).
// loopback (rt_create_multi_loopback, tests only) admits a list that names a GPU more
// than once: the context then exchanges the shards with device copies instead of RCCL.
// rccl (rt_test_create_multi_rccl, tests only): the multi-device driver and its RCCL clique
// even for one listed device (a one-rank ncclCommInitAll), so a one-GPU box runs the pack,
// ncclScatter, render, ncclGather and un-permute sequence the 8-GPU node runs.
int create_multi(int n_devices, const int* devices, bool loopback, rt_context** out, bool rccl = false)
{
    if (!out) return rt_fail(nullptr, RT_ERR_ARG, "rt_create_multi: out is NULL");
    *out = nullptr;
    if (n_devices < 1 || n_devices > 64) return rt_fail(nullptr, RT_ERR_ARG, "rt_create_multi: n_devices must be 1..64");
    for (int d = 0; d < n_devices; d++) {
        const int id = devices ? devices[d] : d;
        if (id < 0) return rt_fail(nullptr, RT_ERR_ARG, "rt_create_multi: negative device id");
        for (int e = 0; e < d; e++)
            if ((devices ? devices[e] : e) == id && !loopback)
                return rt_fail(nullptr, RT_ERR_ARG, "rt_create_multi: device " + std::to_string(id) + " listed twice");
    }
    rt_context* c = new rt_context();
    for (int d = 0; d < n_devices; d++) c->devices.push_back(devices ? devices[d] : d);
    c->device = c->devices[0];
    c->loopback = loopback;
    c->force_multi = rccl;
    rt_read_diag(c);
    int r = rt_backend_create(c);
    if (r) {
        set_global_err(c->err);
        rt_backend_destroy(c);
        delete c;
        return r;
    }
    *out = c;
    return RT_OK;
}
}  // namespace

extern "C" {
int rt_create_multi(int n_devices, const int* devices, rt_context** out)
{
    return create_multi(n_devices, devices, false, out);
}

int rt_create_multi_loopback(int n_devices, const int* devices, rt_context** out)
{
    return create_multi(n_devices, devices, true, out);
}

int rt_test_create_multi_rccl(int n_devices, const int* devices, rt_context** out)
{
    return create_multi(n_devices, devices, false, out, true);
}

int rt_test_fail_device(rt_context* c, int device)
{
    if (!c) return rt_fail(nullptr, RT_ERR_ARG, "rt_test_fail_device: ctx is NULL");
    c->fail_device = device;
    return RT_OK;
}

int rt_test_schedule(rt_context* c, const char* key, double value)
{
    if (!c || !key) return rt_fail(c, RT_ERR_ARG, "rt_test_schedule: ctx or key is NULL");
    RtSchedule& s = c->sched;
    const std::string k = key;
    // (finite for every key; in int range for the integer ones: the cast is otherwise undefined)
    const bool real_key = k == "tail_enter" || k == "fast_spp" || k == "near_scale";
    if (!std::isfinite(value) || (!real_key && (value < -2147483648.0 || value > 2147483647.0)))
        return rt_fail(c, RT_ERR_ARG, "rt_test_schedule: value of " + k + " is out of range");
    const int v = real_key ? 0 : (int)value;
    if (k == "lanes") s.lanes = std::max(0, v);
    else if (k == "tail_paths") s.tail_paths = v;
    else if (k == "tail_enter") s.tail_enter = value;
    else if (k == "tail_rows") s.tail_rows = v;
    else if (k == "drain_rows") s.drain_rows = std::min(4, v);
    else if (k == "heavy_calls") s.heavy_calls = v;
    else if (k == "spec_cam") s.spec_cam = std::min(2, v);
    else if (k == "tail_spec_cam") s.tail_spec_cam = std::min(2, v);
    else if (k == "force_fallback") s.force_fallback = std::max(0, v);
    else if (k == "step_budget") s.step_budget = v;
    else if (k == "fast_k") s.fast_k = v;
    else if (k == "fast_spp") s.fast_spp = value;
    else if (k == "near_scale") s.near_scale = value;
    else if (k == "reset") s = RtSchedule{};
    else return rt_fail(c, RT_ERR_ARG, "rt_test_schedule: unknown key " + k);
    return RT_OK;
}

int rt_test_obj_parallel_min(long bytes)
{
    rt::g_obj_parallel_min.store(bytes < 0 ? -1 : bytes);
    return RT_OK;
}

int rt_test_walk_log(rt_context* c, int min_calls, int sample_every, int capacity)
{
    if (!c || min_calls < 0 || capacity < 0) return rt_fail(c, RT_ERR_ARG, "rt_test_walk_log: bad arguments");
    c->diag.wlog_min = min_calls;
    c->diag.wlog_every = sample_every < 0 ? -1 : std::max(1, sample_every);
    c->diag.wlog_cap = min_calls > 0 ? capacity : 0;
    c->diag.wlog.clear();
    c->diag.wlog_total = 0;
    return RT_OK;
}

long rt_test_walk_log_read(const rt_context* c, float* out, long capacity)
{
    if (!c || capacity < 0 || (capacity > 0 && !out)) return rt_fail(nullptr, RT_ERR_ARG, "rt_test_walk_log_read: bad arguments");
    const long n = (long)(c->diag.wlog.size() / RT_WLOG_FLOATS);
    const long m = std::min(n, capacity);
    if (m > 0) std::memcpy(out, c->diag.wlog.data(), (size_t)m * RT_WLOG_FLOATS * sizeof(float));
    return c->diag.wlog_total;
}

int rt_device_count(const rt_context* ctx) { return ctx ? (ctx->devices.empty() ? 1 : (int)ctx->devices.size()) : RT_ERR_ARG; }

void rt_destroy(rt_context* ctx)
{
    if (!ctx) return;
    rt_backend_destroy(ctx);
    delete ctx;
}

int rt_set_scene(rt_context* c, const float* triangles, int n, const int* material_indices, int n_mi,
                 const float* materials, int n_mats, const int* emissive, int n_em, const float* spheres, int n_sph)
{
    if (!c) return rt_fail(nullptr, RT_ERR_ARG, "rt_set_scene: ctx is NULL");
    if (n < 0 || (n > 0 && !triangles) || n_mats <= 0 || !materials || n_mi < n || (n_mi > 0 && !material_indices) ||
        n_em < 0 || (n_em > 0 && !emissive) || n_sph < 0 || (n_sph > 0 && !spheres))
        return rt_fail(c, RT_ERR_ARG, "rt_set_scene: bad buffer sizes");
    for (int i = 0; i < n_mi; i++)
        if (material_indices[i] < 0 || material_indices[i] >= n_mats)
            return rt_fail(c, RT_ERR_ARG, "rt_set_scene: material index out of range");
    for (int i = 0; i < n_em; i++)
        if (emissive[i] < 0 || emissive[i] >= n) return rt_fail(c, RT_ERR_ARG, "rt_set_scene: emissive id out of range");
    for (int i = 0; i < n_sph; i++) {
        const int prim = (int)spheres[5 * i + 4];
        if (prim < 0 || prim >= n_mi)
            return rt_fail(c, RT_ERR_ARG, "rt_set_scene: sphere primitive index has no material index");
    }
    c->tris.assign(triangles, triangles + 9 * (size_t)n);
    c->mat_idx.assign(material_indices, material_indices + n_mi);
    c->mats.resize(n_mats);
    for (int i = 0; i < n_mats; i++) {
        const float* p = materials + 10 * (size_t)i;
        c->mats[i] = RtMat{p[0], p[1], p[2], p[8], p[4], p[5], p[6], p[9]};
    }
    c->emissive.assign(emissive, emissive + n_em);
    c->spheres.clear();
    for (int i = 0; i < n_sph; i++) {
        const float* p = spheres + 5 * (size_t)i;
        float4_ a{p[0], p[1], p[2], p[3]}, b{0, 0, 0, 0};
        const int prim = (int)p[4];
        std::memcpy(&b.x, &prim, 4);
        c->spheres.push_back(a);
        c->spheres.push_back(b);
    }
    c->have_scene = true;
    c->have_bvh = false;
    c->dirty = true;
    return RT_OK;
}

int rt_set_materials(rt_context* c, const float* materials, int n_mats)
{
    if (!c || !c->have_scene) return rt_fail(c, RT_ERR_STATE, "rt_set_materials: no scene");
    if (n_mats <= 0 || !materials) return rt_fail(c, RT_ERR_ARG, "rt_set_materials: bad buffer");
    for (int32_t mi : c->mat_idx)
        if (mi >= n_mats) return rt_fail(c, RT_ERR_ARG, "rt_set_materials: a material index is out of range");
    c->mats.resize(n_mats);
    for (int i = 0; i < n_mats; i++) {
        const float* p = materials + 10 * (size_t)i;
        c->mats[i] = RtMat{p[0], p[1], p[2], p[8], p[4], p[5], p[6], p[9]};
    }
    c->mats_dirty_only = true;  // the octree, search BVH, triangles and env stay on the device
    return RT_OK;
}

int rt_build_bvh(rt_context* c, int max_depth, int leaf_max)
{
    if (!c || !c->have_scene) return rt_fail(c, RT_ERR_STATE, "rt_build_bvh: no scene");
    if (max_depth > 32 || max_depth < -1 || leaf_max < 1)
        return rt_fail(c, RT_ERR_ARG, "rt_build_bvh: max_depth must be -1..32 (device stack bound), leaf_max >= 1");
    const int n = (int)(c->tris.size() / 9);
    rt::build_octree(c->tris.data(), n, max_depth, leaf_max, c->octree);
    rt::flatten_octree(c->octree, c->tris.data(), n, c->flat);
    if (c->flat.max_depth > 32) return rt_fail(c, RT_ERR_ARG, "rt_build_bvh: octree deeper than 32");
    rt::build_search_bvh(c->flat);
    c->have_bvh = true;
    c->dirty = true;
    return RT_OK;
}

int rt_set_bvh_preorder(rt_context* c, const void* dump, long bytes)
{
    if (!c || !c->have_scene) return rt_fail(c, RT_ERR_STATE, "rt_set_bvh_preorder: no scene");
    if (!dump || bytes <= 0) return rt_fail(c, RT_ERR_ARG, "rt_set_bvh_preorder: empty dump");
    rt::Octree t;
    if (rt::octree_from_dump((const char*)dump, (size_t)bytes, t))
        return rt_fail(c, RT_ERR_ARG, "rt_set_bvh_preorder: malformed pre-order dump");
    const int n = (int)(c->tris.size() / 9);
    for (const auto& nd : t.pool)
        for (int id : nd.tris)
            if (id < 0 || id >= n) return rt_fail(c, RT_ERR_ARG, "rt_set_bvh_preorder: triangle id out of range");
    c->octree = std::move(t);
    rt::flatten_octree(c->octree, c->tris.data(), n, c->flat);
    if (c->flat.max_depth > 32) return rt_fail(c, RT_ERR_ARG, "rt_set_bvh_preorder: octree deeper than 32");
    rt::build_search_bvh(c->flat);
    c->have_bvh = true;
    c->dirty = true;
    return RT_OK;
}

long rt_bvh_dump(const rt_context* c, void* buf, long cap)
{
    if (!c || !c->have_bvh) return RT_ERR_STATE;
    std::vector<char> d = rt::dump_octree(c->octree);
    if (buf && cap >= (long)d.size()) std::memcpy(buf, d.data(), d.size());
    return (long)d.size();
}

int rt_bvh_info(const rt_context* c, long* info)
{
    if (!c || !c->have_bvh || !info) return RT_ERR_STATE;
    info[0] = (long)c->octree.pool.size();
    info[1] = (long)c->flat.nodes.size();
    info[2] = (long)(c->tris.size() / 9);
    info[3] = c->flat.max_depth;
    info[4] = (long)(c->flat.nodes.size() * sizeof(RtNode) + c->flat.tri4.size() * sizeof(float4_) +
                     c->flat.prim2k.size() * 4 + c->flat.parent.size() * 4 + c->flat.leaf_of.size() * 4 +
                     c->flat.bvh4.size() * sizeof(Bvh4Node) + c->flat.bvh_tri4.size() * sizeof(float4_));
    return RT_OK;
}

int rt_set_env(rt_context* c, const float* px, int w, int h, int ch, const float* cdf)
{
    if (!c) return rt_fail(nullptr, RT_ERR_ARG, "rt_set_env: ctx is NULL");
    if (!px || w <= 0 || h <= 0 || (ch != 3 && ch != 4)) return rt_fail(c, RT_ERR_ARG, "rt_set_env: bad image");
    const size_t n = (size_t)w * h;
    c->ew = w;
    c->eh = h;
    c->env_lum.resize(n);
    c->cdf.resize(n);
    rt::env_luminance_cdf(px, w, h, ch, c->env_lum.data(), c->cdf.data());
    if (cdf) c->cdf.assign(cdf, cdf + n);
    // RGB + the texel's luminance in w: the env-map sample reads both with one 16-B load
    c->env.resize(n);
    for (size_t i = 0; i < n; i++) c->env[i] = float4_{px[ch * i], px[ch * i + 1], px[ch * i + 2], c->env_lum[i]};
    c->cdf_row.assign((size_t)((h + 15) & ~15), 0.0f);  // (padded: the fence search loads 16 at a time)
    for (int y = 0; y < h; y++) c->cdf_row[y] = c->cdf[(size_t)y * w + w - 1];
    rt::env_cdf_fences(c->cdf.data(), c->cdf_row.data(), w, h, c->cdf_fence);
    c->cdf_cw = w / 32;
    c->cdf_coarse.resize(std::max<size_t>(1, (size_t)h * c->cdf_cw));
    for (int y = 0; y < h; y++)
        for (int j = 0; j < c->cdf_cw; j++) c->cdf_coarse[(size_t)y * c->cdf_cw + j] = c->cdf[(size_t)y * w + 32 * j + 31];
    c->have_env = true;
    c->dirty = true;
    return RT_OK;
}

int rt_set_camera(rt_context* c, const float view[16], float fov_dist)
{
    if (!c || !view) return rt_fail(c, RT_ERR_ARG, "rt_set_camera: bad arguments");
    std::memcpy(c->cam.m, view, 64);
    c->cam.fov_dist = fov_dist;
    c->have_cam = true;
    return RT_OK;
}

static int check_ready(rt_context* c, int w, int h, int spp, int bounces)
{
    if (!c) return rt_fail(nullptr, RT_ERR_ARG, "ctx is NULL");
    if (!c->have_scene || !c->have_bvh) return rt_fail(c, RT_ERR_STATE, "scene/BVH not set");
    if (!c->have_env) return rt_fail(c, RT_ERR_STATE, "environment map not set");
    if (!c->have_cam) return rt_fail(c, RT_ERR_STATE, "camera not set");
    if (w <= 0 || h <= 0 || spp <= 0 || bounces < 0) return rt_fail(c, RT_ERR_ARG, "bad render size");
    // the reference seeds with the int 31 + x*y*spp (render_kernel.cpp:77)
    if ((double)(w - 1) * (double)(h - 1) * (double)spp + 31.0 > 2147483647.0)
        return rt_fail(c, RT_ERR_ARG, "31 + x*y*spp overflows int (reference seed)");
    if (c->dirty || c->mats_dirty_only) {
        int r = rt_backend_upload(c);
        if (r) return r;
        c->dirty = false;
        c->mats_dirty_only = false;
    }
    return RT_OK;
}

int rt_render(rt_context* c, int w, int h, int spp, int bounces, float* fb)
{
    if (int r = check_ready(c, w, h, spp, bounces)) return r;
    if (!fb) return rt_fail(c, RT_ERR_ARG, "rt_render: fb is NULL");
    return rt_backend_render(c, w, h, spp, bounces, fb, nullptr, 0, 1, nullptr);
}

int rt_render_device(rt_context* c, int w, int h, int spp, int bounces, void* d_fb, int row_offset, int row_stride,
                     void* stream)
{
    if (int r = check_ready(c, w, h, spp, bounces)) return r;
    if (!d_fb || row_stride <= 0 || row_offset < 0 || row_offset >= row_stride)
        return rt_fail(c, RT_ERR_ARG, "rt_render_device: bad shard");
    return rt_backend_render(c, w, h, spp, bounces, nullptr, d_fb, row_offset, row_stride, stream);
}

int rt_render_variants(rt_context* c, int w, int h, int spp, int bounces, int n_var, const float* materials,
                       int n_mats, int row_offset, int row_stride, float* fb, void* const* d_fbs)
{
    if (int r = check_ready(c, w, h, spp, bounces)) return r;
    if (n_var <= 0 || !materials || n_mats <= 0 || (fb == nullptr) == (d_fbs == nullptr))
        return rt_fail(c, RT_ERR_ARG, "rt_render_variants: bad buffers (exactly one of fb_rgba / d_fbs)");
    if (row_stride <= 0 || row_offset < 0 || row_offset >= row_stride)
        return rt_fail(c, RT_ERR_ARG, "rt_render_variants: bad row shard");
    for (int32_t mi : c->mat_idx)
        if (mi >= n_mats) return rt_fail(c, RT_ERR_ARG, "rt_render_variants: a material index is out of range");
    if (d_fbs)
        for (int v = 0; v < n_var; v++)
            if (!d_fbs[v]) return rt_fail(c, RT_ERR_ARG, "rt_render_variants: null device buffer");
    std::vector<RtMat> tabs((size_t)n_var * n_mats);
    for (size_t i = 0; i < tabs.size(); i++) {
        const float* p = materials + 10 * i;
        tabs[i] = RtMat{p[0], p[1], p[2], p[8], p[4], p[5], p[6], p[9]};
    }
    const int r = rt_backend_render_variants(c, w, h, spp, bounces, n_var, tabs, n_mats, row_offset, row_stride, fb, d_fbs);
    c->mats_dirty_only = true;  // the devices' tables hold the last variants: the next render re-sends the bound one
    return r;
}

int rt_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    if (int r = check_ready(c, w, h, spp, bounces)) return r;
    if (n < 0 || (n > 0 && (!xy || !rgba))) return rt_fail(c, RT_ERR_ARG, "rt_render_pixels: bad buffers");
    for (int i = 0; i < n; i++)
        if (xy[2 * i] < 0 || xy[2 * i] >= w || xy[2 * i + 1] < 0 || xy[2 * i + 1] >= h)
            return rt_fail(c, RT_ERR_ARG, "rt_render_pixels: pixel outside the image");
    if (n == 0) return RT_OK;
    return rt_backend_render_pixels(c, w, h, spp, bounces, xy, n, rgba);
}

int rt_intersect(rt_context* c, const float* rays, int n, void* out)
{
    if (!c || !c->have_scene || !c->have_bvh) return rt_fail(c, RT_ERR_STATE, "rt_intersect: scene/BVH not set");
    if (n < 0 || (n > 0 && (!rays || !out))) return rt_fail(c, RT_ERR_ARG, "rt_intersect: bad buffers");
    if (n == 0) return RT_OK;
    if (c->dirty) {
        if (!c->have_env) {
            // a 1x1 black env keeps the device view valid for ray queries
            const float z[3] = {0, 0, 0};
            rt_set_env(c, z, 1, 1, 3, nullptr);
        }
        int r = rt_backend_upload(c);
        if (r) return r;
        c->dirty = false;
        c->mats_dirty_only = false;
    }
    return rt_backend_intersect(c, rays, n, out);
}

int rt_set_intersect_mode(rt_context* c, int use_bvh)
{
    if (!c) return RT_ERR_ARG;
    c->brute = use_bvh == 0;
    c->dirty = true;
    return RT_OK;
}

int rt_set_stats(rt_context* c, int enabled)
{
    if (!c) return RT_ERR_ARG;
    c->stats_enabled = enabled != 0;
    c->stats_seq = enabled == 2;
    return RT_OK;
}

int rt_get_stats(const rt_context* c, unsigned long long* out, int n)
{
    if (!c || !out) return RT_ERR_ARG;
    for (int i = 0; i < n && i < 2 * RT_STAT_COUNT; i++) out[i] = c->stats[i];
    return RT_OK;
}

double rt_last_kernel_ms(const rt_context* c) { return c ? c->last_kernel_ms : -1.0; }

// ------------------------------------------------------------- host helpers
struct rt_mesh {
    rt::Mesh m;
};

int rt_mesh_load(const char* path, rt_mesh** out)
{
    if (!path || !out) return rt_fail(nullptr, RT_ERR_ARG, "rt_mesh_load: bad arguments");
    *out = nullptr;
    rt_mesh* m = new rt_mesh();
    std::string err;
    int r = rt::load_obj(path, m->m, err);
    if (r) {
        delete m;
        return rt_fail(nullptr, RT_ERR_IO, "rt_mesh_load: " + err);
    }
    *out = m;
    return RT_OK;
}

int rt_mesh_counts(const rt_mesh* m, int* nt, int* nm, int* ne)
{
    if (!m) return RT_ERR_ARG;
    if (nt) *nt = m->m.ntris();
    if (nm) *nm = (int)(m->m.mats.size() / 10);
    if (ne) *ne = (int)m->m.emissive.size();
    return RT_OK;
}

int rt_mesh_copy(const rt_mesh* m, float* tris, int* mi, float* mats, int* em)
{
    if (!m) return RT_ERR_ARG;
    if (tris) std::memcpy(tris, m->m.tris.data(), m->m.tris.size() * 4);
    if (mi) std::memcpy(mi, m->m.mat_idx.data(), m->m.mat_idx.size() * 4);
    if (mats) std::memcpy(mats, m->m.mats.data(), m->m.mats.size() * 4);
    if (em) std::memcpy(em, m->m.emissive.data(), m->m.emissive.size() * 4);
    return RT_OK;
}

void rt_mesh_free(rt_mesh* m) { delete m; }

int rt_camera_preset(const char* name, float view[16], float* fov_dist)
{
    if (!name || !view || !fov_dist) return RT_ERR_ARG;
    return rt::camera_preset(name, view, fov_dist) ? rt_fail(nullptr, RT_ERR_ARG, "unknown camera preset") : RT_OK;
}

int rt_env_luminance_cdf(const float* px, int w, int h, int ch, float* lum, float* cdf)
{
    if (!px || w <= 0 || h <= 0 || (ch != 3 && ch != 4) || !lum || !cdf) return RT_ERR_ARG;
    rt::env_luminance_cdf(px, w, h, ch, lum, cdf);
    return RT_OK;
}

long rt_octree_dump(const float* tris, int n, int max_depth, int leaf_max, void* buf, long cap)
{
    if (!tris || n < 0) return RT_ERR_ARG;
    rt::Octree t;
    rt::build_octree(tris, n, max_depth, leaf_max, t);
    std::vector<char> d = rt::dump_octree(t);
    if (buf && cap >= (long)d.size()) std::memcpy(buf, d.data(), d.size());
    return (long)d.size();
}

}  // extern "C"

// ------------------------------------------------------------- image I/O
int rt_read_hdr(const char* path, int flip_y, int* width, int* height, float* pixels_rgba)
{
    if (!path || !width || !height) return rt_fail(nullptr, RT_ERR_ARG, "rt_read_hdr: bad arguments");
    int w = 0, h = 0;
    std::vector<float> rgb;
    std::string err;
    if (rt::read_hdr(path, flip_y != 0, w, h, rgb, err)) return rt_fail(nullptr, RT_ERR_IO, "rt_read_hdr: " + err);
    if (pixels_rgba) {
        if (*width != w || *height != h) return rt_fail(nullptr, RT_ERR_ARG, "rt_read_hdr: buffer size does not match the image");
        for (size_t i = 0; i < (size_t)w * h; i++) {  // Color(r, g, b, 0.0f): utils.cpp:114-120
            pixels_rgba[4 * i] = rgb[3 * i];
            pixels_rgba[4 * i + 1] = rgb[3 * i + 1];
            pixels_rgba[4 * i + 2] = rgb[3 * i + 2];
            pixels_rgba[4 * i + 3] = 0.0f;
        }
    }
    *width = w;
    *height = h;
    return RT_OK;
}

int rt_image_to_rgba8(const float* rgba, long n_pixels, unsigned char* out)
{
    if (n_pixels < 0 || (n_pixels > 0 && (!rgba || !out))) return rt_fail(nullptr, RT_ERR_ARG, "rt_image_to_rgba8: bad arguments");
    rt::rgba8(rgba, (size_t)n_pixels, out);
    return RT_OK;
}

int rt_write_png(const char* path, const float* rgba, int width, int height, int flip_y)
{
    if (!path || (width > 0 && height > 0 && !rgba)) return rt_fail(nullptr, RT_ERR_ARG, "rt_write_png: bad arguments");
    std::string err;
    if (rt::write_png(path, rgba, width, height, flip_y != 0, err)) return rt_fail(nullptr, RT_ERR_IO, "rt_write_png: " + err);
    return RT_OK;
}

