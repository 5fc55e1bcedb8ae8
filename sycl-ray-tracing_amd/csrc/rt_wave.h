// rt_wave.h — the wavefront form of RenderKernel::ray_trace_pixel
// (render_kernel.cpp:75-181), shared by the gfx950 kernels (rt_render.hip)
// and the CPU build of the same code (rt_hostsim.cpp).
//
// Why a wavefront: a bounce of the reference issues up to five scene
// queries (continuation, light shadow, BRDF->light, env shadow, BRDF->env),
// but every RNG draw of the bounce happens before any of them is looked at
// and no query's origin or direction depends on another query's result. So
// one bounce splits into
//   shade    (RNG draws, BRDF / env / light sampling; emits the rays),
//   trace    (closest-hit / occlusion queries, separate kernels),
//   resolve  (the reference's arithmetic on the query results, in its order).
// Every path keeps its RNG state, so each pixel's draws happen in exactly
// the reference's order; pixels are independent, so running them side by
// side changes nothing. The per-path loop below is an exact re-expression of
// the reference's bounce loop, state machine included (MISSED, bounce==1 sky
// rule, emission at bounce 0, `break` on a dead BRDF sample).
//
// Buffers (device memory, one entry per path slot; slot = pixel index of
// the launch's pixel source): 16-B records so a wave's loads coalesce.
#pragma once

#include "rt_fast.h"

namespace rtk {

// Closest-hit kinds first (CONT .. CAM), then the occlusion kinds (ESH, BENV): the trace
// kernels split the queues there. CAM is the next sample's camera ray, traced ahead (below).
enum RayKind { RK_CONT = 0, RK_LSH = 1, RK_BL = 2, RK_CAM = 3, RK_ESH = 4, RK_BENV = 5, RK_COUNT = 6 };

enum PathFlag : uint32_t {
    PF_CONT = 1u,        // a continuation / camera ray is in flight
    PF_END = 2u,         // the sample ends once the pending bounce is resolved
    PF_AUX = 4u,         // a shaded bounce waits to be resolved
    PF_LSH = 8u,         // light shadow ray emitted (and its candidate is valid)
    PF_BL = 16u,         // BRDF->light ray emitted
    PF_ESH = 32u,        // env shadow ray emitted
    PF_BENV = 64u,       // BRDF->env ray emitted
    PF_CAM = 256u,       // the next sample's camera ray is in flight (next_camera)
};
#define RT_FLAG_BITS 12  // p_rd.w = flags | bounce << RT_FLAG_BITS

struct RayRec {  // 32 B queue entry
    float4_ o;  // xyz origin, w = target (slot) bits
    float4_ d;  // xyz direction
};

// Pixel source of a launch: image rows y = off + j*stride (j = slot / W), or
// an explicit (x, y) list (ray_trace_pixel over a pixel set).
struct PixSrc {
    int W, off, stride;
    const int32_t* xy;
};

RT_HD void pix_xy(const PixSrc& src, int i, int& x, int& y)
{
    if (src.xy) {
        x = src.xy[2 * i];
        y = src.xy[2 * i + 1];
    } else {
        const int j = i / src.W;
        x = i - j * src.W;
        y = src.off + j * src.stride;
    }
}

struct WaveView {
    RtSceneView S;
    RtCamera cam;
    PixSrc src;
    int W, H, spp, bounces;
    float cam_o[3];         // xform_point(cam, 0): every camera ray's origin (set_view_consts)
    float aspect;           // (float)W / (float)H
    int far_check;          // the camera lies outside the near box: test every query's origin (rt_fast.h far_origin)
    int n_slots;
    int bl_rays;            // 0: no primitive has an emissive material -> BRDF->light rays can't contribute
    int any_rays;           // 1: occlusion queries may use the any-hit walk (no analytic spheres)
    float4_* fb;            // framebuffer values (read-modify-write at pixel end), see fb_at
    int fb_rs;              // row sources: framebuffer rows from one slot row to the next (lanes alternate rows)
    // path state
    float4_* p_ro;          // ro.xyz, rng bits
    float4_* p_rd;          // rd.xyz, flags | bounce << RT_FLAG_BITS
    float4_* p_thr;         // thr.rgb, sample
    float4_* p_sc;          // sc.rgb
    float4_* p_fin;         // fin.rgb
    // pending bounce (shade -> resolve)
    float4_* q_light;       // light candidate rgb, dist
    float4_* q_bl;          // BRDF->light sample brdf * cos(n, dir) rgb, pdf
    float4_* q_sdir;        // BRDF->light dir xyz
    float4_* q_blo;         // BRDF->light origin xyz (sphere hit normals)
    float4_* q_env;         // env candidate rgb
    float4_* q_benv;        // BRDF->env candidate rgb
    float4_* q_thr;         // thr at the shaded bounce
    // query results
    float* r_cont_t;
    int32_t* r_cont_k;
    float* r_cam_t;         // the next sample's camera ray (RK_CAM), traced ahead
    int32_t* r_cam_k;
    float* r_lsh_t;
    float* r_bl_t;
    int32_t* r_bl_k;
    uint8_t* r_esh;
    uint8_t* r_benv;
    // queues
    RayRec* q[RK_COUNT];    // [shards * seg_cap] each, then (heavy class on) as many of its heavy class
    uint8_t* r_heavy;       // [n_slots] (heavy class on) a query of the slot took >= heavy_calls quad trips
    int heavy_calls;        // k_trace's heavy threshold (0: heavy class off; set before wave_carve)
    int spec_cam;           // 1: trace the next sample's camera ray ahead (next_camera); 0: at the sample's start
    int32_t* counters;      // queue sizes, tickets, live counts (rt_render.hip C_*)
    int32_t* r_park;        // [n_slots] queries of the slot parked (the step skips the slot while > 0)
    RayRec* fb_c[2];        // [RK_COUNT n_slots] closest-hit queries left to the exact walk (d.w = kind), by parity
    RayRec* fb_a[2];        // [2 n_slots] occlusion queries left to the exact walk, by parity
    ParkC* park_c[2];       // parked closest-hit queries, double-buffered by iteration parity
    int32_t* done[2];       // slots whose exact walks finished, by parity (released by the next k_trace)
    ParkA* park_a[2];
    int park_cap;
    int budget;             // steps a query may take per launch before it parks
    uint32_t* spill_r;      // per-lane stack spill areas of the trace kernels
    float* spill_k;
    int spill_lanes;
    uint32_t* fspill_r;     // per-lane spill areas of the search-BVH stacks (RT_FAST_SPILL entries)
    float* fspill_k;
    int fspill_lanes;
    int32_t* iterq;         // stats renders: [iteration][2] = {queries, live slots} (else null)
    unsigned long long* handovers;  // queries k_trace handed to the exact walk, summed over renders (device; else null)
    float4_* wlog;          // stats renders with a walk log (rt_test_walk_log): 3 float4 per long walk, else null
    int32_t* wlog_n;        // records written (may exceed wlog_cap: the rest are dropped)
    int wlog_min, wlog_cap; // quad_visit calls a logged walk takes at least; records at most
    int wlog_every;         // 1, or a sampling modulus over (slot, iteration, kind)
    int iter;               // iteration of this launch
    int tail_paths;         // k_tail: paths per wave
    int drain_rows;         // k_trace: a wave's drain continues its walks as rows when at most this many remain
    // fast lane (run_wave, rt_test_schedule fast_k): one k_step hands the live paths with at most
    // fast_thr samples done (up to fast_cap of them) to the tail kernel on the fast stream
    int32_t* fast_list;     // the handed-over slots
    int32_t* fast_ticket;   // their count (may pass fast_cap: the tail kernel clamps)
    int fast_cap, fast_thr; // fast_cap 0: off (k_tail: the list's length cap)
    int force_fb;           // test knob (RT_FORCE_FALLBACK): a query whose ray hashes to 0 mod force_fb
                            // skips the quad walk and takes the exact octree walk (0: off)
    int shards, seg_cap;    // queues and live lists: `shards` segments of seg_cap entries (device: rt_render.hip)
    const int32_t* act_in;  // active slots this iteration
    int32_t* act_out;
    int n_act_in;
};

// Carves the path-slot buffers for n slots out of one allocation at `base`
// (nullptr: only sizes it). Returns the bytes needed.
#define RT_FAST_SPILL 48  // search-BVH stack entries per lane beyond the LDS window

inline size_t wave_carve(char* base, size_t n, WaveView& W)  // uses W.park_cap, W.spill_lanes, W.fspill_lanes, W.shards, W.seg_cap
{
    size_t o = 0;
    auto take = [&](size_t bytes) -> void* {
        void* p = base ? base + o : nullptr;
        o += (bytes + 255) & ~(size_t)255;
        return p;
    };
    W.p_ro = (float4_*)take(n * 16);
    W.p_rd = (float4_*)take(n * 16);
    W.p_thr = (float4_*)take(n * 16);
    W.p_sc = (float4_*)take(n * 16);
    W.p_fin = (float4_*)take(n * 16);
    W.q_light = (float4_*)take(n * 16);
    W.q_bl = (float4_*)take(n * 16);
    W.q_sdir = (float4_*)take(n * 16);
    W.q_blo = (float4_*)take(n * 16);
    W.q_env = (float4_*)take(n * 16);
    W.q_benv = (float4_*)take(n * 16);
    W.q_thr = (float4_*)take(n * 16);
    W.r_cont_t = (float*)take(n * 4);
    W.r_cont_k = (int32_t*)take(n * 4);
    W.r_cam_t = (float*)take(n * 4);
    W.r_cam_k = (int32_t*)take(n * 4);
    W.r_lsh_t = (float*)take(n * 4);
    W.r_bl_t = (float*)take(n * 4);
    W.r_bl_k = (int32_t*)take(n * 4);
    W.r_esh = (uint8_t*)take(n);
    W.r_benv = (uint8_t*)take(n);
    const size_t qn = (size_t)W.shards * W.seg_cap;  // >= n
    for (int k = 0; k < RK_COUNT; k++) W.q[k] = (RayRec*)take((W.heavy_calls > 0 ? 2 : 1) * qn * sizeof(RayRec));
    W.r_heavy = W.heavy_calls > 0 ? (uint8_t*)take(n) : nullptr;
    W.act_in = (const int32_t*)take(qn * 4);
    W.act_out = (int32_t*)take(qn * 4);
    W.r_park = (int32_t*)take(n * 4);
    for (int k = 0; k < 2; k++) {
        W.fb_c[k] = (RayRec*)take((size_t)RK_COUNT * n * sizeof(RayRec));
        W.fb_a[k] = (RayRec*)take(2 * n * sizeof(RayRec));
        W.park_c[k] = (ParkC*)take((size_t)W.park_cap * sizeof(ParkC));
        W.park_a[k] = (ParkA*)take((size_t)W.park_cap * sizeof(ParkA));
        W.done[k] = (int32_t*)take((7 * n + 2 * (size_t)W.park_cap) * 4);
    }
    W.spill_r = (uint32_t*)take((size_t)W.spill_lanes * RT_STACK_CAP * 4);
    W.spill_k = (float*)take((size_t)W.spill_lanes * RT_STACK_CAP * 4);
    W.fspill_r = (uint32_t*)take((size_t)W.fspill_lanes * RT_FAST_SPILL * 4);
    W.fspill_k = (float*)take((size_t)W.fspill_lanes * RT_FAST_SPILL * 4);
    return o;
}

// The test stressor of rt_test_schedule("force_fallback", k): a query whose ray hashes to
// 0 mod k skips the search-BVH walk for the exact octree walk (k = 0: off).
RT_HD bool forced_fallback(int k, const float4_& o, const float4_& d)
{
    return k > 0 && ((rt_asuint(o.x) ^ rt_asuint(d.y) ^ (rt_asuint(d.z) >> 7)) % (uint32_t)k) == 0u;
}
RT_HD float4_ f4(V3 v, float w) { return float4_{v.x, v.y, v.z, w}; }
RT_HD float4_ f4(Col c, float w) { return float4_{c.r, c.g, c.b, w}; }
RT_HD V3 v3of(const float4_& f) { return v3(f.x, f.y, f.z); }
RT_HD Col colof(const float4_& f) { return Col{f.x, f.y, f.z}; }

// What one path step hands to the queues: per kind the ray (the slot goes into the
// queue record when it is written, rec()).
struct Emit {
    V3 o[RK_COUNT], d[RK_COUNT];
    uint32_t mask;  // bit k: a ray of kind k
    bool active;    // the path stays in flight
    bool heavy;     // the rays go to the heavy class (WaveView::qh)
    RT_HD RayRec rec(int kind, int slot, float dw = 0.0f) const
    {
        RayRec r;
        r.o = float4_{o[kind].x, o[kind].y, o[kind].z, rt_asfloat((uint32_t)slot)};
        r.d = float4_{d[kind].x, d[kind].y, d[kind].z, dw};
        return r;
    }
};

RT_HD void emit(Emit& e, int kind, int slot, V3 o, V3 d)
{
    (void)slot;  // (the step's own slot: written with the record)
    e.o[kind] = o;
    e.d[kind] = d;
    e.mask |= 1u << kind;
}

// k_step's and k_tail's Emit: the rays wait in LDS (this lane's column s: component c of
// kind k at s[(6 k + c) * ST], ST lanes side by side, so a wave's lanes touch consecutive
// words), not in up to 36 VGPRs held from the first emit through the rest of the shading
// code to the append.
template <int ST>
struct EmitLds {
    float* s;
    uint32_t mask;
    bool active;
    bool heavy;
    RT_HD V3 o(int kind) const { return v3(s[(6 * kind) * ST], s[(6 * kind + 1) * ST], s[(6 * kind + 2) * ST]); }
    RT_HD V3 d(int kind) const { return v3(s[(6 * kind + 3) * ST], s[(6 * kind + 4) * ST], s[(6 * kind + 5) * ST]); }
    RT_HD RayRec rec(int kind, int slot, float dw = 0.0f) const
    {
        const V3 ro = o(kind), rd = d(kind);
        RayRec r;
        r.o = float4_{ro.x, ro.y, ro.z, rt_asfloat((uint32_t)slot)};
        r.d = float4_{rd.x, rd.y, rd.z, dw};
        return r;
    }
};

template <int ST>
RT_HD void emit(EmitLds<ST>& e, int kind, int slot, V3 o, V3 d)
{
    (void)slot;
    float* c = e.s + 6 * kind * ST;
    c[0] = o.x;
    c[ST] = o.y;
    c[2 * ST] = o.z;
    c[3 * ST] = d.x;
    c[4 * ST] = d.y;
    c[5 * ST] = d.z;
    e.mask |= 1u << kind;
}

RT_HD V3 xform_point(const RtCamera& c, V3 p)  // mat.cpp:94-111
{
    const float* m = c.m;
    float xt = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yt = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zt = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wt = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    float w = 1.f / wt;
    if (wt == 1.f) return v3(xt, yt, zt);
    return v3(xt * w, yt * w, zt * w);
}

// framebuffer update + exposure / gamma tone-map (:167-180), in place (the one-step
// form of finish_pixel + tonemap_pixel; test builds).
RT_HD void tonemap_into(float* px, Col fin)
{
    px[0] += fin.r;
    px[1] += fin.g;
    px[2] += fin.b;
    const float a = px[3] + 0.0f;
    px[3] = 1.0f + (-((-a) * 1.5f));
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float e = rt_expf((-px[c]) * 1.5f);
        float tm = 1.0f + (-e);
        px[c] = rt_powf(tm, 1.0f / 2.2f);
    }
}

// Register copy of one path slot.
struct PathReg {
    V3 ro, rd;
    Rng rng;
    uint32_t flags;
    int bounce, sample;
    Col thr, sc, fin;
    int last_end;  // the pixel's previous sample: its last shaded bounce (-1: none, -2: no sample yet)
};

RT_HD void load_path(const WaveView& W, int p, PathReg& P)
{
    const float4_ a = W.p_ro[p], b = W.p_rd[p], c = W.p_thr[p], d = W.p_sc[p], e = W.p_fin[p];
    P.ro = v3of(a);
    P.rng.a = rt_asuint(a.w);
    P.rd = v3of(b);
    const uint32_t fb = rt_asuint(b.w);
    P.flags = fb & ((1u << RT_FLAG_BITS) - 1u);
    P.bounce = (int)(fb >> RT_FLAG_BITS);
    P.thr = colof(c);
    P.sample = (int)rt_asuint(c.w);
    P.sc = colof(d);
    P.last_end = (int)rt_asuint(d.w);
    P.fin = colof(e);
}

// fin changes only when a sample ends: the other steps leave its record alone
RT_HD void store_path(const WaveView& W, int p, const PathReg& P, bool fin_changed)
{
    W.p_ro[p] = f4(P.ro, rt_asfloat(P.rng.a));
    W.p_rd[p] = f4(P.rd, rt_asfloat(P.flags | ((uint32_t)P.bounce << RT_FLAG_BITS)));
    W.p_thr[p] = f4(P.thr, rt_asfloat((uint32_t)P.sample));
    W.p_sc[p] = f4(P.sc, rt_asfloat((uint32_t)P.last_end));
    if (fin_changed) W.p_fin[p] = f4(P.fin, 0.0f);
}

// Camera ray of a sample (render_kernel.cpp:88-92, get_camera_ray :56-73): the two
// jitter draws from rng, then the ray.
RT_HD void camera_ray(const WaveView& W, int x, int y, Rng& rng, V3& o, V3& d)
{
    float xj = ((float)x + 0.5f) + rng.next() - 1.0f;
    float yj = ((float)y + 0.5f) + rng.next() - 1.0f;
    float xn = xj / (float)W.W * 2.0f - 1.0f;
    xn *= W.aspect;
    float yn = yj / (float)W.H * 2.0f - 1.0f;
    o = v3(W.cam_o[0], W.cam_o[1], W.cam_o[2]);
    const V3 pd = xform_point(W.cam, v3(xn, yn, W.cam.fov_dist));
    d = normalize(sub(pd, o));
}

// The next sample's camera ray, traced ahead. A sample's draws all happen at its
// shaded bounces, so once a bounce is shaded the RNG state the next sample starts
// from is known if the sample ends there: when the bounce loop ends at this bounce
// (terminated, or the last bounce) it is certain, and when the continuation ray is
// cast it is right exactly when that ray misses (a miss draws nothing), which is how
// most samples end. Casting the next camera ray from a copy of the state beside the
// bounce's own rays lets the step that sees the sample end shade the next sample's
// first hit at once: one step per sample fewer on the path's dependent chain. When
// the continuation hits instead, the camera answer is dropped. The ray is computed
// again, bit for bit the same, when its sample starts (begin_sample_ahead).
template <class E>
RT_HD void next_camera(const WaveView& W, int p, const PathReg& P, E& e, uint32_t& fl)
{
    if (!W.spec_cam || P.sample + 1 >= W.spp) return;
    // spec_cam 2: where the sample may go on (a continuation is cast), only at the bounce
    // where the pixel's previous sample ended (the camera ray: bounce -1)
    if (W.spec_cam == 2 && (fl & PF_CONT) && P.last_end != -2 && P.last_end != P.bounce - 1) return;
    int x, y;
    pix_xy(W.src, p, x, y);
    Rng r = P.rng;
    V3 o, d;
    camera_ray(W, x, y, r, o, d);
    emit(e, RK_CAM, p, o, d);
    fl |= PF_CAM;
}

// Camera ray of the next sample (render_kernel.cpp:88-92, get_camera_ray
// :56-73). Returns false when the pixel is complete (then fb is written).
// With max_bounces == 0 the reference's bounce loop never runs: each sample
// only draws its 2 jitter values and adds black.
template <class E>
RT_HD bool start_sample(const WaveView& W, int p, PathReg& P, E& e)
{
    int x, y;
    pix_xy(W.src, p, x, y);
    for (;;) {
        camera_ray(W, x, y, P.rng, P.ro, P.rd);
        P.thr = col(1.0f);
        P.sc = col(0.0f);
        P.bounce = 0;
        P.flags = 0;
        if (W.bounces > 0) {
            P.flags = PF_CONT;
            emit(e, RK_CONT, p, P.ro, P.rd);
            // (and the one after it, should this camera ray miss: no draws, so it starts here)
            next_camera(W, p, P, e, P.flags);
            return true;
        }
        P.fin = cadd(P.fin, P.sc);
        if (++P.sample == W.spp) return false;
    }
}

// A sample whose camera ray was traced ahead (next_camera): its draws and ray, as
// start_sample computes them, and its camera answer is the continuation to consume.
RT_HD void begin_sample_ahead(const WaveView& W, int p, PathReg& P)
{
    int x, y;
    pix_xy(W.src, p, x, y);
    camera_ray(W, x, y, P.rng, P.ro, P.rd);
    P.thr = col(1.0f);
    P.sc = col(0.0f);
    P.bounce = 0;
    P.flags = PF_CONT;
}

// The per-render constants of start_sample, evaluated once (same operations, so the
// same values): the camera origin xform_point(cam, 0) and the aspect ratio.
RT_HD void set_view_consts(WaveView& W)
{
    const V3 o = xform_point(W.cam, v3(0.0f, 0.0f, 0.0f));
    W.cam_o[0] = o.x;
    W.cam_o[1] = o.y;
    W.cam_o[2] = o.z;
    W.aspect = (float)W.W / (float)W.H;
    // (a render whose camera lies in the near box casts every other ray from a surface of the
    // scene, inside it too: its queries skip the per-query near-box test; W.S set before this)
    W.far_check = far_origin(W.S, o) ? 1 : 0;
}

// Framebuffer entry of slot p: slot rows map to every fb_rs-th framebuffer row.
RT_HD size_t fb_at(const WaveView& W, int p)
{
    if (W.src.xy || W.fb_rs <= 1) return (size_t)p;
    const int j = p / W.src.W;
    return (size_t)j * W.fb_rs * W.src.W + (p - j * W.src.W);
}

// The pixel's end (render_kernel.cpp:167-180) in two parts: finish_pixel adds the
// sample average to the framebuffer when the pixel's last sample ends, and
// tonemap_pixel (the alpha update and the exposure / gamma expf / powf of tonemap_into,
// on the same values in the same order) runs once per pixel after the render's last
// step, in its own converged pass (rt_render.hip k_tonemap, rt_hostsim.cpp), instead
// of inside the divergent step code.
RT_HD void finish_pixel(const WaveView& W, int p, PathReg& P)
{
    const float k = (float)W.spp;
    Col fin = P.fin;
    fin.r /= k;  // Color /= float is a true division (color.h:69-76)
    fin.g /= k;
    fin.b /= k;
    float4_& dst = W.fb[fb_at(W, p)];
    float4_ px = dst;
    px.x += fin.r;
    px.y += fin.g;
    px.z += fin.b;
    dst = px;
}

RT_HD void tonemap_pixel(const WaveView& W, int p)
{
    float4_& dst = W.fb[fb_at(W, p)];
    float4_ px = dst;
    float* v = &px.x;
    const float a = v[3] + 0.0f;
    v[3] = 1.0f + (-((-a) * 1.5f));
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float e = rt_expf((-v[c]) * 1.5f);
        float tm = 1.0f + (-e);
        v[c] = rt_powf(tm, 1.0f / 2.2f);
    }
    dst = px;
}

// Path initialisation: seed + 10 warm-up draws (render_kernel.cpp:77-82),
// first camera ray.
RT_HD void path_init(const WaveView& W, int p, Emit& e)
{
    int x, y;
    pix_xy(W.src, p, x, y);
    PathReg P;
    P.rng.a = (uint32_t)(31 + x * y * W.spp);
    for (int i = 0; i < 10; i++) P.rng.next();
    P.fin = col(0.0f);
    P.sample = 0;
    P.last_end = -2;
    e.mask = 0;
    e.heavy = false;
    e.active = start_sample(W, p, P, e);
    if (!e.active) finish_pixel(W, p, P);
    store_path(W, p, P, true);
}

// Hit record of a closest-hit query (HitInfo fields the integrator reads).
// As hit_from, the triangle's records r0..r2 (tri4[3k..3k+2]) already loaded by the caller.
RT_HD bool hit_from_rec(const RtSceneView& S, V3 o, V3 d, float t, int k, const float4_& r0, const float4_& r1,
                        const float4_& r2, Hit& h)
{
    h.t = t;
    h.k = k;
    h.prim = -1;
    h.mi = -1;
    if (k >= 0) {  // triangle (triangle.h:46-56)
        h.p = add(o, mul(t, d));
        h.n = normalize(cross(ld3(r1), ld3(r2)));
        h.prim = (int)rt_asuint(r0.w);
        if (S.tri_mat) h.mi = (int)rt_asuint(r1.w);
    } else if (k <= -2) {  // sphere (sphere.h:46-48)
        const float4_ s0 = S.spheres[2 * (-2 - k)];
        h.p = add(o, mul(t, d));
        h.n = normalize(sub(h.p, ld3(s0)));
        h.prim = (int)rt_asuint(S.spheres[2 * (-2 - k) + 1].x);
    }
    return t > 0.0f;
}

RT_HD bool hit_from(const RtSceneView& S, V3 o, V3 d, float t, int k, Hit& h)
{
    h.t = t;
    h.k = k;
    h.prim = -1;
    h.mi = -1;
    if (k >= 0) {  // triangle (triangle.h:46-56)
        const float4_ r1 = S.tri4[3 * k + 1];
        const V3 e1 = ld3(r1), e2 = ld3(S.tri4[3 * k + 2]);
        h.p = add(o, mul(t, d));
        h.n = normalize(cross(e1, e2));
        h.prim = (int)rt_asuint(S.tri4[3 * k].w);
        if (S.tri_mat) h.mi = (int)rt_asuint(r1.w);
    } else if (k <= -2) {  // sphere (sphere.h:46-48)
        const float4_ s0 = S.spheres[2 * (-2 - k)];
        h.p = add(o, mul(t, d));
        h.n = normalize(sub(h.p, ld3(s0)));
        h.prim = (int)rt_asuint(S.spheres[2 * (-2 - k) + 1].x);
    }
    return t > 0.0f;
}

// ---------------------------------------------------------------- shade
// The pre-query half of one hit bounce: sample_lights (:633-713),
// sample_environment_map (:569-631) and the continuation sample (:123),
// with every RNG draw in the reference's order. Candidate contributions
// are computed now (they depend only on the draws); resolve() decides with
// the query results whether they count.
template <class E>
RT_HD void shade(const WaveView& W, int p, PathReg& P, const Hit& h, E& e, Stats* st)
{
    const RtSceneView& S = W.S;
    if (st) st->c[RT_STAT_MAT]++;
    const Mat m = load_mat_of(S, h);
    const V3 rd = P.rd;
    uint32_t fl = PF_AUX;

    // ---- sample_lights, light half (sample_random_point_on_lights :715-742)
    if (S.n_emissive > 0) {
        int li = rt_f2i(P.rng.next() * (float)S.n_emissive);
        li = S.emissive[li];
        const int lk = S.prim2k[li];
        const V3 A = ld3(S.tri4[3 * lk]), AB = ld3(S.tri4[3 * lk + 1]), AC = ld3(S.tri4[3 * lk + 2]);
        float r1 = P.rng.next();
        float r2 = P.rng.next();
        float sr1 = rt_sqrtf(r1);
        float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
        V3 Pt = add(add(A, mul(u, AB)), mul(v, AC));
        V3 nrm = cross(AB, AC);
        float ln = length(nrm);
        V3 lnorm = mul(1 / ln, nrm);
        float area = ln * 0.5f;
        float nb = (float)S.n_emissive;
        float lpdf = 1.0f / (nb * area);

        V3 so = add(h.p, mul(1.0e-4f, h.n));
        V3 sd = sub(Pt, so);
        float dist = length(sd);
        V3 sdn = normalize(sd);
        float dl = rt_max(dot(lnorm, neg(sdn)), 0.0f);
        if (dl > 0.0f) {
            // evaluate_shadow_ray (:744-759) is the query; the rest only runs if unshadowed
            if (st) st->c[RT_STAT_MAT]++;
            const Mat em = load_mat(S, li);
            lpdf *= dist * dist;
            lpdf /= dl;
            Col brdf = ct_brdf(m, sdn, neg(rd), h.n);
            float cp = ct_pdf(m, neg(rd), sdn, h.n);
            if (cp != 0.0f) {
                float mis = power_heuristic(lpdf, cp);
                float cosine = dot(h.n, sdn);
                Col light = cdiv(cscale(cmul(cscale(em.emission, cosine), brdf), mis), lpdf);
                W.q_light[p] = f4(light, dist);
                fl |= PF_LSH;
                emit(e, RK_LSH, p, so, sdn);
            }
        }
    }
    // ---- sample_lights, BRDF half (:681-711). With no emissive material (bl_rays 0) the
    // sample can never contribute: only its two RNG draws are kept.
    if (!W.bl_rays) {
        P.rng.next();
        P.rng.next();
    } else {
        V3 sdir = v3(0.0f, 0.0f, 0.0f);
        float dpdf;
        Col brdf = ct_sample(m, neg(rd), h.n, sdir, dpdf, P.rng);
        if (!(brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f)) {
            // brdf * dot(n, sdir): the first product of resolve's bmis (:700), done here so the
            // hit normal need not travel
            W.q_bl[p] = f4(cscale(brdf, dot(h.n, sdir)), dpdf);
            const V3 blo = add(h.p, mul(1.0e-5f, h.n));
            W.q_sdir[p] = f4(sdir, 0.0f);
            W.q_blo[p] = f4(blo, 0.0f);
            fl |= PF_BL;
            emit(e, RK_BL, p, blo, sdir);
        }
    }
    // ---- sample_environment_map (:569-631)
    {
        const float total = S.cdf_total;
        int x, y;
        cdf_search(S, P.rng.next() * total, x, y, st);
        float u = (float)x / (float)S.ew, v = (float)y / (float)S.eh;
        float phi = (float)((double)(u * 2.0f) * 3.14159265358979323846);
        float theta = (float)((double)v * 3.14159265358979323846);
        float st_, ct_, sp_, cp_;
        rt_sincosf(theta, st_, ct_);
        rt_sincosf(phi, sp_, cp_);
        V3 dir = v3(-st_ * cp_, -ct_, -st_ * sp_);
        float cosine = dot(h.n, dir);
        if (cosine > 0.0f) {
            // the texel and its f64-evaluated luminance in one record (env.w = env_lum, rt_set_env)
            if (st) st->c[RT_STAT_ENV]++;
            const float4_ et = S.env[y * S.ew + x];
            float pdf = et.w / total;
            pdf = (float)((double)((pdf * (float)S.ew) * (float)S.eh) /
                          (2.0 * 3.14159265358979323846 * 3.14159265358979323846 * (double)st_));
            const Col rad = Col{et.x, et.y, et.z};
            Col brdf = ct_brdf(m, dir, neg(rd), h.n);
            float bp = ct_pdf(m, neg(rd), dir, h.n);
            float mis = power_heuristic(pdf, bp);
            W.q_env[p] = f4(cdiv(cmul(cscale(cscale(brdf, cosine), mis), rad), pdf), 0.0f);
            fl |= PF_ESH;
            emit(e, RK_ESH, p, add(h.p, mul(1.0e-4f, h.n)), dir);
        }
        float bsp;
        V3 bdir = v3(0.0f, 0.0f, 0.0f);
        Col bis = ct_sample(m, neg(rd), h.n, bdir, bsp, P.rng);
        cosine = rt_max(dot(h.n, bdir), 0.0f);
        if (bsp != 0.0f && cosine > 0.0f) {
            Col sky = env_from_dir(S, bdir, st);
            float th = rt_acosf(bdir.z);
            float sth = rt_sinf(th);
            float epdf = (0.3086f * sky.r + 0.6094f * sky.g + 0.0820f * sky.b) / S.cdf_total;
            epdf *= (float)(S.ew * S.eh);
            epdf = (float)((double)epdf / (2.0 * 3.14159265358979323846 * 3.14159265358979323846 * (double)sth));
            float mis = power_heuristic(bsp, epdf);
            W.q_benv[p] = f4(cdiv(cmul(cscale(cscale(sky, mis), cosine), bis), bsp), 0.0f);
            fl |= PF_BENV;
            emit(e, RK_BENV, p, add(h.p, mul(1.0e-5f, h.n)), bdir);
        }
    }
    // ---- continuation (:123-141)
    float bpdf;
    V3 dir = v3(0.0f, 0.0f, 0.0f);
    Col brdf = ct_sample(m, neg(rd), h.n, dir, bpdf, P.rng);
    // bounce 0: sample_color += material.emission (:126) — sc is still the sample start's 0 and
    // nothing else adds to it before this bounce's resolve, so the same addition happens here
    if (P.bounce == 0) P.sc = cadd(P.sc, m.emission);
    W.q_thr[p] = f4(P.thr, 0.0f);
    if ((brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f) || bpdf < 1.0e-8f || rt_isinf(bpdf)) {
        fl |= PF_END;  // `break` after this bounce's light is added
    } else {
        P.thr = cmul(P.thr, cdiv(cscale(brdf, rt_max(0.0f, dot(dir, h.n))), bpdf));
        P.ro = add(h.p, mul(1.0e-4f, h.n));
        P.rd = dir;
        if (P.bounce + 1 < W.bounces) {
            P.bounce++;
            fl |= PF_CONT;
            emit(e, RK_CONT, p, P.ro, P.rd);
        } else {
            fl |= PF_END;  // the bounce loop is over
        }
    }
    next_camera(W, p, P, e, fl);  // (the next sample starts from this state if the sample ends here)
    P.flags = fl;
}

// --------------------------------------------------------------- resolve
// sc += (light + bmis + brdf_sample + env_sample) * thr with the
// reference's association: lr = light + bmis, er = brdf_sample + env_sample,
// sc = sc + (lr + er) * thr (render_kernel.cpp:113-128).
// The records a resolve reads first, loaded by path_step together with the hit's
// triangle (one memory round trip): the pending bounce's candidates and their query results.
struct ResolveRec {
    float4_ thr, env, benv, light;
    float lsh_t, bl_t;
    uint8_t esh, benv_r;
};
RT_HD void resolve_load(const WaveView& W, int p, uint32_t fl, ResolveRec& R)
{
    const float4_ z = float4_{0.0f, 0.0f, 0.0f, 0.0f};
    R.thr = W.q_thr[p];
    R.env = (fl & PF_ESH) ? W.q_env[p] : z;
    R.benv = (fl & PF_BENV) ? W.q_benv[p] : z;
    R.esh = (fl & PF_ESH) ? W.r_esh[p] : 1;
    R.benv_r = (fl & PF_BENV) ? W.r_benv[p] : 1;
    R.light = (fl & PF_LSH) ? W.q_light[p] : z;
    R.lsh_t = (fl & PF_LSH) ? W.r_lsh_t[p] : 0.0f;
    R.bl_t = (fl & PF_BL) ? W.r_bl_t[p] : 0.0f;
}

RT_HD void resolve(const WaveView& W, int p, PathReg& P, const ResolveRec& R, Stats* st)
{
    const RtSceneView& S = W.S;
    const uint32_t fl = P.flags;
    const float4_ q_thr = R.thr, q_env = R.env, q_benv = R.benv;
    const uint8_t r_esh = R.esh, r_benv = R.benv_r;
    Col light = col(0.0f);
    if (fl & PF_LSH) {
        const float4_ q = R.light;
        const float t = R.lsh_t;
        const bool in_shadow = t > 0.0f && t + 1.0e-4f < q.w;
        if (!in_shadow) light = colof(q);
    }
    Col bmis = col(0.0f);
    if (fl & PF_BL) {
        const float t = R.bl_t;
        if (t > 0.0f) {
            const int k = W.r_bl_k[p];
            const float4_ qb = W.q_bl[p];
            const V3 sdir = v3of(W.q_sdir[p]);
            Hit nh;
            hit_from(S, v3of(W.q_blo[p]), sdir, t, k, nh);
            float ca = rt_max(dot(nh.n, neg(sdir)), 0.0f);
            if (ca > 0.0f) {
                if (st) st->c[RT_STAT_MAT]++;
                const Mat mm = load_mat_of(S, nh);
                const Col e = mm.emission;
                if (e.r > 0 || e.g > 0 || e.b > 0) {
                    float d2 = t * t;
                    // Triangle::area (triangle.cpp:8-11) of the hit triangle; an
                    // emissive *sphere* hit reads past the triangle buffer in the
                    // reference (undefined behaviour): area 0 here.
                    float la = k < 0 ? 0.0f : length(cross(ld3(S.tri4[3 * k + 1]), ld3(S.tri4[3 * k + 2]))) / 2;
                    float lp = d2 / (la * ca);
                    float mis = power_heuristic(qb.w, lp);
                    bmis = cdiv(cscale(cmul(colof(qb), e), mis), qb.w);  // (qb.rgb = brdf * cosine, shade)
                }
            }
        }
    }
    Col env_sample = col(0.0f), brdf_sample = col(0.0f);
    if ((fl & PF_ESH) && !r_esh) env_sample = colof(q_env);
    if ((fl & PF_BENV) && !r_benv) brdf_sample = colof(q_benv);
    const Col lr = cadd(light, bmis);
    const Col er = cadd(brdf_sample, env_sample);
    P.sc = cadd(P.sc, cmul(cadd(lr, er), colof(q_thr)));
}

// One iteration of path slot p: resolve the bounce shaded last iteration,
// consume the continuation query, shade the new hit or end the sample; a sample
// that ends goes on with the next one: its camera answer, when it was traced ahead
// (next_camera), is consumed in the same step (shaded, or that sample ends too and
// the next camera ray is cast), else its camera ray is cast. Fills `e` with the rays
// for the next trace.
template <class E>
RT_HD void path_step(const WaveView& W, int p, E& e, Stats* st)
{
    e.mask = 0;
    e.active = true;
    e.heavy = false;
    // the slot's state, wait count and continuation result in one round trip
    const int park = W.r_park[p];
    const int heavy = W.r_heavy ? W.r_heavy[p] : 0;
    PathReg P;
    load_path(W, p, P);
    const float cont_t = W.r_cont_t[p];
    const int cont_k = W.r_cont_k[p];
    const float cam_t = W.r_cam_t[p];  // (read only with PF_CAM)
    const int cam_k = W.r_cam_k[p];
    if (park != 0) {  // a query of this path is parked: wait (-1: handed to the fast lane, leaves the list)
        e.active = park > 0;
        return;
    }
    if (st) st->c[RT_STAT_STEPS]++;
    if (heavy) {  // its last walk was long: this step's rays head the next streams
        e.heavy = true;
        W.r_heavy[p] = 0;
    }
    // what depends only on the state, loaded together: the bounce to resolve and the hit's triangle
    const uint32_t fl0 = P.flags;
    ResolveRec R;
    if (fl0 & PF_AUX) resolve_load(W, p, fl0, R);
    // (the triangle the step shades: the continuation's hit, else the next sample's camera hit)
    float4_ tr0 = float4_{0.0f, 0.0f, 0.0f, 0.0f}, tr1 = tr0, tr2 = tr0;
    const bool cont_hit = (fl0 & PF_CONT) && cont_t > 0.0f && cont_k >= 0;
    const int tk = cont_hit ? cont_k : ((fl0 & PF_CAM) && cam_t > 0.0f && cam_k >= 0) ? cam_k : -1;
    if (tk >= 0) {
        tr0 = W.S.tri4[3 * tk];
        tr1 = W.S.tri4[3 * tk + 1];
        tr2 = W.S.tri4[3 * tk + 2];
    }
    if (fl0 & PF_AUX) resolve(W, p, P, R, st);
    // the hit this step shades, if any: the continuation's, or else (the sample over) the
    // next sample's camera hit traced ahead; shade() is called from one place only (its
    // registers, not twice its code)
    bool end = (P.flags & PF_END) != 0, fin_changed = false, do_shade = false;
    Hit h;
    if (P.flags & PF_CONT) {
        if (hit_from_rec(W.S, P.ro, P.rd, cont_t, cont_k, tr0, tr1, tr2, h)) {
            do_shade = true;
        } else {
            // MISSED (:143-160): the next loop iteration adds the sky only when
            // it is bounce 1, i.e. the camera ray missed; then `break`.
            if (P.bounce == 0 && W.bounces >= 2) P.sc = cadd(P.sc, cmul(env_from_dir(W.S, P.rd, st), P.thr));
            end = true;
        }
    }
    if (end) {
        fin_changed = true;
        P.last_end = (P.flags & PF_END) ? P.bounce : P.bounce - 1;  // (a missed continuation: the bounce before)
        P.fin = cadd(P.fin, P.sc);
        bool start = ++P.sample < W.spp;
        if (start && (fl0 & PF_CAM)) {  // the next sample, its camera ray traced ahead: its answer now
            begin_sample_ahead(W, p, P);
            if (hit_from_rec(W.S, P.ro, P.rd, cam_t, cam_k, tr0, tr1, tr2, h)) {
                do_shade = true;
                start = false;
            } else {  // (bounce 0 missed: the sky, and that sample is over too)
                if (W.bounces >= 2) P.sc = cadd(P.sc, cmul(env_from_dir(W.S, P.rd, st), P.thr));
                P.last_end = -1;
                P.fin = cadd(P.fin, P.sc);
                start = ++P.sample < W.spp;
            }
        }
        if (!do_shade) e.active = start && start_sample(W, p, P, e);
    }
    if (do_shade) {
        shade(W, p, P, h, e, st);
    } else if (!e.active) {
        finish_pixel(W, p, P);
    }
    store_path(W, p, P, fin_changed);
}

// --------------------------------------------------------------- queries
// Closest-hit query (INTERSECT_SCENE = intersect_scene_bvh :485-502):
// octree, then the sphere loop. Writes (t, k) with k = leaf-order triangle,
// -2 - sphere index, or -1 for none.
RT_HD void spheres_closest(const RtSceneView& S, V3 o, V3 d, float& t, int& k)
{
    for (int i = 0; i < S.n_spheres; i++) {
        Hit sh;
        if (sphere_test(S.spheres, i, o, d, sh))
            if (sh.t < t || t == -1.0f) {
                t = sh.t;
                k = sh.k;
            }
    }
}

RT_HD void query_closest(const RtSceneView& S, V3 o, V3 d, StackEnt* stack, float& t, int& k, Stats* st)
{
    if (S.brute)
        brute_closest(S, o, d, t, k);
    else
        trace_closest(S, o, d, stack, t, k, st);
    spheres_closest(S, o, d, t, k);
}

// Writes a finished closest-hit query (octree best + sphere loop) to its
// result slot; target = slot * 8 + kind. Occlusion kinds reach here only
// when analytic spheres are present (then they use the exact closest logic).
RT_HD void finish_closest(const WaveView& W, uint32_t target, V3 o, V3 d, float t, int k)
{
    spheres_closest(W.S, o, d, t, k);
    const int slot = (int)(target >> 3), kind = (int)(target & 7u);
    if (kind == RK_CONT) {
        W.r_cont_t[slot] = t;
        W.r_cont_k[slot] = k;
    } else if (kind == RK_CAM) {
        W.r_cam_t[slot] = t;
        W.r_cam_k[slot] = k;
    } else if (kind == RK_LSH) {
        W.r_lsh_t[slot] = t;
    } else if (kind == RK_BL) {
        W.r_bl_t[slot] = t;
        W.r_bl_k[slot] = k;
    } else {
        (kind == RK_ESH ? W.r_esh : W.r_benv)[slot] = t > 0.0f ? 1 : 0;
    }
}

RT_HD void finish_any(const WaveView& W, uint32_t target, bool hit)
{
    const int slot = (int)(target >> 3), kind = (int)(target & 7u);
    (kind == RK_ESH ? W.r_esh : W.r_benv)[slot] = hit ? 1 : 0;
}

// The queue item behind a trace work index: closest-hit kernels see
// CONT, LSH, BL (then ESH, BENV when they need the closest logic); the
// occlusion kernel sees ESH, BENV. Returns the ray and its target.
RT_HD RayRec queue_item(const WaveView& W, const int32_t* counts, int first_kind, int last_kind, int i,
                        uint32_t& target)
{
    int kind = first_kind;
    while (kind < last_kind && i >= counts[kind]) {
        i -= counts[kind];
        kind++;
    }
    const RayRec r = W.q[kind][i];
    target = (rt_asuint(r.o.w) << 3) | (uint32_t)kind;
    return r;
}

// Short-stack form; false = stack overflow, re-run query_closest().
template <class STK>
RT_HD bool query_closest_short(const RtSceneView& S, V3 o, V3 d, STK& stk, float& t, int& k, Stats* st)
{
    if (!trace_closest_short(S, o, d, stk, t, k, st)) return false;
    spheres_closest(S, o, d, t, k);
    return true;
}

}  // namespace rtk
