// rt_render.hip — gfx950 backend of librt_hip.so: device buffers, the
// render / ray-query kernels and their launches.
//
// Kernel v1 ("megakernel"): one lane per pixel runs RenderKernel::
// ray_trace_pixel (render_kernel.cpp:75-181) to completion — all samples,
// all bounces, all five ray queries per bounce — via rt_trace.h, then does the
// framebuffer accumulate + tone-map in place. The octree walk keeps its
// explicit stack in private (scratch) memory.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "rt_context.h"
#include "rt_trace.h"

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return rt_fail(ctx, RT_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));     \
    } while (0)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct Backend {
    DevBuf nodes, tri4, prim2k, mat_idx, mats, emissive, spheres, env, env_lum, cdf;
    DevBuf stats;     // RT_STAT_COUNT u64
    DevBuf scratch;   // pixel lists / rays / outputs
    DevBuf fb;        // host-fb staging
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    RtSceneView view{};
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

Backend* be(rt_context* c) { return (Backend*)c->backend; }

// ------------------------------------------------------------------ kernels
template <bool STATS>
__global__ __launch_bounds__(256) void k_render(rtk::Ctx C, float4_* __restrict__ fb, int row_offset, int row_stride,
                                                int rows_local, unsigned long long* __restrict__ stats)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows_local * C.W) return;
    const int j = idx / C.W;
    const int x = idx - j * C.W;
    const int y = row_offset + j * row_stride;
    rtk::StackEnt stack[RT_STACK_CAP];
    rtk::Stats st;
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++) st.c[i] = 0;
    const rtk::Col f = rtk::trace_pixel(C, x, y, stack, STATS ? &st : nullptr);
    float4_ px = fb[idx];
    rtk::tonemap_into(&px.x, f);
    fb[idx] = px;
    if (STATS)
        for (int i = 0; i < RT_STAT_COUNT; i++) atomicAdd(&stats[i], st.c[i]);
}

template <bool STATS>
__global__ __launch_bounds__(256) void k_pixels(rtk::Ctx C, const int* __restrict__ xy, float4_* __restrict__ rgba, int n,
                                                unsigned long long* __restrict__ stats)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    rtk::StackEnt stack[RT_STACK_CAP];
    rtk::Stats st;
    if (STATS)
        for (int k = 0; k < RT_STAT_COUNT; k++) st.c[k] = 0;
    const rtk::Col f = rtk::trace_pixel(C, xy[2 * i], xy[2 * i + 1], stack, STATS ? &st : nullptr);
    float4_ px = rgba[i];
    rtk::tonemap_into(&px.x, f);
    rgba[i] = px;
    if (STATS)
        for (int k = 0; k < RT_STAT_COUNT; k++) atomicAdd(&stats[k], st.c[k]);
}

__global__ __launch_bounds__(256) void k_intersect(RtSceneView S, const float* __restrict__ rays, int32_t* __restrict__ out,
                                                   int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    rtk::StackEnt stack[RT_STACK_CAP];
    const float* r = rays + 6 * (size_t)i;
    rtk::Hit h;
    const bool f = rtk::intersect_scene(S, rtk::v3(r[0], r[1], r[2]), rtk::v3(r[3], r[4], r[5]), stack, h, nullptr);
    int32_t* o = out + 11 * (size_t)i;
    o[0] = f ? 1 : 0;
    o[1] = h.prim;
    o[2] = (int32_t)rt_asuint(h.t);
    const bool any = h.t != -1.0f;
    o[3] = any ? (int32_t)rt_asuint(h.p.x) : 0;
    o[4] = any ? (int32_t)rt_asuint(h.p.y) : 0;
    o[5] = any ? (int32_t)rt_asuint(h.p.z) : 0;
    o[6] = any ? (int32_t)rt_asuint(h.n.x) : 0;
    o[7] = any ? (int32_t)rt_asuint(h.n.y) : 0;
    o[8] = any ? (int32_t)rt_asuint(h.n.z) : 0;
    o[9] = (int32_t)rt_asuint(-1.0f);
    o[10] = (int32_t)rt_asuint(-1.0f);
}

// libm self-test kernel (tests/test_gpu_libm.py): out[i] = f(in[i])
__global__ void k_libm(int fn, const float* __restrict__ in, const float* __restrict__ in2, float* __restrict__ out, int n)
{
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
        default: r = (float)((double)x * 0.31830988618379067154 / (double)in2[i]); break;
    }
    out[i] = r;
}

}  // namespace

// ------------------------------------------------------------------- hooks
int rt_backend_create(rt_context* c)
{
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return rt_fail(c, RT_ERR_NODEV, "librt_hip: no HIP device available (this library has no CPU path)");
    if (c->device < 0 || c->device >= n) return rt_fail(c, RT_ERR_NODEV, "librt_hip: device index out of range");
    HIPCHK(c, hipSetDevice(c->device));
    Backend* b = new Backend();
    c->backend = b;
    HIPCHK(c, hipEventCreate(&b->ev0));
    HIPCHK(c, hipEventCreate(&b->ev1));
    return RT_OK;
}

void rt_backend_destroy(rt_context* c)
{
    Backend* b = be(c);
    if (!b) return;
    (void)hipSetDevice(c->device);
    DevBuf* all[] = {&b->nodes, &b->tri4,    &b->prim2k,  &b->mat_idx, &b->mats,    &b->emissive, &b->spheres,
                     &b->env,   &b->env_lum, &b->cdf,     &b->stats,   &b->scratch, &b->fb};
    for (DevBuf* d : all)
        if (d->p) (void)hipFree(d->p);
    if (b->ev0) (void)hipEventDestroy(b->ev0);
    if (b->ev1) (void)hipEventDestroy(b->ev1);
    delete b;
    c->backend = nullptr;
}

int rt_backend_upload(rt_context* c)
{
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(c->device));
    int r = 0;
    if ((r = upload(c, b->nodes, c->flat.nodes)) || (r = upload(c, b->tri4, c->flat.tri4)) ||
        (r = upload(c, b->prim2k, c->flat.prim2k)) || (r = upload(c, b->mat_idx, c->mat_idx)) ||
        (r = upload(c, b->mats, c->mats)) || (r = upload(c, b->emissive, c->emissive)) ||
        (r = upload(c, b->spheres, c->spheres)) || (r = upload(c, b->env, c->env)) ||
        (r = upload(c, b->env_lum, c->env_lum)) || (r = upload(c, b->cdf, c->cdf)) ||
        (r = ensure(c, b->stats, RT_STAT_COUNT * sizeof(unsigned long long))))
        return r;
    RtSceneView v{};
    v.nodes = (const RtNode*)b->nodes.p;
    v.tri4 = (const float4_*)b->tri4.p;
    v.prim2k = (const int32_t*)b->prim2k.p;
    v.mat_idx = (const int32_t*)b->mat_idx.p;
    v.mats = (const RtMat*)b->mats.p;
    v.emissive = (const int32_t*)b->emissive.p;
    v.spheres = (const float4_*)b->spheres.p;
    v.env = (const float4_*)b->env.p;
    v.env_lum = (const float*)b->env_lum.p;
    v.cdf = (const float*)b->cdf.p;
    v.n_emissive = (int)c->emissive.size();
    v.n_spheres = (int)(c->spheres.size() / 2);
    v.ew = c->ew;
    v.eh = c->eh;
    v.n_tris = (int)(c->tris.size() / 9);
    b->view = v;
    return RT_OK;
}

static int finish_stats(rt_context* c, Backend* b, hipStream_t s)
{
    if (!c->stats_enabled) return RT_OK;
    HIPCHK(c, hipMemcpyAsync(c->stats, b->stats.p, sizeof(c->stats), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return RT_OK;
}

int rt_backend_render(rt_context* c, int w, int h, int spp, int bounces, float* host_fb, void* dev_fb, int row_offset,
                      int row_stride, void* stream)
{
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const int rows_local = (h - row_offset + row_stride - 1) / row_stride;
    const size_t npx = (size_t)rows_local * w;
    float4_* fb = (float4_*)dev_fb;
    if (host_fb) {
        if (int r = ensure(c, b->fb, npx * sizeof(float4_))) return r;
        fb = (float4_*)b->fb.p;
        HIPCHK(c, hipMemcpyAsync(fb, host_fb, npx * sizeof(float4_), hipMemcpyHostToDevice, s));
    }
    if (c->stats_enabled) HIPCHK(c, hipMemsetAsync(b->stats.p, 0, b->stats.bytes, s));
    rtk::Ctx C{b->view, c->cam, w, h, spp, bounces};
    const int threads = 256;
    const int blocks = (int)((npx + threads - 1) / threads);
    HIPCHK(c, hipEventRecord(b->ev0, s));
    if (c->stats_enabled)
        hipLaunchKernelGGL(k_render<true>, dim3(blocks), dim3(threads), 0, s, C, fb, row_offset, row_stride, rows_local,
                           (unsigned long long*)b->stats.p);
    else
        hipLaunchKernelGGL(k_render<false>, dim3(blocks), dim3(threads), 0, s, C, fb, row_offset, row_stride,
                           rows_local, (unsigned long long*)b->stats.p);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(b->ev1, s));
    if (host_fb) {
        HIPCHK(c, hipMemcpyAsync(host_fb, fb, npx * sizeof(float4_), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, b->ev0, b->ev1));
        c->last_kernel_ms = ms;
    } else {
        c->last_kernel_ms = -1.0;  // read with rt_last_kernel_ms after the caller synchronizes
    }
    return finish_stats(c, b, s);
}

int rt_backend_render_pixels(rt_context* c, int w, int h, int spp, int bounces, const int* xy, int n, float* rgba)
{
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bxy = (size_t)n * 8, brgba = (size_t)n * 16;
    if (int r = ensure(c, b->scratch, bxy + brgba)) return r;
    int* dxy = (int*)b->scratch.p;
    float4_* drgba = (float4_*)((char*)b->scratch.p + bxy);
    HIPCHK(c, hipMemcpy(dxy, xy, bxy, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(drgba, rgba, brgba, hipMemcpyHostToDevice));
    if (c->stats_enabled) HIPCHK(c, hipMemset(b->stats.p, 0, b->stats.bytes));
    rtk::Ctx C{b->view, c->cam, w, h, spp, bounces};
    const int threads = 256, blocks = (n + threads - 1) / threads;
    HIPCHK(c, hipEventRecord(b->ev0, 0));
    if (c->stats_enabled)
        hipLaunchKernelGGL(k_pixels<true>, dim3(blocks), dim3(threads), 0, 0, C, dxy, drgba, n,
                           (unsigned long long*)b->stats.p);
    else
        hipLaunchKernelGGL(k_pixels<false>, dim3(blocks), dim3(threads), 0, 0, C, dxy, drgba, n,
                           (unsigned long long*)b->stats.p);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(b->ev1, 0));
    HIPCHK(c, hipMemcpy(rgba, drgba, brgba, hipMemcpyDeviceToHost));
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    c->last_kernel_ms = ms;
    return finish_stats(c, b, 0);
}

int rt_backend_intersect(rt_context* c, const float* rays, int n, void* out)
{
    Backend* b = be(c);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t br = (size_t)n * 24, bo = (size_t)n * 44;
    if (int r = ensure(c, b->scratch, br + bo)) return r;
    float* dr = (float*)b->scratch.p;
    int32_t* dout = (int32_t*)((char*)b->scratch.p + br);
    HIPCHK(c, hipMemcpy(dr, rays, br, hipMemcpyHostToDevice));
    const int threads = 256, blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(k_intersect, dim3(blocks), dim3(threads), 0, 0, b->view, dr, dout, n);
    HIPCHK(c, hipGetLastError());
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

// Kernel time of the last rt_render_device launch (events recorded on its
// stream); call after synchronizing that stream.
extern "C" double rt_device_last_kernel_ms(rt_context* c)
{
    if (!c || !c->backend) return -1.0;
    Backend* b = be(c);
    float ms = 0;
    if (hipEventElapsedTime(&ms, b->ev0, b->ev1) != hipSuccess) return -1.0;
    c->last_kernel_ms = ms;
    return ms;
}
