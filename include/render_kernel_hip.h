// render_kernel_hip.h — header-only C++ drop-in for the reference's RenderKernel
// (TomClabault/SYCL-ray-tracing include/render_kernel.h:21-96), forwarding to the
// C ABI of librt_hip.so (include/rt_hip.h).
//
// Include it INSTEAD of render_kernel.h, with the reference's include/ on the
// include path (it uses the reference's Triangle, SimpleMaterial, Sphere, BVH,
// Image, Camera types), and link -lrt_hip. Same constructor signature
// (render_kernel.h:24-46), set_camera (:48), render (:57, render_kernel.cpp:189-211)
// and ray_trace_pixel (:56, render_kernel.cpp:75-181).
//
// Semantics kept from the reference:
//  * the kernel holds REFERENCES to the caller's buffers (render_kernel.h:81-93):
//    the material vector is re-read on every render() / ray_trace_pixel() and
//    pushed with rt_set_materials when it changed (the cfg5 material sweep edits
//    it between renders without an octree rebuild). The triangles, the BVH& (handed
//    over as a pre-order walk of BVH::_root, so the GPU walks the caller's tree),
//    the sky and its CDF are bound at construction, as a rebuilt BVH would be.
//  * render() mutates the Image& in place: fb += sample average, then the tone-map
//    (render_kernel.cpp:167-180), alpha included.
// Differences: errors throw std::runtime_error (the reference's class has none);
// the devices are chosen by the trailing `device_count` argument or RT_DEVICES
// (default 1): N > 1 shards the frame's rows over devices 0..N-1 with RCCL
// (rt_create_multi), bit-identical to one device.
#ifndef RENDER_KERNEL_HIP_H
#define RENDER_KERNEL_HIP_H

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_hip.h"

#include "bvh.h"
#include "camera.h"
#include "image.h"
#include "simple_material.h"
#include "sphere.h"
#include "triangle.h"

class RenderKernel {
public:
    RenderKernel(int width, int height, int render_samples, int max_bounces, Image& image_buffer,
                 const std::vector<Triangle>& triangle_buffer, const std::vector<SimpleMaterial>& materials_buffer,
                 const std::vector<int>& emissive_triangle_indices_buffer,
                 const std::vector<int>& materials_indices_buffer, const std::vector<Sphere>& analytic_spheres_buffer,
                 BVH& bvh, const Image& skysphere, const std::vector<float>& env_map_cdf, int device_count = 0)
        : m_width(width), m_height(height), m_render_samples(render_samples), m_max_bounces(max_bounces),
          m_frame_buffer(image_buffer), m_materials_buffer(materials_buffer)
    {
        static_assert(sizeof(Triangle) == 9 * sizeof(float), "Triangle is 3 Points (triangle.h:67)");
        static_assert(sizeof(SimpleMaterial) == 10 * sizeof(float), "SimpleMaterial is 2 Colors + 2 floats");
        if (device_count <= 0) {
            const char* e = std::getenv("RT_DEVICES");
            device_count = e ? std::atoi(e) : 1;
        }
        if (device_count > 1)
            check(rt_create_multi(device_count, nullptr, &m_ctx));
        else
            check(rt_create(0, &m_ctx));
        std::vector<float> sph;
        for (const Sphere& s : analytic_spheres_buffer)
            sph.insert(sph.end(), {s.center.x, s.center.y, s.center.z, s.radius, (float)s.primitive_index});
        check(rt_set_scene(m_ctx, reinterpret_cast<const float*>(triangle_buffer.data()), (int)triangle_buffer.size(),
                           materials_indices_buffer.data(), (int)materials_indices_buffer.size(),
                           reinterpret_cast<const float*>(materials_buffer.data()), (int)materials_buffer.size(),
                           emissive_triangle_indices_buffer.data(), (int)emissive_triangle_indices_buffer.size(),
                           sph.data(), (int)analytic_spheres_buffer.size()));
        m_materials_sent = materials_bytes();
        // the caller's octree (BVH::_root is public, bvh.h:276-279), as a pre-order walk
        std::vector<char> dump;
        preorder(bvh._root, dump);
        check(rt_set_bvh_preorder(m_ctx, dump.data(), (long)dump.size()));
        check(rt_set_env(m_ctx, skysphere.data(), skysphere.width(), skysphere.height(), 4,
                         env_map_cdf.empty() ? nullptr : env_map_cdf.data()));
    }

    ~RenderKernel() { rt_destroy(m_ctx); }
    RenderKernel(const RenderKernel&) = delete;
    RenderKernel& operator=(const RenderKernel&) = delete;

    void set_camera(Camera camera)  // render_kernel.h:48
    {
        check(rt_set_camera(m_ctx, &camera.view_matrix.m[0][0], camera.fov_dist));
    }

    void render()  // render_kernel.cpp:189-211
    {
        std::lock_guard<std::mutex> lk(m_mu);
        sync_materials();
        check(rt_render(m_ctx, m_width, m_height, m_render_samples, m_max_bounces, m_frame_buffer.data()));
    }

    // Thread-safe like the reference's (whose render() calls it from an OpenMP parallel-for,
    // render_kernel.cpp:189-211): calls on one kernel are serialized, since they share the
    // context's device buffers and the material-sync state. For throughput, hand pixel
    // batches to rt_render_pixels (or call render()) instead of one pixel per call.
    void ray_trace_pixel(int x, int y) const  // render_kernel.cpp:75-181
    {
        std::lock_guard<std::mutex> lk(m_mu);
        const_cast<RenderKernel*>(this)->sync_materials();
        const int xy[2] = {x, y};
        Color& px = m_frame_buffer.color_data()[y * m_width + x];
        check(rt_render_pixels(m_ctx, m_width, m_height, m_render_samples, m_max_bounces, xy, 1,
                               reinterpret_cast<float*>(&px)));
    }

    int device_count() const { return rt_device_count(m_ctx); }

private:
    static void check(int rc)
    {
        if (rc != RT_OK) throw std::runtime_error(std::string("librt_hip: ") + rt_last_error(nullptr));
    }

    std::vector<char> materials_bytes() const
    {
        const char* p = reinterpret_cast<const char*>(m_materials_buffer.data());
        return std::vector<char>(p, p + m_materials_buffer.size() * sizeof(SimpleMaterial));
    }

    void sync_materials()
    {
        std::vector<char> now = materials_bytes();
        if (now == m_materials_sent) return;
        check(rt_set_materials(m_ctx, reinterpret_cast<const float*>(m_materials_buffer.data()),
                               (int)m_materials_buffer.size()));
        m_materials_sent.swap(now);
    }

    // {int is_leaf, int n, int tris[n], float min[3], max[3], d_near[7], d_far[7]}, children after
    // each internal node (the rt_set_bvh_preorder format)
    static void preorder(const BVH::OctreeNode* n, std::vector<char>& out)
    {
        auto put = [&](const void* p, size_t b) { out.insert(out.end(), (const char*)p, (const char*)p + b); };
        const int leaf = n->_is_leaf ? 1 : 0, cnt = (int)n->_triangles.size();
        put(&leaf, 4);
        put(&cnt, 4);
        put(n->_triangles.data(), 4 * (size_t)cnt);
        put(&n->_min.x, 12);
        put(&n->_max.x, 12);
        put(n->_bounding_volume._d_near.data(), 28);
        put(n->_bounding_volume._d_far.data(), 28);
        if (!n->_is_leaf)
            for (int i = 0; i < 8; i++) preorder(n->_children[i], out);
    }

    rt_context* m_ctx = nullptr;
    int m_width, m_height, m_render_samples, m_max_bounces;
    Image& m_frame_buffer;
    const std::vector<SimpleMaterial>& m_materials_buffer;
    std::vector<char> m_materials_sent;
    mutable std::mutex m_mu;  // one call on the context at a time (ray_trace_pixel is const and may be threaded)
};

#endif  // RENDER_KERNEL_HIP_H
