// ref_driver.cpp — harness around the REFERENCE implementation (test
// infrastructure, container-only).
//
// This file is ours; it links the reference's own render-path sources, which
// stay where they lie under /root/reference (see oracle/ref/Makefile):
// source/{render_kernel,bvh,flattened_bvh,triangle,vec,color,mat,camera,ray}.cpp.
// It exists to produce golden fixtures (tests/golden/) and the
// "reference"-kind CPU timing. Nothing in the product links it.
//
// Scene ingest is the reference's own source/utils.cpp (Utils::parse_obj,
// Utils::compute_env_map_cdf), compiled and linked by the Makefile. Only the
// env image loader is replaced: the HDR asset is absent, so the synthetic sky
// comes in as a raw RGB f32 file (read_env_raw) and is stored as the same
// Image the reference's read_image_float builds (Color(r, g, b, 0),
// utils.cpp:114-120).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <omp.h>

#include "rapidobj.hpp"

#include "bvh.h"
#include "bvh_tests.h"
#include "camera.h"
#include "flattened_bvh.h"
#include "image.h"
#include "parsed_obj.h"
#include "render_kernel.h"
#include "simple_material.h"
#include "sphere.h"
#include "triangle.h"
#include "utils.h"

// ---------------------------------------------------------------- inputs
static ParsedOBJ parse_obj(const std::string& filepath) { return Utils::parse_obj(filepath); }
static std::vector<float> compute_env_map_cdf(const Image& sky) { return Utils::compute_env_map_cdf(sky); }

// main.cpp:20-30 add_sphere_to_scene (main.cpp holds main(), so it is not linked):
// the sphere's material is appended to the materials and its material index to
// material_indices; the sphere's primitive index is the caller's.
static Sphere add_sphere_to_scene(ParsedOBJ& parsed_obj, const Point& center, float radius,
                                  const SimpleMaterial& material, int primitive_index)
{
    int material_index = parsed_obj.materials.size();
    parsed_obj.materials.push_back(material);
    parsed_obj.material_indices.push_back(material_index);
    return Sphere(center, radius, primitive_index);
}

static Image read_env_raw(const char* path)  // raw stand-in for utils.cpp:100-124
{
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(1); }
    int wh[2];
    if (std::fread(wh, 4, 2, f) != 2) std::exit(1);
    std::vector<float> rgb((size_t)wh[0] * wh[1] * 3);
    if (std::fread(rgb.data(), 4, rgb.size(), f) != rgb.size()) std::exit(1);
    std::fclose(f);
    Image out(wh[0], wh[1]);
    for (int i = 0; i < wh[0] * wh[1]; i++)
        out[i] = Color(rgb[i * 3 + 0], rgb[i * 3 + 1], rgb[i * 3 + 2], 0.0f);
    return out;
}

// ---------------------------------------------------------------- helpers
struct Out {
    FILE* f;
    explicit Out(const char* p) : f(std::fopen(p, "wb")) { if (!f) { std::perror(p); std::exit(1); } }
    ~Out() { std::fclose(f); }
    void i32(int v) { std::fwrite(&v, 4, 1, f); }
    void f32(float v) { std::fwrite(&v, 4, 1, f); }
    template <class T> void raw(const T* p, size_t n) { std::fwrite(p, sizeof(T), n, f); }
};

static Camera camera_by_name(const std::string& n)  // camera.cpp:3-8
{
    if (n == "cornell") return Camera::CORNELL_BOX_CAMERA;
    if (n == "ganesha") return Camera::GANESHA_CAMERA;
    if (n == "ite") return Camera::ITE_ORB_CAMERA;
    if (n == "dragon") return Camera::PBRT_DRAGON_CAMERA;
    if (n == "mis") return Camera::MIS_CAMERA;
    if (n == "default") return Camera();
    // "tele:fov:rx:tx:ty:tz": a camera built the way camera.cpp:3-8 builds the presets,
    // Camera(fov, RotationX(rx) * Translation(tx, ty, tz)) (far telephoto fixtures)
    float fov, rx, tx, ty, tz;
    if (std::sscanf(n.c_str(), "tele:%f:%f:%f:%f:%f", &fov, &rx, &tx, &ty, &tz) == 5)
        return Camera(fov, RotationX(rx) * Translation(tx, ty, tz));
    std::fprintf(stderr, "unknown camera %s\n", n.c_str());
    std::exit(1);
}

static void dump_node(Out& o, const BVH::OctreeNode* n)
{
    o.i32(n->_is_leaf ? 1 : 0);
    o.i32((int)n->_triangles.size());
    for (int t : n->_triangles) o.i32(t);
    o.raw(&n->_min.x, 3);
    o.raw(&n->_max.x, 3);
    o.raw(n->_bounding_volume._d_near.data(), 7);
    o.raw(n->_bounding_volume._d_far.data(), 7);
    if (!n->_is_leaf)
        for (int i = 0; i < 8; i++) dump_node(o, n->_children[i]);
}

static void write_hit(Out& o, bool hit, const HitInfo& h)
{
    o.i32(hit ? 1 : 0);
    o.i32(h.primitive_index);
    o.f32(h.t);
    o.raw(&h.inter_point.x, 3);
    o.raw(&h.normal_at_intersection.x, 3);
    o.f32(h.u);
    o.f32(h.v);
}

struct Scene {
    ParsedOBJ obj;
    std::vector<Sphere> spheres;
    BVH* bvh = nullptr;
    Image sky;
    std::vector<float> cdf;
};

// RT_SPHERES="cx,cy,cz,r,er,eg,eb,dr,dg,db,metalness,roughness;..." adds analytic
// spheres the way main.cpp:74 would with add_sphere_to_scene (primitive index of
// sphere k: the triangle count + k, as main.cpp:74 passes triangles.size()).
static void add_env_spheres(Scene& s)
{
    const char* e = std::getenv("RT_SPHERES");
    if (!e) return;
    std::string spec(e);
    size_t pos = 0;
    while (pos < spec.size()) {
        size_t end = spec.find(';', pos);
        if (end == std::string::npos) end = spec.size();
        float v[12];
        if (std::sscanf(spec.substr(pos, end - pos).c_str(), "%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f", &v[0], &v[1], &v[2],
                        &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11]) != 12) {
            std::fprintf(stderr, "bad RT_SPHERES entry\n");
            std::exit(2);
        }
        SimpleMaterial m{Color(v[4], v[5], v[6]), Color(v[7], v[8], v[9]), v[10], v[11]};
        const int prim = (int)s.obj.triangles.size() + (int)s.spheres.size();
        s.spheres.push_back(add_sphere_to_scene(s.obj, Point(v[0], v[1], v[2]), v[3], m, prim));
        pos = end + 1;
    }
}

static void load_scene(Scene& s, const char* obj, const char* env)
{
    s.obj = parse_obj(obj);
    s.bvh = new BVH(&s.obj.triangles);
    add_env_spheres(s);
    if (env) {
        s.sky = read_env_raw(env);
        s.cdf = compute_env_map_cdf(s.sky);
    }
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr,
                     "usage:\n  ref_driver parse <obj> <out>\n  ref_driver bvh <obj> <out>\n"
                     "  ref_driver bvhtests <obj> <out>\n  ref_driver rays <obj> <rays> <out>\n"
                     "  ref_driver brute <obj> <rays> <out>\n  ref_driver camera <name> <out>\n  ref_driver cdf <env> <out>\n"
                     "  ref_driver render <obj> <env> <camera> W H spp bounces <out>\n"
                     "  ref_driver pixels <obj> <env> <camera> W H spp bounces <pixels> <out>\n");
        return 2;
    }
    const std::string cmd = argv[1];
    if (cmd == "camera") {
        Camera c = camera_by_name(argv[2]);
        Out o(argv[3]);
        o.raw(&c.view_matrix.m[0][0], 16);
        o.f32(c.fov_dist);
        return 0;
    }
    if (cmd == "cdf") {
        Image sky = read_env_raw(argv[2]);
        std::vector<float> cdf = compute_env_map_cdf(sky);
        Out o(argv[3]);
        o.i32(sky.width());
        o.i32(sky.height());
        for (int y = 0; y < sky.height(); y++)
            for (int x = 0; x < sky.width(); x++) o.f32(sky.luminance_of_pixel(x, y));
        o.raw(cdf.data(), cdf.size());
        return 0;
    }
    if (cmd == "parse") {
        ParsedOBJ p = parse_obj(argv[2]);
        Out o(argv[3]);
        o.i32((int)p.triangles.size());
        for (const Triangle& t : p.triangles) { o.raw(&t.m_a.x, 3); o.raw(&t.m_b.x, 3); o.raw(&t.m_c.x, 3); }
        o.i32((int)p.material_indices.size());
        o.raw(p.material_indices.data(), p.material_indices.size());
        o.i32((int)p.materials.size());
        for (const SimpleMaterial& m : p.materials) {
            o.raw(&m.emission.r, 4);
            o.raw(&m.diffuse.r, 4);
            o.f32(m.metalness);
            o.f32(m.roughness);
        }
        o.i32((int)p.emissive_triangle_indices.size());
        o.raw(p.emissive_triangle_indices.data(), p.emissive_triangle_indices.size());
        return 0;
    }
    if (cmd == "bvh") {
        ParsedOBJ p = parse_obj(argv[2]);
        BVH bvh(&p.triangles);
        Out o(argv[3]);
        dump_node(o, bvh._root);
        return 0;
    }
    if (cmd == "bvhtests") {
        // source/tests.cpp:16-58,103-152 with the vectors of include/bvh_tests.h
        ParsedOBJ p = parse_obj(argv[2]);
        BVH bvh(&p.triangles);
        FlattenedBVH flat = bvh.flatten();
        Out o(argv[3]);
        auto emit = [&](const std::vector<Ray>& rays, const std::vector<Point>* expect) {
            o.i32((int)rays.size());
            for (size_t i = 0; i < rays.size(); i++) {
                const Ray& r = rays[i];
                o.raw(&r.origin.x, 3);
                o.raw(&r.direction.x, 3);
                Point e = expect ? (*expect)[i] : Point(0, 0, 0);
                o.raw(&e.x, 3);
                HitInfo h1;
                bool b1 = bvh.intersect(r, h1);
                write_hit(o, b1, h1);
                HitInfo h2;
                bool b2 = flat.intersect(r, h2, p.triangles);
                write_hit(o, b2, h2);
            }
        };
        emit(bvh_test_rays_inter, &bvh_test_rays_inter_result_points);
        emit(bvh_test_rays_no_inter, nullptr);
        return 0;
    }
    if (cmd == "rays") {
        ParsedOBJ p = parse_obj(argv[2]);
        BVH bvh(&p.triangles);
        FILE* f = std::fopen(argv[3], "rb");
        int n;
        if (std::fread(&n, 4, 1, f) != 1) return 1;
        std::vector<float> rv((size_t)n * 6);
        if (std::fread(rv.data(), 4, rv.size(), f) != rv.size()) return 1;
        std::fclose(f);
        std::vector<HitInfo> hits(n);
        std::vector<int> found(n);
#pragma omp parallel for schedule(dynamic, 256)
        for (int i = 0; i < n; i++) {
            Ray r(Point(rv[i * 6 + 0], rv[i * 6 + 1], rv[i * 6 + 2]),
                  Vector(rv[i * 6 + 3], rv[i * 6 + 4], rv[i * 6 + 5]));
            found[i] = bvh.intersect(r, hits[i]) ? 1 : 0;
        }
        Out o(argv[4]);
        o.i32(n);
        for (int i = 0; i < n; i++) write_hit(o, found[i], hits[i]);
        return 0;
    }
    if (cmd == "brute") {
        // RenderKernel::intersect_scene (render_kernel.h:65, render_kernel.cpp:453-483): the
        // brute-force triangle loop + sphere loop, public and compiled in every build, on a
        // ray list; spheres (RT_SPHERES) as main.cpp:74 adds them.
        Scene s;
        load_scene(s, argv[2], nullptr);
        FILE* f = std::fopen(argv[3], "rb");
        int n;
        if (!f || std::fread(&n, 4, 1, f) != 1) return 1;
        std::vector<float> rv((size_t)n * 6);
        if (std::fread(rv.data(), 4, rv.size(), f) != rv.size()) return 1;
        std::fclose(f);
        Image fb(1, 1), sky(1, 1);
        std::vector<float> cdf(1, 0.0f);
        RenderKernel rk(1, 1, 1, 1, fb, s.obj.triangles, s.obj.materials, s.obj.emissive_triangle_indices,
                        s.obj.material_indices, s.spheres, *s.bvh, sky, cdf);
        std::vector<HitInfo> hits(n);
        std::vector<int> found(n);
#pragma omp parallel for schedule(dynamic, 16)
        for (int i = 0; i < n; i++) {
            Ray r(Point(rv[i * 6 + 0], rv[i * 6 + 1], rv[i * 6 + 2]),
                  Vector(rv[i * 6 + 3], rv[i * 6 + 4], rv[i * 6 + 5]));
            found[i] = rk.intersect_scene(r, hits[i]) ? 1 : 0;
        }
        Out o(argv[4]);
        o.i32(n);
        for (int i = 0; i < n; i++) write_hit(o, found[i], hits[i]);
        return 0;
    }
    if (cmd == "render" || cmd == "pixels") {
        if (argc < (cmd == "render" ? 10 : 11)) return 2;
        Scene s;
        load_scene(s, argv[2], argv[3]);
        // optional material override (Cook-Torrance sweep, BASELINE config 5):
        // env RT_MAT_OVERRIDE="index:metalness:roughness"
        if (const char* mo = std::getenv("RT_MAT_OVERRIDE")) {
            int mi;
            float me, ro;
            if (std::sscanf(mo, "%d:%f:%f", &mi, &me, &ro) == 3 && mi >= 0 && mi < (int)s.obj.materials.size()) {
                s.obj.materials[mi].metalness = me;
                s.obj.materials[mi].roughness = ro;
            }
        }
        Camera cam = camera_by_name(argv[4]);
        const int W = std::atoi(argv[5]), H = std::atoi(argv[6]);
        const int spp = std::atoi(argv[7]), bounces = std::atoi(argv[8]);
        Image fb(W, H);
        RenderKernel rk(W, H, spp, bounces, fb, s.obj.triangles, s.obj.materials,
                        s.obj.emissive_triangle_indices, s.obj.material_indices, s.spheres, *s.bvh, s.sky,
                        s.cdf);
        rk.set_camera(cam);
        if (cmd == "render") {
            auto t0 = std::chrono::high_resolution_clock::now();
            rk.render();
            auto t1 = std::chrono::high_resolution_clock::now();
            double sec = std::chrono::duration<double>(t1 - t0).count();
            std::fprintf(stderr, "REF_RENDER_SECONDS %.6f threads %d Msamples/s %.4f\n", sec,
                         omp_get_max_threads(), (double)W * H * spp / sec / 1e6);
            Out o(argv[9]);
            o.raw(fb.data(), (size_t)W * H * 4);
        } else {
            FILE* f = std::fopen(argv[9], "rb");
            int n;
            if (std::fread(&n, 4, 1, f) != 1) return 1;
            std::vector<int> px((size_t)n * 2);
            if (std::fread(px.data(), 4, px.size(), f) != px.size()) return 1;
            std::fclose(f);
            auto t0 = std::chrono::high_resolution_clock::now();
#pragma omp parallel for schedule(dynamic, 16)
            for (int i = 0; i < n; i++) rk.ray_trace_pixel(px[i * 2], px[i * 2 + 1]);
            auto t1 = std::chrono::high_resolution_clock::now();
            double sec = std::chrono::duration<double>(t1 - t0).count();
            std::fprintf(stderr, "REF_PIXELS_SECONDS %.6f threads %d Msamples/s %.4f\n", sec,
                         omp_get_max_threads(), (double)n * spp / sec / 1e6);
            Out o(argv[10]);
            o.i32(n);
            for (int i = 0; i < n; i++) {
                Color c = fb[px[i * 2 + 1] * W + px[i * 2]];
                o.raw(&c.r, 4);
            }
        }
        return 0;
    }
    std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 2;
}
