// rt_scene.h — host-side scene preparation for the HIP render kernel.
//
// Everything here reproduces, bit for bit, the host prerequisites the
// reference render kernel consumes:
//   * OBJ/MTL ingest           -> source/utils.cpp:16-98 (+ rapidobj 1.0.1
//                                 quad split rule, rapidobj.hpp:7164-7225)
//   * octree BVH build         -> include/bvh.h:55-125, source/bvh.cpp:19-60
//   * env luminance + CDF      -> include/image.h:80-85, source/utils.cpp:126-142
//   * camera presets           -> include/camera.h:10-40, source/camera.cpp:3-8
// and adds the GPU flattening (layout described in DESIGN.md §3).
#pragma once

#include <atomic>

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "rt_device.h"

namespace rt {

struct Mesh {
    std::vector<float> tris;      // [N][9]  Triangle{m_a, m_b, m_c}
    std::vector<int> mat_idx;     // [N]     material id + 1 (0 = default)
    std::vector<float> mats;      // [M][10] emission rgba, diffuse rgba, metalness, roughness
    std::vector<int> emissive;    // emissive triangle ids
    int ntris() const { return (int)(tris.size() / 9); }
};

// Parses an OBJ (+ its mtllib) like Utils::parse_obj. Returns 0 or a negative
// error; `err` receives a message.
int load_obj(const std::string& path, Mesh& out, std::string& err);       // chunks parsed by the workers
int load_obj_serial(const std::string& path, Mesh& out, std::string& err);  // one pass, file order

// ---------------------------------------------------------------- octree
struct OctNode {
    float mn[3], mx[3];
    float dn[7], df[7];
    int32_t child[8];             // pool indices (internal nodes)
    std::vector<int32_t> tris;    // leaf triangle ids, insertion order
    bool leaf = true;
};

struct Octree {
    std::vector<OctNode> pool;    // pool[0] = root
    int max_depth = 32, leaf_max = 8;
};

// Parallel over worker threads (build_octree, rt_scene.cpp), the same tree as the
// reference's one-triangle-at-a-time insertion (build_octree_serial).
void build_octree(const float* tris, int ntris, int max_depth, int leaf_max, Octree& out);
void build_octree_serial(const float* tris, int ntris, int max_depth, int leaf_max, Octree& out);

// Host worker threads for scene preparation: OMP_NUM_THREADS / RT_HOST_THREADS if
// set, else the hardware threads (at most 16: a GPU box's CPU share).
int worker_count();
// the OBJ size from which load_obj parses in chunks on worker threads (-1: the default,
// 4 MB); tests set 0 through rt_test_obj_parallel_min to run the chunked path on small files
extern std::atomic<long> g_obj_parallel_min;
// fn(task) for task in [0, n) on up to `workers` threads (dynamic, one task at a time).
void parallel_for(int n, int workers, const std::function<void(int)>& fn);
// Pre-order dump identical to oracle/ref/ref_driver.cpp "bvh".
std::vector<char> dump_octree(const Octree& t);
// Inverse of dump_octree: rebuilds an Octree from a caller's pre-order walk
// of BVH::_root (the drop-in path for a reference-built BVH). 0 or <0.
int octree_from_dump(const char* buf, size_t bytes, Octree& out);

// GPU layout (see rt_device.h for the record formats).
struct FlatBvh {
    std::vector<RtNode> nodes;    // nodes[0] = root record
    std::vector<float4_> tri4;    // 3 records per triangle, leaf order
    std::vector<int32_t> prim2k;  // triangle id -> leaf-order index
    std::vector<int32_t> parent;  // record -> parent record (-1: root)
    std::vector<int32_t> leaf_of; // leaf-order index k -> leaf record
    int max_depth = 0;            // deepest non-empty node
    bool chain_monotone = false;  // every record's planes lie within its parent's
    // search BVH over tri4 (build_search_bvh)
    std::vector<BvhNode> bvh;    // binary SAH build
    std::vector<Bvh4Node> bvh4;  // collapsed 4-wide form the device walks (first bvh4_ntop: breadth-first top)
    int bvh4_ntop = 0;
    // 16-wide form (two bvh4 levels per node, rt_device.h Bvh16): 16 child records per node
    std::vector<Bvh4Child> bvh16;
    // oriented slab per child record (build_slabs): {f16 normal x | y << 16, f16 normal z, lo, hi}
    std::vector<float4_> bvh4s, bvh16s;
    std::vector<float4_> bvh_tri4;
};
void flatten_octree(const Octree& t, const float* tris, int ntris, FlatBvh& out);
// Binned-SAH binary BVH over out.tri4 (leaf size <= 4), boxes padded so that
// any triangle the reference's Moller-Trumbore test reports as hit lies in
// the boxes the traversal enters.
void build_search_bvh(FlatBvh& out);
// Oriented slabs of the search BVH's children (out.bvh4s / bvh16s), from bvh4, bvh16 and
// bvh_tri4; build_search_bvh calls it.
void build_slabs(FlatBvh& out);

// ------------------------------------------------------------------ env
// lum[i] = (float)(0.3086*r + 0.6094*g + 0.0820*b) in double (image.h:80-85)
// cdf[i] = cdf[max(i-1,0)] + lum[i] in float, sequential (utils.cpp:126-142)
void env_luminance_cdf(const float* pix, int w, int h, int channels, float* lum, float* cdf);
// Fence tables of the counting CDF search (rt_trace.h cdf_search_fence):
// [1 + h][272] floats, sequence 0 = the row ends, sequence 1 + y = row y;
// per sequence a[] of length m: 16 block ends at 256 (a[256 j + 255]) then
// 256 block ends at 16 (a[16 j + 15]), +inf past m. Left empty when the
// search would not be exact: a NaN or decreasing CDF entry (the reference's
// probe order then matters), w % 16 != 0, or w or h above 4097.
// Image input / output stages (rt_imageio.cpp): Utils::read_image_float on a
// Radiance .hdr (stb_image 2.28 decode, flipY), RGB out; write_image_png's
// 8-bit conversion and a PNG file (flipY).
int read_hdr(const char* path, bool flip_y, int& width, int& height, std::vector<float>& rgb, std::string& err);
void rgba8(const float* rgba, size_t n_px, unsigned char* out);
int write_png(const char* path, const float* rgba, int w, int h, bool flip_y, std::string& err);
void env_cdf_fences(const float* cdf, const float* row_ends, int w, int h, std::vector<float>& out);

// --------------------------------------------------------------- camera
// Fills view[16] (row-major) and fov_dist for a Camera preset name:
// default | cornell | ganesha | ite | dragon | mis. Returns 0 or -1.
int camera_preset(const std::string& name, float view[16], float* fov_dist);

}  // namespace rt
