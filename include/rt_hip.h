/* rt_hip.h — C ABI of librt_hip.so, the MI355X (gfx950) drop-in for the
 * reference's render kernel.
 *
 * Reference interface replaced (TomClabault/SYCL-ray-tracing @ 2024-08-07):
 *   class RenderKernel            include/render_kernel.h:21-96
 *     RenderKernel(...)           include/render_kernel.h:24-46   -> rt_create + rt_set_scene
 *                                                                   + rt_build_bvh / rt_set_bvh_preorder
 *                                                                   + rt_set_env
 *     set_camera(Camera)          include/render_kernel.h:48      -> rt_set_camera
 *     render()                    include/render_kernel.h:57,
 *                                 source/render_kernel.cpp:189-211 -> rt_render / rt_render_device
 *     ray_trace_pixel(x, y)       include/render_kernel.h:56,
 *                                 source/render_kernel.cpp:75-181  -> rt_render_pixels
 *   BVH(triangles, 32, 8)         source/bvh.cpp:19-37            -> rt_build_bvh
 *   BVH::intersect(ray, hit)      source/bvh.cpp:62-65            -> rt_intersect
 *   Camera presets                source/camera.cpp:3-8           -> rt_camera_preset
 *   Utils::parse_obj              source/utils.cpp:16-98          -> rt_mesh_load (+ rt_mesh_*)
 *   Utils::compute_env_map_cdf    source/utils.cpp:126-142        -> rt_env_luminance_cdf
 *
 * Conventions: every function returns 0 (RT_OK) or a negative RT_ERR_*;
 * rt_last_error() gives the message. Inputs are copied (the caller keeps
 * ownership, like the reference's const std::vector& members). Calls are
 * synchronous unless a stream is passed. One context per host thread.
 * Buffer layouts are the reference's in-memory layouts:
 *   triangles  float[n][9]  Triangle{Point m_a, m_b, m_c}       (triangle.h:67)
 *   materials  float[m][10] SimpleMaterial{Color emission (rgba), Color diffuse (rgba),
 *                           metalness, roughness}                (simple_material.h:6-13)
 *   spheres    float[s][5]  Sphere{center xyz, radius, primitive_index (as float)} (sphere.h:7-59)
 *   image      float[h][w][4] Image / Color RGBA                 (image.h:25-178)
 *   view       float[16]    Transform::m row-major, + Camera::fov_dist (camera.h:38-40)
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_ERR_ARG (-1)
#define RT_ERR_HIP (-2)
#define RT_ERR_STATE (-3)
#define RT_ERR_IO (-4)
#define RT_ERR_NODEV (-5)

typedef struct rt_context rt_context;
typedef struct rt_mesh rt_mesh;

/* ---------------------------------------------------------------- context */
int rt_create(int device, rt_context** out);
/* One context over n_devices GPUs of this process (devices[] = HIP ordinals,
 * NULL = 0..n-1; devices[0] is the root). Scene, BVH and env are replicated on
 * every device; a render shards the frame's rows (row j of the request ->
 * device j mod n), ncclScatter's the root framebuffer's rows to their devices,
 * renders every shard on its own device and ncclGather's them back to the root
 * (single-process RCCL clique, ncclCommInitAll). The result is bit-identical to
 * a single-device render. Replaces the OpenMP row loop of RenderKernel::render
 * (render_kernel.cpp:189-211) for a whole node. RT_ERR_NODEV if a device or
 * librccl.so.1 is missing. */
int rt_create_multi(int n_devices, const int* devices, rt_context** out);
int rt_device_count(const rt_context* ctx);
/* TEST ONLY (no reference counterpart). rt_create_multi_loopback: as
 * rt_create_multi, but devices[] may name one GPU more than once and the
 * shards are exchanged by device copies instead of RCCL, so the whole
 * multi-device driver (threads, streams, pack / un-permute) runs on a
 * one-GPU box. rt_test_fail_device: every later multi-device render of ctx
 * fails device d (0..n-1) before its work starts (-1: off), to exercise the
 * per-device error slots. Never called by the product paths. */
int rt_create_multi_loopback(int n_devices, const int* devices, rt_context** out);
/* TEST ONLY. rt_test_create_multi_rccl: as rt_create_multi, but the multi-device
 * driver runs even for one listed device, through a one-rank RCCL clique
 * (ncclCommInitAll over [device]): pack, ncclScatter, render, ncclGather and
 * un-permute, so that a one-GPU box executes the RCCL path the 8-GPU node runs. */
int rt_test_create_multi_rccl(int n_devices, const int* devices, rt_context** out);
int rt_test_fail_device(rt_context* ctx, int device);
/* TEST ONLY. rt_test_schedule: override one wavefront-schedule parameter of
 * ctx's later renders (keys: "lanes", "tail_paths" (0: no tail kernel),
 * "tail_enter", "tail_rows", "drain_rows", "heavy_calls", "spec_cam",
 * "tail_spec_cam", "step_budget", "fast_k" (fast lane: that many of the slowest
 * paths go to a tail kernel early; 0: off), "fast_spp" (... from iteration
 * fast_spp x spp on), "near_scale" (the near box, scene box widened by this x its
 * largest extent: queries from outside it take the exact octree walk), the
 * stressor "force_fallback" (every k-th query by a ray hash skips to the exact
 * octree walk), "reset"). No parameter changes a result; the product never calls
 * it and reads no schedule from the environment. RT_ERR_ARG for an unknown key or
 * a value that is not a finite number in int range. */
int rt_test_schedule(rt_context* ctx, const char* key, double value);
/* TEST ONLY. Walk log of stats renders (rt_set_stats): every search-BVH walk of
 * at least min_calls quad_visit calls (a row trip counts 2) is recorded, up to
 * capacity records (min_calls 0: off); sample_every > 1 keeps only the walks
 * whose (path slot, iteration, kind) hash is 0 modulo it, sample_every < 0 only
 * the k_trace walks left to the exact octree walk (their triangle field then
 * says why: 1 a tie, 2 the octree chain check, 3 the bounded stack). A record is RT_WLOG_FLOATS floats:
 * origin xyz, kind | where << 8 (int bits; where 0 k_trace quads, 1 a k_trace
 * drain's rows, 2 k_tail), direction xyz, calls (int bits), t (closest: the
 * answer, -1 none, -2 left to the exact walk; occlusion: 1 occluded / 0 not),
 * triangle (int bits), iteration (int bits), path slot (int bits).
 * rt_test_walk_log_read copies up to capacity records of the last stats render
 * and returns how many walks qualified (>= the records copied). */
#define RT_WLOG_FLOATS 12
int rt_test_walk_log(rt_context* ctx, int min_calls, int sample_every, int capacity);
long rt_test_walk_log_read(const rt_context* ctx, float* out, long capacity);
void rt_destroy(rt_context* ctx);
const char* rt_last_error(const rt_context* ctx); /* ctx may be NULL: last global error */
int rt_version(void);
/* The build of this library: "src=<hash of its kernel sources> defs=<experiment
 * flags>" (Makefile), so a measurement reports the binary it ran. */
const char* rt_build_id(void);

/* Scene buffers bound by the RenderKernel constructor (render_kernel.h:27-31). */
int rt_set_scene(rt_context* ctx, const float* triangles, int n_triangles, const int* material_indices,
                 int n_material_indices, const float* materials, int n_materials, const int* emissive_triangles,
                 int n_emissive, const float* spheres, int n_spheres);

/* The material buffer alone, for a context whose scene is set: the reference
 * keeps `const std::vector<SimpleMaterial>&` (render_kernel.h:81-93), so a
 * caller may edit materials between render() calls (the cfg5 material sweep);
 * this pushes the new table without rebuilding the octree / search BVH.
 * Material indices must stay in range. */
int rt_set_materials(rt_context* ctx, const float* materials, int n_materials);

/* BVH(&triangles, max_depth, leaf_max_obj_count): native octree build,
 * bit-identical to bvh.h:55-125 (child-box quirk included). */
int rt_build_bvh(rt_context* ctx, int max_depth, int leaf_max_obj_count);
/* Drop-in for a reference-built BVH&: a pre-order walk of BVH::_root, per node
 * {int is_leaf, int n, int tris[n], float min[3], max[3], d_near[7], d_far[7]},
 * children 0..7 after each internal node (INTEGRATION.md shows the walker). */
int rt_set_bvh_preorder(rt_context* ctx, const void* dump, long bytes);
/* Pre-order dump of the context's octree in the same format; returns the size. */
long rt_bvh_dump(const rt_context* ctx, void* buf, long capacity);
/* info[0..4] = octree nodes, GPU child records, triangles, max depth, GPU bytes */
int rt_bvh_info(const rt_context* ctx, long* info);

/* skysphere Image + env_map_cdf (render_kernel.h:33-34). `pixels` has
 * `channels` (3 or 4) floats per texel, row 0 first (as read_image_float
 * leaves it). cdf may be NULL: computed exactly like compute_env_map_cdf. */
int rt_set_env(rt_context* ctx, const float* pixels, int width, int height, int channels, const float* cdf);

/* RenderKernel::set_camera. */
int rt_set_camera(rt_context* ctx, const float view[16], float fov_dist);

/* RenderKernel::render(): fb_rgba (host, w*h*4) is read (accumulated into)
 * and overwritten with the tone-mapped result, exactly as the reference
 * mutates its Image&. */
int rt_render(rt_context* ctx, int width, int height, int samples, int max_bounces, float* fb_rgba);

/* Device-resident render for benchmarking / multi-GPU sharding: renders image
 * rows y = row_offset + j*row_stride (j = 0..) into d_fb (device, rows_local*w*4
 * floats, row j of the shard at offset j*w*4). stream may be NULL (default).
 * Multi-device context: d_fb and stream live on the root device. */
int rt_render_device(rt_context* ctx, int width, int height, int samples, int max_bounces, void* d_fb,
                     int row_offset, int row_stride, void* stream);

/* The Cook-Torrance material sweep (BASELINE config 5) as replicas: n_variants
 * material tables materials[n_variants][n_materials][10] over the bound scene
 * (rt_set_materials semantics for each: no octree / BVH rebuild). Variant v
 * renders rows y = row_offset + j*row_stride of its own frame on device
 * v mod N of the context, each device walking its variants in order on its own
 * stream; the devices run concurrently and exchange nothing. Output: either
 * fb_rgba (host, n_variants blocks of rows_local*w*4 floats, read and overwritten
 * like rt_render's) or d_fbs[v] (device buffers of rows_local*w*4 floats, d_fbs[v]
 * on device v mod N). Synchronous; rt_last_kernel_ms is the slowest device's time.
 * The context's own material table (rt_set_scene / rt_set_materials) is what the
 * next render uses again. Replaces the caller loop of render_kernel.h:81-93
 * (edit the bound std::vector<SimpleMaterial>, render(), repeat). */
int rt_render_variants(rt_context* ctx, int width, int height, int samples, int max_bounces, int n_variants,
                       const float* materials, int n_materials, int row_offset, int row_stride, float* fb_rgba,
                       void* const* d_fbs);

/* ray_trace_pixel for a list of n pixels xy[n][2]: rgba[n][4] holds each
 * pixel's framebuffer value on entry and the tone-mapped value on return. */
int rt_render_pixels(rt_context* ctx, int width, int height, int samples, int max_bounces, const int* xy, int n,
                     float* rgba);

/* BVH::intersect + sphere loop (INTERSECT_SCENE) for n rays rays[n][6]
 * (origin, direction); out[n][11] = {found, primitive, t, point[3],
 * normal[3], u, v} with u = v = -1 (unused downstream). */
int rt_intersect(rt_context* ctx, const float* rays, int n, void* out);

/* USE_BVH (render_kernel.h:13, render_kernel.cpp:504-511): 1 (the reference's
 * build, the default) answers INTERSECT_SCENE with the octree walk
 * (intersect_scene_bvh :485-502); 0 with the brute-force triangle loop
 * (intersect_scene :453-483: closest by strict `<` in buffer order, so the
 * lowest triangle index wins a tie). */
int rt_set_intersect_mode(rt_context* ctx, int use_bvh);

/* Counters of the last render when enabled (RT_STAT_* order, rt_device.h);
 * with n up to 2 * RT_STAT_COUNT the second block is the share of the
 * gfx950 tail kernel (k_tail) in those totals. */
/* enabled = 2: counters of a render whose occlusion walks take one node per trip
 * (the gfx950 walks otherwise pair the stack top's node into the same trip, testing
 * boxes a one-node walk may never reach) and whose walks are all quad walks (no
 * 16-wide row trips in k_trace's drains or the tail kernel): the box tests a walk
 * must make, for the roofline's necessary-bytes figure. Same answers, same frame. */
int rt_set_stats(rt_context* ctx, int enabled);
int rt_get_stats(const rt_context* ctx, unsigned long long* out, int n);
/* Average duration (ms) of the last render kernel measured with HIP events. */
double rt_last_kernel_ms(const rt_context* ctx);

/* ------------------------------------------------- host helpers (no GPU) */
int rt_mesh_load(const char* obj_path, rt_mesh** out);
int rt_mesh_counts(const rt_mesh* m, int* n_triangles, int* n_materials, int* n_emissive);
int rt_mesh_copy(const rt_mesh* m, float* triangles, int* material_indices, float* materials, int* emissive);
void rt_mesh_free(rt_mesh* m);
int rt_camera_preset(const char* name, float view[16], float* fov_dist);
int rt_env_luminance_cdf(const float* pixels, int width, int height, int channels, float* lum, float* cdf);
/* Utils::read_image_float (utils.cpp:100-124) on a Radiance .hdr file, decoded
 * like stb_image 2.28 (stb_image.h:7157-7286) and flipped vertically when
 * flip_y (the reference's default). Call with pixels_rgba == NULL to get the
 * size, then with a w*h*4 float buffer: RGBA, alpha 0 (utils.cpp:119). */
int rt_read_hdr(const char* path, int flip_y, int* width, int* height, float* pixels_rgba);
/* write_image_png (image_io.cpp:165-182): RGBA f32 -> 8 bit exactly as the
 * reference converts (x*255, clamp to [0,255], truncate), rows flipped when
 * flip_y, written as a PNG. rt_image_to_rgba8 is the conversion alone. */
int rt_write_png(const char* path, const float* rgba, int width, int height, int flip_y);
int rt_image_to_rgba8(const float* rgba, long n_pixels, unsigned char* out);
/* TEST ONLY. rt_mesh_load parses files of at least `bytes` in chunks on worker
 * threads (-1: the default, 4 MB; 0: every file, so small test files take the
 * chunked path). */
int rt_test_obj_parallel_min(long bytes);
/* Octree of a triangle buffer without a device (parity tests). */
long rt_octree_dump(const float* triangles, int n_triangles, int max_depth, int leaf_max, void* buf, long capacity);

#ifdef __cplusplus
}
#endif

#endif /* RT_HIP_H */
