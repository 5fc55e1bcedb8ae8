// shim_test.cpp — compiles include/render_kernel_hip.h (the C++ drop-in RenderKernel)
// against the REFERENCE's own headers and types (/root/reference/include) and drives it
// the way the reference's main.cpp:66-122 drives render_kernel.h: parse the OBJ with
// Utils::parse_obj, build BVH(&triangles), compute_env_map_cdf, construct, set_camera,
// render(). Container test (tests/test_shim.py): linked against librt_hostsim.so (the
// same C ABI; the GPU box has no /root/reference). Writes the frame, then checks the
// by-reference material semantics: an in-place edit of the material vector between
// renders gives the frame a fresh kernel over the edited vector gives, and ray_trace_pixel
// called from an OpenMP parallel-for (the reference's render() loop) gives render()'s frame.
//   shim_test <obj> <sky.raw> <camera> W H spp bounces <out.f32>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "image.h"
#include "utils.h"
#include "render_kernel_hip.h"

static Image read_sky_raw(const char* path)  // int w, h; float rgb[h][w][3]
{
    FILE* f = std::fopen(path, "rb");
    if (!f) std::exit(3);
    int wh[2];
    if (std::fread(wh, 4, 2, f) != 2) std::exit(3);
    std::vector<float> rgb((size_t)wh[0] * wh[1] * 3);
    if (std::fread(rgb.data(), 4, rgb.size(), f) != rgb.size()) std::exit(3);
    std::fclose(f);
    Image out(wh[0], wh[1]);
    for (int i = 0; i < wh[0] * wh[1]; i++) out[i] = Color(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.0f);
    return out;
}

int main(int argc, char** argv)
{
    if (argc < 9) return 2;
    const std::string cam_name = argv[3];
    const int W = std::atoi(argv[4]), H = std::atoi(argv[5]), spp = std::atoi(argv[6]), nb = std::atoi(argv[7]);
    ParsedOBJ obj = Utils::parse_obj(argv[1]);
    BVH bvh(&obj.triangles);
    Image sky = read_sky_raw(argv[2]);
    std::vector<float> cdf = Utils::compute_env_map_cdf(sky);
    std::vector<Sphere> spheres;
    Camera cam = cam_name == "dragon" ? Camera::PBRT_DRAGON_CAMERA : Camera::CORNELL_BOX_CAMERA;

    Image fb(W, H);
    std::vector<SimpleMaterial> mats = obj.materials;
    RenderKernel rk(W, H, spp, nb, fb, obj.triangles, mats, obj.emissive_triangle_indices, obj.material_indices,
                    spheres, bvh, sky, cdf);
    rk.set_camera(cam);
    rk.render();
    FILE* f = std::fopen(argv[8], "wb");
    std::fwrite(fb.data(), 4, (size_t)W * H * 4, f);
    std::fclose(f);
    const std::vector<float> first(fb.data(), fb.data() + (size_t)W * H * 4);

    // by-reference materials: edit in place, render again into a fresh frame
    for (size_t i = 1; i < mats.size(); i++) {
        mats[i].metalness = 0.75f;
        mats[i].roughness = 0.2f;
    }
    Image fb2(W, H);
    {
        RenderKernel rk2(W, H, spp, nb, fb2, obj.triangles, mats, obj.emissive_triangle_indices,
                         obj.material_indices, spheres, bvh, sky, cdf);
        rk2.set_camera(cam);
        rk2.render();
    }
    // rk keeps its frame reference: reuse it over a reset frame
    fb = Image(W, H);
    rk.render();
    const bool same = std::memcmp(fb.data(), fb2.data(), (size_t)W * H * 16) == 0;
    const bool edited = std::memcmp(fb.data(), first.data(), (size_t)W * H * 16) != 0;
    // ray_trace_pixel (render_kernel.h:56) over a reset pixel gives the frame's value
    const int px = W / 3, py = H / 2;
    const Color want = fb[py * W + px];
    fb[py * W + px] = Color();
    rk.ray_trace_pixel(px, py);
    const bool pixel_ok = std::memcmp(&fb[py * W + px], &want, 16) == 0 || (want.r != want.r);
    // the reference's own render() pattern (render_kernel.cpp:189-211): ray_trace_pixel from an
    // OpenMP parallel-for over rows, on one kernel (its calls serialize on the context)
    // (every 8th row: one pixel per call is the slow way to drive a context)
    const std::vector<float> after(fb.data(), fb.data() + (size_t)W * H * 4);
    fb = Image(W, H);
#pragma omp parallel for schedule(dynamic)
    for (int y = 0; y < H; y += 8)
        for (int x = 0; x < W; x++) rk.ray_trace_pixel(x, y);
    bool threaded_ok = true;
    for (int y = 0; y < H; y += 8)
        threaded_ok = threaded_ok && std::memcmp(fb.data() + (size_t)y * W * 4, after.data() + (size_t)y * W * 4, (size_t)W * 16) == 0;
    std::printf("SHIM devices %d materials_by_reference %d changed %d pixel %d threaded %d\n", rk.device_count(),
                same ? 1 : 0, edited ? 1 : 0, pixel_ok ? 1 : 0, threaded_ok ? 1 : 0);
    return same && edited && pixel_ok && threaded_ok ? 0 : 1;
}
