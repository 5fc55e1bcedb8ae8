// sanitize_driver.cpp — the CPU build of the render path under ASan + UBSan or
// TSan (`make sanitize`, SURVEY.md §5 "race detection / sanitizers").
//
// One executable links the hostsim backend (the product's device code compiled
// for the host: rt_hostsim.cpp + the C ABI + host ingest), the CPU restatement
// oracle (oracle/cpu_oracle.cpp) and this driver, all built with the sanitizer.
// It runs the paths the CPU test suite covers through Python, as native calls:
//   ingest      rt_mesh_load of cornell_pbr.obj and MIS.obj; octree dump of
//               MIS (3860 triangles, a 12-triangle leaf at depth 32) against the
//               oracle's dump, byte for byte
//   render      a Cornell frame, single context, against the oracle, bitwise
//   multi       the same frame on 2- and 3-"device" contexts (rt_create_multi:
//               one host thread per device, rt_for_devices), bitwise
//   variants    rt_render_variants of 3 tables over 1 and 2 devices, each against
//               a context rendering that table, bitwise
//   failure     rt_test_fail_device: the error surfaces, the context recovers
//   pixels      rt_render_pixels on MIS against the oracle's pixels, bitwise
//   intersect   rt_intersect against oracle_intersect (found, prim, t bits)
//   image io    rt_image_to_rgba8 / rt_write_png of the frame
// Exit status 0 = every check passed (a sanitizer report also fails the run:
// halt_on_error / -fno-sanitize-recover).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"

extern "C" {
void* oracle_scene_create(const float* tris, int ntri, const int* mat_idx, const float* mats, int nmat,
                          const int* emissive, int nem, const float* spheres, int nsph, const float* env_rgb, int ew,
                          int eh, int max_depth, int leaf_max);
void oracle_scene_destroy(void* s);
long oracle_bvh_dump(void* s, char* buf, long cap);
void oracle_intersect(void* s, const float* rays, int n, void* out, uint64_t* counters);
double oracle_render(void* s, const float* view16, float fov_dist, int W, int H, int spp, int bounces, const int* px,
                     long n, float* fb, int nthreads, uint64_t* counters);
}

namespace {
int g_fail = 0;

void check(bool ok, const std::string& what)
{
    std::printf("%-58s %s\n", what.c_str(), ok ? "ok" : "FAIL");
    if (!ok) g_fail++;
}

void rc(int r, const char* what, rt_context* c)
{
    if (r != RT_OK) {
        std::printf("%s failed (%d): %s\n", what, r, rt_last_error(c));
        std::exit(2);
    }
}

struct Mesh {
    std::vector<float> tris, mats;
    std::vector<int> mi, em;
};

Mesh load(const std::string& path)
{
    rt_mesh* m = nullptr;
    rc(rt_mesh_load(path.c_str(), &m), ("rt_mesh_load " + path).c_str(), nullptr);
    int nt = 0, nm = 0, ne = 0;
    rt_mesh_counts(m, &nt, &nm, &ne);
    Mesh o;
    o.tris.resize(9 * (size_t)nt);
    o.mi.resize(nt);
    o.mats.resize(10 * (size_t)nm);
    o.em.resize(ne);
    rt_mesh_copy(m, o.tris.data(), o.mi.data(), o.mats.data(), o.em.data());
    rt_mesh_free(m);
    return o;
}

// a small synthetic sky (tools/scenes.py SKY-S's formula at 64 x 32, with its sun block)
void make_sky(int W, int H, std::vector<float>& rgb, std::vector<float>& rgba)
{
    rgb.assign(3 * (size_t)W * H, 0.0f);
    rgba.assign(4 * (size_t)W * H, 0.0f);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            const float s = (float)y / (float)H;
            float c[3] = {0.3f + 0.5f * s, 0.4f + 0.4f * s, 0.6f + 0.4f * s};
            if (x >= 40 && x < 43 && y >= 25 && y < 28) c[0] = 200.0f, c[1] = 180.0f, c[2] = 150.0f;
            for (int k = 0; k < 3; k++) {
                rgb[3 * ((size_t)y * W + x) + k] = c[k];
                rgba[4 * ((size_t)y * W + x) + k] = c[k];
            }
        }
}

struct Scene {
    Mesh m;
    std::vector<float> sky_rgb, sky_rgba;
    int ew = 64, eh = 32;
    float view[16];
    float fov = 0;
};

rt_context* make_ctx(const Scene& S, const std::vector<int>& devices, const float* mats = nullptr)
{
    rt_context* c = nullptr;
    if (devices.empty())
        rc(rt_create(0, &c), "rt_create", nullptr);
    else
        rc(rt_create_multi((int)devices.size(), devices.data(), &c), "rt_create_multi", nullptr);
    const int nt = (int)S.m.mi.size(), nm = (int)S.m.mats.size() / 10;
    rc(rt_set_scene(c, S.m.tris.data(), nt, S.m.mi.data(), nt, mats ? mats : S.m.mats.data(), nm, S.m.em.data(),
                    (int)S.m.em.size(), nullptr, 0),
       "rt_set_scene", c);
    rc(rt_build_bvh(c, 32, 8), "rt_build_bvh", c);
    rc(rt_set_env(c, S.sky_rgba.data(), S.ew, S.eh, 4, nullptr), "rt_set_env", c);
    rc(rt_set_camera(c, S.view, S.fov), "rt_set_camera", c);
    return c;
}

std::vector<float> blank(int W, int H)
{
    std::vector<float> fb(4 * (size_t)W * H, 0.0f);
    for (size_t i = 3; i < fb.size(); i += 4) fb[i] = 1.0f;
    return fb;
}

bool same_bits(const std::vector<float>& a, const std::vector<float>& b)
{
    return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * 4) == 0;
}

void* oracle_of(const Scene& S, const float* mats = nullptr)
{
    const int nt = (int)S.m.mi.size(), nm = (int)S.m.mats.size() / 10;
    return oracle_scene_create(S.m.tris.data(), nt, S.m.mi.data(), mats ? mats : S.m.mats.data(), nm, S.m.em.data(),
                               (int)S.m.em.size(), nullptr, 0, S.sky_rgb.data(), S.ew, S.eh, 32, 8);
}
}  // namespace

int main(int argc, char** argv)
{
    const std::string dir = argc > 1 ? argv[1] : "scenes";
    const int W = 48, H = 40, spp = 4, nb = 3;

    Scene C;
    C.m = load(dir + "/cornell_pbr.obj");
    make_sky(C.ew, C.eh, C.sky_rgb, C.sky_rgba);
    rc(rt_camera_preset("cornell", C.view, &C.fov), "rt_camera_preset", nullptr);

    // render: single context vs the oracle
    void* oc = oracle_of(C);
    std::vector<float> want = blank(W, H);
    oracle_render(oc, C.view, C.fov, W, H, spp, nb, nullptr, 0, want.data(), 0, nullptr);
    rt_context* c1 = make_ctx(C, {});
    std::vector<float> f1 = blank(W, H);
    rc(rt_render(c1, W, H, spp, nb, f1.data()), "rt_render", c1);
    check(same_bits(f1, want), "render: cornell 48x40x4spp x3 vs oracle (bitwise)");

    // multi: 2 and 3 host "devices" (rt_for_devices threads)
    for (int n : {2, 3}) {
        std::vector<int> ids;
        for (int d = 0; d < n; d++) ids.push_back(d);
        rt_context* cm = make_ctx(C, ids);
        std::vector<float> fm = blank(W, H);
        rc(rt_render(cm, W, H, spp, nb, fm.data()), "rt_render multi", cm);
        check(same_bits(fm, want), "multi: " + std::to_string(n) + " devices vs oracle (bitwise)");
        // failure injection and recovery
        rt_test_fail_device(cm, n - 1);
        std::vector<float> bad = blank(W, H);
        const int r = rt_render(cm, W, H, spp, nb, bad.data());
        check(r == RT_ERR_STATE && std::string(rt_last_error(cm)).find("injected failure") != std::string::npos,
              "failure: device " + std::to_string(n - 1) + " of " + std::to_string(n) + " surfaces");
        rt_test_fail_device(cm, -1);
        std::vector<float> again = blank(W, H);
        rc(rt_render(cm, W, H, spp, nb, again.data()), "rt_render after failure", cm);
        check(same_bits(again, want), "failure: the context renders bitwise again");
        rt_destroy(cm);
    }

    // variants: 3 material tables over 1 and 2 devices vs a context per table
    const int nm = (int)C.m.mats.size() / 10;
    std::vector<float> tabs;
    for (int v = 0; v < 3; v++) {
        std::vector<float> t = C.m.mats;
        for (int i = 1; i < nm; i++) {
            t[10 * i + 8] = (float)v / 3.0f;
            t[10 * i + 9] = 0.05f + 0.3f * (float)v;
        }
        tabs.insert(tabs.end(), t.begin(), t.end());
    }
    std::vector<std::vector<float>> want_v;
    for (int v = 0; v < 3; v++) {
        rt_context* cv = make_ctx(C, {}, tabs.data() + (size_t)v * 10 * nm);
        std::vector<float> f = blank(W, H);
        rc(rt_render(cv, W, H, spp, nb, f.data()), "rt_render variant", cv);
        want_v.push_back(f);
        rt_destroy(cv);
    }
    for (int n : {1, 2}) {
        std::vector<int> ids;
        for (int d = 0; d < n; d++) ids.push_back(d);
        rt_context* cm = make_ctx(C, n == 1 ? std::vector<int>{} : ids);
        std::vector<float> fr;
        for (int v = 0; v < 3; v++) {
            std::vector<float> b = blank(W, H);
            fr.insert(fr.end(), b.begin(), b.end());
        }
        rc(rt_set_stats(cm, 1), "rt_set_stats", cm);
        rc(rt_render_variants(cm, W, H, spp, nb, 3, tabs.data(), nm, 0, 1, fr.data(), nullptr), "rt_render_variants",
           cm);
        bool ok = true;
        for (int v = 0; v < 3; v++)
            ok = ok && std::memcmp(fr.data() + (size_t)v * 4 * W * H, want_v[v].data(), 16 * (size_t)W * H) == 0;
        check(ok, "variants: 3 tables on " + std::to_string(n) + " device(s) (bitwise)");
        std::vector<float> fb = blank(W, H);
        rc(rt_render(cm, W, H, spp, nb, fb.data()), "rt_render after variants", cm);
        check(same_bits(fb, want), "variants: the bound table renders again (bitwise)");
        rt_destroy(cm);
    }

    // image io
    {
        std::vector<unsigned char> px(4 * (size_t)W * H);
        rc(rt_image_to_rgba8(f1.data(), (long)W * H, px.data()), "rt_image_to_rgba8", nullptr);
        const std::string png = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/rt_sanitize.png";
        check(rt_write_png(png.c_str(), f1.data(), W, H, 1) == RT_OK, "image io: rgba8 + png");
        std::remove(png.c_str());
    }
    rt_destroy(c1);
    oracle_scene_destroy(oc);

    // MIS: ingest, octree dump, pixels, intersect
    Scene M;
    M.m = load(dir + "/MIS.obj");
    make_sky(M.ew, M.eh, M.sky_rgb, M.sky_rgba);
    rc(rt_camera_preset("mis", M.view, &M.fov), "rt_camera_preset", nullptr);
    void* om = oracle_of(M);
    {
        const int nt = (int)M.m.mi.size();
        const long n1 = rt_octree_dump(M.m.tris.data(), nt, 32, 8, nullptr, 0);
        std::vector<char> a(n1);
        rt_octree_dump(M.m.tris.data(), nt, 32, 8, a.data(), n1);
        const long n2 = oracle_bvh_dump(om, nullptr, 0);
        std::vector<char> b(n2);
        oracle_bvh_dump(om, b.data(), n2);
        check(n1 == n2 && std::memcmp(a.data(), b.data(), n1) == 0, "ingest: MIS octree dump vs oracle (bytes)");
    }
    rt_context* cmis = make_ctx(M, {});
    {
        const int MW = 64, MH = 64, mspp = 16, mnb = 8;
        std::vector<int> xy;
        for (int i = 0; i < 64; i++) xy.push_back((i * 37) % MW), xy.push_back((i * 11 + 5) % MH);
        const int n = (int)xy.size() / 2;
        std::vector<float> got(4 * (size_t)n, 0.0f), fb = blank(MW, MH);
        for (int i = 0; i < n; i++) got[4 * i + 3] = 1.0f;
        rc(rt_render_pixels(cmis, MW, MH, mspp, mnb, xy.data(), n, got.data()), "rt_render_pixels", cmis);
        oracle_render(om, M.view, M.fov, MW, MH, mspp, mnb, xy.data(), n, fb.data(), 0, nullptr);
        bool ok = true;
        for (int i = 0; i < n; i++)
            ok = ok && std::memcmp(&got[4 * i], &fb[4 * ((size_t)xy[2 * i + 1] * MW + xy[2 * i])], 12) == 0;
        check(ok, "pixels: MIS 64 px x16spp x8 vs oracle (bitwise)");
    }
    {
        const int n = 512;
        std::vector<float> rays(6 * (size_t)n);
        uint32_t s = 12345;
        auto rnd = [&]() { s ^= s << 13, s ^= s >> 17, s ^= s << 5; return (float)(s >> 8) / 16777216.0f; };
        for (int i = 0; i < n; i++) {
            float d[3] = {rnd() - 0.5f, rnd() - 0.5f, rnd() - 0.5f};
            const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            rays[6 * i] = 8.0f * (rnd() - 0.5f), rays[6 * i + 1] = 4.0f * rnd(), rays[6 * i + 2] = 8.0f * (rnd() - 0.5f);
            for (int k = 0; k < 3; k++) rays[6 * i + 3 + k] = d[k] / l;
        }
        std::vector<int32_t> a(11 * (size_t)n), b(11 * (size_t)n);
        rc(rt_intersect(cmis, rays.data(), n, a.data()), "rt_intersect", cmis);
        oracle_intersect(om, rays.data(), n, b.data(), nullptr);
        bool ok = true;
        for (int i = 0; i < n; i++)
            ok = ok && a[11 * i] == b[11 * i] && a[11 * i + 1] == b[11 * i + 1] && a[11 * i + 2] == b[11 * i + 2];
        check(ok, "intersect: 512 MIS rays vs oracle (found, prim, t bits)");
    }
    rt_destroy(cmis);
    oracle_scene_destroy(om);
    std::printf("%s: %d failure(s)\n", argc > 2 ? argv[2] : "sanitize_driver", g_fail);
    return g_fail ? 1 : 0;
}
