// Analysis tool (not product, not a test): per-sample bounce counts of the
// reference integrator, to size a speculative schedule of a pixel's sample
// chain. Builds the oracle's CPU restatement into the same translation unit.
#include "../../oracle/cpu_oracle.cpp"

namespace {
// trace_pixel (cpu_oracle.cpp) with the radiance dropped: per sample, the
// number of hit bounces h (RNG draws = 2 + k*h) and of closest-hit queries.
void chain_pixel(const Ctx& C, int x, int y, uint8_t* hs, uint8_t* qs)
{
    const Scene& S = C.S;
    Rng rng{(uint32_t)(31 + x * y * C.spp)};
    for (int i = 0; i < 10; i++) rng();
    for (int s = 0; s < C.spp; s++) {
        float xj = (x + 0.5f) + rng() - 1.0f;
        float yj = (y + 0.5f) + rng() - 1.0f;
        Ray ray = camera_ray(C, xj, yj);
        int h = 0, q = 0;
        for (int bounce = 0; bounce < C.bounces; bounce++) {
            Hit hit;
            q++;
            if (!intersect_scene(S, ray, hit, nullptr)) break;
            h++;
            const Mat& m = S.mats[S.mat_idx[hit.prim]];
            sample_lights(C, ray, hit, m, rng);
            sample_env(C, ray, hit, m, rng);
            float bpdf;
            V3 dir = v3(0, 0, 0);
            Col brdf = ct_sample(m, -ray.d, hit.n, dir, bpdf, rng);
            if ((brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f) || bpdf < 1.0e-8f || std::isinf(bpdf)) break;
            ray = Ray{hit.p + hit.n * 1.0e-4f, dir};
        }
        hs[s] = (uint8_t)h;
        qs[s] = (uint8_t)q;
    }
}
}  // namespace

extern "C" void probe_chains(void* s, const float* view16, float fov_dist, int W, int H, int spp, int bounces,
                             const int* px, long n, uint8_t* hs, uint8_t* qs)
{
    Cam cam;
    std::memcpy(cam.m, view16, 64);
    cam.fov_dist = fov_dist;
#pragma omp parallel
    {
        Ctx C{*(Scene*)s, cam, W, H, spp, bounces, nullptr, nullptr};
#pragma omp for schedule(dynamic, 4)
        for (long i = 0; i < n; i++)
            chain_pixel(C, px[2 * i], px[2 * i + 1], hs + (size_t)i * spp, qs + (size_t)i * spp);
    }
}
