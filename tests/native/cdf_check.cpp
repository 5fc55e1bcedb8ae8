// cdf_check — the counting CDF search (rt_trace.h fence_count, fence tables
// from rt_scene.cpp env_cdf_fences) against the reference's binary search
// loop (render_kernel.cpp:532-567) on adversarial sequences: long flat runs
// (zero-luminance texels), duplicates at fence positions, values below /
// equal to / above every entry, +inf and NaN values, lengths 1..4096.
// Exit status 0 iff every search agrees.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "rt_scene.h"
#include "rt_trace.h"

static int ref_search(const float* a, int n, float v)  // the reference's loop over [0, n - 1]
{
    int lower = 0, upper = n - 1;
    while (lower < upper) {
        const int mid = (lower + upper) / 2;
        if (v < a[mid])
            upper = mid;
        else
            lower = mid + 1;
    }
    return lower;
}

int main()
{
    std::mt19937 rng(7);
    long bad = 0, checked = 0;
    const int widths[] = {16, 32, 48, 512, 1024, 2048, 4096};
    const int heights[] = {1, 2, 3, 17, 255, 256, 1024, 4097};
    for (int w : widths)
        for (int h : heights) {
            if ((long)w * h > (1l << 22)) continue;
            const size_t n = (size_t)w * h;
            // luminance: mostly zero runs, some equal values, a few large
            std::vector<float> lum(n), cdf(n);
            std::uniform_real_distribution<float> U(0.0f, 1.0f);
            for (size_t i = 0; i < n; i++) {
                const float r = U(rng);
                lum[i] = r < 0.6f ? 0.0f : (r < 0.8f ? 0.25f : r * 3.0f);
            }
            float s = 0.0f;
            for (size_t i = 0; i < n; i++) cdf[i] = s = s + lum[i];
            std::vector<float> rows(((size_t)h + 15) & ~(size_t)15, 0.0f);
            for (int y = 0; y < h; y++) rows[y] = cdf[(size_t)y * w + w - 1];
            std::vector<float> fence;
            rt::env_cdf_fences(cdf.data(), rows.data(), w, h, fence);
            if (fence.empty()) {
                std::printf("no fences for %dx%d\n", w, h);
                return 1;
            }
            std::vector<float> vals = {-1.0f, 0.0f, cdf[0], cdf[n - 1], cdf[n - 1] * 2, INFINITY, -INFINITY, NAN};
            for (int k = 0; k < 2000; k++) vals.push_back(U(rng) * cdf[n - 1]);
            for (int k = 0; k < 500; k++) vals.push_back(cdf[rng() % n]);  // exact entry values (ties)
            for (float v : vals) {
                const int ry = ref_search(rows.data(), h, v);
                const int my = rtk::fence_count(rows.data(), fence.data(), h - 1, v);
                const int rx = ref_search(cdf.data() + (size_t)ry * w, w, v);
                const int mx = rtk::fence_count(cdf.data() + (size_t)ry * w, fence.data() + (size_t)(1 + ry) * 272, w - 1, v);
                checked++;
                if (ry != my || rx != mx) {
                    if (bad < 10) std::printf("mismatch %dx%d v=%a: ref (%d,%d) fence (%d,%d)\n", w, h, v, rx, ry, mx, my);
                    bad++;
                }
            }
        }
    // ineligible tables: NaN entry, decreasing entry, width not a multiple of 16
    std::vector<float> out, a(16, 1.0f), r(16, 0.0f);
    a[3] = NAN;
    rt::env_cdf_fences(a.data(), r.data(), 16, 1, out);
    const bool nan_rejected = out.empty();
    std::vector<float> b(32, 1.0f);
    b[5] = 0.5f;
    rt::env_cdf_fences(b.data(), r.data(), 16, 2, out);
    const bool dec_rejected = out.empty();
    std::printf("cdf_check: %ld searches, %ld mismatches; NaN table rejected %d, decreasing rejected %d\n", checked, bad,
                nan_rejected, dec_rejected);
    return (bad == 0 && nan_rejected && dec_rejected) ? 0 : 1;
}
