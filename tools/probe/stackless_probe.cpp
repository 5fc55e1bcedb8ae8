// stackless_probe.cpp — CPU study: stackless occlusion walks vs the product's short stack
// (north star: "stackless FlattenedBVH traversal").
//
// A walk on the GPU is a chain of dependent memory round trips ("trips": one per inner node
// whose four child records a quad loads, one per leaf whose triangles it loads); a pop from
// the quad's LDS stack is ~100 cycles against a ~0.5-1.3 us trip. This tool replays
// occlusion rays over the product's own search BVH (rt_scene.cpp build_search_bvh + its
// oriented slabs, the rt_fast.h box4 test) and counts the trips of four walks with the
// same answer (any Moller-Trumbore hit; the octree chain check is left out, as it is the
// same for all four):
//   stack      rt_quad.h quad_visit<ANY, PAIR = false>: one node per trip, first hit
//              child next, the other hit children pushed (LDS), pop on a dead end
//   paired     the product's trip: the current node and the stack top's inner node
//   parent     stackless with parent links (Hapala et al. 2011, 4-wide): after a subtree
//              the walk returns to its parent and must load it again to find the next hit
//              child after the one it came from (no stack, one extra trip per return)
//   skip       stackless with skip links (a threaded tree): one child box per trip, a hit
//              descends, a miss or a finished subtree follows the skip link to the next box
//              in depth-first order (no stack, no re-tests, no 4-wide trip)
// Rays: origins on uniformly chosen surface points (1e-4 off the surface, as the
// renderer's shadow origins, render_kernel.cpp:592), directions cosine-distributed about
// the normal (env and BRDF->env occlusion rays) or within ~2 degrees of the tangent plane
// (the grazing rays that make the longest walks, profiles/r05_walk_attrib).
// Usage: stackless_probe OBJ OUT.json [n_rays]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "rt_scene.h"
#include "rt_fast.h"

namespace {

using rtk::V3;

struct Walker {
    const RtSceneView& S;
    std::vector<int> parent, slot;  // 4-wide node -> parent node and its child slot there (root: -1)

    explicit Walker(const RtSceneView& s, int nn) : S(s), parent(nn, -1), slot(nn, -1)
    {
        for (int i = 0; i < nn; i++)
            for (int c = 0; c < 4; c++) {
                const Bvh4Child& ch = S.bvh4[i].ch[c];
                if (ch.cnt == 0) parent[ch.ref] = i, slot[ch.ref] = c;
            }
    }
    void test(int node, const rtk::RayB& rb, V3 o, V3 d, bool* hit) const
    {
        const rtk::Bvh4R n = rtk::load_bvh4(S.bvh4, node);
        float tn[4];
        rtk::box4(S, node, n, rb, o, d, __builtin_inff(), tn, hit);
    }
    bool leaf_hit(int first, int cnt, V3 o, V3 d) const
    {
        for (int j = 0; j < cnt; j++) {
            const float4_* r = S.bvh_tri4 + 3 * (size_t)(first + j);
            float t;
            if (rtk::tri_test_v(rtk::ld3(r[0]), rtk::ld3(r[1]), rtk::ld3(r[2]), o, d, t)) return true;
        }
        return false;
    }
    // stack walk, one node per trip (PAIR false) or the stack top's inner node too (PAIR true)
    long stack_walk(V3 o, V3 d, bool pair, bool& hit_out, int& maxdepth) const
    {
        const rtk::RayB rb = rtk::rayb_setup(o, d);
        std::vector<int> st;  // items: node >= 0, leaf ~(first << 3 | cnt)
        long trips = 0;
        int cur = 0;
        hit_out = false;
        maxdepth = 0;
        for (;;) {
            if (cur >= 0) {
                int nodes[2] = {cur, -1};
                if (pair && !st.empty() && st.back() >= 0) nodes[1] = st.back(), st.pop_back();
                trips++;
                int first = -1;
                for (int k = 0; k < 2; k++) {
                    if (nodes[k] < 0) continue;
                    bool h[4];
                    test(nodes[k], rb, o, d, h);
                    for (int c = 0; c < 4; c++) {
                        if (!h[c]) continue;
                        const Bvh4Child& ch = S.bvh4[nodes[k]].ch[c];
                        const int it = ch.cnt > 0 ? ~((ch.ref << 3) | ch.cnt) : ch.ref;
                        if (first == -1 && it != -1)
                            first = it;
                        else
                            st.push_back(it);
                    }
                }
                maxdepth = std::max(maxdepth, (int)st.size());
                if (first != -1) {
                    cur = first;
                    continue;
                }
            } else {
                trips++;
                const int v = ~cur;
                if (leaf_hit(v >> 3, v & 7, o, d)) {
                    hit_out = true;
                    return trips;
                }
            }
            if (st.empty()) return trips;
            cur = st.back();
            st.pop_back();
        }
    }
    // closest-hit walk with the quad walk's rule (rt_quad.h: nearest hit child next, the rest
    // on the stack by entry distance, entries beyond t*(1 + RT_T2_WINDOW) dropped), started at
    // node `start`; then (ancestor start) for every ancestor of `start` up to the root one more
    // trip tests that ancestor's other children against the window and walks the ones hit.
    // Returns trips; t_out = the closest M-T t (-1 none).
    long closest_walk(V3 o, V3 d, int start, float& t_out) const
    {
        const rtk::RayB rb = rtk::rayb_setup(o, d);
        float best = __builtin_inff();
        long trips = 0;
        std::vector<std::pair<float, int>> st;  // (entry, item)
        auto window = [&]() { return best + best * RT_T2_WINDOW; };
        auto walk_from = [&](int item) {
            int cur = item;
            for (;;) {
                trips++;
                if (cur >= 0) {
                    const rtk::Bvh4R n = rtk::load_bvh4(S.bvh4, cur);
                    float tn[4];
                    bool h[4];
                    rtk::box4(S, cur, n, rb, o, d, window(), tn, h);
                    std::vector<std::pair<float, int>> hit;
                    for (int c = 0; c < 4; c++)
                        if (h[c] && tn[c] <= window())
                            hit.push_back({tn[c], n.cnt[c] > 0 ? ~((n.ref[c] << 3) | n.cnt[c]) : n.ref[c]});
                    std::sort(hit.begin(), hit.end());
                    for (int j = (int)hit.size() - 1; j >= 1; j--) st.push_back(hit[j]);
                    if (!hit.empty()) {
                        cur = hit[0].second;
                        continue;
                    }
                } else {
                    const int v = ~cur;
                    for (int j = 0; j < (v & 7); j++) {
                        const float4_* r = S.bvh_tri4 + 3 * (size_t)((v >> 3) + j);
                        float t;
                        if (rtk::tri_test_v(rtk::ld3(r[0]), rtk::ld3(r[1]), rtk::ld3(r[2]), o, d, t)) best = std::min(best, t);
                    }
                }
                cur = INT32_MIN;
                while (!st.empty()) {
                    const auto e = st.back();
                    st.pop_back();
                    if (e.first <= window()) {
                        cur = e.second;
                        break;
                    }
                }
                if (cur == INT32_MIN) return;
            }
        };
        walk_from(start);
        for (int a = start; a != 0; a = parent[a]) {  // the ancestors' other children
            const int p = parent[a];
            trips++;
            const rtk::Bvh4R n = rtk::load_bvh4(S.bvh4, p);
            float tn[4];
            bool h[4];
            rtk::box4(S, p, n, rb, o, d, window(), tn, h);
            for (int c = 0; c < 4; c++) {
                if (c == slot[a] || !h[c] || !(tn[c] <= window())) continue;
                walk_from(n.cnt[c] > 0 ? ~((n.ref[c] << 3) | n.cnt[c]) : n.ref[c]);
            }
        }
        t_out = best == __builtin_inff() ? -1.0f : best;
        return trips;
    }
    // stackless, parent links: state (node, the child slot the walk last came back from)
    long parent_walk(V3 o, V3 d, bool& hit_out) const
    {
        const rtk::RayB rb = rtk::rayb_setup(o, d);
        long trips = 0;
        int cur = 0, from = -1;
        hit_out = false;
        for (;;) {
            trips++;  // (re)load cur's four children
            bool h[4];
            test(cur, rb, o, d, h);
            int next = -1;
            for (int c = from + 1; c < 4; c++) {
                if (!h[c]) continue;
                const Bvh4Child& ch = S.bvh4[cur].ch[c];
                if (ch.cnt > 0) {  // leaf child: its triangles, then on with the next slot (mask in registers)
                    trips++;
                    if (leaf_hit(ch.ref, ch.cnt, o, d)) {
                        hit_out = true;
                        return trips;
                    }
                    continue;
                }
                next = c;
                break;
            }
            if (next >= 0) {
                cur = S.bvh4[cur].ch[next].ref;
                from = -1;
                continue;
            }
            if (cur == 0) return trips;  // root exhausted
            from = slot[cur];
            cur = parent[cur];
        }
    }
    // stackless, skip links: one child box per trip in depth-first order
    long skip_walk(V3 o, V3 d, bool& hit_out) const
    {
        const rtk::RayB rb = rtk::rayb_setup(o, d);
        long trips = 0;
        hit_out = false;
        // position = (node, child slot); the skip link of a child is the next slot of its node,
        // or (after the last) the skip of the node's own slot in its parent
        int node = 0, c = 0;
        auto advance = [&]() {  // to the next box in DFS order after (node, c)'s subtree
            for (;;) {
                if (++c < 4) return true;
                if (node == 0) return false;
                c = slot[node];
                node = parent[node];
            }
        };
        for (;;) {
            const Bvh4Child& ch = S.bvh4[node].ch[c];
            bool ok = false;
            if (ch.cnt >= 0) {
                trips++;  // one child record (+ its slab)
                const float mn[3] = {ch.lo[0], ch.lo[1], ch.lo[2]}, mx[3] = {ch.hi[0], ch.hi[1], ch.hi[2]};
                float tn, tf;
                ok = rtk::box_hit2(mn, mx, rb, __builtin_inff(), tn, tf) &&
                     rtk::slab_ok(S.bvh4s[4 * (size_t)node + c], o, d, tn, tf);
            }
            if (ok && ch.cnt > 0) {
                trips++;
                if (leaf_hit(ch.ref, ch.cnt, o, d)) {
                    hit_out = true;
                    return trips;
                }
            } else if (ok) {
                node = ch.ref;
                c = 0;
                continue;
            }
            if (!advance()) return trips;
        }
    }
};

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: stackless_probe OBJ OUT.json [n_rays]\n");
        return 2;
    }
    const int n_rays = argc > 3 ? std::atoi(argv[3]) : 200000;
    rt::Mesh m;
    std::string err;
    if (rt::load_obj(argv[1], m, err)) {
        std::fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const int nt = m.ntris();
    rt::Octree oc;
    rt::build_octree(m.tris.data(), nt, 32, 8, oc);
    rt::FlatBvh fb;
    rt::flatten_octree(oc, m.tris.data(), nt, fb);
    rt::build_search_bvh(fb);
    RtSceneView S{};
    S.bvh4 = fb.bvh4.data();
    S.bvh4s = fb.bvh4s.data();
    S.bvh_tri4 = fb.bvh_tri4.data();
    Walker W(S, (int)fb.bvh4.size());
    // the 4-wide node holding each leaf-order triangle k (the "hit leaf" of a ray leaving k)
    std::vector<int> node_of_k(nt, -1);
    for (int i = 0; i < (int)fb.bvh4.size(); i++)
        for (const Bvh4Child& ch : fb.bvh4[i].ch)
            if (ch.cnt > 0)
                for (int j = 0; j < ch.cnt; j++) {
                    int k;  // build_search_bvh stores the leaf-order index in the first record's w
                    std::memcpy(&k, &fb.bvh_tri4[3 * (size_t)(ch.ref + j)].w, 4);
                    if (k >= 0 && k < nt) node_of_k[k] = i;
                }

    FILE* out = std::fopen(argv[2], "w");
    std::fprintf(out, "{\"what\": \"trips (dependent memory round trips) per occlusion walk over the product's search BVH, "
                      "%d rays per set, %s (%d triangles): stack = rt_quad.h one node per trip; paired = the product's "
                      "trip (current node + the stack top's inner node); parent = stackless with parent links (a return "
                      "reloads the parent); skip = stackless with skip links (one child box per trip)\", \"sets\": {",
                 n_rays, argv[1], nt);
    for (int set = 0; set < 2; set++) {
        std::mt19937_64 rng(1234 + set);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        std::vector<double> tr[4];
        long hits = 0, mism = 0;
        int maxdepth_all = 0;
        for (int i = 0; i < n_rays; i++) {
            const int k = (int)(U(rng) * nt) % nt;
            const float* t = &m.tris[9 * (size_t)k];
            double a[3], e1[3], e2[3], nrm[3];
            for (int j = 0; j < 3; j++) a[j] = t[j], e1[j] = t[3 + j] - t[j], e2[j] = t[6 + j] - t[j];
            nrm[0] = e1[1] * e2[2] - e1[2] * e2[1], nrm[1] = e1[2] * e2[0] - e1[0] * e2[2], nrm[2] = e1[0] * e2[1] - e1[1] * e2[0];
            const double ln = std::sqrt(nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2]);
            if (!(ln > 0)) continue;
            for (double& x : nrm) x /= ln;
            double r1 = U(rng), r2 = U(rng);
            if (r1 + r2 > 1) r1 = 1 - r1, r2 = 1 - r2;
            double p[3];
            for (int j = 0; j < 3; j++) p[j] = a[j] + r1 * e1[j] + r2 * e2[j] + 1e-4 * nrm[j];
            // tangent frame
            double tx[3] = {1, 0, 0};
            if (std::fabs(nrm[0]) > 0.9) tx[0] = 0, tx[1] = 1;
            double ty[3] = {nrm[1] * tx[2] - nrm[2] * tx[1], nrm[2] * tx[0] - nrm[0] * tx[2], nrm[0] * tx[1] - nrm[1] * tx[0]};
            const double lt = std::sqrt(ty[0] * ty[0] + ty[1] * ty[1] + ty[2] * ty[2]);
            for (double& x : ty) x /= lt;
            double tz[3] = {ty[1] * nrm[2] - ty[2] * nrm[1], ty[2] * nrm[0] - ty[0] * nrm[2], ty[0] * nrm[1] - ty[1] * nrm[0]};
            const double phi = 2 * M_PI * U(rng);
            double ct = set == 0 ? std::sqrt(U(rng)) : 0.035 * U(rng);  // cosine-weighted / within ~2 degrees
            const double st = std::sqrt(std::max(0.0, 1 - ct * ct));
            double dd[3];
            for (int j = 0; j < 3; j++) dd[j] = ct * nrm[j] + st * (std::cos(phi) * ty[j] + std::sin(phi) * tz[j]);
            const V3 o = rtk::v3((float)p[0], (float)p[1], (float)p[2]);
            const V3 d = rtk::normalize(rtk::v3((float)dd[0], (float)dd[1], (float)dd[2]));
            bool h0, h1, h2, h3;
            int md;
            tr[0].push_back((double)W.stack_walk(o, d, false, h0, md));
            maxdepth_all = std::max(maxdepth_all, md);
            tr[1].push_back((double)W.stack_walk(o, d, true, h1, md));
            tr[2].push_back((double)W.parent_walk(o, d, h2));
            tr[3].push_back((double)W.skip_walk(o, d, h3));
            hits += h0;
            mism += (h0 != h1) + (h0 != h2) + (h0 != h3);
        }
        const char* names[4] = {"stack", "paired", "parent", "skip"};
        std::fprintf(out, "%s\"%s\": {\"rays\": %zu, \"occluded\": %ld, \"answer_mismatches\": %ld, \"max_stack\": %d",
                     set ? ", " : "", set ? "grazing" : "cosine", tr[0].size(), hits, mism, maxdepth_all);
        for (int w = 0; w < 4; w++) {
            std::vector<double> v = tr[w];
            std::sort(v.begin(), v.end());
            double s = 0;
            for (double x : v) s += x;
            const double mean = s / std::max<size_t>(1, v.size());
            std::fprintf(out, ", \"%s\": {\"mean\": %.3f, \"p99\": %.0f, \"max\": %.0f}", names[w], mean,
                         v.empty() ? 0.0 : v[(size_t)(0.99 * (v.size() - 1))], v.empty() ? 0.0 : v.back());
            std::printf("%s %s mean %.2f p99 %.0f max %.0f\n", set ? "grazing" : "cosine", names[w], mean,
                        v.empty() ? 0.0 : v[(size_t)(0.99 * (v.size() - 1))], v.empty() ? 0.0 : v.back());
        }
        std::fprintf(out, "}");
    }
    std::fprintf(out, "}, \"closest\": {");
    // continuation walks from the hit leaf's ancestor: rays leaving a
    // surface triangle; top-down from the root vs started at the ancestor `up` levels above
    // the node holding the triangle, then the ancestors' other children
    for (int set = 0; set < 2; set++) {
        std::mt19937_64 rng(777 + set);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        const int ups[4] = {0, 1, 2, 4};
        std::vector<double> tr[5];
        long mism = 0, used = 0;
        for (int i = 0; i < n_rays / 4; i++) {
            const int k0 = (int)(U(rng) * nt) % nt;  // original index
            const int k = fb.prim2k[k0];
            if (k < 0 || node_of_k[k] < 0) continue;
            const float* t = &m.tris[9 * (size_t)k0];
            double a[3], e1[3], e2[3], nrm[3];
            for (int j = 0; j < 3; j++) a[j] = t[j], e1[j] = t[3 + j] - t[j], e2[j] = t[6 + j] - t[j];
            nrm[0] = e1[1] * e2[2] - e1[2] * e2[1], nrm[1] = e1[2] * e2[0] - e1[0] * e2[2], nrm[2] = e1[0] * e2[1] - e1[1] * e2[0];
            const double ln = std::sqrt(nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2]);
            if (!(ln > 0)) continue;
            for (double& x : nrm) x /= ln;
            double r1 = U(rng), r2 = U(rng);
            if (r1 + r2 > 1) r1 = 1 - r1, r2 = 1 - r2;
            double p[3];
            for (int j = 0; j < 3; j++) p[j] = a[j] + r1 * e1[j] + r2 * e2[j] + 1e-4 * nrm[j];
            double tx[3] = {1, 0, 0};
            if (std::fabs(nrm[0]) > 0.9) tx[0] = 0, tx[1] = 1;
            double ty[3] = {nrm[1] * tx[2] - nrm[2] * tx[1], nrm[2] * tx[0] - nrm[0] * tx[2], nrm[0] * tx[1] - nrm[1] * tx[0]};
            const double lt = std::sqrt(ty[0] * ty[0] + ty[1] * ty[1] + ty[2] * ty[2]);
            for (double& x : ty) x /= lt;
            double tz[3] = {ty[1] * nrm[2] - ty[2] * nrm[1], ty[2] * nrm[0] - ty[0] * nrm[2], ty[0] * nrm[1] - ty[1] * nrm[0]};
            const double phi = 2 * M_PI * U(rng);
            const double ct = set == 0 ? std::sqrt(U(rng)) : 0.035 * U(rng);
            const double sn = std::sqrt(std::max(0.0, 1 - ct * ct));
            double dd[3];
            for (int j = 0; j < 3; j++) dd[j] = ct * nrm[j] + sn * (std::cos(phi) * ty[j] + std::sin(phi) * tz[j]);
            const V3 o = rtk::v3((float)p[0], (float)p[1], (float)p[2]);
            const V3 d = rtk::normalize(rtk::v3((float)dd[0], (float)dd[1], (float)dd[2]));
            float t0;
            tr[0].push_back((double)W.closest_walk(o, d, 0, t0));
            for (int u = 0; u < 4; u++) {
                int st = node_of_k[k];
                for (int l = 0; l < ups[u] && st != 0; l++) st = W.parent[st];
                float t1;
                tr[1 + u].push_back((double)W.closest_walk(o, d, st, t1));
                mism += std::memcmp(&t1, &t0, 4) != 0;
            }
            used++;
        }
        const char* names[5] = {"root", "leaf_node", "up1", "up2", "up4"};
        std::fprintf(out, "%s\"%s\": {\"rays\": %ld, \"answer_mismatches\": %ld", set ? ", " : "",
                     set ? "grazing" : "cosine", used, mism);
        for (int w = 0; w < 5; w++) {
            std::vector<double> v = tr[w];
            std::sort(v.begin(), v.end());
            double sum = 0;
            for (double x : v) sum += x;
            const double mean = sum / std::max<size_t>(1, v.size());
            std::fprintf(out, ", \"%s\": {\"mean\": %.3f, \"p99\": %.0f, \"max\": %.0f}", names[w], mean,
                         v.empty() ? 0.0 : v[(size_t)(0.99 * (v.size() - 1))], v.empty() ? 0.0 : v.back());
            std::printf("closest %s %s mean %.2f p99 %.0f max %.0f\n", set ? "grazing" : "cosine", names[w], mean,
                        v.empty() ? 0.0 : v[(size_t)(0.99 * (v.size() - 1))], v.empty() ? 0.0 : v.back());
        }
        std::fprintf(out, "}");
    }
    std::fprintf(out, "}}\n");
    std::fclose(out);
    return 0;
}
