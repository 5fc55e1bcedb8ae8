// walk_probe.cpp — CPU study of search-BVH walk lengths.
//
// Replays logged rays (tools/walk_attrib.py samples: origin, direction, kind) through a
// one-query walk with the quad walk's visit rule (rt_quad.h quad_visit: nearest hit child
// next, the others on a stack, closest-hit walks keep visiting entries within
// t*(1 + RT_T2_WINDOW); occlusion walks stop at their first hit) and counts its trips (one
// per inner node or leaf visited: one memory round trip each on the GPU), over BVH builds:
//   product  the library's own search BVH (rt_scene.cpp build_search_bvh)
//   sah      binned SAH with this probe's builder (same policy as the product: 16 bins,
//            leaves <= 4, greedy largest-area 4-wide collapse)
//   sbvh     the same plus spatial splits (Stich et al. 2009): a triangle may be referenced
//            by several leaves, each with the box of its part inside the split planes
// Usage: walk_probe OBJ RAYS.bin OUT.json [variants: product sah sbvh sbvh:ALPHA ...]
// RAYS.bin: float32 [n][8] = origin xyz, direction xyz, kind, group.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_scene.h"
#include "rt_fast.h"

namespace {

struct Box {
    float mn[3], mx[3];
    void reset()
    {
        for (int i = 0; i < 3; i++) mn[i] = INFINITY, mx[i] = -INFINITY;
    }
    void grow(const float* p)
    {
        for (int i = 0; i < 3; i++) mn[i] = std::min(mn[i], p[i]), mx[i] = std::max(mx[i], p[i]);
    }
    void grow(const Box& b)
    {
        for (int i = 0; i < 3; i++) mn[i] = std::min(mn[i], b.mn[i]), mx[i] = std::max(mx[i], b.mx[i]);
    }
    bool valid() const { return mx[0] >= mn[0] && mx[1] >= mn[1] && mx[2] >= mn[2]; }
    float area() const
    {
        if (!valid()) return 0.0f;
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
    float c(int a) const { return 0.5f * (mn[a] + mx[a]); }
};
Box isect(const Box& a, const Box& b)
{
    Box r;
    for (int i = 0; i < 3; i++) r.mn[i] = std::max(a.mn[i], b.mn[i]), r.mx[i] = std::min(a.mx[i], b.mx[i]);
    return r;
}

void pad_box(const Box& b, float* mn, float* mx)  // rt_scene.cpp pad_box
{
    float mag = 1.0f;
    for (int i = 0; i < 3; i++) mag = std::max(mag, std::max(std::fabs(b.mn[i]), std::fabs(b.mx[i])));
    const float pad = 1e-4f * mag;
    for (int i = 0; i < 3; i++) mn[i] = b.mn[i] - pad, mx[i] = b.mx[i] + pad;
}

// the 4-wide tree the walk runs on: cnt > 0 leaf (refs[ref .. ref + cnt) are triangle ids), 0 inner, -1 empty
struct N4 {
    float lo[4][3], hi[4][3];
    int ref[4], cnt[4];
    float sn[4][3], s0[4], s1[4];  // optional oriented slab per child (sn = 0: none)
};
struct Tree {
    std::vector<N4> n;
    std::vector<int> refs;
    std::string name;
    double build_s = 0;
    bool slabs = false;
};

struct Tri {
    float a[3], b[3], c[3];
};

// ---------------------------------------------------------------- builder
struct Ref {
    Box b;
    int tri;
};
struct Node2 {
    Box bl, br;
    int l, r, lc, rc;  // child: lc > 0 leaf (first ref = l), 0 inner node l
};

// The part of triangle t inside box `clip`: Sutherland-Hodgman against its six planes.
Box clip_tri(const Tri& t, const Box& clip)
{
    float poly[16][3], tmp[16][3];
    int n = 3;
    std::memcpy(poly[0], t.a, 12), std::memcpy(poly[1], t.b, 12), std::memcpy(poly[2], t.c, 12);
    for (int ax = 0; ax < 3 && n; ax++)
        for (int side = 0; side < 2 && n; side++) {
            const float v = side ? clip.mx[ax] : clip.mn[ax];
            int m = 0;
            for (int i = 0; i < n; i++) {
                const float* p = poly[i];
                const float* q = poly[(i + 1) % n];
                const bool pin = side ? p[ax] <= v : p[ax] >= v;
                const bool qin = side ? q[ax] <= v : q[ax] >= v;
                if (pin) std::memcpy(tmp[m++], p, 12);
                if (pin != qin) {
                    const float s = (v - p[ax]) / (q[ax] - p[ax]);
                    for (int k = 0; k < 3; k++) tmp[m][k] = p[k] + s * (q[k] - p[k]);
                    tmp[m][ax] = v;
                    m++;
                }
            }
            n = std::min(m, 15);
            std::memcpy(poly, tmp, sizeof(float) * 3 * n);
        }
    Box r;
    r.reset();
    for (int i = 0; i < n; i++) r.grow(poly[i]);
    return isect(r, clip);
}

struct Builder {
    const std::vector<Tri>& T;
    int bins = 16, leaf_max = 4;
    bool spatial = false;
    float alpha = 1e-5f;
    float root_area = 1;
    std::vector<Node2> nodes;
    std::vector<int> leaf_refs;
    long splits = 0;
    explicit Builder(const std::vector<Tri>& t) : T(t) {}

    struct Split {
        float cost = INFINITY;
        int axis = -1;
        float pos = 0;  // object: bin index; spatial: plane
        bool spatial = false;
        Box bl, br;
    };

    Split object_split(const std::vector<Ref>& R, const Box& cb) const
    {
        Split best;
        for (int ax = 0; ax < 3; ax++) {
            const float lo = cb.mn[ax], ext = cb.mx[ax] - cb.mn[ax];
            if (!(ext > 0)) continue;
            const float sc = bins / ext;
            std::vector<Box> bb(bins);
            std::vector<int> cnt(bins, 0);
            for (auto& x : bb) x.reset();
            for (const Ref& r : R) {
                const int bi = std::min(bins - 1, (int)((r.b.c(ax) - lo) * sc));
                cnt[bi]++;
                bb[bi].grow(r.b);
            }
            std::vector<Box> rb(bins);
            std::vector<int> rc(bins);
            Box acc;
            acc.reset();
            int ac = 0;
            for (int i = bins - 1; i > 0; i--) acc.grow(bb[i]), ac += cnt[i], rb[i] = acc, rc[i] = ac;
            acc.reset();
            ac = 0;
            for (int i = 0; i < bins - 1; i++) {
                acc.grow(bb[i]);
                ac += cnt[i];
                if (ac == 0 || rc[i + 1] == 0) continue;
                const float cost = acc.area() * ac + rb[i + 1].area() * rc[i + 1];
                if (cost < best.cost) best.cost = cost, best.axis = ax, best.pos = (float)i, best.bl = acc, best.br = rb[i + 1];
            }
        }
        return best;
    }

    Split spatial_split(const std::vector<Ref>& R, const Box& nb) const
    {
        Split best;
        for (int ax = 0; ax < 3; ax++) {
            const float lo = nb.mn[ax], ext = nb.mx[ax] - nb.mn[ax];
            if (!(ext > 0)) continue;
            const float w = ext / bins;
            std::vector<Box> bb(bins);
            std::vector<int> enter(bins, 0), leave(bins, 0);
            for (auto& x : bb) x.reset();
            for (const Ref& r : R) {
                const int b0 = std::max(0, std::min(bins - 1, (int)((r.b.mn[ax] - lo) / w)));
                const int b1 = std::max(b0, std::min(bins - 1, (int)((r.b.mx[ax] - lo) / w)));
                enter[b0]++;
                leave[b1]++;
                for (int b = b0; b <= b1; b++) {
                    Box slab = r.b;
                    slab.mn[ax] = std::max(r.b.mn[ax], lo + w * b);
                    slab.mx[ax] = std::min(r.b.mx[ax], b == bins - 1 ? nb.mx[ax] : lo + w * (b + 1));
                    const Box c = b0 == b1 ? r.b : clip_tri(T[r.tri], slab);
                    if (c.valid()) bb[b].grow(c);
                }
            }
            std::vector<Box> rb(bins);
            std::vector<int> rc(bins);
            Box acc;
            acc.reset();
            int ac = 0;
            for (int i = bins - 1; i > 0; i--) acc.grow(bb[i]), ac += leave[i], rb[i] = acc, rc[i] = ac;
            acc.reset();
            ac = 0;
            for (int i = 0; i < bins - 1; i++) {
                acc.grow(bb[i]);
                ac += enter[i];
                if (ac == 0 || rc[i + 1] == 0) continue;
                const float cost = acc.area() * ac + rb[i + 1].area() * rc[i + 1];
                if (cost < best.cost)
                    best.cost = cost, best.axis = ax, best.pos = lo + w * (i + 1), best.spatial = true, best.bl = acc,
                    best.br = rb[i + 1];
            }
        }
        return best;
    }

    // returns child (ref, cnt) for the slot
    void build(std::vector<Ref> root)
    {
        Box rb;
        rb.reset();
        for (auto& r : root) rb.grow(r.b);
        root_area = rb.area();
        nodes.clear();
        leaf_refs.clear();
        nodes.push_back(Node2{});
        struct Task {
            std::vector<Ref> R;
            int node, side, depth;
        };
        std::vector<Task> st;
        // the root node's two children come from the first split
        std::vector<Ref> L, Rr;
        Box lb, rbx;
        if (!split_refs(root, 0, L, Rr)) {
            L = root;
            Rr.clear();
        }
        st.push_back({std::move(Rr), 0, 1, 1});
        st.push_back({std::move(L), 0, 0, 1});
        while (!st.empty()) {
            Task t = std::move(st.back());
            st.pop_back();
            Node2& p = nodes[t.node];
            Box& box = t.side ? p.br : p.bl;
            int& ref = t.side ? p.r : p.l;
            int& cnt = t.side ? p.rc : p.lc;
            if (t.R.empty()) {
                box.reset();
                ref = 0;
                cnt = -1;
                continue;
            }
            box.reset();
            for (auto& r : t.R) box.grow(r.b);
            std::vector<Ref> A, B;
            if ((int)t.R.size() <= leaf_max || !split_refs(t.R, t.depth, A, B)) {
                ref = (int)leaf_refs.size();
                cnt = (int)t.R.size();
                for (auto& r : t.R) leaf_refs.push_back(r.tri);
                continue;
            }
            const int ni = (int)nodes.size();
            ref = ni;
            cnt = 0;
            nodes.push_back(Node2{});
            st.push_back({std::move(B), ni, 1, t.depth + 1});
            st.push_back({std::move(A), ni, 0, t.depth + 1});
        }
    }

    bool split_refs(const std::vector<Ref>& R, int depth, std::vector<Ref>& A, std::vector<Ref>& B)
    {
        const int n = (int)R.size();
        if (n <= 1) return false;
        Box nb, cb;
        nb.reset();
        cb.reset();
        for (auto& r : R) {
            nb.grow(r.b);
            const float c[3] = {r.b.c(0), r.b.c(1), r.b.c(2)};
            cb.grow(c);
        }
        Split s = object_split(R, cb);
        if (spatial && depth < 48 && s.axis >= 0) {
            const float ov = isect(s.bl, s.br).area();
            if (ov / root_area > alpha) {
                Split sp = spatial_split(R, nb);
                if (sp.cost < s.cost) s = sp;
            }
        } else if (spatial && depth < 48 && s.axis < 0) {
            Split sp = spatial_split(R, nb);
            if (sp.axis >= 0) s = sp;
        }
        A.clear();
        B.clear();
        if (s.axis < 0) {  // coincident centroids: by count
            A.assign(R.begin(), R.begin() + n / 2);
            B.assign(R.begin() + n / 2, R.end());
            return true;
        }
        if (!s.spatial) {
            const float lo = cb.mn[s.axis], sc = bins / (cb.mx[s.axis] - cb.mn[s.axis]);
            for (auto& r : R) (std::min(bins - 1, (int)((r.b.c(s.axis) - lo) * sc)) <= (int)s.pos ? A : B).push_back(r);
        } else {
            splits++;
            for (auto& r : R) {
                if (r.b.mx[s.axis] <= s.pos) {
                    A.push_back(r);
                } else if (r.b.mn[s.axis] >= s.pos) {
                    B.push_back(r);
                } else {
                    Box l = r.b, h = r.b;
                    l.mx[s.axis] = s.pos;
                    h.mn[s.axis] = s.pos;
                    const Box cl = clip_tri(T[r.tri], l), ch = clip_tri(T[r.tri], h);
                    if (cl.valid()) A.push_back(Ref{cl, r.tri});
                    if (ch.valid()) B.push_back(Ref{ch, r.tri});
                }
            }
        }
        if (A.empty() || B.empty()) {
            A.clear();
            B.clear();
            A.assign(R.begin(), R.begin() + n / 2);
            B.assign(R.begin() + n / 2, R.end());
        }
        return true;
    }

    // greedy largest-area collapse to 4-wide (rt_scene.cpp collapse_bvh4), padded boxes
    Tree collapse() const
    {
        Tree t;
        t.refs = leaf_refs;
        struct Slot {
            Box b;
            int ref, cnt;
        };
        auto slots_of = [&](int n, Slot* out) {
            out[0] = {nodes[n].bl, nodes[n].l, nodes[n].lc};
            out[1] = {nodes[n].br, nodes[n].r, nodes[n].rc};
        };
        struct Task {
            int n2, n4;
        };
        std::vector<Task> st{{0, 0}};
        t.n.emplace_back();
        while (!st.empty()) {
            const Task k = st.back();
            st.pop_back();
            Slot c[4];
            int m = 2;
            slots_of(k.n2, c);
            while (m < 4) {
                int best = -1;
                for (int i = 0; i < m; i++)
                    if (c[i].cnt == 0 && (best < 0 || c[i].b.area() > c[best].b.area())) best = i;
                if (best < 0) break;
                Slot two[2];
                slots_of(c[best].ref, two);
                c[best] = two[0];
                c[m++] = two[1];
            }
            N4 nd{};
            Task kids[4];
            int nk = 0;
            for (int i = 0; i < 4; i++) {
                if (i >= m || c[i].cnt < 0) {
                    nd.cnt[i] = -1;
                    nd.ref[i] = 0;
                    for (int a = 0; a < 3; a++) nd.lo[i][a] = INFINITY, nd.hi[i][a] = -INFINITY;
                    continue;
                }
                pad_box(c[i].b, nd.lo[i], nd.hi[i]);
                nd.cnt[i] = c[i].cnt;
                nd.ref[i] = c[i].ref;
                if (c[i].cnt == 0) {
                    kids[nk++] = {c[i].ref, (int)t.n.size()};
                    nd.ref[i] = (int)t.n.size();
                    t.n.emplace_back();
                }
            }
            t.n[k.n4] = nd;
            for (int i = nk - 1; i >= 0; i--) st.push_back(kids[i]);
        }
        return t;
    }
};

Tree product_tree(const rt::FlatBvh& f)
{
    Tree t;
    t.name = "product";
    t.refs.resize(f.bvh_tri4.size() / 3);
    for (size_t i = 0; i < t.refs.size(); i++) t.refs[i] = (int)rt_asuint(f.bvh_tri4[3 * i + 2].w);
    t.n.resize(f.bvh4.size());
    for (size_t i = 0; i < f.bvh4.size(); i++)
        for (int c = 0; c < 4; c++) {
            const Bvh4Child& ch = f.bvh4[i].ch[c];
            for (int a = 0; a < 3; a++) t.n[i].lo[c][a] = ch.lo[a], t.n[i].hi[c][a] = ch.hi[a];
            t.n[i].ref[c] = ch.ref;
            t.n[i].cnt[c] = ch.cnt;
        }
    return t;
}

// Oriented slab per child: the subtree's area-weighted mean triangle normal n and the range
// of n.v over its vertices (padded like the boxes); none when the normals cancel out.
void collect(const Tree& tr, int node, std::vector<int>& out)
{
    const N4& n = tr.n[node];
    for (int c = 0; c < 4; c++) {
        if (n.cnt[c] < 0) continue;
        if (n.cnt[c] > 0)
            for (int j = 0; j < n.cnt[c]; j++) out.push_back(tr.refs[n.ref[c] + j]);
        else
            collect(tr, n.ref[c], out);
    }
}
float g_margin = 0;  // absolute slab margin (0: 2e-4 of the child's magnitude)
void add_slabs(Tree& tr, const std::vector<Tri>& T, float min_align)
{
    tr.slabs = true;
    std::vector<int> tris;
    for (size_t i = 0; i < tr.n.size(); i++) {
        N4& n = tr.n[i];
        for (int c = 0; c < 4; c++) {
            n.sn[c][0] = n.sn[c][1] = n.sn[c][2] = 0;
            if (n.cnt[c] < 0) continue;
            tris.clear();
            if (n.cnt[c] > 0)
                for (int j = 0; j < n.cnt[c]; j++) tris.push_back(tr.refs[n.ref[c] + j]);
            else
                collect(tr, n.ref[c], tris);
            double m[3] = {0, 0, 0}, asum = 0;
            for (int k : tris) {
                const Tri& x = T[k];
                const double e1[3] = {x.b[0] - x.a[0], x.b[1] - x.a[1], x.b[2] - x.a[2]};
                const double e2[3] = {x.c[0] - x.a[0], x.c[1] - x.a[1], x.c[2] - x.a[2]};
                const double cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                for (int a = 0; a < 3; a++) m[a] += cr[a];
                asum += std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
            }
            const double len = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
            if (!(len > min_align * asum) || len == 0) continue;
            float nn[3] = {(float)(m[0] / len), (float)(m[1] / len), (float)(m[2] / len)};
            float lo = INFINITY, hi = -INFINITY, mag = 1.0f;
            for (int k : tris) {
                const Tri& x = T[k];
                for (const float* v : {x.a, x.b, x.c}) {
                    const float dd = nn[0] * v[0] + nn[1] * v[1] + nn[2] * v[2];
                    lo = std::min(lo, dd), hi = std::max(hi, dd);
                    for (int a = 0; a < 3; a++) mag = std::max(mag, std::fabs(v[a]));
                }
            }
            std::memcpy(n.sn[c], nn, 12);
            const float mg = g_margin > 0 ? g_margin : 2e-4f * mag;
            n.s0[c] = lo - mg;
            n.s1[c] = hi + mg;
        }
    }
}

bool g_box_key = false;  // the slab rejects only; the stack key stays the box entry
// box (and slab) entry / exit
bool child_hit(const N4& n, int c, const float* o, const float* d, const float* inv, float tmax, bool slabs, float& tn)
{
    float t0 = 0.0f, t1 = tmax;
    for (int a = 0; a < 3; a++) {
        float x0 = (n.lo[c][a] - o[a]) * inv[a], x1 = (n.hi[c][a] - o[a]) * inv[a];
        if (x0 > x1) std::swap(x0, x1);
        if (!(x0 <= t1 && x1 >= t0)) return false;  // (NaN: a miss)
        t0 = std::max(t0, x0);
        t1 = std::min(t1, x1);
    }
    const float tbox = t0;
    if (slabs && (n.sn[c][0] != 0 || n.sn[c][1] != 0 || n.sn[c][2] != 0)) {
        const float no = n.sn[c][0] * o[0] + n.sn[c][1] * o[1] + n.sn[c][2] * o[2];
        const float nd = n.sn[c][0] * d[0] + n.sn[c][1] * d[1] + n.sn[c][2] * d[2];
        if (nd == 0) {
            if (no < n.s0[c] || no > n.s1[c]) return false;
        } else {
            float x0 = (n.s0[c] - no) / nd, x1 = (n.s1[c] - no) / nd;
            if (x0 > x1) std::swap(x0, x1);
            t0 = std::max(t0, x0);
            t1 = std::min(t1, x1);
            if (t0 > t1) return false;
        }
    }
    tn = g_box_key ? tbox : t0;
    return true;
}

// ---------------------------------------------------------------- walk
struct WalkOut {
    int trips, inner, leaves, tris, empty_inner, empty_leaves;
    float t;
};
WalkOut walk(const Tree& tr, const std::vector<Tri>& T, const float* o3, const float* d3, bool any)
{
    using namespace rtk;
    const V3 o = v3(o3[0], o3[1], o3[2]), d = v3(d3[0], d3[1], d3[2]);
    const RayB rb = rayb_setup(o, d);
    (void)rb;
    const float inv[3] = {1.0f / d3[0], 1.0f / d3[1], 1.0f / d3[2]};
    WalkOut w{0, 0, 0, 0, 0, 0, INFINITY};
    struct E {
        int item;
        float key;
    };
    E stk[512];
    int sp = 0;
    int cur = 0;  // >= 0 node, < 0: ~(leaf ref << 3 | cnt)
    float t = INFINITY;
    for (;;) {
        w.trips++;
        const float tmax = any ? INFINITY : t + t * RT_T2_WINDOW;
        bool pop = true;
        if (cur >= 0) {
            w.inner++;
            const N4& n = tr.n[cur];
            E h[4];
            int nh = 0;
            for (int c = 0; c < 4; c++) {
                if (n.cnt[c] < 0) continue;
                float tn;
                if (child_hit(n, c, o3, d3, inv, tmax, tr.slabs, tn) && tn <= tmax)
                    h[nh++] = {n.cnt[c] > 0 ? ~((n.ref[c] << 3) | n.cnt[c]) : n.ref[c], any ? 0.0f : tn};
            }
            if (!nh) w.empty_inner++;
            if (nh) {
                std::stable_sort(h, h + nh, [](const E& a, const E& b) { return a.key < b.key; });
                for (int j = nh - 1; j >= 1; j--)
                    if (sp < 512) stk[sp++] = h[j];
                cur = h[0].item;
                pop = false;
            }
        } else {
            w.leaves++;
            const int v = ~cur, first = v >> 3, cnt = v & 7;
            const float tb = t;
            bool any_hit = false;
            for (int j = 0; j < cnt; j++) {
                const Tri& x = T[tr.refs[first + j]];
                const V3 a = v3(x.a[0], x.a[1], x.a[2]);
                const V3 e1 = v3(x.b[0] - x.a[0], x.b[1] - x.a[1], x.b[2] - x.a[2]);
                const V3 e2 = v3(x.c[0] - x.a[0], x.c[1] - x.a[1], x.c[2] - x.a[2]);
                float th;
                w.tris++;
                if (tri_test_v(a, e1, e2, o, d, th)) {
                    any_hit = true;
                    if (th < t) t = th;
                }
            }
            (void)tb;
            if (!any_hit) w.empty_leaves++;
            if (any && t < INFINITY) break;
        }
        if (pop) {
            const float tm = any ? INFINITY : t + t * RT_T2_WINDOW;
            cur = INT32_MIN;
            while (sp > 0) {
                --sp;
                if (stk[sp].key <= tm) {
                    cur = stk[sp].item;
                    break;
                }
            }
            if (cur == INT32_MIN) break;
        }
    }
    w.t = t;
    return w;
}

double qtile(std::vector<int> v, double q)
{
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: walk_probe OBJ RAYS.bin OUT.json [product sah sbvh sbvh:ALPHA sah:BINS ...]\n");
        return 2;
    }
    rt::Mesh m;
    std::string err;
    if (rt::load_obj(argv[1], m, err)) {
        std::fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const int nt = m.ntris();
    std::vector<Tri> T(nt);
    for (int i = 0; i < nt; i++) std::memcpy(&T[i], &m.tris[9 * (size_t)i], 36);
    std::vector<float> rays;
    {
        FILE* f = std::fopen(argv[2], "rb");
        if (!f) return 1;
        std::fseek(f, 0, SEEK_END);
        const long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        rays.resize(sz / 4);
        if (std::fread(rays.data(), 4, rays.size(), f) != rays.size()) return 1;
        std::fclose(f);
    }
    const size_t nr = rays.size() / 8;
    std::vector<std::string> variants;
    for (int i = 4; i < argc; i++) variants.push_back(argv[i]);
    if (variants.empty()) variants = {"product", "sah", "sbvh"};
    FILE* out = std::fopen(argv[3], "w");
    std::fprintf(out, "{\"rays\": %zu, \"variants\": [\n", nr);
    bool first = true;
    for (const std::string& v : variants) {
        Tree tr;
        auto t0 = std::chrono::steady_clock::now();
        long nrefs = nt, splits = 0;
        g_box_key = v.find("boxkey") != std::string::npos;
        g_margin = v.find("m1e-3") != std::string::npos ? 1e-3f : v.find("m3e-3") != std::string::npos ? 3e-3f : 0.0f;
        if (v == "product" || v.rfind("product+slab", 0) == 0) {
            rt::Octree oc;
            rt::build_octree(m.tris.data(), nt, 32, 8, oc);
            rt::FlatBvh fb;
            rt::flatten_octree(oc, m.tris.data(), nt, fb);
            t0 = std::chrono::steady_clock::now();
            rt::build_search_bvh(fb);
            tr = product_tree(fb);
            if (v != "product") add_slabs(tr, T, v.size() > 12 && v[12] == ':' ? std::stof(v.substr(13)) : 0.5f);
        } else {
            // "sah" / "sbvh[:alpha]" / "sah:16", or key=value tokens after a comma:
            // bins=N, leaf=N, alpha=X, slab (add slabs, align 0.5), slab=ALIGN
            Builder B(T);
            std::string head = v.substr(0, v.find(','));
            const size_t c = head.find(':');
            const std::string kind = head.substr(0, c);
            if (kind == "sbvh") {
                B.spatial = true;
                if (c != std::string::npos) B.alpha = std::stof(head.substr(c + 1));
            } else if (c != std::string::npos) {
                B.bins = std::stoi(head.substr(c + 1));
            }
            float slab_align = -1.0f;
            for (size_t p = v.find(','); p != std::string::npos; p = v.find(',', p + 1)) {
                const std::string tok = v.substr(p + 1, v.find(',', p + 1) - p - 1);
                const size_t eq = tok.find('=');
                const std::string key = tok.substr(0, eq), val = eq == std::string::npos ? "" : tok.substr(eq + 1);
                if (key == "bins") B.bins = std::stoi(val);
                else if (key == "leaf") B.leaf_max = std::stoi(val);
                else if (key == "alpha") B.alpha = std::stof(val);
                else if (key == "slab") slab_align = val.empty() ? 0.5f : std::stof(val);
            }
            std::vector<Ref> R(nt);
            for (int i = 0; i < nt; i++) {
                R[i].tri = i;
                R[i].b.reset();
                R[i].b.grow(T[i].a), R[i].b.grow(T[i].b), R[i].b.grow(T[i].c);
            }
            B.build(std::move(R));
            tr = B.collapse();
            nrefs = (long)B.leaf_refs.size();
            splits = B.splits;
            if (slab_align >= 0) add_slabs(tr, T, slab_align);
        }
        tr.build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::vector<int> trips[2], all;
        double sum = 0, sum_inner = 0, sum_leaves = 0, sum_tris = 0, sum_ei = 0, sum_el = 0;
        long miss_mismatch = 0;
        for (size_t i = 0; i < nr; i++) {
            const float* r = &rays[8 * i];
            const bool any = r[6] >= 4.0f;
            const WalkOut w = walk(tr, T, r, r + 3, any);
            const int g = r[7] > 0.5f ? 1 : 0;
            trips[g].push_back(w.trips);
            all.push_back(w.trips);
            sum += w.trips;
            sum_inner += w.inner;
            sum_leaves += w.leaves;
            sum_tris += w.tris;
            sum_ei += w.empty_inner;
            sum_el += w.empty_leaves;
            (void)miss_mismatch;
        }
        std::fprintf(stderr, "%-12s inner %.2f (no child entered %.2f) leaves %.2f (no hit %.2f) tris %.2f\n", v.c_str(),
                     sum_inner / std::max<size_t>(1, nr), sum_ei / std::max<size_t>(1, nr), sum_leaves / std::max<size_t>(1, nr),
                     sum_el / std::max<size_t>(1, nr), sum_tris / std::max<size_t>(1, nr));
        std::fprintf(stderr, "%-12s nodes %zu refs %ld splits %ld build %.2fs  mean %.2f  p50 %.0f p90 %.0f p99 %.0f p99.9 %.0f max %.0f\n",
                     v.c_str(), tr.n.size(), nrefs, splits, tr.build_s, sum / std::max<size_t>(1, nr), qtile(all, 0.5),
                     qtile(all, 0.9), qtile(all, 0.99), qtile(all, 0.999), qtile(all, 1.0));
        std::fprintf(out, "%s{\"variant\": \"%s\", \"nodes\": %zu, \"refs\": %ld, \"spatial_splits\": %ld, \"build_s\": %.3f",
                     first ? "" : ",\n", v.c_str(), tr.n.size(), nrefs, splits, tr.build_s);
        for (int g = 0; g < 2; g++) {
            double s = 0;
            for (int x : trips[g]) s += x;
            std::fprintf(out, ", \"group%d\": {\"n\": %zu, \"mean\": %.3f, \"p50\": %.0f, \"p90\": %.0f, \"p99\": %.0f, \"p999\": %.0f, \"max\": %.0f}",
                         g, trips[g].size(), trips[g].empty() ? 0.0 : s / trips[g].size(), qtile(trips[g], 0.5),
                         qtile(trips[g], 0.9), qtile(trips[g], 0.99), qtile(trips[g], 0.999), qtile(trips[g], 1.0));
        }
        std::fprintf(out, "}");
        first = false;
        std::fflush(out);
    }
    std::fprintf(out, "\n]}\n");
    std::fclose(out);
    return 0;
}
