// cpu_oracle.cpp — CPU RESTATEMENT of the reference render path.
//
// TEST INFRASTRUCTURE ONLY. This is the parity checker for the HIP product
// (tests/, __graft_entry__.smoke()) and the "port" CPU baseline in bench.py.
// Nothing in sycl-ray-tracing_amd/ links or calls it.
//
// It restates, function by function, /root/reference at 2024-08-07 with the
// same float/double evaluation order and the system glibc libm, and is
// pinned bit-exactly to the compiled reference (oracle/_ref/ref_driverO2)
// through the fixtures in tests/golden/ (tests/test_oracle_pinned.py).
//
// Build: g++ -O2 -fopenmp -ffp-contract=off -shared (oracle/Makefile).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <queue>
#include <vector>

#include <omp.h>

namespace {

// ------------------------------------------------------- include/vec.h
struct V3 {
    float x, y, z;
};
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }  // vec.h:75,131
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }  // vec.h:96,106,126
inline V3 operator-(V3 v) { return v3(-v.x, -v.y, -v.z); }                        // vec.h:101
inline V3 operator*(float k, V3 v) { return v3(k * v.x, k * v.y, k * v.z); }      // vec.h:80,136
inline V3 operator*(V3 v, float k) { return k * v; }                               // vec.h:85,141
inline float dot(V3 u, V3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }        // vec.h:186-189
inline float length(V3 v) { return std::sqrt(dot(v, v)); }                         // vec.h:157-165
inline V3 normalize(V3 v)                                                          // vec.h:172-176
{
    float kk = 1.0f / length(v);
    return kk * v;
}
inline V3 cross(V3 u, V3 v)  // vec.h:178-184
{
    return v3((u.y * v.z) - (u.z * v.y), (u.z * v.x) - (u.x * v.z), (u.x * v.y) - (u.y * v.x));
}
inline V3 vmin(V3 a, V3 b) { return v3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)); }  // vec.cpp:506-509
inline V3 vmax(V3 a, V3 b) { return v3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)); }  // vec.cpp:511-514

// ------------------------------------------------------ include/color.h
struct Col {
    float r, g, b;
};
inline Col col(float v) { return Col{v, v, v}; }
inline Col operator+(Col a, Col b) { return Col{a.r + b.r, a.g + b.g, a.b + b.b}; }  // color.h:419
inline Col operator-(Col a, Col b) { return Col{a.r + (-b.r), a.g + (-b.g), a.b + (-b.b)}; }  // color.h:429
inline Col operator*(Col a, Col b) { return Col{a.r * b.r, a.g * b.g, a.b * b.b}; }  // color.h:434
inline Col operator*(float k, Col c) { return Col{c.r * k, c.g * k, c.b * k}; }    // color.h:439
inline Col operator*(Col c, float k) { return k * c; }                               // color.h:444
inline Col operator/(Col c, float k)                                                 // color.h:459-463
{
    float kk = 1 / k;
    return kk * c;
}
inline bool is_black(Col c) { return c.r == 0.0f && c.g == 0.0f && c.b == 0.0f; }  // color.h:313-316
inline float luminance(Col c) { return 0.3086f * c.r + 0.6094f * c.g + 0.0820f * c.b; }  // color.h:368-371

// ------------------------------------------------- include/xorshift.h
struct Rng {  // xorshift.h:10-31
    uint32_t a;
    uint32_t draws = 0;  // (analysis only: draws so far, oracle_render_log)
    float operator()()
    {
        draws++;
        uint32_t x = a;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        a = x;
        return std::min(x / (float)std::numeric_limits<unsigned int>::max(), 1.0f - 1.0e-6f);
    }
};

// ---------------------------------------- include/ray.h, hit_info.h
struct Ray {
    V3 o, d;
};
struct Hit {  // hit_info.h:6-15
    V3 p{0, 0, 0}, n{0, 0, 0};
    float t = -1.0f, u = -1.0f, v = -1.0f;
    int prim = -1;
};

struct Tri {
    V3 a, b, c;
};
struct Mat {
    Col emission, diffuse;
    float metalness, roughness;
};
struct Sph {
    V3 c;
    float r;
    int prim;
};

// -------------------------------------------------- include/triangle.h
bool tri_intersect(const Tri& tr, const Ray& ray, Hit& h)  // triangle.h:16-60
{
    const float EPSILON = 0.0000001f;
    V3 edge1 = tr.b - tr.a, edge2 = tr.c - tr.a;
    V3 hh = cross(ray.d, edge2);
    float a = dot(edge1, hh);
    if (a > -EPSILON && a < EPSILON) return false;
    float f = 1.0f / a;
    V3 s = ray.o - tr.a;
    float u = f * dot(s, hh);
    if (u < 0.0f || u > 1.0f) return false;
    V3 q = cross(s, edge1);
    float v = f * dot(ray.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot(edge2, q);
    if (t > EPSILON) {
        h.p = ray.o + ray.d * t;
        h.n = normalize(cross(edge1, edge2));
        h.t = t;
        h.u = u;
        h.v = v;
        return true;
    }
    return false;
}
float tri_area(const Tri& t) { return length(cross(t.b - t.a, t.c - t.a)) / 2; }  // triangle.cpp:8-11
V3 tri_centroid(const Tri& t)                                                     // triangle.cpp:3-6
{
    V3 s = vmin(t.a, vmin(t.b, t.c)) + vmax(t.a, vmax(t.b, t.c));
    float kk = 1.f / 2;  // Point operator/ (vec.h:90-94)
    return kk * s;
}

// ---------------------------------------------------- include/sphere.h
bool sph_intersect(const Sph& sp, const Ray& ray, Hit& h)  // sphere.h:11-52
{
    V3 L = ray.o - sp.c;
    const float a = 1.0f;
    float b = 2.0f * dot(ray.d, L);
    float c = dot(L, L) - sp.r * sp.r;
    float delta = b * b - 4.0f * a * c;
    if (delta < 0.0f) return false;
    const float a2 = 2.0f * a;
    if (delta == 0.0f)
        h.t = -b / a2;
    else {
        float sq = std::sqrt(delta);
        float t1 = (-b - sq) / a2, t2 = (-b + sq) / a2;
        if (t1 < t2) {
            h.t = t1;
            if (h.t < 0.0f) h.t = t2;
        }
    }
    if (h.t < 0.0f) return false;
    h.p = ray.o + ray.d * h.t;
    h.n = normalize(h.p - sp.c);
    h.prim = sp.prim;
    return true;
}

// -------------------------------- include/bounding_volume.h, bvh.cpp
const float S3 = std::sqrt(3.0f) / 3;
const V3 PLANE_N[7] = {v3(1, 0, 0),   v3(0, 1, 0),    v3(0, 0, 1),   v3(S3, S3, S3),
                       v3(-S3, S3, S3), v3(-S3, -S3, S3), v3(S3, -S3, S3)};  // bvh.cpp:8-16

struct Vol {
    float dn[7], df[7];
    Vol()
    {
        for (int i = 0; i < 7; i++) dn[i] = INFINITY, df[i] = -INFINITY;
    }
    void extend(const float* n, const float* f)  // bounding_volume.h:39-46
    {
        for (int i = 0; i < 7; i++) dn[i] = std::min(dn[i], n[i]), df[i] = std::max(df[i], f[i]);
    }
    void extend(const Tri& t)  // bounding_volume.h:53-66, 25-37
    {
        float n[7], f[7];
        for (int i = 0; i < 7; i++) n[i] = INFINITY, f[i] = -INFINITY;
        const V3* p = &t.a;
        for (int i = 0; i < 7; i++)
            for (int j = 0; j < 3; j++) {
                float d = dot(PLANE_N[i], p[j]);
                n[i] = std::min(n[i], d);
                f[i] = std::max(f[i], d);
            }
        extend(n, f);
    }
    bool intersect(float& tn, float& tf, const float* den, const float* num) const  // :101-126
    {
        tn = -INFINITY;
        tf = INFINITY;
        for (int i = 0; i < 7; i++) {
            float d = den[i];
            if (d == 0.0f) continue;
            float a = (dn[i] - num[i]) / d, b = (df[i] - num[i]) / d;
            if (d < 0.0f) std::swap(a, b);
            tn = std::max(tn, a);
            tf = std::min(tf, b);
            if (tf < tn) return false;
        }
        return true;
    }
};

struct Counters {
    uint64_t rays = 0, vol_tests = 0, vol_tests_empty = 0, tri_tests = 0, leaf_visits = 0;
};

struct Node {  // bvh.h:19-209
    bool leaf = true;
    std::vector<int> tris;
    Node* ch[8] = {};
    V3 mn, mx;
    Vol vol;
    Node(V3 a, V3 b) : mn(a), mx(b) {}
    ~Node()
    {
        if (!leaf)
            for (auto* c : ch) delete c;
    }
    void create_children()  // bvh.h:67-81 (child _min offsets reproduced as written)
    {
        float mx_ = (mn.x + mx.x) / 2, my = (mn.y + mx.y) / 2, mz = (mn.z + mx.z) / 2;
        ch[0] = new Node(mn, v3(mx_, my, mz));
        ch[1] = new Node(v3(mx_, mn.y, mn.z), v3(mx.x, my, mz));
        ch[2] = new Node(mn + v3(0, my, 0), v3(mx_, mx.y, mz));
        ch[3] = new Node(v3(mx_, my, mn.z), v3(mx.x, mx.y, mz));
        ch[4] = new Node(mn + v3(0, 0, mz), v3(mx_, my, mx.z));
        ch[5] = new Node(v3(mx_, mn.y, mz), v3(mx.x, my, mx.z));
        ch[6] = new Node(mn + v3(0, my, mz), v3(mx_, mx.y, mx.z));
        ch[7] = new Node(v3(mx_, my, mz), mx);
    }
    void insert(const std::vector<Tri>& T, int id, int depth, int maxd, int leafmax)  // bvh.h:83-107
    {
        bool exceeded = maxd != -1 && depth == maxd;
        if (leaf || exceeded) {
            tris.push_back(id);
            if ((int)tris.size() > leafmax && !exceeded) {
                leaf = false;
                create_children();
                for (int t : tris) insert_to_children(T, t, depth, maxd, leafmax);
                tris.clear();
                tris.shrink_to_fit();
            }
        } else
            insert_to_children(T, id, depth, maxd, leafmax);
    }
    void insert_to_children(const std::vector<Tri>& T, int id, int depth, int maxd, int leafmax)  // :109-125
    {
        V3 c = tri_centroid(T[id]);
        float mx_ = (mn.x + mx.x) / 2, my = (mn.y + mx.y) / 2, mz = (mn.z + mx.z) / 2;
        int o = 0;
        if (c.x > mx_) o += 1;
        if (c.y > my) o += 2;
        if (c.z > mz) o += 4;
        ch[o]->insert(T, id, depth + 1, maxd, leafmax);
    }
    Vol compute_volume(const std::vector<Tri>& T)  // bvh.h:55-65
    {
        if (leaf)
            for (int t : tris) vol.extend(T[t]);
        else
            for (int i = 0; i < 8; i++) {
                Vol v = ch[i]->compute_volume(T);
                vol.extend(v.dn, v.df);
            }
        return vol;
    }
    struct QE {  // bvh.h:23-36
        const Node* node;
        float t;
        bool operator>(const QE& o) const { return t > o.t; }
    };
    bool intersect(const std::vector<Tri>& T, const Ray& ray, Hit& hit, float& t_near, const float* den,
                   const float* num, Counters* cnt) const  // bvh.h:142-209
    {
        float t_far, trash;
        if (!vol.intersect(trash, t_far, den, num)) return false;
        if (leaf) {
            if (cnt) cnt->leaf_visits++;
            for (int id : tris) {
                Hit lh;
                if (cnt) cnt->tri_tests++;
                if (tri_intersect(T[id], ray, lh))
                    if (lh.t < hit.t || hit.t == -1) {
                        hit = lh;
                        hit.prim = id;
                    }
            }
            t_near = hit.t;
            return t_near > 0;
        }
        std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
        for (int i = 0; i < 8; i++) {
            float d;
            if (cnt) {
                bool empty = ch[i]->leaf && ch[i]->tris.empty();
                (empty ? cnt->vol_tests_empty : cnt->vol_tests)++;
            }
            if (ch[i]->vol.intersect(d, t_far, den, num)) q.emplace(QE{ch[i], d});
        }
        bool found = false;
        float closest = 100000000, inter = 100000000;
        while (!q.empty()) {
            QE top = q.top();
            q.pop();
            if (top.node->intersect(T, ray, hit, inter, den, num, cnt)) {
                closest = std::min(closest, inter);
                found = true;
                if (q.empty() || closest < q.top().t) {
                    t_near = closest;
                    return true;
                }
            }
        }
        if (!found) return false;
        t_near = closest;
        return true;
    }
};

struct Scene {
    std::vector<Tri> tris;
    std::vector<int> mat_idx, emissive;
    std::vector<Mat> mats;
    std::vector<Sph> sph;
    Node* root = nullptr;
    int ew = 0, eh = 0;
    std::vector<Col> env;
    std::vector<float> env_lum, cdf;
    bool brute = false;  // INTERSECT_SCENE with USE_BVH 0 (render_kernel.h:13, render_kernel.cpp:504-511)
    ~Scene() { delete root; }
};

bool bvh_intersect(const Scene& S, const Ray& ray, Hit& hit, Counters* cnt)  // bvh.cpp:62-65, bvh.h:127-140
{
    float den[7], num[7], trash;
    for (int i = 0; i < 7; i++) {
        den[i] = dot(PLANE_N[i], ray.d);
        num[i] = dot(PLANE_N[i], ray.o);
    }
    if (cnt) cnt->rays++, cnt->vol_tests++;
    return S.root->intersect(S.tris, ray, hit, trash, den, num, cnt);
}

// RenderKernel::intersect_scene, the brute-force loop (render_kernel.cpp:453-483)
bool intersect_scene_brute(const Scene& S, const Ray& ray, Hit& closest)
{
    closest.t = -1.0f;
    for (int i = 0; i < (int)S.tris.size(); i++) {
        Hit h;
        if (tri_intersect(S.tris[i], ray, h))
            if (h.t < closest.t || closest.t == -1.0f) {
                closest = h;
                closest.prim = i;
            }
    }
    for (const Sph& sp : S.sph) {
        Hit lh;
        if (sph_intersect(sp, ray, lh))
            if (lh.t < closest.t || closest.t == -1.0f) closest = lh;
    }
    return closest.t > 0.0f;
}

bool intersect_scene(const Scene& S, const Ray& ray, Hit& h, Counters* cnt)  // render_kernel.cpp:485-502
{
    if (S.brute) return intersect_scene_brute(S, ray, h);
    bvh_intersect(S, ray, h, cnt);
    for (const Sph& sp : S.sph) {
        Hit lh;
        if (sph_intersect(sp, ray, lh))
            if (lh.t < h.t || h.t == -1.0f) h = lh;
    }
    return h.t > 0.0f;
}

// ---------------------------------------------- source/render_kernel.cpp
struct Cam {
    float m[4][4];
    float fov_dist;
};

struct Ctx {
    const Scene& S;
    Cam cam;
    int W, H, spp, bounces;
    Counters* cnt;
    uint64_t* env_lookups;
};

V3 xform_point(const Cam& c, V3 p)  // mat.cpp:94-111
{
    float xt = c.m[0][0] * p.x + c.m[0][1] * p.y + c.m[0][2] * p.z + c.m[0][3];
    float yt = c.m[1][0] * p.x + c.m[1][1] * p.y + c.m[1][2] * p.z + c.m[1][3];
    float zt = c.m[2][0] * p.x + c.m[2][1] * p.y + c.m[2][2] * p.z + c.m[2][3];
    float wt = c.m[3][0] * p.x + c.m[3][1] * p.y + c.m[3][2] * p.z + c.m[3][3];
    float w = 1.f / wt;
    if (wt == 1.f) return v3(xt, yt, zt);
    return v3(xt * w, yt * w, zt * w);
}

Ray camera_ray(const Ctx& C, float x, float y)  // render_kernel.cpp:56-73
{
    float xn = x / C.W * 2 - 1;
    xn *= (float)C.W / C.H;
    float yn = y / C.H * 2 - 1;
    V3 o = xform_point(C.cam, v3(0.0f, 0.0f, 0.0f));
    V3 p = xform_point(C.cam, v3(xn, yn, C.cam.fov_dist));
    return Ray{o, normalize(p - o)};
}

V3 rotate_around_normal(V3 n, V3 l)  // render_kernel.cpp:5-22
{
    float sign = std::copysign(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float b = n.x * n.y * a;
    V3 b1 = v3(1.0f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    V3 b2 = v3(b, sign + n.y * n.y * a, -n.y);
    return l.x * b1 + l.y * b2 + l.z * n;
}

Col fresnel_schlick(Col F0, float NoV) { return F0 + (col(1.0f) - F0) * std::pow((1.0f - NoV), 5.0f); }  // :218-221
float ggx_d(float alpha, float NoH)                                                                  // :223-233
{
    NoH = std::min(NoH, 0.999999f);
    float alpha2 = alpha * alpha;
    float NoH2 = NoH * NoH;
    float b = (NoH2 * (alpha2 - 1.0f) + 1.0f);
    return alpha2 * M_1_PI / (b * b);
}
float g1(float k, float d) { return d / (d * (1.0f - k) + k); }  // :235-238
float smith(float r2, float NoV, float NoL)                       // :240-245
{
    float k = r2 / 2.0f;
    return g1(k, NoL) * g1(k, NoV);
}

float ct_pdf(const Mat& m, V3 V, V3 L, V3 N)  // :247-258
{
    V3 H = normalize(V + L);
    float alpha = m.roughness * m.roughness;
    float VoH = std::max(0.0f, dot(V, H));
    float NoH = std::max(0.0f, dot(N, H));
    float D = ggx_d(alpha, NoH);
    return D * NoH / (4.0f * VoH);
}

Col ct_brdf(const Mat& m, V3 L, V3 V, V3 N)  // :260-301
{
    Col out = col(0.0f);
    Col base = m.diffuse;
    V3 H = normalize(V + L);
    float NoV = std::max(0.0f, dot(N, V));
    float NoL = std::max(0.0f, dot(N, L));
    float NoH = std::max(0.0f, dot(N, H));
    float VoH = std::max(0.0f, dot(H, V));
    if (NoV > 0.0f && NoL > 0.0f && NoH > 0.0f) {
        float metal = m.metalness, alpha = m.roughness * m.roughness;
        Col F0 = col(0.04f * (1.0f - metal)) + metal * base;
        Col F = fresnel_schlick(F0, VoH);
        float D = ggx_d(alpha, NoH);
        float G = smith(alpha, NoV, NoL);
        Col kD = col(1.0f - metal);
        kD = kD * (col(1.0f) - F);
        Col diffuse = kD * base / (float)M_PI;
        Col spec = (F * D * G) / (4.0f * NoV * NoL);
        out = diffuse + spec;
    }
    return out;
}

Col ct_sample(const Mat& m, V3 V, V3 N, V3& out_dir, float& pdf, Rng& rng)  // :392-451
{
    pdf = 0.0f;
    float metal = m.metalness, alpha = m.roughness * m.roughness;
    float r1 = rng(), r2 = rng();
    float phi = 2.0f * (float)M_PI * r1;
    float theta = std::acos((1.0f - r2) / (r2 * (alpha * alpha - 1.0f) + 1.0f));
    float sin_theta = std::sin(theta);
    V3 local = v3(std::cos(phi) * sin_theta, std::sin(phi) * sin_theta, std::cos(theta));
    V3 mn = rotate_around_normal(N, local);
    if (dot(mn, N) < 0.0f) return col(0.0f);
    V3 L = normalize(2.0f * dot(mn, V) * mn - V);
    V3 H = mn;
    out_dir = L;
    Col out = col(0.0f);
    Col base = m.diffuse;
    float NoV = std::max(0.0f, dot(N, V));
    float NoL = std::max(0.0f, dot(N, L));
    float NoH = std::max(0.0f, dot(N, H));
    float VoH = std::max(0.0f, dot(H, V));
    if (NoV > 0.0f && NoL > 0.0f && NoH > 0.0f) {
        float D = ggx_d(alpha, NoH);
        Col F0 = col(0.04f * (1.0f - metal)) + metal * base;
        Col F = fresnel_schlick(F0, VoH);
        float G = smith(alpha, NoV, NoL);
        Col kD = col(1.0f - metal);
        kD = kD * (col(1.0f) - F);
        Col diffuse = kD * base / (float)M_PI;
        Col spec = (F * D * G) / (4.0f * NoV * NoL);
        pdf = D * NoH / (4.0f * VoH);
        out = diffuse + spec;
    }
    return out;
}

float power_heuristic(float a, float b)  // :513-518
{
    float a2 = a * a;
    return a2 / (a2 + b * b);
}

Col env_from_dir(const Ctx& C, V3 d)  // :520-530
{
    const Scene& S = C.S;
    float u = 0.5f + std::atan2(d.z, d.x) / (2.0f * (float)M_PI);
    float v = 0.5f + std::asin(d.y) / (float)M_PI;
    int x = std::max(std::min((int)(u * S.ew), S.ew - 1), 0);
    int y = std::max(std::min((int)(v * S.eh), S.eh - 1), 0);
    return S.env[y * S.ew + x];
}

void cdf_search(const Scene& S, float value, int& x, int& y)  // :532-567
{
    int lower = 0, upper = S.eh - 1, xi = S.ew - 1;
    while (lower < upper) {
        int yi = (lower + upper) / 2;
        if (value < S.cdf[yi * S.ew + xi])
            upper = yi;
        else
            lower = yi + 1;
    }
    y = std::max(std::min(lower, S.eh), 0);
    lower = 0;
    upper = S.ew - 1;
    while (lower < upper) {
        int xm = (lower + upper) / 2;
        if (value < S.cdf[y * S.ew + xm])
            upper = xm;
        else
            lower = xm + 1;
    }
    x = std::max(std::min(lower, S.ew), 0);
}

Col sample_env(const Ctx& C, const Ray& ray, const Hit& h, const Mat& m, Rng& rng)  // :569-631
{
    const Scene& S = C.S;
    float total = S.cdf[S.cdf.size() - 1];
    int x, y;
    cdf_search(S, rng() * total, x, y);
    float u = (float)x / S.ew, v = (float)y / S.eh;
    float phi = u * 2.0f * M_PI;
    float theta = v * M_PI;
    Col env_sample = col(0.0f);
    float st = std::sin(theta), ctt = std::cos(theta);
    V3 dir = v3(-st * std::cos(phi), -ctt, -st * std::sin(phi));
    float cosine = dot(h.n, dir);
    if (cosine > 0.0f) {
        Hit trash;
        if (!intersect_scene(S, Ray{h.p + h.n * 1.0e-4f, dir}, trash, C.cnt)) {
            float pdf = S.env_lum[std::min(y, S.eh - 1) * S.ew + std::min(x, S.ew - 1)] / total;
            pdf = (pdf * S.ew * S.eh) / (2.0f * M_PI * M_PI * st);
            int xc = std::min(std::max(x, 0), S.ew - 1), yc = std::min(std::max(y, 0), S.eh - 1);  // image.h:165-177
            Col rad = S.env[yc * S.ew + xc];
            Col brdf = ct_brdf(m, dir, -ray.d, h.n);
            float bp = ct_pdf(m, -ray.d, dir, h.n);
            float mis = power_heuristic(pdf, bp);
            env_sample = brdf * cosine * mis * rad / pdf;
        }
    }
    float bsp;
    V3 bdir = v3(0, 0, 0);
    Col bis = ct_sample(m, -ray.d, h.n, bdir, bsp, rng);
    cosine = std::max(dot(h.n, bdir), 0.0f);
    Col brdf_sample = col(0.0f);
    if (bsp != 0.0f && cosine > 0.0f) {
        Hit trash;
        if (!intersect_scene(S, Ray{h.p + h.n * 1.0e-5f, bdir}, trash, C.cnt)) {
            Col sky = env_from_dir(C, bdir);
            float th = std::acos(bdir.z);
            float sth = std::sin(th);
            float epdf = luminance(sky) / S.cdf[S.cdf.size() - 1];
            epdf *= S.ew * S.eh;
            epdf /= (2.0f * M_PI * M_PI * sth);
            float mis = power_heuristic(bsp, epdf);
            brdf_sample = sky * mis * cosine * bis / bsp;
        }
    }
    return brdf_sample + env_sample;
}

Col sample_lights(const Ctx& C, const Ray& ray, const Hit& h, const Mat& m, Rng& rng)  // :633-713
{
    const Scene& S = C.S;
    Col light = col(0.0f);
    if (S.emissive.size() > 0) {
        // sample_random_point_on_lights :715-742
        int li = rng() * S.emissive.size();
        li = S.emissive[li];
        const Tri& tr = S.tris[li];
        float r1 = rng(), r2 = rng();
        float sr1 = std::sqrt(r1);
        float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
        V3 AB = tr.b - tr.a, AC = tr.c - tr.a;
        V3 P = tr.a + AB * u + AC * v;
        V3 nrm = cross(AB, AC);
        float ln = length(nrm);
        float kk = 1 / ln;
        V3 lnorm = kk * nrm;
        float area = ln * 0.5f;
        float nb = S.emissive.size();
        float lpdf = 1.0f / (nb * area);

        V3 so = h.p + h.n * 1.0e-4f;
        V3 sd = P - so;
        float dist = length(sd);
        V3 sdn = normalize(sd);
        Ray sray{so, sdn};
        float dl = std::max(dot(lnorm, -sdn), 0.0f);
        if (dl > 0.0f) {
            Hit sh;  // evaluate_shadow_ray :744-759
            bool in_shadow = false;
            if (intersect_scene(S, sray, sh, C.cnt)) in_shadow = sh.t + 1.0e-4f < dist;
            if (!in_shadow) {
                const Mat& em = S.mats[S.mat_idx[li]];
                lpdf *= dist * dist;
                lpdf /= dl;
                Col brdf = ct_brdf(m, sray.d, -ray.d, h.n);
                float cp = ct_pdf(m, -ray.d, sdn, h.n);
                if (cp != 0.0f) {
                    float mis = power_heuristic(lpdf, cp);
                    float cosine = dot(h.n, sdn);
                    light = em.emission * cosine * brdf * mis / lpdf;
                }
            }
        }
    }
    Col bmis = col(0.0f);
    V3 sdir = v3(0, 0, 0);
    float dpdf;
    Col brdf = ct_sample(m, -ray.d, h.n, sdir, dpdf, rng);
    if (!is_black(brdf)) {
        Hit nh;
        if (intersect_scene(S, Ray{h.p + h.n * 1.0e-5f, sdir}, nh, C.cnt)) {
            float ca = std::max(dot(nh.n, -sdir), 0.0f);
            if (ca > 0.0f) {
                const Mat& mm = S.mats[S.mat_idx[nh.prim]];
                Col e = mm.emission;
                if (e.r > 0 || e.g > 0 || e.b > 0) {
                    float d2 = nh.t * nh.t;
                    float la = tri_area(S.tris[nh.prim]);
                    float lpdf = d2 / (la * ca);
                    float mis = power_heuristic(dpdf, lpdf);
                    float cosine = dot(h.n, sdir);
                    bmis = brdf * cosine * e * mis / dpdf;
                }
            }
        }
    }
    return light + bmis;
}

// draws_log (analysis only, oracle_render_log): the RNG draws of each sample, spp entries
void trace_pixel(const Ctx& C, int x, int y, float* fb, uint16_t* draws_log = nullptr)  // render_kernel.cpp:75-181
{
    const Scene& S = C.S;
    Rng rng{(uint32_t)(31 + x * y * C.spp)};
    for (int i = 0; i < 10; i++) rng();
    Col fin = col(0.0f);
    for (int s = 0; s < C.spp; s++) {
        const uint32_t d0 = rng.draws;
        float xj = (x + 0.5f) + rng() - 1.0f;
        float yj = (y + 0.5f) + rng() - 1.0f;
        Ray ray = camera_ray(C, xj, yj);
        Col thr = col(1.0f), sc = col(0.0f);
        int state = 0;  // 0 BOUNCE, 1 MISSED, 2 TERMINATED
        for (int bounce = 0; bounce < C.bounces; bounce++) {
            if (state == 0) {
                Hit h;
                if (intersect_scene(S, ray, h, C.cnt)) {
                    const Mat& m = S.mats[S.mat_idx[h.prim]];
                    Col lr = sample_lights(C, ray, h, m, rng);
                    Col er = sample_env(C, ray, h, m, rng);
                    float bpdf;
                    V3 dir = v3(0, 0, 0);
                    Col brdf = ct_sample(m, -ray.d, h.n, dir, bpdf, rng);
                    if (bounce == 0) sc = sc + m.emission;
                    sc = sc + (lr + er) * thr;
                    if ((brdf.r == 0.0f && brdf.g == 0.0f && brdf.b == 0.0f) || bpdf < 1.0e-8f || std::isinf(bpdf)) {
                        state = 2;
                        break;
                    }
                    thr = thr * (brdf * std::max(0.0f, dot(dir, h.n)) / bpdf);
                    ray = Ray{h.p + h.n * 1.0e-4f, dir};
                    state = 0;
                } else
                    state = 1;
            } else if (state == 1) {
                if (bounce == 1) sc = sc + env_from_dir(C, ray.d) * thr;
                break;
            } else
                break;
        }
        fin = fin + sc;
        if (draws_log) draws_log[s] = (uint16_t)(rng.draws - d0);
    }
    float k = (float)C.spp;
    fin.r /= k;
    fin.g /= k;
    fin.b /= k;
    float* px = fb + 4 * ((size_t)y * C.W + x);
    px[0] += fin.r;
    px[1] += fin.g;
    px[2] += fin.b;
    // alpha: final_color.a = 0 is added, then exp/pow keep alpha (color.h:465-473)
    float a = px[3] + 0.0f;
    px[3] = 1.0f + (-((-a) * 1.5f));
    for (int c = 0; c < 3; c++) {
        float e = std::exp((-px[c]) * 1.5f);
        float tm = 1.0f + (-e);
        px[c] = std::pow(tm, 1.0f / 2.2f);
    }
}

}  // namespace

// ------------------------------------------------------------------ C API
extern "C" {

void* oracle_scene_create(const float* tris, int ntri, const int* mat_idx, const float* mats, int nmat,
                          const int* emissive, int nem, const float* spheres, int nsph, const float* env_rgb,
                          int ew, int eh, int max_depth, int leaf_max)
{
    Scene* S = new Scene();
    S->tris.resize(ntri);
    std::memcpy(S->tris.data(), tris, sizeof(float) * 9 * (size_t)ntri);
    // one material index per triangle, then one per sphere (main.cpp:20-30
    // add_sphere_to_scene appends them in that order)
    S->mat_idx.assign(mat_idx, mat_idx + ntri + nsph);
    S->mats.resize(nmat);
    for (int i = 0; i < nmat; i++) {
        const float* p = mats + 10 * i;  // emission rgba, diffuse rgba, metalness, roughness
        S->mats[i] = Mat{Col{p[0], p[1], p[2]}, Col{p[4], p[5], p[6]}, p[8], p[9]};
    }
    S->emissive.assign(emissive, emissive + nem);
    for (int i = 0; i < nsph; i++) {
        const float* p = spheres + 5 * i;
        S->sph.push_back(Sph{v3(p[0], p[1], p[2]), p[3], (int)p[4]});
    }
    // BVH::BVH (bvh.cpp:19-37) + build_bvh (bvh.cpp:52-60)
    V3 mn = v3(INFINITY, INFINITY, INFINITY), mx = v3(-INFINITY, -INFINITY, -INFINITY);
    for (const Tri& t : S->tris) {
        const V3* p = &t.a;
        for (int i = 0; i < 3; i++) mn = vmin(mn, p[i]), mx = vmax(mx, p[i]);
    }
    S->root = new Node(mn, mx);
    for (int id = 0; id < ntri; id++) S->root->insert(S->tris, id, 0, max_depth, leaf_max);
    S->root->compute_volume(S->tris);
    // env: read_image_float (utils.cpp:100-124) + compute_env_map_cdf (utils.cpp:126-142)
    if (env_rgb && ew > 0 && eh > 0) {
        S->ew = ew;
        S->eh = eh;
        S->env.resize((size_t)ew * eh);
        S->env_lum.resize((size_t)ew * eh);
        S->cdf.resize((size_t)ew * eh);
        for (size_t i = 0; i < S->env.size(); i++) {
            S->env[i] = Col{env_rgb[3 * i], env_rgb[3 * i + 1], env_rgb[3 * i + 2]};
            const Col& c = S->env[i];
            S->env_lum[i] = 0.3086 * c.r + 0.6094 * c.g + 0.0820 * c.b;  // image.h:80-85
        }
        S->cdf[0] = 0.0f;
        for (int i = 0; i < ew * eh; i++) S->cdf[i] = S->cdf[std::max(i - 1, 0)] + S->env_lum[i];
    }
    return S;
}

void oracle_scene_destroy(void* s) { delete (Scene*)s; }

// USE_BVH (render_kernel.h:13): 1 = octree (the reference's build), 0 = brute-force loop
void oracle_set_use_bvh(void* s, int use_bvh) { ((Scene*)s)->brute = use_bvh == 0; }

// Pre-order dump of the octree: per node {leaf, ntris, tris..., 6 floats min/max, 14 floats planes},
// the same record format as oracle/ref/ref_driver.cpp "bvh". Returns bytes written (or needed).
static void dump_rec(const Node* n, std::vector<char>& out)
{
    auto put = [&](const void* p, size_t b) { out.insert(out.end(), (const char*)p, (const char*)p + b); };
    int leaf = n->leaf ? 1 : 0, nt = (int)n->tris.size();
    put(&leaf, 4);
    put(&nt, 4);
    put(n->tris.data(), 4 * n->tris.size());
    put(&n->mn, 12);
    put(&n->mx, 12);
    put(n->vol.dn, 28);
    put(n->vol.df, 28);
    if (!n->leaf)
        for (auto* c : n->ch) dump_rec(c, out);
}
long oracle_bvh_dump(void* s, char* buf, long cap)
{
    std::vector<char> out;
    dump_rec(((Scene*)s)->root, out);
    if (buf && cap >= (long)out.size()) std::memcpy(buf, out.data(), out.size());
    return (long)out.size();
}

// rays: n x {ox,oy,oz,dx,dy,dz}; out: n x {found, prim, t, px,py,pz, nx,ny,nz, u, v} (11 x 4 B)
void oracle_intersect(void* s, const float* rays, int n, void* out, uint64_t* counters)
{
    const Scene& S = *(Scene*)s;
    Counters tot;
#pragma omp parallel
    {
        Counters c;
#pragma omp for schedule(dynamic, 256)
        for (int i = 0; i < n; i++) {
            Ray r{v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5])};
            Hit h;
            bool f = intersect_scene(S, r, h, counters ? &c : nullptr);
            int32_t* o = (int32_t*)out + 11 * (size_t)i;
            o[0] = f ? 1 : 0;
            o[1] = h.prim;
            std::memcpy(o + 2, &h.t, 4);
            std::memcpy(o + 3, &h.p, 12);
            std::memcpy(o + 6, &h.n, 12);
            std::memcpy(o + 9, &h.u, 4);
            std::memcpy(o + 10, &h.v, 4);
        }
#pragma omp critical
        {
            tot.rays += c.rays;
            tot.vol_tests += c.vol_tests;
            tot.vol_tests_empty += c.vol_tests_empty;
            tot.tri_tests += c.tri_tests;
            tot.leaf_visits += c.leaf_visits;
        }
    }
    if (counters) {
        counters[0] = tot.rays;
        counters[1] = tot.vol_tests;
        counters[2] = tot.vol_tests_empty;
        counters[3] = tot.tri_tests;
        counters[4] = tot.leaf_visits;
    }
}

// Renders the listed pixels (n x {x,y}) into a W x H RGBA framebuffer `fb`
// (read-modify-write, like RenderKernel::ray_trace_pixel). px == nullptr
// renders the whole frame (RenderKernel::render, render_kernel.cpp:189-211).
// counters (optional, 5 x u64): rays, vol tests, empty-vol tests, tri tests, leaf visits.
double oracle_render(void* s, const float* view16, float fov_dist, int W, int H, int spp, int bounces,
                     const int* px, long n, float* fb, int nthreads, uint64_t* counters)
{
    const Scene& S = *(Scene*)s;
    Cam cam;
    std::memcpy(cam.m, view16, 64);
    cam.fov_dist = fov_dist;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    Counters tot;
    const double t0 = omp_get_wtime();
#pragma omp parallel
    {
        Counters c;
        Ctx C{S, cam, W, H, spp, bounces, counters ? &c : nullptr, nullptr};
        if (px) {
#pragma omp for schedule(dynamic, 16)
            for (long i = 0; i < n; i++) trace_pixel(C, px[2 * i], px[2 * i + 1], fb);
        } else {
#pragma omp for schedule(dynamic)
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) trace_pixel(C, x, y, fb);
        }
#pragma omp critical
        {
            tot.rays += c.rays;
            tot.vol_tests += c.vol_tests;
            tot.vol_tests_empty += c.vol_tests_empty;
            tot.tri_tests += c.tri_tests;
            tot.leaf_visits += c.leaf_visits;
        }
    }
    const double t1 = omp_get_wtime();
    if (counters) {
        counters[0] = tot.rays;
        counters[1] = tot.vol_tests;
        counters[2] = tot.vol_tests_empty;
        counters[3] = tot.tri_tests;
        counters[4] = tot.leaf_visits;
    }
    return t1 - t0;
}

// Analysis only (tools/chain_model.py): oracle_render over a pixel list, logging each
// sample's RNG draw count into draws_log[n][spp] — the per-pixel sample chain the GPU
// wavefront walks in order.
void oracle_render_log(void* s, const float* view16, float fov_dist, int W, int H, int spp, int bounces,
                       const int* px, long n, float* fb, uint16_t* draws_log)
{
    const Scene& S = *(Scene*)s;
    Cam cam;
    std::memcpy(cam.m, view16, 64);
    cam.fov_dist = fov_dist;
#pragma omp parallel
    {
        Ctx C{S, cam, W, H, spp, bounces, nullptr, nullptr};
#pragma omp for schedule(dynamic, 16)
        for (long i = 0; i < n; i++) trace_pixel(C, px[2 * i], px[2 * i + 1], fb, draws_log + (size_t)i * spp);
    }
}

}  // extern "C"
