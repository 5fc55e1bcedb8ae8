// rt_scene.cpp — host scene preparation (see rt_scene.h). Compiled with
// -ffp-contract=off and no -march so every float operation is a single IEEE
// SSE operation, as in the reference build.
#include "rt_scene.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <unordered_map>

namespace rt {

std::atomic<long> g_obj_parallel_min{-1};

int worker_count()
{
    for (const char* v : {"RT_HOST_THREADS", "OMP_NUM_THREADS"})
        if (const char* e = std::getenv(v))
            if (int n = std::atoi(e); n > 0) return std::min(n, 256);
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hw, 16u));
}

void parallel_for(int n, int workers, const std::function<void(int)>& fn)
{
    workers = std::max(1, std::min(workers, n));
    if (workers == 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<int> next{0};
    auto run = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) fn(i);
    };
    std::vector<std::thread> th;
    for (int w = 1; w < workers; w++) th.emplace_back(run);
    run();
    for (auto& t : th) t.join();
}

// ======================================================================= OBJ
namespace {

struct MtlMat {
    float kd[3] = {0, 0, 0}, ke[3] = {0, 0, 0};
    float pr = 0.0f, pm = 0.0f;
    int illum = 0;
};

bool read_file(const std::string& path, std::string& out)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n >= 0 && std::fread(&out[0], 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

inline const char* skip_ws(const char* p, const char* e)
{
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
    return p;
}

// Reads one token as float with correct rounding (strtof), like rapidobj's
// parser does for the "%f" decimal strings in these files.
inline bool read_float(const char*& p, const char* e, float& v)
{
    p = skip_ws(p, e);
    if (p >= e || *p == '\n') return false;
    char* end;
    v = std::strtof(p, &end);
    if (end == p) return false;
    p = end;
    return true;
}

std::string dirname_of(const std::string& path)
{
    size_t s = path.find_last_of('/');
    return s == std::string::npos ? std::string(".") : path.substr(0, s);
}

int load_mtl(const std::string& path, std::vector<MtlMat>& mats, std::unordered_map<std::string, int>& names,
             std::string& err)
{
    std::string text;
    if (!read_file(path, text)) {
        err = "cannot read material library " + path;
        return -2;
    }
    std::istringstream in(text);
    std::string line;
    MtlMat* cur = nullptr;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* p = line.c_str();
        const char* e = p + line.size();
        p = skip_ws(p, e);
        if (p >= e || *p == '#') continue;
        const char* k = p;
        while (p < e && *p != ' ' && *p != '\t') p++;
        std::string key(k, p);
        if (key == "newmtl") {
            p = skip_ws(p, e);
            std::string name(p, e);
            while (!name.empty() && (name.back() == ' ' || name.back() == '\t')) name.pop_back();
            names[name] = (int)mats.size();
            mats.emplace_back();
            cur = &mats.back();
        } else if (!cur) {
            continue;
        } else if (key == "Kd" || key == "Ke") {
            float* dst = key == "Kd" ? cur->kd : cur->ke;
            float v[3];
            int n = 0;
            while (n < 3 && read_float(p, e, v[n])) n++;
            if (n == 1) v[1] = v[2] = v[0];
            if (n >= 1) std::memcpy(dst, v, sizeof v);
        } else if (key == "Pr") {
            read_float(p, e, cur->pr);
        } else if (key == "Pm") {
            read_float(p, e, cur->pm);
        } else if (key == "illum") {
            cur->illum = std::atoi(skip_ws(p, e));
        }
    }
    return 0;
}

// OBJ index: 1-based, negative = relative to the current end.
inline bool read_index(const char*& p, const char* e, int nverts, int& out)
{
    p = skip_ws(p, e);
    if (p >= e || *p == '\n' || *p == '#') return false;
    char* end;
    long v = std::strtol(p, &end, 10);
    if (end == p) return false;
    p = end;
    while (p < e && *p != ' ' && *p != '\t' && *p != '\r') p++;  // skip /vt/vn
    out = v > 0 ? (int)(v - 1) : (int)(nverts + v);
    return true;
}

}  // namespace

int load_obj_serial(const std::string& path, Mesh& out, std::string& err)
{
    std::string text;
    if (!read_file(path, text)) {
        err = "cannot read " + path;
        return -1;
    }
    std::vector<float> pos;
    pos.reserve(text.size() / 8);
    std::vector<MtlMat> mtl;
    std::unordered_map<std::string, int> names;
    int cur_mat = -1;
    out = Mesh();
    const char* p = text.data();
    const char* end = p + text.size();
    std::vector<int> face;
    while (p < end) {
        const char* le = (const char*)std::memchr(p, '\n', end - p);
        if (!le) le = end;
        const char* q = skip_ws(p, le);
        if (q + 1 < le && q[0] == 'v' && (q[1] == ' ' || q[1] == '\t')) {
            q += 1;
            float v[3];
            for (int i = 0; i < 3; i++)
                if (!read_float(q, le, v[i])) {
                    err = "bad vertex line";
                    return -3;
                }
            pos.insert(pos.end(), v, v + 3);
        } else if (q + 1 < le && q[0] == 'f' && (q[1] == ' ' || q[1] == '\t')) {
            q += 1;
            face.clear();
            int idx;
            const int nv = (int)(pos.size() / 3);
            while (read_index(q, le, nv, idx)) face.push_back(idx);
            if (face.size() < 3) {
                err = "face with fewer than 3 vertices";
                return -3;
            }
            for (int i : face)
                if (i < 0 || i >= nv) {
                    err = "face index out of range";
                    return -3;
                }
            auto emit = [&](int i0, int i1, int i2) {
                const int id[3] = {i0, i1, i2};
                for (int k = 0; k < 3; k++) out.tris.insert(out.tris.end(), &pos[3 * id[k]], &pos[3 * id[k]] + 3);
                out.mat_idx.push_back(cur_mat + 1);  // utils.cpp:51-56
                bool em = false;
                if (cur_mat >= 0) {
                    const float* ke = mtl[cur_mat].ke;
                    em = ke[0] > 0 || ke[1] > 0 || ke[2] > 0;  // utils.cpp:58-69
                }
                if (em) out.emissive.push_back(out.ntris() - 1);
            };
            if (face.size() == 3) {
                emit(face[0], face[1], face[2]);
            } else if (face.size() == 4) {
                // rapidobj::Triangulate quad rule (rapidobj.hpp:7164-7225): split on the
                // shorter diagonal, d02 < d13 computed in float.
                const float* P0 = &pos[3 * face[0]];
                const float* P1 = &pos[3 * face[1]];
                const float* P2 = &pos[3 * face[2]];
                const float* P3 = &pos[3 * face[3]];
                float e02x = P0[0] - P2[0], e02y = P0[1] - P2[1], e02z = P0[2] - P2[2];
                float e13x = P1[0] - P3[0], e13y = P1[1] - P3[1], e13z = P1[2] - P3[2];
                float d02 = e02x * e02x + e02y * e02y + e02z * e02z;
                float d13 = e13x * e13x + e13y * e13y + e13z * e13z;
                bool less = d02 < d13;
                emit(face[0], face[1], less ? face[2] : face[3]);
                emit(less ? face[0] : face[1], face[2], face[3]);
            } else {
                err = "polygons with more than 4 vertices are not supported (rapidobj earcut path)";
                return -4;
            }
        } else if (q + 6 < le && std::strncmp(q, "usemtl", 6) == 0 && (q[6] == ' ' || q[6] == '\t')) {
            q = skip_ws(q + 6, le);
            std::string name(q, le);
            while (!name.empty() && (name.back() == ' ' || name.back() == '\t' || name.back() == '\r')) name.pop_back();
            auto it = names.find(name);
            cur_mat = it == names.end() ? -1 : it->second;
        } else if (q + 6 < le && std::strncmp(q, "mtllib", 6) == 0 && (q[6] == ' ' || q[6] == '\t')) {
            q = skip_ws(q + 6, le);
            std::string name(q, le);
            while (!name.empty() && (name.back() == ' ' || name.back() == '\t' || name.back() == '\r')) name.pop_back();
            int r = load_mtl(dirname_of(path) + "/" + name, mtl, names, err);
            if (r) return r;
        }
        p = le + 1;
    }
    // SimpleMaterial list (utils.cpp:73-95)
    auto push_mat = [&](float er, float eg, float eb, float dr, float dg, float db, float metal, float rough) {
        const float m[10] = {er, eg, eb, 1.0f, dr, dg, db, 1.0f, metal, rough};
        out.mats.insert(out.mats.end(), m, m + 10);
    };
    push_mat(1.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    for (const MtlMat& m : mtl) {
        float rough = std::max(1.0e-2f, m.pr);
        float metal = m.pm;
        if (m.illum == 0) {
            rough = 1.0f;
            metal = 0.0f;
        }
        push_mat(m.ke[0], m.ke[1], m.ke[2], m.kd[0], m.kd[1], m.kd[2], metal, rough);
    }
    return 0;
}

// Parallel form of load_obj_serial: the text is cut into chunks at line ends;
// workers parse each chunk's vertex and face lines (faces keep their raw OBJ
// indices, their line offset and the chunk-local vertex count, for relative
// indices), the mtllib / usemtl lines are replayed in file order on one thread (so
// a usemtl resolves against the libraries loaded before it), and workers then
// check and emit each chunk's faces at their final offsets. Every failure is
// positioned (the byte offset of its line: a bad vertex or short face while
// parsing, a library that does not load at its mtllib line, an out-of-range index
// or a face of more than 4 vertices at its face line, in load_obj_serial's check
// order), and the first in file order is reported, as the serial loader stops at
// the first failing line.
namespace {
struct ObjErr {
    size_t at = SIZE_MAX;
    int code = 0;
    std::string msg;
    void set(size_t a, int c, const std::string& m)
    {
        if (a < at) at = a, code = c, msg = m;
    }
};
struct ObjChunk {
    const char *b, *e;
    std::vector<float> verts;
    std::vector<long> idx;           // raw OBJ indices of the chunk's faces, concatenated
    std::vector<int> fsize, fvloc;   // per face: vertex count, chunk-local vertex count before it
    std::vector<size_t> fpos;        // per face: byte offset of its line
    struct Ev {
        int kind;  // 0 usemtl, 1 mtllib
        int face;  // chunk-local face index it precedes
        size_t at;
        std::string name;
    };
    std::vector<Ev> ev;
    ObjErr perr;  // the chunk's parse error (its parse stops there)
    // phase 2 results
    size_t vbase = 0, tbase = 0;
    bool live = false;  // at or before the first chunk with a parse / library error
    std::vector<std::pair<int, int>> mat_at;  // (local face, material) transitions
    int mat0 = -1;
    std::vector<int> emissive;
    ObjErr ferr;  // the chunk's first face error (index range, > 4 vertices)
};
}  // namespace

int load_obj(const std::string& path, Mesh& out, std::string& err)
{
    std::string text;
    if (!read_file(path, text)) {
        err = "cannot read " + path;
        return -1;
    }
    const int workers = worker_count();
    const long pm = g_obj_parallel_min.load();  // (rt_test_obj_parallel_min: tests force the chunked path)
    const size_t par_min = pm >= 0 ? (size_t)pm : (size_t)4 << 20;
    if (text.size() < par_min || workers < 2) return load_obj_serial(path, out, err);
    out = Mesh();
    const char* T = text.data();
    const size_t N = text.size();
    const int nch = 4 * workers;
    std::vector<ObjChunk> ch(nch);
    {
        size_t pos = 0;
        for (int c = 0; c < nch; c++) {
            size_t end = c + 1 == nch ? N : std::max(pos, N * (c + 1) / nch);
            while (end < N && T[end - 1] != '\n') end++;
            ch[c].b = T + pos;
            ch[c].e = T + end;
            pos = end;
        }
    }
    parallel_for(nch, workers, [&](int c) {
        ObjChunk& C = ch[c];
        const char* p = C.b;
        while (p < C.e) {
            const char* le = (const char*)std::memchr(p, '\n', C.e - p);
            if (!le) le = C.e;
            const char* q = skip_ws(p, le);
            if (q + 1 < le && q[0] == 'v' && (q[1] == ' ' || q[1] == '\t')) {
                q += 1;
                float v[3];
                bool ok = true;
                for (int i = 0; i < 3 && ok; i++) ok = read_float(q, le, v[i]);
                if (!ok) {
                    C.perr.set((size_t)(p - T), -3, "bad vertex line");
                    break;
                }
                C.verts.insert(C.verts.end(), v, v + 3);
            } else if (q + 1 < le && q[0] == 'f' && (q[1] == ' ' || q[1] == '\t')) {
                q += 1;
                int n = 0;
                for (;;) {
                    const char* r = skip_ws(q, le);
                    if (r >= le || *r == '\n' || *r == '#') break;
                    char* end;
                    const long v = std::strtol(r, &end, 10);
                    if (end == r) break;
                    q = end;
                    while (q < le && *q != ' ' && *q != '\t' && *q != '\r') q++;  // skip /vt/vn
                    C.idx.push_back(v);
                    n++;
                }
                if (n < 3) {
                    C.idx.resize(C.idx.size() - n);
                    C.perr.set((size_t)(p - T), -3, "face with fewer than 3 vertices");
                    break;
                }
                C.fsize.push_back(n);  // (> 4 vertices: an error once its indices are checked, below)
                C.fvloc.push_back((int)(C.verts.size() / 3));
                C.fpos.push_back((size_t)(p - T));
            } else if (q + 6 < le && (std::strncmp(q, "usemtl", 6) == 0 || std::strncmp(q, "mtllib", 6) == 0) &&
                       (q[6] == ' ' || q[6] == '\t')) {
                const int kind = q[0] == 'u' ? 0 : 1;
                q = skip_ws(q + 6, le);
                std::string name(q, le);
                while (!name.empty() && (name.back() == ' ' || name.back() == '\t' || name.back() == '\r')) name.pop_back();
                C.ev.push_back({kind, (int)C.fsize.size(), (size_t)(p - T), std::move(name)});
            }
            p = le + 1;
        }
    });
    // file order: offsets, materials (mtllib / usemtl replayed); chunks after the first
    // parse or library error are not needed (the serial loader stops there)
    std::vector<MtlMat> mtl;
    std::unordered_map<std::string, int> names;
    int cur = -1;
    size_t vb = 0, tb = 0;
    ObjErr first;  // the first failure in file order
    for (ObjChunk& C : ch) {
        C.vbase = vb;
        C.tbase = tb;
        C.mat0 = cur;
        C.live = true;
        for (auto& ev : C.ev) {
            if (ev.kind == 1) {
                std::string e2;
                if (int r = load_mtl(dirname_of(path) + "/" + ev.name, mtl, names, e2)) {
                    first.set(ev.at, r, e2);
                    break;
                }
            } else {
                auto it = names.find(ev.name);
                cur = it == names.end() ? -1 : it->second;
                C.mat_at.push_back({ev.face, cur});
            }
        }
        first.set(C.perr.at, C.perr.code, C.perr.msg);
        vb += C.verts.size() / 3;
        for (int n : C.fsize) tb += n == 3 ? 1 : 2;
        if (first.at != SIZE_MAX) break;
    }
    std::vector<float> pos(3 * vb);
    out.tris.resize(9 * tb);
    out.mat_idx.resize(tb);
    parallel_for(nch, workers, [&](int c) {
        const ObjChunk& C = ch[c];
        if (C.live) std::memcpy(pos.data() + 3 * C.vbase, C.verts.data(), C.verts.size() * 4);
    });
    const size_t stop_at = first.at;  // faces at or after it are never reached by the serial loader
    parallel_for(nch, workers, [&](int c) {
        ObjChunk& C = ch[c];
        if (!C.live) return;
        size_t t = C.tbase, o = 0;
        size_t m = 0;
        int mat = C.mat0;
        for (size_t f = 0; f < C.fsize.size() && C.fpos[f] < stop_at; f++) {
            while (m < C.mat_at.size() && C.mat_at[m].first <= (int)f) mat = C.mat_at[m++].second;
            const int n = C.fsize[f];
            const long nv = (long)(C.vbase + C.fvloc[f]);
            int face[4];
            bool bad = false;
            for (int k = 0; k < n; k++) {  // (load_obj_serial: the index range first, then the vertex count)
                const long v = C.idx[o + k];
                const int i = v > 0 ? (int)(v - 1) : (int)(nv + v);
                if (i < 0 || i >= nv) bad = true;
                if (k < 4) face[k] = i;
            }
            o += n;
            if (bad) {
                C.ferr.set(C.fpos[f], -3, "face index out of range");
                return;
            }
            if (n > 4) {
                C.ferr.set(C.fpos[f], -4, "polygons with more than 4 vertices are not supported (rapidobj earcut path)");
                return;
            }
            auto emit = [&](int i0, int i1, int i2) {
                const int id[3] = {i0, i1, i2};
                for (int k = 0; k < 3; k++) std::memcpy(&out.tris[9 * t + 3 * k], &pos[3 * (size_t)id[k]], 12);
                out.mat_idx[t] = mat + 1;  // utils.cpp:51-56
                if (mat >= 0) {
                    const float* ke = mtl[mat].ke;
                    if (ke[0] > 0 || ke[1] > 0 || ke[2] > 0) C.emissive.push_back((int)t);  // utils.cpp:58-69
                }
                t++;
            };
            if (n == 3) {
                emit(face[0], face[1], face[2]);
            } else {  // rapidobj::Triangulate quad rule (rapidobj.hpp:7164-7225), as load_obj_serial
                const float* P0 = &pos[3 * (size_t)face[0]];
                const float* P1 = &pos[3 * (size_t)face[1]];
                const float* P2 = &pos[3 * (size_t)face[2]];
                const float* P3 = &pos[3 * (size_t)face[3]];
                float e02x = P0[0] - P2[0], e02y = P0[1] - P2[1], e02z = P0[2] - P2[2];
                float e13x = P1[0] - P3[0], e13y = P1[1] - P3[1], e13z = P1[2] - P3[2];
                float d02 = e02x * e02x + e02y * e02y + e02z * e02z;
                float d13 = e13x * e13x + e13y * e13y + e13z * e13z;
                bool less = d02 < d13;
                emit(face[0], face[1], less ? face[2] : face[3]);
                emit(less ? face[0] : face[1], face[2], face[3]);
            }
        }
    });
    for (const ObjChunk& C : ch) first.set(C.ferr.at, C.ferr.code, C.ferr.msg);
    if (first.at != SIZE_MAX) {
        err = first.msg;
        return first.code;
    }
    for (const ObjChunk& C : ch) out.emissive.insert(out.emissive.end(), C.emissive.begin(), C.emissive.end());
    // SimpleMaterial list (utils.cpp:73-95)
    auto push_mat = [&](float er, float eg, float eb, float dr, float dg, float db, float metal, float rough) {
        const float mm[10] = {er, eg, eb, 1.0f, dr, dg, db, 1.0f, metal, rough};
        out.mats.insert(out.mats.end(), mm, mm + 10);
    };
    push_mat(1.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    for (const MtlMat& m : mtl) {
        float rough = std::max(1.0e-2f, m.pr);
        float metal = m.pm;
        if (m.illum == 0) {
            rough = 1.0f;
            metal = 0.0f;
        }
        push_mat(m.ke[0], m.ke[1], m.ke[2], m.kd[0], m.kd[1], m.kd[2], metal, rough);
    }
    return 0;
}

// ==================================================================== octree
namespace {

const float S3 = std::sqrt(3.0f) / 3;
const float PN[7][3] = {{1, 0, 0},   {0, 1, 0},    {0, 0, 1},   {S3, S3, S3},
                        {-S3, S3, S3}, {-S3, -S3, S3}, {S3, -S3, S3}};  // bvh.cpp:8-16

inline float pdot(int i, const float* p) { return PN[i][0] * p[0] + PN[i][1] * p[1] + PN[i][2] * p[2]; }
inline float fmin_(float a, float b) { return (b < a) ? b : a; }  // std::min
inline float fmax_(float a, float b) { return (a < b) ? b : a; }  // std::max

void root_box(const float* tris, int ntris, float* mn, float* mx)  // bvh.cpp:19-37
{
    for (int k = 0; k < 3; k++) mn[k] = INFINITY, mx[k] = -INFINITY;
    for (int t = 0; t < ntris; t++)
        for (int j = 0; j < 3; j++)
            for (int k = 0; k < 3; k++) {
                float v = tris[9 * (size_t)t + 3 * j + k];
                mn[k] = fmin_(mn[k], v);
                mx[k] = fmax_(mx[k], v);
            }
}

struct Builder {
    const float* T;
    Octree& t;
    Builder(const float* tris, Octree& tree) : T(tris), t(tree) {}

    int new_node(const float* mn, const float* mx)
    {
        OctNode n;
        std::memcpy(n.mn, mn, 12);
        std::memcpy(n.mx, mx, 12);
        for (int i = 0; i < 7; i++) n.dn[i] = INFINITY, n.df[i] = -INFINITY;
        for (int i = 0; i < 8; i++) n.child[i] = -1;
        t.pool.push_back(std::move(n));
        return (int)t.pool.size() - 1;
    }
    void create_children(int ni)  // bvh.h:67-81, including the child _min offsets as written
    {
        float mn[3], mx[3];
        std::memcpy(mn, t.pool[ni].mn, 12);
        std::memcpy(mx, t.pool[ni].mx, 12);
        const float cx = (mn[0] + mx[0]) / 2, cy = (mn[1] + mx[1]) / 2, cz = (mn[2] + mx[2]) / 2;
        const float b[8][6] = {
            {mn[0], mn[1], mn[2], cx, cy, cz},
            {cx, mn[1], mn[2], mx[0], cy, cz},
            {mn[0] + 0.0f, mn[1] + cy, mn[2] + 0.0f, cx, mx[1], cz},
            {cx, cy, mn[2], mx[0], mx[1], cz},
            {mn[0] + 0.0f, mn[1] + 0.0f, mn[2] + cz, cx, cy, mx[2]},
            {cx, mn[1], cz, mx[0], cy, mx[2]},
            {mn[0] + 0.0f, mn[1] + cy, mn[2] + cz, cx, mx[1], mx[2]},
            {cx, cy, cz, mx[0], mx[1], mx[2]},
        };
        for (int i = 0; i < 8; i++) {
            int c = new_node(b[i], b[i] + 3);
            t.pool[ni].child[i] = c;
        }
    }
    void insert(int ni, int id, int depth)  // bvh.h:83-107
    {
        const bool exceeded = t.max_depth != -1 && depth == t.max_depth;
        if (t.pool[ni].leaf || exceeded) {
            t.pool[ni].tris.push_back(id);
            if ((int)t.pool[ni].tris.size() > t.leaf_max && !exceeded) {
                t.pool[ni].leaf = false;
                create_children(ni);
                std::vector<int32_t> moved;
                moved.swap(t.pool[ni].tris);
                for (int tid : moved) insert_to_children(ni, tid, depth);
            }
        } else
            insert_to_children(ni, id, depth);
    }
    // Top-down form of the insertions for node ni at `depth` receiving ids[0..n)
    // (ascending): the same tree insert() builds from the same ids in order (see
    // build_octree). The ids are partitioned stably in place, tmp[0..n) is scratch.
    void build_from(int ni, int32_t* ids, int n, int32_t* tmp, int depth, const float* cen)
    {
        const bool exceeded = t.max_depth != -1 && depth == t.max_depth;
        if (exceeded || n <= t.leaf_max) {
            t.pool[ni].tris.assign(ids, ids + n);
            return;
        }
        t.pool[ni].leaf = false;
        create_children(ni);
        const OctNode& nd = t.pool[ni];
        const float m0 = (nd.mn[0] + nd.mx[0]) / 2, m1 = (nd.mn[1] + nd.mx[1]) / 2, m2 = (nd.mn[2] + nd.mx[2]) / 2;
        int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; i++) {
            const float* c = cen + 3 * (size_t)ids[i];
            const int o = (c[0] > m0 ? 1 : 0) + (c[1] > m1 ? 2 : 0) + (c[2] > m2 ? 4 : 0);
            tmp[i] = o;
            cnt[o]++;
        }
        int off[9];
        off[0] = 0;
        for (int o = 0; o < 8; o++) off[o + 1] = off[o] + cnt[o];
        int pos[8];
        for (int o = 0; o < 8; o++) pos[o] = off[o];
        for (int i = 0; i < n; i++) {  // stable scatter into tmp, then back
            const int o = tmp[i];
            tmp[i] = ids[i] | (o << 28);  // (ids < 2^28: checked by the caller)
        }
        for (int i = 0; i < n; i++) ids[pos[tmp[i] >> 28]++] = tmp[i] & 0x0fffffff;
        int kids[8];
        for (int o = 0; o < 8; o++) kids[o] = t.pool[ni].child[o];
        for (int o = 0; o < 8; o++) build_from(kids[o], ids + off[o], cnt[o], tmp + off[o], depth + 1, cen);
    }
    void insert_to_children(int ni, int id, int depth)  // bvh.h:109-125
    {
        const float* a = T + 9 * (size_t)id;
        float c[3];
        for (int k = 0; k < 3; k++) {
            // Triangle::bbox_centroid (triangle.cpp:3-6): (min + max) * (1.f / 2)
            float lo = fmin_(a[k], fmin_(a[3 + k], a[6 + k]));
            float hi = fmax_(a[k], fmax_(a[3 + k], a[6 + k]));
            c[k] = (1.f / 2) * (lo + hi);
        }
        const OctNode& n = t.pool[ni];
        int o = 0;
        if (c[0] > (n.mn[0] + n.mx[0]) / 2) o += 1;
        if (c[1] > (n.mn[1] + n.mx[1]) / 2) o += 2;
        if (c[2] > (n.mn[2] + n.mx[2]) / 2) o += 4;
        insert(n.child[o], id, depth + 1);
    }
    void compute_volume(int ni)  // bvh.h:55-65 (iterative post-order)
    {
        std::vector<std::pair<int, int>> st{{ni, 0}};
        while (!st.empty()) {
            auto& [n, k] = st.back();
            OctNode& nd = t.pool[n];
            if (nd.leaf) {
                for (int id : nd.tris) {
                    const float* a = T + 9 * (size_t)id;
                    float tn[7], tf[7];
                    for (int i = 0; i < 7; i++) tn[i] = INFINITY, tf[i] = -INFINITY;
                    for (int i = 0; i < 7; i++)
                        for (int j = 0; j < 3; j++) {
                            float d = pdot(i, a + 3 * j);
                            tn[i] = fmin_(tn[i], d);
                            tf[i] = fmax_(tf[i], d);
                        }
                    for (int i = 0; i < 7; i++) nd.dn[i] = fmin_(nd.dn[i], tn[i]), nd.df[i] = fmax_(nd.df[i], tf[i]);
                }
                st.pop_back();
                continue;
            }
            if (k < 8) {
                int c = nd.child[k++];
                st.push_back({c, 0});
                continue;
            }
            for (int i = 0; i < 8; i++) {
                const OctNode& ch = t.pool[nd.child[i]];
                for (int p = 0; p < 7; p++) nd.dn[p] = fmin_(nd.dn[p], ch.dn[p]), nd.df[p] = fmax_(nd.df[p], ch.df[p]);
            }
            st.pop_back();
        }
    }
};

}  // namespace

// Serial build: the reference's insertion order, one triangle at a time (bvh.cpp:52-60).
void build_octree_serial(const float* tris, int ntris, int max_depth, int leaf_max, Octree& out)
{
    out.pool.clear();
    out.pool.reserve((size_t)ntris / 2 + 16);
    out.max_depth = max_depth;
    out.leaf_max = leaf_max;
    float mn[3], mx[3];
    root_box(tris, ntris, mn, mx);
    Builder b(tris, out);
    b.new_node(mn, mx);
    for (int id = 0; id < ntris; id++) b.insert(0, id, 0);  // bvh.cpp:52-60
    b.compute_volume(0);
}

// Parallel build, identical tree. With insertion in id order (bvh.cpp:52-60), a
// node receives exactly the triangles whose centroids route to it through its
// ancestors' (fixed) boxes; it splits iff more than leaf_max of them arrive
// below max_depth; and its list is in ascending id order (a split re-inserts the
// list in order, later ids are larger). So the octree is built top-down: a node's
// ascending id list is partitioned (stably) into its 8 children's, and subtrees
// below the first levels are built on worker threads into their own pools. Leaf
// volumes fold their triangles in list order and internal volumes their children
// 0..7, as bvh.h:55-65 does, so the planes are the same floats.
void build_octree(const float* tris, int ntris, int max_depth, int leaf_max, Octree& out)
{
    out.pool.clear();
    out.max_depth = max_depth;
    out.leaf_max = leaf_max;
    const int workers = worker_count();
    if (ntris < 65536 || workers < 2 || ntris >= (1 << 28)) {
        build_octree_serial(tris, ntris, max_depth, leaf_max, out);
        return;
    }
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!std::getenv("RT_VERBOSE")) return;
        auto T1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[octree] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(T1 - T0).count());
        T0 = T1;
    };
    // Triangle::bbox_centroid (triangle.cpp:3-6), as insert_to_children computes it
    std::vector<float> cen(3 * (size_t)ntris);
    parallel_for(workers, workers, [&](int w) {
        const int b = (int)((long)ntris * w / workers), e = (int)((long)ntris * (w + 1) / workers);
        for (int id = b; id < e; id++) {
            const float* a = tris + 9 * (size_t)id;
            for (int k = 0; k < 3; k++) {
                float lo = fmin_(a[k], fmin_(a[3 + k], a[6 + k]));
                float hi = fmax_(a[k], fmax_(a[3 + k], a[6 + k]));
                cen[3 * (size_t)id + k] = (1.f / 2) * (lo + hi);
            }
        }
    });
    struct Sub {
        int node;  // pool slot of the subtree root (in the top pool)
        int depth;
        std::vector<int32_t> ids;
        Octree part;  // the subtree, built by a worker
    };
    Builder top(tris, out);
    float mn[3], mx[3];
    root_box(tris, ntris, mn, mx);
    top.new_node(mn, mx);
    std::vector<int32_t> all(ntris);
    for (int i = 0; i < ntris; i++) all[i] = i;
    // expand the top levels breadth-first until there are enough subtrees to share out
    std::vector<Sub> frontier;
    frontier.push_back(Sub{0, 0, std::move(all), {}});
    const size_t want = 16 * (size_t)workers;
    for (int level = 0; level < 6 && frontier.size() < want; level++) {
        std::vector<Sub> next;
        bool grew = false;
        for (Sub& sb : frontier) {
            OctNode& n = out.pool[sb.node];
            const bool exceeded = max_depth != -1 && sb.depth == max_depth;
            if (exceeded || (int)sb.ids.size() <= leaf_max) {
                next.push_back(std::move(sb));
                continue;
            }
            n.leaf = false;
            top.create_children(sb.node);
            const OctNode& nn = out.pool[sb.node];
            const float m0 = (nn.mn[0] + nn.mx[0]) / 2, m1 = (nn.mn[1] + nn.mx[1]) / 2, m2 = (nn.mn[2] + nn.mx[2]) / 2;
            std::vector<int32_t> parts[8];
            for (int id : sb.ids) {
                const float* c = &cen[3 * (size_t)id];
                const int o = (c[0] > m0 ? 1 : 0) + (c[1] > m1 ? 2 : 0) + (c[2] > m2 ? 4 : 0);
                parts[o].push_back(id);
            }
            for (int o = 0; o < 8; o++) next.push_back(Sub{out.pool[sb.node].child[o], sb.depth + 1, std::move(parts[o]), {}});
            grew = true;
        }
        frontier.swap(next);
        if (!grew) break;
    }
    lap("centroids + top levels");
    // subtrees on the workers, largest first
    std::vector<int> order(frontier.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return frontier[a].ids.size() > frontier[b].ids.size(); });
    parallel_for((int)order.size(), workers, [&](int j) {
        Sub& sb = frontier[order[j]];
        Octree& part = sb.part;
        part.max_depth = max_depth;
        part.leaf_max = leaf_max;
        part.pool.reserve(sb.ids.size() / 2 + 16);
        Builder b(tris, part);
        const OctNode& r = out.pool[sb.node];
        b.new_node(r.mn, r.mx);
        std::vector<int32_t> tmp(sb.ids.size());
        b.build_from(0, sb.ids.data(), (int)sb.ids.size(), tmp.data(), sb.depth, cen.data());
        b.compute_volume(0);
    });
    lap("subtrees");
    // graft the subtrees into the top pool (their roots replace the frontier slots):
    // part node i > 0 of subtree j -> base[j] + i - 1, moved by the workers
    std::vector<size_t> base(frontier.size() + 1);
    base[0] = out.pool.size();
    for (size_t j = 0; j < frontier.size(); j++) base[j + 1] = base[j] + frontier[j].part.pool.size() - 1;
    out.pool.resize(base[frontier.size()]);
    parallel_for((int)frontier.size(), workers, [&](int j) {
        Sub& sb = frontier[j];
        std::vector<OctNode>& pp = sb.part.pool;
        auto remap = [&](OctNode& n) {
            if (!n.leaf)
                for (int i = 0; i < 8; i++) n.child[i] = n.child[i] == 0 ? sb.node : (int32_t)(base[j] + n.child[i] - 1);
        };
        for (size_t i = 1; i < pp.size(); i++) {
            remap(pp[i]);
            out.pool[base[j] + i - 1] = std::move(pp[i]);
        }
        remap(pp[0]);
        out.pool[sb.node] = std::move(pp[0]);
        std::vector<OctNode>().swap(pp);
    });
    lap("graft");
    // volumes of the top levels (their frontier children are done)
    std::vector<int> st;
    std::vector<int> post;
    st.push_back(0);
    std::vector<char> is_front(out.pool.size(), 0);
    for (const Sub& sb : frontier) is_front[sb.node] = 1;
    while (!st.empty()) {
        const int n = st.back();
        st.pop_back();
        if (is_front[n] || out.pool[n].leaf) continue;
        post.push_back(n);
        for (int i = 0; i < 8; i++) st.push_back(out.pool[n].child[i]);
    }
    for (size_t i = post.size(); i-- > 0;) {
        OctNode& nd = out.pool[post[i]];
        for (int c = 0; c < 8; c++) {
            const OctNode& ch = out.pool[nd.child[c]];
            for (int p = 0; p < 7; p++) nd.dn[p] = fmin_(nd.dn[p], ch.dn[p]), nd.df[p] = fmax_(nd.df[p], ch.df[p]);
        }
    }
}

std::vector<char> dump_octree(const Octree& t)
{
    std::vector<char> out;
    auto put = [&](const void* p, size_t n) { out.insert(out.end(), (const char*)p, (const char*)p + n); };
    std::vector<int> st{0};
    while (!st.empty()) {
        int ni = st.back();
        st.pop_back();
        const OctNode& n = t.pool[ni];
        int leaf = n.leaf ? 1 : 0, nt = (int)n.tris.size();
        put(&leaf, 4);
        put(&nt, 4);
        put(n.tris.data(), 4 * n.tris.size());
        put(n.mn, 12);
        put(n.mx, 12);
        put(n.dn, 28);
        put(n.df, 28);
        if (!n.leaf)
            for (int i = 7; i >= 0; i--) st.push_back(n.child[i]);
    }
    return out;
}

int octree_from_dump(const char* buf, size_t bytes, Octree& out)
{
    out.pool.clear();
    size_t o = 0;
    // stack of (parent, child slot) to attach the next record to
    std::vector<std::pair<int, int>> st;
    bool first = true;
    while (o < bytes) {
        if (o + 8 > bytes) return -1;
        int leaf, nt;
        std::memcpy(&leaf, buf + o, 4);
        std::memcpy(&nt, buf + o + 4, 4);
        o += 8;
        if (nt < 0 || o + 4 * (size_t)nt + 80 > bytes) return -1;
        OctNode n;
        n.leaf = leaf != 0;
        n.tris.resize(nt);
        std::memcpy(n.tris.data(), buf + o, 4 * (size_t)nt);
        o += 4 * (size_t)nt;
        std::memcpy(n.mn, buf + o, 12);
        std::memcpy(n.mx, buf + o + 12, 12);
        std::memcpy(n.dn, buf + o + 24, 28);
        std::memcpy(n.df, buf + o + 52, 28);
        o += 80;
        for (int i = 0; i < 8; i++) n.child[i] = -1;
        out.pool.push_back(std::move(n));
        const int me = (int)out.pool.size() - 1;
        if (!first) {
            if (st.empty()) return -1;
            auto [par, slot] = st.back();
            st.pop_back();
            out.pool[par].child[slot] = me;
        }
        first = false;
        if (!out.pool[me].leaf)
            for (int i = 7; i >= 0; i--) st.push_back({me, i});
    }
    return st.empty() && !first ? 0 : -1;
}

void flatten_octree(const Octree& t, const float* tris, int ntris, FlatBvh& out)
{
    out.nodes.clear();
    out.tri4.clear();
    out.parent.clear();
    out.leaf_of.clear();
    out.prim2k.assign(ntris, -1);
    out.max_depth = 0;
    auto empty = [&](int ni) { return t.pool[ni].leaf && t.pool[ni].tris.empty(); };
    auto fill = [&](RtNode& r, int ni) {
        std::memcpy(r.dn, t.pool[ni].dn, 28);
        std::memcpy(r.df, t.pool[ni].df, 28);
        r.ref = 0;
        r.cnt = 0;
    };
    // Depth-first: a node's children block is allocated when the node is
    // expanded, so siblings are contiguous and a subtree stays close in memory.
    struct Item {
        int ni, rec, depth;
    };
    out.nodes.push_back(RtNode{});
    out.parent.push_back(-1);
    fill(out.nodes[0], 0);
    std::vector<Item> st{{0, 0, 0}};
    while (!st.empty()) {
        Item it = st.back();
        st.pop_back();
        const OctNode& n = t.pool[it.ni];
        if (!empty(it.ni)) out.max_depth = std::max(out.max_depth, it.depth);
        if (n.leaf) {
            out.nodes[it.rec].ref = (uint32_t)(out.tri4.size() / 3);
            out.nodes[it.rec].cnt = RT_LEAF_BIT | (uint32_t)n.tris.size();
            for (int id : n.tris) {
                out.leaf_of.push_back(it.rec);
                const float* a = tris + 9 * (size_t)id;
                float4_ r0{a[0], a[1], a[2], 0.0f}, r1{a[3] - a[0], a[4] - a[1], a[5] - a[2], 0.0f},
                    r2{a[6] - a[0], a[7] - a[1], a[8] - a[2], 0.0f};
                std::memcpy(&r0.w, &id, 4);
                out.prim2k[id] = (int)(out.tri4.size() / 3);
                out.tri4.push_back(r0);
                out.tri4.push_back(r1);
                out.tri4.push_back(r2);
            }
            continue;
        }
        int kids[8], nk = 0;
        for (int i = 0; i < 8; i++)
            if (!empty(n.child[i])) kids[nk++] = n.child[i];
        const int base = (int)out.nodes.size();
        out.nodes[it.rec].ref = (uint32_t)base;
        out.nodes[it.rec].cnt = (uint32_t)nk;
        out.nodes.resize(base + nk);
        out.parent.resize(base + nk, it.rec);
        for (int k = 0; k < nk; k++) fill(out.nodes[base + k], kids[k]);
        for (int k = nk - 1; k >= 0; k--) st.push_back({kids[k], base + k, it.depth + 1});
    }
}

// ============================================================ search BVH
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
    float area() const
    {
        if (!(mx[0] >= mn[0])) return 0.0f;
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};
struct Prim {
    Box b;
    float c[3];
    int k;
};
constexpr int kBins = 16, kLeafMax = 4;

// Pads a box so every point the reference's Moller-Trumbore test can accept
// for its triangles (barycentric / t round-off ~1e-6 relative to coordinate
// magnitudes) is strictly inside, and the traversal's float slab test on the
// padded box cannot miss such a point.
// (How far the reference's test reaches outside a triangle grows with the ray's distance and
// its grazing angle, not with the coordinates: DESIGN.md §4 "Far origins and grazing hits".
// A floor of 1e-4 x the scene's magnitude on every pad, 10x this one for the dragon's boxes,
// cut the probe's near grazing misses only ~5x: profiles/r06_far_origin.json.)
void pad_box(const Box& b, float* mn, float* mx)
{
    float mag = 1.0f;
    for (int i = 0; i < 3; i++) mag = std::max(mag, std::max(std::fabs(b.mn[i]), std::fabs(b.mx[i])));
    const float pad = 1e-4f * mag;
    for (int i = 0; i < 3; i++) mn[i] = b.mn[i] - pad, mx[i] = b.mx[i] + pad;
}

struct SahBuilder {
    std::vector<Prim>& P;
    std::vector<BvhNode>& nodes;
    int workers = 1;
    static constexpr int kParMin = 1 << 15;  // ranges binned by the workers (top levels)
    explicit SahBuilder(std::vector<Prim>& p, std::vector<BvhNode>& n) : P(p), nodes(n) {}

    // centroid bins of [b, e) on one axis (min / max merges: any chunk order gives the same boxes)
    void bin(int ax, int b, int e, float lo, float sc, Box* bb, int* cnt) const
    {
        for (int i = 0; i < kBins; i++) bb[i].reset(), cnt[i] = 0;
        auto run = [&](int cb, int ce, Box* xb, int* xc) {  // (bins in locals: no false sharing)
            Box lb[kBins];
            int lc[kBins] = {0};
            for (auto& x : lb) x.reset();
            for (int i = cb; i < ce; i++) {
                const int bi = std::min(kBins - 1, (int)((P[i].c[ax] - lo) * sc));
                lc[bi]++;
                lb[bi].grow(P[i].b);
            }
            for (int i = 0; i < kBins; i++) xb[i] = lb[i], xc[i] = lc[i];
        };
        if (e - b < kParMin || workers < 2) {
            run(b, e, bb, cnt);
            return;
        }
        const int nch = workers;
        std::vector<Box> pb((size_t)nch * kBins);
        std::vector<int> pc((size_t)nch * kBins, 0);
        for (auto& x : pb) x.reset();
        parallel_for(nch, workers, [&](int c) {
            run(b + (int)((long)(e - b) * c / nch), b + (int)((long)(e - b) * (c + 1) / nch), &pb[(size_t)c * kBins],
                &pc[(size_t)c * kBins]);
        });
        for (int c = 0; c < nch; c++)
            for (int i = 0; i < kBins; i++) bb[i].grow(pb[(size_t)c * kBins + i]), cnt[i] += pc[(size_t)c * kBins + i];
    }

    void bounds(int b, int e, Box& bb, Box& cb) const
    {
        bb.reset();
        cb.reset();
        if (e - b < kParMin || workers < 2) {
            for (int i = b; i < e; i++) bb.grow(P[i].b), cb.grow(P[i].c);
            return;
        }
        std::vector<Box> xb(workers), xc(workers);
        parallel_for(workers, workers, [&](int c) {
            Box lb, lc;
            lb.reset();
            lc.reset();
            const int cb0 = b + (int)((long)(e - b) * c / workers), ce = b + (int)((long)(e - b) * (c + 1) / workers);
            for (int i = cb0; i < ce; i++) lb.grow(P[i].b), lc.grow(P[i].c);
            xb[c] = lb;
            xc[c] = lc;
        });
        for (int c = 0; c < workers; c++) bb.grow(xb[c]), cb.grow(xc[c]);
    }

    // Splits [b, e) in place; returns the split point or -1 for a leaf.
    int split(int b, int e, const Box& cb)
    {
        const int n = e - b;
        if (n <= kLeafMax) return -1;
        float best = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int ax = 0; ax < 3; ax++) {
            const float lo = cb.mn[ax], ext = cb.mx[ax] - cb.mn[ax];
            if (!(ext > 0.0f)) continue;
            Box bb[kBins];
            int cnt[kBins];
            const float sc = kBins / ext;
            bin(ax, b, e, lo, sc, bb, cnt);
            float rarea[kBins];
            int rcnt[kBins];
            Box acc;
            acc.reset();
            int ac = 0;
            for (int i = kBins - 1; i > 0; i--) {
                acc.grow(bb[i]);
                ac += cnt[i];
                rarea[i] = acc.area();
                rcnt[i] = ac;
            }
            acc.reset();
            ac = 0;
            for (int i = 0; i < kBins - 1; i++) {
                acc.grow(bb[i]);
                ac += cnt[i];
                if (ac == 0 || rcnt[i + 1] == 0) continue;
                const float cost = acc.area() * ac + rarea[i + 1] * rcnt[i + 1];
                if (cost < best) best = cost, best_axis = ax, best_bin = i;
            }
        }
        int mid;
        if (best_axis < 0) {
            mid = b + n / 2;  // all centroids coincide: split by count
        } else {
            const float lo = cb.mn[best_axis], sc = kBins / (cb.mx[best_axis] - cb.mn[best_axis]);
            auto it = std::partition(P.begin() + b, P.begin() + e, [&](const Prim& p) {
                return std::min(kBins - 1, (int)((p.c[best_axis] - lo) * sc)) <= best_bin;
            });
            mid = (int)(it - P.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        return mid;
    }

    struct Task {
        int b, e, node, side;  // side: 0 left child slot, 1 right child slot of `node`
    };

    // One task of the depth-first build into `nd`: fills the slot, pushes the children.
    void process(std::vector<BvhNode>& nd, const Task& t, std::vector<Task>& st)
    {
        BvhNode& parent = nd[t.node];
        float* mn = t.side ? parent.rmin : parent.lmin;
        float* mx = t.side ? parent.rmax : parent.lmax;
        int32_t& ref = t.side ? parent.right : parent.left;
        int32_t& cnt = t.side ? parent.rcount : parent.lcount;
        if (t.e <= t.b) {  // empty slot (count -1): never entered
            for (int i = 0; i < 3; i++) mn[i] = INFINITY, mx[i] = -INFINITY;
            ref = 0;
            cnt = -1;
            return;
        }
        Box bb, cb;
        bounds(t.b, t.e, bb, cb);
        pad_box(bb, mn, mx);
        const int m = split(t.b, t.e, cb);
        if (m < 0) {
            ref = t.b;  // leaf entries are P[t.b .. t.e) in final order
            cnt = t.e - t.b;
            return;
        }
        const int ni = (int)nd.size();
        ref = ni;
        cnt = 0;
        nd.push_back(BvhNode{});  // (invalidates `parent`; not used below)
        st.push_back({m, t.e, ni, 1});
        st.push_back({t.b, m, ni, 0});
    }

    // Top levels here (their binning on the workers), then the subtrees below
    // `cutoff` primitives on the workers into their own node arrays, grafted back.
    // The tree (splits, leaf order of P) is the serial build's; only the binary
    // node numbering differs, which collapse_bvh4 (depth-first) does not see.
    void run()
    {
        auto T00 = std::chrono::steady_clock::now();
        const int n = (int)P.size();
        nodes.clear();
        nodes.push_back(BvhNode{});
        std::vector<Task> st;
        // root: split the whole set into the root node's two children
        Box bb, cb;
        bounds(0, n, bb, cb);
        int mid = n > 1 ? split(0, n, cb) : -1;
        if (mid < 0) mid = n;  // tiny scene: one leaf in the left slot, empty right
        st.push_back({mid, n, 0, 1});
        st.push_back({0, mid, 0, 0});
        const int cutoff = (workers > 1 && n >= 65536) ? std::max(4096, n / (3 * workers)) : -1;
        std::vector<Task> deferred;
        while (!st.empty()) {
            const Task t = st.back();
            st.pop_back();
            if (t.e - t.b <= cutoff && t.e - t.b > kLeafMax) {
                deferred.push_back(t);
                continue;
            }
            process(nodes, t, st);
        }
        auto T0 = std::chrono::steady_clock::now();
        if (std::getenv("RT_VERBOSE"))
            std::fprintf(stderr, "[sah] top %.1f ms: %zu nodes, %zu deferred (cutoff %d)\n",
                         std::chrono::duration<double, std::milli>(T0 - T00).count(), nodes.size(), deferred.size(), cutoff);
        if (deferred.empty()) return;
        std::vector<std::vector<BvhNode>> local(deferred.size());
        std::vector<int> order(deferred.size());
        for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
            return deferred[x].e - deferred[x].b > deferred[y].e - deferred[y].b;
        });
        parallel_for((int)deferred.size(), workers, [&](int j) {
            const int k = order[j];
            std::vector<BvhNode>& nd = local[k];
            nd.push_back(BvhNode{});  // local 0: stands in for the task's parent
            std::vector<Task> ls{{deferred[k].b, deferred[k].e, 0, deferred[k].side}};
            while (!ls.empty()) {
                const Task t = ls.back();
                ls.pop_back();
                process(nd, t, ls);
            }
        });
        if (std::getenv("RT_VERBOSE"))
            std::fprintf(stderr, "[sah] subtrees %.1f ms\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count());
        for (size_t k = 0; k < deferred.size(); k++) {
            const std::vector<BvhNode>& nd = local[k];
            const int base = (int)nodes.size() - 1;  // local i > 0 -> base + i
            auto fix = [&](int32_t& ref, int32_t cnt) {
                if (cnt == 0) ref += base;
            };
            for (size_t i = 1; i < nd.size(); i++) {
                BvhNode x = nd[i];
                fix(x.left, x.lcount);
                fix(x.right, x.rcount);
                nodes.push_back(x);
            }
            BvhNode& p = nodes[deferred[k].node];
            const BvhNode& v = nd[0];
            if (deferred[k].side) {
                std::memcpy(p.rmin, v.rmin, 12), std::memcpy(p.rmax, v.rmax, 12);
                p.right = v.right + (v.rcount == 0 ? base : 0), p.rcount = v.rcount;
            } else {
                std::memcpy(p.lmin, v.lmin, 12), std::memcpy(p.lmax, v.lmax, 12);
                p.left = v.left + (v.lcount == 0 ? base : 0), p.lcount = v.lcount;
            }
        }
    }
};
}  // namespace

// Collapses the binary BVH into a 4-wide one: a node adopts its children,
// then repeatedly opens its largest-area inner child in favour of that
// child's two children, while it has fewer than four. Boxes are copied
// unchanged (still conservatively padded); leaves keep their entries.
static void collapse_bvh4(const std::vector<BvhNode>& b2, std::vector<Bvh4Node>& b4)
{
    struct Slot {
        float mn[3], mx[3];
        int32_t ref, cnt;
        float area() const
        {
            const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
            return dx * dy + dy * dz + dz * dx;
        }
    };
    auto slots_of = [&](int n, Slot* out) {
        const BvhNode& x = b2[n];
        for (int i = 0; i < 3; i++) out[0].mn[i] = x.lmin[i], out[0].mx[i] = x.lmax[i];
        for (int i = 0; i < 3; i++) out[1].mn[i] = x.rmin[i], out[1].mx[i] = x.rmax[i];
        out[0].ref = x.left, out[0].cnt = x.lcount;
        out[1].ref = x.right, out[1].cnt = x.rcount;
    };
    b4.clear();
    if (b2.empty()) return;
    struct Task {
        int n2, n4;
    };
    std::vector<Task> st{{0, 0}};
    b4.emplace_back();
    while (!st.empty()) {
        const Task t = st.back();
        st.pop_back();
        Slot c[4];
        int m = 2;
        slots_of(t.n2, c);
        while (m < 4) {
            int best = -1;
            for (int i = 0; i < m; i++)
                if (c[i].cnt == 0 && (best < 0 || c[i].area() > c[best].area())) best = i;
            if (best < 0) break;
            Slot two[2];
            slots_of(c[best].ref, two);
            c[best] = two[0];
            c[m++] = two[1];
        }
        Bvh4Node nd{};
        for (int i = 0; i < 4; i++) {
            if (i >= m || c[i].cnt < 0) {
                for (int a = 0; a < 3; a++) nd.ch[i].lo[a] = INFINITY, nd.ch[i].hi[a] = -INFINITY;
                nd.ch[i].ref = 0;
                nd.ch[i].cnt = -1;
                continue;
            }
            for (int a = 0; a < 3; a++) nd.ch[i].lo[a] = c[i].mn[a], nd.ch[i].hi[a] = c[i].mx[a];
            nd.ch[i].cnt = c[i].cnt;
            nd.ch[i].ref = c[i].ref;
        }
        // inner children get consecutive slots; their subtrees follow depth-first
        Task kids[4];
        int nk = 0;
        for (int i = 0; i < 4; i++)
            if (nd.ch[i].cnt == 0) {
                kids[nk++] = {nd.ch[i].ref, (int)b4.size()};
                nd.ch[i].ref = (int)b4.size();
                b4.emplace_back();
            }
        b4[t.n4] = nd;
        for (int i = nk - 1; i >= 0; i--) st.push_back(kids[i]);
    }
}

// Moves the first `k` nodes of a breadth-first walk of the 4-wide tree to the front
// (in that order; the rest keep their depth-first order), so that the levels every
// walk starts with are one contiguous block the kernels can stage in LDS. Returns
// how many nodes that is.
static int bvh4_top_first(std::vector<Bvh4Node>& b4, int k)
{
    const int n = (int)b4.size();
    std::vector<int> bfs;
    bfs.push_back(0);
    for (size_t i = 0; i < bfs.size() && (int)bfs.size() < k; i++)
        for (int c = 0; c < 4 && (int)bfs.size() < k; c++)
            if (b4[bfs[i]].ch[c].cnt == 0) bfs.push_back(b4[bfs[i]].ch[c].ref);
    std::vector<int> to(n, -1);
    int next = 0;
    for (int v : bfs) to[v] = next++;
    for (int v = 0; v < n; v++)
        if (to[v] < 0) to[v] = next++;
    std::vector<Bvh4Node> out(n);
    for (int v = 0; v < n; v++) {
        Bvh4Node nd = b4[v];
        for (auto& c : nd.ch)
            if (c.cnt == 0) c.ref = to[c.ref];
        out[to[v]] = nd;
    }
    b4.swap(out);
    return (int)bfs.size();
}

// The 16-wide form of the 4-wide tree, index for index: 16-wide node i holds 4-wide node
// i's leaf children and the children of its inner children (up to 16; empty slots cnt -1
// with an inverted box), an inner record's ref being the 4-wide node index (= its 16-wide
// node). Any item of a 4-wide walk is an item of a 16-wide walk, so a quad walk's stack can
// be continued by a row (rt_render.hip trace_stream). Boxes and leaves copied unchanged.
static void build_bvh16(const std::vector<Bvh4Node>& b4, std::vector<Bvh4Child>& b16)
{
    Bvh4Child empty{};
    for (int a = 0; a < 3; a++) empty.lo[a] = INFINITY, empty.hi[a] = -INFINITY;
    empty.ref = 0;
    empty.cnt = -1;
    b16.assign(b4.size() * RT_BVH16_W, empty);
    const int n = (int)b4.size();
    const int nw = worker_count();
    parallel_for(nw, nw, [&](int w) {
        for (int i = (int)((long)n * w / nw); i < (int)((long)n * (w + 1) / nw); i++) {
            Bvh4Child* rec = &b16[(size_t)i * RT_BVH16_W];
            int m = 0;
            for (const Bvh4Child& c : b4[i].ch) {
                if (c.cnt < 0) continue;
                if (c.cnt > 0) {
                    rec[m++] = c;
                } else {
                    for (const Bvh4Child& g : b4[c.ref].ch)
                        if (g.cnt >= 0) rec[m++] = g;
                }
            }
        }
    });
}

// f32 <-> f16 bits (round to nearest even; finite inputs of magnitude <= 1 here)
static uint16_t f16_bits(float f)
{
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const int exp = (int)((x >> 23) & 0xff) - 127 + 15;
    uint32_t man = x & 0x7fffffu;
    if (exp <= 0) {  // subnormal half (or zero)
        if (exp < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - exp;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)exp << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

// Oriented slabs of the search BVH's children (rt_fast.h slab_ok): a child's subtree covers a
// contiguous run of bvh_tri4 (the SAH build partitions the triangles in place), whose
// area-weighted mean normal n (when the normals do not cancel: |sum| > half the summed
// areas) quantized to f16 gives the slab {x : lo <= n.x <= hi} over the run's vertices
// a, a + e1, a + e2 (exactly the triangle Moller-Trumbore tests), widened by a margin that
// covers the kernel's f32 evaluation of n.o + t n.d along a ray from the near box (the scene's
// box + 0.5 x its largest extent: queries from farther take the exact walk, rt_fast.h
// far_origin) and the Moller-Trumbore hit's distance from its triangle's plane (DESIGN.md §4:
// ~eps |o - a| off the plane; the margin is 1e-4 of the child's magnitude + 1e-5 of the scene's).
// A ray segment inside the child's box that lies entirely on one side of the slab cannot
// reach a hit there: such children are not entered. Grazing rays above a curved tessellated
// surface enter many boxes but few slabs (the long search-BVH walks, profiles/r05_walk_*).
void build_slabs(FlatBvh& out)
{
    const int nn = (int)out.bvh4.size();
    const int nt = (int)(out.bvh_tri4.size() / 3);
    out.bvh4s.assign((size_t)nn * 4, float4_{0.0f, 0.0f, -INFINITY, INFINITY});
    out.bvh16s.assign((size_t)nn * RT_BVH16_W, float4_{0.0f, 0.0f, -INFINITY, INFINITY});
    if (nn == 0 || nt == 0) return;
    // triangle runs of every node (children's runs are adjacent)
    std::vector<int> lo(nn, INT32_MAX), hi(nn, 0);
    std::vector<int> order;  // post-order
    {
        std::vector<std::pair<int, int>> st{{0, 0}};
        while (!st.empty()) {
            auto& [v, k] = st.back();
            if (k < 4) {
                const Bvh4Child& c = out.bvh4[v].ch[k++];
                if (c.cnt == 0) st.push_back({c.ref, 0});
                continue;
            }
            order.push_back(v);
            st.pop_back();
        }
    }
    for (int v : order)
        for (const Bvh4Child& c : out.bvh4[v].ch) {
            if (c.cnt < 0) continue;
            const int f = c.cnt > 0 ? c.ref : lo[c.ref], l = c.cnt > 0 ? c.ref + c.cnt : hi[c.ref];
            lo[v] = std::min(lo[v], f), hi[v] = std::max(hi[v], l);
        }
    // prefix sums of the (double) normals cross(e1, e2) and their lengths
    std::vector<double> ps((size_t)(nt + 1) * 4, 0.0);
    for (int k = 0; k < nt; k++) {
        const float4_* r = &out.bvh_tri4[3 * (size_t)k];
        const double e1[3] = {r[1].x, r[1].y, r[1].z}, e2[3] = {r[2].x, r[2].y, r[2].z};
        const double cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        for (int a = 0; a < 3; a++) ps[4 * (size_t)(k + 1) + a] = ps[4 * (size_t)k + a] + cr[a];
        ps[4 * (size_t)(k + 1) + 3] = ps[4 * (size_t)k + 3] + std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    }
    float scene_mag = 1.0f;
    for (const Bvh4Child& c : out.bvh4[0].ch)
        if (c.cnt >= 0)
            for (int a = 0; a < 3; a++) scene_mag = std::max(scene_mag, std::max(std::fabs(c.lo[a]), std::fabs(c.hi[a])));
    auto slab_of = [&](const Bvh4Child& c) -> float4_ {
        float4_ s{0.0f, 0.0f, -INFINITY, INFINITY};
        if (c.cnt < 0) return s;
        const int f = c.cnt > 0 ? c.ref : lo[c.ref], l = c.cnt > 0 ? c.ref + c.cnt : hi[c.ref];
        double m[3];
        for (int a = 0; a < 3; a++) m[a] = ps[4 * (size_t)l + a] - ps[4 * (size_t)f + a];
        const double area = ps[4 * (size_t)l + 3] - ps[4 * (size_t)f + 3];
        const double len = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
        if (!(len > 0.5 * area) || !(len > 0.0)) return s;
        uint16_t hb[3];
        double n[3];
        for (int a = 0; a < 3; a++) {
            hb[a] = f16_bits((float)(m[a] / len));
            // the quantized component as the kernel decodes it
            const uint32_t e = (hb[a] >> 10) & 31u, man = hb[a] & 1023u;
            const double mag = e == 0 ? std::ldexp((double)man, -24) : std::ldexp((double)(1024u + man), (int)e - 25);
            n[a] = (hb[a] & 0x8000u) ? -mag : mag;
        }
        double dlo = INFINITY, dhi = -INFINITY;
        for (int k = f; k < l; k++) {
            const float4_* r = &out.bvh_tri4[3 * (size_t)k];
            const double av[3] = {r[0].x, r[0].y, r[0].z};
            const double e1[3] = {r[1].x, r[1].y, r[1].z}, e2[3] = {r[2].x, r[2].y, r[2].z};
            const double p0 = n[0] * av[0] + n[1] * av[1] + n[2] * av[2];
            const double p1 = p0 + n[0] * e1[0] + n[1] * e1[1] + n[2] * e1[2];
            const double p2 = p0 + n[0] * e2[0] + n[1] * e2[1] + n[2] * e2[2];
            dlo = std::min(dlo, std::min(p0, std::min(p1, p2)));
            dhi = std::max(dhi, std::max(p0, std::max(p1, p2)));
        }
        float cmag = 1.0f;
        for (int a = 0; a < 3; a++) cmag = std::max(cmag, std::max(std::fabs(c.lo[a]), std::fabs(c.hi[a])));
        const double margin = 1e-4 * cmag + 1e-5 * scene_mag;
        const uint32_t w0 = (uint32_t)hb[0] | ((uint32_t)hb[1] << 16), w1 = hb[2];
        std::memcpy(&s.x, &w0, 4);
        std::memcpy(&s.y, &w1, 4);
        s.z = (float)(dlo - margin);
        s.w = (float)(dhi + margin);
        // (float rounding of the bounds outwards)
        if ((double)s.z > dlo - margin) s.z = std::nextafter(s.z, -INFINITY);
        if ((double)s.w < dhi + margin) s.w = std::nextafter(s.w, INFINITY);
        return s;
    };
    const int nw = worker_count();
    parallel_for(std::min(nn, 4 * nw), nw, [&](int w) {
        const int W = std::min(nn, 4 * nw);
        for (int i = (int)((long)nn * w / W); i < (int)((long)nn * (w + 1) / W); i++)
            for (int c = 0; c < 4; c++) out.bvh4s[4 * (size_t)i + c] = slab_of(out.bvh4[i].ch[c]);
    });
    // bvh16 order (build_bvh16): node i's leaf children, then its inner children's children
    parallel_for(nw, nw, [&](int w) {
        for (int i = (int)((long)nn * w / nw); i < (int)((long)nn * (w + 1) / nw); i++) {
            float4_* rec = &out.bvh16s[(size_t)i * RT_BVH16_W];
            int m = 0;
            for (int c = 0; c < 4; c++) {
                const Bvh4Child& ch = out.bvh4[i].ch[c];
                if (ch.cnt < 0) continue;
                if (ch.cnt > 0) {
                    rec[m++] = out.bvh4s[4 * (size_t)i + c];
                } else {
                    for (int g = 0; g < 4; g++)
                        if (out.bvh4[ch.ref].ch[g].cnt >= 0) rec[m++] = out.bvh4s[4 * (size_t)ch.ref + g];
                }
            }
        }
    });
}

void build_search_bvh(FlatBvh& out)
{
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!std::getenv("RT_VERBOSE")) return;
        auto T1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[search bvh] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(T1 - T0).count());
        T0 = T1;
    };
    // plane nesting along every parent link (enables rt_fast.h's one-test chain check)
    out.chain_monotone = true;
    for (size_t r = 1; r < out.nodes.size() && out.chain_monotone; r++) {
        const RtNode& c = out.nodes[r];
        const RtNode& p = out.nodes[out.parent[r]];
        for (int i = 0; i < 7; i++)
            if (!(p.dn[i] <= c.dn[i] && p.df[i] >= c.df[i])) out.chain_monotone = false;
    }
    const int n = (int)(out.tri4.size() / 3);
    std::vector<Prim> P(n);
    const int nw = worker_count();
    parallel_for(nw, nw, [&](int w) {
    for (int k = (int)((long)n * w / nw); k < (int)((long)n * (w + 1) / nw); k++) {
        const float4_* r = &out.tri4[3 * (size_t)k];
        const float a[3] = {r[0].x, r[0].y, r[0].z};
        // vertices as the reference's Triangle holds them: b = a + e1, c = a + e2
        // may differ from the originals in the last ulp; pad_box absorbs it.
        const float b[3] = {r[0].x + r[1].x, r[0].y + r[1].y, r[0].z + r[1].z};
        const float c[3] = {r[0].x + r[2].x, r[0].y + r[2].y, r[0].z + r[2].z};
        P[k].b.reset();
        P[k].b.grow(a);
        P[k].b.grow(b);
        P[k].b.grow(c);
        for (int i = 0; i < 3; i++) P[k].c[i] = 0.5f * (P[k].b.mn[i] + P[k].b.mx[i]);
        P[k].k = k;
    }
    });
    lap("chain check + prims");
    SahBuilder B(P, out.bvh);
    B.workers = worker_count();
    if (n > 0) B.run();
    lap("SAH build");
    out.bvh_tri4.resize(3 * (size_t)n);
    parallel_for(nw, nw, [&](int w) {
    for (int i = (int)((long)n * w / nw); i < (int)((long)n * (w + 1) / nw); i++) {
        const int k = P[i].k;
        out.bvh_tri4[3 * (size_t)i] = out.tri4[3 * (size_t)k];
        std::memcpy(&out.bvh_tri4[3 * (size_t)i].w, &k, 4);
        out.bvh_tri4[3 * (size_t)i + 1] = out.tri4[3 * (size_t)k + 1];
        std::memcpy(&out.bvh_tri4[3 * (size_t)i + 1].w, &out.leaf_of[k], 4);  // octree leaf record
        out.bvh_tri4[3 * (size_t)i + 2] = out.tri4[3 * (size_t)k + 2];
        out.bvh_tri4[3 * (size_t)i + 2].w = out.tri4[3 * (size_t)k].w;  // original triangle index (brute-force ties)
    }
    });
    if (out.bvh.empty()) {  // no triangles: a root with two empty slots
        BvhNode r{};
        for (int i = 0; i < 3; i++) r.lmin[i] = r.rmin[i] = INFINITY, r.lmax[i] = r.rmax[i] = -INFINITY;
        r.lcount = r.rcount = -1;
        out.bvh.push_back(r);
    }
    lap("leaf records");
    collapse_bvh4(out.bvh, out.bvh4);
    out.bvh4_ntop = bvh4_top_first(out.bvh4, 256);
    build_bvh16(out.bvh4, out.bvh16);
    lap("collapse");
    build_slabs(out);
    lap("slabs");
}

// ======================================================================= env
void env_cdf_fences(const float* cdf, const float* row_ends, int w, int h, std::vector<float>& out)
{
    out.clear();
    const size_t n = (size_t)w * h;
    if (w % 16 != 0 || w - 1 > 4096 || h - 1 > 4096) return;
    for (size_t i = 0; i < n; i++)
        if (std::isnan(cdf[i]) || (i > 0 && !(cdf[i] >= cdf[i - 1]))) return;
    out.assign((size_t)(1 + h) * 272, INFINITY);
    auto build = [&](const float* a, int m, float* t) {
        for (int j = 0; j < 16; j++)
            if (256 * j + 255 < m) t[j] = a[256 * j + 255];
        for (int j = 0; j < 256; j++)
            if (16 * j + 15 < m) t[16 + j] = a[16 * j + 15];
    };
    build(row_ends, h - 1, out.data());
    for (int y = 0; y < h; y++) build(cdf + (size_t)y * w, w - 1, out.data() + (size_t)(1 + y) * 272);
}

void env_luminance_cdf(const float* pix, int w, int h, int channels, float* lum, float* cdf)
{
    const size_t n = (size_t)w * h;
    for (size_t i = 0; i < n; i++) {
        const float* c = pix + channels * i;
        lum[i] = 0.3086 * c[0] + 0.6094 * c[1] + 0.0820 * c[2];  // image.h:80-85
    }
    if (n == 0) return;
    cdf[0] = 0.0f;
    for (size_t i = 0; i < n; i++) cdf[i] = cdf[i > 0 ? i - 1 : 0] + lum[i];  // utils.cpp:126-142
}

// ==================================================================== camera
namespace {
struct Xf {
    float m[4][4];
};
Xf xf_rows(float a00, float a01, float a02, float a03, float a10, float a11, float a12, float a13, float a20, float a21,
           float a22, float a23, float a30, float a31, float a32, float a33)
{
    return Xf{{{a00, a01, a02, a03}, {a10, a11, a12, a13}, {a20, a21, a22, a23}, {a30, a31, a32, a33}}};
}
Xf compose(const Xf& a, const Xf& b)  // mat.cpp:364-372
{
    Xf m;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            m.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] + a.m[i][3] * b.m[3][j];
    return m;
}
float radians_(float deg) { return ((float)M_PI / 180.f) * deg; }  // mat.cpp:10-13
Xf rotation_x(float a)                                             // mat.cpp:210-220
{
    volatile float r = radians_(a);  // runtime libm call, as the reference makes it
    float s = sinf(r), c = cosf(r);
    return xf_rows(1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1);
}
Xf translation(float x, float y, float z) { return xf_rows(1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1); }
const Xf DEFAULT_CS = xf_rows(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 0, 0, 0, 0, 1);  // camera.cpp:3
}  // namespace

int camera_preset(const std::string& name, float view[16], float* fov_dist)
{
    Xf v;
    float fov_rad;
    const float fov = 45;
    if (name == "default") {  // Camera() (camera.h:18-23)
        v = DEFAULT_CS;
        fov_rad = fov / 180.0f * (float)M_PI;
    } else {
        Xf t;
        if (name == "cornell")
            t = translation(0, 1, 3.5);
        else if (name == "ganesha")
            t = compose(rotation_x(-15), translation(-0.0205, 0.67, 1));
        else if (name == "ite")
            t = compose(rotation_x(-45), translation(0, 0.15, 1.5));
        else if (name == "dragon")
            t = compose(rotation_x(-45), translation(0, -1, 10.5));
        else if (name == "mis")
            t = compose(rotation_x(-10), translation(0, -3, 10.5));
        else
            return -1;
        v = compose(t, DEFAULT_CS);  // Camera(float, Transform) (camera.h:30-36)
        fov_rad = fov / 180.0f * M_PI;
    }
    volatile float half = fov_rad / 2.0f;
    *fov_dist = 1.0f / std::tan((float)half);
    std::memcpy(view, v.m, 64);
    return 0;
}

}  // namespace rt
