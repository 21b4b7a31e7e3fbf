// obj_io.cpp — Wavefront OBJ import into a flattened Scene.
//
// Follows the reference's importer (src/framework/io/MeshWavefrontIO.cc:258-467)
// where it affects the triangle ids the tracer reports: polygons are
// fan-triangulated as (v0, v[i-1], v[i]) (:359-360), indices may be negative
// (relative to the current end of the list), and triangles are grouped per
// material submesh in order of first use, then flattened submesh by submesh
// (reference src/rt/Scene.cc:63-82). Texture coordinates and normals are parsed
// and ignored: the tracer only needs positions.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <array>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "scene.hpp"

namespace mrt {

namespace {

// One face index (reference :317-340): negative = relative to the current end
// of the list; an index outside the list maps to -1 ("no vertex", which the
// reference turns into a vertex at the origin) instead of failing the file.
bool parse_index(const char*& p, int count, int* out) {
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p) return false;
    p = end;
    long idx = (v < 0) ? count + v : v - 1;
    *out = (idx < 0 || idx >= count) ? -1 : (int)idx;
    return true;
}

// loadMtl (reference MeshWavefrontIO.cc:114-200): "newmtl" opens a material
// (diffuse defaults to (0.75, 0.75, 0.75, 1), Mesh.hh:92), "Kd r g b" sets its
// diffuse rgb, "d a" its alpha; the rest (Ka, Ks, Ns, maps) does not reach the
// colour tables and is skipped.
void load_mtl(const std::string& path, std::map<std::string, std::array<float, 4>>& mats) {
    std::ifstream in(path);
    if (!in) return;   // the reference ignores a missing library too
    std::array<float, 4>* cur = nullptr;
    std::string line;
    while (std::getline(in, line)) {
        const char* p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        if (std::strncmp(p, "newmtl ", 7) == 0) {
            std::string name = p + 7;
            name.erase(0, name.find_first_not_of(" \t"));
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ')) name.pop_back();
            cur = &mats.emplace(name, std::array<float, 4>{0.75f, 0.75f, 0.75f, 1.0f}).first->second;
        } else if (cur && std::strncmp(p, "Kd ", 3) == 0) {
            float r, g, b;
            if (std::sscanf(p + 3, "%f %f %f", &r, &g, &b) == 3) { (*cur)[0] = r; (*cur)[1] = g; (*cur)[2] = b; }
        } else if (cur && std::strncmp(p, "d ", 2) == 0) {
            float a;
            if (std::sscanf(p + 2, "%f", &a) == 1) (*cur)[3] = a;
        }
    }
}

}  // namespace

bool load_obj(const std::string& path, Scene& out, std::string* err) {
    std::ifstream in(path);
    if (!in) {
        if (err) *err = "cannot open " + path;
        return false;
    }
    out = Scene();
    out.name = path;
    std::vector<std::vector<Vec3i>> submeshes;
    std::map<std::string, int> materialSubmesh;
    std::map<std::string, std::array<float, 4>> materials;
    const size_t slash = path.find_last_of("/\\");
    const std::string dir = slash == std::string::npos ? std::string(".") : path.substr(0, slash);   // String::getDirName
    // Submesh bookkeeping of the reference (:258-395): faces collect in `pending`
    // and are appended to the current submesh when a usemtl switches away from
    // it (or at the end of the file). A usemtl naming a material of the loaded
    // libraries selects that material's submesh (created on first use); any other
    // name selects none, so the faces that follow join the default submesh (the
    // one created by the first face seen without a material).
    std::map<std::string, int>& matSubmesh = materialSubmesh;
    int current = -1, defaultSubmesh = -1;
    std::vector<Vec3i> pending;
    auto flush = [&]() {
        if (current != -1) submeshes[current].insert(submeshes[current].end(), pending.begin(), pending.end());
        pending.clear();
    };
    int texCount = 0, normalCount = 0;
    std::string line;
    auto trailing_blank = [](const char* p) {
        while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
        return *p == 0;
    };
    while (std::getline(in, line)) {
        const char* p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            // "v x y z" exactly (reference :276-283: a fourth value makes the line invalid, skipped)
            float x, y, z;
            int n = 0;
            if (std::sscanf(p + 2, "%f %f %f%n", &x, &y, &z, &n) == 3 && trailing_blank(p + 2 + n))
                out.vertices.emplace_back(x, y, z);
        } else if (p[0] == 'v' && p[1] == 't') {
            ++texCount;
        } else if (p[0] == 'v' && p[1] == 'n') {
            ++normalCount;
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            p += 2;
            std::vector<int> poly;
            bool ok = true;
            while (*p) {
                while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
                if (!*p) break;
                int vi = 0, dummy = 0;
                if (!parse_index(p, (int)out.vertices.size(), &vi)) { ok = false; break; }
                if (*p == '/') {   // skip /vt and /vn
                    ++p;
                    if (*p != '/' && !parse_index(p, texCount, &dummy)) { ok = false; break; }
                    if (*p == '/') { ++p; if (!parse_index(p, normalCount, &dummy)) { ok = false; break; } }
                }
                poly.push_back(vi);   // -1: resolved to the origin vertex after the last 'v' line
            }
            if (!ok) continue;   // unparsable face: skipped, like the reference's invalid lines
            if (current == -1) {
                if (defaultSubmesh == -1) {
                    defaultSubmesh = (int)submeshes.size();
                    submeshes.emplace_back();
                }
                current = defaultSubmesh;
            }
            for (size_t i = 2; i < poly.size(); i++) pending.push_back(Vec3i{poly[0], poly[i - 1], poly[i]});
        } else if (std::strncmp(p, "mtllib ", 7) == 0) {
            std::string name = p + 7;
            name.erase(0, name.find_first_not_of(" \t"));
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ')) name.pop_back();
            // Resolved against the OBJ's directory (:386-397); a missing library loads nothing.
            if (!name.empty()) load_mtl(dir + "/" + name, materials);
        } else if (std::strncmp(p, "usemtl ", 7) == 0) {
            std::string name = p + 7;
            name.erase(0, name.find_first_not_of(" \t"));
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ')) name.pop_back();
            flush();
            current = -1;
            if (materials.count(name)) {
                auto it = matSubmesh.find(name);
                if (it == matSubmesh.end()) {
                    it = matSubmesh.emplace(name, (int)submeshes.size()).first;
                    submeshes.emplace_back();
                }
                current = it->second;
            }
        }
    }
    flush();
    // Index -1 is the reference's vertex at the origin (:345-347); it is appended
    // after every position, so it does not shift the relative indices above.
    bool needOrigin = false;
    for (auto& sm : submeshes)
        for (auto& t : sm)
            for (int k = 0; k < 3; k++) needOrigin |= t[k] < 0;
    if (needOrigin) {
        const int origin = (int)out.vertices.size();
        out.vertices.emplace_back(0.f, 0.f, 0.f);
        for (auto& sm : submeshes)
            for (auto& t : sm)
                for (int k = 0; k < 3; k++)
                    if (t[k] < 0) t[k] = origin;
    }
    std::vector<std::array<float, 4>> smDiffuse(submeshes.size(), std::array<float, 4>{0.75f, 0.75f, 0.75f, 1.0f});
    bool anyMaterial = false;
    for (const auto& kv : materialSubmesh) {
        auto m = materials.find(kv.first);
        if (m != materials.end()) { smDiffuse[kv.second] = m->second; anyMaterial = true; }
    }
    for (size_t i = 0; i < submeshes.size(); i++) {
        out.triangles.insert(out.triangles.end(), submeshes[i].begin(), submeshes[i].end());
        if (anyMaterial)
            for (size_t k = 0; k < submeshes[i].size(); k++)
                out.triDiffuse.insert(out.triDiffuse.end(), smDiffuse[i].begin(), smDiffuse[i].end());
    }
    out.compute_normals();
    const AABB b = out.bounds();
    const Vec3f c = (b.mn + b.mx) * 0.5f;
    const float r = length(b.mx - b.mn) * 0.5f;
    out.camera.position = c + Vec3f(0.f, 0.f, 2.5f * r);
    out.camera.forward = Vec3f(0.f, 0.f, -1.f);
    out.camera.up = Vec3f(0.f, 1.f, 0.f);
    out.camera.fov = 45.f;
    out.camera.nearDist = 0.001f * r;
    out.camera.farDist = 10.f * r;
    return true;
}

}  // namespace mrt
