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

bool parse_index(const char*& p, int count, int* out) {
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p) return false;
    p = end;
    long idx = (v < 0) ? count + v : v - 1;
    if (idx < 0 || idx >= count) return false;
    *out = (int)idx;
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
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? std::string(".") : path.substr(0, slash);
    int current = -1, defaultSubmesh = -1;
    int texCount = 0, normalCount = 0;
    std::string line;
    long lineNo = 0;
    while (std::getline(in, line)) {
        ++lineNo;
        const char* p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            float x, y, z;
            if (std::sscanf(p + 2, "%f %f %f", &x, &y, &z) != 3) goto bad;
            out.vertices.emplace_back(x, y, z);
        } else if (p[0] == 'v' && p[1] == 't') {
            ++texCount;
        } else if (p[0] == 'v' && p[1] == 'n') {
            ++normalCount;
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            p += 2;
            std::vector<int> poly;
            while (*p) {
                while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
                if (!*p) break;
                int vi = 0;
                if (!parse_index(p, (int)out.vertices.size(), &vi)) goto bad;
                if (*p == '/') {   // skip /vt and /vn
                    ++p;
                    if (*p != '/') { int dummy; if (!parse_index(p, texCount, &dummy)) goto bad; }
                    if (*p == '/') { ++p; int dummy; if (!parse_index(p, normalCount, &dummy)) goto bad; }
                }
                poly.push_back(vi);
            }
            if (poly.size() < 3) continue;
            if (current == -1) {
                if (defaultSubmesh == -1) {
                    defaultSubmesh = (int)submeshes.size();
                    submeshes.emplace_back();
                }
                current = defaultSubmesh;
            }
            for (size_t i = 2; i < poly.size(); i++) submeshes[current].push_back(Vec3i{poly[0], poly[i - 1], poly[i]});
        } else if (std::strncmp(p, "mtllib ", 7) == 0) {
            std::string name = p + 7;
            name.erase(0, name.find_first_not_of(" \t"));
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ')) name.pop_back();
            if (!name.empty()) load_mtl(dir + "/" + name, materials);
        } else if (std::strncmp(p, "usemtl", 6) == 0) {
            std::string name = p + 6;
            name.erase(0, name.find_first_not_of(" \t"));
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ')) name.pop_back();
            auto it = materialSubmesh.find(name);
            if (it == materialSubmesh.end()) {
                it = materialSubmesh.emplace(name, (int)submeshes.size()).first;
                submeshes.emplace_back();
            }
            current = it->second;
        }
        continue;
    bad:
        if (err) *err = path + ":" + std::to_string(lineNo) + ": malformed line";
        return false;
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
