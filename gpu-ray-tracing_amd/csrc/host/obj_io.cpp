// obj_io.cpp — Wavefront OBJ (+ MTL) import into a flattened Scene.
//
// Restates the reference importer (src/framework/io/MeshWavefrontIO.cc:97-467)
// wherever it decides the Scene's bytes, because those bytes decide the BVH, the
// triangle ids the tracer reports and the bvhcache file name (Scene::hash,
// Scene.cc:93-101):
//   * lines as BufferedInputStream::readLine(true, true) returns them (Stream.cc:89-144):
//     '\r' dropped, tabs turned into spaces, a trailing backslash joins the next line;
//   * numbers through the framework's own parsers (String.cc:396-509): parseFloat
//     accumulates digits in float32 (v*10 + d, then scale *= 0.1f; v += scale*d, then
//     v *= powf(10, e)), which is not strtof — vertex bits follow the reference's;
//   * "v x y z" with exactly three values, "vt" with at least two, "vn" with exactly three
//     (other forms are invalid lines, skipped, and take no index);
//   * face corners "p[/t[/n]]": indices relative to the lists read so far (negative from
//     the end, 0 or out of range = none), one mesh vertex per distinct (p, t, n) triple in
//     order of first use (the reference's vertexHash, :317-348) at position p (or the origin);
//     polygons fan-triangulated (v0, v[i-1], v[i]) (:359-360); a corner that does not parse
//     invalidates the face, but the corners before it still made their vertices;
//   * submeshes: faces collect until a "usemtl" switches away; a usemtl naming a loaded
//     material selects that material's submesh (created on first use), any other name
//     selects none, so following faces join the default submesh (:350-384);
//   * "mtllib" resolved against the OBJ's directory (String::getDirName: "." when none);
//     "newmtl" of an existing name keeps the current material (:131-138); Kd writes the
//     values it parsed even when the line is invalid (parseFloats writes as it goes).
// Texture maps abort the reference (fail("parseTexture shouldn't be called")); here they
// are ignored. Texture coordinates and normals only number vertices: the tracer needs
// positions.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <array>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "scene.hpp"

namespace mrt {

namespace {

// ---- BufferedInputStream::readLine(combineWithBackslash, normalizeWhitespace) ----
class LineReader {
public:
    explicit LineReader(std::istream& in) : in_(in) {}
    bool next(std::string& out) {
        out.clear();
        int c = in_.get();
        if (c == EOF) return false;
        bool pendingBackslash = false;
        for (;; c = in_.get()) {
            if (c == EOF) {
                if (pendingBackslash) out.push_back('\\');
                break;
            }
            const unsigned char chr = (unsigned char)c;
            if (chr >= 32 && chr != '\\' && !pendingBackslash) {
                out.push_back((char)chr);
            } else if (chr == '\n') {
                if (!pendingBackslash) break;
                out.push_back(' ');
                pendingBackslash = false;
            } else if (chr != '\r') {
                if (pendingBackslash) {
                    out.push_back('\\');
                    pendingBackslash = false;
                }
                if (chr == '\t') out.push_back(' ');
                else if (chr == '\\') pendingBackslash = true;
                else out.push_back((char)chr);
            }
        }
        return true;
    }

private:
    std::istream& in_;
};

// ---- the framework's parsers (String.cc:356-509, MeshWavefrontIO.cc:97-110) ----
void parse_space(const char*& p) {
    while (*p == ' ' || *p == '\t') p++;
}

bool parse_char(const char*& p, char c) {
    if (*p != c) return false;
    p++;
    return true;
}

bool parse_literal(const char*& p, const char* s) {
    const char* t = p;
    while (*s && *t == *s) {
        t++;
        s++;
    }
    if (*s) return false;
    p = t;
    return true;
}

bool parse_int(const char*& p, int32_t& value) {
    const char* t = p;
    int32_t v = 0;
    const bool neg = !parse_char(t, '+') && parse_char(t, '-');
    if (*t < '0' || *t > '9') return false;
    while (*t >= '0' && *t <= '9') v = (int32_t)((uint32_t)v * 10u + (uint32_t)(*t++ - '0'));
    value = neg ? -v : v;
    p = t;
    return true;
}

bool parse_float(const char*& p, float& value) {
    const char* t = p;
    const bool neg = !parse_char(t, '+') && parse_char(t, '-');
    float v = 0.0f;
    int digits = 0;
    while (*t >= '0' && *t <= '9') {
        v = v * 10.0f + (float)(*t++ - '0');
        digits++;
    }
    if (parse_char(t, '.')) {
        float scale = 1.0f;
        while (*t >= '0' && *t <= '9') {
            scale *= 0.1f;
            v += scale * (float)(*t++ - '0');
            digits++;
        }
    }
    if (!digits) return false;
    p = t;
    if (*p == '#') {
        uint32_t bits = 0;
        if (parse_literal(p, "#INF")) bits = neg ? 0xFF800000u : 0x7F800000u;
        else if (parse_literal(p, "#SNAN")) bits = neg ? 0xFF800001u : 0x7F800001u;
        else if (parse_literal(p, "#QNAN")) bits = neg ? 0xFFC00001u : 0x7FC00001u;
        else if (parse_literal(p, "#IND")) bits = neg ? 0xFFC00000u : 0x7FC00000u;
        if (bits) {
            std::memcpy(&value, &bits, 4);
            return true;
        }
    }
    int32_t e = 0;
    if ((parse_char(t, 'e') || parse_char(t, 'E')) && parse_int(t, e)) {
        p = t;
        if (e) v *= powf(10.0f, (float)e);
    }
    value = neg ? -v : v;
    return true;
}

bool parse_floats(const char*& p, float* values, int num) {   // writes as it goes, like the reference
    const char* t = p;
    for (int i = 0; i < num; i++) {
        if (i) parse_space(t);
        if (!parse_float(t, values[i])) return false;
    }
    p = t;
    return true;
}

// ---- loadMtl (MeshWavefrontIO.cc:114-250): the fields that reach Scene's colour tables ----
using Material = std::array<float, 4>;   // diffuse rgba; default (0.75, 0.75, 0.75, 1) (Mesh.hh)

void load_mtl(const std::string& path, std::map<std::string, Material>& mats) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return;   // FileRO error: nothing loaded (the reference clears the error too)
    LineReader lines(in);
    std::string line;
    Material* mat = nullptr;
    while (lines.next(line)) {
        const char* p = line.c_str();
        parse_space(p);
        if (!*p || parse_literal(p, "#")) continue;
        if (parse_literal(p, "newmtl ")) {
            parse_space(p);
            if (*p && !mats.count(p)) mat = &mats.emplace(p, Material{0.75f, 0.75f, 0.75f, 1.0f}).first->second;
        } else if (!mat) {
            continue;
        } else if (parse_literal(p, "Kd ")) {
            parse_space(p);
            if (!parse_literal(p, "spectral ") && !parse_literal(p, "xyz ")) parse_floats(p, mat->data(), 3);
        } else if (parse_literal(p, "d ")) {
            parse_space(p);
            parse_float(p, (*mat)[3]);
        }
    }
}

struct PtnHash {
    size_t operator()(const std::array<int32_t, 3>& k) const {
        return ((size_t)(uint32_t)k[0] * 0x9E3779B97F4A7C15ull) ^ ((size_t)(uint32_t)k[1] << 21) ^
               ((size_t)(uint32_t)k[2] * 0xC2B2AE3D27D4EB4Full);
    }
};

}  // namespace

bool load_obj(const std::string& path, Scene& out, std::string* err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        if (err) *err = "cannot open " + path;
        return false;
    }
    out = Scene();
    out.name = path;
    const size_t slash = path.find_last_of("/\\");
    const std::string dir = slash == std::string::npos ? std::string(".") : path.substr(0, slash);   // getDirName

    std::vector<Vec3f> positions;
    int32_t texCount = 0, normalCount = 0;
    std::unordered_map<std::array<int32_t, 3>, int32_t, PtnHash> vertexHash;
    std::vector<std::vector<Vec3i>> submeshes;
    std::map<std::string, int> materialSubmesh;
    std::map<std::string, Material> materials;
    int current = -1, defaultSubmesh = -1;
    std::vector<Vec3i> pending;   // the reference's indexTmp
    auto flush = [&]() {
        if (current != -1) submeshes[current].insert(submeshes[current].end(), pending.begin(), pending.end());
        pending.clear();
    };
    std::vector<int32_t> corners;

    LineReader lines(in);
    std::string line;
    while (lines.next(line)) {
        const char* p = line.c_str();
        parse_space(p);
        if (!*p || parse_literal(p, "#")) continue;
        if (parse_literal(p, "v ")) {
            parse_space(p);
            float v[3];
            if (parse_floats(p, v, 3)) {
                parse_space(p);
                if (!*p) positions.emplace_back(v[0], v[1], v[2]);
            }
        } else if (parse_literal(p, "vt ")) {
            parse_space(p);
            float v[2], dummy;
            if (parse_floats(p, v, 2)) {
                parse_space(p);
                while (parse_float(p, dummy)) parse_space(p);
                if (!*p) texCount++;
            }
        } else if (parse_literal(p, "vn ")) {
            parse_space(p);
            float v[3];
            if (parse_floats(p, v, 3)) {
                parse_space(p);
                if (!*p) normalCount++;
            }
        } else if (parse_literal(p, "f ")) {
            parse_space(p);
            corners.clear();
            while (*p) {
                std::array<int32_t, 3> ptn{0, 0, 0};
                if (!parse_int(p, ptn[0])) break;
                for (int i = 1; i < 4 && parse_literal(p, "/"); i++) {
                    int32_t tmp = 0;
                    parse_int(p, tmp);
                    if (i < 3) ptn[i] = tmp;
                }
                parse_space(p);
                const int32_t size[3] = {(int32_t)positions.size(), texCount, normalCount};
                for (int i = 0; i < 3; i++) {
                    if (ptn[i] < 0) ptn[i] += size[i];
                    else ptn[i]--;
                    if (ptn[i] < 0 || ptn[i] >= size[i]) ptn[i] = -1;
                }
                auto it = vertexHash.find(ptn);
                if (it == vertexHash.end()) {
                    it = vertexHash.emplace(ptn, (int32_t)out.vertices.size()).first;
                    out.vertices.push_back(ptn[0] == -1 ? Vec3f(0.0f) : positions[ptn[0]]);
                }
                corners.push_back(it->second);
            }
            if (!*p) {
                if (current == -1) {
                    if (defaultSubmesh == -1) {
                        defaultSubmesh = (int)submeshes.size();
                        submeshes.emplace_back();
                    }
                    current = defaultSubmesh;
                }
                for (size_t i = 2; i < corners.size(); i++) pending.push_back(Vec3i{corners[0], corners[i - 1], corners[i]});
            }
        } else if (parse_literal(p, "usemtl ")) {
            parse_space(p);
            flush();
            current = -1;
            if (materials.count(p)) {
                auto it = materialSubmesh.find(p);
                if (it == materialSubmesh.end()) {
                    it = materialSubmesh.emplace(p, (int)submeshes.size()).first;
                    submeshes.emplace_back();
                }
                current = it->second;
            }
        } else if (parse_literal(p, "mtllib ")) {
            parse_space(p);
            if (*p) load_mtl(dir + "/" + p, materials);
        }
    }
    flush();

    std::vector<Material> smDiffuse(submeshes.size(), Material{0.75f, 0.75f, 0.75f, 1.0f});
    bool anyMaterial = false;
    for (const auto& kv : materialSubmesh) {
        smDiffuse[kv.second] = materials[kv.first];
        anyMaterial = true;
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
