// scene.hpp — flattened triangle scene (reference src/rt/Scene.{hh,cc}:35-101)
// plus the deterministic synthetic stand-ins for the README scenes (the real
// OBJ assets are not in this environment).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "math.hpp"

namespace mrt {

struct Vec3i {
    int32_t x = 0, y = 0, z = 0;
    int32_t operator[](int i) const { return (&x)[i]; }
    int32_t& operator[](int i) { return (&x)[i]; }
};

struct Camera {
    Vec3f position;
    Vec3f forward;   // view direction (camera looks down -z of its frame along this)
    Vec3f up;
    float fov = 45.0f;   // vertical field of view, degrees (CameraControls m_fov)
    float nearDist = 0.001f;
    float farDist = 3.0f;
};

struct Scene {
    std::string name;
    std::vector<Vec3f> vertices;      // getVtxPosBuffer
    std::vector<Vec3i> triangles;     // getTriVtxIndexBuffer
    std::vector<Vec3f> triNormals;    // getTriNormalBuffer (unit face normals)
    std::vector<float> triDiffuse;    // 4 per triangle: its submesh's Material::diffuse (empty = default 0.75 grey)
    Camera camera;                    // a framing camera for the benchmark
    float aoRadius = 5.0f;            // --ao-radius used with this scene

    int num_triangles() const { return (int)triangles.size(); }
    int num_vertices() const { return (int)vertices.size(); }
    void compute_normals();           // Scene.cc:63-82 (cross of the two edges, normalized)
    AABB bounds() const;
};

// Synthetic generators. `name` is one of: "mori", "bunny", "conference",
// "sponza", "hairball", "sphere" (param = subdivision), "random" (param = tris).
// The README scenes hit their published triangle counts exactly.
bool make_synthetic_scene(const std::string& name, int64_t param, uint64_t seed, Scene& out, std::string* err);

// Wavefront OBJ import (reference src/framework/io/MeshWavefrontIO.cc:258-467):
// fan triangulation of polygons, negative (relative) indices, v/vt/vn forms.
bool load_obj(const std::string& path, Scene& out, std::string* err);

// Published triangle counts of the README scenes (README.md:48-58).
int64_t published_triangle_count(const std::string& name);

}  // namespace mrt
