// host_api.cpp — the C-ABI of include/mrt_host.h over the host C++ pieces.
#include <cstdio>
#include <cstring>
#include <vector>
#include <exception>
#include <memory>
#include <string>

#include "../../../include/mrt_host.h"
#include "bvh.hpp"
#include "fwhash.hpp"
#include "raygen.hpp"
#include "scene.hpp"

struct mrth_scene {
    mrt::Scene scene;
};
struct mrth_bvh {
    mrt::Compact2 c2;
    mrth_bvh_stats stats{};
};

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
mrt::Vec3f v3(const float* p) { return mrt::Vec3f(p[0], p[1], p[2]); }
}  // namespace

extern "C" {

const char* mrth_last_error(void) { return g_err.c_str(); }

int mrth_scene_synthetic(const char* name, int64_t param, uint64_t seed, mrth_scene** out) {
    if (!name || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    try {
        auto s = std::make_unique<mrth_scene>();
        std::string err;
        if (!mrt::make_synthetic_scene(name, param, seed, s->scene, &err)) return fail(MRTH_ERR_GENERATOR, err);
        *out = s.release();
        return MRTH_OK;
    } catch (const std::exception& e) {
        return fail(MRTH_ERR_GENERATOR, e.what());
    }
}

int mrth_scene_load_obj(const char* path, mrth_scene** out) {
    if (!path || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    auto s = std::make_unique<mrth_scene>();
    std::string err;
    if (!mrt::load_obj(path, s->scene, &err)) return fail(MRTH_ERR_IO, err);
    *out = s.release();
    return MRTH_OK;
}

int mrth_scene_from_arrays(const float* vertices, int64_t nv, const int32_t* tris, int64_t nt, mrth_scene** out) {
    if (!out || nv < 0 || nt < 0 || (nv && !vertices) || (nt && !tris)) return fail(MRTH_ERR_INVALID_ARG, "bad arrays");
    auto s = std::make_unique<mrth_scene>();
    s->scene.name = "arrays";
    s->scene.vertices.resize(nv);
    for (int64_t i = 0; i < nv; i++) s->scene.vertices[i] = v3(vertices + 3 * i);
    s->scene.triangles.resize(nt);
    for (int64_t i = 0; i < nt; i++) {
        for (int k = 0; k < 3; k++)
            if (tris[3 * i + k] < 0 || tris[3 * i + k] >= nv) return fail(MRTH_ERR_INVALID_ARG, "vertex index out of range");
        s->scene.triangles[i] = mrt::Vec3i{tris[3 * i], tris[3 * i + 1], tris[3 * i + 2]};
    }
    s->scene.compute_normals();
    *out = s.release();
    return MRTH_OK;
}

void mrth_scene_destroy(mrth_scene* s) { delete s; }
int64_t mrth_scene_num_triangles(const mrth_scene* s) { return s ? (int64_t)s->scene.triangles.size() : -1; }
int64_t mrth_scene_num_vertices(const mrth_scene* s) { return s ? (int64_t)s->scene.vertices.size() : -1; }

int mrth_scene_copy_arrays(const mrth_scene* s, float* vertices, int32_t* triangles, float* normals) {
    if (!s) return fail(MRTH_ERR_INVALID_ARG, "null scene");
    if (vertices) std::memcpy(vertices, s->scene.vertices.data(), s->scene.vertices.size() * 12);
    if (triangles) std::memcpy(triangles, s->scene.triangles.data(), s->scene.triangles.size() * 12);
    if (normals) std::memcpy(normals, s->scene.triNormals.data(), s->scene.triNormals.size() * 12);
    return MRTH_OK;
}

namespace {
// Vec4f::toABGR, host variant (reference Math.cc:45-52): clamp, scale by 2^56 in
// double, times 255, round half up in fixed point.
uint32_t host_to_abgr(const float v[4]) {
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        const float c = v[i] < 0.0f ? 0.0f : (v[i] > 1.0f ? 1.0f : v[i]);
        const uint64_t q = (uint64_t)((double)c * 72057594037927936.0);   // exp2(56)
        r |= (uint32_t)((((q * 255u) >> 55) + 1) >> 1) << (8 * i);
    }
    return r;
}
}  // namespace

int mrth_scene_tri_colors(const mrth_scene* s, uint32_t* material, uint32_t* shaded) {
    if (!s) return fail(MRTH_ERR_INVALID_ARG, "null scene");
    // Scene::Scene (reference Scene.cc:37,68-80): each triangle's submesh material
    // (OBJ .mtl Kd/d), or the default MeshBase::Material (Mesh.hh:92: diffuse (0.75, 0.75, 0.75, 1)).
    static const float kDefault[4] = {0.75f, 0.75f, 0.75f, 1.0f};
    const mrt::Vec3f light = mrt::normalize(mrt::Vec3f{1.0f, 2.0f, 3.0f});
    const size_t nt = s->scene.triNormals.size();
    const bool perTri = s->scene.triDiffuse.size() == 4 * nt;
    for (size_t i = 0; i < nt; i++) {
        const float* diffuse = perTri ? &s->scene.triDiffuse[4 * i] : kDefault;
        if (material) material[i] = host_to_abgr(diffuse);
        if (shaded) {
            const float k = mrt::dot(s->scene.triNormals[i], light) * 0.5f + 0.5f;
            const float c[4] = {diffuse[0] * k, diffuse[1] * k, diffuse[2] * k, 1.0f};
            shaded[i] = host_to_abgr(c);
        }
    }
    return MRTH_OK;
}

uint32_t mrth_fw_hash_buffer(const void* ptr, int64_t size) {
    return (ptr || size == 0) && size >= 0 ? mrt::fw::hash_buffer(ptr, size) : 0u;
}

uint32_t mrth_scene_hash(const mrth_scene* s) {
    if (!s) return 0;
    // Scene::hash (Scene.cc:93-101) over the five buffers Scene::Scene fills (:37-80).
    const mrt::Scene& sc = s->scene;
    const size_t nt = sc.triangles.size();
    std::vector<uint32_t> material(nt), shaded(nt);
    mrth_scene_tri_colors(s, material.data(), shaded.data());
    using mrt::fw::hash_buffer;
    static_assert(sizeof(mrt::Vec3i) == 12 && sizeof(mrt::Vec3f) == 12, "Scene buffers are packed 12-byte records");
    return mrt::fw::hash_bits6(hash_buffer(sc.triangles.data(), (int64_t)nt * 12),
                               hash_buffer(sc.triNormals.data(), (int64_t)sc.triNormals.size() * 12),
                               hash_buffer(material.data(), (int64_t)nt * 4), hash_buffer(shaded.data(), (int64_t)nt * 4),
                               hash_buffer(sc.vertices.data(), (int64_t)sc.vertices.size() * 12));
}

int mrth_bvh_cache_name(const mrth_scene* s, const mrth_build_params* p, char out[16]) {
    if (!s || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    mrth_build_params d;
    mrth_default_build_params(&d);
    if (!p) p = &d;
    using namespace mrt::fw;
    // Platform("GPU") with setLeafPreferences(min, max) (Renderer.cc:53-54; Platform.hh:43,69):
    // hashBits(hash<String>(name), costs, hashBits(triBatch 1, nodeBatch 1, minLeaf, maxLeaf)).
    const uint32_t platform = hash_bits6(hash_buffer("GPU", 3), float_bits(p->sah_node_cost),
                                         float_bits(p->sah_triangle_cost),
                                         hash_bits6(1u, 1u, (uint32_t)p->min_leaf_size, (uint32_t)p->max_leaf_size));
    const uint32_t params = hash_bits(float_bits(p->split_alpha));   // BVH::BuildParams::computeHash (BVH.hh:82-85)
    const uint32_t kLayoutCompact2 = 5;                              // BVHLayout_Compact2 (CudaTracerKernels.hh:124)
    const uint32_t h = hash_bits6(mrth_scene_hash(s), platform, params, kLayoutCompact2);
    std::snprintf(out, 16, "%08x.dat", h);   // Renderer.cc:180
    return MRTH_OK;
}

int mrth_scene_camera(const mrth_scene* s, mrth_camera* cam, float* aoRadius) {
    if (!s || !cam) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    const mrt::Camera& c = s->scene.camera;
    for (int i = 0; i < 3; i++) {
        cam->position[i] = c.position[i];
        cam->forward[i] = c.forward[i];
        cam->up[i] = c.up[i];
    }
    cam->fov_deg = c.fov;
    cam->near_dist = c.nearDist;
    cam->far_dist = c.farDist;
    if (aoRadius) *aoRadius = s->scene.aoRadius;
    return MRTH_OK;
}

void mrth_default_build_params(mrth_build_params* p) {
    if (!p) return;
    const mrt::BuildParams d;
    p->sah_node_cost = d.sahNodeCost;
    p->sah_triangle_cost = d.sahTriangleCost;
    p->min_leaf_size = d.minLeafSize;
    p->max_leaf_size = d.maxLeafSize;
    p->split_alpha = d.splitAlpha;
    p->threads = 0;
}

int mrth_bvh_build(const mrth_scene* s, const mrth_build_params* p, mrth_bvh** out) {
    if (!s || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    mrt::BuildParams bp;
    if (p) {
        bp.sahNodeCost = p->sah_node_cost;
        bp.sahTriangleCost = p->sah_triangle_cost;
        bp.minLeafSize = p->min_leaf_size;
        bp.maxLeafSize = p->max_leaf_size;
        bp.splitAlpha = p->split_alpha;
        bp.threads = p->threads;
        if (bp.minLeafSize < 1 || bp.maxLeafSize < bp.minLeafSize) return fail(MRTH_ERR_INVALID_ARG, "bad leaf sizes");
    }
    try {
        auto b = std::make_unique<mrth_bvh>();
        mrt::BvhStats st;
        std::unique_ptr<mrt::BvhNode> root = mrt::build_sbvh(s->scene, bp, &st);
        mrt::create_compact2(*root, s->scene, b->c2);
        b->stats.inner_nodes = st.innerNodes;
        b->stats.leaf_nodes = st.leafNodes;
        b->stats.tri_refs = st.triRefs;
        b->stats.max_depth = st.maxDepth;
        b->stats.sah_cost = st.sahCost;
        b->stats.build_seconds = st.buildSeconds;
        *out = b.release();
        return MRTH_OK;
    } catch (const std::exception& e) {
        return fail(MRTH_ERR_GENERATOR, std::string("build failed: ") + e.what());
    }
}

int mrth_bvh_load(const char* path, mrth_bvh** out) {
    if (!path || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    auto b = std::make_unique<mrth_bvh>();
    std::string err;
    if (!mrt::load_dat(path, b->c2, &err)) return fail(MRTH_ERR_IO, err);
    b->stats.inner_nodes = (int64_t)b->c2.nodes.size() / 16;
    *out = b.release();
    return MRTH_OK;
}

int mrth_bvh_save(const mrth_bvh* b, const char* path) {
    if (!b || !path) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    std::string err;
    if (!mrt::save_dat(path, b->c2, &err)) return fail(MRTH_ERR_IO, err);
    return MRTH_OK;
}

int mrth_bvh_from_buffers(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes,
                          const int32_t* triIndex, int64_t triIndexBytes, mrth_bvh** out) {
    if (!out || !nodes || !woop || !triIndex || nodeBytes % 64 || woopBytes % 16 || triIndexBytes % 4)
        return fail(MRTH_ERR_INVALID_ARG, "bad Compact2 buffers");
    auto b = std::make_unique<mrth_bvh>();
    b->c2.nodes.resize(nodeBytes / 4);
    b->c2.woop.resize(woopBytes / 4);
    b->c2.triIndex.resize(triIndexBytes / 4);
    std::memcpy(b->c2.nodes.data(), nodes, nodeBytes);
    std::memcpy(b->c2.woop.data(), woop, woopBytes);
    std::memcpy(b->c2.triIndex.data(), triIndex, triIndexBytes);
    b->stats.inner_nodes = nodeBytes / 64;
    *out = b.release();
    return MRTH_OK;
}

void mrth_bvh_destroy(mrth_bvh* b) { delete b; }

int mrth_bvh_buffers(const mrth_bvh* b, const void** nodes, int64_t* nodeBytes, const void** woop,
                     int64_t* woopBytes, const int32_t** triIndex, int64_t* triIndexBytes) {
    if (!b) return fail(MRTH_ERR_INVALID_ARG, "null bvh");
    if (nodes) *nodes = b->c2.nodes.data();
    if (nodeBytes) *nodeBytes = b->c2.node_bytes();
    if (woop) *woop = b->c2.woop.data();
    if (woopBytes) *woopBytes = b->c2.woop_bytes();
    if (triIndex) *triIndex = b->c2.triIndex.data();
    if (triIndexBytes) *triIndexBytes = b->c2.tri_index_bytes();
    return MRTH_OK;
}

int mrth_bvh_get_stats(const mrth_bvh* b, mrth_bvh_stats* out) {
    if (!b || !out) return fail(MRTH_ERR_INVALID_ARG, "null argument");
    *out = b->stats;
    return MRTH_OK;
}

void mrth_woopify(const float v0[3], const float v1[3], const float v2[3], float out[12]) {
    mrt::Vec4f w[3];
    mrt::woopify(v3(v0), v3(v1), v3(v2), w);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) out[r * 4 + c] = w[r][c];
}

int mrth_pixel_table(int32_t w, int32_t h, int32_t* indexToPixel) {
    if (w <= 0 || h <= 0 || !indexToPixel) return fail(MRTH_ERR_INVALID_ARG, "bad size");
    const std::vector<int32_t> t = mrt::pixel_table(w, h);
    std::memcpy(indexToPixel, t.data(), t.size() * 4);
    return MRTH_OK;
}

static mrt::Camera to_camera(const mrth_camera* cam) {
    mrt::Camera c;
    c.position = v3(cam->position);
    c.forward = v3(cam->forward);
    c.up = v3(cam->up);
    c.fov = cam->fov_deg;
    c.nearDist = cam->near_dist;
    c.farDist = cam->far_dist;
    return c;
}

int mrth_primary_rays(const mrth_camera* cam, int32_t w, int32_t h, void* rays, int32_t* slotToId) {
    if (!cam || w <= 0 || h <= 0 || !rays) return fail(MRTH_ERR_INVALID_ARG, "bad arguments");
    mrt::gen_primary_rays(to_camera(cam), w, h, static_cast<mrt::Ray*>(rays), slotToId);
    return MRTH_OK;
}

int mrth_primary_rays_subpixel(const mrth_camera* cam, int32_t w, int32_t h, float jx, float jy, void* rays,
                               int32_t* slotToId) {
    if (!cam || w <= 0 || h <= 0 || !rays) return fail(MRTH_ERR_INVALID_ARG, "bad arguments");
    if (!(jx >= 0.0f && jx < 1.0f && jy >= 0.0f && jy < 1.0f)) return fail(MRTH_ERR_INVALID_ARG, "subpixel offset outside [0, 1)");
    mrt::gen_primary_rays(to_camera(cam), w, h, static_cast<mrt::Ray*>(rays), slotToId, jx, jy);
    return MRTH_OK;
}

int mrth_camera_decode_signature(const char* sig, mrth_camera* cam, float* speed, int32_t* keepAligned) {
    if (!sig || !cam) return fail(MRTH_ERR_INVALID_ARG, "bad arguments");
    mrt::CameraSignature c;
    if (!mrt::decode_camera_signature(sig, &c)) return fail(MRTH_ERR_INVALID_ARG, "CameraControls: Invalid signature!");
    for (int i = 0; i < 3; i++) {
        cam->position[i] = c.position[i];
        cam->forward[i] = c.forward[i];
        cam->up[i] = c.up[i];
    }
    cam->fov_deg = c.fov;
    cam->near_dist = c.nearDist;
    cam->far_dist = c.farDist;
    if (speed) *speed = c.speed;
    if (keepAligned) *keepAligned = c.keepAligned ? 1 : 0;
    return MRTH_OK;
}

int mrth_camera_nscreen_to_world(const mrth_camera* cam, int32_t w, int32_t h, float out[16]) {
    if (!cam || w <= 0 || h <= 0 || !out) return fail(MRTH_ERR_INVALID_ARG, "bad arguments");
    const mrt::Mat4f m = mrt::nscreen_to_world(to_camera(cam), w, h);
    for (int i = 0; i < 16; i++) out[i] = m.m[i];
    return MRTH_OK;
}

int mrth_ao_rays(const void* primaryRays, const void* primaryResults, int64_t numPrimary, const mrth_scene* s,
                 int32_t numSamples, float maxDist, uint32_t seed, void* outRays) {
    if (!primaryRays || !primaryResults || !s || !outRays || numPrimary < 0 || numSamples < 1)
        return fail(MRTH_ERR_INVALID_ARG, "bad arguments");
    mrt::gen_ao_rays(static_cast<const mrt::Ray*>(primaryRays), static_cast<const mrt::RayResult*>(primaryResults),
                     numPrimary, s->scene.triNormals.data(), (int64_t)s->scene.triNormals.size(), numSamples, maxDist,
                     seed, static_cast<mrt::Ray*>(outRays));
    return MRTH_OK;
}

int64_t mrth_count_hits(const void* results, int64_t n) {
    if (!results || n < 0) return -1;
    return mrt::count_hits(static_cast<const mrt::RayResult*>(results), n);
}

}  // extern "C"
