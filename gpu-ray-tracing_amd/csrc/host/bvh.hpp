// bvh.hpp — SBVH build (restating the reference SplitBVHBuilder) and the
// Compact2 GPU layout (restating CudaBVH::createCompact / woopifyTri), plus
// the reference's bvhcache .dat stream format.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "scene.hpp"

namespace mrt {

// Build parameters: reference Platform("GPU") with setLeafPreferences(1, 8)
// (Renderer.cc:53-54, Platform.hh:38-79) and BVH::BuildParams splitAlpha 1e-5
// (BVH.hh:70-90).
struct BuildParams {
    float sahNodeCost = 1.0f;
    float sahTriangleCost = 1.0f;
    int nodeBatchSize = 1;
    int triBatchSize = 1;
    int minLeafSize = 1;
    int maxLeafSize = 8;
    float splitAlpha = 1.0e-5f;
    int threads = 0;          // 0 = hardware concurrency; the output does not depend on it
};

struct BvhNode {
    AABB bounds;
    std::unique_ptr<BvhNode> child[2];   // both null for a leaf
    std::vector<int32_t> tris;           // leaf triangle ids, in reference order
    bool is_leaf() const { return !child[0]; }
};

struct BvhStats {
    int64_t innerNodes = 0;
    int64_t leafNodes = 0;
    int64_t triRefs = 0;       // triangle references in leaves (>= tris with spatial splits)
    int64_t maxDepth = 0;
    float sahCost = 0.0f;
    double buildSeconds = 0.0;
};

// SplitBVHBuilder::run (SplitBVHBuilder.cc:55-100). Deterministic: the result
// is independent of the number of threads.
std::unique_ptr<BvhNode> build_sbvh(const Scene& scene, const BuildParams& params, BvhStats* stats);

// BVHLayout_Compact2 buffers (CudaBVH.hh:40-55).
struct Compact2 {
    std::vector<int32_t> nodes;      // 16 ints (64 B) per inner node
    std::vector<int32_t> woop;       // 4 ints per float4 slot
    std::vector<int32_t> triIndex;   // 1 int per woop float4 slot
    int64_t node_bytes() const { return (int64_t)nodes.size() * 4; }
    int64_t woop_bytes() const { return (int64_t)woop.size() * 4; }
    int64_t tri_index_bytes() const { return (int64_t)triIndex.size() * 4; }
};

// CudaBVH::createCompact(bvh, 16) (CudaBVH.cc:270-357). A root that is a leaf
// (scenes of at most maxLeafSize triangles) is wrapped in an inner node whose
// second child is an empty leaf — the reference asserted instead (:289).
void create_compact2(const BvhNode& root, const Scene& scene, Compact2& out);

// CudaBVH::woopifyTri (CudaBVH.cc:361-380): rows Z, U, V of the inverse of
// [v0-v2, v1-v2, cross(v0-v2, v1-v2), v2].
void woopify(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, Vec4f out[3]);

// bvhcache .dat: S32 layout, then per buffer S64 byte count + bytes, little
// endian (CudaBVH.cc:79-97,113-116; Buffer.cc:327-360). Layout 5 = Compact2.
bool save_dat(const std::string& path, const Compact2& c, std::string* err);
bool load_dat(const std::string& path, Compact2& c, std::string* err);

constexpr int32_t kLayoutCompact2 = 5;

}  // namespace mrt
