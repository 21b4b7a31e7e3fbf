// raygen.hpp — host ray generation and the reference's Ray / RayResult records.
#pragma once
#include <cstdint>
#include <vector>

#include "scene.hpp"

namespace mrt {

// reference src/rt/Util.hh:64-73 — 32 B, the trace reads it as 2 x float4.
struct Ray {
    float ox, oy, oz, tmin;
    float dx, dy, dz, tmax;
};
static_assert(sizeof(Ray) == 32, "Ray must be 32 bytes");

// reference src/rt/Util.hh:79-89 — 16 B; the trace writes {id, t} only.
struct RayResult {
    int32_t id;
    float t;
    int32_t padA;
    int32_t padB;
};
static_assert(sizeof(RayResult) == 16, "RayResult must be 16 bytes");

Mat4f nscreen_to_world(const Camera& cam, int w, int h);
std::vector<int32_t> pixel_table(int w, int h);
void gen_primary_rays(const Camera& cam, int w, int h, Ray* out, int32_t* slotToId, float jx = 0.5f, float jy = 0.5f);
void gen_ao_rays(const Ray* inRays, const RayResult* inResults, int64_t numInput, const Vec3f* triNormals,
                 int64_t numTris, int numSamples, float maxDist, uint32_t seed, Ray* out);
int64_t count_hits(const RayResult* results, int64_t n);

}  // namespace mrt
