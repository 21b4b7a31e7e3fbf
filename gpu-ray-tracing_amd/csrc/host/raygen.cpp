// raygen.cpp — camera matrices, the Morton-swizzled pixel table and the
// primary / AO / diffuse ray generators, on the host.
//
// Restates (with IEEE host arithmetic instead of the reference's
// --use_fast_math device code, so results agree statistically, not bitwise;
// the per-ray arithmetic lives in ../raygen_common.hpp, shared with the gfx950
// generators of csrc/raygen_kernel.hip):
//   camera      CameraControls::getOrientation/getWorldToCamera (CameraControls.cc:263-296),
//               Mat4f::perspective / fitToView (Math.cc:66-93),
//               nscreenToWorld = invert(fitToView(-1, 2, size) * worldToClip) (Renderer.cc:126-129)
//   pixels      PixelTable::recalculate (PixelTable.cc:70-161): 8x8 blocks in Morton order,
//               pixels swizzled inside each block, then the bottom and right remainder stripes
//   primary     rayGenPrimaryKernel (RayGenKernels.cu:79-113)
//   AO/diffuse  rayGenAOKernel (RayGenKernels.cu:117-227): back off 1e-4 along the primary ray,
//               normal flipped toward the viewer, Halton(2,3) sample rotated by a Jenkins-hash
//               angle per ray, tmax = -1 for primary misses (degenerate rays)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "raygen.hpp"
#include "../raygen_common.hpp"

namespace mrt {

namespace {

constexpr float kPiF = 3.14159265358979323846f;

Mat4f world_to_camera(const Camera& c) {   // CameraControls.cc:263-296
    const Vec3f col2 = -normalize(c.forward);
    const Vec3f col0 = normalize(cross(c.up, col2));
    const Vec3f col1 = normalize(cross(col2, col0));
    const Vec3f pos(dot(col0, c.position), dot(col1, c.position), dot(col2, c.position));   // orient^T * position
    Mat4f r;
    r.set_row(0, Vec4f(col0, -pos.x));
    r.set_row(1, Vec4f(col1, -pos.y));
    r.set_row(2, Vec4f(col2, -pos.z));
    return r;
}

Mat4f perspective(float fov, float nearDist, float farDist) {   // Math.cc:79-93
    const float f = fw_rcp(std::tan(fov * kPiF / 360.0f));
    const float d = fw_rcp(nearDist - farDist);
    Mat4f r;
    r.set_row(0, Vec4f(f, 0.0f, 0.0f, 0.0f));
    r.set_row(1, Vec4f(0.0f, f, 0.0f, 0.0f));
    r.set_row(2, Vec4f(0.0f, 0.0f, (nearDist + farDist) * d, 2.0f * nearDist * farDist * d));
    r.set_row(3, Vec4f(0.0f, 0.0f, -1.0f, 0.0f));
    return r;
}

Mat4f fit_to_view(float w, float h) {   // Math.cc:66-75 with pos = -1, size = 2
    const float s = fw_min(w / 2.0f, h / 2.0f);
    return Mat4f::scale(Vec3f(2.0f / w, 2.0f / h, 1.0f)) * Mat4f::scale(Vec3f(s, s, 1.0f)) *
           Mat4f::translate(Vec3f(0.0f, 0.0f, 0.0f));
}

template <class F>
void parallel_for(int64_t n, F&& body) {
    const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 65536 || threads == 1) {
        body(0, n);
        return;
    }
    std::vector<std::thread> pool;
    const int64_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        const int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
        if (lo < hi) pool.emplace_back([&, lo, hi] { body(lo, hi); });
    }
    for (auto& th : pool) th.join();
}

}  // namespace

Mat4f nscreen_to_world(const Camera& cam, int w, int h) {
    const Mat4f worldToClip = perspective(cam.fov, cam.nearDist, cam.farDist) * world_to_camera(cam);
    return inverted(fit_to_view((float)w, (float)h) * worldToClip);
}

std::vector<int32_t> pixel_table(int w, int h) {   // PixelTable.cc:70-161 ("smart mode")
    std::vector<int32_t> idxToPos((size_t)w * h);
    int idx = 0;
    const int bheight = h & ~7;
    const int bwidth = w & ~7;
    int maxdim = std::max(bwidth, bheight);
    maxdim |= maxdim >> 1;
    maxdim |= maxdim >> 2;
    maxdim |= maxdim >> 4;
    maxdim |= maxdim >> 8;
    maxdim |= maxdim >> 16;
    maxdim = (maxdim + 1) >> 1;
    const int width8 = bwidth >> 3, height8 = bheight >> 3;
    for (int i = 0; i < maxdim * maxdim; i++) {
        int tx = 0, ty = 0, val = i, bit = 1;
        while (val) {
            if (val & 1) tx |= bit;
            if (val & 2) ty |= bit;
            bit += bit;
            val >>= 2;
        }
        if (tx < width8 && ty < height8)
            for (int inner = 0; inner < 64; inner++) {
                const int ix = ((inner & 1) >> 0) | ((inner & 4) >> 1) | ((inner & 16) >> 2);
                const int iy = ((inner & 2) >> 1) | ((inner & 8) >> 2) | ((inner & 32) >> 3);
                idxToPos[idx++] = (ty * 8 + iy) * w + (tx * 8 + ix);
            }
    }
    for (int px = 0; px < bwidth; px++)
        for (int py = bheight; py < h; py++) idxToPos[idx++] = px + py * w;
    for (int py = 0; py < h; py++)
        for (int px = bwidth; px < w; px++) idxToPos[idx++] = px + py * w;
    return idxToPos;
}

void gen_primary_rays(const Camera& cam, int w, int h, Ray* out, int32_t* slotToId, float jx, float jy) {
    const Mat4f m = nscreen_to_world(cam, w, h);
    const std::vector<int32_t> table = pixel_table(w, h);
    const rg::V3 origin = rg::make(cam.position.x, cam.position.y, cam.position.z);
    parallel_for((int64_t)w * h, [&](int64_t lo, int64_t hi) {
        for (int64_t task = lo; task < hi; task++) {
            const int pixel = table[task];
            const rg::RayRec r = rg::primary_ray(m.m, origin, cam.farDist, w, h, pixel, jx, jy);
            std::memcpy(&out[task], &r, sizeof(Ray));
            if (slotToId) slotToId[task] = pixel;
        }
    });
}

void gen_ao_rays(const Ray* inRays, const RayResult* inResults, int64_t numInput, const Vec3f* triNormals,
                 int64_t numTris, int numSamples, float maxDist, uint32_t seed, Ray* out) {
    static_assert(sizeof(Vec3f) == 12, "normals are packed float triples");
    const float* normals = reinterpret_cast<const float*>(triNormals);
    parallel_for(numInput, [&](int64_t lo, int64_t hi) {
        for (int64_t task = lo; task < hi; task++) {
            rg::RayRec in;
            std::memcpy(&in, &inRays[task], sizeof(in));
            const rg::AOBasis b =
                rg::ao_basis(in, inResults[task].id, inResults[task].t, normals, numTris, seed, (uint32_t)task);
            for (int i = 0; i < numSamples; i++) {
                const rg::RayRec r = rg::ao_sample(b, i, maxDist);
                std::memcpy(&out[task * numSamples + i], &r, sizeof(Ray));
            }
        }
    });
}

int64_t count_hits(const RayResult* results, int64_t n) {   // countHitsKernel (RendererKernels.cu:114-162)
    int64_t hits = 0;
    for (int64_t i = 0; i < n; i++) hits += (results[i].id >= 0);
    return hits;
}

}  // namespace mrt
