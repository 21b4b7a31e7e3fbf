// raygen.cpp — camera matrices, the Morton-swizzled pixel table and the
// primary / AO / diffuse ray generators, on the host.
//
// Restates (with IEEE host arithmetic instead of the reference's
// --use_fast_math device code, so results agree statistically, not bitwise):
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
#include <thread>
#include <vector>

#include "raygen.hpp"

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

inline void jenkins_mix(uint32_t& a, uint32_t& b, uint32_t& c) {   // RayGenKernels.cu:36-47
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
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

void gen_primary_rays(const Camera& cam, int w, int h, Ray* out, int32_t* slotToId) {
    const Mat4f m = nscreen_to_world(cam, w, h);
    const std::vector<int32_t> table = pixel_table(w, h);
    parallel_for((int64_t)w * h, [&](int64_t lo, int64_t hi) {
        for (int64_t task = lo; task < hi; task++) {
            const int pixel = table[task];
            const Vec4f ns(2.0f * ((float)(pixel % w) + 0.5f) / (float)w - 1.0f,
                           2.0f * ((float)(pixel / w) + 0.5f) / (float)h - 1.0f, 0.0f, 1.0f);
            const Vec4f wp4 = m * ns;
            const Vec3f wp = Vec3f(wp4.x, wp4.y, wp4.z) / wp4.w;
            const Vec3f dir = normalize(wp - cam.position);
            Ray& r = out[task];
            r.ox = cam.position.x; r.oy = cam.position.y; r.oz = cam.position.z; r.tmin = 0.0f;
            r.dx = dir.x; r.dy = dir.y; r.dz = dir.z; r.tmax = cam.farDist;
            if (slotToId) slotToId[task] = pixel;
        }
    });
}

void gen_ao_rays(const Ray* inRays, const RayResult* inResults, int64_t numInput, const Vec3f* triNormals,
                 int64_t numTris, int numSamples, float maxDist, uint32_t seed, Ray* out) {
    parallel_for(numInput, [&](int64_t lo, int64_t hi) {
        for (int64_t task = lo; task < hi; task++) {
            const Ray& ir = inRays[task];
            const RayResult& res = inResults[task];
            const Vec3f o(ir.ox, ir.oy, ir.oz), d(ir.dx, ir.dy, ir.dz);
            const Vec3f origin = o + d * fw_max(res.t - 1.0e-4f, 0.0f);

            const int tri = res.id;
            Vec3f normal(1.0f, 0.0f, 0.0f);
            if (tri >= 0 && tri < numTris) normal = triNormals[tri];
            if (dot(normal, d) > 0.0f) normal = -normal;

            const Vec3f na = vabs(normal);
            const float nm = fw_max(fw_max(na.x, na.y), na.z);
            Vec3f perp(normal.y, -normal.x, 0.0f);
            if (nm == na.z) perp = Vec3f(0.0f, normal.z, -normal.y);
            else if (nm == na.x) perp = Vec3f(-normal.z, 0.0f, normal.x);
            perp = normalize(perp);
            const Vec3f biperp = cross(normal, perp);

            uint32_t ha = seed + (uint32_t)task, hb = 0x9e3779b9u, hc = 0x9e3779b9u;
            jenkins_mix(ha, hb, hc);
            jenkins_mix(ha, hb, hc);
            const float angle = 2.0f * kPiF * (float)hc * 0x1p-32f;
            const float ca = std::cos(angle), sa = std::sin(angle);
            const Vec3f t0 = perp * ca + biperp * sa;
            const Vec3f t1 = perp * -sa + biperp * ca;

            for (int i = 0; i < numSamples; i++) {
                float x = 0.0f, xadd = 1.0f;
                for (unsigned hc2 = (unsigned)i + 1; hc2 != 0; hc2 >>= 1) {
                    xadd *= 0.5f;
                    if (hc2 & 1) x += xadd;
                }
                float y = 0.0f, yadd = 1.0f;
                for (int hc3 = i + 1; hc3 != 0; hc3 /= 3) {
                    yadd *= 1.0f / 3.0f;
                    y += (float)(hc3 % 3) * yadd;
                }
                const float a2 = 2.0f * kPiF * y;
                const float r = std::sqrt(x);
                x = r * std::cos(a2);
                y = r * std::sin(a2);
                const float z = std::sqrt(1.0f - x * x - y * y);
                const Vec3f dir = normalize(t0 * x + t1 * y + normal * z);
                Ray& orr = out[task * numSamples + i];
                orr.ox = origin.x; orr.oy = origin.y; orr.oz = origin.z; orr.tmin = 0.0f;
                orr.dx = dir.x; orr.dy = dir.y; orr.dz = dir.z;
                orr.tmax = (tri == -1) ? -1.0f : maxDist;
            }
        }
    });
}

int64_t count_hits(const RayResult* results, int64_t n) {   // countHitsKernel (RendererKernels.cu:114-162)
    int64_t hits = 0;
    for (int64_t i = 0; i < n; i++) hits += (results[i].id != -1);
    return hits;
}

}  // namespace mrt
