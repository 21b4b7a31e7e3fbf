// raygen_common.hpp — the per-ray arithmetic of the reference's ray generators,
// shared verbatim by the host generator (csrc/host/raygen.cpp, g++) and the
// gfx950 kernels (csrc/raygen_kernel.hip, hipcc), so both produce the same
// rays from the same inputs:
//   primary_ray   rayGenPrimaryKernel (reference RayGenKernels.cu:79-113)
//   ao_basis/ao_sample  rayGenAOKernel (RayGenKernels.cu:117-227)
//   jenkins_mix   RayGenKernels.cu:36-47
// Evaluation order follows the reference framework's vector types
// (VectorBase::dot / normalized, Mat4f * Vec4f, Math.hh:996-1007): sums start
// from 0 and accumulate left to right; normalize multiplies by 1 * rcp(length).
// Both sides are built with -ffp-contract=off. Differences that remain: the
// device flushes denormals (FTZ) and its cosf/sinf are not glibc's, so AO/diffuse
// directions agree to a few ulp, primary rays bit for bit (denormals aside).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define MRT_HD __host__ __device__
#else
#define MRT_HD
#endif

namespace mrt {
namespace rg {

struct V3 {
    float x, y, z;
};

// Ray / RayResult records (reference Util.hh:64-89).
struct RayRec {
    float ox, oy, oz, tmin;
    float dx, dy, dz, tmax;
};

MRT_HD inline V3 make(float x, float y, float z) { return V3{x, y, z}; }
MRT_HD inline V3 add(V3 a, V3 b) { return make(a.x + b.x, a.y + b.y, a.z + b.z); }
MRT_HD inline V3 sub(V3 a, V3 b) { return make(a.x - b.x, a.y - b.y, a.z - b.z); }
MRT_HD inline V3 scale(V3 a, float s) { return make(a.x * s, a.y * s, a.z * s); }
MRT_HD inline V3 neg(V3 a) { return make(-a.x, -a.y, -a.z); }
MRT_HD inline float dot(V3 a, V3 b) {
    float r = 0.0f;
    r += a.x * b.x;
    r += a.y * b.y;
    r += a.z * b.z;
    return r;
}
MRT_HD inline V3 cross(V3 a, V3 b) { return make(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
MRT_HD inline float fw_max(float a, float b) { return (a > b) ? a : b; }
MRT_HD inline float fw_rcp(float a) { return (a != 0.0f) ? 1.0f / a : 0.0f; }
MRT_HD inline V3 normalize(V3 a) { return scale(a, 1.0f * fw_rcp(sqrtf(dot(a, a)))); }
MRT_HD inline V3 vabs(V3 a) { return make(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }

MRT_HD inline float rg_cos(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return cosf(x);
#else
    return std::cos(x);
#endif
}
MRT_HD inline float rg_sin(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return sinf(x);
#else
    return std::sin(x);
#endif
}

constexpr float kPi = 3.14159265358979323846f;

// m: column-major 4x4 nscreen-to-world matrix, (r, c) at m[c * 4 + r]. (jx, jy):
// position inside the pixel; the reference always uses the centre (0.5, 0.5).
MRT_HD inline RayRec primary_ray(const float* m, V3 origin, float maxDist, int w, int h, int pixel, float jx = 0.5f,
                                 float jy = 0.5f) {
    const float ns[4] = {2.0f * ((float)(pixel % w) + jx) / (float)w - 1.0f,
                         2.0f * ((float)(pixel / w) + jy) / (float)h - 1.0f, 0.0f, 1.0f};
    float wp4[4];
    for (int i = 0; i < 4; i++) {
        float rr = 0.0f;
        for (int j = 0; j < 4; j++) rr += m[j * 4 + i] * ns[j];
        wp4[i] = rr;
    }
    const V3 wp = make(wp4[0] / wp4[3], wp4[1] / wp4[3], wp4[2] / wp4[3]);
    const V3 dir = normalize(sub(wp, origin));
    return RayRec{origin.x, origin.y, origin.z, 0.0f, dir.x, dir.y, dir.z, maxDist};
}

MRT_HD inline void jenkins_mix(uint32_t& a, uint32_t& b, uint32_t& c) {
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

// Per input ray: the backed-off origin, the viewer-facing normal and the two
// tangents rotated by the ray's Jenkins-hash angle.
struct AOBasis {
    V3 origin, normal, t0, t1;
    bool miss;
};

MRT_HD inline AOBasis ao_basis(const RayRec& in, int32_t id, float t, const float* normals, int64_t numTris,
                               uint32_t seed, uint32_t task) {
    AOBasis b;
    const V3 o = make(in.ox, in.oy, in.oz), d = make(in.dx, in.dy, in.dz);
    b.origin = add(o, scale(d, fw_max(t - 1.0e-4f, 0.0f)));
    V3 normal = make(1.0f, 0.0f, 0.0f);
    if (id >= 0 && id < numTris) normal = make(normals[3 * (int64_t)id], normals[3 * (int64_t)id + 1], normals[3 * (int64_t)id + 2]);
    if (dot(normal, d) > 0.0f) normal = neg(normal);
    const V3 na = vabs(normal);
    const float nm = fw_max(fw_max(na.x, na.y), na.z);
    V3 perp = make(normal.y, -normal.x, 0.0f);
    if (nm == na.z) perp = make(0.0f, normal.z, -normal.y);
    else if (nm == na.x) perp = make(-normal.z, 0.0f, normal.x);
    perp = normalize(perp);
    const V3 biperp = cross(normal, perp);
    uint32_t ha = seed + task, hb = 0x9e3779b9u, hc = 0x9e3779b9u;
    jenkins_mix(ha, hb, hc);
    jenkins_mix(ha, hb, hc);
    const float angle = 2.0f * kPi * (float)hc * 0x1p-32f;
    const float ca = rg_cos(angle), sa = rg_sin(angle);
    b.t0 = add(scale(perp, ca), scale(biperp, sa));
    b.t1 = add(scale(perp, -sa), scale(biperp, ca));
    b.normal = normal;
    b.miss = id == -1;
    return b;
}

// Sample i: Halton (2, 3) point warped onto the cosine hemisphere around the normal.
// ao_sample_xyz is the part that depends on i only (so a generator may compute it once
// per sample index and share it), ao_sample_dir the rotation into the ray's basis.
MRT_HD inline V3 ao_sample_xyz(int i) {
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
    const float a2 = 2.0f * kPi * y;
    const float r = sqrtf(x);
    x = r * rg_cos(a2);
    y = r * rg_sin(a2);
    const float z = sqrtf(1.0f - x * x - y * y);
    return make(x, y, z);
}

MRT_HD inline RayRec ao_sample_dir(const AOBasis& b, V3 s, float maxDist) {
    const V3 dir = normalize(add(add(scale(b.t0, s.x), scale(b.t1, s.y)), scale(b.normal, s.z)));
    return RayRec{b.origin.x, b.origin.y, b.origin.z, 0.0f, dir.x, dir.y, dir.z, b.miss ? -1.0f : maxDist};
}

MRT_HD inline RayRec ao_sample(const AOBasis& b, int i, float maxDist) {
    return ao_sample_dir(b, ao_sample_xyz(i), maxDist);
}

}  // namespace rg
}  // namespace mrt
