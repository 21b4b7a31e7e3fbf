// math.hpp — the few float vector/matrix operations the host side needs,
// restated with the reference framework's exact evaluation order so that the
// BVH builder and the Woop transform produce the same bits the reference's
// host code would (reference src/framework/base/Math.hh, Defs.hh:140-160,
// src/rt/Util.hh:37-57). Host min/max are the reference's FW::min/max:
// (a < b) ? a : b and (a > b) ? a : b, NOT fminf/fmaxf.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace mrt {

inline float fw_min(float a, float b) { return (a < b) ? a : b; }
inline float fw_max(float a, float b) { return (a > b) ? a : b; }
inline float fw_rcp(float a) { return (a != 0.0f) ? 1.0f / a : 0.0f; }   // Math.hh:113
inline uint32_t float_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float bits_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

struct Vec3f {
    float x = 0.f, y = 0.f, z = 0.f;
    Vec3f() = default;
    Vec3f(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit Vec3f(float a) : x(a), y(a), z(a) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
    float min_comp() const { return fw_min(fw_min(x, y), z); }   // VectorBase::min()
    float max_comp() const { return fw_max(fw_max(x, y), z); }
    float sum() const { return (x + y) + z; }
};
inline Vec3f operator+(const Vec3f& a, const Vec3f& b) { return Vec3f(a.x + b.x, a.y + b.y, a.z + b.z); }
inline Vec3f operator-(const Vec3f& a, const Vec3f& b) { return Vec3f(a.x - b.x, a.y - b.y, a.z - b.z); }
inline Vec3f operator*(const Vec3f& a, const Vec3f& b) { return Vec3f(a.x * b.x, a.y * b.y, a.z * b.z); }
inline Vec3f operator*(const Vec3f& a, float s) { return Vec3f(a.x * s, a.y * s, a.z * s); }
inline Vec3f operator/(const Vec3f& a, float s) { return Vec3f(a.x / s, a.y / s, a.z / s); }
inline Vec3f operator-(const Vec3f& a) { return Vec3f(-a.x, -a.y, -a.z); }
inline Vec3f vmin(const Vec3f& a, const Vec3f& b) { return Vec3f(fw_min(a.x, b.x), fw_min(a.y, b.y), fw_min(a.z, b.z)); }
inline Vec3f vmax(const Vec3f& a, const Vec3f& b) { return Vec3f(fw_max(a.x, b.x), fw_max(a.y, b.y), fw_max(a.z, b.z)); }
inline Vec3f cross(const Vec3f& a, const Vec3f& b) {   // Math.hh:338
    return Vec3f(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float dot(const Vec3f& a, const Vec3f& b) {   // VectorBase::dot: r = 0; r += a[i]*b[i]
    float r = 0.0f;
    r += a.x * b.x;
    r += a.y * b.y;
    r += a.z * b.z;
    return r;
}
inline float length(const Vec3f& a) { return std::sqrt(dot(a, a)); }
inline Vec3f normalize(const Vec3f& a) { return a * (1.0f * fw_rcp(length(a))); }   // VectorBase::normalized
inline Vec3f vabs(const Vec3f& a) { return Vec3f(std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)); }

struct Vec4f {
    float x = 0.f, y = 0.f, z = 0.f, w = 0.f;
    Vec4f() = default;
    Vec4f(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    Vec4f(const Vec3f& v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};

// Axis-aligned box (reference src/rt/Util.hh:37-57).
struct AABB {
    Vec3f mn{FLT_MAX, FLT_MAX, FLT_MAX};
    Vec3f mx{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    AABB() = default;
    AABB(const Vec3f& a, const Vec3f& b) : mn(a), mx(b) {}
    void grow(const Vec3f& p) { mn = vmin(mn, p); mx = vmax(mx, p); }
    void grow(const AABB& b) { grow(b.mn); grow(b.mx); }
    void intersect(const AABB& b) { mn = vmax(mn, b.mn); mx = vmin(mx, b.mx); }
    bool valid() const { return mn.x <= mx.x && mn.y <= mx.y && mn.z <= mx.z; }
    float area() const {
        if (!valid()) return 0.0f;
        const Vec3f d = mx - mn;
        return (d.x * d.y + d.y * d.z + d.z * d.x) * 2.0f;
    }
};

// Column-major 4x4 float matrix; (r, c) at m[c * 4 + r] (Math.hh:674-692).
struct Mat4f {
    float m[16];
    Mat4f() { set_identity(); }
    void set_identity() {
        for (int i = 0; i < 16; i++) m[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    }
    float& operator()(int r, int c) { return m[c * 4 + r]; }
    float operator()(int r, int c) const { return m[c * 4 + r]; }
    void set_col(int c, const Vec4f& v) { for (int r = 0; r < 4; r++) (*this)(r, c) = v[r]; }
    void set_row(int r, const Vec4f& v) { for (int c = 0; c < 4; c++) (*this)(r, c) = v[c]; }
    Vec4f row(int r) const { return Vec4f((*this)(r, 0), (*this)(r, 1), (*this)(r, 2), (*this)(r, 3)); }

    static Mat4f scale(const Vec3f& s) {
        Mat4f r;
        r(0, 0) = s.x; r(1, 1) = s.y; r(2, 2) = s.z;
        return r;
    }
    static Mat4f translate(const Vec3f& t) {
        Mat4f r;
        r(0, 3) = t.x; r(1, 3) = t.y; r(2, 3) = t.z;
        return r;
    }
};

inline Mat4f operator*(const Mat4f& a, const Mat4f& b) {   // Math.hh:1031-1044
    Mat4f r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float rr = 0.0f;
            for (int k = 0; k < 4; k++) rr += a(i, k) * b(k, j);
            r(i, j) = rr;
        }
    return r;
}

inline Vec4f operator*(const Mat4f& a, const Vec4f& v) {   // Math.hh:996-1007
    Vec4f r;
    for (int i = 0; i < 4; i++) {
        float rr = 0.0f;
        for (int j = 0; j < 4; j++) rr += a(i, j) * v[j];
        r[i] = rr;
    }
    return r;
}

// 3x3 determinant in the reference's term order (Math.hh:935-940).
inline float det3(const float v[3][3]) {
    return v[0][0] * v[1][1] * v[2][2] - v[0][0] * v[1][2] * v[2][1] + v[1][0] * v[2][1] * v[0][2] -
           v[1][0] * v[2][2] * v[0][1] + v[2][0] * v[0][1] * v[1][2] - v[2][0] * v[0][2] * v[1][1];
}

// Cofactor inverse with the reference's quirk: d accumulates L * det, and the
// result is r * rcp(d) * L (Math.hh:962-984).
inline Mat4f inverted(const Mat4f& a) {
    Mat4f r;
    float d = 0.0f;
    float si = 1.0f;
    for (int i = 0; i < 4; i++) {
        float sj = si;
        for (int j = 0; j < 4; j++) {
            float sub[3][3];
            for (int k = 0; k < 3; k++)
                for (int l = 0; l < 3; l++) sub[k][l] = a((k < j) ? k : k + 1, (l < i) ? l : l + 1);
            const float dd = det3(sub) * sj;
            r(i, j) = dd;
            d += dd * a(j, i);
            sj = -sj;
        }
        si = -si;
    }
    const float rd = fw_rcp(d);
    for (int i = 0; i < 16; i++) r.m[i] = (r.m[i] * rd) * 4.0f;
    return r;
}

// A decoded camera signature (CameraControls m_position .. m_keepAligned,
// CameraControls.cc:374-419); camera.cpp.
struct CameraSignature {
    Vec3f position, forward, up;
    float speed = 0.f, fov = 0.f, nearDist = 0.f, farDist = 0.f;
    bool keepAligned = false;
};
bool decode_camera_signature(const char* sig, CameraSignature* out);

}  // namespace mrt
