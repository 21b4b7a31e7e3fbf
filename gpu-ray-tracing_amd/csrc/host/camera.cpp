// camera.cpp — the reference's camera signature: the 6-bit text encoding the
// App's --camera argument carries (grtcmdline.txt), decoded exactly as
// CameraControls::decodeSignature / decodeFloat / decodeDirection / decodeBits
// do (src/framework/3d/CameraControls.cc:374-419, 502-554).
//
//   decodeBits       one character -> 6 bits: '/'..':' = 0..11, 'A'..'Z' = 12..37, 'a'..'z' = 38..63
//   decodeFloat      six characters, little end first (bits i*6.. of the float's bit pattern)
//   decodeDirection  a face character (bit 0-1: major axis, bit 2: negative, bit 3: axis-aligned),
//                    then the two minor components divided by the major one (absent when aligned),
//                    normalised (VectorBase::normalized: v * (1 * rcp(length))) and rotated back
//   signature        "position xyz, forward, up, speed, fov, near, far, keepAligned" with optional
//                    surrounding quotes, a trailing comma and whitespace; anything else fails
#include <cstdint>
#include <cstring>

#include "math.hpp"

namespace mrt {

namespace {

bool decode_bits(const char*& src, uint32_t* out) {
    const char c = *src;
    if (c >= '/' && c <= ':') *out = (uint32_t)(c - '/');
    else if (c >= 'A' && c <= 'Z') *out = (uint32_t)(c - 'A' + 12);
    else if (c >= 'a' && c <= 'z') *out = (uint32_t)(c - 'a' + 38);
    else return false;
    ++src;
    return true;
}

bool decode_float(const char*& src, float* out) {
    uint32_t bits = 0;
    for (int i = 0; i < 32; i += 6) {
        uint32_t b = 0;
        if (!decode_bits(src, &b)) return false;
        bits |= b << i;
    }
    std::memcpy(out, &bits, 4);
    return true;
}

bool decode_direction(const char*& src, Vec3f* out) {
    uint32_t face = 0;
    if (!decode_bits(src, &face)) return false;
    Vec3f tuv;
    tuv.x = ((face & 4) == 0) ? 1.0f : -1.0f;
    if ((face & 8) == 0) {
        if (!decode_float(src, &tuv.y) || !decode_float(src, &tuv.z)) return false;
    }
    tuv = normalize(tuv);
    switch (face & 3) {
        case 0: *out = tuv; break;
        case 1: *out = Vec3f(tuv.z, tuv.x, tuv.y); break;
        default: *out = Vec3f(tuv.y, tuv.z, tuv.x); break;
    }
    return true;
}

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n'; }

}  // namespace

bool decode_camera_signature(const char* sig, CameraSignature* out) {
    if (!sig || !out) return false;
    const char* src = sig;
    while (is_space(*src)) src++;
    if (*src == '"') src++;
    CameraSignature c;
    uint32_t keep = 0;
    if (!decode_float(src, &c.position.x) || !decode_float(src, &c.position.y) || !decode_float(src, &c.position.z) ||
        !decode_direction(src, &c.forward) || !decode_direction(src, &c.up) || !decode_float(src, &c.speed) ||
        !decode_float(src, &c.fov) || !decode_float(src, &c.nearDist) || !decode_float(src, &c.farDist) ||
        !decode_bits(src, &keep))
        return false;
    c.keepAligned = keep != 0;
    if (*src == '"') src++;
    if (*src == ',') src++;
    while (is_space(*src)) src++;
    if (*src) return false;   // "CameraControls: Invalid signature!"
    *out = c;
    return true;
}

}  // namespace mrt
