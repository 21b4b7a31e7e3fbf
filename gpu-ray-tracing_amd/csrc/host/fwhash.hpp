// fwhash.hpp — the reference framework's hash functions (src/framework/base/Hash.hh:181-201,
// Hash.cc:34-112), which name the reference's bvhcache files: Renderer::getCudaBVH
// (Renderer.cc:178-186) writes "<bvhCachePath>/%08x.dat" with
// hashBits(scene.hash(), platform.computeHash(), buildParams.computeHash(), layout).
#pragma once
#include <cstdint>
#include <string>

namespace mrt {
namespace fw {

constexpr uint32_t kHashMagic = 0x9e3779b9u;   // FW_HASH_MAGIC

inline void jenkins_mix(uint32_t& a, uint32_t& b, uint32_t& c) {   // FW_JENKINS_MIX
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

// hashBits(a, b = MAGIC, c = 0) and hashBits(a, b, c, d, e = 0, f = 0) (Hash.hh:195-196).
inline uint32_t hash_bits(uint32_t a, uint32_t b = kHashMagic, uint32_t c = 0) {
    c += kHashMagic;
    jenkins_mix(a, b, c);
    return c;
}
inline uint32_t hash_bits6(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e = 0, uint32_t f = 0) {
    c += kHashMagic;
    jenkins_mix(a, b, c);
    a += d;
    b += e;
    c += f;
    jenkins_mix(a, b, c);
    return c;
}

// hashBuffer (Hash.cc:34-76): 12-byte little-endian blocks, then the tail, then
// c += (the tail's length — not the buffer's) and one last mix. hashBufferAlign
// (:80-112) gives the same value for 4-byte-aligned sizes.
uint32_t hash_buffer(const void* ptr, int64_t size);

inline uint32_t float_bits(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}

}  // namespace fw
}  // namespace mrt
