// fwhash.cpp — hashBuffer of the reference framework (src/framework/base/Hash.cc:34-76).
#include "fwhash.hpp"

namespace mrt {
namespace fw {

uint32_t hash_buffer(const void* ptr, int64_t size) {
    const uint8_t* src = static_cast<const uint8_t*>(ptr);
    uint32_t a = kHashMagic, b = kHashMagic, c = kHashMagic;
    auto word = [](const uint8_t* p) {
        return (uint32_t)p[0] + ((uint32_t)p[1] << 8) + ((uint32_t)p[2] << 16) + ((uint32_t)p[3] << 24);
    };
    while (size >= 12) {
        a += word(src);
        b += word(src + 4);
        c += word(src + 8);
        jenkins_mix(a, b, c);
        src += 12;
        size -= 12;
    }
    switch (size) {   // the reference's fall-through tail
        case 11: c += (uint32_t)src[10] << 16; [[fallthrough]];
        case 10: c += (uint32_t)src[9] << 8; [[fallthrough]];
        case 9: c += src[8]; [[fallthrough]];
        case 8: b += (uint32_t)src[7] << 24; [[fallthrough]];
        case 7: b += (uint32_t)src[6] << 16; [[fallthrough]];
        case 6: b += (uint32_t)src[5] << 8; [[fallthrough]];
        case 5: b += src[4]; [[fallthrough]];
        case 4: a += (uint32_t)src[3] << 24; [[fallthrough]];
        case 3: a += (uint32_t)src[2] << 16; [[fallthrough]];
        case 2: a += (uint32_t)src[1] << 8; [[fallthrough]];
        case 1: a += src[0]; [[fallthrough]];
        case 0: break;
    }
    c += (uint32_t)size;
    jenkins_mix(a, b, c);
    return c;
}

}  // namespace fw
}  // namespace mrt
