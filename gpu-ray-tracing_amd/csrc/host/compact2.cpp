// compact2.cpp — BVHLayout_Compact2 serialisation of a BVH tree, the Woop
// triangle transform, and the reference's bvhcache .dat stream format.
//
// create_compact2 restates CudaBVH::createCompact(bvh, 16)
// (src/rt/cuda/CudaBVH.cc:270-357): depth-first with an explicit LIFO stack;
// an inner child gets the float4 index of its 64-B record (appended when the
// child is discovered), a leaf child gets ~(float4 index of its first Woop
// row); every leaf's triangles are followed by one (-0,-0,-0,-0) terminator;
// triIndex holds (origIdx, 0, 0) per triangle and 0 per terminator.
#include <cstdio>
#include <cstring>
#include <fstream>

#include "bvh.hpp"

namespace mrt {

void woopify(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, Vec4f out[3]) {   // CudaBVH.cc:361-380
    Mat4f mtx;
    mtx.set_col(0, Vec4f(v0 - v2, 0.0f));
    mtx.set_col(1, Vec4f(v1 - v2, 0.0f));
    mtx.set_col(2, Vec4f(cross(v0 - v2, v1 - v2), 0.0f));
    mtx.set_col(3, Vec4f(v2, 1.0f));
    mtx = inverted(mtx);
    out[0] = Vec4f(mtx(2, 0), mtx(2, 1), mtx(2, 2), -mtx(2, 3));
    out[1] = mtx.row(0);
    out[2] = mtx.row(1);
}

namespace {

void put_box_pair(int32_t* dst, const AABB& b0, const AABB& b1) {
    const float v[12] = {b0.mn.x, b0.mx.x, b0.mn.y, b0.mx.y,   // (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
                         b1.mn.x, b1.mx.x, b1.mn.y, b1.mx.y,   // (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
                         b0.mn.z, b0.mx.z, b1.mn.z, b1.mx.z};  // (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
    std::memcpy(dst, v, sizeof v);
}

}  // namespace

void create_compact2(const BvhNode& rootIn, const Scene& scene, Compact2& out) {
    out.nodes.clear();
    out.woop.clear();
    out.triIndex.clear();

    // A leaf root gets an inner parent with an empty second leaf.
    BvhNode wrapper;
    const BvhNode* root = &rootIn;
    BvhNode emptyLeaf;
    if (rootIn.is_leaf()) {
        emptyLeaf.bounds = rootIn.bounds;
        root = &wrapper;
    }
    auto child_of = [&](const BvhNode* n, int i) -> const BvhNode* {
        if (n == &wrapper) return i == 0 ? &rootIn : &emptyLeaf;
        return n->child[i].get();
    };

    struct Entry {
        const BvhNode* node;
        int64_t idx;   // in 16-int node records
    };
    std::vector<Entry> stack;
    stack.push_back({root, 0});
    out.nodes.resize(16, 0);

    while (!stack.empty()) {
        const Entry e = stack.back();
        stack.pop_back();
        const AABB* cbox[2];
        int32_t cidx[2];
        for (int i = 0; i < 2; i++) {
            const BvhNode* child = child_of(e.node, i);
            cbox[i] = &child->bounds;
            if (!child->is_leaf()) {
                const int64_t rec = (int64_t)out.nodes.size() / 16;
                cidx[i] = (int32_t)(rec * 4);   // float4 index (getNumBytes() / 16)
                stack.push_back({child, rec});
                out.nodes.resize(out.nodes.size() + 16, 0);
                continue;
            }
            cidx[i] = ~(int32_t)(out.woop.size() / 4);
            for (const int32_t tri : child->tris) {
                const Vec3i& t = scene.triangles[tri];
                Vec4f w[3];
                woopify(scene.vertices[t.x], scene.vertices[t.y], scene.vertices[t.z], w);
                if (w[0].x == 0.0f) w[0].x = 0.0f;   // -0.0 would read as a terminator
                for (int r = 0; r < 3; r++)
                    for (int c = 0; c < 4; c++) out.woop.push_back((int32_t)float_bits(w[r][c]));
                out.triIndex.push_back(tri);
                out.triIndex.push_back(0);
                out.triIndex.push_back(0);
            }
            for (int c = 0; c < 4; c++) out.woop.push_back((int32_t)0x80000000);   // terminator
            out.triIndex.push_back(0);
        }
        int32_t* dst = &out.nodes[(size_t)e.idx * 16];
        put_box_pair(dst, *cbox[0], *cbox[1]);
        dst[12] = cidx[0];
        dst[13] = cidx[1];
        dst[14] = 0;
        dst[15] = 0;
    }
}

bool save_dat(const std::string& path, const Compact2& c, std::string* err) {
    std::ofstream f(path, std::ios::binary);
    if (!f) {
        if (err) *err = "cannot write " + path;
        return false;
    }
    auto put32 = [&](uint32_t v) { unsigned char b[4]; for (int i = 0; i < 4; i++) b[i] = (unsigned char)(v >> (8 * i)); f.write((const char*)b, 4); };
    auto put64 = [&](uint64_t v) { unsigned char b[8]; for (int i = 0; i < 8; i++) b[i] = (unsigned char)(v >> (8 * i)); f.write((const char*)b, 8); };
    auto putBuf = [&](const std::vector<int32_t>& v) {
        put64((uint64_t)v.size() * 4);
        for (int32_t x : v) put32((uint32_t)x);
    };
    put32((uint32_t)kLayoutCompact2);
    putBuf(c.nodes);
    putBuf(c.woop);
    putBuf(c.triIndex);
    if (!f) {
        if (err) *err = "write failed: " + path;
        return false;
    }
    return true;
}

bool load_dat(const std::string& path, Compact2& c, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        if (err) *err = "cannot open " + path;
        return false;
    }
    auto get = [&](int n, uint64_t* v) {
        unsigned char b[8] = {};
        if (!f.read((char*)b, n)) return false;
        *v = 0;
        for (int i = 0; i < n; i++) *v |= (uint64_t)b[i] << (8 * i);
        return true;
    };
    uint64_t layout = 0;
    if (!get(4, &layout) || (int32_t)layout != kLayoutCompact2) {
        if (err) *err = "not a Compact2 bvhcache file (layout != 5): " + path;
        return false;
    }
    std::vector<int32_t>* bufs[3] = {&c.nodes, &c.woop, &c.triIndex};
    for (auto* b : bufs) {
        uint64_t bytes = 0;
        if (!get(8, &bytes) || bytes % 4 != 0 || bytes > (1ull << 40)) {
            if (err) *err = "corrupt buffer header in " + path;
            return false;
        }
        b->resize(bytes / 4);
        if (bytes && !f.read((char*)b->data(), (std::streamsize)bytes)) {   // little-endian host
            if (err) *err = "truncated bvhcache file " + path;
            return false;
        }
    }
    return true;
}

}  // namespace mrt
