// wide_bvh.cpp — the 4-wide node array the production traversal reads, derived
// at bind time from the bound Compact2 tree (CudaBVH.cc:270-357 layout).
//
// Collapse: every wide node starts from a binary inner node's two children and
// repeatedly replaces its inner child of largest surface area by that child's
// two children until it holds four (leaves stay leaves; a node may keep fewer
// children, the rest are absent). Child boxes are the binary tree's boxes,
// bit for bit, so the slab test of a wide child is the binary step's test of
// that same box. Wide nodes are numbered depth first (a node's first inner child
// follows it), 128 B each, one cache line:
//   float4 0  (c0.lo.x, c0.hi.x, c1.lo.x, c1.hi.x)     float4 1  (c2.lo.x, c2.hi.x, c3.lo.x, c3.hi.x)
//   float4 2  the same for y                           float4 3
//   float4 4  the same for z                           float4 5
//   float4 6  child refs (int): inner = float4 index of the wide node (8 per node),
//             leaf = ~(woop float4 index [| count << 27, below]), absent = 0x76543210
//             (an absent child's planes are NaN: its slab test always fails)
//   float4 7  unused (zero)
// Leaves, Woop triangles and triIndex are the Compact2 ones. Given the first word of
// every Woop slot (leaf_counts_fit), a leaf ref carries its triangle count:
// ~(woop index | count << 27) with count 1..15 (0 = not counted: the leaf ends at
// its terminator, as in the binary step), so the leaf loop neither loads the
// terminator nor a triangle slot past it.
//
// The quantized form (build_wide4q) stores the same four children in 64 B, four
// 16-B loads instead of seven (the traversal is bound by 16-B lane loads,
// profiles/round2_tuning.md):
//   float4 0  origin (x, y, z) = the union box's lower corner; w = three biased
//             exponents (byte k = e_k + 127; the axis step is 2^e_k)
//   float4 1  (qlo.x, qhi.x, qlo.y, qhi.y)  one byte per child (child c = byte c)
//   float4 2  (qlo.z, qhi.z, 0, 0)
//   float4 3  child refs: inner = float4 index of the wide node (4 per node),
//             leaf = as in the exact form, absent = 0x76543210
// A child plane decodes as fma(q, 2^e, origin) in f32 with denormals flushed —
// the kernel's arithmetic exactly — and q is chosen so that the decoded lower
// plane is <= the Compact2 plane and the decoded upper plane >= it. The decoded
// box therefore contains the binary box, its slab interval contains the binary
// one (the slab values are monotonic in the plane), and the traversal tests a
// superset of the leaves the binary traversal tests.
#include <algorithm>
#include <atomic>
#include <thread>
#include <utility>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "trace_kernel.hpp"

namespace mrt {

namespace {

struct Child {
    int32_t ref;
    float lo[3], hi[3];
};

float as_float(int32_t i) {
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

void binary_children(const int32_t* nodes, int32_t ref, Child out[2]) {
    const int32_t* n = nodes + (int64_t)(ref / 4) * 16;
    out[0] = Child{n[12], {as_float(n[0]), as_float(n[2]), as_float(n[8])}, {as_float(n[1]), as_float(n[3]), as_float(n[9])}};
    out[1] = Child{n[13], {as_float(n[4]), as_float(n[6]), as_float(n[10])}, {as_float(n[5]), as_float(n[7]), as_float(n[11])}};
}

double half_area(const Child& c) {
    const double x = (double)c.hi[0] - c.lo[0], y = (double)c.hi[1] - c.lo[1], z = (double)c.hi[2] - c.lo[2];
    return x * y + y * z + z * x;
}

// The children of the wide node rooted at binary node `ref`.
int collapse(const int32_t* nodes, int32_t ref, Child out[4]) {
    Child two[2];
    binary_children(nodes, ref, two);
    out[0] = two[0];
    out[1] = two[1];
    int n = 2;
    while (n < 4) {
        int best = -1;
        double bestArea = -1.0;
        for (int i = 0; i < n; i++)
            if (out[i].ref >= 0 && half_area(out[i]) > bestArea) {
                bestArea = half_area(out[i]);
                best = i;
            }
        if (best < 0) break;
        binary_children(nodes, out[best].ref, two);
        for (int i = n; i > best + 1; i--) out[i] = out[i - 1];   // the two grandchildren take best's place
        out[best] = two[0];
        out[best + 1] = two[1];
        n++;
    }
    return n;
}

// The ref a wide child stores for Compact2 leaf ref `ref` (see above).
int32_t wide_leaf_ref(int32_t ref, const int32_t* woopX, int64_t woopSlots) {
    if (!woopX) return ref;
    const int64_t slot = ~(int64_t)ref;
    int32_t count = 0;
    for (int32_t k = 0; k <= 15; k++) {
        const int64_t s = slot + 3 * (int64_t)k;
        if (s >= woopSlots) break;
        if (woopX[s] == (int32_t)0x80000000) {
            count = k;
            break;
        }
    }
    return ~(int32_t)(slot | ((int64_t)count << kWideLeafAddrBits));
}

// f32 with denormals flushed to (signed) zero, as the kernel computes.
float ftz(float x) { return std::fabs(x) < FLT_MIN ? std::copysign(0.0f, x) : x; }

float decode(int q, float step, float origin) { return ftz(std::fmaf((float)q, step, origin)); }

// Quantizes one axis of up to four children. False when no exponent fits.
bool quantize_axis(const float* lo, const float* hi, int n, float* origin, int* biasedExp, uint8_t* qlo, uint8_t* qhi) {
    float o = INFINITY, top = -INFINITY;
    for (int c = 0; c < n; c++) {
        o = std::fmin(o, ftz(lo[c]));
        top = std::fmax(top, ftz(hi[c]));
    }
    if (!std::isfinite(o) || !std::isfinite(top)) return false;
    o = ftz(o);
    const double extent = (double)top - (double)o;
    int e = -126;
    if (extent > 0) e = std::max(-126, (int)std::ceil(std::log2(extent / 255.0)));
    for (; e <= 127; e++) {
        const float step = std::ldexp(1.0f, e);
        bool ok = true;
        for (int c = 0; c < n && ok; c++) {
            const float l = ftz(lo[c]), h = ftz(hi[c]);
            int a = (int)std::floor(((double)l - o) / step);
            a = std::min(255, std::max(0, a));
            while (a > 0 && decode(a, step, o) > l) a--;
            int b = (int)std::ceil(((double)h - o) / step);
            b = std::min(255, std::max(0, b));
            while (b < 255 && decode(b, step, o) < h) b++;
            if (decode(a, step, o) > l || decode(b, step, o) < h) ok = false;
            qlo[c] = (uint8_t)a;
            qhi[c] = (uint8_t)b;
        }
        if (ok) {
            *origin = o;
            *biasedExp = e + 127;
            return true;
        }
    }
    return false;
}

// The binary roots of the wide nodes under `root` (inclusive), depth first.
void preorder(const int32_t* nodes, int32_t root, std::vector<int32_t>& order) {
    std::vector<int32_t> stack{root};
    Child ch[4];
    while (!stack.empty()) {
        const int32_t ref = stack.back();
        stack.pop_back();
        order.push_back(ref);
        const int n = collapse(nodes, ref, ch);
        for (int i = n - 1; i >= 0; i--)
            if (ch[i].ref >= 0) stack.push_back(ch[i].ref);
    }
}

// Runs fn(i) for i in [0, n) on up to hardware_concurrency() threads (bind-time
// work on trees of millions of nodes: VERDICT r2 #7).
template <class F>
void parallel_for(int64_t n, F fn) {
    // the process's CPU share: OMP_NUM_THREADS where set (the GPU boxes: 16; their
    // hardware_concurrency() counts the whole machine), else the hardware threads, at most 16
    int64_t cap = std::max(1u, std::thread::hardware_concurrency());
    if (const char* e = std::getenv("OMP_NUM_THREADS")) cap = std::max<int64_t>(1, std::atoll(e));
    const int64_t threads = std::max<int64_t>(1, std::min<int64_t>({n, cap, 16}));
    if (threads == 1 || n < 2) {
        for (int64_t i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<int64_t> next{0};
    std::vector<std::thread> pool;
    for (int64_t k = 0; k < threads; k++)
        pool.emplace_back([&]() {
            for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i);
        });
    for (auto& t : pool) t.join();
}

// Depth-first wide numbering: binary node -> wide index, and the binary roots in
// order. The top kSplitLevels wide levels are walked here; every subtree below them
// is walked on its own thread, then the subtrees' local orders are placed at their
// preorder offsets (the same numbering as one sequential walk).
void number_wide(const int32_t* nodes, int64_t numNodes, std::vector<int32_t>& wideOf, std::vector<int32_t>& order) {
    constexpr int kSplitLevels = 4;   // up to 4^4 subtree tasks
    wideOf.assign((size_t)numNodes, -1);
    order.clear();
    std::vector<int32_t> top;                       // >= 0: a wide root above the split; < 0: ~task
    std::vector<int32_t> tasks;                     // the binary roots of the subtree tasks
    std::vector<std::pair<int32_t, int>> stack{{0, 0}};
    Child ch[4];
    while (!stack.empty()) {
        const auto [ref, depth] = stack.back();
        stack.pop_back();
        if (depth == kSplitLevels) {
            top.push_back(~(int32_t)tasks.size());
            tasks.push_back(ref);
            continue;
        }
        top.push_back(ref);
        const int n = collapse(nodes, ref, ch);
        for (int i = n - 1; i >= 0; i--)
            if (ch[i].ref >= 0) stack.push_back({ch[i].ref, depth + 1});
    }
    std::vector<std::vector<int32_t>> sub(tasks.size());
    parallel_for((int64_t)tasks.size(), [&](int64_t i) { preorder(nodes, tasks[(size_t)i], sub[(size_t)i]); });
    std::vector<int64_t> base(tasks.size(), 0);
    for (int32_t e : top) {
        if (e >= 0) {
            order.push_back(e);
        } else {
            base[(size_t)~e] = (int64_t)order.size();
            order.insert(order.end(), sub[(size_t)~e].begin(), sub[(size_t)~e].end());
        }
    }
    parallel_for((int64_t)((order.size() + 65535) / 65536), [&](int64_t c) {
        const size_t end = std::min(order.size(), (size_t)(c + 1) * 65536);
        for (size_t w = (size_t)c * 65536; w < end; w++) wideOf[(size_t)(order[w] / 4)] = (int32_t)w;
    });
}

}  // namespace

bool leaf_counts_fit(int64_t woopSlots) { return woopSlots <= ((int64_t)1 << kWideLeafAddrBits); }

int64_t wide_stack_bound(const uint32_t* wide, int64_t numWide, int nodeWords) {
    if (numWide <= 0) return 0;
    const int refBase = nodeWords == 32 ? 24 : 12;   // the child refs' first word
    const int refScale = nodeWords / 4;               // float4s per node: ref = node index * refScale
    int64_t bound = 0;
    std::vector<std::pair<int64_t, int64_t>> todo{{0, 0}};   // (wide node, entries on the stack when visited)
    while (!todo.empty()) {
        const auto [w, depth] = todo.back();
        todo.pop_back();
        const uint32_t* o = wide + w * nodeWords;
        int present = 0;
        for (int c = 0; c < 4; c++) present += (int32_t)o[refBase + c] != kEntrypointSentinel;
        const int64_t below = depth + std::max(0, present - 1);   // this node pushes all but the child it enters
        bound = std::max(bound, below);
        for (int c = 0; c < 4; c++) {
            const int32_t ref = (int32_t)o[refBase + c];
            if (ref >= 0 && ref != kEntrypointSentinel && ref / refScale < numWide) todo.push_back({ref / refScale, below});
        }
    }
    return bound;
}

bool build_wide4q(const int32_t* nodes, int64_t numNodes, std::vector<uint32_t>* out, const int32_t* woopX,
                  int64_t woopSlots) {
    out->clear();
    if (numNodes <= 0) return true;
    std::vector<int32_t> wideOf, order;
    number_wide(nodes, numNodes, wideOf, order);
    out->assign(order.size() * 16, 0u);
    std::atomic<bool> ok{true};
    parallel_for((int64_t)((order.size() + 4095) / 4096), [&](int64_t chunk) {
    Child ch[4];
    const size_t end = std::min(order.size(), (size_t)(chunk + 1) * 4096);
    for (size_t w = (size_t)chunk * 4096; w < end; w++) {
        const int n = collapse(nodes, order[w], ch);
        uint32_t* o = out->data() + w * 16;
        uint32_t exps = 0;
        for (int k = 0; k < 3; k++) {
            float lo[4], hi[4], origin = 0.0f;
            uint8_t qlo[4] = {0, 0, 0, 0}, qhi[4] = {0, 0, 0, 0};
            int be = 0;
            for (int c = 0; c < n; c++) {
                lo[c] = ch[c].lo[k];
                hi[c] = ch[c].hi[k];
            }
            if (!quantize_axis(lo, hi, n, &origin, &be, qlo, qhi)) {
                ok = false;
                return;
            }
            std::memcpy(&o[k], &origin, 4);
            exps |= (uint32_t)be << (8 * k);
            uint32_t wl = 0, wh = 0;
            for (int c = 0; c < 4; c++) {
                wl |= (uint32_t)qlo[c] << (8 * c);
                wh |= (uint32_t)qhi[c] << (8 * c);
            }
            o[4 + 2 * k] = wl;
            o[5 + 2 * k] = wh;
        }
        o[3] = exps;
        for (int c = 0; c < 4; c++) {
            int32_t ref = kEntrypointSentinel;
            if (c < n) ref = ch[c].ref >= 0 ? wideOf[(size_t)(ch[c].ref / 4)] * 4 : wide_leaf_ref(ch[c].ref, woopX, woopSlots);
            o[12 + c] = (uint32_t)ref;
        }
    }
    });
    if (!ok) out->clear();
    return ok;
}

std::vector<uint32_t> build_wide4(const int32_t* nodes, int64_t numNodes, const int32_t* woopX, int64_t woopSlots) {
    std::vector<uint32_t> out;
    if (numNodes <= 0) return out;
    // Pass 1: number the wide nodes depth first (binary node -> wide index).
    std::vector<int32_t> wideOf, order;
    number_wide(nodes, numNodes, wideOf, order);
    // Pass 2: write the nodes.
    out.assign(order.size() * 32, 0u);
    parallel_for((int64_t)((order.size() + 4095) / 4096), [&](int64_t chunk) {
    Child ch[4];
    const size_t end = std::min(order.size(), (size_t)(chunk + 1) * 4096);
    for (size_t w = (size_t)chunk * 4096; w < end; w++) {
        const int n = collapse(nodes, order[w], ch);
        uint32_t* o = out.data() + w * 32;
        for (int c = 0; c < 4; c++) {
            const int f4 = c >> 1, pair = (c & 1) * 2;   // children 0,1 in float4 0/2/4, 2,3 in 1/3/5
            // an absent child: NaN planes (every slab test of it fails) and the sentinel ref
            const float qnan = std::numeric_limits<float>::quiet_NaN();
            float lo[3] = {qnan, qnan, qnan}, hi[3] = {qnan, qnan, qnan};
            int32_t ref = kEntrypointSentinel;
            if (c < n) {
                for (int k = 0; k < 3; k++) {
                    lo[k] = ch[c].lo[k];
                    hi[k] = ch[c].hi[k];
                }
                ref = ch[c].ref >= 0 ? wideOf[(size_t)(ch[c].ref / 4)] * 8 : wide_leaf_ref(ch[c].ref, woopX, woopSlots);
            }
            for (int k = 0; k < 3; k++) {
                std::memcpy(&o[(2 * k + f4) * 4 + pair], &lo[k], 4);
                std::memcpy(&o[(2 * k + f4) * 4 + pair + 1], &hi[k], 4);
            }
            o[6 * 4 + c] = (uint32_t)ref;
        }
    }
    });
    return out;
}

}  // namespace mrt
