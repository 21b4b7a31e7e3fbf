// sbvh.cpp — spatial-split BVH builder.
//
// Restates the reference's SplitBVHBuilder (src/rt/bvh/SplitBVHBuilder.cc:55-485,
// Stich et al. 2009) including the parts that decide output bits: the
// order of the reference's median-3 quicksort (src/framework/base/Sort.cc:
// 63-239) with the (centroid sum, triIdx) comparator — a strict total order
// within a node, so std::sort reproduces it — the SAH tie-break on
// i^2 + (n-i)^2, degenerate-reference removal by swap-with-last, the 128-bin
// spatial search with float->int bin truncation, and the duplicate / unsplit
// decision. Where the reference kept one global reference stack and built the
// right child before the left one, this build gives every node its own copy
// of the segment it owns, which yields the same subtree bits and lets large
// subtrees build on separate threads.
#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "bvh.hpp"

namespace mrt {

namespace {

constexpr int kMaxDepth = 64;          // SplitBVHBuilder.hh:41-45
constexpr int kMaxSpatialDepth = 48;
constexpr int kNumSpatialBins = 128;
constexpr int kParallelMinRefs = 1024; // subtrees at least this large may run on their own thread
constexpr size_t kRadixSortRefs = 4096;  // nodes at least this large radix-sort their references
constexpr int kParallelBinRefs = 32768;  // nodes at least this large bin their spatial-split search on threads
constexpr int kBinThreads = 4;

struct Ref {
    int32_t triIdx = -1;
    AABB bounds;
};
struct NodeSpec {
    int numRef = 0;
    AABB bounds;
};
struct ObjectSplit {
    float sah = FLT_MAX;
    int sortDim = 0;
    int numLeft = 0;
    AABB leftBounds, rightBounds;
};
struct SpatialSplit {
    float sah = FLT_MAX;
    int dim = 0;
    float pos = 0.0f;
};
struct SpatialBin {
    AABB bounds;
    int enter = 0;
    int exit = 0;
    bool grown = false;   // bounds.grow() was called (an empty AABB grown in turns the bin infinite, as in the reference)
};

// (S32) of a float as x86-64 cvttss2si computes it: truncation, and the
// "integer indefinite" 0x80000000 for NaN and out-of-range values.
inline int trunc_to_int(float x) {
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT_MIN;
    return (int)x;
}
inline int clampi(int v, int lo, int hi) { return std::min(std::max(v, lo), hi); }

// FW::sort over a Ref array ordered by (min+max)[dim], then triIdx
// (SplitBVHBuilder.cc:75-84 with Sort.cc:63-239). Within one node every
// triangle has at most one reference (a spatial split sends a duplicated
// triangle's two halves to different children), so (key, triIdx) is a strict
// total order and the sorted permutation is unique: std::sort returns exactly
// the reference's median-3 quicksort result (checked by the builder's golden
// Compact2 fixtures and the per-scene hashes in tests/test_oracle.py).
void sort_refs(std::vector<Ref>& refs, int dim) {
    // The same order as 64-bit integer keys — the float key's order-preserving
    // bits (-0 folded into +0, which compares equal to it), then triIdx — with
    // the position as payload: 16-B records sort far faster than 28-B Refs with a
    // float add per compare. Large nodes: LSD radix sort (16-bit digits, passes
    // whose digit is constant skipped); small ones: std::sort.
    struct KeyPos { uint64_t key; uint32_t pos; };
    const size_t n = refs.size();
    if (n < 2) return;
    std::vector<KeyPos> a(n);
    for (size_t i = 0; i < n; i++) {
        float c = refs[i].bounds.mn[dim] + refs[i].bounds.mx[dim];
        c = c + 0.0f;   // -0 -> +0
        uint32_t u;
        std::memcpy(&u, &c, 4);
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        a[i] = {((uint64_t)u << 32) | (uint32_t)refs[i].triIdx, (uint32_t)i};
    }
    if (n < kRadixSortRefs) {
        std::sort(a.begin(), a.end(), [](const KeyPos& x, const KeyPos& y) { return x.key < y.key; });
    } else {
        std::vector<KeyPos> b(n);
        std::vector<uint32_t> count(1 << 16);
        for (int shift = 0; shift < 64; shift += 16) {
            std::fill(count.begin(), count.end(), 0u);
            for (size_t i = 0; i < n; i++) count[(a[i].key >> shift) & 0xFFFF]++;
            if (count[(a[0].key >> shift) & 0xFFFF] == n) continue;   // one digit value: the pass is the identity
            uint32_t sum = 0;
            for (uint32_t& c : count) { const uint32_t t = c; c = sum; sum += t; }
            for (size_t i = 0; i < n; i++) b[count[(a[i].key >> shift) & 0xFFFF]++] = a[i];
            a.swap(b);
        }
    }
    std::vector<Ref> out(n);
    for (size_t i = 0; i < n; i++) out[i] = refs[a[i].pos];
    refs.swap(out);
}

using Axes = std::array<std::vector<Ref>, 3>;

class Builder {
public:
    Builder(const Scene& s, const BuildParams& p) : sc_(s), p_(p) {
        // Default: OMP_NUM_THREADS when set (the GPU hosts export their CPU share
        // there; hardware_concurrency() counts the whole machine), else all cores.
        int threads = p.threads;
        if (threads <= 0) {
            const char* env = std::getenv("OMP_NUM_THREADS");
            threads = env ? std::atoi(env) : 0;
        }
        if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
        freeThreads_.store(std::max(0, threads - 1));
    }

    std::unique_ptr<BvhNode> run() {   // SplitBVHBuilder.cc:55-100
        NodeSpec root;
        std::vector<Ref> refs(sc_.triangles.size());
        for (size_t i = 0; i < refs.size(); i++) {
            refs[i].triIdx = (int32_t)i;
            const Vec3i& t = sc_.triangles[i];
            for (int j = 0; j < 3; j++) refs[i].bounds.grow(sc_.vertices[t[j]]);
            root.bounds.grow(refs[i].bounds);
        }
        root.numRef = (int)refs.size();
        minOverlap_ = root.bounds.area() * p_.splitAlpha;
        numTris_ = sc_.triangles.size();
        // The node's references sorted along each axis, kept through the splits
        // (a subset of a uniquely ordered array is ordered): three sorts in total
        // instead of four per node.
        Axes axes;
        for (int d = 0; d < 3; d++) axes[d] = refs;
        {
            std::thread tx([&] { sort_refs(axes[0], 0); });
            std::thread ty([&] { sort_refs(axes[1], 1); });
            sort_refs(axes[2], 2);
            tx.join();
            ty.join();
        }
        return build(std::move(refs), std::move(axes), root, 0);
    }

private:
    float tri_cost(int n) const {
        return (float)(((n + p_.triBatchSize - 1) / p_.triBatchSize) * p_.triBatchSize) * p_.sahTriangleCost;
    }
    float node_cost(int n) const {
        return (float)(((n + p_.nodeBatchSize - 1) / p_.nodeBatchSize) * p_.nodeBatchSize) * p_.sahNodeCost;
    }

    // SplitBVHBuilder.cc:113-174. `refs` is exactly the node's segment of the
    // reference's m_refStack, in the same order.
    std::unique_ptr<BvhNode> build(std::vector<Ref> refs, Axes axes, NodeSpec spec, int level) {
        // Remove degenerates (:120-129).
        std::vector<int32_t> removed;
        for (int i = (int)refs.size() - 1; i >= 0; i--) {
            const Vec3f size = refs[i].bounds.mx - refs[i].bounds.mn;
            if (size.min_comp() < 0.0f || size.sum() == size.max_comp()) {
                removed.push_back(refs[i].triIdx);
                refs[i] = refs.back();
                refs.pop_back();
            }
        }
        spec.numRef = (int)refs.size();
        if (!removed.empty()) {   // the same references leave the sorted arrays (triIdx is unique in a node)
            std::vector<uint8_t>& mark = marks();
            for (int32_t t : removed) mark[t] = 1;
            for (auto& a : axes)
                a.erase(std::remove_if(a.begin(), a.end(), [&](const Ref& r) { return mark[r.triIdx] != 0; }), a.end());
            for (int32_t t : removed) mark[t] = 0;
        }

        if (spec.numRef <= p_.minLeafSize || level >= kMaxDepth) return make_leaf(refs, spec);

        const float area = spec.bounds.area();
        const float leafSAH = area * tri_cost(spec.numRef);
        const float nodeSAH = area * node_cost(2);
        const ObjectSplit object = find_object_split(axes, nodeSAH);
        refs = axes[2];   // the reference's sweeps leave the node's references sorted along z

        SpatialSplit spatial;
        if (level < kMaxSpatialDepth) {
            AABB overlap = object.leftBounds;
            overlap.intersect(object.rightBounds);
            if (overlap.area() >= minOverlap_) spatial = find_spatial_split(refs, spec, nodeSAH);
        }

        const float minSAH = fw_min(fw_min(leafSAH, object.sah), spatial.sah);
        if (minSAH == leafSAH && spec.numRef <= p_.maxLeafSize) return make_leaf(refs, spec);

        NodeSpec left, right;
        if (minSAH == spatial.sah) perform_spatial_split(left, right, refs, spatial);
        if (!left.numRef || !right.numRef) {
            perform_object_split(left, right, refs, spec, object);
            refs = axes[object.sortDim];   // the sort's result: the node's references are the same set
        }

        std::vector<Ref> rightRefs(refs.begin() + left.numRef, refs.end());
        refs.resize(left.numRef);
        Axes leftAxes, rightAxes;
        split_axes(axes, refs, rightRefs, leftAxes, rightAxes);
        axes = Axes();

        auto node = std::make_unique<BvhNode>();
        node->bounds = spec.bounds;
        std::unique_ptr<BvhNode> rightNode;
        std::thread worker;
        if (right.numRef >= kParallelMinRefs && left.numRef >= kParallelMinRefs && take_thread()) {
            worker = std::thread([&, lvl = level + 1] { rightNode = build(std::move(rightRefs), std::move(rightAxes), right, lvl); });
        } else {
            rightNode = build(std::move(rightRefs), std::move(rightAxes), right, level + 1);
        }
        std::unique_ptr<BvhNode> leftNode = build(std::move(refs), std::move(leftAxes), left, level + 1);
        if (worker.joinable()) {
            worker.join();
            freeThreads_.fetch_add(1);
        }
        node->child[0] = std::move(leftNode);
        node->child[1] = std::move(rightNode);
        return node;
    }

    bool take_thread() {
        int f = freeThreads_.load();
        while (f > 0)
            if (freeThreads_.compare_exchange_weak(f, f - 1)) return true;
        return false;
    }

    // createLeaf (:178-187): triangles in m_refStack.removeLast() order.
    std::unique_ptr<BvhNode> make_leaf(const std::vector<Ref>& refs, const NodeSpec& spec) {
        auto leaf = std::make_unique<BvhNode>();
        leaf->bounds = spec.bounds;
        leaf->tris.reserve(refs.size());
        for (int i = (int)refs.size() - 1; i >= 0; i--) leaf->tris.push_back(refs[i].triIdx);
        return leaf;
    }

    // findObjectSplit (:191-231): per axis, a right-to-left bound sweep over the
    // references in sorted order (kept sorted through the splits, see run()).
    ObjectSplit find_object_split(const Axes& axes, float nodeSAH) const {
        ObjectSplit split;
        const int n = (int)axes[0].size();
        float bestTieBreak = FLT_MAX;
        std::vector<AABB> rightBounds(std::max(n - 1, 1));
        for (int dim = 0; dim < 3; dim++) {
            const std::vector<Ref>& sorted = axes[dim];
            AABB rb;
            for (int i = n - 1; i > 0; i--) {
                rb.grow(sorted[i].bounds);
                rightBounds[i - 1] = rb;
            }
            AABB lb;
            for (int i = 1; i < n; i++) {
                lb.grow(sorted[i - 1].bounds);
                const float sah = nodeSAH + lb.area() * tri_cost(i) + rightBounds[i - 1].area() * tri_cost(n - i);
                const float tieBreak = (float)i * (float)i + (float)(n - i) * (float)(n - i);
                if (sah < split.sah || (sah == split.sah && tieBreak < bestTieBreak)) {
                    split.sah = sah;
                    split.sortDim = dim;
                    split.numLeft = i;
                    split.leftBounds = lb;
                    split.rightBounds = rightBounds[i - 1];
                    bestTieBreak = tieBreak;
                }
            }
        }
        return split;
    }

    // The children's sorted arrays. A reference that went to one side whole keeps
    // its bounds, hence its key, and its place in each parent array (a stable
    // partition); the two clipped halves of a duplicated triangle get new keys
    // and are sorted in and merged.
    void split_axes(const Axes& axes, const std::vector<Ref>& leftRefs, const std::vector<Ref>& rightRefs,
                    Axes& leftAxes, Axes& rightAxes) {
        std::vector<uint8_t>& mark = marks();   // bit 0: on the left, bit 1: on the right
        for (const Ref& r : leftRefs) mark[r.triIdx] |= 1;
        for (const Ref& r : rightRefs) mark[r.triIdx] |= 2;
        std::vector<Ref> dupLeft, dupRight;
        for (const Ref& r : leftRefs)
            if (mark[r.triIdx] == 3) dupLeft.push_back(r);
        for (const Ref& r : rightRefs)
            if (mark[r.triIdx] == 3) dupRight.push_back(r);
        for (int d = 0; d < 3; d++) {
            std::vector<Ref> l, rr;
            l.reserve(leftRefs.size());
            rr.reserve(rightRefs.size());
            for (const Ref& r : axes[d]) {
                const uint8_t m = mark[r.triIdx];
                if (m == 1) l.push_back(r);
                else if (m == 2) rr.push_back(r);
            }
            merge_sorted(l, dupLeft, d, leftAxes[d]);
            merge_sorted(rr, dupRight, d, rightAxes[d]);
        }
        for (const Ref& r : leftRefs) mark[r.triIdx] = 0;
        for (const Ref& r : rightRefs) mark[r.triIdx] = 0;
    }

    static void merge_sorted(std::vector<Ref>& base, std::vector<Ref> extra, int dim, std::vector<Ref>& out) {
        if (extra.empty()) {
            out = std::move(base);
            return;
        }
        sort_refs(extra, dim);
        out.resize(base.size() + extra.size());
        std::merge(base.begin(), base.end(), extra.begin(), extra.end(), out.begin(), [dim](const Ref& a, const Ref& b) {
            const float ca = a.bounds.mn[dim] + a.bounds.mx[dim];
            const float cb = b.bounds.mn[dim] + b.bounds.mx[dim];
            return ca < cb || (ca == cb && a.triIdx < b.triIdx);
        });
    }

    // Per-thread scratch indexed by triIdx, all zero between uses.
    std::vector<uint8_t>& marks() {
        thread_local std::vector<uint8_t> m;
        if (m.size() < numTris_) m.assign(numTris_, 0);
        return m;
    }

    // performObjectSplit (:235-245).
    void perform_object_split(NodeSpec& left, NodeSpec& right, std::vector<Ref>& refs, const NodeSpec& spec,
                              const ObjectSplit& split) const {
        (void)refs;   // the node's references sorted along split.sortDim are the caller's axes[sortDim]
        left.numRef = split.numLeft;
        left.bounds = split.leftBounds;
        right.numRef = spec.numRef - split.numLeft;
        right.bounds = split.rightBounds;
    }

    // findSpatialSplit (:249-327).
    SpatialSplit find_spatial_split(const std::vector<Ref>& refs, const NodeSpec& spec, float nodeSAH) const {
        const Vec3f origin = spec.bounds.mn;
        const Vec3f binSize = (spec.bounds.mx - origin) * (1.0f / (float)kNumSpatialBins);
        const Vec3f invBinSize(1.0f / binSize.x, 1.0f / binSize.y, 1.0f / binSize.z);

        // Binning (the search's cost: one splitReference per bin plane a reference
        // crosses). Bin bounds are min/max unions and the counts sums, so any
        // partition of the references gives the same bins: large nodes bin in
        // chunks on their own threads and merge.
        auto bin_refs = [&](size_t begin, size_t end, std::vector<SpatialBin>& out) {
            out.assign(3 * kNumSpatialBins, SpatialBin());
            for (size_t k = begin; k < end; k++) {
                const Ref& ref = refs[k];
                const Vec3f lo = (ref.bounds.mn - origin) * invBinSize;
                const Vec3f hi = (ref.bounds.mx - origin) * invBinSize;
                int firstBin[3], lastBin[3];
                for (int d = 0; d < 3; d++) {
                    firstBin[d] = clampi(trunc_to_int(lo[d]), 0, kNumSpatialBins - 1);
                    lastBin[d] = clampi(trunc_to_int(hi[d]), firstBin[d], kNumSpatialBins - 1);
                }
                for (int dim = 0; dim < 3; dim++) {
                    Ref curr = ref;
                    for (int i = firstBin[dim]; i < lastBin[dim]; i++) {
                        Ref l, r;
                        split_reference(l, r, curr, dim, origin[dim] + binSize[dim] * (float)(i + 1));
                        out[dim * kNumSpatialBins + i].bounds.grow(l.bounds);
                        out[dim * kNumSpatialBins + i].grown = true;
                        curr = r;
                    }
                    out[dim * kNumSpatialBins + lastBin[dim]].bounds.grow(curr.bounds);
                    out[dim * kNumSpatialBins + lastBin[dim]].grown = true;
                    out[dim * kNumSpatialBins + firstBin[dim]].enter++;
                    out[dim * kNumSpatialBins + lastBin[dim]].exit++;
                }
            }
        };
        std::vector<SpatialBin> bins;
        const size_t n = refs.size();
        const int chunks = n >= (size_t)kParallelBinRefs ? kBinThreads : 1;
        if (chunks == 1) {
            bin_refs(0, n, bins);
        } else {
            std::vector<std::vector<SpatialBin>> part(chunks);
            std::vector<std::thread> th;
            for (int c = 1; c < chunks; c++) th.emplace_back(bin_refs, n * c / chunks, n * (c + 1) / chunks, std::ref(part[c]));
            bin_refs(0, n / chunks, part[0]);
            for (auto& t : th) t.join();
            bins = std::move(part[0]);
            for (int c = 1; c < chunks; c++)
                for (size_t b = 0; b < bins.size(); b++) {
                    if (part[c][b].grown) {   // an untouched chunk bin is the empty AABB: growing by it is not a no-op
                        bins[b].bounds.grow(part[c][b].bounds);
                        bins[b].grown = true;
                    }
                    bins[b].enter += part[c][b].enter;
                    bins[b].exit += part[c][b].exit;
                }
        }
        auto bin = [&](int dim, int i) -> SpatialBin& { return bins[dim * kNumSpatialBins + i]; };

        SpatialSplit split;
        AABB rightBounds[kNumSpatialBins - 1];
        for (int dim = 0; dim < 3; dim++) {
            AABB rb;
            for (int i = kNumSpatialBins - 1; i > 0; i--) {
                rb.grow(bin(dim, i).bounds);
                rightBounds[i - 1] = rb;
            }
            AABB lb;
            int leftNum = 0;
            int rightNum = spec.numRef;
            for (int i = 1; i < kNumSpatialBins; i++) {
                lb.grow(bin(dim, i - 1).bounds);
                leftNum += bin(dim, i - 1).enter;
                rightNum -= bin(dim, i - 1).exit;
                const float sah = nodeSAH + lb.area() * tri_cost(leftNum) + rightBounds[i - 1].area() * tri_cost(rightNum);
                if (sah < split.sah) {
                    split.sah = sah;
                    split.dim = dim;
                    split.pos = origin[dim] + binSize[dim] * (float)i;
                }
            }
        }
        return split;
    }

    // performSpatialSplit (:331-421).
    void perform_spatial_split(NodeSpec& left, NodeSpec& right, std::vector<Ref>& refs, const SpatialSplit& split) const {
        const int leftStart = 0;
        int leftEnd = leftStart;
        int rightStart = (int)refs.size();
        left.bounds = right.bounds = AABB();

        for (int i = leftEnd; i < rightStart; i++) {
            if (refs[i].bounds.mx[split.dim] <= split.pos) {   // entirely left
                left.bounds.grow(refs[i].bounds);
                std::swap(refs[i], refs[leftEnd++]);
            } else if (refs[i].bounds.mn[split.dim] >= split.pos) {   // entirely right
                right.bounds.grow(refs[i].bounds);
                std::swap(refs[i], refs[--rightStart]);
                i--;
            }
        }

        while (leftEnd < rightStart) {   // straddlers: duplicate or unsplit
            Ref lref, rref;
            split_reference(lref, rref, refs[leftEnd], split.dim, split.pos);

            AABB lub = left.bounds, rub = right.bounds, ldb = left.bounds, rdb = right.bounds;
            lub.grow(refs[leftEnd].bounds);
            rub.grow(refs[leftEnd].bounds);
            ldb.grow(lref.bounds);
            rdb.grow(rref.bounds);

            const int size = (int)refs.size();
            const float lac = tri_cost(leftEnd - leftStart);
            const float rac = tri_cost(size - rightStart);
            const float lbc = tri_cost(leftEnd - leftStart + 1);
            const float rbc = tri_cost(size - rightStart + 1);

            const float unsplitLeftSAH = lub.area() * lbc + right.bounds.area() * rac;
            const float unsplitRightSAH = left.bounds.area() * lac + rub.area() * rbc;
            const float duplicateSAH = ldb.area() * lbc + rdb.area() * rbc;
            const float minSAH = fw_min(fw_min(unsplitLeftSAH, unsplitRightSAH), duplicateSAH);

            if (minSAH == unsplitLeftSAH) {
                left.bounds = lub;
                leftEnd++;
            } else if (minSAH == unsplitRightSAH) {
                right.bounds = rub;
                std::swap(refs[leftEnd], refs[--rightStart]);
            } else {
                left.bounds = ldb;
                right.bounds = rdb;
                refs[leftEnd++] = lref;
                refs.push_back(rref);
            }
        }
        left.numRef = leftEnd - leftStart;
        right.numRef = (int)refs.size() - rightStart;
    }

    // splitReference (:425-470).
    void split_reference(Ref& left, Ref& right, const Ref& ref, int dim, float pos) const {
        left.triIdx = right.triIdx = ref.triIdx;
        left.bounds = right.bounds = AABB();
        const Vec3i& inds = sc_.triangles[ref.triIdx];
        const Vec3f* v1 = &sc_.vertices[inds.z];
        for (int i = 0; i < 3; i++) {
            const Vec3f* v0 = v1;
            v1 = &sc_.vertices[inds[i]];
            const float v0p = (*v0)[dim];
            const float v1p = (*v1)[dim];
            if (v0p <= pos) left.bounds.grow(*v0);
            if (v0p >= pos) right.bounds.grow(*v0);
            if ((v0p < pos && v1p > pos) || (v0p > pos && v1p < pos)) {
                const float t = fw_min(fw_max((pos - v0p) / (v1p - v0p), 0.0f), 1.0f);
                const float s = 1.0f - t;
                const Vec3f p((*v0).x * s + (*v1).x * t, (*v0).y * s + (*v1).y * t, (*v0).z * s + (*v1).z * t);
                left.bounds.grow(p);
                right.bounds.grow(p);
            }
        }
        left.bounds.mx[dim] = pos;
        right.bounds.mn[dim] = pos;
        left.bounds.intersect(ref.bounds);
        right.bounds.intersect(ref.bounds);
    }

    const Scene& sc_;
    const BuildParams& p_;
    float minOverlap_ = 0.0f;
    size_t numTris_ = 0;
    std::atomic<int> freeThreads_{0};
};

void collect_stats(const BvhNode& n, int depth, float rootArea, const BuildParams& p, BvhStats& s) {
    s.maxDepth = std::max<int64_t>(s.maxDepth, depth);
    const float prob = rootArea > 0.0f ? n.bounds.area() / rootArea : 0.0f;
    if (n.is_leaf()) {
        s.leafNodes++;
        s.triRefs += (int64_t)n.tris.size();
        s.sahCost += prob * (float)n.tris.size() * p.sahTriangleCost;
        return;
    }
    s.innerNodes++;
    s.sahCost += prob * 2.0f * p.sahNodeCost;
    collect_stats(*n.child[0], depth + 1, rootArea, p, s);
    collect_stats(*n.child[1], depth + 1, rootArea, p, s);
}

}  // namespace

std::unique_ptr<BvhNode> build_sbvh(const Scene& scene, const BuildParams& params, BvhStats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    Builder b(scene, params);
    std::unique_ptr<BvhNode> root = b.run();
    if (stats) {
        *stats = BvhStats();
        collect_stats(*root, 0, root->bounds.area(), params, *stats);
        stats->buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return root;
}

}  // namespace mrt
