// trace_kernel.hpp — launch interface between the C-ABI glue (mrt_api.cpp)
// and the gfx950 traversal kernels (trace_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

namespace mrt {

// Bottom-of-stack marker; the traversal ends when it is popped
// (reference CudaTracerKernels.hh:107-111 EntrypointSentinel).
constexpr int kEntrypointSentinel = 0x76543210;

// Total per-lane stack capacity (reference STACK_SIZE 64,
// kepler_dynamic_fetch.cu:47). The top kLdsStack entries live in LDS, the
// rest spill to a per-lane slab in HBM.
constexpr int kStackCapacity = 64;
constexpr int kMaxQueues = 8;
constexpr int kQueueStrideWords = 64;      // one 256-B line per queue head
#ifndef MRT_BLOCK_THREADS
#define MRT_BLOCK_THREADS 256
#endif
constexpr int kBlockThreads = MRT_BLOCK_THREADS;   // wave64s per workgroup x 64 (default 4 waves)
// Queue heads: kMaxQueues per-XCD heads, the shared queue's head and the served mask (bit q:
// some wave has taken from queue q), one 256-B line each, zeroed per launch.
constexpr int kServedLine = kMaxQueues + 1;
constexpr int kQueueLines = kMaxQueues + 2;
// Largest node / woop buffer a tracer binds (32-bit buffer offsets).
constexpr int64_t kMaxBufferBytes = 0xFFFFFFC0ll;

// Everything one launch needs; passed by value as the kernel argument.
struct TraceArgs {
    const float4* rays;        // Ray[n] as 2 x float4
    int2* results;             // RayResult[n] viewed as int2 pairs; slot 2*i = {id, t}
    const float4* nodes;       // Compact2 nodes
    const float4* woop;        // Woop triangles
    const int* triIndex;       // remap table
    uint32_t nodeBytes;        // buffer-resource ranges (range-checked loads)
    uint32_t woopBytes;
    int numRays;
    int numQueues;             // 1..8 ray queues (per-XCD heads)
    int sharedRays;            // numQueues > 1: the batch's last rays in one queue every XCD's waves take
                               // from once their own queue is dry (head kMaxQueues)
    int queueBlockLog2;        // numQueues > 1: 0 = contiguous shares, k = 2^k-ray blocks dealt cyclically
    int fetchThreshold;        // refill when fewer live lanes than this
    int specSlack;             // speculative: leave the node loop once <= this many lanes lack a leaf
    int staticRounds;          // queue modes: static strided rounds of the grid before the queues
    int wideLeafCounts;        // the wide leaf refs carry triangle counts (wide_bvh.cpp)
    int laneGroupsLog2;        // strided mode: a wave's lanes take rays from 2^k spread-out sub-ranges
    int totalLanes;            // grid lanes (stride of the spill slab)
    int stackCap;              // stack entries incl. the sentinel (kStackCapacity, or the wide tree's bound)
    int stackBound;            // entries (sentinel excluded) a depth-first walk of the bound tree can hold
                               // (wide_stack_bound; stackCap - 1 for the binary order): the frontier tail
                               // keeps this much headroom before it expands more than one entry per step
    int tailLanes;            // exact 4-wide speculative kernels: a wave that cannot refill and is down to
                               // this many live lanes finishes them in the frontier tail (0 = off)
    int raySort;               // cfg.ray_sort: a one-round static launch deals each workgroup's 256-ray tile
                               // to its waves by direction octant (exact 4-wide kernels)
    int xccMask;               // test hook (cfg.queue_xcc_mask): > 0 = a wave's queue is (XCC_ID & mask) %
                               // numQueues, so the queues above mask have no waves of their own
    unsigned* queues;          // numQueues heads, kQueueStrideWords apart, zeroed per launch
    int* spill;                // (stackCap - S) * totalLanes ints
    int* status;               // [0] = stack overflow count (entries pushed past stackCap)
    int4* stats;               // per-ray {nodes, tris, leaves, 0} (STATS variants)
};

// Node formats the traversal reads (wide_bvh.cpp): the bound Compact2 nodes, or
// the 4-wide nodes derived from them at bind time, exact (128 B) or quantized (64 B).
enum : int { kNodeCompact2 = 0, kNodeWide4 = 1, kNodeWide4Q = 2 };

// Variant selector (all combinations are instantiated in trace_kernel.hip).
struct TraceVariant {
    bool anyHit;
    bool speculative;   // reference warp-wide postponement (ballot) vs per-lane
    bool exactRcp;      // IEEE 1/x vs v_rcp_f32
    bool stats;
    int ldsStack;       // 8, 16 or 32 LDS entries per lane
    int nodes = 0;      // kNodeCompact2, or a 4-wide form derived from it (speculative mode only)
    bool tail = false;  // kNodeWide4 with leaf counts: the instantiation with the frontier tail
};

// The 4-wide node array derived from a Compact2 node array (numNodes inner nodes,
// 16 int32 each): 32 uint32 (128 B) per wide node, layout in wide_bvh.cpp.
// woopX (the first word of each of woopSlots Woop slots, or null): with it the
// leaf refs carry their triangle counts (wide_bvh.cpp); pass it only when
// leaf_counts_fit(woopSlots) (woop indices below 2^27).
constexpr int kWideLeafAddrBits = 27;
bool leaf_counts_fit(int64_t woopSlots);
std::vector<uint32_t> build_wide4(const int32_t* nodes, int64_t numNodes, const int32_t* woopX = nullptr,
                                  int64_t woopSlots = 0);
// The most stack entries (sentinel excluded) a traversal of a 4-wide node array
// can hold: the maximum over nodes of the pushes of all their ancestors plus
// their own (each node pushes all but one of its children when every child is
// hit, and any child may be the one visited first). nodeWords: 32 (exact form)
// or 16 (quantized).
int64_t wide_stack_bound(const uint32_t* wide, int64_t numWide, int nodeWords);
// The quantized 4-wide form: 16 uint32 (64 B) per wide node. False (and no
// output) when some child box has no finite quantization (non-finite planes).
bool build_wide4q(const int32_t* nodes, int64_t numNodes, std::vector<uint32_t>* out, const int32_t* woopX = nullptr,
                  int64_t woopSlots = 0);

// Launch one persistent trace. grid = number of 256-thread workgroups.
hipError_t launch_trace(const TraceVariant& v, const TraceArgs& a, int gridBlocks, hipStream_t s);

// Resident 256-thread workgroups per CU for a variant (occupancy query).
hipError_t trace_occupancy(const TraceVariant& v, int* blocksPerCU);

// Static facts about a variant's code object (for occupancy sizing/reporting).
hipError_t trace_kernel_attributes(const TraceVariant& v, hipFuncAttributes* attr);

// Exhaustive check of the EXACT variants' reciprocal against 1.0f / x (all 2^32
// inputs); adds the number of mismatching bit patterns to *mismatchesDev.
hipError_t selftest_exact_rcp(unsigned long long* mismatchesDev, hipStream_t s);

// Thread-local error detail behind mrt_last_error_detail() (csrc/mrt_api.cpp).
int api_fail(int code, const std::string& what);
const char* api_last_error();

}  // namespace mrt
