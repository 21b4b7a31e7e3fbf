// mrt_api.cpp — the C-ABI of include/mrt.h: per-device tracer contexts, the
// persistent-grid sizing, the workspace (queue heads, stack spill slab) and
// the reference-compatible entry points of CudaTracerKernels.hh:42-52.
//
// The library never owns the caller's BVH/ray/result buffers (reference
// ownership: CudaBVH.cc:101-109, RayBuffer.cc:42-81). It owns only its
// workspace, sized for the persistent grid it launches.
#include <hip/hip_runtime.h>
#include <climits>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mrt.h"
#include "trace_kernel.hpp"

namespace mrt {
struct Workspace;
}

struct mrt_tracer {
    int device = 0;
    int numCUs = 0;
    int numXccs = 1;   // XCDs of the device (partition): the per-XCD queue candidate's queue count
    std::mutex mu;

    // Bound Compact2 BVH (borrowed device pointers).
    bool bound = false;
    const void* nodes = nullptr;
    int64_t nodeBytes = 0;
    const void* woop = nullptr;
    int64_t woopBytes = 0;
    const int32_t* triIndex = nullptr;
    int64_t triIndexBytes = 0;

    mrt_launch_cfg cfg{};

    // 4-wide nodes derived from the bound Compact2 tree (cfg.wide; wide_bvh.cpp),
    // owned by the tracer and rebuilt when the BVH or the setting changes.
    void* wideNodes = nullptr;
    int64_t wideBytes = 0;
    int wideBuiltFor = -1;   // the cfg.wide value the current array was built for
    int wideFormat = mrt::kNodeCompact2;   // the form wideNodes holds (kNodeWide4 / kNodeWide4Q)
    bool wideLeafCounts = false;           // its leaf refs carry triangle counts
    // Stack entries (sentinel included) the wide traversal gets: the wide tree's
    // worst case (wide_stack_bound) + 1, at least the reference's 64. A wide node
    // pushes up to three children where the binary step pushes one, so a tree that
    // fits the reference's stack in binary order could otherwise overflow in wide
    // order; sized this way no ray of the bound tree can overflow it.
    int wideStackCap = mrt::kStackCapacity;
    int wideStackBound = mrt::kStackCapacity - 1;   // wide_stack_bound of the derived tree (the tail's headroom)
    double bindMs = 0.0;                   // wall time of the last bind / wide derivation (mrt_trace_info)

    // Launch scratch, one set per stream the handle has launched on: the stack
    // spill slab, the queue heads and the overflow counter are written by a
    // running trace, so two traces in flight on different streams must not
    // share them (the handle's mutex only covers enqueueing).
    std::vector<mrt::Workspace*> workspaces;
    uint64_t useClock = 0;   // launches of this handle (the workspaces' LRU order; guarded by mu)
    hipEvent_t evStart = nullptr, evStop = nullptr;

    // Occupancy per kernel variant (index variant_key(), below 256), queried once
    // (hipOccupancy* is a host round-trip that would otherwise sit on every launch).
    int occ[512] = {};

    // cfg.autotune: per (batch size, variant) the ray-distribution schedule the
    // measured launches chose (mrt_api.cpp autotune_*), reset on bind/set_config.
    std::map<std::pair<int, int>, struct TuneState*> tunes;
};

// Launch-schedule autotuning state of one (batch size, kernel variant).
struct TuneState {
    // Stage 1: kSchedules ray-distribution schedules; stage 2: the stage-1 winner and
    // the runner-up, each with the speculation slack at 4 and 6, without the frontier
    // tail (with it if the tracer's default is off), with 16 lane groups, and with 2
    // lane groups at slack 6 (candidates kSchedules .. + kStage2 - 1 modify the winner,
    // the next kStage2 the runner-up; a settled choice is stored canonically as modifier
    // kSchedules + k of the schedule it modifies, so saved tables keep their meaning).
    // Stage 3: the stage-2 winner's modifier on each other schedule (kStage3 candidates from
    // kStage3First): e.g. 16 lane groups paid off at 16 waves/CU though the two stage-1 leaders
    // were 20 and 12 waves/CU (bunny primary 640x480).
    static constexpr int kSchedules = 8;
    static constexpr int kStage2 = 5;
    static constexpr int kStage3First = kSchedules + 2 * kStage2;
    static constexpr int kStage3 = kSchedules - 2;
    static constexpr int kCandidates = kStage3First + kStage3;
    static constexpr int kSamples = 8;   // timed launches per candidate; the median ranks them
    // A candidate runs kRun consecutive launches at a time, the first untimed: a launch right
    // after another schedule's inherits its cache and queue state (round 6: one launch per
    // candidate ranked a 42-us batch's schedules 3.5 % off their steady-state order).
    static constexpr int kRun = 4;
    int launches = 0;    // exploring launches so far (the first round of candidates runs untimed:
                         // the clocks and caches are still settling)
    int runPos = 0;      // position of the next launch in its candidate's run
    float times[kCandidates][kSamples];
    int samples[kCandidates] = {};
    int next = 0;        // candidate the next exploring launch uses
    int rule = 0;        // the candidate equal to the fixed rule (effective_cfg) for this batch
    int stage1 = -1;     // the stage-1 winner, once every schedule has kSamples samples (once locked:
                         // the schedule the locked modifier applies to)
    int stage1b = -1;    // the stage-1 runner-up (stage 2 modifies it too; VERDICT r5 #4: the headline's
                         // saved schedule is the 8-waves/CU schedule with 2 lane groups, whose base
                         // alone loses to 20 waves/CU in stage 1)
    int stage2 = -1;     // the stage-2 pick (a modifier of stage1 or stage1b), once stage 2's have kSamples
    int s3mod = -1;      // its modifier k, tried on the schedules in s3sched (stage 3)
    int s3sched[kStage3] = {};
    int locked = -1;     // the chosen candidate (canonical: kSchedules + k of stage1), once settled
    void* stream = nullptr;          // the stream this batch size was first launched on
    bool multiStream = false;        // launched on several streams: not explored (settled schedule or the rule)
    bool inherited = false;          // took a nearby batch size's schedule (kTuneInherit): not exported
    struct Pending {
        hipEvent_t start = nullptr, stop = nullptr;
        int cand = -1;   // -1 = slot free
    } pending[16];   // launches in flight with a timing (back-to-back launches complete later)
    float median(int c) const {
        float v[kSamples];
        const int n = std::min(samples[c], kSamples);
        std::copy(times[c], times[c] + n, v);
        std::sort(v, v + n);
        return n ? (n % 2 ? v[n / 2] : 0.5f * (v[n / 2 - 1] + v[n / 2])) : 1e30f;
    }
};

namespace mrt {
namespace {
thread_local std::string g_lastError;
}  // namespace

// Shared with the ray-generation entry points (csrc/raygen_kernel.hip).
int api_fail(int code, const std::string& what) {
    g_lastError = what;
    return code;
}
const char* api_last_error() { return g_lastError.c_str(); }

struct Workspace {
    void* stream = nullptr;       // the hipStream_t this scratch was last used on
    unsigned* queues = nullptr;   // kMaxQueues * kQueueStrideWords words
    int* status = nullptr;        // [0] = stack overflows of asynchronous launches since the last reset
                                  // (sticky); [kTimedSlot] = the current blocking launch's own count
    int* spill = nullptr;
    size_t spillInts = 0;
    // -DMRT_DONE_EVENT: recorded after every launch that uses this scratch, so waiting
    // for it never touches the stream (see workspace_wait)
    hipEvent_t done = nullptr;
    bool launched = false;        // a launch may still be using this scratch
    uint64_t lastUse = 0;         // launch counter value of the last use (LRU reuse)
};
constexpr int kTimedSlot = 16;    // a separate 64-B line of Workspace::status
// The per-launch completion event only tells the host that the launch has finished
// (workspace reuse, destroy, overflow reads): no system-scope fence, which would
// write back and invalidate the caches between back-to-back launches.
#ifdef MRT_DONE_EVENT
#ifndef MRT_DONE_EVENT_FLAGS
#define MRT_DONE_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
constexpr unsigned kDoneEventFlags = MRT_DONE_EVENT_FLAGS;
#endif
// Events that only time launches (the autotuner's, the blocking call's start).
#ifndef MRT_TIMING_EVENT_FLAGS
#define MRT_TIMING_EVENT_FLAGS hipEventDisableSystemFence
#endif
constexpr unsigned kTimingEventFlags = MRT_TIMING_EVENT_FLAGS;
// Scratch sets per handle: a trace on a new stream reuses the least recently used
// set (after its last launch has completed) once this many exist.
constexpr int kMaxWorkspaces = 8;
}  // namespace mrt

namespace {

int fail(int code, const std::string& what) { return mrt::api_fail(code, what); }

int hipFail(hipError_t e, const char* what) {
    return fail(MRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define MRT_HIP(call)                                  \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) return hipFail(e_, #call); \
    } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// The production (speculative) traversal reads 4-wide nodes derived at bind time
// (profiles/round2_tuning.md, "4-wide nodes").
constexpr int kDefaultWide = 1;
// The speculative traversal turns to its leaves once at most two lanes of the
// wave still search for one, instead of waiting for the last lane (reference
// kepler_dynamic_fetch.cu:300-315): +3...+9 % on primary, diffuse and AO batches,
// -3 % on AO 1280x960 (profiles/round2_tuning.md).
constexpr int kDefaultSpecSlack = 2;
// Launch schedules are tuned per batch size (autotune_*, below): equal or faster on
// every workload once settled (+9...+16 % on bunny/dragon primary batches).
constexpr int kDefaultAutotune = 1;
// The frontier tail (trace_kernel.hip frontier_tail): a wave that cannot refill and is
// down to at most this many live lanes finishes them 64/R lanes per ray. On by default:
// hairball diffuse 640x480 0.314 -> 0.225 ms, Mori AO 0.055 -> 0.044, bunny primary
// +5 %; conference AO and sponza diffuse lose 2-4 % (profiles/round3_frontier_ab.txt),
// where the autotuner's stage 2 can turn it off.
#ifndef MRT_DEFAULT_TAIL_LANES
#define MRT_DEFAULT_TAIL_LANES 16
#endif
// Lane groups the autotuner's stage 2 tries (profiles/round3_lanegroups.txt).
constexpr int kTunedLaneGroups = 16;
// What the autotuner's stage 2 tries when tail_lanes is left at its default (16: off).
constexpr int kTunedTailLanes = 16;
constexpr int kDefaultTailLanes = MRT_DEFAULT_TAIL_LANES;

mrt_launch_cfg default_cfg() {
    mrt_launch_cfg c;
    c.waves_per_cu = 0;   // auto: sized from the batch (grid_blocks)
    c.fetch_threshold = 0;   // strided mode: a wave refills once all its lanes are done
    c.num_queues = -1;       // static strided assignment (see trace_kernel.hip); 1..8 = atomic queues
    c.lds_stack = 16;
    c.lane_groups = 1;
    c.wide = kDefaultWide;
    c.spec_slack = kDefaultSpecSlack;
    c.static_rounds = 1;
    c.autotune = kDefaultAutotune;
    c.tail_lanes = kDefaultTailLanes;
    c.queue_shared = 0;
    c.queue_block = 0;
    c.ray_sort = 0;
    c.queue_xcc_mask = 0;
    return c;
}

bool valid_cfg(const mrt_launch_cfg& c) {
    return (c.waves_per_cu == 0 || (c.waves_per_cu >= 4 && c.waves_per_cu <= 32)) && c.fetch_threshold >= 0 && c.fetch_threshold <= 64 &&
           (c.num_queues == -1 || (c.num_queues >= 1 && c.num_queues <= mrt::kMaxQueues)) &&
           (c.lds_stack == 8 || c.lds_stack == 16 || c.lds_stack == 32) &&
           c.lane_groups >= 1 && c.lane_groups <= 64 && (c.lane_groups & (c.lane_groups - 1)) == 0 &&
           (c.wide >= 0 && c.wide <= 2) && c.spec_slack >= 0 && c.spec_slack <= 63 &&
           c.static_rounds >= 1 && c.static_rounds <= 64 && (c.autotune == 0 || c.autotune == 1) &&
           c.tail_lanes >= 0 && c.tail_lanes <= 16 &&
           c.queue_shared >= 0 && c.queue_shared <= 100 && c.queue_block >= 0 && c.queue_block <= (1 << 20) &&
           (c.queue_block & (c.queue_block - 1)) == 0 && (c.queue_block == 0 || c.queue_block >= 64) &&
           c.queue_xcc_mask >= 0 && c.queue_xcc_mask <= 15 && (c.ray_sort == 0 || c.ray_sort == 1);
}

// The frontier tail runs in the exact 4-wide kernels whose leaf refs carry counts.
bool with_tail(const mrt_tracer* t, const mrt::TraceVariant& v, const mrt_launch_cfg& c) {
    return c.tail_lanes > 0 && v.nodes == mrt::kNodeWide4 && t->wideLeafCounts;
}

mrt::TraceVariant variant_for(const mrt_tracer* t, uint32_t flags) {
    mrt::TraceVariant v;
    v.anyHit = (flags & MRT_TRACE_ANY_HIT) != 0;
    v.exactRcp = (flags & MRT_TRACE_EXACT_RCP) != 0;
    v.speculative = (flags & MRT_TRACE_LOCKSTEP_OFF) == 0;
    v.stats = (flags & MRT_TRACE_STATS) != 0;
    v.ldsStack = t->cfg.lds_stack;
    // The per-lane (lockstep-off) order is the reference's binary order: it keeps
    // the Compact2 nodes, and with them the oracle's exact per-ray counters.
    v.nodes = (t->cfg.wide != 0 && t->wideNodes != nullptr && v.speculative) ? t->wideFormat : mrt::kNodeCompact2;
    v.tail = with_tail(t, v, t->cfg);
    return v;
}

// Rays per lane the automatic grid aims for: a frame-sized batch is bound by
// its slowest rays, whose step latency grows with the number of co-resident
// waves, so small batches get fewer waves per CU; big batches fill the CU.
// Measured on MI355X (tools/sweep.py, profiles/round1_sweep.txt): batches that
// fit one ray per lane at 32 waves/CU run fastest fully static (conference AO
// 640x480: 0.061 ms vs 0.077 at 8 waves); above that, 8 waves/CU is best up to
// ~1M rays (bunny primary 1024x768), 16 at 3M, 32 at 12M rays.
constexpr int kAutoRaysPerLane = 12;
// Static strided rounds: 20 waves/CU (5 per SIMD). More resident waves evict
// each other's nodes and triangles from the vector L1 (28 waves/CU: hairball
// -22 %, profiles/round2_tuning.md); the register budget of the 4-wide kernels
// is sized for exactly this occupancy.
constexpr int kStridedWaves = 20;
constexpr int kAutoMinWaves = 8;

// Persistent grid: as many 256-thread workgroups per CU as the config asks for
// (or the batch size suggests) and the code object's occupancy admits; every
// workgroup is resident at once.
constexpr int kSecondaryKey = 512;   // tuning keys only: variant_key | kSecondaryKey for MRT_TRACE_SECONDARY batches
int variant_key(const mrt::TraceVariant& v) {
    const int lds = v.ldsStack == 8 ? 0 : v.ldsStack == 16 ? 1 : 2;
    static_assert((15 | (2 << 4) | (mrt::kNodeWide4Q << 6) | (1 << 8)) < (int)(sizeof(mrt_tracer::occ) / sizeof(int)),
                  "every variant_key indexes mrt_tracer::occ");
    return (v.anyHit ? 1 : 0) | (v.speculative ? 2 : 0) | (v.exactRcp ? 4 : 0) | (v.stats ? 8 : 0) | (lds << 4) |
           (v.nodes << 6) | (v.tail ? 256 : 0);   // < 512 = the size of mrt_tracer::occ
}

// The launch configuration a trace uses: the tracer's, except that with every
// ray-distribution knob at its default a batch over a BVH that does not fit the
// 256 MB Infinity Cache runs on one global ray queue with refills at 48 live
// lanes. Its rays are long (HBM-latency bound), so the refill atomics are rare,
// and dynamic fetch evens out the per-lane sequences whose static imbalance
// otherwise leaves much of a launch with a decaying number of live lanes. Small
// batches (at most 3 rays per lane of a 16-wave grid) get 12 waves/CU, so that even
// they refill; larger ones 16. Measured (profiles/round2_tuning.md): hairball
// diffuse 640x480 0.365 -> 0.301 ms, primary 1024x768 0.72 -> 0.42 ms, diffuse
// 1920x1080 1.04 -> 0.82 ms. Cache-resident batches keep the static strided
// rounds: there the same queue costs up to 2.6x (contended atomics).
constexpr int64_t kMallBytes = 256ll << 20;
constexpr int kBigQueueThreshold = 48;
#ifndef MRT_BIG_QUEUE_WAVES
#define MRT_BIG_QUEUE_WAVES 16
#endif
constexpr int kBigQueueWaves = MRT_BIG_QUEUE_WAVES;
constexpr int kBigQueueWavesSmall = 12;
constexpr int kBigQueueSmallRaysPerLane = 3;   // of the 16-wave grid

mrt_launch_cfg effective_cfg(const mrt_tracer* t, int numRays) {
    mrt_launch_cfg c = t->cfg;
    const bool defaults = c.num_queues < 0 && c.waves_per_cu == 0 && c.fetch_threshold == 0 && c.lane_groups == 1;
    if (defaults && t->nodeBytes + t->woopBytes > kMallBytes) {
        const int64_t lanes16 = (int64_t)std::max(1, t->numCUs) * kBigQueueWaves * 64;
        c.num_queues = 1;
        c.fetch_threshold = kBigQueueThreshold;
        c.waves_per_cu = (int64_t)numRays <= kBigQueueSmallRaysPerLane * lanes16 ? kBigQueueWavesSmall : kBigQueueWaves;
    }
    return c;
}

int grid_blocks(mrt_tracer* t, const mrt_launch_cfg& cfg, const mrt::TraceVariant& v, int numRays, int* outBlocksPerCU) {
    int& occ = t->occ[variant_key(v)];
    if (occ <= 0 && (mrt::trace_occupancy(v, &occ) != hipSuccess || occ <= 0)) occ = 1;
    int waves = cfg.waves_per_cu;
    if (waves == 0 && cfg.num_queues < 0) {
        // Static strided assignment: 28 waves/CU (7 workgroups) measured best or
        // within 2 % of best from 307k to 12.6M rays (profiles/round1_sweep.txt).
        waves = kStridedWaves;
    } else if (waves == 0) {
        const long long cus = std::max(1, t->numCUs);
        if ((long long)numRays <= 32LL * 64 * cus) {
            // The whole batch fits the first (static, atomic-free) round at full
            // occupancy: one ray per lane, no dynamic fetch at all.
            waves = 32;
        } else {
            const long long lanesPerCU = (long long)numRays / kAutoRaysPerLane / cus;
            waves = (int)std::min<long long>(32, std::max<long long>(kAutoMinWaves, (lanesPerCU + 63) / 64));
        }
    }
    constexpr int wavesPerBlock = mrt::kBlockThreads / 64;
    const int want = std::max(1, (waves + wavesPerBlock - 1) / wavesPerBlock);
    const int perCU = std::min(want, occ);
    if (outBlocksPerCU) *outBlocksPerCU = perCU;
    return perCU * t->numCUs;
}

// Waits for the last launch that used `w` without touching the stream it ran on (the
// caller may have destroyed it): a device-wide synchronize. A completion event recorded
// after every launch (-DMRT_DONE_EVENT) would let the wait cover this handle's launches
// only, but an event between back-to-back launches costs each of them 1-3 % (measured:
// conference AO 0.0352 -> 0.0361 ms, bunny 640x480 0.0945 -> 0.0959 ms,
// profiles/round3_tuning.md); the waits are rare (bind, set_config, destroy, overflow
// reads, a ninth stream).
int workspace_wait(mrt::Workspace* w) {
    if (!w->launched) return MRT_OK;
#ifdef MRT_DONE_EVENT
    MRT_HIP(hipEventSynchronize(w->done));
#else
    MRT_HIP(hipDeviceSynchronize());
    w->launched = false;
#endif
    return MRT_OK;
}

// Every launch of this handle has completed (bind, set_config and destroy).
int wait_all_workspaces(mrt_tracer* t) {
    for (mrt::Workspace* w : t->workspaces)
        if (int rc = workspace_wait(w)) return rc;
    return MRT_OK;
}

// The scratch of `stream`: its own set, else a new one, else (kMaxWorkspaces
// reached) the least recently used set once its last launch has completed —
// grown to the grid's spill slab.
int workspace_for(mrt_tracer* t, void* stream, int totalLanes, int ldsStack, int stackCap, mrt::Workspace** out) {
    mrt::Workspace* w = nullptr;
    for (mrt::Workspace* x : t->workspaces)
        if (x->stream == stream) w = x;
    if (!w && (int)t->workspaces.size() >= mrt::kMaxWorkspaces) {
        for (mrt::Workspace* x : t->workspaces)
            if (!w || x->lastUse < w->lastUse) w = x;
        if (int rc = workspace_wait(w)) return rc;   // its previous stream's launch may still run
        w->stream = stream;
    }
    if (!w) {
        w = new mrt::Workspace();
        w->stream = stream;
        t->workspaces.push_back(w);
        MRT_HIP(hipMalloc(&w->queues, mrt::kQueueLines * mrt::kQueueStrideWords * sizeof(unsigned)));
        MRT_HIP(hipMalloc(&w->status, 64 * sizeof(int)));
        MRT_HIP(hipMemset(w->status, 0, 64 * sizeof(int)));
#ifdef MRT_DONE_EVENT
        MRT_HIP(hipEventCreateWithFlags(&w->done, mrt::kDoneEventFlags));
#endif
    }
    w->lastUse = ++t->useClock;
    const size_t need = (size_t)(stackCap - ldsStack) * (size_t)totalLanes;
    if (need > w->spillInts) {
        // A smaller slab may still be in use by this scratch's previous launch.
        if (int rc = workspace_wait(w)) return rc;
        if (w->spill) MRT_HIP(hipFree(w->spill));
        w->spill = nullptr;
        w->spillInts = 0;
        MRT_HIP(hipMalloc(&w->spill, need * sizeof(int)));
        w->spillInts = need;
    }
    if (!t->evStart) {
        // the blocking call's timing pair: no system-scope fence around the kernel (it would
        // flush the caches and be timed with it); the stop event releases to device scope,
        // so the overflow count read after it is current
        MRT_HIP(hipEventCreateWithFlags(&t->evStart, mrt::kTimingEventFlags));
        MRT_HIP(hipEventCreateWithFlags(&t->evStop, hipEventReleaseToDevice));
    }
    *out = w;
    return MRT_OK;
}

// Largest wide-traversal stack a tracer sizes its spill slab for (entries per lane).
constexpr int kMaxWideStack = 1024;

// (Re)derives the 4-wide nodes of the bound BVH when cfg.wide asks for them;
// bind, unbind and set_config call it with the handle's mutex held. Synchronous
// (bind-time work: the Compact2 nodes come to the host, collapse, go back).
int refresh_wide(mrt_tracer* t) {
    const int want = t->bound ? t->cfg.wide : 0;
    if (want == t->wideBuiltFor) return MRT_OK;
    DeviceGuard guard(t->device);
    // launches in flight may still read the old array: wait for this handle's own
    if (int rc = wait_all_workspaces(t)) return rc;
    if (t->wideNodes) MRT_HIP(hipFree(t->wideNodes));
    t->wideNodes = nullptr;
    t->wideBytes = 0;
    t->wideBuiltFor = -1;
    t->wideFormat = mrt::kNodeCompact2;
    t->wideStackCap = mrt::kStackCapacity;
    t->wideStackBound = mrt::kStackCapacity - 1;
    if (want) {
        std::vector<int32_t> host((size_t)(t->nodeBytes / 4));
        MRT_HIP(hipMemcpy(host.data(), t->nodes, (size_t)t->nodeBytes, hipMemcpyDeviceToHost));
        // The first word of every Woop slot (the terminators): the leaf refs carry counts.
        const int64_t slots = t->woopBytes / 16;
        const bool counts = mrt::leaf_counts_fit(slots);
        std::vector<int32_t> woopX;
        if (counts) {
            woopX.resize((size_t)slots);
            MRT_HIP(hipMemcpy2D(woopX.data(), 4, t->woop, 16, 4, (size_t)slots, hipMemcpyDeviceToHost));
        }
        const int32_t* wx = counts ? woopX.data() : nullptr;
        std::vector<uint32_t> wide;
        int format = mrt::kNodeWide4;
        // The quantized form when asked for and every box quantizes; else the exact one.
        if (want == 2 && mrt::build_wide4q(host.data(), t->nodeBytes / 64, &wide, wx, slots)) format = mrt::kNodeWide4Q;
        else wide = mrt::build_wide4(host.data(), t->nodeBytes / 64, wx, slots);
        t->wideLeafCounts = counts;
        const int nodeWords = format == mrt::kNodeWide4 ? 32 : 16;
        const int64_t need = mrt::wide_stack_bound(wide.data(), (int64_t)wide.size() / nodeWords, nodeWords);
        if (need + 1 > kMaxWideStack) {   // a degenerate tree: keep the binary traversal and its reference capacity
            t->wideBuiltFor = want;
            return MRT_OK;
        }
        t->wideStackCap = std::max<int>(mrt::kStackCapacity, (int)need + 1);
        t->wideStackBound = (int)need;
        const int64_t bytes = (int64_t)wide.size() * 4;
        if (bytes > mrt::kMaxBufferBytes) return fail(MRT_ERR_TOO_LARGE, "4-wide node array above the 32-bit range");
        MRT_HIP(hipMalloc(&t->wideNodes, (size_t)bytes));
        MRT_HIP(hipMemcpy(t->wideNodes, wide.data(), (size_t)bytes, hipMemcpyHostToDevice));
        t->wideBytes = bytes;
        t->wideFormat = format;
    }
    t->wideBuiltFor = want;
    return MRT_OK;
}

// ---- launch-schedule autotuning (cfg.autotune) ---------------------------------
// The ray-distribution schedule that wins depends on the frame: on how the
// expensive rays fall on the static rounds, on the ray length and on the BVH's
// cache residency (profiles/round2_tuning.md: static rounds, fewer waves, per-XCD
// queues and the global queue each win somewhere by 5-70 %). With cfg.autotune
// and the distribution knobs at their defaults, the first launches of a batch
// size cycle through these eight candidates, each timed with an event pair that is
// read back on a later launch (never blocking); after kSamples launches each the
// fastest and the runner-up are timed again, each with the stage-2 modifiers (the
// speculation slack at 4 and 6, the tail toggled, 16 lane groups, 2 lane groups at
// slack 6), and the fastest is kept for that batch size. Closest hits are the same hits under
// every schedule, except that which of two triangles at exactly the same t wins follows the
// traversal order, and so can the hit an any-hit ray reports (any valid hit). A
// reproducible run pins the schedule: autotune 0, or the schedules saved per BVH
// (mrt_tracer_tune_export / _import, mrt/tuned_schedules.json for the bench).
constexpr int kMaxTuned = 64;   // batch sizes tuned per handle; others use the rule
constexpr int64_t kTuneInherit = 32;   // a new batch size within 1/32 of a settled one takes its schedule
// Candidate 2's per-XCD queue blocks (rays), shared tail (%) and refill threshold. No shared tail: on a
// frame in pixel order it bought 0.6 %, and on a buffer ordered costly-first (the strong-scaling shards,
// mrt.dist priority) its last rays retire at once and every XCD's waves then contend for one queue head
// (T_1 3.44 -> 3.20 ms, 8-rank shards 0.490 -> 0.445 ms without it; profiles/round4_shared_queue.txt).
constexpr int kXcdQueueBlock = 8192;
constexpr int kXcdQueueShared = 0;
constexpr int kXcdQueueThreshold = 56;

// The schedule and modifier (-1: none) of candidate c: stage 1 a schedule, stage 2 a modifier of
// the stage-1 winner or runner-up, stage 3 the stage-2 modifier on another schedule. A settled
// candidate is canonical: kSchedules + k modifies st->stage1.
void tune_decode(const TuneState* st, int c, int* sched, int* mod) {
    if (c < TuneState::kSchedules) {
        *sched = c;
        *mod = -1;
    } else if (c < TuneState::kStage3First) {
        const bool second = c >= TuneState::kSchedules + TuneState::kStage2;
        *sched = second ? st->stage1b : st->stage1;
        *mod = (c - TuneState::kSchedules) % TuneState::kStage2;
    } else {
        *sched = st->s3sched[c - TuneState::kStage3First];
        *mod = st->s3mod;
    }
}

mrt_launch_cfg tune_candidate(const mrt_tracer* t, const mrt_launch_cfg& base, int c, const TuneState* st) {
    int sched = c, k = -1;
    if (st) tune_decode(st, c, &sched, &k);
    if (k >= 0) {
        // stage 2/3: a schedule with the wave turning to its leaves once <= 4 (6)
        // lanes still search, with the frontier tail toggled, or with its lanes taking rays from 16
        // distant parts of each strided chunk (only for knobs the caller left at their defaults)
        mrt_launch_cfg x = tune_candidate(t, base, sched, nullptr);
        if (k < 2 && base.spec_slack == kDefaultSpecSlack) x.spec_slack = k == 0 ? 4 : 6;
        if (k == 2 && base.tail_lanes == kDefaultTailLanes) x.tail_lanes = kDefaultTailLanes ? 0 : kTunedTailLanes;
        // lane groups mix a wave's rays from distant image regions: fewer waves hold a whole
        // tile of expensive rays (a silhouette), so more of them reach the frontier tail early
        // (bunny primary 640x480 0.086 -> 0.069 ms, sponza diffuse +8 %; conference AO -7 %)
        if (k == 3) x.lane_groups = kTunedLaneGroups;
        // two lane groups with slack 6: the coherent primary batches keep most of their tile
        // coherence and still shed their expensive half-tiles early (bunny primary 1024x768
        // +3 %, profiles/round4_head_knobs.txt)
        if (k == 4 && base.lane_groups == 1 && base.spec_slack == kDefaultSpecSlack) {
            x.lane_groups = 2;
            x.spec_slack = 6;
        }
        return x;
    }
    mrt_launch_cfg x = base;
    x.fetch_threshold = 0;
    x.waves_per_cu = 0;
    x.num_queues = -1;
    x.queue_block = 0;
    x.queue_shared = 0;
    switch (sched) {
        case 0: break;                                                      // static rounds, 20 waves/CU
        case 1: x.waves_per_cu = 8; break;                                  // static rounds, fewer waves
        case 2:   // per-XCD queues of 8192-ray blocks dealt cyclically (every XCD samples the whole frame,
                  // its L2 holds its own blocks' nodes and triangles), no shared tail queue,
                  // refills at 56 live lanes, 20 waves/CU: a multi-million-ray launch over a BVH above the
                  // Infinity Cache (hairball 2 M rays: 0.630 -> 0.547 ms, fabric bytes 1.07 -> 0.74 GB at
                  // 4096-ray blocks, profiles/round4_queue_ab.txt; 8192: 1.4 % faster again and the
                  // strong-scaling shards' best, round4_order_sweep.txt)
            x.num_queues = std::max(1, std::min(t->numXccs, mrt::kMaxQueues));   // one per XCD, never more
            x.queue_block = kXcdQueueBlock;
            x.queue_shared = kXcdQueueShared;
            x.fetch_threshold = kXcdQueueThreshold;
            x.waves_per_cu = kStridedWaves;
            break;
        case 3: x.num_queues = 1; x.fetch_threshold = kBigQueueThreshold; x.waves_per_cu = kBigQueueWaves; break;   // global queue
        case 4: x.num_queues = 1; x.fetch_threshold = 48; x.waves_per_cu = 12; break;
        case 5: x.waves_per_cu = 16; break;
        case 6: x.waves_per_cu = 12; break;
        default:   // the global queue at full occupancy: a lone multi-million-ray launch over a BVH
                   // above the Infinity Cache (hairball 2 M rays 0.728 -> 0.712 ms), whose frontier
                   // tail drains it; slower when launches overlap on two streams (the rule's 16)
            x.num_queues = 1;
            x.fetch_threshold = kBigQueueThreshold;
            x.waves_per_cu = kStridedWaves;
            break;
    }
    return x;
}

// A candidate replaces the incumbent (the fixed rule in stage 1, the stage-1 winner
// in stage 2) only when its median is this much faster: candidates within a few
// per cent of each other no longer settle differently from run to run.
constexpr float kTuneMargin = 0.03f;

int tune_pick(const TuneState* st, int incumbent, int first, int last) {
    int best = incumbent;
    for (int c = first; c < last; c++)
        if (c != incumbent && st->median(c) < st->median(best)) best = c;
    return st->median(best) < (1.0f - kTuneMargin) * st->median(incumbent) ? best : incumbent;
}

void tune_collect(TuneState* st) {
    for (auto& p : st->pending) {
        if (p.cand < 0 || hipEventQuery(p.stop) != hipSuccess) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess && st->samples[p.cand] < TuneState::kSamples)
            st->times[p.cand][st->samples[p.cand]++] = ms;
        p.cand = -1;
    }
    if (st->locked >= 0) return;
    auto sampled = [&](int first, int last) {
        for (int c = first; c < last; c++)
            if (st->samples[c] < TuneState::kSamples) return false;
        return true;
    };
    if (st->stage1 < 0) {
        if (!sampled(0, TuneState::kSchedules)) return;
        st->stage1 = tune_pick(st, st->rule, 0, TuneState::kSchedules);
        for (int c = 0; c < TuneState::kSchedules; c++)
            if (c != st->stage1 && (st->stage1b < 0 || st->median(c) < st->median(st->stage1b))) st->stage1b = c;
        st->next = TuneState::kSchedules;
        st->runPos = 0;
        return;
    }
    if (st->stage2 < 0) {
        if (!sampled(TuneState::kSchedules, TuneState::kStage3First)) return;
        st->samples[st->stage1] = std::min(st->samples[st->stage1], TuneState::kSamples);
        const int pick = tune_pick(st, st->stage1, TuneState::kSchedules, TuneState::kStage3First);
        if (pick < TuneState::kSchedules) {   // no modifier beats the stage-1 winner: settled
            st->locked = pick;
            return;
        }
        int sched, mod;
        tune_decode(st, pick, &sched, &mod);
        st->stage2 = pick;
        st->s3mod = mod;
        for (int c = 0, i = 0; c < TuneState::kSchedules; c++)
            if (c != st->stage1 && c != st->stage1b) st->s3sched[i++] = c;
        st->next = TuneState::kStage3First;
        st->runPos = 0;
        return;
    }
    if (!sampled(TuneState::kStage3First, TuneState::kCandidates)) return;
    const int pick = tune_pick(st, st->stage2, TuneState::kStage3First, TuneState::kCandidates);
    int sched, mod;
    tune_decode(st, pick, &sched, &mod);
    st->stage1 = sched;   // canonical: modifier kSchedules + mod of schedule stage1
    st->locked = TuneState::kSchedules + mod;
}

void tune_reset(mrt_tracer* t) {
    for (auto& kv : t->tunes) {
        for (auto& p : kv.second->pending) {
            if (p.start) (void)hipEventSynchronize(p.stop);
            if (p.start) (void)hipEventDestroy(p.start);
            if (p.stop) (void)hipEventDestroy(p.stop);
        }
        delete kv.second;
    }
    t->tunes.clear();
}

// Largest batch one launch takes: ray/result addressing and the strided round
// arithmetic stay inside int32 with room for the grid (bigger batches are split
// by the caller, as the reference Renderer does at 2^21 rays, Renderer.cc:46).
constexpr int32_t kMaxRaysPerLaunch = 1 << 30;

int trace_impl(mrt_tracer* t, const void* rays, void* results, int32_t numRays, uint32_t flags, int32_t* stats,
               void* stream, mrt_trace_info* info) {
    if (!t) return fail(MRT_ERR_INVALID_ARG, "null tracer");
    if (numRays < 0) return fail(MRT_ERR_INVALID_ARG, "numRays < 0");
    if (flags & ~0x1Fu) return fail(MRT_ERR_INVALID_ARG, "unknown trace flag");
    std::lock_guard<std::mutex> lock(t->mu);
    if (info) std::memset(info, 0, sizeof(*info));
    if (numRays == 0) return MRT_OK;   // reference CudaTracer.cc:123-125: no rays => 0 ms
    if (!t->bound) return fail(MRT_ERR_NOT_BOUND, "trace before bind (no BVH)");
    if (!rays || !results) return fail(MRT_ERR_INVALID_ARG, "null ray/result buffer");
    if ((flags & MRT_TRACE_STATS) && !stats) return fail(MRT_ERR_INVALID_ARG, "MRT_TRACE_STATS without stats buffer");

    if (numRays > kMaxRaysPerLaunch) return fail(MRT_ERR_TOO_LARGE, "more than 2^30 rays in one launch: split the batch");

    DeviceGuard guard(t->device);
    mrt::TraceVariant v = variant_for(t, flags);   // its key (the tracer's tail setting) keys the tuning
    int perCU = 0;
    mrt_launch_cfg cfg = effective_cfg(t, numRays);
    // autotuning: the schedule candidate this launch uses, and its timing slot
    TuneState* tune = nullptr;
    TuneState::Pending* slot = nullptr;
    int cand = -1;
    const mrt_launch_cfg& uc = t->cfg;
    if (uc.autotune && uc.num_queues < 0 && uc.waves_per_cu == 0 && uc.fetch_threshold == 0 && uc.lane_groups == 1 &&
        !(flags & MRT_TRACE_STATS)) {
        // secondary rays (MRT_TRACE_SECONDARY) settle their own schedule: a diffuse batch of a primary
        // batch's size runs differently (round-5 README table: Mori primary 4829 Mrays/s on the diffuse
        // batch's schedule, 5814 on its own)
        const auto key = std::make_pair(numRays, variant_key(v) | ((flags & MRT_TRACE_SECONDARY) ? kSecondaryKey : 0));
        auto it = t->tunes.find(key);
        if (it != t->tunes.end()) {
            tune = it->second;
        } else if ((int)t->tunes.size() < kMaxTuned) {
            tune = new TuneState();
            tune->stream = stream;
            // the candidate that equals the fixed rule for this batch (effective_cfg)
            tune->rule = cfg.num_queues == 1 ? (cfg.waves_per_cu == kBigQueueWaves ? 3 : 4) : 0;
            // A batch within 1/kTuneInherit of a settled batch size of the same variant takes
            // that schedule instead of exploring (the nearest one): the strong-scaling shards of
            // one frame differ by a block or two (2,064,384 .. 2,080,768 rays against the saved
            // 2,073,600), and ~100 exploring launches per shard size would fall in the timed steps.
            int64_t bestGap = -1;
            for (const auto& kv : t->tunes) {
                if (kv.first.second != key.second || kv.second->locked < 0) continue;
                const int64_t gap = std::llabs((int64_t)kv.first.first - numRays);
                if (gap * kTuneInherit > (int64_t)kv.first.first || (bestGap >= 0 && gap >= bestGap)) continue;
                bestGap = gap;
                tune->stage1 = kv.second->stage1;
                tune->locked = kv.second->locked;
                tune->inherited = true;
            }
            t->tunes[key] = tune;
        }
        // A batch size launched on several streams is not explored there: its launches
        // overlap, and a candidate's time alone no longer ranks the pipeline. It runs its
        // settled schedule (saved, inherited, or settled on one stream) if it has one, else
        // the fixed rule (the bench's two-stream hairball 8 spp buffer: 4.23 ms on the rule,
        // 3.48 on the per-XCD block-cyclic schedule).
        if (tune && !tune->stream) tune->stream = stream;   // an imported schedule: first used here
        if (tune && tune->stream != stream) tune->multiStream = true;
        if (tune && tune->multiStream && tune->locked < 0) tune = nullptr;
    }
    if (tune) {
        tune_collect(tune);
        if (tune->locked >= 0) {
            cand = tune->locked;
        } else {
            // runs of kRun launches per candidate, cycling over the current stage's candidates;
            // the first launch of a run (and the whole first cycle of stage 1) is untimed
            cand = tune->next;
            const bool timed = tune->runPos > 0 && tune->launches >= TuneState::kSchedules * TuneState::kRun;
            tune->launches++;
            if (++tune->runPos == TuneState::kRun) {
                tune->runPos = 0;
                const int first = tune->stage1 < 0 ? 0 : (tune->stage2 < 0 ? TuneState::kSchedules : TuneState::kStage3First);
                const int last = tune->stage1 < 0 ? TuneState::kSchedules
                                                  : (tune->stage2 < 0 ? TuneState::kStage3First : TuneState::kCandidates);
                tune->next = first + (tune->next + 1 - first) % (last - first);
            }
            if (timed)
                for (auto& p : tune->pending)
                    if (p.cand < 0) {
                        slot = &p;
                        break;
                    }
            if (slot && !slot->start) {
                MRT_HIP(hipEventCreateWithFlags(&slot->start, mrt::kTimingEventFlags));
                MRT_HIP(hipEventCreateWithFlags(&slot->stop, mrt::kTimingEventFlags));
            }
        }
        cfg = tune_candidate(t, cfg, cand, tune);
    }
    v.tail = with_tail(t, v, cfg);   // a tuned candidate may run without the tail
    const int blocks = grid_blocks(t, cfg, v, numRays, &perCU);
    const int totalLanes = blocks * mrt::kBlockThreads;
    const bool wide = v.nodes != mrt::kNodeCompact2;
    const int stackCap = wide ? t->wideStackCap : mrt::kStackCapacity;
    mrt::Workspace* ws = nullptr;
    if (int rc = workspace_for(t, stream, totalLanes, v.ldsStack, stackCap, &ws)) return rc;

    mrt::TraceArgs a{};
    a.rays = static_cast<const float4*>(rays);
    a.results = static_cast<int2*>(results);
    a.nodes = static_cast<const float4*>(wide ? t->wideNodes : t->nodes);
    a.woop = static_cast<const float4*>(t->woop);
    a.triIndex = t->triIndex;
    a.nodeBytes = (uint32_t)(wide ? t->wideBytes : t->nodeBytes);
    a.woopBytes = (uint32_t)t->woopBytes;
    a.numRays = numRays;
    a.numQueues = cfg.num_queues < 0 ? 0 : std::min(cfg.num_queues, std::max(1, numRays));
    // queue_shared percent of the rays past the first round go to the shared queue
    a.sharedRays = a.numQueues > 1 ? (int)((int64_t)numRays * cfg.queue_shared / 100) : 0;
    a.queueBlockLog2 = a.numQueues > 1 && cfg.queue_block > 0 ? __builtin_ctz((unsigned)cfg.queue_block) : 0;
    // the live-lane refill applies to the queue modes only (static rounds hand out one ray per
    // lane per round, to every lane at once): a strided launch reports and uses 0
    a.fetchThreshold = a.numQueues > 0 ? cfg.fetch_threshold : 0;
    a.specSlack = cfg.spec_slack;
    a.staticRounds = cfg.static_rounds;
    a.wideLeafCounts = wide && t->wideLeafCounts;
    a.laneGroupsLog2 = __builtin_ctz((unsigned)cfg.lane_groups);
    a.totalLanes = totalLanes;
    a.stackCap = stackCap;
    a.stackBound = wide ? t->wideStackBound : stackCap - 1;
    a.tailLanes = cfg.tail_lanes;
    a.xccMask = cfg.queue_xcc_mask;
    a.raySort = cfg.ray_sort;
    a.queues = ws->queues;
    a.spill = ws->spill;
    // The blocking call counts this launch's overflows in a slot of its own; the
    // asynchronous one adds to the sticky counter (mrt_tracer_stack_overflows).
    a.status = info ? ws->status + mrt::kTimedSlot : ws->status;
    a.stats = reinterpret_cast<int4*>(stats);

    hipStream_t s = static_cast<hipStream_t>(stream);
    // Queue heads restart at zero for every launch; strided mode has none.
    if (a.numQueues > 0)
        MRT_HIP(hipMemsetAsync(ws->queues, 0, mrt::kQueueLines * mrt::kQueueStrideWords * sizeof(unsigned), s));
    if (info) MRT_HIP(hipMemsetAsync(ws->status + mrt::kTimedSlot, 0, sizeof(int), s));
    if (info) MRT_HIP(hipEventRecord(t->evStart, s));
    if (slot) MRT_HIP(hipEventRecord(slot->start, s));
    MRT_HIP(mrt::launch_trace(v, a, blocks, s));
#ifdef MRT_DONE_EVENT
    MRT_HIP(hipEventRecord(ws->done, s));
#endif
    ws->launched = true;
    if (slot) {
        MRT_HIP(hipEventRecord(slot->stop, s));
        slot->cand = cand;
    }
    if (info) {
        // stage-2 candidates (another speculation slack) carry their stage-1 schedule in bits 8+
        // canonical: a modifier k of the schedule it modifies, kSchedules + k | schedule << 8
        int sched = cand, mod = -1;
        tune_decode(tune, cand, &sched, &mod);
        info->autotune_candidate = mod >= 0 ? (TuneState::kSchedules + mod) | (sched << 8) : cand;
        info->autotune_locked = tune && tune->locked >= 0 ? 1 : 0;
        info->stack_capacity = stackCap;
        MRT_HIP(hipEventRecord(t->evStop, s));
        MRT_HIP(hipEventSynchronize(t->evStop));
        MRT_HIP(hipEventElapsedTime(&info->kernel_ms, t->evStart, t->evStop));
        info->grid_waves = totalLanes / 64;
        info->block_threads = mrt::kBlockThreads;
        info->lds_stack_entries = v.ldsStack;
        info->wide = wide ? 4 : 2;
        info->node_bytes = v.nodes == mrt::kNodeWide4 ? 128 : 64;
        info->num_queues = a.numQueues;
        info->fetch_threshold = a.fetchThreshold;
        int overflow = 0;
        MRT_HIP(hipMemcpy(&overflow, ws->status + mrt::kTimedSlot, sizeof(int), hipMemcpyDeviceToHost));
        info->stack_overflows = overflow;
        if (overflow)
            return fail(MRT_ERR_STACK_OVERFLOW,
                        std::to_string(overflow) + " stack pushes past the " + std::to_string(stackCap) +
                            "-entry traversal stack (stack_capacity): those rays' results are incomplete (BVH "
                            "deeper than the reference's STACK_SIZE 64 allows in the binary order)");
    }
    return MRT_OK;
}

// ---- implicit per-device tracers (convenience + reference-compat API) ----
constexpr int kMaxDevices = 64;
std::mutex g_devMu;
mrt_tracer* g_devTracer[kMaxDevices] = {};

mrt_tracer* device_tracer(int* err) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        *err = fail(MRT_ERR_NO_DEVICE, "no current HIP device");
        return nullptr;
    }
    std::lock_guard<std::mutex> lock(g_devMu);
    if (!g_devTracer[dev]) {
        mrt_tracer* t = nullptr;
        *err = mrt_tracer_create(dev, &t);
        if (*err) return nullptr;
        g_devTracer[dev] = t;
    }
    *err = MRT_OK;
    return g_devTracer[dev];
}

// cutilSafeCall-style fatal error for the compat entry points
// (reference cutil_inline_runtime.h:32-42).
void compat_check(int rc, const char* file, int line) {
    if (rc != MRT_OK) {
        std::fprintf(stderr, "[%s,%d] (HIP error %d: %s)\n", file, line, rc, mrt_last_error_detail());
        std::exit(-1);
    }
}

}  // namespace

extern "C" {

int mrt_version(void) { return 100; }

const char* mrt_error_string(int err) {
    switch (err) {
        case MRT_OK: return "ok";
        case MRT_ERR_INVALID_ARG: return "invalid argument";
        case MRT_ERR_NOT_BOUND: return "no BVH bound";
        case MRT_ERR_HIP: return "HIP runtime error";
        case MRT_ERR_NO_DEVICE: return "no HIP device";
        case MRT_ERR_TOO_LARGE: return "buffer or batch too large";
        case MRT_ERR_STACK_OVERFLOW: return "traversal stack overflow";
        default: return "unknown error";
    }
}

const char* mrt_last_error_detail(void) { return mrt::api_last_error(); }

int mrt_selftest_exact_rcp(uint64_t* mismatches) {
    if (!mismatches) return fail(MRT_ERR_INVALID_ARG, "null argument");
    unsigned long long* d = nullptr;
    MRT_HIP(hipMalloc(&d, sizeof(*d)));
    hipError_t e = hipMemset(d, 0, sizeof(*d));
    if (e == hipSuccess) e = mrt::selftest_exact_rcp(d, nullptr);
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hipFail(e, "selftest_exact_rcp");
    *mismatches = h;
    return MRT_OK;
}

int mrt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int mrt_tracer_create(int device, mrt_tracer** out) {
    if (!out) return fail(MRT_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(MRT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(MRT_ERR_INVALID_ARG, "device index out of range");
    int cus = 0, xccs = 0;
    MRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    // XCDs of this device (partition): the HIP attribute, else 32 CUs per MI355X XCD
    if (hipDeviceGetAttribute(&xccs, hipDeviceAttributeNumberOfXccs, device) != hipSuccess || xccs <= 0)
        xccs = std::max(1, cus / 32);
    mrt_tracer* t = new mrt_tracer();
    t->device = device;
    t->numCUs = cus;
    t->numXccs = std::max(1, std::min(xccs, mrt::kMaxQueues));
    t->cfg = default_cfg();
    *out = t;
    return MRT_OK;
}

int mrt_tracer_destroy(mrt_tracer* t) {
    if (!t) return MRT_OK;
    {
        DeviceGuard guard(t->device);
        if (t->wideNodes) (void)hipFree(t->wideNodes);
        (void)wait_all_workspaces(t);   // event waits: the streams may already be destroyed
        for (mrt::Workspace* w : t->workspaces) {
            if (w->done) (void)hipEventDestroy(w->done);
            if (w->queues) (void)hipFree(w->queues);
            if (w->status) (void)hipFree(w->status);
            if (w->spill) (void)hipFree(w->spill);
            delete w;
        }
        if (t->evStart) (void)hipEventDestroy(t->evStart);
        if (t->evStop) (void)hipEventDestroy(t->evStop);
        tune_reset(t);
    }
    delete t;
    return MRT_OK;
}

int mrt_tracer_bind(mrt_tracer* t, const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes,
                    const int32_t* triIndex, int64_t triIndexBytes) {
    if (!t || !nodes || !woop || !triIndex) return fail(MRT_ERR_INVALID_ARG, "null BVH buffer");
    if (nodeBytes < 64 || woopBytes < 16 || triIndexBytes < 4 || (nodeBytes % 64) || (woopBytes % 16) ||
        (triIndexBytes % 4))
        return fail(MRT_ERR_INVALID_ARG, "BVH buffer sizes are not Compact2-shaped");
    if (nodeBytes > mrt::kMaxBufferBytes || woopBytes > mrt::kMaxBufferBytes)
        return fail(MRT_ERR_TOO_LARGE, "Compact2 buffer above the 32-bit buffer-offset range");
    if (triIndexBytes / 4 != woopBytes / 16) return fail(MRT_ERR_INVALID_ARG, "triIndex must hold one int per woop float4");
    std::lock_guard<std::mutex> lock(t->mu);
    t->nodes = nodes;
    t->nodeBytes = nodeBytes;
    t->woop = woop;
    t->woopBytes = woopBytes;
    t->triIndex = triIndex;
    t->triIndexBytes = triIndexBytes;
    t->bound = true;
    t->wideBuiltFor = -1;   // a new BVH: its wide nodes are derived now (if configured)
    DeviceGuard guard(t->device);
    tune_reset(t);          // and its schedules are tuned again
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = refresh_wide(t);
    t->bindMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int mrt_tracer_unbind(mrt_tracer* t) {
    if (!t) return fail(MRT_ERR_INVALID_ARG, "null tracer");
    std::lock_guard<std::mutex> lock(t->mu);
    t->bound = false;
    t->nodes = t->woop = nullptr;
    t->triIndex = nullptr;
    return refresh_wide(t);
}

int mrt_tracer_set_config(mrt_tracer* t, const mrt_launch_cfg* cfg) {
    if (!t || !cfg) return fail(MRT_ERR_INVALID_ARG, "null argument");
    mrt_launch_cfg c = *cfg;
    const mrt_launch_cfg d = default_cfg();
    if (c.waves_per_cu == 0) c.waves_per_cu = d.waves_per_cu;
    if (c.num_queues == 0) c.num_queues = d.num_queues;
    if (c.lds_stack == 0) c.lds_stack = d.lds_stack;
    if (c.lane_groups == 0) c.lane_groups = d.lane_groups;
    if (c.wide < 0) c.wide = d.wide;   // -1 = library default
    if (c.spec_slack < 0) c.spec_slack = d.spec_slack;
    if (c.static_rounds == 0) c.static_rounds = d.static_rounds;
    if (c.autotune < 0) c.autotune = d.autotune;
    if (c.tail_lanes < 0) c.tail_lanes = d.tail_lanes;
    if (c.queue_shared < 0) c.queue_shared = d.queue_shared;
    if (c.queue_block < 0) c.queue_block = d.queue_block;
    if (c.queue_xcc_mask < 0) c.queue_xcc_mask = d.queue_xcc_mask;
    if (c.ray_sort < 0) c.ray_sort = d.ray_sort;
    if (!valid_cfg(c)) return fail(MRT_ERR_INVALID_ARG, "launch config out of range");
    std::lock_guard<std::mutex> lock(t->mu);
    t->cfg = c;
    DeviceGuard guard(t->device);
    tune_reset(t);
    const auto t0 = std::chrono::steady_clock::now();
    const int built = t->wideBuiltFor;
    const int rc = refresh_wide(t);
    if (t->wideBuiltFor != built)
        t->bindMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int mrt_tracer_get_config(const mrt_tracer* t, mrt_launch_cfg* cfg) {
    if (!t || !cfg) return fail(MRT_ERR_INVALID_ARG, "null argument");
    *cfg = t->cfg;
    return MRT_OK;
}

int mrt_tracer_bind_info(const mrt_tracer* t, mrt_bind_info* info) {
    if (!t || !info) return fail(MRT_ERR_INVALID_ARG, "null argument");
    info->bind_ms = t->bindMs;
    info->wide_bytes = t->wideNodes ? t->wideBytes : 0;
    info->wide_format = t->wideNodes ? t->wideFormat : mrt::kNodeCompact2;
    info->stack_capacity = t->wideNodes ? t->wideStackCap : mrt::kStackCapacity;
    info->stack_bound = t->wideNodes ? t->wideStackBound : mrt::kStackCapacity - 1;
    return MRT_OK;
}

// candidate field: the locked candidate | the stage-1 winner << 8 (stage-2 candidates
// are the stage-1 schedule with another speculation slack)
int mrt_tracer_tune_export(const mrt_tracer* t, mrt_tuned_schedule* out, int32_t capacity, int32_t* count) {
    if (!t || !count || (capacity > 0 && !out)) return fail(MRT_ERR_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> lock(const_cast<mrt_tracer*>(t)->mu);
    int n = 0;
    for (const auto& kv : t->tunes) {
        // inherited entries were tuned for another batch (size and ray distribution): not saved as tuned
        if (kv.second->locked < 0 || kv.second->inherited) continue;
        if (n < capacity)
            out[n] = mrt_tuned_schedule{kv.first.first, kv.first.second,
                                        kv.second->locked | (std::max(0, kv.second->stage1) << 8), MRT_TUNE_VERSION};
        n++;
    }
    *count = n;
    return MRT_OK;
}

int mrt_tracer_tune_import(mrt_tracer* t, const mrt_tuned_schedule* in, int32_t count) {
    if (!t || (count > 0 && !in) || count < 0) return fail(MRT_ERR_INVALID_ARG, "null argument");
    for (int i = 0; i < count; i++) {
        const int locked = in[i].candidate & 0xff, stage1 = in[i].candidate >> 8;
        if (in[i].version != MRT_TUNE_VERSION || in[i].num_rays <= 0 || locked >= TuneState::kSchedules + TuneState::kStage2 ||
            stage1 < 0 || stage1 >= TuneState::kSchedules)
            return fail(MRT_ERR_INVALID_ARG, "tuned schedule from another library version or out of range");
    }
    std::lock_guard<std::mutex> lock(t->mu);
    for (int i = 0; i < count; i++) {
        const auto key = std::make_pair((int)in[i].num_rays, (int)in[i].variant);
        auto it = t->tunes.find(key);
        if (it == t->tunes.end()) {
            if ((int)t->tunes.size() >= kMaxTuned) return fail(MRT_ERR_TOO_LARGE, "more tuned batch sizes than kMaxTuned");
            it = t->tunes.emplace(key, new TuneState()).first;
        }
        it->second->stage1 = in[i].candidate >> 8;
        it->second->locked = in[i].candidate & 0xff;
        it->second->inherited = false;   // a schedule saved for this very key: exported again
    }
    return MRT_OK;
}

int mrt_tracer_trace(mrt_tracer* t, const void* rays, void* results, int32_t numRays, uint32_t flags,
                     int32_t* stats, void* stream) {
    return trace_impl(t, rays, results, numRays, flags, stats, stream, nullptr);
}

int mrt_tracer_trace_timed(mrt_tracer* t, const void* rays, void* results, int32_t numRays, uint32_t flags,
                           int32_t* stats, void* stream, mrt_trace_info* info) {
    mrt_trace_info local;
    return trace_impl(t, rays, results, numRays, flags, stats, stream, info ? info : &local);
}

int mrt_tracer_stack_overflows(mrt_tracer* t, int64_t* count, int32_t reset) {
    if (!t || !count) return fail(MRT_ERR_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> lock(t->mu);
    DeviceGuard guard(t->device);
    int64_t total = 0;
    for (mrt::Workspace* w : t->workspaces) {
        int n = 0;
        if (int rc = workspace_wait(w)) return rc;
        MRT_HIP(hipMemcpy(&n, w->status, sizeof(int), hipMemcpyDeviceToHost));
        total += n;
        if (reset) MRT_HIP(hipMemset(w->status, 0, sizeof(int)));
    }
    *count = total;
    return MRT_OK;
}

int mrt_derive_wide_nodes(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes, int32_t form,
                          void* out, int64_t outCapacity, int64_t* outBytes) {
    if (!nodes || !outBytes || nodeBytes <= 0 || nodeBytes % 64 != 0 || (form != 1 && form != 2) ||
        (woop && (woopBytes <= 0 || woopBytes % 16 != 0)))
        return fail(MRT_ERR_INVALID_ARG, "derive_wide_nodes: bad arguments");
    // the first word of every Woop slot, when the leaf refs can carry counts
    const int64_t slots = woop ? woopBytes / 16 : 0;
    std::vector<int32_t> woopX;
    if (woop && mrt::leaf_counts_fit(slots)) {
        woopX.resize((size_t)slots);
        for (int64_t i = 0; i < slots; i++) woopX[(size_t)i] = static_cast<const int32_t*>(woop)[4 * i];
    }
    const int32_t* wx = woopX.empty() ? nullptr : woopX.data();
    std::vector<uint32_t> wide;
    const auto* n = static_cast<const int32_t*>(nodes);
    if (form == 2) {
        if (!mrt::build_wide4q(n, nodeBytes / 64, &wide, wx, slots))
            return fail(MRT_ERR_INVALID_ARG, "a box has no finite quantization");
    } else {
        wide = mrt::build_wide4(n, nodeBytes / 64, wx, slots);
    }
    *outBytes = (int64_t)wide.size() * 4;
    if (out) {
        if (outCapacity < *outBytes) return fail(MRT_ERR_TOO_LARGE, "derive_wide_nodes: output buffer too small");
        std::memcpy(out, wide.data(), (size_t)*outBytes);
    }
    return MRT_OK;
}

int mrt_bind_bvh(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes,
                 const int32_t* triIndex, int64_t triIndexBytes) {
    int err = 0;
    mrt_tracer* t = device_tracer(&err);
    if (!t) return err;
    return mrt_tracer_bind(t, nodes, nodeBytes, woop, woopBytes, triIndex, triIndexBytes);
}

int mrt_unbind_bvh(void) {
    int err = 0;
    mrt_tracer* t = device_tracer(&err);
    if (!t) return err;
    return mrt_tracer_unbind(t);
}

int mrt_trace(const void* rays, void* results, int32_t numRays, int32_t anyHit, void* stream, float* outMs) {
    int err = 0;
    mrt_tracer* t = device_tracer(&err);
    if (!t) return err;
    const uint32_t flags = anyHit ? MRT_TRACE_ANY_HIT : 0u;
    if (!outMs) return trace_impl(t, rays, results, numRays, flags, nullptr, stream, nullptr);
    mrt_trace_info info;
    const int rc = trace_impl(t, rays, results, numRays, flags, nullptr, stream, &info);
    *outMs = info.kernel_ms;
    return rc;
}

// ---- reference-compatible entry points --------------------------------------

void bind_CudaBVHTexture(void* nodeBuf, int64_t nodeBufSize, void* triWoopBuf, int64_t triWoopSize,
                         int32_t* triIndexBuf, int64_t triIndexSize) {
    compat_check(mrt_bind_bvh(nodeBuf, nodeBufSize, triWoopBuf, triWoopSize, triIndexBuf, triIndexSize), __FILE__,
                 __LINE__);
}

void unbind_CudaBVHTexture(void) { compat_check(mrt_unbind_bvh(), __FILE__, __LINE__); }

float launch_tracingKernel(int32_t nthreads, int32_t* blockSize, int numRays, bool anyHit, void* rays,
                           void* results, void* nodesA, void* nodesB, void* nodesC, void* nodesD, void* trisA,
                           void* trisB, void* trisC, int32_t* triIndices) {
    // The reference ignored nthreads/blockSize (CudaKernel::setGrid rewrote
    // them) and read the BVH through the textures bound earlier; the node/tri
    // pointers are accepted for ABI compatibility only.
    (void)nthreads; (void)blockSize; (void)nodesA; (void)nodesB; (void)nodesC; (void)nodesD;
    (void)trisA; (void)trisB; (void)trisC; (void)triIndices;
    float ms = 0.0f;
    compat_check(mrt_trace(rays, results, numRays, anyHit ? 1 : 0, nullptr, &ms), __FILE__, __LINE__);
    return ms;
}

void copy_tracing_results(void* result_host, void* result_dev, int32_t size) {
    const hipError_t e = hipMemcpy(result_host, result_dev, (size_t)size * 16u, hipMemcpyDeviceToHost);
    if (e != hipSuccess) compat_check(hipFail(e, "hipMemcpy"), __FILE__, __LINE__);
}

void launch_rayGenPrimaryKernel(int32_t nthreads, mrt_raygen_primary_input* in) {
    (void)nthreads;
    if (!in) compat_check(fail(MRT_ERR_INVALID_ARG, "null RayGenPrimaryInput"), __FILE__, __LINE__);
    compat_check(mrt_raygen_primary(in->nscreenToWorld, in->origin, in->maxDist, in->w, in->h, in->indexToPixel,
                                    in->rays, in->slotToID, in->idToSlot, nullptr),
                 __FILE__, __LINE__);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) compat_check(hipFail(e, "hipDeviceSynchronize"), __FILE__, __LINE__);
}

void launch_rayGenAOKernel(int32_t nthreads, mrt_raygen_ao_input* in) {
    (void)nthreads;
    if (!in || in->firstInputSlot < 0)
        compat_check(fail(MRT_ERR_INVALID_ARG, "bad RayGenAOInput"), __FILE__, __LINE__);
    // inSlot = taskIdx + firstInputSlot; the hash and the output slots use taskIdx (RayGenKernels.cu:128-131,163)
    const char* inRays = static_cast<const char*>(in->inRays);
    const char* inResults = static_cast<const char*>(in->inResults);
    compat_check(mrt_raygen_ao(inRays ? inRays + (int64_t)in->firstInputSlot * 32 : nullptr,
                               inResults ? inResults + (int64_t)in->firstInputSlot * 16 : nullptr, in->numInputRays,
                               static_cast<const float*>(in->normals), INT64_MAX, in->numSamples, in->maxDist,
                               in->randomSeed, in->outRays, in->outIDToSlot, in->outSlotToID, nullptr),
                 __FILE__, __LINE__);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) compat_check(hipFail(e, "hipDeviceSynchronize"), __FILE__, __LINE__);
}

void launch_reconstructKernel(int32_t nthreads, mrt_reconstruct_input* in) {
    (void)nthreads;   // the reference's CudaKernel::setGrid(nthreads) shape; ours is fixed
    if (!in) compat_check(fail(MRT_ERR_INVALID_ARG, "null ReconstructInput"), __FILE__, __LINE__);
    const int32_t type = in->isAO ? MRT_RAY_AO : (in->isDiffuse ? MRT_RAY_DIFFUSE : MRT_RAY_PRIMARY);
    compat_check(mrt_reconstruct(type, in->numRaysPerPrimary, in->firstPrimary, in->numPrimary, in->primarySlotToID,
                                 in->primaryResults, in->batchIDToSlot, in->batchResults, in->triMaterialColor,
                                 in->triShadedColor, in->pixels, nullptr),
                 __FILE__, __LINE__);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) compat_check(hipFail(e, "hipDeviceSynchronize"), __FILE__, __LINE__);
}

int32_t launch_countHitsKernel(int32_t threads, const int32_t* blockSize, mrt_count_hits_input* in) {
    (void)threads; (void)blockSize;   // launch shape of the reference (RendererKernels.cu:191-199)
    if (!in) compat_check(fail(MRT_ERR_INVALID_ARG, "null CountHitsInput"), __FILE__, __LINE__);
    int32_t* d = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&d), sizeof(int32_t));
    if (e != hipSuccess) compat_check(hipFail(e, "hipMalloc"), __FILE__, __LINE__);
    compat_check(mrt_count_hits(in->rayResults, in->numRays, d, nullptr), __FILE__, __LINE__);
    int32_t n = 0;
    e = hipMemcpy(&n, d, sizeof(int32_t), hipMemcpyDeviceToHost);
    const hipError_t f = hipFree(d);
    if (e != hipSuccess) compat_check(hipFail(e, "hipMemcpy"), __FILE__, __LINE__);
    if (f != hipSuccess) compat_check(hipFail(f, "hipFree"), __FILE__, __LINE__);
    return n;
}

}  // extern "C"
