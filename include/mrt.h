/*
 * mrt.h — C-ABI of the MI355X BVH ray-traversal engine (the hot path).
 *
 * This is the drop-in boundary for the reference's tracing kernel module:
 *   reference  src/rt/kernels/CudaTracerKernels.hh:42-52   (extern "C" prototypes)
 *   reference  src/rt/kernels/kepler_dynamic_fetch.cu:417-479 (their implementations)
 *   caller     src/rt/cuda/CudaTracer.cc:119-177            (CudaTracer::traceBatch)
 *
 * Data formats are the reference's, byte for byte:
 *   - nodes    : CudaBVH BVHLayout_Compact2 node array, 64 B per inner node
 *                (reference src/rt/cuda/CudaBVH.hh:40-55, CudaBVH.cc:270-357)
 *   - woop     : Woop triangle rows (Z,U,V as float4) + one float4 terminator
 *                (x bits == 0x80000000) after every leaf
 *   - triIndex : one int32 per woop float4 slot (origIdx for the Z row)
 *   - rays     : Ray[n], 32 B = float4(orig.xyz, tmin) + float4(dir.xyz, tmax)
 *                (reference src/rt/Util.hh:64-73)
 *   - results  : RayResult[n], 16 B = int id, float t, int pad[2]; the trace
 *                writes only {id, t} (reference src/rt/Util.hh:79-89,
 *                CudaTracerKernels.hh:197 STORE_RESULT)
 *
 * All buffer pointers are DEVICE pointers owned by the caller (the library
 * borrows them; reference ownership model CudaBVH.cc:101-109, RayBuffer.cc:42-81).
 * Every function returns 0 on success or a positive MRT_ERR_* code; the
 * reference instead printed and exit(-1)'d (cutil_inline_runtime.h:32-42) —
 * the compat entry points at the bottom keep that behaviour.
 */
#ifndef MRT_H
#define MRT_H

#include <stdint.h>
#include <stddef.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------ */
enum {
    MRT_OK = 0,
    MRT_ERR_INVALID_ARG = 1,   /* null pointer / negative size / bad flag   */
    MRT_ERR_NOT_BOUND = 2,     /* trace before bind (CudaTracer.cc:129)      */
    MRT_ERR_HIP = 3,           /* a HIP runtime call failed                  */
    MRT_ERR_NO_DEVICE = 4,     /* no GPU visible                             */
    MRT_ERR_TOO_LARGE = 5,     /* buffer beyond the 4 GiB buffer-offset range, or > 2^30 rays per launch */
    MRT_ERR_STACK_OVERFLOW = 6 /* a ray needed more than the reference's 64 stack entries
                                  (kepler_dynamic_fetch.cu:47 STACK_SIZE): its result is incomplete */
};

/* ---- trace flags (bit set) -------------------------------------------- */
enum {
    MRT_TRACE_ANY_HIT = 1u << 0,  /* any-hit early out; reference anyHit=!needClosestHit (CudaTracer.cc:172) */
    MRT_TRACE_EXACT_RCP = 1u << 1,/* correctly rounded 1/x in the Woop test & ray setup (parity mode);
                                     default is the hardware v_rcp_f32 (the reference used rcp.approx)  */
    MRT_TRACE_LOCKSTEP_OFF = 1u << 2, /* per-lane (non-speculative) while-while: every lane follows the
                                     single-ray order exactly (deterministic any-hit, exact counters)  */
    MRT_TRACE_STATS = 1u << 3,    /* also write per-ray {inner nodes, tris tested, leaves, latency in 10 ns ticks} int4s */
    MRT_TRACE_SECONDARY = 1u << 4 /* tuning hint, no effect on results: the batch holds secondary rays (AO, diffuse,
                                     later bounces). The autotuner keeps their schedule apart from a primary batch
                                     of the same size and kernel variant (saved / exported with variant | 512) */
};

/* One per HIP device. Re-entrant: launches on different streams get separate
 * scratch (stack spill slab, queue heads, overflow counter), so traces on
 * several streams of one handle may run concurrently. */
typedef struct mrt_tracer mrt_tracer;

/* Tuning knobs of the persistent launch (0 = library default). */
typedef struct mrt_launch_cfg {
    int32_t waves_per_cu;      /* persistent waves per CU (grid = CUs * waves_per_cu); 0 = auto (by batch size).
                                  With num_queues, waves_per_cu, fetch_threshold and lane_groups all at their
                                  defaults, a batch over a BVH larger than the 256 MB Infinity Cache uses
                                  one global queue, refills at 48 live lanes, 12 waves/CU up to 3 rays per
                                  lane of a 16-wave grid, else 16 (mrt_trace_info reports what a launch used) */
    int32_t fetch_threshold;   /* queue modes (num_queues >= 1): refill a wave when fewer than this many of its
                                  64 lanes are live (0 = when all are done; reference DYNAMIC_FETCH_THRESHOLD
                                  20 of 32, kepler_dynamic_fetch.cu:48). Static strided rounds ignore it   */
    int32_t num_queues;        /* -1 (default) = static strided rounds, no atomics; 1..8 = the reference's
                                  dynamic fetch: a static first round, then one atomic per wave refill
                                  on the queue of the wave's XCD (xcc % num_queues), no stealing of rays
                                  from a served queue; a queue no wave has taken from when a wave's own
                                  queue is dry (an XCD without workgroups of the launch, e.g. a CPX/DPX
                                  partition) is adopted by that wave, so every ray is traced whatever
                                  the placement. The autotuner's per-XCD candidate uses one queue per
                                  XCD of the device (hipDeviceAttributeNumberOfXccs)                   */
    int32_t lds_stack;         /* traversal-stack entries per lane kept in LDS: 8, 16 or 32       */
    int32_t lane_groups;       /* strided mode: a wave's 64 lanes take rays from this many (1..64, power of
                                  two) distant sub-ranges of the batch instead of 64 consecutive rays */
    int32_t wide;              /* the speculative traversal reads 4-wide nodes derived from the bound
                                  Compact2 tree at bind time (half the dependent node fetches; closest hits
                                  equal the binary traversal's except exact-t ties): 1 = exact child boxes
                                  (128-B nodes), 2 = child boxes quantized outward to 8 bits per plane
                                  (64-B nodes; a superset of the binary traversal's leaves, falls back to 1
                                  when a box has no finite quantization); 0 = the Compact2 nodes
                                  themselves; -1 = library default. The per-lane
                                  (MRT_TRACE_LOCKSTEP_OFF) mode always walks the Compact2 nodes */
    int32_t spec_slack;        /* speculative mode: a wave turns from its inner nodes to its postponed leaves
                                  once at most this many of its lanes are still without a leaf (0..63; the
                                  reference waits for all, i.e. 0; default 2; -1 = library default) */
    int32_t static_rounds;     /* queue modes (num_queues >= 1): rays handed out in this many static strided
                                  rounds of the grid before the queues take over (1..64; 0 = default 1) */
    int32_t autotune;          /* 1 = with the distribution knobs above at their defaults, the first launches
                                  of each batch size (per kernel variant, up to 64 sizes) time eight ray-
                                  distribution schedules (static rounds at 20, 16, 12 or 8 waves/CU, per-XCD
                                  block-cyclic queues, the global queue at 20, 16 or 12 waves/CU), then
                                  the winner and the runner-up, each with spec_slack 4 and 6, without the
                                  frontier tail, with 16 lane groups, and with 2 lane groups at spec_slack 6 (each
                                  knob only when left at its default), then the best such modifier on the
                                  six other schedules (stage 3); each candidate runs four launches at a time
                                  (the first untimed) until it has eight timed samples, without blocking,
                                  after one untimed round; the median ranks them and a candidate
                                  replaces the fixed rule (stage 1) or the previous stage's winner only
                                  when 3 % faster. A new batch size within 1/32 of a settled one of the
                                  same variant and ray class (MRT_TRACE_SECONDARY batches are a class
                                  of their own) takes the nearest settled schedule without exploring —
                                  a schedule tuned on another ray distribution of that class; such
                                  inherited entries are not exported by mrt_tracer_tune_export (an
                                  imported schedule for the same key replaces one and is). A batch
                                  size launched on more than one stream is not explored: it runs its settled
                                  schedule if it has one, else the fixed rule; reset by bind and set_config (default 1; mrt_tracer_tune_export /
                                  _import save and restore the choices). 0 = the fixed rule only; -1 = default */
    int32_t tail_lanes;        /* exact 4-wide speculative traversal: a wave that cannot refill (its strided
                                  round, or its queue drained) and is down to at most this many tracing
                                  lanes finishes those rays in the frontier tail: 64/R lanes per ray for R
                                  rays (at least four), up to 16/R pending nodes or four-triangle leaf chunks
                                  per ray per memory round trip, regrouping as rays finish (0..16; 0 = off;
                                  default 16; -1 = default; the autotuner tries 0 when left at the default) */
    int32_t queue_shared;      /* num_queues > 1: this percentage of the batch's rays (its end) goes to one
                                  shared queue that a wave takes from once its XCD's queue is dry; the
                                  rest is dealt in per-XCD contiguous shares (0..100; default 0; -1 =
                                  default)                                                             */
    int32_t queue_block;       /* num_queues > 1: 0 = each queue's share is contiguous; a power of two >= 64 =
                                  the shares are this many rays' blocks dealt cyclically (block i to queue
                                  i mod num_queues), so every XCD samples the whole frame (default 0;
                                  -1 = default)                                                        */
    int32_t ray_sort;          /* 1 = a static launch whose batch fits one round of the grid (e.g. 307 200 rays
                                  at 20 waves/CU) deals each workgroup's 256 consecutive rays to its four
                                  waves by direction octant, degenerate (tmax < 0) rays last, instead of
                                  the strided deal (exact 4-wide traversal only); 0 = off (default; -1 =
                                  default). Results are unchanged: every ray is traced once either way.
                                  With ray_sort = 1 the strided deal ignores lane_groups (in every launch,
                                  also one whose batch needs several rounds, where the sort is skipped) */
    int32_t queue_xcc_mask;    /* test hook, 0 = off (default; -1 = default): 1..15 = a wave takes from queue
                                  (XCC_ID & mask) % num_queues, so with mask 3 and 8 queues, queues 4..7
                                  have no waves of their own (the unserved-queue sweep must trace them) */
} mrt_launch_cfg;

/* Per-launch statistics reported back to the host (optional). */
typedef struct mrt_trace_info {
    float   kernel_ms;         /* event-timed duration of the trace launch (if requested)        */
    int32_t grid_waves;        /* persistent waves launched                                       */
    int32_t block_threads;     /* threads per workgroup                                           */
    int32_t lds_stack_entries; /* per-lane traversal-stack entries held in LDS                    */
    int32_t wide;              /* node width the launch traversed: 2 (Compact2) or 4              */
    int32_t num_queues;        /* ray queues the launch used (0 = static strided rounds)          */
    int32_t fetch_threshold;   /* live-lane refill threshold the launch used (0 for static strided rounds:
                                  the refill applies to the queue modes only)                        */
    int32_t stack_overflows;   /* entries pushed past stack_capacity in this launch (then the call returns
                                  MRT_ERR_STACK_OVERFLOW; 0 for any SBVH of depth <= 64)            */
    int32_t node_bytes;        /* bytes per node the launch read: 64 (Compact2 or quantized 4-wide), 128 */
    int32_t autotune_candidate; /* cfg.autotune: the schedule candidate this launch used, else -1 (the fixed
                                  rule): 0..7 a ray-distribution schedule; 8..12 a stage-2 modifier of
                                  the stage-1 schedule s, encoded as modifier | s << 8 (8/9: spec_slack
                                  4/6, 10: the frontier tail toggled, 11: 16 lane groups, 12: 2 lane
                                  groups at spec_slack 6; bench.py schedule_name spells them out)    */
    int32_t autotune_locked;   /* 1 once the batch size's schedule is chosen                      */
    int32_t stack_capacity;    /* stack entries (sentinel included) the launch had: 64 = the reference's
                                  for the binary order; the wide orders get the bound tree's worst case
                                  (never less than 64), so no ray of a tree overflows there          */
} mrt_trace_info;

/* What the last bind derived (mrt_tracer_bind_info). */
typedef struct mrt_bind_info {
    double  bind_ms;           /* wall time of the last bind / set_config's wide-node derivation      */
    int64_t wide_bytes;        /* bytes of the derived 4-wide node array (0 = the Compact2 nodes)      */
    int32_t wide_format;       /* 0 = Compact2, 1 = exact 4-wide (128 B), 2 = quantized 4-wide (64 B)  */
    int32_t stack_capacity;    /* stack entries the wide traversal gets (see mrt_trace_info)          */
    int32_t stack_bound;       /* entries (sentinel excluded) a depth-first walk of the bound tree can hold:
                                  the wide tree's worst case (63 for the binary order). The frontier tail
                                  expands several entries per step only while this much room stays free,
                                  so it never needs more than stack_capacity either                     */
} mrt_bind_info;

/* One settled launch schedule of the autotuner (cfg.autotune): the candidate a batch
 * size and kernel variant chose. Opaque apart from num_rays; valid for the library
 * version MRT_TUNE_VERSION and the BVH it was tuned on (the caller keys a saved
 * table by the BVH, e.g. next to its .dat cache). */
typedef struct mrt_tuned_schedule {
    int32_t num_rays;
    int32_t variant;
    int32_t candidate;
    int32_t version;           /* MRT_TUNE_VERSION when exported; others are refused on import */
} mrt_tuned_schedule;
enum { MRT_TUNE_VERSION = 11 };   /* 11: round 6 (schedules re-tuned on the round-6 library) */

/* ---- handle API -------------------------------------------------------- */
int  mrt_tracer_create(int device, mrt_tracer** out);
int  mrt_tracer_destroy(mrt_tracer* t);

/* Bind a Compact2 BVH (device pointers, borrowed). Replaces bind_CudaBVHTexture
 * (CudaTracerKernels.hh:44); unlike the reference it may be called again to
 * re-bind a new BVH (the reference never re-bound, CudaTracer.cc:142-146). */
int  mrt_tracer_bind(mrt_tracer* t,
                     const void* nodes, int64_t nodeBytes,
                     const void* woop, int64_t woopBytes,
                     const int32_t* triIndex, int64_t triIndexBytes);
int  mrt_tracer_unbind(mrt_tracer* t);

int  mrt_tracer_set_config(mrt_tracer* t, const mrt_launch_cfg* cfg);
int  mrt_tracer_get_config(const mrt_tracer* t, mrt_launch_cfg* cfg);
int  mrt_tracer_bind_info(const mrt_tracer* t, mrt_bind_info* info);

/* The autotuner's settled schedules (up to capacity; *count = how many exist), and
 * the reverse: schedules saved from an earlier run of the same BVH are locked at
 * once (no exploring launches, the same schedule every run). Import after bind
 * (bind and set_config forget every schedule). */
int  mrt_tracer_tune_export(const mrt_tracer* t, mrt_tuned_schedule* out, int32_t capacity, int32_t* count);
int  mrt_tracer_tune_import(mrt_tracer* t, const mrt_tuned_schedule* in, int32_t count);

/* Stream-ordered trace of numRays (<= 2^30) rays (device pointers). stream is a
 * hipStream_t (NULL = the null stream). stats may be NULL unless
 * MRT_TRACE_STATS is set (then: int32[4*numRays]). Asynchronous: a stack
 * overflow cannot be returned here; it accumulates in a sticky per-stream
 * counter that mrt_tracer_stack_overflows reads. */
int  mrt_tracer_trace(mrt_tracer* t, const void* rays, void* results, int32_t numRays,
                      uint32_t flags, int32_t* stats, void* stream);

/* Same, but blocking and event-timed around the launch only — the
 * reference's launch_tracingKernel contract (kepler_dynamic_fetch.cu:432-474).
 * Returns MRT_ERR_STACK_OVERFLOW (results written, info filled) when a ray of
 * this launch needed more than stack_capacity entries (64 in the binary order). */
int  mrt_tracer_trace_timed(mrt_tracer* t, const void* rays, void* results, int32_t numRays,
                            uint32_t flags, int32_t* stats, void* stream, mrt_trace_info* info);

/* Stack overflows of asynchronous launches since the last reset, summed over the
 * handle's streams (synchronises them). reset != 0 zeroes the counters. */
int  mrt_tracer_stack_overflows(mrt_tracer* t, int64_t* count, int32_t reset);

/* Host-only (no device): the 4-wide node array a tracer derives at bind time
 * from a Compact2 node array (host memory). form 1 = exact child boxes, 128 B per
 * node; form 2 = child boxes quantized outward, 64 B per node (layouts in
 * csrc/wide_bvh.cpp). With the Woop array (host memory, may be NULL) the leaf refs
 * carry their triangle counts, as the tracer's own array does when the woop
 * indices fit 27 bits. *outBytes = the array's size; it is copied to out when
 * out != NULL and outCapacity suffices (else MRT_ERR_TOO_LARGE). Form 2 returns
 * MRT_ERR_INVALID_ARG when some box has no finite quantization. */
int  mrt_derive_wide_nodes(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes, int32_t form,
                           void* out, int64_t outCapacity, int64_t* outBytes);

/* Diagnostics: run the EXACT variants' reciprocal (v_rcp_f32 + one FMA Newton step)
 * against the correctly rounded 1.0f / x for all 2^32 inputs on the current device;
 * *mismatches = number of differing bit patterns (0 expected). Blocking. */
int  mrt_selftest_exact_rcp(uint64_t* mismatches);

/* ---- device ray generation and hit counting (the trace's producers and consumer) ----
 * Stream-ordered on the calling thread's current HIP device. Buffers are device
 * pointers; the camera matrix and origin are host values. Per-ray arithmetic is
 * the host generator's (mrt_host.h mrth_primary_rays / mrth_ao_rays): primary
 * rays are bit-identical to it (device denormals flush to zero), AO/diffuse
 * directions agree to a few ulp (device cosf/sinf). */

/* RayGen::primary + rayGenPrimaryKernel (RayGen.cc:50-72, RayGenKernels.cu:79-113).
 * nscreenToWorld: column-major 4x4 (mrth_camera_nscreen_to_world). indexToPixel:
 * w*h pixel ids in trace order (mrth_pixel_table). slotToId/idToSlot may be NULL. */
int  mrt_raygen_primary(const float nscreenToWorld[16], const float origin[3], float maxDist, int32_t w, int32_t h,
                        const int32_t* indexToPixel, void* rays, int32_t* slotToId, int32_t* idToSlot, void* stream);

/* The same rays sampled at (jx, jy) in [0, 1)^2 inside each pixel instead of its centre
 * (0.5, 0.5): distinct, equally coherent batches of one view, e.g. one sample per rank
 * when a frame's rays are sharded over GPUs (bench.py). */
int  mrt_raygen_primary_subpixel(const float nscreenToWorld[16], const float origin[3], float maxDist, int32_t w,
                                 int32_t h, float jx, float jy, const int32_t* indexToPixel, void* rays,
                                 int32_t* slotToId, int32_t* idToSlot, void* stream);

/* RayGen::ao + rayGenAOKernel (RayGen.cc:77-120, RayGenKernels.cu:117-227): numSamples
 * hemisphere rays per input ray (origin backed off 1e-4 along the input ray, Halton
 * (2,3) samples rotated by a Jenkins hash of seed + ray index, tmax = -1 for input
 * misses). triNormals: 3 floats per triangle. Closest-hit use (diffuse): maxDist = far. */
int  mrt_raygen_ao(const void* inRays, const void* inResults, int32_t numInputRays, const float* triNormals,
                   int64_t numTris, int32_t numSamples, float maxDist, uint32_t seed, void* outRays,
                   int32_t* outIdToSlot, int32_t* outSlotToId, void* stream);

/* A whole frame's AO/diffuse rays, generated for a list of blocks of the frame's ray order
 * instead of batch by batch: the frame's RayGen::batching sequence (RayGen.cc:124-142) —
 * batch k = input rays [k*batchInputRays, (k+1)*batchInputRays), seeded by batchSeeds[k]
 * (host array, one glibc rand() per batch, RayGen.cc:106), numSamples rays per input ray
 * — numbers its rays g = input * numSamples + sample; output ray j is ray
 * blocks[j / blockRays] * blockRays + j % blockRays of it, bit-identical to the ray the
 * batches hold there (mrt_raygen_ao of batch k). blocks: device int32[numBlocks], any
 * order (e.g. a rank's shard, its costly blocks first). Only the frame's last block can
 * be partial; when listed it must be the last entry, and numOutRays = the listed rays
 * ((numBlocks-1)*blockRays + its length; else numBlocks*blockRays). At most 256 batches.
 * A block id outside [0, blocks in the frame) is not checked on the host (the list is device
 * memory): its output rays are left unwritten. */
int  mrt_raygen_ao_blocks(const void* inRays, const void* inResults, int32_t numInputRays, const float* triNormals,
                          int64_t numTris, int32_t numSamples, float maxDist, const uint32_t* batchSeeds,
                          int32_t numBatches, int32_t batchInputRays, const int32_t* blocks, int32_t numBlocks,
                          int32_t blockRays, int64_t numOutRays, void* outRays, void* stream);

/* One rank's blocks of a frame's AO/diffuse ray order for mrt_raygen_ao_blocks (multi-GPU
 * sharding: no reference counterpart — the reference is single-GPU). The frame's
 * numPrimary*numSamples rays are cut into blockRays-ray blocks, block i to rank i % world;
 * order 0 lists the rank's blocks in frame order, order 1 live blocks first: decreasing
 * number of live rays (samples whose primary ray hit, read from primaryResults — the primary
 * pass's RayResult[numPrimary]; a missed primary's samples are degenerate, tmax = -1), ties in
 * frame order, the frame's partial last block last (live counts quantized to 12 bits when
 * blockRays > 4094; order 1 holds at most 16384 blocks per rank). blocks: device
 * int32[capacity] (NULL: only *numBlocks / *numRays are set); *numBlocks and *numRays (host) =
 * the rank's blocks and the rays they hold, known without the device. Stream-ordered, no host sync. */
int  mrt_shard_blocks(const void* primaryResults, int32_t numPrimary, int32_t numSamples, int32_t blockRays,
                      int32_t world, int32_t rank, int32_t order, int32_t* blocks, int32_t capacity,
                      int32_t* numBlocks, int64_t* numRays, void* stream);

/* countHitsKernel (RendererKernels.cu:112-162): *hitCount (device int32) = number of
 * results with id >= 0. */
int  mrt_count_hits(const void* results, int32_t numRays, int32_t* hitCount, void* stream);

/* ray types of a batch (reference RayType_Primary / _AO / _Diffuse, App.cc) */
enum { MRT_RAY_PRIMARY = 0, MRT_RAY_AO = 1, MRT_RAY_DIFFUSE = 2 };

/* reconstructKernel (RendererKernels.cu:60-108; ReconstructInput RendererKernels.hh:46-61,
 * filled by Renderer.cc:421-445): one ABGR pixel per primary ray of the batch, at
 * pixels[primarySlotToId[firstPrimary + i]], i < numPrimary. Primary: shaded colour of
 * the hit triangle or the background (0.2, 0.4, 0.8); AO: the fraction of unblocked
 * rays (background where the primary missed); diffuse: the average shaded colour of
 * the bounce hits (white for misses) times the primary hit's material colour. Batch
 * rays of primary task i are batchIdToSlot[i * numRaysPerPrimary + k] (primary:
 * batchIdToSlot[pixel id]); batchIdToSlot NULL = identity layout (mrt_raygen_ao's).
 * Results are RayResult (16 B); colour tables one ABGR uint32 per triangle
 * (mrth_scene_tri_colors). Colour arithmetic is the reference's device code: float
 * sums in ray order, truncating toABGR. */
int  mrt_reconstruct(int32_t rayType, int32_t numRaysPerPrimary, int32_t firstPrimary, int32_t numPrimary,
                     const int32_t* primarySlotToId, const void* primaryResults, const int32_t* batchIdToSlot,
                     const void* batchResults, const uint32_t* triMaterialColor, const uint32_t* triShadedColor,
                     uint32_t* pixels, void* stream);

/* ---- per-device convenience API (one implicit tracer per device) -------- */
int  mrt_bind_bvh(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes,
                  const int32_t* triIndex, int64_t triIndexBytes);
int  mrt_unbind_bvh(void);
int  mrt_trace(const void* rays, void* results, int32_t numRays, int32_t anyHit, void* stream,
               float* outMs /* may be NULL: then asynchronous */);

/* Host-side introspection. */
const char* mrt_error_string(int err);
const char* mrt_last_error_detail(void);     /* thread-local text of the last failure */
int  mrt_version(void);                      /* 100 * major + minor                     */
int  mrt_device_count(void);

/* ---- reference-compatible entry points (same names, same arguments) ----
 * CudaTracerKernels.hh:44-52. Errors print "[file,line] (HIP error N: msg)"
 * and exit(-1) like cutilSafeCall. float4/int4/RayResult are passed as void*
 * and Vec2i& as a pointer to two int32 (ABI-identical). */
void  bind_CudaBVHTexture(void* nodeBuf, int64_t nodeBufSize, void* triWoopBuf, int64_t triWoopSize,
                          int32_t* triIndexBuf, int64_t triIndexSize);
void  unbind_CudaBVHTexture(void);
float launch_tracingKernel(int32_t nthreads, int32_t* blockSize, int numRays, bool anyHit,
                           void* rays, void* results,
                           void* nodesA, void* nodesB, void* nodesC, void* nodesD,
                           void* trisA, void* trisB, void* trisC, int32_t* triIndices);
void  copy_tracing_results(void* result_host, void* result_dev, int32_t size);

/* RendererKernels.hh:46-69 input structs, field for field (same C layout: three int32,
 * three bools, then 8-byte-aligned pointers). The reference passes them by C++
 * reference, which is ABI-identical to a pointer. Both launchers synchronise like
 * the reference's (cudaDeviceSynchronize) and ignore its launch-shape arguments. */
typedef struct mrt_reconstruct_input {
    int32_t   numRaysPerPrimary, firstPrimary, numPrimary;
    bool      isPrimary, isAO, isDiffuse;
    int32_t*  primarySlotToID;
    void*     primaryResults;
    int32_t*  batchIDToSlot;
    void*     batchResults;
    uint32_t* triMaterialColor;
    uint32_t* triShadedColor;
    uint32_t* pixels;
} mrt_reconstruct_input;

typedef struct mrt_count_hits_input {
    int32_t numRays;
    void*   rayResults;
    int32_t raysPerThread;
} mrt_count_hits_input;

/* RayGenKernels.hh:40-68 input structs, field for field: Vec3f = 3 floats, Mat4f =
 * 16 floats column-major, then 8-byte-aligned pointers. */
typedef struct mrt_raygen_primary_input {
    float    origin[3];
    float    nscreenToWorld[16];
    int32_t  w, h;
    float    maxDist;
    void*    rays;
    int32_t* idToSlot;
    int32_t* slotToID;
    int32_t* indexToPixel;
} mrt_raygen_primary_input;

typedef struct mrt_raygen_ao_input {
    int32_t  firstInputSlot, numInputRays, numSamples;
    float    maxDist;
    uint32_t randomSeed;
    void*    inRays;
    void*    inResults;
    void*    outRays;
    int32_t* outIDToSlot;
    int32_t* outSlotToID;
    void*    normals;          /* const Vec3f*: one per triangle, unbounded like the reference's */
} mrt_raygen_ao_input;

/* launch_rayGenPrimaryKernel / launch_rayGenAOKernel (RayGenKernels.cu:295-330); blocking */
void    launch_rayGenPrimaryKernel(int32_t nthreads, mrt_raygen_primary_input* in);
void    launch_rayGenAOKernel(int32_t nthreads, mrt_raygen_ao_input* in);

/* launch_reconstructKernel (RendererKernels.cu:166-186) */
void    launch_reconstructKernel(int32_t nthreads, mrt_reconstruct_input* in);
/* launch_countHitsKernel (RendererKernels.cu:189-215): returns the hit count */
int32_t launch_countHitsKernel(int32_t threads, const int32_t* blockSize, mrt_count_hits_input* in);

#ifdef __cplusplus
}
#endif

#endif /* MRT_H */
