// raygen_kernel.hip — the trace's producers and consumer on the device (gfx950):
// primary rays, AO/diffuse hemisphere rays and the hit count, so a frame
// (primary -> trace -> AO -> trace) never leaves HBM.
//
//   mrt_raygen_primary  <- RayGen::primary + rayGenPrimaryKernel (reference RayGen.cc:50-72,
//                          RayGenKernels.cu:79-113)
//   mrt_raygen_ao       <- RayGen::ao + rayGenAOKernel (RayGen.cc:77-120, RayGenKernels.cu:117-227)
//   mrt_count_hits      <- countHitsKernel / launch_countHitsKernel (RendererKernels.cu:112-162,189-)
//   mrt_reconstruct     <- reconstructKernel / launch_reconstructKernel (RendererKernels.cu:60-108,
//                          Renderer.cc:421-445)
//
// The per-ray arithmetic is csrc/raygen_common.hpp, the same code the host
// generator runs. These are streaming kernels (32 B written per ray, 16-48 B
// read): one thread per output ray, 256-thread blocks, no LDS. The hit count
// is a shuffle reduction, one partial per block and a one-block final sum (no
// contended atomics).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mrt.h"
#include "raygen_common.hpp"
#include "trace_kernel.hpp"

namespace mrt {
namespace {

constexpr int kThreads = 256;

struct PrimaryArgs {
    float m[16];   // column-major nscreen-to-world
    float ox, oy, oz, maxDist;
    float jx, jy;   // sample position inside the pixel
    int w, h;
    const int32_t* indexToPixel;
    rg::RayRec* rays;
    int32_t* slotToId;
    int32_t* idToSlot;
};

__global__ __launch_bounds__(kThreads) void primary_kernel(PrimaryArgs a) {
    const int task = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (task >= a.w * a.h) return;
    const int pixel = a.indexToPixel[task];
    a.rays[task] = rg::primary_ray(a.m, rg::make(a.ox, a.oy, a.oz), a.maxDist, a.w, a.h, pixel, a.jx, a.jy);
    if (a.slotToId) a.slotToId[task] = pixel;
    if (a.idToSlot) a.idToSlot[pixel] = task;
}

struct AOArgs {
    const rg::RayRec* inRays;
    const int2* inResults;   // RayResult viewed as int2 pairs: slot 2*i = {id, t bits}
    int numInput;
    const float* normals;
    int64_t numTris;
    int numSamples;
    float maxDist;
    uint32_t seed;
    rg::RayRec* outRays;
    int32_t* outIdToSlot;
    int32_t* outSlotToId;
};

__global__ __launch_bounds__(kThreads) void ao_kernel(AOArgs a) {
    const int task = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (task >= a.numInput) return;
    const int2 res = a.inResults[2 * task];
    const rg::AOBasis b =
        rg::ao_basis(a.inRays[task], res.x, __int_as_float(res.y), a.normals, a.numTris, a.seed, (uint32_t)task);
    const int64_t out = (int64_t)task * a.numSamples;
    for (int i = 0; i < a.numSamples; i++) {
        a.outRays[out + i] = rg::ao_sample(b, i, a.maxDist);
        if (a.outIdToSlot) a.outIdToSlot[out + i] = (int32_t)(out + i);
        if (a.outSlotToId) a.outSlotToId[out + i] = (int32_t)(out + i);
    }
}

// One thread per OUTPUT ray (numSamples > 1): consecutive lanes write consecutive
// 32 B rays (coalesced), each recomputing its input ray's basis (a few dozen
// ALU ops and three L2-resident reads). ao_sample(b, i) depends only on (b, i),
// so the rays are the same bits as ao_kernel's.
__global__ __launch_bounds__(kThreads) void ao_per_sample_kernel(AOArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (gid >= (int64_t)a.numInput * a.numSamples) return;
    const int task = (int)(gid / a.numSamples), i = (int)(gid - (int64_t)task * a.numSamples);
    const int2 res = a.inResults[2 * task];
    const rg::AOBasis b =
        rg::ao_basis(a.inRays[task], res.x, __int_as_float(res.y), a.normals, a.numTris, a.seed, (uint32_t)task);
    a.outRays[gid] = rg::ao_sample(b, i, a.maxDist);
    if (a.outIdToSlot) a.outIdToSlot[gid] = (int32_t)gid;
    if (a.outSlotToId) a.outSlotToId[gid] = (int32_t)gid;
}

// A frame's secondary rays in block order (mrt_raygen_ao_blocks). The frame's
// RayGen::batching sequence (RayGen.cc:124-142) numbers its rays g = p * S + i
// (input ray p, sample i); batch k holds the inputs [k * P, (k + 1) * P) and hashes
// seed_k + (p - k * P) (RayGen.cc:106, RayGenKernels.cu:122-134). Output ray j is
// ray g = blocks[j / B] * B + j % B of that sequence, so a list of blocks in any
// order comes out as the same bits the batches would hold at those positions —
// a rank's shard generated directly in its trace order, no gather of a frame
// buffer. One thread per output ray: consecutive lanes write consecutive 32-B
// rays; a block id and an input ray are shared by B and S consecutive lanes.
constexpr int kMaxBatchSeeds = 256;
struct AOBlocksArgs {
    const rg::RayRec* inRays;
    const int2* inResults;
    int numInput;
    const float* normals;
    int64_t numTris;
    int numSamples;
    float maxDist;
    int batchInputs;          // P: input rays per batch
    int blockRays;            // B
    int64_t totalRays;        // numInput * numSamples
    int64_t outRays;          // output rays of this launch
    const int32_t* blocks;
    rg::RayRec* out;
    uint32_t seeds[kMaxBatchSeeds];
};

__global__ __launch_bounds__(kThreads) void ao_blocks_kernel(AOBlocksArgs a) {
    const int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.outRays) return;
    const int64_t k = j / a.blockRays;
    const int64_t g = (int64_t)a.blocks[k] * a.blockRays + (j - k * a.blockRays);
    // past the frame's end: the (last-listed) partial block; a block id outside the frame writes nothing
    if (g < 0 || g >= a.totalRays) return;
    const int p = (int)(g / a.numSamples), i = (int)(g - (int64_t)p * a.numSamples);
    const int batch = p / a.batchInputs;
    const int2 res = a.inResults[2 * p];
    const rg::AOBasis b = rg::ao_basis(a.inRays[p], res.x, __int_as_float(res.y), a.normals, a.numTris,
                                       a.seeds[batch], (uint32_t)(p - batch * a.batchInputs));
    a.out[j] = rg::ao_sample(b, i, a.maxDist);
}

// The same rays when a workgroup's kTileRays outputs lie inside one block (blockRays a
// multiple of kTileRays) and hold whole input rays (numSamples divides kTileRays, at most
// kThreads input rays and at most kThreads samples per ray): each input ray's basis (two trig calls, a normalize, the hash, three
// dependent loads) is computed once by one thread and each sample's hemisphere point once
// per sample index, both through LDS — not once per output ray (S = 8: 8x fewer basis
// evaluations) — then each thread writes kTileRays / kThreads rays (coalesced). Same
// arithmetic, same bits. Four rays per thread: a 2 M-ray shard is 2 025 workgroups, one
// round of the device, so the dependent load chain is paid once, not four times.
constexpr int kTileRays = 1024;
__global__ __launch_bounds__(kThreads) void ao_blocks_tiled_kernel(AOBlocksArgs a) {
    __shared__ rg::AOBasis basis[kThreads];
    __shared__ rg::V3 sample[kThreads];
    const int t = (int)threadIdx.x;
    const int64_t j0 = (int64_t)blockIdx.x * kTileRays;
    const int64_t k = j0 / a.blockRays;
    const int64_t g0 = (int64_t)a.blocks[k] * a.blockRays + (j0 - k * a.blockRays);   // a multiple of S
    if (g0 < 0 || g0 >= a.totalRays) return;   // a block id outside the frame (workgroup-uniform): nothing
    const int S = a.numSamples;
    const int perWg = kTileRays / S;
    const int p0 = (int)(g0 / S);
    if (t < perWg && p0 + t < a.numInput) {
        const int p = p0 + t;
        const int batch = p / a.batchInputs;
        const int2 res = a.inResults[2 * p];
        basis[t] = rg::ao_basis(a.inRays[p], res.x, __int_as_float(res.y), a.normals, a.numTris, a.seeds[batch],
                                (uint32_t)(p - batch * a.batchInputs));
    }
    if (kThreads - 1 - t < S) sample[kThreads - 1 - t] = rg::ao_sample_xyz(kThreads - 1 - t);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kTileRays / kThreads; u++) {
        const int o = u * kThreads + t;
        if (j0 + o >= a.outRays || g0 + o >= a.totalRays) break;
        a.out[j0 + o] = rg::ao_sample_dir(basis[o / S], sample[o % S], a.maxDist);
    }
}

// mrt_shard_blocks: a rank's blocks of the frame's secondary-ray order (block i to rank
// i % world) and their trace order. Two launches, no host sync:
//   block_live_kernel   one wave per listed block: its live rays = the samples of its input
//                       rays whose primary hit (RayGenKernels.cu:117-227: a missed primary's
//                       samples get tmax = -1), as the sort key B - live (the frame's partial
//                       last block: the largest key, so it sorts last);
//   block_order_kernel  one workgroup: a stable LSD radix sort of the list by that key in LDS
//                       (three 4-bit digit passes; per-thread digit counts over contiguous chunks
//                       keep equal keys in list = frame order), then the ordered block ids.
constexpr int kOrderThreads = 1024;
constexpr int kOrderMax = 16384;      // list entries the one-workgroup sort holds
constexpr int kKeyMax = 4095;         // 12-bit keys

struct ShardArgs {
    const int2* results;     // primary RayResult viewed as int2 pairs
    int numPrimary, numSamples, blockRays, world, rank, numBlocks;   // numBlocks: listed (this rank's)
    int64_t totalRays;
    int32_t* out;            // the block list; first the keys (block_live_kernel), then the ordered ids
};

__device__ inline int shard_block_id(const ShardArgs& a, int j) { return a.rank + j * a.world; }

__global__ __launch_bounds__(kThreads) void block_live_kernel(ShardArgs a) {
    const int lane = (int)(threadIdx.x & 63);
    const int j = (int)((blockIdx.x * kThreads + threadIdx.x) >> 6);
    if (j >= a.numBlocks) return;
    const int64_t g0 = (int64_t)shard_block_id(a, j) * a.blockRays;
    const int64_t g1 = min(g0 + a.blockRays, a.totalRays);
    const int64_t p0 = g0 / a.numSamples, p1 = (g1 - 1) / a.numSamples;   // input rays touching the block
    int live = 0;
    for (int64_t p = p0 + lane; p <= p1; p += 64) {
        if (a.results[2 * p].x >= 0) {
            const int64_t lo = max(g0, p * a.numSamples), hi = min(g1, (p + 1) * a.numSamples);
            live += (int)(hi - lo);
        }
    }
    for (int off = 32; off > 0; off >>= 1) live += __shfl_xor(live, off, 64);
    if (lane == 0) {
        int key = a.blockRays - live;   // decreasing live = increasing key
        if (a.blockRays > kKeyMax - 1)  // quantized to 12 bits (mrt.dist.live_sort_key restates it)
            key = (int)(((int64_t)key * (kKeyMax - 1) + a.blockRays - 1) / a.blockRays);
        if (g1 - g0 < a.blockRays) key = kKeyMax;   // the partial last block sorts last
        a.out[j] = key;
    }
}

// Inclusive prefix sum over a wave's 64 lanes in six DPP adds (row_shr 1/2/4/8 within each
// 16-lane row, then row_bcast 15/31 across rows): VALU only, no LDS permutes.
__device__ inline int wave_scan_incl(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

__global__ __launch_bounds__(kOrderThreads) void block_order_kernel(ShardArgs a) {
    constexpr int kWaves = kOrderThreads / 64;
    __shared__ uint16_t key[kOrderMax];
    __shared__ uint16_t idx[2][kOrderMax];
    __shared__ int waveTot[kWaves][16];
    __shared__ int wavePre[kWaves][16];
    static_assert((16 * kWaves) % 64 == 0, "the prefix wave walks (digit, wave) entries 64 at a time");
    const int t = (int)threadIdx.x, lane = t & 63, wave = t >> 6, n = a.numBlocks;
    for (int i = t; i < n; i += kOrderThreads) {
        key[i] = (uint16_t)a.out[i];
        idx[0][i] = (uint16_t)i;
    }
    const int chunk = (n + kOrderThreads - 1) / kOrderThreads;
    const int lo = min(n, t * chunk), hi = min(n, lo + chunk);
    int src = 0;
    for (int shift = 0; shift < 12; shift += 4, src ^= 1) {
        __syncthreads();
        // this thread's digit counts over its contiguous chunk of the current order (registers:
        // the digit selects by compare, no dynamic register indexing)
        int c[16];
#pragma unroll
        for (int e = 0; e < 16; e++) c[e] = 0;
        for (int i = lo; i < hi; i++) {
            const int d = (key[idx[src][i]] >> shift) & 15;
#pragma unroll
            for (int e = 0; e < 16; e++) c[e] += d == e;
        }
        // exclusive offsets in (digit, thread) order: digit totals before d, plus this digit's
        // counts of the threads before t — a wave scan per digit, the waves' totals through LDS,
        // their (digit, wave) exclusive prefix by one wave, read back once per digit
        int pre[16];
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int v = wave_scan_incl(c[e]);
            pre[e] = v - c[e];
            if (lane == 63) waveTot[wave][e] = v;
        }
        __syncthreads();
        if (wave == 0) {   // lane l < 16 * kWaves / 64 ... one entry (digit e, wave w) per step, in order
            int run = 0;
            for (int e0 = 0; e0 < 16 * kWaves; e0 += 64) {
                const int q = e0 + lane, e = q / kWaves, w = q - e * kWaves;
                const int v = waveTot[w][e];
                const int incl = wave_scan_incl(v);
                wavePre[w][e] = run + incl - v;
                run += __builtin_amdgcn_readlane(incl, 63);
            }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 16; e++) pre[e] += wavePre[wave][e];
        for (int i = lo; i < hi; i++) {
            const uint16_t v = idx[src][i];
            const int d = (key[v] >> shift) & 15;
            int pos = 0;
#pragma unroll
            for (int e = 0; e < 16; e++) {
                pos = d == e ? pre[e] : pos;
                pre[e] += d == e;
            }
            idx[src ^ 1][pos] = v;
        }
    }
    __syncthreads();
    for (int i = t; i < n; i += kOrderThreads) a.out[i] = shard_block_id(a, idx[src][i]);
}

__global__ __launch_bounds__(kThreads) void block_list_kernel(ShardArgs a) {
    const int j = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (j < a.numBlocks) a.out[j] = shard_block_id(a, j);
}

// Per block: hits among its rays (id >= 0, RendererKernels.cu:131), one partial.
__global__ __launch_bounds__(kThreads) void count_partial_kernel(const int4* results, int n, int perBlock,
                                                                int32_t* partial) {
    __shared__ int waveSum[kThreads / 64];
    const int begin = (int)blockIdx.x * perBlock;
    const int end = min(begin + perBlock, n);
    int c = 0;
    for (int i = begin + (int)threadIdx.x; i < end; i += kThreads) c += results[i].x >= 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) waveSum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kThreads / 64; w++) t += waveSum[w];
        partial[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kThreads) void count_final_kernel(const int32_t* partial, int m, int32_t* out) {
    __shared__ int waveSum[kThreads / 64];
    int c = 0;
    for (int i = (int)threadIdx.x; i < m; i += kThreads) c += partial[i];
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) waveSum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kThreads / 64; w++) t += waveSum[w];
        *out = t;
    }
}

struct ReconstructArgs {
    int numRaysPerPrimary, firstPrimary, numPrimary, rayType;
    const int32_t* primarySlotToId;
    const int4* primaryResults;
    const int32_t* batchIdToSlot;   // NULL: identity (the device/host generators' layout)
    const int4* batchResults;
    const uint32_t* triMaterialColor;
    const uint32_t* triShadedColor;
    uint32_t* pixels;
};

// fromABGR / toABGR of RendererKernels.cu:38-56 (device variant: truncating, not rounding).
__device__ inline float4 from_abgr(uint32_t c) {
    const float k = 1.0f / 255.0f;
    return make_float4((float)(c & 0xFF) * k, (float)((c >> 8) & 0xFF) * k, (float)((c >> 16) & 0xFF) * k,
                       (float)(c >> 24) * k);
}
__device__ inline uint32_t to_abgr(float4 v) {
    return (uint32_t)(fminf(fmaxf(v.x, 0.0f), 1.0f) * 255.0f) |
           ((uint32_t)(fminf(fmaxf(v.y, 0.0f), 1.0f) * 255.0f) << 8) |
           ((uint32_t)(fminf(fmaxf(v.z, 0.0f), 1.0f) * 255.0f) << 16) |
           ((uint32_t)(fminf(fmaxf(v.w, 0.0f), 1.0f) * 255.0f) << 24);
}

__device__ inline void add_sample(float4& c, int tri, bool isPrimary, bool isAO, const uint32_t* shaded) {
    float4 add;
    if (tri == -1) add = isPrimary ? make_float4(0.2f, 0.4f, 0.8f, 1.0f) : make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    else add = isAO ? make_float4(0.0f, 0.0f, 0.0f, 1.0f) : from_abgr(shaded[tri]);
    c.x += add.x; c.y += add.y; c.z += add.z; c.w += add.w;
}

// Average -> AO background -> diffuse modulation -> one ABGR pixel (RendererKernels.cu:96-107).
__device__ inline void finish_pixel(const ReconstructArgs& a, float4 c, int primarySlot) {
    const float4 bg = make_float4(0.2f, 0.4f, 0.8f, 1.0f);
    const float inv = 1.0f / (float)a.numRaysPerPrimary;
    c.x *= inv; c.y *= inv; c.z *= inv; c.w *= inv;
    const int tri = a.primaryResults[primarySlot].x;
    if (a.rayType == MRT_RAY_AO && tri == -1) c = bg;
    if (a.rayType == MRT_RAY_DIFFUSE) {
        const float4 m = tri == -1 ? bg : from_abgr(a.triMaterialColor[tri]);
        c.x *= m.x; c.y *= m.y; c.z *= m.z; c.w *= m.w;
    }
    a.pixels[a.primarySlotToId[primarySlot]] = to_abgr(c);
}

// One thread per primary ray of the batch: average the batch rays' colours
// (background / white / shaded triangle colour), modulate by the primary hit's
// material for diffuse, write one ABGR pixel (RendererKernels.cu:60-108).
// General form: any batchIdToSlot (gathers), and the primary batch.
__global__ __launch_bounds__(kThreads) void reconstruct_kernel(ReconstructArgs a) {
    const int task = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (task >= a.numPrimary) return;
    const int n = a.numRaysPerPrimary;
    const bool isPrimary = a.rayType == MRT_RAY_PRIMARY, isAO = a.rayType == MRT_RAY_AO;
    const int primarySlot = a.firstPrimary + task;
    const int batchBase = isPrimary ? a.primarySlotToId[primarySlot] : task * n;
    float4 c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int i = 0; i < n; i++) {
        const int slot = a.batchIdToSlot ? a.batchIdToSlot[batchBase + i] : (isPrimary ? primarySlot : batchBase + i);
        add_sample(c, a.batchResults[slot].x, isPrimary, isAO, a.triShadedColor);
    }
    finish_pixel(a, c, primarySlot);
}

// Identity-layout AO/diffuse batches (mrt_raygen_ao's): the block's n rays per
// primary are one contiguous run of results, so the hit ids are staged through
// LDS with coalesced loads (consecutive lanes, consecutive results) in tiles of
// kTileSamples per primary, then each thread sums its own samples in ray order
// (bit-identical to reconstruct_kernel). Row stride kTileSamples + 1 keeps the
// per-thread LDS reads conflict-free.
constexpr int kTileSamples = 16;
__global__ __launch_bounds__(kThreads) void reconstruct_tiled_kernel(ReconstructArgs a) {
    __shared__ int ids[kThreads * (kTileSamples + 1)];
    const int n = a.numRaysPerPrimary;
    const bool isAO = a.rayType == MRT_RAY_AO;
    const int taskBase = (int)blockIdx.x * kThreads;
    const int nTasks = min(kThreads, a.numPrimary - taskBase);
    const int t = (int)threadIdx.x;
    float4 c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int s0 = 0; s0 < n; s0 += kTileSamples) {
        const int ns = min(kTileSamples, n - s0);
        const int cnt = nTasks * ns;
        __syncthreads();
        for (int e = t; e < cnt; e += kThreads) {
            const int tt = e / ns, ss = e - tt * ns;
            ids[tt * (kTileSamples + 1) + ss] = a.batchResults[(int64_t)(taskBase + tt) * n + s0 + ss].x;
        }
        __syncthreads();
        if (t < nTasks)
            for (int ss = 0; ss < ns; ss++) add_sample(c, ids[t * (kTileSamples + 1) + ss], false, isAO, a.triShadedColor);
    }
    if (t < nTasks) finish_pixel(a, c, a.firstPrimary + taskBase + t);
}

int hip_fail(hipError_t e, const char* what) {
    return api_fail(MRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int kCountBlocks = 1024;

}  // namespace
}  // namespace mrt

using namespace mrt;

extern "C" {

int mrt_raygen_primary(const float nscreenToWorld[16], const float origin[3], float maxDist, int32_t w, int32_t h,
                       const int32_t* indexToPixel, void* rays, int32_t* slotToId, int32_t* idToSlot, void* stream) {
    return mrt_raygen_primary_subpixel(nscreenToWorld, origin, maxDist, w, h, 0.5f, 0.5f, indexToPixel, rays, slotToId,
                                       idToSlot, stream);
}

int mrt_raygen_primary_subpixel(const float nscreenToWorld[16], const float origin[3], float maxDist, int32_t w,
                                int32_t h, float jx, float jy, const int32_t* indexToPixel, void* rays,
                                int32_t* slotToId, int32_t* idToSlot, void* stream) {
    if (!nscreenToWorld || !origin || !indexToPixel || !rays) return api_fail(MRT_ERR_INVALID_ARG, "null argument");
    if (w <= 0 || h <= 0 || (int64_t)w * h > INT32_MAX) return api_fail(MRT_ERR_INVALID_ARG, "bad image size");
    if (!(jx >= 0.0f && jx < 1.0f && jy >= 0.0f && jy < 1.0f)) return api_fail(MRT_ERR_INVALID_ARG, "subpixel offset outside [0, 1)");
    PrimaryArgs a{};
    a.jx = jx;
    a.jy = jy;
    for (int i = 0; i < 16; i++) a.m[i] = nscreenToWorld[i];
    a.ox = origin[0]; a.oy = origin[1]; a.oz = origin[2];
    a.maxDist = maxDist;
    a.w = w; a.h = h;
    a.indexToPixel = indexToPixel;
    a.rays = static_cast<rg::RayRec*>(rays);
    a.slotToId = slotToId;
    a.idToSlot = idToSlot;
    const int n = w * h;
    hipLaunchKernelGGL(primary_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MRT_OK : hip_fail(e, "raygen primary launch");
}

int mrt_raygen_ao(const void* inRays, const void* inResults, int32_t numInputRays, const float* triNormals,
                  int64_t numTris, int32_t numSamples, float maxDist, uint32_t seed, void* outRays,
                  int32_t* outIdToSlot, int32_t* outSlotToId, void* stream) {
    if (numInputRays < 0 || numSamples < 1) return api_fail(MRT_ERR_INVALID_ARG, "bad ray/sample count");
    if (numInputRays == 0) return MRT_OK;
    if (!inRays || !inResults || !outRays || (numTris > 0 && !triNormals))
        return api_fail(MRT_ERR_INVALID_ARG, "null argument");
    if ((int64_t)numInputRays * numSamples > INT32_MAX) return api_fail(MRT_ERR_TOO_LARGE, "too many output rays");
    AOArgs a{};
    a.inRays = static_cast<const rg::RayRec*>(inRays);
    a.inResults = static_cast<const int2*>(inResults);
    a.numInput = numInputRays;
    a.normals = triNormals;
    a.numTris = numTris;
    a.numSamples = numSamples;
    a.maxDist = maxDist;
    a.seed = seed;
    a.outRays = static_cast<rg::RayRec*>(outRays);
    a.outIdToSlot = outIdToSlot;
    a.outSlotToId = outSlotToId;
    if (numSamples > 1) {
        const int64_t total = (int64_t)numInputRays * numSamples;
        hipLaunchKernelGGL(ao_per_sample_kernel, dim3((unsigned)((total + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           static_cast<hipStream_t>(stream), a);
    } else {
        hipLaunchKernelGGL(ao_kernel, dim3((numInputRays + kThreads - 1) / kThreads), dim3(kThreads), 0,
                           static_cast<hipStream_t>(stream), a);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MRT_OK : hip_fail(e, "raygen ao launch");
}

int mrt_raygen_ao_blocks(const void* inRays, const void* inResults, int32_t numInputRays, const float* triNormals,
                         int64_t numTris, int32_t numSamples, float maxDist, const uint32_t* batchSeeds,
                         int32_t numBatches, int32_t batchInputRays, const int32_t* blocks, int32_t numBlocks,
                         int32_t blockRays, int64_t numOutRays, void* outRays, void* stream) {
    if (numInputRays < 0 || numSamples < 1 || numBlocks < 0 || blockRays < 1 || batchInputRays < 1 || numOutRays < 0)
        return api_fail(MRT_ERR_INVALID_ARG, "bad ray/sample/block count");
    const int64_t total = (int64_t)numInputRays * numSamples;
    if (total > INT32_MAX) return api_fail(MRT_ERR_TOO_LARGE, "too many frame rays");
    const int64_t needBatches = ((int64_t)numInputRays + batchInputRays - 1) / batchInputRays;
    if (numBatches < needBatches) return api_fail(MRT_ERR_INVALID_ARG, "fewer batch seeds than batches");
    if (needBatches > kMaxBatchSeeds) return api_fail(MRT_ERR_TOO_LARGE, "more than 256 batches in the frame");
    const int64_t nb = (total + blockRays - 1) / blockRays;
    if (numBlocks > nb) return api_fail(MRT_ERR_INVALID_ARG, "more blocks listed than the frame has");
    if (numOutRays > (int64_t)numBlocks * blockRays || numOutRays < (int64_t)(numBlocks > 0 ? numBlocks - 1 : 0) * blockRays)
        return api_fail(MRT_ERR_INVALID_ARG, "numOutRays does not match the listed blocks");
    if (numOutRays == 0) return MRT_OK;
    if (!inRays || !inResults || !outRays || !blocks || !batchSeeds || (numTris > 0 && !triNormals))
        return api_fail(MRT_ERR_INVALID_ARG, "null argument");
    AOBlocksArgs a{};
    a.inRays = static_cast<const rg::RayRec*>(inRays);
    a.inResults = static_cast<const int2*>(inResults);
    a.numInput = numInputRays;
    a.normals = triNormals;
    a.numTris = numTris;
    a.numSamples = numSamples;
    a.maxDist = maxDist;
    a.batchInputs = batchInputRays;
    a.blockRays = blockRays;
    a.totalRays = total;
    a.outRays = numOutRays;
    a.blocks = blocks;
    a.out = static_cast<rg::RayRec*>(outRays);
    for (int64_t k = 0; k < needBatches; k++) a.seeds[k] = batchSeeds[k];
    if (blockRays % kTileRays == 0 && kTileRays % numSamples == 0 && kTileRays / numSamples <= kThreads &&
        numSamples <= kThreads)   // the tile's input rays and its sample points each fit one LDS slot per thread
        hipLaunchKernelGGL(ao_blocks_tiled_kernel, dim3((unsigned)((numOutRays + kTileRays - 1) / kTileRays)),
                           dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(ao_blocks_kernel, dim3((unsigned)((numOutRays + kThreads - 1) / kThreads)), dim3(kThreads),
                           0, static_cast<hipStream_t>(stream), a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MRT_OK : hip_fail(e, "raygen ao blocks launch");
}

int mrt_shard_blocks(const void* primaryResults, int32_t numPrimary, int32_t numSamples, int32_t blockRays,
                     int32_t world, int32_t rank, int32_t order, int32_t* blocks, int32_t capacity, int32_t* numBlocks,
                     int64_t* numRays, void* stream) {
    if (numPrimary < 0 || numSamples < 1 || blockRays < 1 || world < 1 || rank < 0 || rank >= world ||
        (order != 0 && order != 1) || !numBlocks || !numRays)
        return api_fail(MRT_ERR_INVALID_ARG, "bad shard arguments");
    const int64_t total = (int64_t)numPrimary * numSamples;
    if (total > INT32_MAX) return api_fail(MRT_ERR_TOO_LARGE, "too many frame rays");
    const int64_t nb = (total + blockRays - 1) / blockRays;
    const int64_t mine = nb > rank ? (nb - 1 - rank) / world + 1 : 0;
    const bool lastMine = mine > 0 && (nb - 1) % world == rank;
    *numBlocks = (int32_t)mine;
    *numRays = mine * blockRays - (lastMine ? nb * blockRays - total : 0);
    if (mine == 0 || !blocks) return MRT_OK;   // blocks NULL: a size query
    if (capacity < mine) return api_fail(MRT_ERR_TOO_LARGE, "block list capacity below the shard's blocks");
    if (order == 1 && mine > kOrderMax)
        return api_fail(MRT_ERR_TOO_LARGE, "live-first order holds at most 16384 blocks per rank (use larger blocks)");
    if (order == 1 && !primaryResults) return api_fail(MRT_ERR_INVALID_ARG, "null primary results");
    hipStream_t s = static_cast<hipStream_t>(stream);
    ShardArgs a{};
    a.results = static_cast<const int2*>(primaryResults);
    a.numPrimary = numPrimary;
    a.numSamples = numSamples;
    a.blockRays = blockRays;
    a.world = world;
    a.rank = rank;
    a.numBlocks = (int)mine;
    a.totalRays = total;
    a.out = blocks;
    if (order == 0) {
        hipLaunchKernelGGL(block_list_kernel, dim3((unsigned)((mine + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, a);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MRT_OK : hip_fail(e, "shard block list launch");
    }
    hipLaunchKernelGGL(block_live_kernel, dim3((unsigned)((mine * 64 + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL(block_order_kernel, dim3(1), dim3(kOrderThreads), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MRT_OK : hip_fail(e, "shard order launch");
}

int mrt_count_hits(const void* results, int32_t numRays, int32_t* hitCount, void* stream) {
    if (!hitCount || numRays < 0 || (numRays > 0 && !results)) return api_fail(MRT_ERR_INVALID_ARG, "bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int perBlock = ((numRays + kCountBlocks - 1) / kCountBlocks + kThreads - 1) / kThreads * kThreads;
    const int blocks = perBlock > 0 ? (numRays + perBlock - 1) / perBlock : 0;
    // Stream-ordered scratch for the per-block partials (no state shared between calls).
    int32_t* partial = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&partial), (size_t)(blocks + 1) * sizeof(int32_t), s);
    if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(count partials)");
    if (blocks > 0)
        hipLaunchKernelGGL(count_partial_kernel, dim3(blocks), dim3(kThreads), 0, s,
                           static_cast<const int4*>(results), numRays, perBlock, partial);
    hipLaunchKernelGGL(count_final_kernel, dim3(1), dim3(kThreads), 0, s, partial, blocks, hitCount);
    e = hipGetLastError();
    const hipError_t f = hipFreeAsync(partial, s);
    if (e != hipSuccess) return hip_fail(e, "count hits launch");
    return f == hipSuccess ? MRT_OK : hip_fail(f, "hipFreeAsync(count partials)");
}

int mrt_reconstruct(int32_t rayType, int32_t numRaysPerPrimary, int32_t firstPrimary, int32_t numPrimary,
                    const int32_t* primarySlotToId, const void* primaryResults, const int32_t* batchIdToSlot,
                    const void* batchResults, const uint32_t* triMaterialColor, const uint32_t* triShadedColor,
                    uint32_t* pixels, void* stream) {
    if (rayType < MRT_RAY_PRIMARY || rayType > MRT_RAY_DIFFUSE) return api_fail(MRT_ERR_INVALID_ARG, "bad ray type");
    if (numRaysPerPrimary < 1 || firstPrimary < 0 || numPrimary < 0 ||
        (rayType == MRT_RAY_PRIMARY && numRaysPerPrimary != 1))
        return api_fail(MRT_ERR_INVALID_ARG, "bad batch shape");
    if ((int64_t)numPrimary * numRaysPerPrimary > INT32_MAX || (int64_t)firstPrimary + numPrimary > INT32_MAX)
        return api_fail(MRT_ERR_TOO_LARGE, "too many rays");
    if (numPrimary == 0) return MRT_OK;
    if (!primarySlotToId || !primaryResults || !batchResults || !pixels ||
        (rayType != MRT_RAY_AO && !triShadedColor) || (rayType == MRT_RAY_DIFFUSE && !triMaterialColor))
        return api_fail(MRT_ERR_INVALID_ARG, "null argument");
    ReconstructArgs a{};
    a.numRaysPerPrimary = numRaysPerPrimary;
    a.firstPrimary = firstPrimary;
    a.numPrimary = numPrimary;
    a.rayType = rayType;
    a.primarySlotToId = primarySlotToId;
    a.primaryResults = static_cast<const int4*>(primaryResults);
    a.batchIdToSlot = batchIdToSlot;
    a.batchResults = static_cast<const int4*>(batchResults);
    a.triMaterialColor = triMaterialColor;
    a.triShadedColor = triShadedColor;
    a.pixels = pixels;
    const dim3 grid((numPrimary + kThreads - 1) / kThreads);
    if (rayType != MRT_RAY_PRIMARY && !batchIdToSlot)
        hipLaunchKernelGGL(reconstruct_tiled_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(reconstruct_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MRT_OK : hip_fail(e, "reconstruct launch");
}

}  // extern "C"
