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
