// packet_kernel.hip — wave-packet traversal of the exact 4-wide nodes (gfx950).
//
// The per-lane kernel (trace_kernel.hip) gives each of a wave's 64 lanes its own walk:
// every step is a 16-B vector load per node row per lane, and the wave pays for its
// slowest lane's path. A batch of coherent rays (primary rays in Morton order: a wave's
// 64 rays are one 8x8 pixel tile) walks nearly the same nodes on every lane, so here the
// wave walks the tree ONCE for its 64 rays:
//   * the node or triangle being visited is wave-uniform, read with scalar loads into
//     SGPRs (one 112-B node or 48-B triangle per step for the whole wave, no per-lane
//     address, no TA/TD traffic), the slab and Woop tests run per lane on those SGPRs;
//   * each visit carries the 64-bit mask of the lanes whose own traversal reaches it (they
//     hit every box on its path); a child is entered by the lanes that hit its box, nearest
//     child first (the entry distance of the first such lane), the others go on a
//     wave-uniform stack in LDS as (ref, lane mask) pairs;
//   * a lane tests a leaf's triangles only when it hit the leaf's box, so every lane tests
//     a subset of the leaves its own depth-first walk tests and all of those that can hold
//     its closest hit: closest hits are the per-lane kernel's (exact-t ties aside), results
//     and arithmetic (slab planes, Woop test, exact or v_rcp reciprocal) are identical.
// Closest-hit only; the leaf refs must carry their triangle counts (wide_bvh.cpp). Waves
// take 64-ray tiles: one static tile each, then one atomic per wave per tile from the head
// of their XCD's share (no stealing; the last share to drain is the slowest XCD's).
#include "trace_kernel.hpp"

namespace mrt {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
// Node and triangle rows through the constant address space: with a wave-uniform index
// these are scalar loads (s_load_dwordx4/x8/x16 into SGPRs). The BVH is read-only for the
// whole launch.
typedef float v4f __attribute__((ext_vector_type(4)));
typedef const v4f __attribute__((address_space(4)))* CF4;

__device__ __forceinline__ int f2i(float f) { return __float_as_int(f); }
__device__ __forceinline__ float i2f(int i) { return __int_as_float(i); }

// The slab test's min/max as in trace_kernel.hip (reference spanBeginKepler/spanEndKepler).
__device__ __forceinline__ float span_begin(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    const int z = max(min(f2i(c0), f2i(c1)), f2i(d));
    return i2f(max(max(f2i(fminf(a0, a1)), f2i(fminf(b0, b1))), z));
}
__device__ __forceinline__ float span_end(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    const int z = min(max(f2i(c0), f2i(c1)), f2i(d));
    return i2f(min(min(f2i(fmaxf(a0, a1)), f2i(fmaxf(b0, b1))), z));
}

template <bool EXACT>
__device__ __forceinline__ float recip(float x) {
    if constexpr (EXACT) {   // correctly rounded under FTZ (trace_kernel.hip rcp_exact)
        const float r0 = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r0, 1.0f);
        const float r1 = __builtin_fmaf(r0, e, r0);
        return (e != e) ? r0 : r1;
    } else {
        return __builtin_amdgcn_rcpf(x);
    }
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

template <bool EXACT>
__global__ __launch_bounds__(kBlockThreads) void packet_kernel(TraceArgs a) {
    constexpr int kW = kBlockThreads / 64;
    __shared__ int stackRef[kW * kPacketStack];
    __shared__ uint64_t stackMask[kW * kPacketStack];
    const int lane = (int)(threadIdx.x & 63);
    const int w = (int)(threadIdx.x >> 6);
    int* const sref = stackRef + w * kPacketStack;
    uint64_t* const smask = stackMask + w * kPacketStack;
    const CF4 nodes = (CF4)(uintptr_t)a.nodes;
    const CF4 woop = (CF4)(uintptr_t)a.woop;
    const __amdgpu_buffer_rsrc_t triRsrc =   // one int per woop float4, range-checked like trace_kernel.hip
        __builtin_amdgcn_make_buffer_rsrc((void*)a.triIndex, 0, (int)(a.woopBytes / 4u), 0x00020000);

    // Tiles: group g = blockIdx % 8 (one XCD under the round-robin placement) owns the
    // contiguous tiles [g*C, (g+1)*C); its waves take one each statically, then count on
    // through the group's head (queues[g]).
    const int numTiles = (a.numRays + 63) >> 6;
    const int groups = ((gridDim.x & 7u) == 0) ? 8 : 1;
    const int group = (int)(blockIdx.x % (unsigned)groups);
    const int groupWaves = (int)gridDim.x / groups * kW;
    const int per = (numTiles + groups - 1) / groups;
    const int tBegin = min(group * per, numTiles), tEnd = min(tBegin + per, numTiles);
    int local = (int)(blockIdx.x / (unsigned)groups) * kW + w;

    while (tBegin + local < tEnd) {
        const int rayidx = (tBegin + local) * 64 + lane;
        const bool has = rayidx < a.numRays;
        float ox = 0.f, oy = 0.f, oz = 0.f, tmin = 0.f, dx = 0.f, dy = 0.f, dz = 0.f, hitT = -1.f;
        if (has) {
            const float4 o = a.rays[2 * (size_t)rayidx + 0];
            const float4 d = a.rays[2 * (size_t)rayidx + 1];
            ox = o.x; oy = o.y; oz = o.z; tmin = o.w;
            dx = d.x; dy = d.y; dz = d.z; hitT = d.w;
        }
        // reference kepler_dynamic_fetch.cu:123-140 (2^-80 clamp, 1/d, o * (1/d) unfused)
        const float ooeps = 0x1p-80f;
        const float idirx = recip<EXACT>(fabsf(dx) > ooeps ? dx : copysignf(ooeps, dx));
        const float idiry = recip<EXACT>(fabsf(dy) > ooeps ? dy : copysignf(ooeps, dy));
        const float idirz = recip<EXACT>(fabsf(dz) > ooeps ? dz : copysignf(ooeps, dz));
        const float oodx = ox * idirx, oody = oy * idiry, oodz = oz * idirz;
        const f2 ix = {idirx, idirx}, iy = {idiry, idiry}, iz = {idirz, idirz};
        const f2 nx = {-oodx, -oodx}, ny = {-oody, -oody}, nz = {-oodz, -oodz};
        int hitIndex = -1;

        uint64_t cur = __ballot(has);   // the lanes whose walk reaches the current node
        int node = 0;                   // the root; < 0: a leaf ref
        int sp = 0;
        for (;;) {
            const bool part = (cur >> lane) & 1ull;
            if (node >= 0) {
                const CF4 n = nodes + node;
                const v4f qx01 = n[0], qx23 = n[1], qy01 = n[2], qy23 = n[3], qz01 = n[4], qz23 = n[5], qc = n[6];
                float key[4];
                const v4f* const qx[2] = {&qx01, &qx23};
                const v4f* const qy[2] = {&qy01, &qy23};
                const v4f* const qz[2] = {&qz01, &qz23};
#pragma unroll
                for (int h = 0; h < 2; h++) {   // trace_kernel.hip boxes4, child 2h and 2h+1
                    const f2 ax = __builtin_elementwise_fma(f2{qx[h]->x, qx[h]->y}, ix, nx);
                    const f2 bx = __builtin_elementwise_fma(f2{qx[h]->z, qx[h]->w}, ix, nx);
                    const f2 ay = __builtin_elementwise_fma(f2{qy[h]->x, qy[h]->y}, iy, ny);
                    const f2 by = __builtin_elementwise_fma(f2{qy[h]->z, qy[h]->w}, iy, ny);
                    const f2 az = __builtin_elementwise_fma(f2{qz[h]->x, qz[h]->y}, iz, nz);
                    const f2 bz = __builtin_elementwise_fma(f2{qz[h]->z, qz[h]->w}, iz, nz);
                    const float amin = span_begin(ax.x, ax.y, ay.x, ay.y, az.x, az.y, tmin);
                    const float amax = span_end(ax.x, ax.y, ay.x, ay.y, az.x, az.y, hitT);
                    const float bmin = span_begin(bx.x, bx.y, by.x, by.y, bz.x, bz.y, tmin);
                    const float bmax = span_end(bx.x, bx.y, by.x, by.y, bz.x, bz.y, hitT);
                    key[2 * h] = (part && amax >= amin) ? amin : __builtin_inff();
                    key[2 * h + 1] = (part && bmax >= bmin) ? bmin : __builtin_inff();
                }
                int ref[4] = {f2i(qc.x), f2i(qc.y), f2i(qc.z), f2i(qc.w)};
                uint64_t m[4];
                float rk[4];   // a child's rank: the entry distance of the first lane that enters it
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    m[c] = __ballot(key[c] != __builtin_inff());
                    rk[c] = m[c] ? __builtin_amdgcn_readlane(key[c], (int)__builtin_ctzll(m[c])) : __builtin_inff();
                }
                // five compare-exchanges sort the (rank, ref, mask) triples; the missed children last
                auto cx = [&](int i, int j) {
                    if (rk[j] < rk[i]) {
                        const float k = rk[i]; rk[i] = rk[j]; rk[j] = k;
                        const int r = ref[i]; ref[i] = ref[j]; ref[j] = r;
                        const uint64_t mm = m[i]; m[i] = m[j]; m[j] = mm;
                    }
                };
                cx(0, 1);
                cx(2, 3);
                cx(0, 2);
                cx(1, 3);
                cx(1, 2);
                if (m[0]) {
                    // the farther hit children onto the stack, farthest first; the nearest next
#pragma unroll
                    for (int c = 3; c >= 1; c--) {
                        if (m[c]) {
                            if (sp < kPacketStack) {
                                if (lane == 0) {
                                    sref[sp] = ref[c];
                                    smask[sp] = m[c];
                                }
                                ++sp;
                            } else if (lane == 0) {
                                atomicAdd(a.status, 1);   // cannot happen within stackBound (host check)
                            }
                        }
                    }
                    node = ref[0];
                    cur = m[0];
                    continue;
                }
            } else {
                // a leaf: its triangles, each tested by the lanes that hit the leaf's box
                // (trace_kernel.hip triangle; reference :315-396)
                const uint32_t lr = ~(uint32_t)node;
                const int count = (int)(lr >> kWideLeafAddrBits);
                const int first = (int)(lr & ((1u << kWideLeafAddrBits) - 1u));
                for (int j = 0; j < count; j++) {
                    const CF4 tri = woop + (first + 3 * j);
                    const v4f v00 = tri[0], v11 = tri[1], v22 = tri[2];
                    const float Oz = __builtin_fmaf(-oz, v00.z, __builtin_fmaf(-oy, v00.y, __builtin_fmaf(-ox, v00.x, v00.w)));
                    const float Dz = __builtin_fmaf(dz, v00.z, __builtin_fmaf(dx, v00.x, dy * v00.y));
                    const float t = Oz * recip<EXACT>(Dz);
                    const float Ox = __builtin_fmaf(oz, v11.z, __builtin_fmaf(oy, v11.y, __builtin_fmaf(ox, v11.x, v11.w)));
                    const float Dx = __builtin_fmaf(dz, v11.z, __builtin_fmaf(dx, v11.x, dy * v11.y));
                    const float u = __builtin_fmaf(Dx, t, Ox);
                    const float Oy = __builtin_fmaf(oz, v22.z, __builtin_fmaf(oy, v22.y, __builtin_fmaf(ox, v22.x, v22.w)));
                    const float Dy = __builtin_fmaf(dz, v22.z, __builtin_fmaf(dx, v22.x, dy * v22.y));
                    const float v = __builtin_fmaf(t, Dy, Oy);
                    const bool accept = part & (t > tmin) & (t < hitT) & (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f);
                    hitT = accept ? t : hitT;
                    hitIndex = accept ? first + 3 * j : hitIndex;
                }
            }
            if (sp == 0) break;
            --sp;
            node = uniform(sref[sp]);
            cur = uniform64(smask[sp]);
        }

        if (has) {
            const int id = hitIndex == -1 ? -1 : __builtin_amdgcn_raw_buffer_load_b32(triRsrc, (uint32_t)hitIndex * 4u, 0, 0);
            a.results[2 * (size_t)rayidx] = make_int2(id, f2i(hitT));
        }

        // the next tile: the first round is static, then one atomic per wave on the group's head
        int next = 0;
        if (lane == 0) next = (int)atomicAdd(&a.queues[group * kQueueStrideWords], 1u);
        local = groupWaves + uniform(__shfl(next, 0));
    }
}

}  // namespace

hipError_t launch_packet(bool exactRcp, const TraceArgs& a, int gridBlocks, hipStream_t s) {
    if (gridBlocks <= 0) return hipErrorInvalidValue;
    if (exactRcp)
        hipLaunchKernelGGL(packet_kernel<true>, dim3(gridBlocks), dim3(kBlockThreads), 0, s, a);
    else
        hipLaunchKernelGGL(packet_kernel<false>, dim3(gridBlocks), dim3(kBlockThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t packet_occupancy(bool exactRcp, int* blocksPerCU) {
    const void* fn = exactRcp ? reinterpret_cast<const void*>(packet_kernel<true>)
                              : reinterpret_cast<const void*>(packet_kernel<false>);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocksPerCU, fn, kBlockThreads, 0);
}

}  // namespace mrt
