// ubench_levels.hip — calibration of the cache-level counters the bench's
// per-level roofline reads (TCP_TOTAL_CACHE_ACCESSES, TCP_TCC_READ_REQ, TCC_REQ,
// TCC_HIT/MISS, TCC_EA0_RDREQ, FETCH_SIZE), on the trace kernel's own access
// shapes with a known byte count, from three footprints: one XCD's L2 (2 MiB),
// the Infinity Cache (64 MiB) and HBM (2 GiB).
//
//   shape L (node-like): every lane reads one whole random 128-B line as eight
//     16-B buffer loads (the 4-wide node fetch: 7-8 dwordx4 of one line);
//   shape S (sparse):    every lane reads one random 16-B slot per load (a
//     lane's first triangle row of a leaf).
//
// Each (shape, footprint) kernel has its own name (template tags), runs once to
// warm the footprint and once measured; the program prints the dispatch order,
// the bytes each measured launch requested and its time. Run it under separate
// rocprofv3 --pmc passes (tools/calib_levels.sh) and divide counters by the
// known request counts.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_levels tools/ubench_levels.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__device__ __forceinline__ float4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// TAG: 0..2 footprint, +0 line shape / +8 sparse shape, +16 warm pass
template <int TAG>
__global__ __launch_bounds__(256) void levels_kernel(const float4* table, uint32_t lines, int iters, float4* out) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)table, 0, (int)0x7fffffff, 0x00020000);   // offsets < 2^31
    uint32_t h = (blockIdx.x * 256u + threadIdx.x + 1u) * 2654435761u;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr bool sparse = (TAG & 8) != 0;
    for (int i = 0; i < iters; i++) {
        h = h * 1664525u + 1013904223u;
        const uint32_t line = (h >> 3) % lines;
        if constexpr (sparse) {
            const float4 a = ld16(r, line * 128u + (h & 7u) * 16u);
            acc.x += a.x;
            acc.y += a.w;
        } else {
            const uint32_t o = line * 128u;
            const float4 a = ld16(r, o), b = ld16(r, o + 16u), c = ld16(r, o + 32u), d = ld16(r, o + 48u);
            const float4 e = ld16(r, o + 64u), f = ld16(r, o + 80u), g = ld16(r, o + 96u), k = ld16(r, o + 112u);
            acc.x += a.x + b.y + c.z + d.w;
            acc.y += e.x + f.y + g.z + k.w;
        }
    }
    if (acc.x == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = acc;   // keeps the loads; never true here
}

template <int TAG>
float run(const float4* table, uint32_t lines, int iters, float4* out, int blocks, hipEvent_t e0, hipEvent_t e1) {
    levels_kernel<TAG | 16><<<blocks, 256>>>(table, lines, iters, out);   // warm: the footprint into its level
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    levels_kernel<TAG><<<blocks, 256>>>(table, lines, iters, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 4;   // 16 waves/CU
    const size_t lanes = (size_t)blocks * 256;
    const size_t sizes[3] = {2ull << 20, 64ull << 20, 2048ull << 20};
    float4* table;
    float4* out;
    CHECK(hipMalloc(&table, sizes[2]));
    CHECK(hipMemset(table, 0, sizes[2]));
    CHECK(hipMalloc(&out, lanes * 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("# %d CUs, %d workgroups x 256, %zu lanes; each footprint: warm launch, then measured launch\n", cus,
                blocks, lanes);
    std::printf("# kernel tag, footprint MiB, shape, wave loads, lane 16-B loads, bytes requested, ms, GB/s\n");
    const int itL = 64, itS = 256;
    float ms[6];
    ms[0] = run<0>(table, (uint32_t)(sizes[0] / 128), itL, out, blocks, e0, e1);
    ms[1] = run<1>(table, (uint32_t)(sizes[1] / 128), itL, out, blocks, e0, e1);
    ms[2] = run<2>(table, (uint32_t)(sizes[2] / 128), itL, out, blocks, e0, e1);
    ms[3] = run<8>(table, (uint32_t)(sizes[0] / 128), itS, out, blocks, e0, e1);
    ms[4] = run<9>(table, (uint32_t)(sizes[1] / 128), itS, out, blocks, e0, e1);
    ms[5] = run<10>(table, (uint32_t)(sizes[2] / 128), itS, out, blocks, e0, e1);
    for (int k = 0; k < 6; k++) {
        const bool sparse = k >= 3;
        const size_t laneLoads = lanes * (sparse ? itS : 8 * itL);
        const size_t waveLoads = laneLoads / 64;
        const double bytes = (double)laneLoads * 16;
        std::printf("%d %zu %s %zu %zu %.0f %.4f %.1f\n", (sparse ? 8 : 0) + k % 3, sizes[k % 3] >> 20,
                    sparse ? "sparse16" : "line128", waveLoads, laneLoads, bytes, ms[k], bytes / (ms[k] * 1e-3) / 1e9);
    }
    CHECK(hipFree(table));
    CHECK(hipFree(out));
    return 0;
}
