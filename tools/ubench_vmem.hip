// ubench_vmem.hip — what does one buffer_load_dwordx4 wave instruction cost the
// vector-memory data path on gfx950 when only some lanes are active?
//
// Every wave issues `iters` dependent rounds of 4 independent 16-B buffer loads
// (the shape of the trace kernel's node/triangle fetches) at pseudo-random
// 16-B-aligned offsets inside an L1-resident table; only lanes < `active` run the
// loop (exec-masked, as divergent lanes are in the traversal). Reported: CU
// cycles per wave-instruction at 20 waves/CU (2.4 GHz nominal clock). If the
// cost falls with fewer active lanes, the data path charges per lane; if it stays,
// it charges per instruction.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_vmem tools/ubench_vmem.hip
//   tools/ubench_vmem [table_kib]
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

__global__ __launch_bounds__(256) void vmem_kernel(const float4* table, int tableSlots, int iters, int active,
                                                   float4* out) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)table, 0, tableSlots * 16, 0x00020000);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < active) {
        uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
        for (int i = 0; i < iters; i++) {
            // four independent loads, then one dependent address update
            const uint32_t base = (h % (uint32_t)(tableSlots - 4)) * 16u;
            const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base, 0, 0));
            const float4 b = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base + 16u, 0, 0));
            const float4 c = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base + 32u, 0, 0));
            const float4 d = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base + 48u, 0, 0));
            acc.x += a.x + b.y;
            acc.y += c.z + d.w;
            h = h * 1664525u + 1013904223u + __float_as_uint(a.w + d.x);
        }
    }
    if (acc.x == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = acc;   // keep the loads; never true
}

int main(int argc, char** argv) {
    const int tableKiB = argc > 1 ? std::atoi(argv[1]) : 16;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int tableSlots = tableKiB * 1024 / 16;
    float4* table;
    float4* out;
    CHECK(hipMalloc(&table, (size_t)tableSlots * 16));
    CHECK(hipMemset(table, 0, (size_t)tableSlots * 16));
    const int blocks = cus * 5;   // 5 x 4 waves = 20 waves/CU
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 16));
    const int iters = 2000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("table %d KiB, %d CUs, 20 waves/CU, %d rounds x 4 dwordx4 loads per wave\n", tableKiB, cus, iters);
    const int actives[] = {64, 48, 32, 16, 8, 4, 1};
    for (int active : actives) {
        vmem_kernel<<<blocks, 256>>>(table, tableSlots, iters, active, out);   // warm
        CHECK(hipEventRecord(e0));
        vmem_kernel<<<blocks, 256>>>(table, tableSlots, iters, active, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double instrPerCU = 20.0 * iters * 4;
        const double cyc = ms * 1e-3 * 2.4e9 / instrPerCU;
        std::printf("active lanes %2d: %8.3f ms  %6.2f CU cycles per wave load  %7.1f GB/s of active-lane data per CU\n",
                    active, ms, cyc, instrPerCU * active * 16 / (ms * 1e-3) / 1e9);
    }
    CHECK(hipFree(table));
    CHECK(hipFree(out));
    return 0;
}
