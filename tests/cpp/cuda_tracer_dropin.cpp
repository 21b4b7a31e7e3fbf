// cuda_tracer_dropin.cpp — the reference's host side, linked against libmrt.so.
//
// A C++ caller written the way the reference's CudaTracer::traceBatch()
// (src/rt/cuda/CudaTracer.cc:119-177) calls its kernel module: the four
// prototypes of src/rt/kernels/CudaTracerKernels.hh:42-52 with the reference's
// own parameter types (float4*, S64, Vec2i&, int4*, RayResult*), resolved at
// link time by libmrt.so instead of kepler_dynamic_fetch.o. Test program for
// tests/test_gpu_parity.py::test_cpp_host_links_reference_prototypes (the
// INTEGRATION.md "drop-in at link level" claim, exercised).
//
//   cuda_tracer_dropin NODES WOOP TRIINDEX RAYS ANYHIT OUT
// reads raw little-endian buffers (Compact2 nodes / woop / triIndex, Ray[n]),
// traces them and writes RayResult[n] (16 B each) to OUT.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int32_t S32;
typedef int64_t S64;
struct Vec2i { S32 x, y; };                              // framework/base/Math.hpp
struct RayResult { S32 id; float t; S32 padA, padB; };   // src/rt/Util.hh:79-89

// src/rt/kernels/CudaTracerKernels.hh:42-52, verbatim parameter types.
extern "C" {
void bind_CudaBVHTexture(float4* nodeBuf, S64 nodeBufSize, float4* triWoopBuf, S64 triWoopSize, int* triIndexBuf,
                         S64 triIndexSize);
void unbind_CudaBVHTexture(void);
float launch_tracingKernel(S32 nthreads, Vec2i& blockSize, int numRays, bool anyHit, float4* rays, int4* results,
                           float4* nodesA, float4* nodesB, float4* nodesC, float4* nodesD, float4* trisA,
                           float4* trisB, float4* trisC, int* triIndices);
void copy_tracing_results(RayResult* result_host, RayResult* result_dev, S32 size);
}

namespace {

std::vector<char> slurp(const char* path) {
    std::FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<char> b((size_t)n);
    if (n && std::fread(b.data(), 1, (size_t)n, f) != (size_t)n) { std::perror(path); std::exit(2); }
    std::fclose(f);
    return b;
}

template <class T> T* upload(const std::vector<char>& b) {
    void* p = nullptr;
    if (hipMalloc(&p, b.size() ? b.size() : 16) != hipSuccess) { std::fprintf(stderr, "hipMalloc failed\n"); std::exit(3); }
    if (!b.empty()) (void)hipMemcpy(p, b.data(), b.size(), hipMemcpyHostToDevice);
    return static_cast<T*>(p);
}

// The reference's CudaTracer, reduced to what traceBatch needs (CudaTracer.cc:119-177).
class CudaTracer {
public:
    void setBVH(float4* nodes, S64 nodeBytes, float4* woop, S64 woopBytes, int* triIndex, S64 triIndexBytes) {
        m_nodes = nodes; m_woop = woop; m_triIndex = triIndex;
        bind_CudaBVHTexture(nodes, nodeBytes, woop, woopBytes, triIndex, triIndexBytes);   // CudaTracer.cc:142-146
    }
    ~CudaTracer() { unbind_CudaBVHTexture(); }                                          // CudaTracer.cc:77-81
    float traceBatch(float4* rays, int4* results, int numRays, bool needClosestHit) {
        if (numRays == 0) return 0.0f;                                                   // CudaTracer.cc:123-125
        Vec2i blockSize = {32, 4};
        return launch_tracingKernel(90 * 32 * 8, blockSize, numRays, !needClosestHit, rays, results, m_nodes,
                                    nullptr, nullptr, nullptr, m_woop, nullptr, nullptr, m_triIndex);
    }
private:
    float4* m_nodes = nullptr;
    float4* m_woop = nullptr;
    int* m_triIndex = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s NODES WOOP TRIINDEX RAYS ANYHIT OUT\n", argv[0]);
        return 2;
    }
    const auto nodes = slurp(argv[1]), woop = slurp(argv[2]), tri = slurp(argv[3]), rays = slurp(argv[4]);
    const bool anyHit = std::atoi(argv[5]) != 0;
    const int n = (int)(rays.size() / 32);
    float4* dNodes = upload<float4>(nodes);
    float4* dWoop = upload<float4>(woop);
    int* dTri = upload<int>(tri);
    float4* dRays = upload<float4>(rays);
    int4* dRes = upload<int4>(std::vector<char>((size_t)n * sizeof(RayResult), 0));
    float ms;
    {
        CudaTracer tracer;
        tracer.setBVH(dNodes, (S64)nodes.size(), dWoop, (S64)woop.size(), dTri, (S64)tri.size());
        ms = tracer.traceBatch(dRays, dRes, n, !anyHit);
    }
    std::vector<RayResult> host((size_t)n);
    copy_tracing_results(host.data(), reinterpret_cast<RayResult*>(dRes), n);
    std::FILE* f = std::fopen(argv[6], "wb");
    if (!f || std::fwrite(host.data(), sizeof(RayResult), host.size(), f) != host.size()) { std::perror(argv[6]); return 2; }
    std::fclose(f);
    std::printf("traced %d rays in %.4f ms\n", n, ms);
    (void)hipFree(dNodes); (void)hipFree(dWoop); (void)hipFree(dTri); (void)hipFree(dRays); (void)hipFree(dRes);
    return 0;
}
