// Layer-boundary cost on gfx950: a chain of L dependent "layers" (each reads the previous
// layer's buffer of S bytes and writes its own) run as
//   A) L kernels captured in one HIP graph (the ELBO step's structure), and
//   B) ONE persistent kernel with a grid-wide barrier between layers (atomic arrival counter,
//      device-scope release / acquire fences), all workgroups resident;
// reports microseconds per layer.  Tells whether a multi-layer persistent codec kernel can beat
// kernel boundaries (multi-XCD L2 writeback / invalidate at every boundary either way).
// Build: hipcc --offload-arch=gfx950 -O3 tools/boundary_bench.hip -o /tmp/boundary_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void layer_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int n4) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
        float4 v = src[i];
        v.x += 1.f;
        dst[i] = v;
    }
}

__global__ __launch_bounds__(256) void layer_kernel_nt(const float4* __restrict__ src, float4* __restrict__ dst, int n4) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
        float4 v = src[i];
        v.x += 1.f;
        __builtin_nontemporal_store(v.x, &dst[i].x);
        __builtin_nontemporal_store(v.y, &dst[i].y);
        __builtin_nontemporal_store(v.z, &dst[i].z);
        __builtin_nontemporal_store(v.w, &dst[i].w);
    }
}

__device__ __forceinline__ void grid_barrier(unsigned* cnt, unsigned target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);   // this WG's writes visible
        while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void persistent_kernel(float4* bufs, int n4, int layers, unsigned* cnt, unsigned base) {
    for (int l = 0; l < layers; ++l) {
        const float4* src = bufs + (size_t)(l & 1) * n4;
        float4* dst = bufs + (size_t)((l + 1) & 1) * n4;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
            float4 v = src[i];
            v.x += 1.f;
            dst[i] = v;
        }
        grid_barrier(cnt, base + (unsigned)(l + 1) * gridDim.x);
    }
}

__global__ void empty_kernel() {}

int main() {
    const int L = 46;
    const size_t sizes[] = {256 << 10, 2 << 20, 6 << 20, 10 << 20};
    const int grids[] = {288, 1024};
    float4* bufs;
    unsigned* cnt;
    CHECK(hipMalloc(&bufs, 2 * (10 << 20)));
    CHECK(hipMalloc(&cnt, 256));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // empty kernels in a graph
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int l = 0; l < L; ++l) hipLaunchKernelGGL(empty_kernel, dim3(288), dim3(256), 0, s);
        CHECK(hipStreamEndCapture(s, &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e0, s));
        for (int r = 0; r < 50; ++r) CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("graph of %d empty kernels (288 WGs): %.2f us per kernel\n", L, 1e3 * ms / 50 / L);
    }
    for (size_t S : sizes) {
        const int n4 = (int)(S / 16);
        for (int G : grids) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int l = 0; l < L; ++l)
                hipLaunchKernelGGL(layer_kernel, dim3(G), dim3(256), 0, s, bufs + (size_t)(l & 1) * n4,
                                   bufs + (size_t)((l + 1) & 1) * n4, n4);
            CHECK(hipStreamEndCapture(s, &g));
            CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(ge, s));
            CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < 20; ++r) CHECK(hipGraphLaunch(ge, s));
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms_g;
            CHECK(hipEventElapsedTime(&ms_g, e0, e1));
            // non-temporal stores
            float ms_nt = 0;
            {
                hipGraph_t g2;
                hipGraphExec_t ge2;
                CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
                for (int l = 0; l < L; ++l)
                    hipLaunchKernelGGL(layer_kernel_nt, dim3(G), dim3(256), 0, s, bufs + (size_t)(l & 1) * n4,
                                       bufs + (size_t)((l + 1) & 1) * n4, n4);
                CHECK(hipStreamEndCapture(s, &g2));
                CHECK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
                for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(ge2, s));
                CHECK(hipEventRecord(e0, s));
                for (int r = 0; r < 20; ++r) CHECK(hipGraphLaunch(ge2, s));
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                CHECK(hipEventElapsedTime(&ms_nt, e0, e1));
            }
            printf("S %6zu KB  grid %5d: graph nt-stores %.2f us/layer\n", S >> 10, G, 1e3 * ms_nt / 20 / L);
            // persistent
            float ms_p = 0;
            CHECK(hipMemsetAsync(cnt, 0, 256, s));
            for (int r = 0; r < 21; ++r) {
                if (r == 1) CHECK(hipEventRecord(e0, s));
                hipLaunchKernelGGL(persistent_kernel, dim3(G), dim3(256), 0, s, bufs, n4, L, cnt, (unsigned)(r * L * G));
            }
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipEventElapsedTime(&ms_p, e0, e1));
            printf("S %6zu KB  grid %5d: graph %.2f us/layer (%.0f GB/s)   persistent %.2f us/layer (%.0f GB/s)\n",
                   S >> 10, G, 1e3 * ms_g / 20 / L, 2.0 * S / (1e-3 * ms_g / 20 / L) / 1e9, 1e3 * ms_p / 20 / L,
                   2.0 * S / (1e-3 * ms_p / 20 / L) / 1e9);
        }
    }
    return 0;
}
