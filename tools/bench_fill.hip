// Per-CU LDS fill rate of the load forms a conv tile stage can use (gfx950).
// Each 256-thread workgroup fills CHUNK bytes of LDS from a 64 MiB source
// (L2 / Infinity-Cache resident after the first pass), then writes one word so
// the loads are live.  Build: hipcc --offload-arch=gfx950 -O3 tools/bench_fill.hip -o /tmp/bench_fill
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHUNK (32 * 1024)
#define NF (CHUNK / 4)

__device__ __forceinline__ void glds(const float* g, float* l, int size) {
    if (size == 4)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 4, 0, 0);
    else
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// mode 0: glds dword contiguous, 1: glds dwordx4 contiguous, 2: glds dword rows of 18 (pitch 64 in global),
// 3: global_load_dword x8 -> ds_write_b32, 4: global_load_dwordx4 x4 -> ds_write_b128,
// 5: glds dwordx4 rows of 24 floats (6 chunks) with pitch 64
template <int MODE>
__global__ __launch_bounds__(256) void fill(const float* __restrict__ src, float* out, int nsrc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int tid = threadIdx.x, wb = tid & ~63;
    const float* base = src + ((size_t)blockIdx.x * NF * 2) % (size_t)(nsrc - 2 * NF);
    if (MODE == 0) {
        for (int e0 = 0; e0 < NF; e0 += 256) glds(base + e0 + tid, sm + e0 + wb, 4);
    } else if (MODE == 1) {
        for (int e0 = 0; e0 < NF; e0 += 1024) glds(base + e0 + 4 * tid, sm + e0 + 4 * wb, 16);
    } else if (MODE == 2) {
        for (int e0 = 0; e0 < NF; e0 += 256) {
            const int e = e0 + tid, r = e / 18, c = e - r * 18;
            glds(base + r * 64 + c, sm + e0 + wb, 4);
        }
    } else if (MODE == 3) {
        for (int e0 = 0; e0 < NF; e0 += 2048) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = base[e0 + u * 256 + tid];
#pragma unroll
            for (int u = 0; u < 8; ++u) sm[e0 + u * 256 + tid] = v[u];
        }
    } else if (MODE == 4) {
        for (int e0 = 0; e0 < NF; e0 += 4096) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const float4*)(base + e0 + u * 1024 + 4 * tid);
#pragma unroll
            for (int u = 0; u < 4; ++u) *(float4*)(sm + e0 + u * 1024 + 4 * tid) = v[u];
        }
    } else {
        for (int e0 = 0; e0 < NF; e0 += 1024) {
            const int q = (e0 >> 2) + tid, r = q / 6, c = q - r * 6;
            glds(base + r * 64 + 4 * c, sm + e0 + 4 * wb, 16);
        }
    }
    __syncthreads();
    if (tid == 0) out[blockIdx.x] = sm[(blockIdx.x * 97) % NF];
}

template <int MODE>
void run(const float* src, float* out, int nsrc, int nblocks, const char* name) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fill<MODE>, dim3(nblocks), dim3(256), CHUNK, 0, src, out, nsrc);
    hipEventRecord(a);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fill<MODE>, dim3(nblocks), dim3(256), CHUNK, 0, src, out, nsrc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = 1e3 * ms / reps;
    const double bytes = (double)nblocks * CHUNK;
    printf("%-36s blocks %5d  %8.2f us  %8.1f GB/s chip  %6.1f GB/s per CU\n", name, nblocks, us, bytes / us / 1e3,
           bytes / us / 1e3 / 256);
}

int main() {
    const int nsrc = 16 << 20;   // 64 MiB of floats
    float *src, *out;
    hipMalloc(&src, (size_t)nsrc * 4);
    hipMalloc(&out, 1 << 20);
    hipMemset(src, 0, (size_t)nsrc * 4);
    for (int nb : {256, 1024, 4096}) {
        run<0>(src, out, nsrc, nb, "glds dword contiguous");
        run<1>(src, out, nsrc, nb, "glds dwordx4 contiguous");
        run<2>(src, out, nsrc, nb, "glds dword rows of 18");
        run<5>(src, out, nsrc, nb, "glds dwordx4 rows of 24");
        run<3>(src, out, nsrc, nb, "load dword x8 + ds_write_b32");
        run<4>(src, out, nsrc, nb, "load dwordx4 x4 + ds_write_b128");
    }
    return 0;
}
