// Layer-boundary cost on gfx950: a chain of L dependent "layers" (each reads the previous layer's
// buffer of S bytes and writes its own, and -- like a train-mode BatchNorm layer of the codec --
// publishes per-workgroup fp64 channel partial sums that every workgroup of the next layer reads
// back) run as
//   A) L kernels captured in one HIP graph (the ELBO step's structure): write-through (sc1) data
//      stores, fp64 stat atomics into 16 replicas, the next kernel sums the replicas;
//   B) ONE persistent kernel with an XCD-hierarchical grid barrier between layers: workgroups
//      grouped by blockIdx % 8 (the XCD under round-robin dispatch; any partition is correct), one
//      arrival counter per group on its own 128-B line, the group's last arriver bumps the top
//      counter, the top's last arriver publishes the epoch in a generation word that waiters poll
//      with relaxed sc1 loads + s_sleep.  Data and stat hand-off by write-through stores / memory-side
//      atomics and sc1 loads (no L2 writeback / invalidate fences needed: the guide's valid form);
//   C) as B with plain data stores and an agent release fence before arriving + acquire after.
// Every spin is bounded (give-up flag).  Reports microseconds per layer.  r02's version made every
// workgroup add to ONE counter with release/acquire fences per poll (serialised same-address
// atomics: 16 us at 288 workgroups); this one measures the barrier the persistent-codec design
// would actually use.
// Build: hipcc --offload-arch=gfx950 -O3 tools/boundary_bench.hip -o tools/boundary_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            printf("%s: %s\n", #x, hipGetErrorString(e));                         \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int NCH = 8;        // BN channels published per layer
constexpr int NREP = 16;      // stat replicas (as the codec's GPI_REPLICAS)
constexpr int SPIN_MAX = 1 << 22;

struct Sync {                  // zeroed by a memset before every launch
    unsigned grp[8][32];       // one 128-B line per group counter
    unsigned top[32];
    unsigned gen[32];
    unsigned fail[32];
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4_wt(float4* p, float4 v) {
    const f32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ float4 ld4_sc1(const float4* p) {
    f32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return float4{v[0], v[1], v[2], v[3]};
}

// ---------------------------------------------------------------- A) one kernel per layer
__global__ __launch_bounds__(256) void layer_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int n4,
                                                    const double* __restrict__ st_in, double* st_out) {
    __shared__ double coef[NCH];
    if (threadIdx.x < NCH) {          // the previous layer's statistics: sum of the replicas
        double s = 0.0;
        for (int r = 0; r < NREP; ++r) s += st_in[r * NCH + threadIdx.x];
        coef[threadIdx.x] = s;
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
        float4 v = src[i];
        v.x += (float)coef[i & (NCH - 1)] * 1e-30f;
        acc += v.x;
        st4_wt(&dst[i], v);
    }
    if (threadIdx.x < NCH) atomicAdd(&st_out[(blockIdx.x % NREP) * NCH + threadIdx.x], (double)acc);
}

__global__ void zero_stats(double* st, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) st[i] = 0.0;
}

// ---------------------------------------------------------------- B / C) persistent
template <bool FENCES>
__device__ __forceinline__ bool grid_barrier(Sync* s, unsigned epoch) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const int g = blockIdx.x & 7;
        const unsigned n_g = (gridDim.x - g + 7) / 8;      // workgroups with blockIdx % 8 == g
        unsigned old;
        if (FENCES)
            old = __hip_atomic_fetch_add(&s->grp[g][0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        else
            old = __hip_atomic_fetch_add(&s->grp[g][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == epoch * n_g - 1) {                      // last of its group
            const unsigned n_top = gridDim.x < 8 ? gridDim.x : 8;
            const unsigned t = __hip_atomic_fetch_add(&s->top[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (t == epoch * n_top - 1) __hip_atomic_store(&s->gen[0], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        int spin = 0;
        while (__hip_atomic_load(&s->gen[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
            __builtin_amdgcn_s_sleep(1);
            if (++spin > SPIN_MAX) {
                __hip_atomic_store(&s->fail[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
        }
        if (FENCES) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

template <bool FENCES>
__global__ __launch_bounds__(256) void persistent_kernel(float4* bufs, int n4, int layers, Sync* s, double* stats) {
    __shared__ double coef[NCH];
    __shared__ int okf;
    for (int l = 0; l < layers; ++l) {
        const float4* src = bufs + (size_t)(l & 1) * n4;
        float4* dst = bufs + (size_t)((l + 1) & 1) * n4;
        const double* st_in = stats + (size_t)(l & 1) * NREP * NCH;
        double* st_out = stats + (size_t)((l + 1) & 1) * NREP * NCH;
        if (threadIdx.x < NCH) {
            double sum = 0.0;
            for (int r = 0; r < NREP; ++r)
                sum += __hip_atomic_load(&st_in[r * NCH + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            coef[threadIdx.x] = sum;
        }
        __syncthreads();
        float acc = 0.f;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
            float4 v = FENCES ? src[i] : ld4_sc1(&src[i]);
            v.x += (float)coef[i & (NCH - 1)] * 1e-30f;
            acc += v.x;
            if (FENCES) dst[i] = v;
            else st4_wt(&dst[i], v);
        }
        if (threadIdx.x < NCH) atomicAdd(&st_out[(blockIdx.x % NREP) * NCH + threadIdx.x], (double)acc);
        // the stat atomics and write-through stores must have left the CU before arriving
        __builtin_amdgcn_s_waitcnt(0);
        const bool ok = grid_barrier<FENCES>(s, (unsigned)(l + 1));
        if (threadIdx.x == 0) okf = ok;
        __syncthreads();
        if (!okf) return;
    }
}

__global__ void empty_kernel() {}

int main() {
    const int L = 46;
    const size_t sizes[] = {64 << 10, 256 << 10, 2 << 20, 10 << 20};
    const int grids[] = {256, 288, 512, 1024};
    float4* bufs;
    Sync* sync;
    double* stats;
    CHECK(hipMalloc(&bufs, 2 * (10 << 20)));
    CHECK(hipMalloc(&sync, sizeof(Sync)));
    CHECK(hipMalloc(&stats, 2 * NREP * NCH * sizeof(double)));
    CHECK(hipMemset(stats, 0, 2 * NREP * NCH * sizeof(double)));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
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
            // A) graph of layer kernels (stats zeroed by a small kernel per layer, as the codec's
            //    statistics scratch is reset once per step)
            hipGraph_t g;
            hipGraphExec_t ge;
            CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int l = 0; l < L; ++l) {
                double* st_out = stats + (size_t)((l + 1) & 1) * NREP * NCH;
                const double* st_in = stats + (size_t)(l & 1) * NREP * NCH;
                hipLaunchKernelGGL(layer_kernel, dim3(G), dim3(256), 0, s, bufs + (size_t)(l & 1) * n4,
                                   bufs + (size_t)((l + 1) & 1) * n4, n4, st_in, st_out);
            }
            CHECK(hipStreamEndCapture(s, &g));
            CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(ge, s));
            CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < 20; ++r) CHECK(hipGraphLaunch(ge, s));
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms_g;
            CHECK(hipEventElapsedTime(&ms_g, e0, e1));
            float ms_p[2] = {0.f, 0.f};
            unsigned fail[2] = {0, 0};
            for (int f = 0; f < 2; ++f) {
                for (int r = 0; r < 21; ++r) {
                    if (r == 1) CHECK(hipEventRecord(e0, s));
                    CHECK(hipMemsetAsync(sync, 0, sizeof(Sync), s));
                    if (f == 0)
                        hipLaunchKernelGGL(persistent_kernel<false>, dim3(G), dim3(256), 0, s, bufs, n4, L, sync, stats);
                    else
                        hipLaunchKernelGGL(persistent_kernel<true>, dim3(G), dim3(256), 0, s, bufs, n4, L, sync, stats);
                }
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                CHECK(hipEventElapsedTime(&ms_p[f], e0, e1));
                Sync h;
                CHECK(hipMemcpy(&h, sync, sizeof(Sync), hipMemcpyDeviceToHost));
                fail[f] = h.fail[0];
            }
            printf("S %6zu KB grid %5d: graph %.2f us/layer   persistent xcd-barrier (write-through) %.2f us/layer%s"
                   "   (+fences) %.2f us/layer%s\n",
                   S >> 10, G, 1e3 * ms_g / 20 / L, 1e3 * ms_p[0] / 20 / L, fail[0] ? " GAVE UP" : "",
                   1e3 * ms_p[1] / 20 / L, fail[1] ? " GAVE UP" : "");
            fflush(stdout);
        }
    }
    return 0;
}
