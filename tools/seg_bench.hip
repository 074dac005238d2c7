// Small-plane codec segment: per-layer cost of a chain of L BN-coupled layers, each workgroup owning
// ONE sample's tile (T floats: 13 x 16 x 16 at 16^2, 10 x 8 x 8 at 8^2), as
//   A) L kernels captured in one HIP graph -- every layer loads its sample's tile from HBM (the
//      operand round trip every codec launch pays), sums the 16 stat replicas of the previous layer,
//      transforms the tile (BN + ReLU + a 3-tap row stencil), stores it write-through (sc1) and adds
//      its per-channel fp64 partial sums into the replicas;
//   D) ONE persistent kernel in which the tile stays in LDS across layers: only the fp64 channel sums
//      cross the grid barrier (the output still goes to HBM write-through, as the backward needs it);
//      D1 with the XCD-hierarchical barrier of tools/boundary_bench.hip (group counter -> top counter ->
//      generation word), D2 with a sharded counter (one 128-B line per blockIdx % 8 group; arrivals add
//      to their group's shard, every waiter polls all 8 shards with sc1 loads by 8 lanes of one wave).
// Correctness under load: every workgroup adds 1.0 to field 0 of channel 0 per layer, so after the
// barrier the replica sum must equal the grid; a smaller value is counted as a stale read.
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/seg_bench.hip -o tools/seg_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                     \
        }                                                                 \
    } while (0)

constexpr int NCH = 8;       // BN channels per layer
constexpr int NREP = 16;     // stat replicas
constexpr int SPIN_MAX = 1 << 20;

struct Sync {
    unsigned grp[8][32];     // XCD-group / shard counters, one 128-B line each
    unsigned top[32];
    unsigned gen[32];
    unsigned fail[32];
    unsigned stale[32];
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4_wt(float* p, f32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one layer's work on the LDS tile: coefficients from the replica sums, BN + ReLU + 3-tap row stencil
// into `out` (LDS), write-through store of `out` to HBM, per-channel partial sums -> replicas
__device__ __forceinline__ void layer_body(const float* tile, float* out, int T, const double* st_in, double* st_out,
                                          float* dst, float* coef, float* red, unsigned* stale, int grid) {
    const int tid = threadIdx.x;
    if (tid < NCH) {
        double s = 0.0, q = 0.0;
#pragma unroll
        for (int r = 0; r < NREP; ++r) {
            s += ld_sc1(&st_in[(r * NCH + tid) * 2]);
            q += ld_sc1(&st_in[(r * NCH + tid) * 2 + 1]);
        }
        if (tid == 0 && s < (double)grid - 0.5) atomicAdd(stale, 1u);
        coef[2 * tid] = (float)(1.0 / (1.0 + q * 1e-30));
        coef[2 * tid + 1] = (float)(s * 1e-30);
    }
    __syncthreads();
    const int per_ch = T / NCH;
    float ps[NCH], pq[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) ps[c] = pq[c] = 0.f;
    for (int i4 = tid; i4 < T / 4; i4 += 256) {
        const int i = 4 * i4, c = i / per_ch;
        const float a = coef[2 * c], b = coef[2 * c + 1];
        f32x4 v;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = i + u;
            const float l = j > 0 ? tile[j - 1] : 0.f, m = tile[j], r = j + 1 < T ? tile[j + 1] : 0.f;
            v[u] = fmaxf(fmaf(a, 0.25f * l + 0.5f * m + 0.25f * r, b), 0.f);
        }
        *reinterpret_cast<f32x4*>(out + i) = v;
        st4_wt(dst + i, v);
#pragma unroll
        for (int cc = 0; cc < NCH; ++cc) {
            if (cc == c) {
                ps[cc] += (v[0] + v[1]) + (v[2] + v[3]);
                pq[cc] += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
            }
        }
    }
    // block sums of the 16 partials (wave shuffles + LDS), one fp64 atomic per value per workgroup
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
        for (int o = 32; o > 0; o >>= 1) {
            ps[cc] += __shfl_xor(ps[cc], o, 64);
            pq[cc] += __shfl_xor(pq[cc], o, 64);
        }
    }
    const int lane = tid & 63, w = tid >> 6;
    if (lane == 0) {
#pragma unroll
        for (int cc = 0; cc < NCH; ++cc) {
            red[w * 2 * NCH + 2 * cc] = ps[cc];
            red[w * 2 * NCH + 2 * cc + 1] = pq[cc];
        }
    }
    __syncthreads();
    if (tid < 2 * NCH) {
        const float v = (red[tid] + red[2 * NCH + tid]) + (red[4 * NCH + tid] + red[6 * NCH + tid]);
        // field 0 of channel 0 also counts the workgroup (the stale-read check of the next layer)
        const double add = (double)v * 1e-30 + (tid == 0 ? 1.0 : 0.0);
        atomicAdd(&st_out[((blockIdx.x % NREP) * NCH + (tid >> 1)) * 2 + (tid & 1)], add);
    }
}

// ---------------------------------------------------------------- A) graph of layer kernels
__global__ __launch_bounds__(256) void layer_kernel(const float* __restrict__ src, float* __restrict__ dst, int T,
                                                    const double* st_in, double* st_out, Sync* s) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* tile = smem;
    float* out = tile + T;
    float* coef = out + T;
    float* red = coef + 2 * NCH;
    const float* sb = src + (size_t)blockIdx.x * T;
    for (int i4 = threadIdx.x; i4 < T / 4; i4 += 256)
        reinterpret_cast<float4*>(tile)[i4] = reinterpret_cast<const float4*>(sb)[i4];
    __syncthreads();
    layer_body(tile, out, T, st_in, st_out, dst + (size_t)blockIdx.x * T, coef, red, &s->stale[0], gridDim.x);
}

// zero the stats of layer l + 2 (so the graph can be replayed); seeds layer 0's count
__global__ void stats_init(double* st, int L, int grid) {
    for (int i = threadIdx.x; i < (L + 1) * NREP * NCH * 2; i += blockDim.x) st[i] = 0.0;
    __syncthreads();
    if (threadIdx.x == 0) st[0] = (double)grid;
}

// ---------------------------------------------------------------- D) persistent, tile in LDS
template <int MODE>   // 1: XCD-hierarchical barrier, 2: sharded counter
__device__ __forceinline__ bool grid_barrier(Sync* s, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores / atomics have left the CU
    __syncthreads();                                    // ... and every other wave's
    __shared__ int okf;
    if (threadIdx.x < 64) {
        const int g = blockIdx.x & 7;
        const unsigned G = gridDim.x;
        bool ok = true;
        if (MODE == 1) {
            if (threadIdx.x == 0) {
                const unsigned n_g = (G - g + 7) / 8;
                const unsigned old = __hip_atomic_fetch_add(&s->grp[g][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old == epoch * n_g - 1) {
                    const unsigned n_top = G < 8 ? G : 8;
                    const unsigned t = __hip_atomic_fetch_add(&s->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (t == epoch * n_top - 1)
                        __hip_atomic_store(&s->gen[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                int spin = 0;
                while (__hip_atomic_load(&s->gen[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spin > SPIN_MAX) { ok = false; break; }
                }
            }
        } else {
            const int lane = threadIdx.x;
            if (lane == 0) __hip_atomic_fetch_add(&s->grp[g][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // lanes 0..7 poll shard `lane`: done when every shard has all its group's arrivals of this epoch
            const unsigned n_l = lane < 8 ? (G > (unsigned)lane ? (G - lane + 7) / 8 : 0) : 0;
            const unsigned want = epoch * n_l;
            int spin = 0;
            for (;;) {
                unsigned v = want;
                if (lane < 8) v = __hip_atomic_load(&s->grp[lane][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool mine = v >= want;
                if (__all(mine)) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spin > SPIN_MAX) { ok = false; break; }
            }
        }
        if (threadIdx.x == 0) {
            if (!ok) __hip_atomic_store(&s->fail[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            okf = ok;
        }
    }
    __syncthreads();
    return okf != 0;
}

template <int MODE>
__global__ __launch_bounds__(256) void persistent_kernel(const float* __restrict__ src, float* bufs, int T, int L,
                                                         double* stats, Sync* s) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* t0 = smem;
    float* t1 = t0 + T;
    float* coef = t1 + T;
    float* red = coef + 2 * NCH;
    const float* sb = src + (size_t)blockIdx.x * T;
    for (int i4 = threadIdx.x; i4 < T / 4; i4 += 256)
        reinterpret_cast<float4*>(t0)[i4] = reinterpret_cast<const float4*>(sb)[i4];
    __syncthreads();
    for (int l = 0; l < L; ++l) {
        float* in = (l & 1) ? t1 : t0;
        float* out = (l & 1) ? t0 : t1;
        float* dst = bufs + ((size_t)(l & 1) * gridDim.x + blockIdx.x) * T;
        layer_body(in, out, T, stats + (size_t)l * NREP * NCH * 2, stats + (size_t)(l + 1) * NREP * NCH * 2, dst,
                   coef, red, &s->stale[0], gridDim.x);
        if (!grid_barrier<MODE>(s, (unsigned)(l + 1))) return;
    }
}

int main() {
    const int L = 16;
    const int Ts[] = {13 * 256, 10 * 64};
    const int grids[] = {256, 288};
    float *src, *bufs;
    double* stats;
    Sync* sync;
    const size_t maxT = 13 * 256, maxG = 288;
    CHECK(hipMalloc(&src, maxT * maxG * 4));
    CHECK(hipMalloc(&bufs, 2 * maxT * maxG * 4));
    CHECK(hipMalloc(&stats, (L + 1) * NREP * NCH * 2 * sizeof(double)));
    CHECK(hipMalloc(&sync, sizeof(Sync)));
    CHECK(hipMemset(src, 0, maxT * maxG * 4));
    CHECK(hipMemset(sync, 0, sizeof(Sync)));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int REPS = 50;
    for (int T : Ts) {
        for (int G : grids) {
            const size_t lds_a = (2 * T + 2 * NCH + 8 * NCH) * 4, lds_p = lds_a;
            // A) graph
            hipGraph_t g;
            hipGraphExec_t ge;
            CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            hipLaunchKernelGGL(stats_init, dim3(1), dim3(256), 0, st, stats, L, G);
            for (int l = 0; l < L; ++l) {
                const float* in = l == 0 ? src : bufs + (size_t)((l + 1) & 1) * maxT * maxG;
                float* out = bufs + (size_t)(l & 1) * maxT * maxG;
                hipLaunchKernelGGL(layer_kernel, dim3(G), dim3(256), lds_a, st, in, out, T,
                                   stats + (size_t)l * NREP * NCH * 2, stats + (size_t)(l + 1) * NREP * NCH * 2, sync);
            }
            CHECK(hipStreamEndCapture(st, &g));
            CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CHECK(hipMemset(sync, 0, sizeof(Sync)));
            for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(ge, st));
            CHECK(hipEventRecord(e0, st));
            for (int r = 0; r < REPS; ++r) CHECK(hipGraphLaunch(ge, st));
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms_a;
            CHECK(hipEventElapsedTime(&ms_a, e0, e1));
            Sync h;
            CHECK(hipMemcpy(&h, sync, sizeof(Sync), hipMemcpyDeviceToHost));
            const unsigned stale_a = h.stale[0];
            // D1 / D2) persistent: one graph of {memset sync, stats_init, persistent kernel}
            float ms_d[2];
            unsigned fail[2], stale[2];
            for (int m = 0; m < 2; ++m) {
                hipGraph_t gp;
                hipGraphExec_t gpe;
                CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
                CHECK(hipMemsetAsync(sync, 0, offsetof(Sync, fail), st));
                hipLaunchKernelGGL(stats_init, dim3(1), dim3(256), 0, st, stats, L, G);
                if (m == 0)
                    hipLaunchKernelGGL(persistent_kernel<1>, dim3(G), dim3(256), lds_p, st, src, bufs, T, L, stats, sync);
                else
                    hipLaunchKernelGGL(persistent_kernel<2>, dim3(G), dim3(256), lds_p, st, src, bufs, T, L, stats, sync);
                CHECK(hipStreamEndCapture(st, &gp));
                CHECK(hipGraphInstantiate(&gpe, gp, nullptr, nullptr, 0));
                CHECK(hipMemset(sync, 0, sizeof(Sync)));
                for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(gpe, st));
                CHECK(hipEventRecord(e0, st));
                for (int r = 0; r < REPS; ++r) CHECK(hipGraphLaunch(gpe, st));
                CHECK(hipEventRecord(e1, st));
                CHECK(hipEventSynchronize(e1));
                CHECK(hipEventElapsedTime(&ms_d[m], e0, e1));
                CHECK(hipMemcpy(&h, sync, sizeof(Sync), hipMemcpyDeviceToHost));
                fail[m] = h.fail[0];
                stale[m] = h.stale[0];
            }
            // the per-replay fixed cost (graph launch, stats_init, memset) is in every arm: report per layer
            // of the whole replay and the difference
            printf("T %5d floats grid %3d: A graph %.2f us/layer (stale %u) | D1 xcd-barrier %.2f us/layer (stale %u%s)"
                   " | D2 sharded %.2f us/layer (stale %u%s)\n",
                   T, G, 1e3 * ms_a / REPS / L, stale_a, 1e3 * ms_d[0] / REPS / L, stale[0], fail[0] ? " GAVE UP" : "",
                   1e3 * ms_d[1] / REPS / L, stale[1], fail[1] ? " GAVE UP" : "");
            fflush(stdout);
            CHECK(hipGraphExecDestroy(ge));
            CHECK(hipGraphDestroy(g));
        }
    }
    return 0;
}
