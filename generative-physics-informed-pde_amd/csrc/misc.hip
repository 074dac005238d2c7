// Step plumbing kernels: gradient finalisation, flat Adam, device RNG.
#include "common.h"
#include <string.h>

using namespace gpi;

namespace {

__global__ __launch_bounds__(256) void grad_finalize_kernel(double* __restrict__ gacc, float* grad, int64_t n,
                                                            int flags, int64_t* step) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (step && i == 0) *step += 1;
    if (i >= n) return;
    const float g = (float)gacc[i];
    grad[i] = (flags & GPI_FINALIZE_ACCUMULATE) ? grad[i] + g : g;
    if (flags & GPI_FINALIZE_ZERO) gacc[i] = 0.0;
}

__global__ __launch_bounds__(256) void step_epilogue_kernel(gpi_step_epilogue_desc d) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (d.step && i == 0) *d.step += 1;
    if (i < d.n) {
        float g = (float)d.gacc[i];
        // the data-parallel error slot: this rank's hand-off timeout, summed over the ranks by the all-reduce
        if (i == d.err_slot && d.wait_err && __hip_atomic_load(d.wait_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            g = 1.f;
        d.grad[i] = (d.flags & GPI_FINALIZE_ACCUMULATE) ? d.grad[i] + g : g;
        if (d.flags & GPI_FINALIZE_ZERO) d.gacc[i] = 0.0;
    }
    if (i < d.n_scratch) {
        if (i < d.n_terms) d.terms_dst[i] = d.scratch[i];
        d.scratch[i] = 0.0;
    }
    if (i < d.n_idx) d.idx_dst[i] = d.idx_src[i];
    if (i * 4 < d.drop_n) {                      // gpi_dropout_masks' draw, Philox block i
        const uint64_t base = d.drop_offset ? *d.drop_offset : 0;
        const uint4_ r = philox(base + (uint64_t)i, d.drop_sub, d.drop_seed);
        const float u[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
        const float scale = 1.f / (1.f - d.drop_p);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i * 4 + k < d.drop_n) d.drop_out[i * 4 + k] = u[k] < d.drop_p ? 0.f : scale;
    }
}

// torch.optim.Adam's element update (torch/optim/adam.py single-tensor path, no weight decay /
// amsgrad / maximize), every rounding spelled out with explicit FMAs so that the separate Adam launch
// and the fused epilogue + Adam launch compute bit-identical results:
//   m.lerp_(g, 1 - beta1);  v.mul_(beta2).addcmul_(g, g, 1 - beta2);
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ void adam_element(float g, float& p, float& m, float& v, float beta1, float beta2,
                                             float eps, float step_size, float bc2_sqrt) {
    m = fmaf(1.f - beta1, g - m, m);
    v = fmaf(1.f - beta2, g * g, v * beta2);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = fmaf(-step_size, m / denom, p);
}

// The step epilogue with Adam fused in (single-process steps: no all-reduce between the gradient
// delivery and the update): element i's fp64 gradient -> grad[i] -> Adam on p[i], m[i], v[i], plus the
// epilogue's scratch / subset / dropout duties.  The step counter and the RNG offset are read by every
// workgroup (bias corrections, the dropout draw) and advanced once all of them have read them: by the
// last workgroup to finish (arrival counter *done, reset by that workgroup for the next launch).
__device__ __forceinline__ bool epilogue_wait(const uint32_t* flag, const int64_t* epoch, uint32_t* err);

// the sticky error word of a cross-stream wait (gpi_adam_desc.wait_err): set -> no parameter update
__device__ __forceinline__ bool wait_failed(const uint32_t* err) {
    return err && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// (grid-stride over at most GPI_EPILOGUE_MAX_WG workgroups: with one element per thread the grid of a 256^2
// step -- q_X rows of 32 x 2 x 65536 floats, ~16 k workgroups -- would fill every CU slot with workgroups
// spinning in epilogue_wait while the side stream still had kernels to dispatch)
// The skip decision is per workgroup: each re-reads the sticky error word after its own wait, so a workgroup
// that passes its wait after another one's timeout has been stored skips as well.  Only a timeout stored in the
// same instant as another workgroup's final re-read (the flag arriving just as the spin budget of ~10 s runs out)
// can leave part of that step's update applied -- the host raises on the word either way and no later step
// updates (the word is sticky): the "untouched" guarantee is best-effort within that window.
__global__ __launch_bounds__(256) void step_epilogue_adam_kernel(gpi_step_epilogue_desc d, gpi_adam_desc a,
                                                                 uint32_t* done, int64_t m_items) {
    bool skip = false;
    if (d.wait_flag) skip = epilogue_wait(d.wait_flag, a.step, d.wait_err);
    else if (a.wait_err) {
        __shared__ uint32_t s_bad;
        if (threadIdx.x == 0) s_bad = wait_failed(a.wait_err) ? 1u : 0u;
        __syncthreads();
        skip = s_bad != 0u;
    }
    const int64_t t = *a.step + 1;              // the step number after this step's increment
    const uint64_t base = d.drop_offset ? *d.drop_offset : 0;
    const float lr = *a.lr;
    const double bc1 = 1.0 - pow((double)a.beta1, (double)t);
    const double bc2 = 1.0 - pow((double)a.beta2, (double)t);
    const float step_size = (float)((double)lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float scale = 1.f / (1.f - d.drop_p);
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m_items; i += stride) {
        if (i < d.n) {
            const float g = (float)d.gacc[i];
            d.grad[i] = g;
            d.gacc[i] = 0.0;
            if (!skip) {
                float p = a.p[i], m = a.m[i], v = a.v[i];
                adam_element(g, p, m, v, a.beta1, a.beta2, a.eps, step_size, bc2_sqrt);
                a.m[i] = m;
                a.v[i] = v;
                a.p[i] = p;
            }
        }
        if (i < d.n_scratch) {
            if (i < d.n_terms) d.terms_dst[i] = d.scratch[i];
            d.scratch[i] = 0.0;
        }
        if (i < d.n_idx) d.idx_dst[i] = d.idx_src[i];
        if (i * 4 < d.drop_n) {
            const uint4_ r = philox(base + (uint64_t)i, d.drop_sub, d.drop_seed);
            const float u[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i * 4 + k < d.drop_n) d.drop_out[i * 4 + k] = u[k] < d.drop_p ? 0.f : scale;
        }
    }
    // every thread's reads of *step / *drop_offset are complete (their values were consumed above), so
    // a relaxed arrival suffices: the last arriver's writes come after every workgroup's reads
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            *const_cast<int64_t*>(a.step) = t;
            if (a.rng_offset) *a.rng_offset += a.rng_advance;
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// torch.optim.Adam single-tensor math (torch/optim/adam.py, defaults:
// no weight decay, no amsgrad, maximize=False).
__global__ __launch_bounds__(256) void adam_kernel(gpi_adam_desc d) {
    if (d.rng_offset && blockIdx.x == 0 && threadIdx.x == 0) *d.rng_offset += d.rng_advance;
    if (wait_failed(d.wait_err)) return;        // a timed-out hand-off: the gradient may be incomplete
    if (d.skip_if && *d.skip_if != 0.f) {      // ... on another rank (the all-reduced error slot)
        if (d.wait_err && blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(d.wait_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int64_t t = *d.step;
    const float lr = *d.lr;
    const double bc1 = 1.0 - pow((double)d.beta1, (double)t);
    const double bc2 = 1.0 - pow((double)d.beta2, (double)t);
    const float step_size = (float)((double)lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < d.n; i += (int64_t)gridDim.x * 256) {
        float p = d.p[i], m = d.m[i], v = d.v[i];
        adam_element(d.g[i], p, m, v, d.beta1, d.beta2, d.eps, step_size, bc2_sqrt);
        d.m[i] = m;
        d.v[i] = v;
        d.p[i] = p;
    }
}

__device__ __forceinline__ void randn_body(int64_t q, float* out, int64_t n, uint64_t seed, uint64_t base,
                                           uint64_t sub) {   // one Philox block q -> 4 normals
    if (q * 4 >= n) return;
    const uint4_ r = philox(base + (uint64_t)q, sub, seed);
    const float u0 = u01(r.x), u1 = u01(r.y), u2 = u01(r.z), u3 = u01(r.w);
    const float r0 = sqrtf(-2.f * logf(u0)), r1 = sqrtf(-2.f * logf(u2));
    const float t0 = 6.2831853071795864f * u1, t1 = 6.2831853071795864f * u3;
    float v[4] = {r0 * cosf(t0), r0 * sinf(t0), r1 * cosf(t1), r1 * sinf(t1)};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (q * 4 + k < n) out[q * 4 + k] = v[k];
}

__device__ __forceinline__ void dropout_body(int64_t q, float* out, int64_t n, float p, float scale, uint64_t seed,
                                             uint64_t base, uint64_t sub) {   // one Philox block -> 4 channels
    if (q * 4 >= n) return;
    const uint4_ r = philox(base + (uint64_t)q, sub, seed);
    const float u[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (q * 4 + k < n) out[q * 4 + k] = u[k] < p ? 0.f : scale;
}

__global__ __launch_bounds__(256) void randn_kernel(float* out, int64_t n, uint64_t seed, const uint64_t* offset,
                                                    uint64_t sub) {
    randn_body((int64_t)blockIdx.x * 256 + threadIdx.x, out, n, seed, offset ? *offset : 0, sub);
}

__global__ __launch_bounds__(256) void dropout_mask_kernel(float* out, int64_t n, float p, float scale, uint64_t seed,
                                                          const uint64_t* offset, uint64_t sub) {
    dropout_body((int64_t)blockIdx.x * 256 + threadIdx.x, out, n, p, scale, seed, offset ? *offset : 0, sub);
}

__global__ void rng_advance_kernel(uint64_t* offset, uint64_t by) { *offset += by; }

// random subset: the first k of the n indices ordered by (Philox key, index) -- a uniformly random
// k-subset in random order.  Each element's position is its rank, the number of (key, index) pairs
// below its own, counted in parallel: every workgroup draws all n keys into LDS and ranks EPB
// elements, TPE = 256 / EPB threads per element over strided slices of the keys, partial counts
// summed across the TPE lanes.  Same result as sorting the pairs (ranks of distinct pairs are
// distinct), without the sort's log^2 n dependent barrier steps in one workgroup (15 us at n = 1024).
__device__ __forceinline__ void subset_rank_body(int blk, uint32_t* hk, int32_t* out, int32_t n, int32_t k,
                                                 uint64_t seed, uint64_t base, uint64_t sub, int32_t epb) {
    for (int j = threadIdx.x; j < n; j += 256) hk[j] = philox(base + (uint64_t)j, sub, seed).x;
    __syncthreads();
    const int tpe = 256 / epb;
    const int e = threadIdx.x / tpe, part = threadIdx.x - e * tpe;
    const int i = blk * epb + e;
    int cnt = 0;
    if (i < n) {
        const uint32_t ki = hk[i];
        for (int j = part; j < n; j += tpe) {
            const uint32_t kj = hk[j];
            cnt += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
        }
    }
    // tpe consecutive lanes (a power of two <= 64 within one wave) hold one element's partial counts
    for (int m = 1; m < tpe; m <<= 1) cnt += __shfl_xor(cnt, m, 64);
    if (i < n && part == 0 && cnt < k) out[cnt] = i;
}

__global__ __launch_bounds__(256) void subset_rank_kernel(int32_t* out, int32_t n, int32_t k, uint64_t seed,
                                                          const uint64_t* offset, uint64_t sub, int32_t epb) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hk[];
    subset_rank_body(blockIdx.x, hk, out, n, k, seed, offset ? *offset : 0, sub, epb);
}

// elements per workgroup of the one-launch subset: about n / 256 (>= 4, <= 64, a power of two): enough
// workgroups to spread the n^2 comparisons, few enough that the n key draws per workgroup stay cheap
int subset_epb(int32_t n) {
    int32_t epb = 4;                      // >= 4: an element's 256 / epb lanes stay inside one wave
    while (epb < 64 && epb * 256 < n) epb <<= 1;
    return epb;
}

struct DrawArgs {
    gpi_draw_item it[GPI_MAX_DRAWS];
    int32_t first_block[GPI_MAX_DRAWS + 1];
    int32_t epb;
    int32_t n;
};

// gpi_draws: the items' workgroups by block range; every item's arithmetic is its own kernel's
__global__ __launch_bounds__(256) void draws_kernel(DrawArgs a, const uint64_t* offset) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hk[];
    int k = 0;
#pragma unroll
    for (int j = 1; j < GPI_MAX_DRAWS; ++j) k += (j < a.n && (int)blockIdx.x >= a.first_block[j]) ? 1 : 0;
    const gpi_draw_item it = a.it[k];
    const int blk = blockIdx.x - a.first_block[k];
    const uint64_t base = offset ? *offset : 0;
    const int64_t q = (int64_t)blk * 256 + threadIdx.x;
    if (it.kind == GPI_DRAW_RANDN) randn_body(q, (float*)it.out, it.n, it.seed, base, it.sub);
    else if (it.kind == GPI_DRAW_DROPOUT) dropout_body(q, (float*)it.out, it.n, it.p, 1.f / (1.f - it.p), it.seed, base, it.sub);
    else subset_rank_body(blk, hk, (int32_t*)it.out, (int32_t)it.n, (int32_t)it.k, it.seed, base, it.sub, a.epb);
}

// Any pool size (gpi_random_subset_ws): the same order -- the first k of the n indices by (Philox key,
// index) -- without all n keys in one workgroup's LDS.  The keys are uniform 32-bit values, so a
// histogram of their top 16 bits finds the bin b* where the count of smaller-or-equal keys first reaches
// k; every key whose top bits are <= b* is a candidate (about k + n / 65536 of them), every other key
// is larger than all candidates, so the first k pairs in the global order are the first k among the
// candidates, ranked as above.  Five small launches: zero, histogram, scan (b*), compact, rank.
constexpr int SUB_BINS = 1 << 16;

__global__ __launch_bounds__(256) void subset_zero_kernel(uint32_t* w, int32_t nwords) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < nwords) w[i] = 0u;
}

__global__ __launch_bounds__(256) void subset_hist_kernel(uint32_t* hist, int32_t n, uint64_t seed,
                                                          const uint64_t* offset, uint64_t sub) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint64_t base = offset ? *offset : 0;
    atomicAdd(&hist[philox(base + (uint64_t)j, sub, seed).x >> 16], 1u);
}

// one workgroup of 1024 threads, thread t owning bins [64 t, 64 t + 64): ctl[0] = b*, ctl[1] = 0
__global__ __launch_bounds__(1024) void subset_scan_kernel(const uint32_t* hist, uint32_t* ctl, int32_t k) {
    __shared__ uint32_t part[1024];
    const int t = threadIdx.x;
    uint32_t s = 0;
    for (int b = 0; b < 64; ++b) s += hist[64 * t + b];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {      // inclusive Hillis-Steele scan
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const uint32_t ex = part[t] - s;
    if (ex < (uint32_t)k && (uint32_t)k <= part[t]) {
        uint32_t c = ex;
        for (int b = 0; b < 64; ++b) {
            c += hist[64 * t + b];
            if (c >= (uint32_t)k) {
                ctl[0] = (uint32_t)(64 * t + b);
                break;
            }
        }
    }
    if (t == 0) ctl[1] = 0u;
}

__global__ __launch_bounds__(256) void subset_compact_kernel(uint2* cand, uint32_t* ctl, int32_t n, uint64_t seed,
                                                             const uint64_t* offset, uint64_t sub) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint64_t base = offset ? *offset : 0;
    const uint32_t key = philox(base + (uint64_t)j, sub, seed).x;
    if ((key >> 16) <= ctl[0]) {
        const uint32_t slot = atomicAdd(&ctl[1], 1u);
        cand[slot] = make_uint2(key, (uint32_t)j);
    }
}

// one wave per candidate (grid-stride over the waves): its rank among all C candidates.  O(C^2) compares
// (C ~ k + n / 65536): the path draws k of a few hundred to a few thousand (the reference's subset and
// batch sizes), where this is a handful of microseconds; a k of tens of thousands would want a
// segmented radix sort of the candidates instead.
__global__ __launch_bounds__(256) void subset_cand_rank_kernel(int32_t* out, const uint2* cand, const uint32_t* ctl,
                                                               int32_t k) {
    const int C = (int)ctl[1];
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * 4;
    for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < C; w += nw) {
        const uint2 me = cand[w];
        int cnt = 0;
        for (int j = lane; j < C; j += 64) {
            const uint2 o = cand[j];
            cnt += (o.x < me.x || (o.x == me.x && o.y < me.y)) ? 1 : 0;
        }
        for (int m = 32; m > 0; m >>= 1) cnt += __shfl_xor(cnt, m, 64);
        if (lane == 0 && cnt < k) out[cnt] = (int32_t)me.y;
    }
}

// Cross-stream hand-off by a device counter (gpi_stream_signal / gpi_stream_wait).  The signal kernel runs
// after every earlier kernel of its stream has completed and released its writes (the queue's kernel
// boundary), so one relaxed agent-scope increment publishes them (no load, fire and forget); the waiter
// spins on that word with sc1 loads until it reaches the step's count and exits, and the stream's next
// kernel starts with the usual acquire.  Every step signals each flag exactly once, so the count after
// step t's signal is t + 1 with t = the step counter, which changes only in the step's final epilogue,
// after every hand-off of the step.  Every spin is bounded: on a timeout the waiter sets *err and
// returns (the results are then garbage, the host reads the flag, nothing hangs).
constexpr int WAIT_SPIN_MAX = 1 << 24;

// every workgroup: one lane polls the flag (relaxed sc1 loads), then ONE agent acquire so that the
// workgroup's later plain loads see what the signalling stream wrote, then the workgroup barrier
__device__ __forceinline__ bool count_reached(const uint32_t* flag, uint32_t want) {
    return (int32_t)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) >= 0;
}

// returns true (every thread) when this wait timed out or an earlier one did (the sticky *err)
__device__ __forceinline__ bool epilogue_wait(const uint32_t* flag, const int64_t* epoch, uint32_t* err) {
    __shared__ uint32_t s_bad;
    if (threadIdx.x == 0) {
        const uint32_t want = (uint32_t)(*epoch + 1);
        uint32_t bad = 0u;
        for (int i = 0; !count_reached(flag, want); ++i) {
            __builtin_amdgcn_s_sleep(2);
            if (i > WAIT_SPIN_MAX) {
                if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bad = 1u;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (wait_failed(err)) bad = 1u;
        s_bad = bad;
    }
    __syncthreads();
    return s_bad != 0u;
}

__global__ void stream_signal_kernel(uint32_t* flag) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void stream_wait_kernel(const uint32_t* flag, const int64_t* epoch, uint32_t* err) {
    if (threadIdx.x != 0) return;
    const uint32_t want = (uint32_t)(*epoch + 1);
    for (int i = 0; !count_reached(flag, want); ++i) {
        __builtin_amdgcn_s_sleep(2);
        if (i > WAIT_SPIN_MAX) {
            if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

__global__ void stream_wait_ge_kernel(const int64_t* a, const int64_t* b, uint32_t* err) {
    if (threadIdx.x != 0) return;
    const int64_t want = __hip_atomic_load(b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want; ++i) {
        __builtin_amdgcn_s_sleep(2);
        if (i > WAIT_SPIN_MAX) {
            if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

// gpi_queue_probe: a short bounded spin for the flag's first increment; records whether it came
constexpr int PROBE_SPIN_MAX = 1 << 16;
__global__ void queue_probe_kernel(const uint32_t* flag, uint32_t* seen) {
    if (threadIdx.x != 0) return;
    uint32_t ok = 0;
    for (int i = 0; i < PROBE_SPIN_MAX; ++i) {
        if (count_reached(flag, 1u)) {
            ok = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_store(seen, ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" int gpi_queue_probe(const uint32_t* flag, uint32_t* seen, void* stream) {
    if (!flag || !seen) return GPI_ERR_ARG;
    hipLaunchKernelGGL(queue_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, seen);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_stream_wait_ge(const int64_t* a, const int64_t* b, uint32_t* err, void* stream) {
    if (!a || !b) return GPI_ERR_ARG;
    hipLaunchKernelGGL(stream_wait_ge_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, err);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_stream_signal(uint32_t* flag, const int64_t* epoch, void* stream) {
    if (!flag || !epoch) return GPI_ERR_ARG;
    hipLaunchKernelGGL(stream_signal_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flag);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_stream_wait(const uint32_t* flag, const int64_t* epoch, uint32_t* err, void* stream) {
    if (!flag || !epoch) return GPI_ERR_ARG;
    hipLaunchKernelGGL(stream_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, epoch, err);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_version(void) { return 1; }

extern "C" int gpi_replicas(void) { return GPI_REPLICAS; }

// ---------------------------------------------------------------- SyncBN seam exchange (gpi_bn_exchange)
// Lane t < 2 G n of one wave owns message element (group g, channel c, field f).  Cross-process words (the
// flags, the peers' buffers) are touched only by system-scope atomics: the stores write through to the owner's
// memory, the loads bypass this GPU's caches; the data stores are complete (vmcnt) before the flag's release.
__global__ __launch_bounds__(64) void bn_exchange_kernel(gpi_bn_exchange_desc d) {
    const int t = threadIdx.x;
    const int m = GPI_MAX_GROUPS * d.n * 2;
    const int g = t / (2 * d.n), c = (t >> 1) - g * d.n, f = t & 1;
    double* rec0 = (double*)d.stats + ((int64_t)g * d.n_stats + d.stat0 + c) * 4 + d.f0 + f;
    const int64_t rstride = (int64_t)GPI_MAX_GROUPS * d.n_stats * 4;   // doubles per replica
    double v = 0.0;
    if (d.mode != GPI_BNX_UNFOLD && t < m) {
        double r[GPI_REPLICAS];
#pragma unroll
        for (int k = 0; k < GPI_REPLICAS; ++k) r[k] = rec0[k * rstride];
#pragma unroll
        for (int k = 0; k < GPI_REPLICAS; ++k) v += r[k];              // replica order
    }
    if (d.mode == GPI_BNX_FOLD) {
        if (t < m) d.msg[t] = v;
        return;
    }
    if (d.mode == GPI_BNX_UNFOLD) {
        if (t < m) v = d.msg[t];
    } else {
        const uint32_t seq = *d.seq + 1u;
        const int slot = (int)(seq & 1u) * GPI_BNX_MSG;
        if (t < m)
            __hip_atomic_store(d.peer_buf[d.rank] + slot + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_waitcnt(0);                                  // this lane's message store is done
        __syncthreads();
        __shared__ uint32_t s_bad;
        if (t == 0) {
            // (no release fence: the message went out by write-through system-scope stores that are complete;
            // a fence would write back this XCD's whole L2)
            __hip_atomic_store(d.peer_flag[d.rank], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            uint32_t bad = 0u;
            for (int p = 0; p < d.world && !bad; ++p) {
                for (int i = 0; (int32_t)(__hip_atomic_load(d.peer_flag[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                                          seq) < 0; ++i) {
                    __builtin_amdgcn_s_sleep(2);
                    if (i > WAIT_SPIN_MAX) {
                        bad = 1u;
                        if (d.err) __hip_atomic_store(d.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            *d.seq = seq;       // (the peers' messages are read by system-scope loads below: no acquire fence)
            s_bad = bad;
        }
        __syncthreads();
        v = 0.0;
        if (t < m) {
            double r[GPI_MAX_RANKS];
            for (int p = 0; p < d.world; ++p)
                r[p] = __hip_atomic_load(d.peer_buf[p] + slot + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int p = 0; p < d.world; ++p) v += r[p];                // rank order
        }
        (void)s_bad;
    }
    if (t < m) {
        rec0[0] = v * d.scale[g];
#pragma unroll
        for (int k = 1; k < GPI_REPLICAS; ++k) rec0[k * rstride] = 0.0;
    }
}

extern "C" int gpi_struct_sizes(int64_t* out, int n) {
    const int64_t s[] = {(int64_t)sizeof(gpi_stat), (int64_t)sizeof(gpi_groups), (int64_t)sizeof(gpi_conv_desc),
                         (int64_t)sizeof(gpi_codec_ctx), (int64_t)sizeof(gpi_reduce_item), (int64_t)sizeof(gpi_head_desc),
                         (int64_t)sizeof(gpi_gemm_item), (int64_t)sizeof(gpi_rom_desc), (int64_t)sizeof(gpi_residual_desc),
                         (int64_t)sizeof(gpi_adam_desc), (int64_t)sizeof(gpi_vo_query_desc),
                         (int64_t)sizeof(gpi_vo_moments_desc), (int64_t)sizeof(gpi_vo_condition_desc),
                         (int64_t)sizeof(gpi_vo_precision_desc), (int64_t)sizeof(gpi_gp_sample_desc),
                         (int64_t)sizeof(gpi_vo_galerkin_desc), (int64_t)sizeof(gpi_step_epilogue_desc),
                         (int64_t)sizeof(gpi_fom_desc), (int64_t)sizeof(gpi_random_field_desc),
                         (int64_t)sizeof(gpi_vo_sparse), (int64_t)sizeof(gpi_draw_item),
                         (int64_t)sizeof(gpi_bn_exchange_desc)};
    const int k = (int)(sizeof(s) / sizeof(s[0]));
    if (!out || n < k) return GPI_ERR_ARG;
    for (int i = 0; i < k; ++i) out[i] = s[i];
    return k;
}

extern "C" const char* gpi_error_string(int code) {
    switch (code) {
        case GPI_OK: return "ok";
        case GPI_ERR_ARG: return "invalid argument";
        case GPI_ERR_LAUNCH: return "kernel launch failed";
        case GPI_ERR_UNSUPPORTED: return "unsupported configuration";
        default: return "unknown error";
    }
}

extern "C" int gpi_grad_finalize(double* gacc, float* grad, int64_t n, int flags, int64_t* step, void* stream) {
    if (!gacc || !grad || n < 0) return GPI_ERR_ARG;
    const int64_t nb = n > 0 ? (n + 255) / 256 : 1;
    hipLaunchKernelGGL(grad_finalize_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, gacc, grad, n,
                       flags, step);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_step_epilogue(const gpi_step_epilogue_desc* d, void* stream) {
    if (!d || d->n < 0 || d->n_scratch < 0 || d->n_idx < 0 || d->n_terms < 0 || d->n_terms > d->n_scratch) return GPI_ERR_ARG;
    if ((d->n && (!d->gacc || !d->grad)) || (d->n_scratch && !d->scratch) || (d->n_terms && !d->terms_dst) ||
        (d->n_idx && (!d->idx_src || !d->idx_dst)))
        return GPI_ERR_ARG;
    if (d->drop_n < 0 || (d->drop_n && (!d->drop_out || !(d->drop_p >= 0.f && d->drop_p < 1.f)))) return GPI_ERR_ARG;
    int64_t m = d->n > d->n_scratch ? d->n : d->n_scratch;
    if (d->n_idx > m) m = d->n_idx;
    if ((d->drop_n + 3) / 4 > m) m = (d->drop_n + 3) / 4;
    const int64_t nb = m > 0 ? (m + 255) / 256 : 1;
    hipLaunchKernelGGL(step_epilogue_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_step_epilogue_adam(const gpi_step_epilogue_desc* d, const gpi_adam_desc* a, uint32_t* done,
                                      void* stream) {
    if (!d || !a || !done || d->n < 0 || d->n_scratch < 0 || d->n_idx < 0 || d->n_terms < 0 || d->n_terms > d->n_scratch)
        return GPI_ERR_ARG;
    if (!d->gacc || !d->grad || (d->n_scratch && !d->scratch) || (d->n_terms && !d->terms_dst) ||
        (d->n_idx && (!d->idx_src || !d->idx_dst)))
        return GPI_ERR_ARG;
    if (d->drop_n < 0 || (d->drop_n && (!d->drop_out || !(d->drop_p >= 0.f && d->drop_p < 1.f)))) return GPI_ERR_ARG;
    // the fused form owns the counter (Adam's) and always zeroes the accumulator; the update covers
    // exactly the gradient's elements
    if (d->flags != GPI_FINALIZE_ZERO || d->step || !a->p || !a->g || !a->m || !a->v || !a->lr || !a->step ||
        a->n != d->n || a->g != d->grad || (d->drop_n && d->drop_offset && a->rng_offset &&
                                              d->drop_offset != a->rng_offset))
        return GPI_ERR_ARG;
    int64_t m = d->n > d->n_scratch ? d->n : d->n_scratch;
    if (d->n_idx > m) m = d->n_idx;
    if ((d->drop_n + 3) / 4 > m) m = (d->drop_n + 3) / 4;
    int64_t nb = m > 0 ? (m + 255) / 256 : 1;
    if (nb > GPI_EPILOGUE_MAX_WG) nb = GPI_EPILOGUE_MAX_WG;
    hipLaunchKernelGGL(step_epilogue_adam_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, *d, *a, done,
                       m);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_adam(const gpi_adam_desc* d, void* stream) {
    if (!d || !d->p || !d->g || !d->m || !d->v || !d->lr || !d->step || d->n < 0) return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    int64_t nb = (d->n + 255) / 256;
    if (nb > 2048) nb = 2048;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_randn(float* out, int64_t n, uint64_t seed, const uint64_t* offset, uint64_t sub, void* stream) {
    if (!out || n < 0) return GPI_ERR_ARG;
    if (n == 0) return GPI_OK;
    const int64_t nq = (n + 3) / 4;
    hipLaunchKernelGGL(randn_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, n,
                       seed, offset, sub);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_dropout_masks(float* out, int64_t n, float p, uint64_t seed, const uint64_t* offset, uint64_t sub,
                                 void* stream) {
    if (!out || n < 0 || !(p >= 0.f && p < 1.f)) return GPI_ERR_ARG;
    if (n == 0) return GPI_OK;
    const int64_t nq = (n + 3) / 4;
    hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out,
                       n, p, 1.f / (1.f - p), seed, offset, sub);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_rng_advance(uint64_t* offset, uint64_t by, void* stream) {
    if (!offset) return GPI_ERR_ARG;
    hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, offset, by);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_random_subset_workspace(int32_t n, int64_t* bytes) {
    if (n <= 0 || !bytes) return GPI_ERR_ARG;
    *bytes = (int64_t)sizeof(uint32_t) * (SUB_BINS + 64) + (int64_t)sizeof(uint2) * n;
    return GPI_OK;
}

extern "C" int gpi_random_subset(int32_t* out, int32_t n, int32_t k, uint64_t seed, const uint64_t* offset,
                                 uint64_t sub, void* stream);

extern "C" int gpi_random_subset_ws(int32_t* out, int32_t n, int32_t k, uint64_t seed, const uint64_t* offset,
                                    uint64_t sub, void* workspace, int64_t ws_bytes, void* stream) {
    if (!out || n <= 0 || k < 0 || k > n) return GPI_ERR_ARG;
    if (k == 0) return GPI_OK;
    if (n <= 16384) return gpi_random_subset(out, n, k, seed, offset, sub, stream);
    int64_t need = 0;
    gpi_random_subset_workspace(n, &need);
    if (!workspace || ws_bytes < need || ((uintptr_t)workspace & 15)) return GPI_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    uint32_t* hist = (uint32_t*)workspace;
    uint32_t* ctl = hist + SUB_BINS;
    uint2* cand = (uint2*)(ctl + 64);
    const unsigned gn = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(subset_zero_kernel, dim3((SUB_BINS + 64 + 255) / 256), dim3(256), 0, st, hist, SUB_BINS + 64);
    hipLaunchKernelGGL(subset_hist_kernel, dim3(gn), dim3(256), 0, st, hist, n, seed, offset, sub);
    hipLaunchKernelGGL(subset_scan_kernel, dim3(1), dim3(1024), 0, st, hist, ctl, k);
    hipLaunchKernelGGL(subset_compact_kernel, dim3(gn), dim3(256), 0, st, cand, ctl, n, seed, offset, sub);
    hipLaunchKernelGGL(subset_cand_rank_kernel, dim3(512), dim3(256), 0, st, out, cand, ctl, k);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_random_subset(int32_t* out, int32_t n, int32_t k, uint64_t seed, const uint64_t* offset,
                                 uint64_t sub, void* stream) {
    if (!out || n <= 0 || k < 0 || k > n || n > 16384) return GPI_ERR_ARG;
    if (k == 0) return GPI_OK;
    const int32_t epb = subset_epb(n);
    const size_t lds = sizeof(uint32_t) * n;
    if (lds > 64 * 1024) return GPI_ERR_ARG;
    hipLaunchKernelGGL(subset_rank_kernel, dim3((unsigned)((n + epb - 1) / epb)), dim3(256), lds, (hipStream_t)stream,
                       out, n, k, seed, offset, sub, epb);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_draws(const gpi_draw_item* items, int n_items, const uint64_t* offset, void* stream) {
    if (!items || n_items < 0 || n_items > GPI_MAX_DRAWS) return GPI_ERR_ARG;
    DrawArgs a;
    a.n = n_items;
    a.epb = 4;
    size_t lds = 0;
    int nb = 0, n_sub = 0;
    for (int k = 0; k < n_items; ++k) {
        const gpi_draw_item& it = items[k];
        a.it[k] = it;
        a.first_block[k] = nb;
        if (!it.out || it.n < 0) return GPI_ERR_ARG;
        if (it.kind == GPI_DRAW_RANDN) {
            nb += (int)((((it.n + 3) / 4) + 255) / 256);
        } else if (it.kind == GPI_DRAW_DROPOUT) {
            if (!(it.p >= 0.f && it.p < 1.f)) return GPI_ERR_ARG;
            nb += (int)((((it.n + 3) / 4) + 255) / 256);
        } else if (it.kind == GPI_DRAW_SUBSET) {
            if (it.n <= 0 || it.n > 16384 || it.k < 0 || it.k > it.n || ++n_sub > 1) return GPI_ERR_ARG;
            a.epb = subset_epb((int32_t)it.n);
            lds = sizeof(uint32_t) * (size_t)it.n;
            if (it.k > 0) nb += (int)((it.n + a.epb - 1) / a.epb);
        } else {
            return GPI_ERR_ARG;
        }
    }
    for (int k = n_items; k <= GPI_MAX_DRAWS; ++k) a.first_block[k] = nb;
    if (nb == 0) return GPI_OK;
    hipLaunchKernelGGL(draws_kernel, dim3((unsigned)nb), dim3(256), lds, (hipStream_t)stream, a, offset);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_bn_exchange(const gpi_bn_exchange_desc* d, void* stream) {
    if (!d || !d->stats || d->n < 1 || d->n > GPI_MAX_COUT || d->stat0 < 0 || d->stat0 + d->n > d->n_stats ||
        (d->f0 != 0 && d->f0 != 2) || d->mode < GPI_BNX_FOLD || d->mode > GPI_BNX_PEER)
        return GPI_ERR_ARG;
    if (d->mode != GPI_BNX_PEER && !d->msg) return GPI_ERR_ARG;
    if (d->mode != GPI_BNX_FOLD && !d->scale) return GPI_ERR_ARG;
    if (d->mode == GPI_BNX_PEER) {
        if (d->world < 1 || d->world > GPI_MAX_RANKS || d->rank < 0 || d->rank >= d->world || !d->seq) return GPI_ERR_ARG;
        for (int p = 0; p < d->world; ++p)
            if (!d->peer_buf[p] || !d->peer_flag[p]) return GPI_ERR_ARG;
    }
    hipLaunchKernelGGL(bn_exchange_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_peer_alloc(int64_t bytes, void** ptr, void* ipc_handle) {
    if (bytes <= 0 || !ptr || !ipc_handle) return GPI_ERR_ARG;
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
    if (hipMalloc(ptr, (size_t)bytes) != hipSuccess) return GPI_ERR_LAUNCH;
    if (hipMemset(*ptr, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipIpcGetMemHandle((hipIpcMemHandle_t*)ipc_handle, *ptr) != hipSuccess) {
        (void)hipFree(*ptr);
        *ptr = nullptr;
        return GPI_ERR_LAUNCH;
    }
    return GPI_OK;
}

extern "C" int gpi_peer_open(const void* ipc_handle, void** ptr) {
    if (!ipc_handle || !ptr) return GPI_ERR_ARG;
    hipIpcMemHandle_t h;
    memcpy(&h, ipc_handle, sizeof(h));
    if (hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return GPI_ERR_LAUNCH;
    return GPI_OK;
}

extern "C" int gpi_peer_close(void* ptr, int own) {
    if (!ptr) return GPI_ERR_ARG;
    return (own ? hipFree(ptr) : hipIpcCloseMemHandle(ptr)) == hipSuccess ? GPI_OK : GPI_ERR_LAUNCH;
}
