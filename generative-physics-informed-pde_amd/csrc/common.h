// Shared device helpers for libgpi_hip.so (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "gpi.h"

#define GPI_LOG2PI 1.8378770664093453f

#define GPI_CHECK_LAUNCH()                                   \
    do {                                                     \
        if (hipGetLastError() != hipSuccess) return GPI_ERR_LAUNCH; \
    } while (0)

namespace gpi {

// DPP step: v + (v moved by ctrl within the rows of row_mask; other rows add 0)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xf, false);
    return v + __int_as_float(t);
}

// Wave64 sum by the DPP ladder (no LDS traffic): quad pairs, quads, rows of 8 and 16
// by row rotation, then row_bcast15 / row_bcast31 fold rows 0..3 into lane 63,
// whose value is returned to every lane.
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_add<0xb1, 0xf>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4e, 0xf>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x124, 0xf>(v);   // row_ror:4
    v = dpp_add<0x128, 0xf>(v);   // row_ror:8
    v = dpp_add<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
    v = dpp_add<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of NV per-thread values into red[0..NV) (caller syncs after).
// scratch: >= NV * (blockDim/64) floats.
// The NV wave sums run step-major (every value through one DPP step before the next step): NV
// independent DPP ops per step keep the VALU busy instead of one dependent ladder per value with
// the DPP wait states in between (value-major took ~1500 cycles for 16 values).
template <int CTRL, int ROW_MASK, int NV>
__device__ __forceinline__ void dpp_step(float (&v)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = dpp_add<CTRL, ROW_MASK>(v[i]);
}

// v[i] <- wave sum of v[i] (uniform), for NV values at once (step-major).
template <int NV>
__device__ __forceinline__ void wave_sums(float (&v)[NV]) {
    dpp_step<0xb1, 0xf>(v);    // quad_perm [1,0,3,2]
    dpp_step<0x4e, 0xf>(v);    // quad_perm [2,3,0,1]
    dpp_step<0x124, 0xf>(v);   // row_ror:4
    dpp_step<0x128, 0xf>(v);   // row_ror:8
    dpp_step<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
    dpp_step<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[i]), 63));
}

template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* scratch, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    wave_sums(v);
#pragma unroll
    for (int i = 0; i < NV; ++i)
        if (lane == 0) scratch[i * nw + wid] = v[i];
    __syncthreads();
    if ((int)threadIdx.x < NV) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += scratch[threadIdx.x * nw + w];
        red[threadIdx.x] = s;
    }
}

__device__ __forceinline__ int floordiv2(int x) { return x >> 1; }   // arithmetic shift = floor
__device__ __forceinline__ int ceildiv2(int x) { return -((-x) >> 1); }

// Group of sample s.  Branch-free over all GPI_MAX_GROUPS starts: every start is read up front, so the
// kernel-argument loads join the entry batch (a data-dependent loop over the by-value argument array
// costs one dependent scalar-load round trip per iteration).
__device__ __forceinline__ int group_of(const gpi_groups& g, int s) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < GPI_MAX_GROUPS; ++j) k += (j < g.n_groups && s >= g.start[j]) ? 1 : 0;
    return k;
}

// arr[i] of a by-value kernel-argument array with a runtime index, as a select over all entries
// (an indexed access would be a dependent scalar load after i is known)
template <typename T, int N>
__device__ __forceinline__ T karg_sel(const T (&arr)[N], int i) {
    T v = arr[0];
#pragma unroll
    for (int j = 1; j < N; ++j) v = (i == j) ? arr[j] : v;
    return v;
}

// train-mode BN coefficients from fp64 sums (biased variance, torch semantics)
__device__ __forceinline__ void bn_mean_invstd(const gpi_stat& st, double n, float eps, float& mean,
                                               float& invstd) {
    double m = st.sum / n;
    double var = st.sumsq / n - m * m;
    if (var < 0.0) var = 0.0;
    mean = (float)m;
    invstd = (float)(1.0 / sqrt(var + (double)eps));
}

// ---------------------------------------------------------------- Philox4x32-10
struct uint4_ { uint32_t x, y, z, w; };

__device__ __forceinline__ uint4_ philox(uint64_t ctr_lo, uint64_t ctr_hi, uint64_t key) {
    uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
    uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

__device__ __forceinline__ float u01(uint32_t x) {   // (0, 1]
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

}  // namespace gpi
