// Dense (per-sample) part of the ELBO and its backward.
//
// One workgroup per sample runs the whole per-sample chain in LDS:
//   encoder FC -> ReLU -> (mu, logsigma) heads      (Encoder.py:175-182, codec.py:495-504)
//   z = mu + exp(logsigma) eps, KL                  (bottleneck/utils.py:216-219,246-248)
//   or z from q_z, KL                               (components.py:167-172,192-193)
//   decoder latent map                              (Decoder.py:213,293)
//   gp(z), X~ = q_X sample, log-lik, entropy        (generative.py:464-478, components.py:195-197,224-229)
//   or X~ = gp(z) (lockX)                           (generative.py:429-459,300-339)
// The backward writes per-sample deltas; the shared-weight gradients
// (sum over samples of delta (x) input) are formed by gpi_outer_gemm, the
// per-sample variational parameters' gradients are written directly.
#include "common.h"
#include <stdlib.h>

using namespace gpi;

namespace {

#ifndef GPI_HEAD_HT
#define GPI_HEAD_HT 128
#endif
constexpr int HT = GPI_HEAD_HT;   // threads per sample
constexpr int VMAX = 512;   // max vector length

__device__ __forceinline__ float block_sum128(float v, float* scratch) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float t = scratch[0];
#pragma unroll
    for (int w = 1; w < HT / 64; ++w) t += scratch[w];
    return t;
}

// The weight reads are the latency chain of these kernels (one sample per workgroup, weights from
// L2): every dependent round trip costs ~0.5 us, so each thread issues a whole batch of weight loads
// before its FMAs, batches are as wide as the registers allow (64 rows / columns), two matrices
// that read the same input share one pass (mu and logsigma heads), and a transposed product
// whose column count leaves threads idle splits its rows over thread groups.  A kernel that
// prefetches every weight at entry was measured 2x slower (r03: fully unrolled, run-once code).

// y0[j] = b0[j] + W0[j,:] . x for j < J0, then y1[j] = b1[j] + W1[j,:] . x for j < J1 (thread per row)
__device__ __forceinline__ void matvec2(const float* __restrict__ W0, const float* __restrict__ b0, float* y0,
                                        int J0, const float* __restrict__ W1, const float* __restrict__ b1,
                                        float* y1, int J1, const float* x, int K) {
    const bool vec = (K & 3) == 0 && ((reinterpret_cast<uintptr_t>(W0) | reinterpret_cast<uintptr_t>(W1)) & 15) == 0;
    for (int j = threadIdx.x; j < J0 + J1; j += HT) {
        const bool first = j < J0;
        const int jr = first ? j : j - J0;
        const float* bias = first ? b0 : b1;
        const float* w = (first ? W0 : W1) + (int64_t)jr * K;
        float a[4] = {bias ? bias[jr] : 0.f, 0.f, 0.f, 0.f};
        int k = 0;
        if (vec) {
            const float4* w4 = reinterpret_cast<const float4*>(w);
            for (; k + 64 <= K; k += 64) {
                float4 wv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) wv[u] = w4[(k >> 2) + u];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    a[0] = fmaf(wv[u].x, x[k + 4 * u], a[0]);
                    a[1] = fmaf(wv[u].y, x[k + 4 * u + 1], a[1]);
                    a[2] = fmaf(wv[u].z, x[k + 4 * u + 2], a[2]);
                    a[3] = fmaf(wv[u].w, x[k + 4 * u + 3], a[3]);
                }
            }
            for (; k + 16 <= K; k += 16) {
                float4 wv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) wv[u] = w4[(k >> 2) + u];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a[0] = fmaf(wv[u].x, x[k + 4 * u], a[0]);
                    a[1] = fmaf(wv[u].y, x[k + 4 * u + 1], a[1]);
                    a[2] = fmaf(wv[u].z, x[k + 4 * u + 2], a[2]);
                    a[3] = fmaf(wv[u].w, x[k + 4 * u + 3], a[3]);
                }
            }
        }
        for (; k + 16 <= K; k += 16) {
            float wv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) wv[u] = w[k + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u & 3] = fmaf(wv[u], x[k + u], a[u & 3]);
        }
        for (; k < K; ++k) a[k & 3] = fmaf(w[k], x[k], a[k & 3]);
        (first ? y0 : y1)[jr] = (a[0] + a[1]) + (a[2] + a[3]);
    }
}

__device__ __forceinline__ void matvec(const float* __restrict__ W, const float* __restrict__ b, const float* x,
                                       int J, int K, float* y) {
    matvec2(W, b, y, J, W, b, y, 0, x, K);
}

// rows j0 <= j < j1 of W^T d into a[] (column k), batches of 32 loads in flight
__device__ __forceinline__ void mt_rows(const float* __restrict__ W, const float* d, int K, int k, int j0, int j1,
                                        float (&a)[4]) {
    const float* w = W + (int64_t)j0 * K + k;
    int j = j0;
    for (; j + 32 <= j1; j += 32, w += (int64_t)32 * K) {
        float wv[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) wv[u] = w[(int64_t)u * K];
#pragma unroll
        for (int u = 0; u < 32; ++u) a[u & 3] = fmaf(wv[u], d[j + u], a[u & 3]);
    }
    for (; j + 8 <= j1; j += 8, w += (int64_t)8 * K) {
        float wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) wv[u] = w[(int64_t)u * K];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u & 3] = fmaf(wv[u], d[j + u], a[u & 3]);
    }
    for (; j < j1; ++j, w += K) a[j & 3] = fmaf(*w, d[j], a[j & 3]);
}

// y[k] (+)= sum_j W0[j,k] d0[j] + sum_j W1[j,k] d1[j] (thread per column).  With K <= HT/2 the rows
// are split over P = min(4, HT/K) thread groups whose partial sums meet in `part` (>= HT floats);
// the call then holds a __syncthreads, so every thread of the workgroup must make it.
__device__ __forceinline__ void matvec_t2(const float* __restrict__ W0, const float* d0, int J0,
                                          const float* __restrict__ W1, const float* d1, int J1, int K, float* y,
                                          bool accumulate, float* part) {
    const int J = J0 + J1;
    const int P = K <= HT / 2 ? min(4, HT / K) : 1;
    if (P == 1) {
        for (int k = threadIdx.x; k < K; k += HT) {
            float a[4] = {accumulate ? y[k] : 0.f, 0.f, 0.f, 0.f};
            mt_rows(W0, d0, K, k, 0, J0, a);
            mt_rows(W1, d1, K, k, 0, J1, a);
            y[k] = (a[0] + a[1]) + (a[2] + a[3]);
        }
        return;
    }
    const int Jp = (((J + P - 1) / P) + 7) & ~7;       // rows per group, batch-aligned
    const int p = threadIdx.x / K, k = threadIdx.x - p * K;
    if (p < P) {
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        const int j0 = p * Jp, j1 = min(J, j0 + Jp);
        mt_rows(W0, d0, K, k, min(j0, J0), min(j1, J0), a);
        mt_rows(W1, d1, K, k, max(j0, J0) - J0, max(j1, J0) - J0, a);
        part[threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
    }
    __syncthreads();
    if (threadIdx.x < K) {
        float t = accumulate ? y[threadIdx.x] : 0.f;
        for (int q = 0; q < P; ++q) t += part[q * K + threadIdx.x];
        y[threadIdx.x] = t;
    }
}

// The variational segment of workspace row q (>= 0): its parameter rows, flags, scales, term slots.
struct QSeg {
    int row, flags;
    int64_t qz_mu, qz_ls, qx_mu, qx_ls;
    float kl_scale, lx_scale;
    double* terms;   // [KL_q, logL_X, entropy][GPI_REPLICAS]
};

__device__ __forceinline__ QSeg qseg(const gpi_head_desc& d, int q) {
    QSeg g;
    if (q >= d.n_q) {
        g.row = q - d.n_q;
        g.flags = d.flags2;
        g.qz_mu = d.qz_mu2; g.qz_ls = d.qz_ls2; g.qx_mu = d.qx_mu2; g.qx_ls = d.qx_ls2;
        g.kl_scale = d.kl_scale_q2; g.lx_scale = d.lx_scale2;
        g.terms = d.terms2;
    } else {
        g.row = q;
        g.flags = d.flags;
        g.qz_mu = d.qz_mu; g.qz_ls = d.qz_ls; g.qx_mu = d.qx_mu; g.qx_ls = d.qx_ls;
        g.kl_scale = d.kl_scale_q; g.lx_scale = d.lx_scale;
        g.terms = d.terms + GPI_REPLICAS;
    }
    return g;
}

__global__ __launch_bounds__(HT) void head_fwd_kernel(gpi_head_desc d, const float* __restrict__ P, float* ws) {
    __shared__ float v0[VMAX], v1[VMAX], v2[VMAX], v3[VMAX];
    __shared__ float scratch[4];
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const bool enc = s < d.n_enc;
    const int q = s - d.n_enc;                  // workspace row over both variational segments
    const QSeg g = qseg(d, q);
    const int dz = d.d_z;
    float* z = v2;

    if (enc) {
        if (d.flags & GPI_HEAD_ENC) {
            const float* f = ws + d.feat + (int64_t)s * d.d_feat;
            for (int k = tid; k < d.d_feat; k += HT) v0[k] = f[k];
            __syncthreads();
            matvec(P + d.fc_w, P + d.fc_b, v0, d.d_feat, d.d_feat, v1);
            __syncthreads();
            for (int k = tid; k < d.d_feat; k += HT) {
                ws[d.hpre + (int64_t)s * d.d_feat + k] = v1[k];
                v1[k] = fmaxf(v1[k], 0.f);
            }
            __syncthreads();
            matvec2(P + d.mu_w, P + d.mu_b, v0, dz, P + d.ls_w, P + d.ls_b, v3, dz, v1, d.d_feat);   // mu, logsigma
            __syncthreads();
            for (int k = tid; k < dz; k += HT) {
                ws[d.zmu + (int64_t)s * dz + k] = v0[k];
                ws[d.zls + (int64_t)s * dz + k] = v3[k];
            }
        } else {
            for (int k = tid; k < dz; k += HT) {
                v0[k] = ws[d.zmu + (int64_t)s * dz + k];
                v3[k] = ws[d.zls + (int64_t)s * dz + k];
            }
        }
        __syncthreads();
        if (d.flags & GPI_HEAD_REPARAM) {
            float kl = 0.f;
            for (int k = tid; k < dz; k += HT) {
                const float mu = v0[k], ls = v3[k];
                const float e = expf(ls);
                const float zz = fmaf(e, ws[d.eps_z + (int64_t)s * dz + k], mu);
                z[k] = zz;
                ws[d.z + (int64_t)s * dz + k] = zz;
                kl += 1.f + 2.f * ls - mu * mu - e * e;
            }
            kl = block_sum128(kl, scratch);
            if (tid == 0) atomicAdd(d.terms + 0 * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, -0.5 * (double)kl);
        } else {
            for (int k = tid; k < dz; k += HT) z[k] = ws[d.z + (int64_t)s * dz + k];
        }
    } else {
        if (g.flags & GPI_HEAD_QZ) {
            float kl = 0.f;
            for (int k = tid; k < dz; k += HT) {
                const float mu = P[g.qz_mu + (int64_t)g.row * dz + k], ls = P[g.qz_ls + (int64_t)g.row * dz + k];
                const float e = expf(ls);
                const float zz = fmaf(e, ws[d.eps_z + (int64_t)s * dz + k], mu);
                z[k] = zz;
                ws[d.z + (int64_t)s * dz + k] = zz;
                kl += 1.f + 2.f * ls - mu * mu - e * e;
            }
            kl = block_sum128(kl, scratch);
            if (tid == 0) atomicAdd(g.terms + 0 * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, -0.5 * (double)kl);
        } else {
            for (int k = tid; k < dz; k += HT) z[k] = ws[d.z + (int64_t)s * dz + k];
        }
    }
    __syncthreads();
    if (d.flags & GPI_HEAD_LATENT) {
        float* lat = ws + d.lat + (int64_t)s * d.d_lat;
        matvec(P + d.lat_w, P + d.lat_b, z, d.d_lat, dz, v1);
        __syncthreads();
        for (int j = tid; j < d.d_lat; j += HT) lat[j] = v1[j];
    }
    if (!enc && (g.flags & GPI_HEAD_GP)) {
        const bool lockx = g.flags & GPI_HEAD_LOCKX;             // uniform per workgroup
        float lx = 0.f, ent = 0.f;
        __syncthreads();
        matvec(P + d.gp_w, P + d.gp_b, z, d.d_x, dz, v3);           // gp(z)
        __syncthreads();
        for (int t = tid; t < d.d_x; t += HT) {
            const float a = v3[t];
            const int64_t qi = (int64_t)q * d.d_x + t;              // workspace row
            if (lockx) {                                           // X~ = gp(z) (generative.py:432)
                ws[d.mux + qi] = a;
                ws[d.xs + qi] = a;
                continue;
            }
            const int64_t pi = (int64_t)g.row * d.d_x + t;          // q_X parameter row
            const float lsq = P[g.qx_ls + pi];
            const float xs = fmaf(expf(lsq), ws[d.eps_x + qi], P[g.qx_mu + pi]);
            ws[d.mux + qi] = a;
            ws[d.xs + qi] = xs;
            const float gls = P[d.gp_ls + t];
            const float r = xs - a;
            lx += -0.5f * (2.f * gls + r * r * expf(-2.f * gls) + GPI_LOG2PI);
            ent += lsq;
        }
        if (lockx) return;
        lx = block_sum128(lx, scratch);
        ent = block_sum128(ent, scratch);
        if (tid == 0) {
            atomicAdd(g.terms + 1 * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, (double)lx);
            atomicAdd(g.terms + 2 * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, (double)ent);
        }
    }
}

__global__ __launch_bounds__(HT) void head_bwd_kernel(gpi_head_desc d, const float* __restrict__ P, float* ws,
                                                      double* gacc, int s_off) {
    __shared__ float v0[VMAX], v1[VMAX], v2[VMAX], v3[VMAX];
    __shared__ float part[HT];
    const int s = blockIdx.x + s_off;
    const int tid = threadIdx.x;
    const bool enc = s < d.n_enc;
    const int q = s - d.n_enc;
    const QSeg g = qseg(d, q);
    const int dz = d.d_z;
    float* dz_ = v0;   // dJ/dz

    // latent map: dz = lat_w^T glat
    if (d.flags & GPI_HEAD_LATENT) {
        const float* gl = ws + d.glat + (int64_t)s * d.d_lat;
        for (int j = tid; j < d.d_lat; j += HT) v1[j] = gl[j];
        __syncthreads();
        matvec_t2(P + d.lat_w, v1, d.d_lat, P, v1, 0, dz, dz_, false, part);
    } else {
        for (int k = tid; k < dz; k += HT) dz_[k] = ws[d.gz + (int64_t)s * dz + k];
    }
    __syncthreads();

    if (!enc && (g.flags & GPI_HEAD_GP)) {
        const bool lockx = g.flags & GPI_HEAD_LOCKX;
        for (int t = tid; t < d.d_x; t += HT) {
            const int64_t qi = (int64_t)q * d.d_x + t;
            if (lockx) {                                    // dJ/dmu_X = dJ/dX~ (the ROM adjoint)
                const float gm = ws[d.gxs + qi];
                v2[t] = gm;
                ws[d.gmux + qi] = gm;
                continue;
            }
            const int64_t pi = (int64_t)g.row * d.d_x + t;
            const float gls = P[d.gp_ls + t];
            const float e2 = expf(-2.f * gls);
            const float xs = ws[d.xs + qi], mux = ws[d.mux + qi];
            const float r = xs - mux;
            const float gm = -g.lx_scale * r * e2;            // dJ/dmu_X
            v2[t] = gm;
            ws[d.gmux + qi] = gm;
            atomicAdd(gacc + d.gp_ls + t, (double)(g.lx_scale * (1.f - r * r * e2)));
            const float dxs = ws[d.gxs + qi] + g.lx_scale * r * e2;   // dJ/dX~
            const float lsq = P[g.qx_ls + pi];
            gacc[g.qx_mu + pi] += (double)dxs;
            gacc[g.qx_ls + pi] += (double)(dxs * expf(lsq) * ws[d.eps_x + qi] - g.lx_scale);
        }
        __syncthreads();
        matvec_t2(P + d.gp_w, v2, d.d_x, P, v2, 0, dz, dz_, true, part);
        __syncthreads();
    }

    if (!enc) {
        if (g.flags & GPI_HEAD_QZ) {
            for (int k = tid; k < dz; k += HT) {
                const int64_t qi = (int64_t)g.row * dz + k;
                const float mu = P[g.qz_mu + qi], ls = P[g.qz_ls + qi];
                const float e = expf(ls);
                gacc[g.qz_mu + qi] += (double)(dz_[k] + g.kl_scale * mu);
                gacc[g.qz_ls + qi] += (double)(dz_[k] * e * ws[d.eps_z + (int64_t)s * dz + k] +
                                               g.kl_scale * (e * e - 1.f));
            }
        }
        return;
    }

    // encoder samples: reparametrisation + KL
    for (int k = tid; k < dz; k += HT) {
        float dmu = dz_[k], dls = 0.f;
        const float mu = ws[d.zmu + (int64_t)s * dz + k], ls = ws[d.zls + (int64_t)s * dz + k];
        if (d.flags & GPI_HEAD_REPARAM) {
            const float e = expf(ls);
            dls = dz_[k] * e * ws[d.eps_z + (int64_t)s * dz + k] + d.kl_scale_enc * (e * e - 1.f);
            dmu += d.kl_scale_enc * mu;
        } else {
            dls = ws[d.dzls + (int64_t)s * dz + k];   // caller-provided d/dlogsigma
        }
        v1[k] = dmu;
        v2[k] = dls;
        ws[d.dzmu + (int64_t)s * dz + k] = dmu;
        ws[d.dzls + (int64_t)s * dz + k] = dls;
    }
    __syncthreads();
    if (!(d.flags & GPI_HEAD_ENC)) return;
    // heads: dh = mu_w^T dmu + ls_w^T dls ; ReLU ; FC
    matvec_t2(P + d.mu_w, v1, dz, P + d.ls_w, v2, dz, d.d_feat, v3, false, part);
    __syncthreads();
    for (int k = tid; k < d.d_feat; k += HT) {
        const float hp = ws[d.hpre + (int64_t)s * d.d_feat + k];
        const float g = hp > 0.f ? v3[k] : 0.f;
        v3[k] = g;
        ws[d.dhpre + (int64_t)s * d.d_feat + k] = g;
    }
    __syncthreads();
    matvec_t2(P + d.fc_w, v3, d.d_feat, P, v3, 0, d.d_feat, v0, false, part);
    __syncthreads();
    for (int k = tid; k < d.d_feat; k += HT) ws[d.gfeat + (int64_t)s * d.d_feat + k] = v0[k];
}

struct GemmArgs {
    gpi_gemm_item it[GPI_MAX_GEMM_ITEMS];
    int32_t first_block[GPI_MAX_GEMM_ITEMS + 1];
    int32_t tiles_n[GPI_MAX_GEMM_ITEMS];
    int32_t n;
};

// C (M x (N+1)) tile 16 x 16 per workgroup; column N is the bias (B = 1).
// item.flags bit 0: apply ReLU to B (h = relu(hpre)).
__global__ __launch_bounds__(256) void outer_gemm_kernel(GemmArgs a, const float* __restrict__ ws, double* gacc) {
    __shared__ float As[32][17], Bs[32][17];
    int k = 0;
    while (k + 1 < a.n && (int)blockIdx.x >= a.first_block[k + 1]) ++k;
    const gpi_gemm_item it = a.it[k];
    const int local = blockIdx.x - a.first_block[k];
    const int tm = local / a.tiles_n[k], tn = local - tm * a.tiles_n[k];
    const int m0 = tm * 16, n0 = tn * 16;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const bool relu_b = it.flags & 1;
    float acc = 0.f;
    for (int sb = 0; sb < it.S; sb += 32) {
        for (int e = threadIdx.x; e < 32 * 16; e += 256) {
            const int r = e >> 4, cc = e & 15;
            const int s = sb + r;
            float av = 0.f, bv = 0.f;
            if (s < it.S) {
                if (m0 + cc < it.M) av = ws[it.a_off + (int64_t)s * it.lda + m0 + cc];
                const int n = n0 + cc;
                if (n < it.N) {
                    bv = ws[it.b_off + (int64_t)s * it.ldb + n];
                    if (relu_b) bv = fmaxf(bv, 0.f);
                } else if (n == it.N) {
                    bv = 1.f;
                }
            }
            As[r][cc] = av;
            Bs[r][cc] = bv;
        }
        __syncthreads();
#pragma unroll 8
        for (int r = 0; r < 32; ++r) acc = fmaf(As[r][ty], Bs[r][tx], acc);
        __syncthreads();
    }
    const int m = m0 + ty, n = n0 + tx;
    if (m < it.M) {
        if (n < it.N) gacc[it.c_off + (int64_t)m * it.N + n] += (double)acc;
        else if (n == it.N && it.bias_off >= 0) gacc[it.bias_off + m] += (double)acc;
    }
}

// ---------------------------------------------------------------------------------- MFMA form
// The dense layers as batched products on the matrix cores (v_mfma_f32_16x16x4_f32: exact f32, a
// k-ordered fmaf chain per output).  One workgroup per tile of TS = 16 samples (encoder samples and
// variational samples in separate tiles), four waves.  A contraction Y[s][j] = sum_k A(j, k) X[s][k]
// runs as 16 x 16 blocks -- rows j = output features, columns = the tile's samples, reduction over the
// input features -- in which lane (i = lane & 15, g = lane >> 4) supplies A(16 jb + i, k) and X[i][k]
// for k = 16 c + 4 g + t (t = 0..3: one aligned float4 of each per 16-wide chunk c) and receives
// Y[i][16 jb + 4 g + r], r = 0..3 (four consecutive outputs of one sample: one float4 store).  X is
// the previous stage's output in LDS, one row per sample, zero outside the valid rows / columns; each
// wave issues all weight loads of its blocks (straight from L2: every tile reads the same matrices)
// before its first MFMA.  The shared-weight gradients (sum over samples of delta (x) input) are the
// same product with the samples as the reduction index (outer_gemm_mfma).

typedef float hf32x4 __attribute__((ext_vector_type(4)));
constexpr int TS = 16;                 // samples per tile
constexpr int MW = 256;                // max output width / contraction length of a wide row buffer
constexpr int LPW = MW + 4;            // LDS pitch (floats) of a wide row buffer
constexpr int MZ = 128;                // max d_z
constexpr int LPZ = MZ + 4;
constexpr int KC = 4;                  // 16-wide k chunks of weight operands in flight per block
// (the kernels stay at <= 128 VGPRs, 4 waves per SIMD: they share the CUs with the step's other stream,
// whose fused epilogue + Adam may be spinning there on a hand-off flag -- a kernel needing a whole SIMD's
// register file would wait for that spin to end, i.e. forever: measured, test_gpu_handoff)

__device__ __forceinline__ hf32x4 mfma16(float a, float b, hf32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[u] += A(16 jb[u] + i, k) X[i][k] over k < K for the NB blocks jb[u] (< 0: skipped) of one matrix.
// WT = false: A(j, k) = W[j K + k] (a torch Linear weight [J][K], rows 16-byte aligned: flat.py);
// WT = true:  A(j, k) = W[k J + j] (the transposed product with a [K][J] weight).  Rows j >= J read 0.
template <bool WT, int NB>
__device__ __forceinline__ void contract(const float* __restrict__ W, int J, int K, const int (&jb)[NB],
                                         const float* X, int px, hf32x4 (&acc)[NB]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    for (int c0 = 0; c0 < K; c0 += 16 * KC) {
        hf32x4 a[NB][KC];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int j = 16 * jb[u] + i;
            const bool jok = jb[u] >= 0 && j < J;
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int k = c0 + 16 * c + 4 * g;
                a[u][c] = hf32x4{0.f, 0.f, 0.f, 0.f};
                if (jok && k < K) {
                    // (32-bit element offsets from the uniform matrix base: scalar base + one VGPR per load)
                    if constexpr (!WT) {
                        a[u][c] = *reinterpret_cast<const hf32x4*>(W + (j * K + k));
                    } else {
                        const int o = k * J + j;
                        a[u][c] = hf32x4{W[o], W[o + J], W[o + 2 * J], W[o + 3 * J]};
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            if (c0 + 16 * c < K) {     // wave-uniform
                const hf32x4 b = *reinterpret_cast<const hf32x4*>(X + i * px + c0 + 16 * c + 4 * g);
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    acc[u] = mfma16(a[u][c].x, b.x, acc[u]);
                    acc[u] = mfma16(a[u][c].y, b.y, acc[u]);
                    acc[u] = mfma16(a[u][c].z, b.z, acc[u]);
                    acc[u] = mfma16(a[u][c].w, b.w, acc[u]);
                }
            }
        }
    }
}

// One stage over nv virtual blocks: wave w takes blocks w, w + 4, ... two at a time (two independent
// accumulator chains); src(vb, W, J, jb) names the matrix and block of virtual block vb; epi(vb, acc).
template <bool WT, typename Src, typename Epi>
__device__ __forceinline__ void mstage(int nv, int K, const float* X, int px, Src src, Epi epi) {
    const int wv = threadIdx.x >> 6;
    for (int v0 = wv; v0 < nv; v0 += 8) {
        const int v1 = v0 + 4;
        const float *W0, *W1;
        int J0, J1, jb0, jb1;
        src(v0, W0, J0, jb0);
        if (v1 < nv) src(v1, W1, J1, jb1);
        hf32x4 acc0[1] = {hf32x4{0.f, 0.f, 0.f, 0.f}}, acc1[1] = {hf32x4{0.f, 0.f, 0.f, 0.f}};
        if (v1 < nv && W0 == W1 && J0 == J1) {
            hf32x4 acc[2] = {acc0[0], acc1[0]};
            const int jb[2] = {jb0, jb1};
            contract<WT, 2>(W0, J0, K, jb, X, px, acc);
            acc0[0] = acc[0];
            acc1[0] = acc[1];
        } else {
            const int jbA[1] = {jb0};
            contract<WT, 1>(W0, J0, K, jbA, X, px, acc0);
            if (v1 < nv) {
                const int jbB[1] = {jb1};
                contract<WT, 1>(W1, J1, K, jbB, X, px, acc1);
            }
        }
        epi(v0, acc0[0]);
        if (v1 < nv) epi(v1, acc1[0]);
    }
}

struct HTile {
    int s0, n, enc;   // first sample, valid samples, encoder tile
};

__device__ __forceinline__ HTile head_tile(const gpi_head_desc& d, int t) {
    const int et = (d.n_enc + TS - 1) / TS;
    HTile T;
    if (t < et) {
        T.s0 = TS * t;
        T.n = min(TS, d.n_enc - T.s0);
        T.enc = 1;
    } else {
        T.s0 = d.n_enc + TS * (t - et);
        T.n = min(TS, d.n_enc + d.n_q + d.n_q2 - T.s0);
        T.enc = 0;
    }
    return T;
}

__device__ __forceinline__ void zero_lds(float* p, int n) {   // n: multiple of 4, p 16-byte aligned
    for (int e = threadIdx.x; e < n / 4; e += 256) reinterpret_cast<float4*>(p)[e] = float4{0.f, 0.f, 0.f, 0.f};
}

// rows s0 .. s0 + n of a [*, w] workspace matrix into LDS rows (pitch px), w % 4 == 0
__device__ __forceinline__ void rows_to_lds(const float* src, int s0, int n, int w, float* dst, int px) {
    const int w4 = w >> 2;
    for (int e = threadIdx.x; e < n * w4; e += 256) {
        const int i = e / w4, c = e - i * w4;
        *reinterpret_cast<float4*>(dst + i * px + 4 * c) =
            *reinterpret_cast<const float4*>(src + (int64_t)(s0 + i) * w + 4 * c);
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(128))) void head_fwd_mfma(gpi_head_desc d, const float* __restrict__ P, float* ws) {
    __shared__ __attribute__((aligned(16))) float sX[TS * LPW], sH[TS * LPW], sMU[TS * LPZ], sLS[TS * LPZ],
        sZ[TS * LPZ];
    __shared__ float scratch[32], red[8];
    const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
    const HTile T = head_tile(d, blockIdx.x);
    const int dz = d.d_z, df = d.d_feat;
    zero_lds(sX, TS * LPW);
    zero_lds(sH, TS * LPW);
    zero_lds(sMU, TS * LPZ);
    zero_lds(sLS, TS * LPZ);
    zero_lds(sZ, TS * LPZ);
    __syncthreads();
    float kl[2] = {0.f, 0.f};   // per variational segment (encoder tile: [0])
    if (T.enc) {
        if (d.flags & GPI_HEAD_ENC) {
            rows_to_lds(ws + d.feat, T.s0, T.n, df, sX, LPW);
            __syncthreads();
            // FC + bias -> hpre (workspace), ReLU -> sH
            mstage<false>((df + 15) >> 4, df, sX, LPW,
                [&](int v, const float*& W, int& J, int& jb) { W = P + d.fc_w; J = df; jb = v; },
                [&](int v, hf32x4 a) {
                    const int j = 16 * v + 4 * g;
                    if (i < T.n && j < df) {
                        const float* b = P + d.fc_b + j;
                        const hf32x4 y{a.x + b[0], a.y + b[1], a.z + b[2], a.w + b[3]};
                        *reinterpret_cast<hf32x4*>(ws + d.hpre + (int64_t)(T.s0 + i) * df + j) = y;
                        *reinterpret_cast<hf32x4*>(sH + i * LPW + j) =
                            hf32x4{fmaxf(y.x, 0.f), fmaxf(y.y, 0.f), fmaxf(y.z, 0.f), fmaxf(y.w, 0.f)};
                    }
                });
            __syncthreads();
            // (mu, logsigma) heads: virtual blocks [0, nbz) of fc_mean, [nbz, 2 nbz) of fc_logvar
            const int nbz = (dz + 15) >> 4;
            mstage<false>(2 * nbz, df, sH, LPW,
                [&](int v, const float*& W, int& J, int& jb) {
                    W = P + (v < nbz ? d.mu_w : d.ls_w);
                    J = dz;
                    jb = v < nbz ? v : v - nbz;
                },
                [&](int v, hf32x4 a) {
                    const bool m = v < nbz;
                    const int j = 16 * (m ? v : v - nbz) + 4 * g;
                    if (i < T.n && j < dz) {
                        const float* b = P + (m ? d.mu_b : d.ls_b) + j;
                        const hf32x4 y{a.x + b[0], a.y + b[1], a.z + b[2], a.w + b[3]};
                        *reinterpret_cast<hf32x4*>(ws + (m ? d.zmu : d.zls) + (int64_t)(T.s0 + i) * dz + j) = y;
                        *reinterpret_cast<hf32x4*>((m ? sMU : sLS) + i * LPZ + j) = y;
                    }
                });
        } else {
            rows_to_lds(ws + d.zmu, T.s0, T.n, dz, sMU, LPZ);
            rows_to_lds(ws + d.zls, T.s0, T.n, dz, sLS, LPZ);
        }
        __syncthreads();
        for (int e = tid; e < T.n * dz; e += 256) {
            const int si = e / dz, k = e - si * dz;
            const int64_t o = (int64_t)(T.s0 + si) * dz + k;
            if (d.flags & GPI_HEAD_REPARAM) {
                const float mu = sMU[si * LPZ + k], ls = sLS[si * LPZ + k];
                const float ex = expf(ls);
                const float zz = fmaf(ex, ws[d.eps_z + o], mu);
                sZ[si * LPZ + k] = zz;
                ws[d.z + o] = zz;
                kl[0] += 1.f + 2.f * ls - mu * mu - ex * ex;
            } else {
                sZ[si * LPZ + k] = ws[d.z + o];
            }
        }
    } else {
        for (int e = tid; e < T.n * dz; e += 256) {
            const int si = e / dz, k = e - si * dz;
            const int s = T.s0 + si, q = s - d.n_enc;
            const QSeg sg = qseg(d, q);
            if (sg.flags & GPI_HEAD_QZ) {
                const float mu = P[sg.qz_mu + (int64_t)sg.row * dz + k], ls = P[sg.qz_ls + (int64_t)sg.row * dz + k];
                const float ex = expf(ls);
                const float zz = fmaf(ex, ws[d.eps_z + (int64_t)s * dz + k], mu);
                sZ[si * LPZ + k] = zz;
                ws[d.z + (int64_t)s * dz + k] = zz;
                kl[q >= d.n_q] += 1.f + 2.f * ls - mu * mu - ex * ex;
            } else {
                sZ[si * LPZ + k] = ws[d.z + (int64_t)s * dz + k];
            }
        }
    }
    block_sum<2>(kl, scratch, red);
    __syncthreads();
    if (tid == 0) {
        const int r = blockIdx.x % GPI_REPLICAS;
        if (T.enc) {
            if (d.flags & GPI_HEAD_REPARAM) atomicAdd(d.terms + 0 * GPI_REPLICAS + r, -0.5 * (double)red[0]);
        } else {
            // segments present in the tile, with their q_z KL
            const int qa = T.s0 - d.n_enc, qb = qa + T.n;
            if (qa < d.n_q && (d.flags & GPI_HEAD_QZ)) atomicAdd(d.terms + GPI_REPLICAS + r, -0.5 * (double)red[0]);
            if (qb > d.n_q && (d.flags2 & GPI_HEAD_QZ)) atomicAdd(d.terms2 + r, -0.5 * (double)red[1]);
        }
    }
    // decoder latent map (all samples) -> workspace
    if (d.flags & GPI_HEAD_LATENT) {
        const int dl = d.d_lat;
        mstage<false>((dl + 15) >> 4, dz, sZ, LPZ,
            [&](int v, const float*& W, int& J, int& jb) { W = P + d.lat_w; J = dl; jb = v; },
            [&](int v, hf32x4 a) {
                const int j = 16 * v + 4 * g;
                if (i < T.n && j < dl) {
                    const float* b = P + d.lat_b + j;
                    *reinterpret_cast<hf32x4*>(ws + d.lat + (int64_t)(T.s0 + i) * dl + j) =
                        hf32x4{a.x + b[0], a.y + b[1], a.z + b[2], a.w + b[3]};
                }
            });
    }
    if (T.enc) return;
    const bool gp1 = (d.flags & GPI_HEAD_GP) != 0, gp2 = (d.flags2 & GPI_HEAD_GP) != 0;
    if (!gp1 && !gp2) return;
    // effective-property map gp(z) -> sX, then per element: X~ (q_X sample or gp(z) itself), log-lik, entropy
    const int dx = d.d_x;
    mstage<false>((dx + 15) >> 4, dz, sZ, LPZ,
        [&](int v, const float*& W, int& J, int& jb) { W = P + d.gp_w; J = dx; jb = v; },
        [&](int v, hf32x4 a) {
            const int j = 16 * v + 4 * g;
            if (i < T.n && j < dx) {
                const float* b = P + d.gp_b + j;
                *reinterpret_cast<hf32x4*>(sX + i * LPW + j) = hf32x4{a.x + b[0], a.y + b[1], a.z + b[2], a.w + b[3]};
            }
        });
    __syncthreads();
    float acc4[4] = {0.f, 0.f, 0.f, 0.f};   // logL_X, entropy of segment 1; of segment 2
    for (int e = tid; e < T.n * dx; e += 256) {
        const int si = e / dx, t = e - si * dx;
        const int s = T.s0 + si, q = s - d.n_enc;
        const QSeg sg = qseg(d, q);
        if (!(sg.flags & GPI_HEAD_GP)) continue;
        const float a = sX[si * LPW + t];
        const int64_t qi = (int64_t)q * dx + t;                 // workspace row
        if (sg.flags & GPI_HEAD_LOCKX) {                       // X~ = gp(z) (generative.py:432)
            ws[d.mux + qi] = a;
            ws[d.xs + qi] = a;
            continue;
        }
        const int64_t pi = (int64_t)sg.row * dx + t;           // q_X parameter row
        const float lsq = P[sg.qx_ls + pi];
        const float xs = fmaf(expf(lsq), ws[d.eps_x + qi], P[sg.qx_mu + pi]);
        ws[d.mux + qi] = a;
        ws[d.xs + qi] = xs;
        const float gls = P[d.gp_ls + t];
        const float rr = xs - a;
        const int h = q >= d.n_q ? 2 : 0;
        acc4[h] += -0.5f * (2.f * gls + rr * rr * expf(-2.f * gls) + GPI_LOG2PI);
        acc4[h + 1] += lsq;
    }
    if ((gp1 && (d.flags & GPI_HEAD_LOCKX)) && (!gp2 || (d.flags2 & GPI_HEAD_LOCKX))) return;   // uniform
    block_sum<4>(acc4, scratch, red);
    __syncthreads();
    if (tid == 0) {
        const int r = blockIdx.x % GPI_REPLICAS;
        const int qa = T.s0 - d.n_enc, qb = qa + T.n;
        if (qa < d.n_q && gp1 && !(d.flags & GPI_HEAD_LOCKX)) {
            atomicAdd(d.terms + 2 * GPI_REPLICAS + r, (double)red[0]);
            atomicAdd(d.terms + 3 * GPI_REPLICAS + r, (double)red[1]);
        }
        if (qb > d.n_q && gp2 && !(d.flags2 & GPI_HEAD_LOCKX)) {
            atomicAdd(d.terms2 + 1 * GPI_REPLICAS + r, (double)red[2]);
            atomicAdd(d.terms2 + 2 * GPI_REPLICAS + r, (double)red[3]);
        }
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(128))) void head_bwd_mfma(gpi_head_desc d, const float* __restrict__ P, float* ws,
                                                     double* gacc, int t_off) {
    __shared__ __attribute__((aligned(16))) float sG[TS * LPW], sGM[TS * LPW], sDZ[TS * LPZ], sDMU[TS * LPZ],
        sDLS[TS * LPZ];
    const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
    const HTile T = head_tile(d, blockIdx.x + t_off);
    const int dz = d.d_z, df = d.d_feat, dl = d.d_lat, dx = d.d_x;
    zero_lds(sG, TS * LPW);
    zero_lds(sGM, TS * LPW);
    zero_lds(sDZ, TS * LPZ);
    zero_lds(sDMU, TS * LPZ);
    zero_lds(sDLS, TS * LPZ);
    __syncthreads();
    const bool lat = (d.flags & GPI_HEAD_LATENT) != 0;
    if (lat) rows_to_lds(ws + d.glat, T.s0, T.n, dl, sG, LPW);
    else rows_to_lds(ws + d.gz, T.s0, T.n, dz, sDZ, LPZ);
    // the tile's samples with a gp term (variational tiles): dJ/dmu_X -> sGM, the q_X rows' and
    // logsigma_X's gradients; one thread per feature t runs over the tile's samples in order
    const int qa = T.s0 - d.n_enc, qb = qa + T.n;
    const bool gp = !T.enc && ((qa < d.n_q && (d.flags & GPI_HEAD_GP)) || (qb > d.n_q && (d.flags2 & GPI_HEAD_GP)));
    if (gp) {
        for (int t = tid; t < dx; t += 256) {
            double gls_sum = 0.0;
            bool any = false;
            for (int si = 0; si < T.n; ++si) {
                const int q = qa + si;
                const QSeg sg = qseg(d, q);
                if (!(sg.flags & GPI_HEAD_GP)) continue;
                const int64_t qi = (int64_t)q * dx + t;
                if (sg.flags & GPI_HEAD_LOCKX) {               // dJ/dmu_X = dJ/dX~ (the ROM adjoint)
                    const float gm = ws[d.gxs + qi];
                    sGM[si * LPW + t] = gm;
                    ws[d.gmux + qi] = gm;
                    continue;
                }
                const int64_t pi = (int64_t)sg.row * dx + t;
                const float gls = P[d.gp_ls + t];
                const float e2 = expf(-2.f * gls);
                const float xs = ws[d.xs + qi], mux = ws[d.mux + qi];
                const float r = xs - mux;
                const float gm = -sg.lx_scale * r * e2;         // dJ/dmu_X
                sGM[si * LPW + t] = gm;
                ws[d.gmux + qi] = gm;
                gls_sum += (double)(sg.lx_scale * (1.f - r * r * e2));
                any = true;
                const float dxs = ws[d.gxs + qi] + sg.lx_scale * r * e2;   // dJ/dX~
                const float lsq = P[sg.qx_ls + pi];
                gacc[sg.qx_mu + pi] += (double)dxs;
                gacc[sg.qx_ls + pi] += (double)(dxs * expf(lsq) * ws[d.eps_x + qi] - sg.lx_scale);
            }
            if (any) atomicAdd(gacc + d.gp_ls + t, gls_sum);
        }
    }
    __syncthreads();
    // dJ/dz = lat_w^T glat (+ gp_w^T dJ/dmu_X), or the caller's gz (+ the gp part)
    if (lat || gp) {
        mstage<true>((dz + 15) >> 4, lat ? dl : dx, lat ? sG : sGM, LPW,
            [&](int v, const float*& W, int& J, int& jb) { W = P + (lat ? d.lat_w : d.gp_w); J = dz; jb = v; },
            [&](int v, hf32x4 a) {
                if (lat && gp) {
                    hf32x4 acc[1] = {a};
                    const int jb[1] = {v};
                    contract<true, 1>(P + d.gp_w, dz, dx, jb, sGM, LPW, acc);
                    a = acc[0];
                }
                const int j = 16 * v + 4 * g;
                if (i < T.n) {
                    hf32x4* p = reinterpret_cast<hf32x4*>(sDZ + i * LPZ + j);
                    *p = lat ? a : *p + a;
                }
            });
    }
    __syncthreads();
    if (!T.enc) {
        for (int e = tid; e < T.n * dz; e += 256) {
            const int si = e / dz, k = e - si * dz;
            const int s = T.s0 + si, q = s - d.n_enc;
            const QSeg sg = qseg(d, q);
            if (!(sg.flags & GPI_HEAD_QZ)) continue;
            const int64_t qi = (int64_t)sg.row * dz + k;
            const float mu = P[sg.qz_mu + qi], ls = P[sg.qz_ls + qi];
            const float ex = expf(ls);
            const float dzv = sDZ[si * LPZ + k];
            gacc[sg.qz_mu + qi] += (double)(dzv + sg.kl_scale * mu);
            gacc[sg.qz_ls + qi] += (double)(dzv * ex * ws[d.eps_z + (int64_t)s * dz + k] + sg.kl_scale * (ex * ex - 1.f));
        }
        return;
    }
    // encoder samples: reparametrisation + KL
    for (int e = tid; e < T.n * dz; e += 256) {
        const int si = e / dz, k = e - si * dz;
        const int64_t o = (int64_t)(T.s0 + si) * dz + k;
        float dmu = sDZ[si * LPZ + k], dls;
        const float mu = ws[d.zmu + o], ls = ws[d.zls + o];
        if (d.flags & GPI_HEAD_REPARAM) {
            const float ex = expf(ls);
            dls = sDZ[si * LPZ + k] * ex * ws[d.eps_z + o] + d.kl_scale_enc * (ex * ex - 1.f);
            dmu += d.kl_scale_enc * mu;
        } else {
            dls = ws[d.dzls + o];   // caller-provided d/dlogsigma
        }
        sDMU[si * LPZ + k] = dmu;
        sDLS[si * LPZ + k] = dls;
        ws[d.dzmu + o] = dmu;
        ws[d.dzls + o] = dls;
    }
    __syncthreads();
    if (!(d.flags & GPI_HEAD_ENC)) return;
    // heads: dh = fc_mean^T dmu + fc_logvar^T dls, ReLU mask of the stored pre-activation -> sGM
    mstage<true>((df + 15) >> 4, dz, sDMU, LPZ,
        [&](int v, const float*& W, int& J, int& jb) { W = P + d.mu_w; J = df; jb = v; },
        [&](int v, hf32x4 a) {
            hf32x4 acc[1] = {a};
            const int jb[1] = {v};
            contract<true, 1>(P + d.ls_w, df, dz, jb, sDLS, LPZ, acc);
            a = acc[0];
            const int j = 16 * v + 4 * g;
            if (i < T.n && j < df) {
                const int64_t o = (int64_t)(T.s0 + i) * df + j;
                const hf32x4 hp = *reinterpret_cast<const hf32x4*>(ws + d.hpre + o);
                const hf32x4 y{hp.x > 0.f ? a.x : 0.f, hp.y > 0.f ? a.y : 0.f, hp.z > 0.f ? a.z : 0.f,
                               hp.w > 0.f ? a.w : 0.f};
                *reinterpret_cast<hf32x4*>(sG + i * LPW + j) = y;
                *reinterpret_cast<hf32x4*>(ws + d.dhpre + o) = y;
            }
        });
    __syncthreads();
    // FC: gfeat = fc_w^T dh (sG's columns past d_feat hold stale glat values; their A operands are 0)
    mstage<true>((df + 15) >> 4, df, sG, LPW,
        [&](int v, const float*& W, int& J, int& jb) { W = P + d.fc_w; J = df; jb = v; },
        [&](int v, hf32x4 a) {
            const int j = 16 * v + 4 * g;
            if (i < T.n && j < df)
                *reinterpret_cast<hf32x4*>(ws + d.gfeat + (int64_t)(T.s0 + i) * df + j) = a;
        });
}

// gacc[c_off + m N + n] += sum_s A[s][m] B[s][n] for one 16 x 16 output tile (column N: the bias, B = 1):
// the samples split over the four waves in contiguous quarters (4 samples per MFMA, every operand load of
// a 64-sample group in flight at once), the waves' partial tiles summed in LDS in wave order.
struct GemmArgsM {
    gpi_gemm_item it[GPI_MAX_GEMM_ITEMS];
    int32_t first_block[GPI_MAX_GEMM_ITEMS + 1];
    int32_t tiles_n[GPI_MAX_GEMM_ITEMS];
    int32_t n;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(128))) void outer_gemm_mfma(GemmArgsM a, const float* __restrict__ ws, double* gacc) {
    __shared__ float part[4][16][17];
    int k = 0;
    while (k + 1 < a.n && (int)blockIdx.x >= a.first_block[k + 1]) ++k;
    const gpi_gemm_item it = a.it[k];
    const int local = blockIdx.x - a.first_block[k];
    const int tm = local / a.tiles_n[k], tn = local - tm * a.tiles_n[k];
    const int m0 = tm * 16, n0 = tn * 16;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
    const bool relu_b = it.flags & 1;
    const int q = (((it.S + 3) >> 2) + 3) >> 2;           // MFMA steps (4 samples each) per wave
    const int sb = wv * q * 4, se = min(it.S, sb + q * 4);
    const int m = m0 + i, n = n0 + i;
    const bool mok = m < it.M;
    hf32x4 acc = {0.f, 0.f, 0.f, 0.f};
    constexpr int GS = 16;                                 // steps in flight
    for (int s0 = sb; s0 < se; s0 += 4 * GS) {
        float av[GS], bv[GS];
#pragma unroll
        for (int u = 0; u < GS; ++u) {
            const int s = s0 + 4 * u + g;
            av[u] = 0.f;
            bv[u] = 0.f;
            if (s < se) {
                if (mok) av[u] = ws[it.a_off + (int64_t)s * it.lda + m];
                if (n < it.N) {
                    const float b = ws[it.b_off + (int64_t)s * it.ldb + n];
                    bv[u] = relu_b ? fmaxf(b, 0.f) : b;
                } else if (n == it.N) {
                    bv[u] = 1.f;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < GS; ++u)
            if (s0 + 4 * u < se) acc = mfma16(av[u], bv[u], acc);   // wave-uniform
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wv][4 * g + r][i] = acc[r];
    __syncthreads();
    const int mr = tid >> 4, nc = tid & 15;
    const float c = ((part[0][mr][nc] + part[1][mr][nc]) + part[2][mr][nc]) + part[3][mr][nc];
    const int mm = m0 + mr, nn = n0 + nc;
    if (mm < it.M) {   // (one writer per element: fire-and-forget atomics instead of a load round trip)
        if (nn < it.N) atomicAdd(gacc + it.c_off + (int64_t)mm * it.N + nn, (double)c);
        else if (nn == it.N && it.bias_off >= 0) atomicAdd(gacc + it.bias_off + mm, (double)c);
    }
}

// ---- the prefetched form for the codec families' widths (d_feat, d_z, d_lat, d_x all multiples of 16:
// highres 80 / 64 / 64 / 128, highres32 64 / 16 / 64 / 32): 512 threads, one 16-row output block per wave
// and stage, and EVERY global operand of the tile -- each wave's weight blocks of every stage, the biases,
// the element-wise operands (noise, variational rows, the stored pre-activations) -- issued at entry, so
// a tile pays one global round trip and then runs its chain of MFMA stages through LDS (the first form
// above waited for each stage's weights in turn: 15.7 / 13.2 us per launch against the VALU kernels'
// 8.3 / 9.7, profiles/r06a_*).
constexpr int HT2 = 512;

template <int NC>
struct Ops {
    hf32x4 a[NC];
};

// A operands of output block jb (< 0: zeros) of a J x K product, K <= 16 NC (16-wide chunks, lane (i, g):
// rows 16 jb + i, k = 16 c + 4 g + t): WT = false reads W[j K + k] (float4), WT = true W[k J + j]
template <bool WT, int NC>
__device__ __forceinline__ void wload(const float* __restrict__ W, int J, int K, int jb, Ops<NC>& o) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int j = 16 * jb + i;
    const bool jok = jb >= 0 && j < J;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int k = 16 * c + 4 * g;
        o.a[c] = hf32x4{0.f, 0.f, 0.f, 0.f};
        if (jok && k < K) {
            if constexpr (!WT) {
                o.a[c] = *reinterpret_cast<const hf32x4*>(W + (j * K + k));
            } else {
                const int q = k * J + j;
                o.a[c] = hf32x4{W[q], W[q + J], W[q + 2 * J], W[q + 3 * J]};
            }
        }
    }
}

template <int NC>
__device__ __forceinline__ hf32x4 wmma(const Ops<NC>& o, const float* X, int px, hf32x4 acc) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const hf32x4 b = *reinterpret_cast<const hf32x4*>(X + i * px + 16 * c + 4 * g);
        acc = mfma16(o.a[c].x, b.x, acc);
        acc = mfma16(o.a[c].y, b.y, acc);
        acc = mfma16(o.a[c].z, b.z, acc);
        acc = mfma16(o.a[c].w, b.w, acc);
    }
    return acc;
}

// the bias of the lane's four outputs 16 jb + 4 g + r of block jb (< 0: zeros), J % 4 == 0
__device__ __forceinline__ hf32x4 bload(const float* __restrict__ b, int J, int jb) {
    const int g = (threadIdx.x & 63) >> 4, j = 16 * jb + 4 * g;
    hf32x4 v{0.f, 0.f, 0.f, 0.f};
    if (jb >= 0 && j < J) v = hf32x4{b[j], b[j + 1], b[j + 2], b[j + 3]};
    return v;
}

__device__ __forceinline__ void zero_lds2(float* p, int n) {   // 512 threads
    for (int e = threadIdx.x; e < n / 4; e += HT2) reinterpret_cast<float4*>(p)[e] = float4{0.f, 0.f, 0.f, 0.f};
}

template <int CF, int CZ, int CL, int CX>
__global__ __launch_bounds__(HT2) __attribute__((amdgpu_num_vgpr(128))) void head_fwd_mfma2(gpi_head_desc d,
                                                                                          const float* __restrict__ P,
                                                                                          float* ws) {
    constexpr int DF = 16 * CF, DZ = 16 * CZ, DL = 16 * CL, DX = 16 * CX;
    constexpr int PF = DF + 4, PZ = DZ + 4, PX = DX + 4;
    constexpr int EU = (TS * DZ + HT2 - 1) / HT2, XU = (TS * DX + HT2 - 1) / HT2, FU = (TS * DF / 4 + HT2 - 1) / HT2;
    static_assert(CF <= 8 && 2 * CZ <= 8 && CL <= 8 && CX <= 8, "one block per wave and stage");
    __shared__ __attribute__((aligned(16))) float sX[TS * PF], sH[TS * PF], sMU[TS * PZ], sLS[TS * PZ], sZ[TS * PZ],
        sG[TS * PX];
    __shared__ float scratch[64], red[8];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
    const HTile T = head_tile(d, blockIdx.x);
    const int qa = T.s0 - d.n_enc;
    const bool enc_fc = T.enc && (d.flags & GPI_HEAD_ENC);
    const bool reparam = T.enc && (d.flags & GPI_HEAD_REPARAM);
    const bool lat = (d.flags & GPI_HEAD_LATENT) != 0;
    const bool gp1 = qa < d.n_q && (d.flags & GPI_HEAD_GP), gp2 = qa + T.n > d.n_q && (d.flags2 & GPI_HEAD_GP);
    const bool gp = !T.enc && (gp1 || gp2);
    // ---- every global operand in flight first
    Ops<CF> aF, aH;
    Ops<CZ> aL, aG;
    hf32x4 bF{0.f, 0.f, 0.f, 0.f}, bH = bF, bL = bF, bG = bF;
    const int hb = w < CZ ? w : w - CZ;                 // heads: waves [0, CZ) fc_mean, [CZ, 2 CZ) fc_logvar
    if (enc_fc) {
        wload<false>(P + d.fc_w, DF, DF, w < CF ? w : -1, aF);
        wload<false>(P + (w < CZ ? d.mu_w : d.ls_w), DZ, DF, w < 2 * CZ ? hb : -1, aH);
        bF = bload(P + d.fc_b, DF, w < CF ? w : -1);
        bH = bload(P + (w < CZ ? d.mu_b : d.ls_b), DZ, w < 2 * CZ ? hb : -1);
    }
    if (lat) {
        wload<false>(P + d.lat_w, DL, DZ, w < CL ? w : -1, aL);
        bL = bload(P + d.lat_b, DL, w < CL ? w : -1);
    }
    if (gp) {
        wload<false>(P + d.gp_w, DX, DZ, w < CX ? w : -1, aG);
        bG = bload(P + d.gp_b, DX, w < CX ? w : -1);
    }
    float4 fv[FU];
    if (enc_fc) {
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int e = tid + HT2 * u, si = e / (DF / 4), c = e - si * (DF / 4);
            fv[u] = si < T.n ? *reinterpret_cast<const float4*>(ws + d.feat + (int64_t)(T.s0 + si) * DF + 4 * c)
                             : float4{0.f, 0.f, 0.f, 0.f};
        }
    }
    // (sample, z) elements: noise, and the variational rows (q tiles), the stored z (no reparametrisation) or
    // the caller's mu / logsigma (encoder tiles without the FC)
    float eE[EU], eM[EU], eL[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
        eE[u] = eM[u] = eL[u] = 0.f;
        if (si >= T.n) continue;
        const int s = T.s0 + si;
        const int64_t o = (int64_t)s * DZ + k;
        if (T.enc) {
            if (reparam) {
                eE[u] = ws[d.eps_z + o];
                if (!enc_fc) {
                    eM[u] = ws[d.zmu + o];
                    eL[u] = ws[d.zls + o];
                }
            } else {
                eM[u] = ws[d.z + o];
            }
        } else {
            const QSeg sg = qseg(d, qa + si);
            if (sg.flags & GPI_HEAD_QZ) {
                eE[u] = ws[d.eps_z + o];
                eM[u] = P[sg.qz_mu + (int64_t)sg.row * DZ + k];
                eL[u] = P[sg.qz_ls + (int64_t)sg.row * DZ + k];
            } else {
                eM[u] = ws[d.z + o];
            }
        }
    }
    // (sample, x) elements of the gp term: q_X mean / logsigma, noise, logsigma_X
    float xM[XU], xL[XU], xE[XU], xG[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        xM[u] = xL[u] = xE[u] = xG[u] = 0.f;
        const int e = tid + HT2 * u, si = e / DX, t = e - si * DX;
        if (!gp || si >= T.n) continue;
        const QSeg sg = qseg(d, qa + si);
        if (!(sg.flags & GPI_HEAD_GP) || (sg.flags & GPI_HEAD_LOCKX)) continue;
        const int64_t pi = (int64_t)sg.row * DX + t;
        xM[u] = P[sg.qx_mu + pi];
        xL[u] = P[sg.qx_ls + pi];
        xE[u] = ws[d.eps_x + (int64_t)(qa + si) * DX + t];
        xG[u] = P[d.gp_ls + t];
    }
    zero_lds2(sX, TS * PF);
    zero_lds2(sH, TS * PF);
    zero_lds2(sZ, TS * PZ);
    zero_lds2(sG, TS * PX);
    __syncthreads();
    if (enc_fc) {
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int e = tid + HT2 * u, si = e / (DF / 4), c = e - si * (DF / 4);
            if (si < TS) *reinterpret_cast<float4*>(sX + si * PF + 4 * c) = fv[u];
        }
        __syncthreads();
        // FC + bias -> hpre (workspace), ReLU -> sH
        if (w < CF) {
            const hf32x4 a = wmma(aF, sX, PF, hf32x4{0.f, 0.f, 0.f, 0.f}) + bF;
            const int j = 16 * w + 4 * g;
            if (i < T.n) {
                *reinterpret_cast<hf32x4*>(ws + d.hpre + (int64_t)(T.s0 + i) * DF + j) = a;
                *reinterpret_cast<hf32x4*>(sH + i * PF + j) =
                    hf32x4{fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f)};
            }
        }
        __syncthreads();
        // (mu, logsigma) heads
        if (w < 2 * CZ) {
            const hf32x4 a = wmma(aH, sH, PF, hf32x4{0.f, 0.f, 0.f, 0.f}) + bH;
            const int j = 16 * hb + 4 * g;
            if (i < T.n) {
                *reinterpret_cast<hf32x4*>(ws + (w < CZ ? d.zmu : d.zls) + (int64_t)(T.s0 + i) * DZ + j) = a;
                *reinterpret_cast<hf32x4*>((w < CZ ? sMU : sLS) + i * PZ + j) = a;
            }
        }
        __syncthreads();
    }
    // z (reparametrisation or the q_z draw) and the KL terms
    float kl[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
        if (si >= T.n) continue;
        const int64_t o = (int64_t)(T.s0 + si) * DZ + k;
        float zz = eM[u];
        bool draw = reparam;
        float mu = eM[u], ls = eL[u];
        int h = 0;
        if (T.enc) {
            if (enc_fc) {
                mu = sMU[si * PZ + k];
                ls = sLS[si * PZ + k];
            }
        } else {
            const QSeg sg = qseg(d, qa + si);
            draw = (sg.flags & GPI_HEAD_QZ) != 0;
            h = qa + si >= d.n_q;
        }
        if (draw) {
            const float ex = expf(ls);
            zz = fmaf(ex, eE[u], mu);
            ws[d.z + o] = zz;
            kl[h] += 1.f + 2.f * ls - mu * mu - ex * ex;
        }
        sZ[si * PZ + k] = zz;
    }
    block_sum<2>(kl, scratch, red);
    __syncthreads();
    if (tid == 0) {
        const int r = blockIdx.x % GPI_REPLICAS;
        if (T.enc) {
            if (reparam) atomicAdd(d.terms + r, -0.5 * (double)red[0]);
        } else {
            if (qa < d.n_q && (d.flags & GPI_HEAD_QZ)) atomicAdd(d.terms + GPI_REPLICAS + r, -0.5 * (double)red[0]);
            if (qa + T.n > d.n_q && (d.flags2 & GPI_HEAD_QZ)) atomicAdd(d.terms2 + r, -0.5 * (double)red[1]);
        }
    }
    // decoder latent map -> workspace; effective-property map gp(z) -> sG
    if (lat && w < CL) {
        const hf32x4 a = wmma(aL, sZ, PZ, hf32x4{0.f, 0.f, 0.f, 0.f}) + bL;
        if (i < T.n) *reinterpret_cast<hf32x4*>(ws + d.lat + (int64_t)(T.s0 + i) * DL + 16 * w + 4 * g) = a;
    }
    if (!gp) return;
    if (w < CX) {
        const hf32x4 a = wmma(aG, sZ, PZ, hf32x4{0.f, 0.f, 0.f, 0.f}) + bG;
        if (i < T.n) *reinterpret_cast<hf32x4*>(sG + i * PX + 16 * w + 4 * g) = a;
    }
    __syncthreads();
    float acc4[4] = {0.f, 0.f, 0.f, 0.f};   // logL_X, entropy of segment 1; of segment 2
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int e = tid + HT2 * u, si = e / DX, t = e - si * DX;
        if (si >= T.n) continue;
        const int q = qa + si;
        const QSeg sg = qseg(d, q);
        if (!(sg.flags & GPI_HEAD_GP)) continue;
        const float a = sG[si * PX + t];
        const int64_t qi = (int64_t)q * DX + t;
        if (sg.flags & GPI_HEAD_LOCKX) {                       // X~ = gp(z) (generative.py:432)
            ws[d.mux + qi] = a;
            ws[d.xs + qi] = a;
            continue;
        }
        const float xs = fmaf(expf(xL[u]), xE[u], xM[u]);
        ws[d.mux + qi] = a;
        ws[d.xs + qi] = xs;
        const float gls = xG[u];
        const float rr = xs - a;
        const int h = q >= d.n_q ? 2 : 0;
        acc4[h] += -0.5f * (2.f * gls + rr * rr * expf(-2.f * gls) + GPI_LOG2PI);
        acc4[h + 1] += xL[u];
    }
    const bool lx1 = gp1 && !(d.flags & GPI_HEAD_LOCKX), lx2 = gp2 && !(d.flags2 & GPI_HEAD_LOCKX);
    if (!lx1 && !lx2) return;   // uniform
    block_sum<4>(acc4, scratch, red);
    __syncthreads();
    if (tid == 0) {
        const int r = blockIdx.x % GPI_REPLICAS;
        if (lx1) {
            atomicAdd(d.terms + 2 * GPI_REPLICAS + r, (double)red[0]);
            atomicAdd(d.terms + 3 * GPI_REPLICAS + r, (double)red[1]);
        }
        if (lx2) {
            atomicAdd(d.terms2 + 1 * GPI_REPLICAS + r, (double)red[2]);
            atomicAdd(d.terms2 + 2 * GPI_REPLICAS + r, (double)red[3]);
        }
    }
}

template <int CF, int CZ, int CL, int CX>
__global__ __launch_bounds__(HT2) __attribute__((amdgpu_num_vgpr(128))) void head_bwd_mfma2(gpi_head_desc d,
                                                                                          const float* __restrict__ P,
                                                                                          float* ws, double* gacc,
                                                                                          int t_off) {
    constexpr int DF = 16 * CF, DZ = 16 * CZ, DL = 16 * CL, DX = 16 * CX;
    constexpr int PF = DF + 4, PZ = DZ + 4, PL = DL + 4, PX = DX + 4;
    constexpr int EU = (TS * DZ + HT2 - 1) / HT2, XU = (TS * DX + HT2 - 1) / HT2, LU = (TS * DL / 4 + HT2 - 1) / HT2;
    static_assert(CF <= 8 && CZ <= 4 && CL <= 8 && CX <= 8, "one block per wave and stage");
    __shared__ __attribute__((aligned(16))) float sG[TS * PL], sGM[TS * PX], sC[TS * PX], sDZ[TS * PZ],
        sP[TS * PZ], sDMU[TS * PZ], sDLS[TS * PZ], sDH[TS * PF];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
    const HTile T = head_tile(d, blockIdx.x + t_off);
    const int qa = T.s0 - d.n_enc;
    const bool lat = (d.flags & GPI_HEAD_LATENT) != 0;
    const bool enc_fc = T.enc && (d.flags & GPI_HEAD_ENC);
    const bool gp1 = qa < d.n_q && (d.flags & GPI_HEAD_GP), gp2 = qa + T.n > d.n_q && (d.flags2 & GPI_HEAD_GP);
    const bool gp = !T.enc && (gp1 || gp2);
    // ---- every global operand in flight first
    // dJ/dz blocks: waves [0, CZ) the latent map's part (lat_w^T glat), waves [4, 4 + CZ) the gp part
    Ops<CL> aLT;
    Ops<CX> aGT;
    if (lat) wload<true>(P + d.lat_w, DZ, DL, w < CZ ? w : -1, aLT);
    if (gp) wload<true>(P + d.gp_w, DZ, DX, (w >= 4 && w < 4 + CZ) ? w - 4 : -1, aGT);
    // encoder tiles: dh blocks (fc_mean^T dmu + fc_logvar^T dls) and the FC's input gradient, waves [0, CF)
    Ops<CZ> aMT, aST;
    Ops<CF> aFT;
    hf32x4 hp{0.f, 0.f, 0.f, 0.f};
    if (enc_fc) {
        wload<true>(P + d.mu_w, DF, DZ, w < CF ? w : -1, aMT);
        wload<true>(P + d.ls_w, DF, DZ, w < CF ? w : -1, aST);
        wload<true>(P + d.fc_w, DF, DF, w < CF ? w : -1, aFT);
        if (w < CF && i < T.n) hp = *reinterpret_cast<const hf32x4*>(ws + d.hpre + (int64_t)(T.s0 + i) * DF + 16 * w + 4 * g);
    }
    // the latent map's output gradient (or the caller's dJ/dz) rows
    float4 lv[LU > 0 ? LU : 1];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
        const int e = tid + HT2 * u, si = e / (DL / 4), c = e - si * (DL / 4);
        lv[u] = (lat && si < T.n) ? *reinterpret_cast<const float4*>(ws + d.glat + (int64_t)(T.s0 + si) * DL + 4 * c)
                                  : float4{0.f, 0.f, 0.f, 0.f};
    }
    // (sample, z) elements: mu / logsigma (encoder: workspace; q: q_z rows), noise, the caller's dJ/dz
    float eM[EU], eL[EU], eE[EU], eZ[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
        eM[u] = eL[u] = eE[u] = eZ[u] = 0.f;
        if (si >= T.n) continue;
        const int64_t o = (int64_t)(T.s0 + si) * DZ + k;
        if (!lat) eZ[u] = ws[d.gz + o];
        if (T.enc) {
            eM[u] = ws[d.zmu + o];
            eL[u] = ws[d.zls + o];
            if (d.flags & GPI_HEAD_REPARAM) eE[u] = ws[d.eps_z + o];
            else eE[u] = ws[d.dzls + o];      // caller-provided d/dlogsigma
        } else {
            const QSeg sg = qseg(d, qa + si);
            if (sg.flags & GPI_HEAD_QZ) {
                eM[u] = P[sg.qz_mu + (int64_t)sg.row * DZ + k];
                eL[u] = P[sg.qz_ls + (int64_t)sg.row * DZ + k];
                eE[u] = ws[d.eps_z + o];
            }
        }
    }
    // (sample, x) elements of the gp term
    float xS[XU], xMu[XU], xGx[XU], xE[XU], xL[XU], xG[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        xS[u] = xMu[u] = xGx[u] = xE[u] = xL[u] = xG[u] = 0.f;
        const int e = tid + HT2 * u, si = e / DX, t = e - si * DX;
        if (!gp || si >= T.n) continue;
        const int q = qa + si;
        const QSeg sg = qseg(d, q);
        if (!(sg.flags & GPI_HEAD_GP)) continue;
        const int64_t qi = (int64_t)q * DX + t;
        xGx[u] = ws[d.gxs + qi];
        if (sg.flags & GPI_HEAD_LOCKX) continue;
        xS[u] = ws[d.xs + qi];
        xMu[u] = ws[d.mux + qi];
        xE[u] = ws[d.eps_x + qi];
        xL[u] = P[sg.qx_ls + (int64_t)sg.row * DX + t];
        xG[u] = P[d.gp_ls + t];
    }
    zero_lds2(sG, TS * PL);
    zero_lds2(sGM, TS * PX);
    zero_lds2(sC, TS * PX);
    zero_lds2(sDMU, TS * PZ);
    zero_lds2(sDLS, TS * PZ);
    zero_lds2(sDH, TS * PF);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < LU; ++u) {
        const int e = tid + HT2 * u, si = e / (DL / 4), c = e - si * (DL / 4);
        if (si < TS) *reinterpret_cast<float4*>(sG + si * PL + 4 * c) = lv[u];
    }
    // gp term: dJ/dmu_X -> sGM (and gmux), the q_X rows' gradients, logsigma_X's contributions -> sC
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int e = tid + HT2 * u, si = e / DX, t = e - si * DX;
        if (!gp || si >= T.n) continue;
        const int q = qa + si;
        const QSeg sg = qseg(d, q);
        if (!(sg.flags & GPI_HEAD_GP)) continue;
        const int64_t qi = (int64_t)q * DX + t;
        if (sg.flags & GPI_HEAD_LOCKX) {                      // dJ/dmu_X = dJ/dX~ (the ROM adjoint)
            sGM[si * PX + t] = xGx[u];
            ws[d.gmux + qi] = xGx[u];
            continue;
        }
        const int64_t pi = (int64_t)sg.row * DX + t;
        const float e2 = expf(-2.f * xG[u]);
        const float r = xS[u] - xMu[u];
        const float gm = -sg.lx_scale * r * e2;              // dJ/dmu_X
        sGM[si * PX + t] = gm;
        ws[d.gmux + qi] = gm;
        sC[si * PX + t] = sg.lx_scale * (1.f - r * r * e2);
        const float dxs = xGx[u] + sg.lx_scale * r * e2;     // dJ/dX~
        // (per-sample rows, one writer each: the atomic is a fire-and-forget read-modify-write, no load round
        // trip inside the kernel)
        atomicAdd(gacc + sg.qx_mu + pi, (double)dxs);
        atomicAdd(gacc + sg.qx_ls + pi, (double)(dxs * expf(xL[u]) * xE[u] - sg.lx_scale));
    }
    __syncthreads();
    if (lat && w < CZ) {
        const hf32x4 a = wmma(aLT, sG, PL, hf32x4{0.f, 0.f, 0.f, 0.f});
        if (i < T.n) *reinterpret_cast<hf32x4*>(sDZ + i * PZ + 16 * w + 4 * g) = a;
    }
    if (gp && w >= 4 && w < 4 + CZ) {
        const hf32x4 a = wmma(aGT, sGM, PX, hf32x4{0.f, 0.f, 0.f, 0.f});
        if (i < T.n) *reinterpret_cast<hf32x4*>(sP + i * PZ + 16 * (w - 4) + 4 * g) = a;
    }
    // logsigma_X: the tile's contributions per feature, summed over its samples in order (fp64)
    const bool lx = (gp1 && !(d.flags & GPI_HEAD_LOCKX)) || (gp2 && !(d.flags2 & GPI_HEAD_LOCKX));
    if (lx && tid < DX) {
        double sum = 0.0;
        for (int si = 0; si < T.n; ++si) sum += (double)sC[si * PX + tid];
        atomicAdd(gacc + d.gp_ls + tid, sum);
    }
    __syncthreads();
    // dJ/dz = latent part (or the caller's) + gp part, then the variational / encoder rows
    float dzv[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
        dzv[u] = 0.f;
        if (si >= T.n) continue;
        dzv[u] = lat ? sDZ[si * PZ + k] : eZ[u];
        if (gp) dzv[u] += sP[si * PZ + k];
    }
    if (!T.enc) {
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
            if (si >= T.n) continue;
            const QSeg sg = qseg(d, qa + si);
            if (!(sg.flags & GPI_HEAD_QZ)) continue;
            const int64_t qi = (int64_t)sg.row * DZ + k;
            const float ex = expf(eL[u]);
            atomicAdd(gacc + sg.qz_mu + qi, (double)(dzv[u] + sg.kl_scale * eM[u]));
            atomicAdd(gacc + sg.qz_ls + qi, (double)(dzv[u] * ex * eE[u] + sg.kl_scale * (ex * ex - 1.f)));
        }
        return;
    }
    // encoder samples: reparametrisation + KL
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int e = tid + HT2 * u, si = e / DZ, k = e - si * DZ;
        if (si >= T.n) continue;
        const int64_t o = (int64_t)(T.s0 + si) * DZ + k;
        float dmu = dzv[u], dls;
        if (d.flags & GPI_HEAD_REPARAM) {
            const float ex = expf(eL[u]);
            dls = dzv[u] * ex * eE[u] + d.kl_scale_enc * (ex * ex - 1.f);
            dmu += d.kl_scale_enc * eM[u];
        } else {
            dls = eE[u];
        }
        sDMU[si * PZ + k] = dmu;
        sDLS[si * PZ + k] = dls;
        ws[d.dzmu + o] = dmu;
        ws[d.dzls + o] = dls;
    }
    if (!enc_fc) return;
    __syncthreads();
    // heads: dh = fc_mean^T dmu + fc_logvar^T dls, ReLU mask of the stored pre-activation
    if (w < CF) {
        hf32x4 a = wmma(aMT, sDMU, PZ, hf32x4{0.f, 0.f, 0.f, 0.f});
        a = wmma(aST, sDLS, PZ, a);
        const hf32x4 y{hp.x > 0.f ? a.x : 0.f, hp.y > 0.f ? a.y : 0.f, hp.z > 0.f ? a.z : 0.f, hp.w > 0.f ? a.w : 0.f};
        if (i < T.n) {
            *reinterpret_cast<hf32x4*>(sDH + i * PF + 16 * w + 4 * g) = y;
            *reinterpret_cast<hf32x4*>(ws + d.dhpre + (int64_t)(T.s0 + i) * DF + 16 * w + 4 * g) = y;
        }
    }
    __syncthreads();
    // FC: the encoder features' gradient fc_w^T dh
    if (w < CF) {
        const hf32x4 a = wmma(aFT, sDH, PF, hf32x4{0.f, 0.f, 0.f, 0.f});
        if (i < T.n) *reinterpret_cast<hf32x4*>(ws + d.gfeat + (int64_t)(T.s0 + i) * DF + 16 * w + 4 * g) = a;
    }
}

// the prefetched form's widths (0: none): d_feat / d_z / d_lat / d_x = 16 x (CF, CZ, CL, CX)
int head_family(const gpi_head_desc* d) {
    const bool enc = (d->flags & GPI_HEAD_ENC) && d->n_enc > 0;
    const int df = enc ? d->d_feat : 0;
    if ((df == 80 || !enc) && d->d_z == 64 && d->d_lat == 64 && d->d_x == 128) return 1;
    if ((df == 64 || !enc) && d->d_z == 16 && d->d_lat == 64 && d->d_x == 32) return 2;
    return 0;
}

// the MFMA kernels' preconditions: widths that fit the LDS row buffers, float4-aligned rows
bool head_mfma_ok(const gpi_head_desc* d) {
    static const int on = [] {
        const char* v = getenv("GPI_HEAD_MFMA");
        return v && *v ? atoi(v) : 1;
    }();
    if (!on || (d->flags & GPI_HEAD_VALU)) return false;
    const bool enc = (d->flags & GPI_HEAD_ENC) && d->n_enc > 0;
    if (d->d_z > MZ || (d->d_z & 3) || d->d_lat > MW || (d->d_lat & 3) || d->d_x > MW || (d->d_x & 3)) return false;
    if (enc && (d->d_feat > MW || (d->d_feat & 3))) return false;
    const int64_t offs[] = {enc ? d->fc_w : 0, enc ? d->mu_w : 0, enc ? d->ls_w : 0, enc ? d->feat : 0,
                            enc ? d->gfeat : 0, enc ? d->hpre : 0, enc ? d->dhpre : 0,
                            (d->flags & GPI_HEAD_LATENT) ? d->lat_w : 0, (d->flags & GPI_HEAD_LATENT) ? d->lat : 0,
                            (d->flags & GPI_HEAD_LATENT) ? d->glat : 0, d->zmu, d->zls, d->gz};
    for (int64_t o : offs)
        if (o & 3) return false;
    return true;
}

bool head_ok(const gpi_head_desc* d) {
    return d && d->d_z > 0 && d->d_z <= VMAX && d->d_feat <= VMAX && d->d_lat <= VMAX && d->d_x <= VMAX &&
           d->n_enc >= 0 && d->n_q >= 0 && d->n_q2 >= 0 && (d->n_enc + d->n_q + d->n_q2) > 0 && d->terms &&
           (d->n_q2 == 0 || d->terms2);
}

}  // namespace

extern "C" int gpi_head_forward(const gpi_head_desc* d, const float* params, float* ws, void* stream) {
    if (!head_ok(d) || !params || !ws) return GPI_ERR_ARG;
    if (head_mfma_ok(d)) {
        const int nt = (d->n_enc + TS - 1) / TS + (d->n_q + d->n_q2 + TS - 1) / TS;
        static const int pf = [] {
            const char* v = getenv("GPI_HEAD_PREFETCH");
            return v && *v ? atoi(v) : 1;
        }();
        const int fam = pf ? head_family(d) : 0;
        if (fam) {
            if (fam == 1) hipLaunchKernelGGL((head_fwd_mfma2<5, 4, 4, 8>), dim3(nt), dim3(HT2), 0, (hipStream_t)stream, *d, params, ws);
            else hipLaunchKernelGGL((head_fwd_mfma2<4, 1, 4, 2>), dim3(nt), dim3(HT2), 0, (hipStream_t)stream, *d, params, ws);
            GPI_CHECK_LAUNCH();
            return GPI_OK;
        }
        hipLaunchKernelGGL(head_fwd_mfma, dim3(nt), dim3(256), 0, (hipStream_t)stream, *d, params, ws);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    hipLaunchKernelGGL(head_fwd_kernel, dim3(d->n_enc + d->n_q + d->n_q2), dim3(HT), 0, (hipStream_t)stream, *d, params, ws);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_head_backward(const gpi_head_desc* d, const float* params, float* ws, double* gacc,
                                 void* stream) {
    if (!head_ok(d) || !params || !ws || !gacc) return GPI_ERR_ARG;
    const bool pe = d->flags & GPI_HEAD_PART_ENC, pq = d->flags & GPI_HEAD_PART_Q;
    if (pe && pq) return GPI_ERR_ARG;
    const int nq = d->n_q + d->n_q2;
    const int nb = pe ? d->n_enc : (pq ? nq : d->n_enc + nq), s_off = pq ? d->n_enc : 0;
    if (nb == 0) return GPI_OK;
    if (head_mfma_ok(d)) {
        const int et = (d->n_enc + TS - 1) / TS, qt = (nq + TS - 1) / TS;
        const int ntl = pe ? et : (pq ? qt : et + qt), t_off = pq ? et : 0;
        static const int pf = [] {
            const char* v = getenv("GPI_HEAD_PREFETCH");
            return v && *v ? atoi(v) : 1;
        }();
        const int fam = pf ? head_family(d) : 0;
        if (fam) {
            if (fam == 1)
                hipLaunchKernelGGL((head_bwd_mfma2<5, 4, 4, 8>), dim3(ntl), dim3(HT2), 0, (hipStream_t)stream, *d, params, ws,
                                   gacc, t_off);
            else
                hipLaunchKernelGGL((head_bwd_mfma2<4, 1, 4, 2>), dim3(ntl), dim3(HT2), 0, (hipStream_t)stream, *d, params, ws,
                                   gacc, t_off);
            GPI_CHECK_LAUNCH();
            return GPI_OK;
        }
        hipLaunchKernelGGL(head_bwd_mfma, dim3(ntl), dim3(256), 0, (hipStream_t)stream, *d, params, ws, gacc, t_off);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    hipLaunchKernelGGL(head_bwd_kernel, dim3(nb), dim3(HT), 0, (hipStream_t)stream, *d, params, ws, gacc, s_off);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_outer_gemm(const gpi_gemm_item* items, int n_items, const float* ws, double* gacc,
                              void* stream) {
    if (!items || n_items < 0 || n_items > GPI_MAX_GEMM_ITEMS || !ws || !gacc) return GPI_ERR_ARG;
    if (n_items == 0) return GPI_OK;
    GemmArgs a;
    a.n = n_items;
    int nb = 0;
    for (int k = 0; k < n_items; ++k) {
        a.it[k] = items[k];
        a.first_block[k] = nb;
        const int tm = (items[k].M + 15) / 16, tn = (items[k].N + 1 + 15) / 16;
        a.tiles_n[k] = tn;
        nb += tm * tn;
    }
    a.first_block[n_items] = nb;
    static const int mf = [] {
        const char* v = getenv("GPI_HEAD_MFMA");
        return v && *v ? atoi(v) : 1;
    }();
    if (mf && !(items[0].flags & 2)) {
        GemmArgsM am;
        am.n = a.n;
        for (int k = 0; k < n_items; ++k) {
            am.it[k] = a.it[k];
            am.first_block[k] = a.first_block[k];
            am.tiles_n[k] = a.tiles_n[k];
        }
        am.first_block[n_items] = nb;
        hipLaunchKernelGGL(outer_gemm_mfma, dim3(nb), dim3(256), 0, (hipStream_t)stream, am, ws, gacc);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    hipLaunchKernelGGL(outer_gemm_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, ws, gacc);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
