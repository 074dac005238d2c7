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

bool head_ok(const gpi_head_desc* d) {
    return d && d->d_z > 0 && d->d_z <= VMAX && d->d_feat <= VMAX && d->d_lat <= VMAX && d->d_x <= VMAX &&
           d->n_enc >= 0 && d->n_q >= 0 && d->n_q2 >= 0 && (d->n_enc + d->n_q + d->n_q2) > 0 && d->terms &&
           (d->n_q2 == 0 || d->terms2);
}

}  // namespace

extern "C" int gpi_head_forward(const gpi_head_desc* d, const float* params, float* ws, void* stream) {
    if (!head_ok(d) || !params || !ws) return GPI_ERR_ARG;
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
    hipLaunchKernelGGL(outer_gemm_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, ws, gacc);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
