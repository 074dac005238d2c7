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

// ------------------------------------------------------------------ folded codec convolutions
// (gpi_head_forward_folded / gpi_head_backward_folded: the encoder's last conv and the decoder's first
// one computed by the head's per-sample workgroup; same arithmetic as conv.hip's kernels)
constexpr int FOLD_CIN = 16, FOLD_COUT = 8, FOLD_HW = 8;      // planes of at most 8 x 8
constexpr int FOLD_PAD_IMG = FOLD_CIN * (FOLD_HW + 2) * (FOLD_HW + 2);   // padded input image
constexpr int FOLD_W = FOLD_COUT * FOLD_CIN * 9;
constexpr int FOLD_OUT = FOLD_COUT * FOLD_HW * FOLD_HW;
constexpr int FOLD_IN = FOLD_CIN * FOLD_HW * FOLD_HW;

struct FoldLds {
    float img[FOLD_PAD_IMG];     // padded activation (feat) / latent image (lat), later the dY image
    float w[FOLD_W];             // weights [cout][cin][3][3]
    float o[FOLD_OUT];           // outputs / gradients [cout][HWo] or [cin][HWi]
    float o2[2 * FOLD_IN];       // input-gradient channel-sum operands: dbn | dbn x-hat
    float sc[FOLD_CIN], sh[FOLD_CIN], gam[FOLD_CIN], mean[FOLD_CIN], inv[FOLD_CIN];
    float oc[4 * FOLD_COUT];     // output BN-backward coefficients: mean, inv, mS, mSx
    float ds[FOLD_COUT];         // Dropout2d scales of the output channels
};

// the GPI_REPLICAS records of field f of (group grp, stat st), summed in conv.hip stat_finish's order
// (per half the even and the odd replicas, then the halves), which tests/gpu_masks.py reproduces
__device__ __forceinline__ double fold_stat(const gpi_codec_ctx& c, int grp, int64_t st, int f) {
    const int64_t rs = (int64_t)GPI_MAX_GROUPS * c.n_stats * 4;          // doubles per replica
    const double* p = &c.stats[(int64_t)grp * c.n_stats + st].sum + f;
    double h[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
            s0 += p[(8 * hh + r) * rs];
            s1 += p[(8 * hh + r + 1) * rs];
        }
        h[hh] = s0 + s1;
    }
    return h[0] + h[1];
}

// conv.hip mean_invstd: every rounding spelled out
__device__ __forceinline__ void fold_mean_invstd(double s, double s2, double n, float eps, float& mean, float& inv) {
    const double m = s / n;
    double var = fma(-m, m, s2 / n);
    if (var < 0.0) var = 0.0;
    mean = (float)m;
    inv = (float)(1.0 / sqrt(var + (double)eps));
}

__device__ __forceinline__ int fold_group(const gpi_codec_ctx& c, int s, int& gsz) {
    const int g = group_of(c.groups, s);
    gsz = karg_sel(c.groups.start, g + 1) - karg_sel(c.groups.start, g);
    return g;
}

// weights [cout][cin][9] of c into F.w; the input BN coefficients (gamma, beta, batch statistics of
// the sample's group) into F.sc / F.sh / F.gam / F.mean / F.inv (threads < cin)
__device__ __forceinline__ void fold_stage_params(const gpi_conv_desc& c, const gpi_codec_ctx& x, const float* P,
                                                  FoldLds& F, int s) {
    const int tid = threadIdx.x;
    const int nw = c.cout * c.cin * 9;
    for (int e = tid; e < nw; e += HT) F.w[e] = P[c.w_off + e];
    if (c.in_bn && tid < c.cin) {
        int gsz;
        const int g = fold_group(x, s, gsz);
        const double s1 = fold_stat(x, g, c.in_stat + tid, 0), s2 = fold_stat(x, g, c.in_stat + tid, 1);
        float mean, inv;
        fold_mean_invstd(s1, s2, (double)gsz * c.h_in * c.w_in, x.bn_eps, mean, inv);
        const float gam = P[c.gamma_off + tid], bet = P[c.beta_off + tid];
        F.gam[tid] = gam;
        F.mean[tid] = mean;
        F.inv[tid] = inv;
        F.sc[tid] = gam * inv;
        F.sh[tid] = fmaf(-(mean * gam), inv, bet);
    }
    if (tid >= 64 && tid < 64 + c.cout)
        F.ds[tid - 64] = c.drop_off >= 0 ? x.ws[c.drop_off + (int64_t)s * c.cout + (tid - 64)] : 1.f;
}

// Plane geometry of a folded conv: power-of-two sides (host-checked), so every pixel decomposition is a
// shift; the stride is a template parameter (no runtime division anywhere in these loops).
struct FoldGeom {
    int lwi, lhwi, lwo, lhwo, Wp, Hp, PP;      // log2 widths / plane sizes, padded pitch / rows / plane
};

__device__ __forceinline__ int ilog2(int v) { return 31 - __clz(v); }

__device__ __forceinline__ FoldGeom fold_geom(const gpi_conv_desc& c) {
    FoldGeom g;
    g.lwi = ilog2(c.w_in);
    g.lhwi = ilog2(c.h_in * c.w_in);
    g.lwo = ilog2(c.w_out);
    g.lhwo = ilog2(c.h_out * c.w_out);
    g.Wp = c.w_in + 2;
    g.Hp = c.h_in + 2;
    g.PP = g.Hp * g.Wp;
    return g;
}

// the padded input image of sample s: BN + ReLU of the raw input (in_bn) or the raw input itself;
// src: the raw input in the program's layout (or, src_lds, already in LDS as [cin][HWi]).  The zero
// border is written by the first pass; callers sync before reading.
__device__ __forceinline__ void fold_input_image(const gpi_conv_desc& c, const float* ws, FoldLds& F, int s,
                                                 const float* src_lds) {
    const FoldGeom G = fold_geom(c);
    const int HWi = 1 << G.lhwi;
    for (int e = threadIdx.x; e < c.cin * G.PP; e += HT) F.img[e] = 0.f;
    __syncthreads();
    for (int e = threadIdx.x; e < c.cin * HWi; e += HT) {
        const int ci = e >> G.lhwi, p = e & (HWi - 1), y = p >> G.lwi, x = p & (c.w_in - 1);
        float v = src_lds ? src_lds[e] : ws[c.in_off + ((int64_t)s * c.in_ctot + c.in_c0) * HWi + e];
        if (c.in_bn) v = fmaxf(fmaf(v, F.sc[ci], F.sh[ci]), 0.f);
        F.img[ci * G.PP + (y + 1) * G.Wp + x + 1] = v;
    }
}

// forward of the folded conv for sample s: F.o[co * HWo + p] = dropout(conv(img)); stored to the
// output buffer; with a stats epilogue the per-channel fp32 sums go to the group's replica record
template <int S>
__device__ __forceinline__ void fold_forward_s(const gpi_conv_desc& c, const gpi_codec_ctx& x, FoldLds& F, int s,
                                               float* out_copy) {
    const int tid = threadIdx.x;
    const FoldGeom G = fold_geom(c);
    const int HWo = 1 << G.lhwo;
    for (int e = tid; e < c.cout * HWo; e += HT) {
        const int co = e >> G.lhwo, p = e & (HWo - 1), oy = p >> G.lwo, ox = p & (c.w_out - 1);
        float acc = 0.f;
        const float* im0 = F.img + (oy * S) * G.Wp + ox * S;
        const float* w0 = F.w + co * c.cin * 9;
        for (int ci = 0; ci < c.cin; ++ci) {
            const float* im = im0 + ci * G.PP;
            const float* w = w0 + ci * 9;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) acc = fmaf(w[ky * 3 + kx], im[ky * G.Wp + kx], acc);
        }
        acc *= F.ds[co];
        F.o[e] = acc;
        if (out_copy) out_copy[e] = acc;
        x.ws[c.out_off + ((int64_t)s * c.out_ctot + c.out_c0) * HWo + e] = acc;
    }
    if (c.epilogue != GPI_EPI_STORE_STATS || c.out_stat < 0) return;
    __syncthreads();
    // per channel: 16 lanes sum its pixels, fold by shuffles, one fp64 atomic per (channel, field)
    int gsz;
    const int g = fold_group(x, s, gsz);
    for (int co = tid >> 4; co < c.cout; co += HT / 16) {
        const int part = tid & 15;
        float a = 0.f, b = 0.f;
        for (int p = part; p < HWo; p += 16) {
            const float v = F.o[co * HWo + p];
            a += v;
            b += v * v;
        }
#pragma unroll
        for (int m = 8; m > 0; m >>= 1) {
            a += __shfl_xor(a, m, 64);
            b += __shfl_xor(b, m, 64);
        }
        if (part == 0) {
            gpi_stat* st = x.stats + ((int64_t)(blockIdx.x % GPI_REPLICAS) * GPI_MAX_GROUPS + g) * x.n_stats +
                           c.out_stat + co;
            atomicAdd(&st->sum, (double)a);
            atomicAdd(&st->sumsq, (double)b);
        }
    }
}

__device__ __forceinline__ void fold_forward(const gpi_conv_desc& c, const gpi_codec_ctx& x, FoldLds& F, int s,
                                             float* out_copy) {
    if (c.stride == 2) fold_forward_s<2>(c, x, F, s, out_copy);
    else fold_forward_s<1>(c, x, F, s, out_copy);
}

// backward of the folded conv for sample s, given its output gradient dY in F.o ([cout][HWo], already
// BN-backward'ed and dropout-scaled) and the padded input image in F.img (the activation): weight
// gradient slab row s, input gradient (ReLU mask, S_in (+)= gamma dbn) to gin and to gin_copy
// ([cin][HWi], may be nullptr), dgamma / dbeta partials and the input's BN-backward sums
template <int S>
__device__ __forceinline__ void fold_backward_s(const gpi_conv_desc& c, const gpi_codec_ctx& x, FoldLds& F, int s,
                                                float* gin_copy) {
    const int tid = threadIdx.x;
    const FoldGeom G = fold_geom(c);
    const int HWi = 1 << G.lhwi, HWo = 1 << G.lhwo;
    const int J = c.cin * 9, rowlen = c.cout * J + (c.in_bn ? 2 * c.cin : 0);
    float* slab = c.wpart_off >= 0 ? x.wpart + c.wpart_off + (int64_t)s * rowlen : nullptr;
    // weight gradient: dW[co][ci][ky][kx] = sum_p dY[co][p] img[ci][oy S + ky][ox S + kx]; item (ci, tap)
    // of every output channel per thread (the division by 9 is by a constant)
    if (slab) {
        for (int r = tid; r < J; r += HT) {
            const int ci = r / 9, t = r - 9 * ci, ky = t / 3, kx = t - 3 * ky;
            const float* im = F.img + ci * G.PP + ky * G.Wp + kx;
            for (int co = 0; co < c.cout; ++co) {
                const float* g = F.o + co * HWo;
                float a0 = 0.f, a1 = 0.f;
                for (int p = 0; p < HWo; p += 2) {
                    const int oy = p >> G.lwo, ox = p & (c.w_out - 1);
                    a0 = fmaf(g[p], im[(oy * S) * G.Wp + ox * S], a0);
                    a1 = fmaf(g[p + 1], im[(oy * S) * G.Wp + (ox + 1) * S], a1);
                }
                slab[co * J + r] = a0 + a1;
            }
        }
    }
    if (c.gin_off < 0) return;
    // input gradient: pixel (iy, ix) receives output (oy, ox) through tap (ky, kx) iff
    // oy S - 1 + ky = iy and ox S - 1 + kx = ix
    for (int e = tid; e < c.cin * HWi; e += HT) {
        const int ci = e >> G.lhwi, p = e & (HWi - 1), iy = p >> G.lwi, ix = p & (c.w_in - 1);
        float a = 0.f;
        for (int co = 0; co < c.cout; ++co) {
            const float* w = F.w + (co * c.cin + ci) * 9;
            const float* g = F.o + co * HWo;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const int ty = iy + 1 - ky;
                if (ty < 0 || (S == 2 && (ty & 1))) continue;
                const int oy = S == 2 ? ty >> 1 : ty;
                if (oy >= c.h_out) continue;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const int tx = ix + 1 - kx;
                    if (tx < 0 || (S == 2 && (tx & 1))) continue;
                    const int ox = S == 2 ? tx >> 1 : tx;
                    if (ox >= c.w_out) continue;
                    a = fmaf(w[ky * 3 + kx], g[(oy << G.lwo) + ox], a);
                }
            }
        }
        float* gp = x.ws + c.gin_off + ((int64_t)s * c.in_ctot + c.in_c0) * HWi + e;
        const float prev = c.gin_accumulate ? *gp : 0.f;
        if (c.in_bn) {
            const float av = F.img[ci * G.PP + (iy + 1) * G.Wp + ix + 1];
            const float dbn = av > 0.f ? a : 0.f;
            const float lbet = F.sh[ci] + F.mean[ci] * F.sc[ci];       // conv.hip: beta from the coefficients
            F.o2[e] = dbn;
            F.o2[FOLD_IN + e] = dbn * ((av - lbet) * (1.f / F.gam[ci]));
            *gp = prev + F.gam[ci] * dbn;
        } else {
            *gp = prev + a;
            if (gin_copy) gin_copy[e] = a;
        }
    }
    if (!c.in_bn) return;
    __syncthreads();
    int gsz;
    const int g = fold_group(x, s, gsz);
    for (int ci = tid >> 4; ci < c.cin; ci += HT / 16) {
        const int part = tid & 15;
        float sd = 0.f, sdx = 0.f;
        for (int p = part; p < HWi; p += 16) {
            sd += F.o2[ci * HWi + p];
            sdx += F.o2[FOLD_IN + ci * HWi + p];
        }
#pragma unroll
        for (int m = 8; m > 0; m >>= 1) {
            sd += __shfl_xor(sd, m, 64);
            sdx += __shfl_xor(sdx, m, 64);
        }
        if (part == 0) {
            if (slab) {
                slab[c.cout * J + ci] = sdx;                 // dgamma partial
                slab[c.cout * J + c.cin + ci] = sd;          // dbeta partial
            }
            gpi_stat* st = x.stats + ((int64_t)(blockIdx.x % GPI_REPLICAS) * GPI_MAX_GROUPS + g) * x.n_stats +
                           c.in_stat + ci;
            const double gm = F.gam[ci];
            atomicAdd(&st->ssum, gm * (double)sd);
            atomicAdd(&st->sxsum, gm * (double)sdx);
        }
    }
}

__device__ __forceinline__ void fold_backward(const gpi_conv_desc& c, const gpi_codec_ctx& x, FoldLds& F, int s,
                                              float* gin_copy) {
    if (c.stride == 2) fold_backward_s<2>(c, x, F, s, gin_copy);
    else fold_backward_s<1>(c, x, F, s, gin_copy);
}

__global__ __launch_bounds__(HT) void head_fwd_kernel(gpi_head_desc d, const float* __restrict__ P, float* ws,
                                                      gpi_head_fold Fd) {
    __shared__ float v0[VMAX], v1[VMAX], v2[VMAX], v3[VMAX];
    __shared__ float scratch[4];
    __shared__ FoldLds FL;
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const bool enc = s < d.n_enc;
    const int q = s - d.n_enc;                  // workspace row over both variational segments
    const QSeg g = qseg(d, q);
    const int dz = d.d_z;
    float* z = v2;

    if (enc) {
        if (d.flags & GPI_HEAD_ENC) {
            if (Fd.has_feat) {
                // the encoder's last conv: its (dropout-scaled) output is this sample's feature row
                fold_stage_params(Fd.feat, Fd.enc_ctx, P, FL, s);
                __syncthreads();
                fold_input_image(Fd.feat, ws, FL, s, nullptr);
                __syncthreads();
                fold_forward(Fd.feat, Fd.enc_ctx, FL, s, v0);
            } else {
                const float* f = ws + d.feat + (int64_t)s * d.d_feat;
                for (int k = tid; k < d.d_feat; k += HT) v0[k] = f[k];
            }
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
        if (Fd.has_lat) {
            // the decoder's first conv on the latent image (its output and batch sums)
            fold_stage_params(Fd.lat, Fd.dec_ctx, P, FL, s);
            __syncthreads();
            fold_input_image(Fd.lat, ws, FL, s, v1);
            __syncthreads();
            fold_forward(Fd.lat, Fd.dec_ctx, FL, s, nullptr);
        }
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
                                                      double* gacc, int s_off, gpi_head_fold Fd) {
    __shared__ float v0[VMAX], v1[VMAX], v2[VMAX], v3[VMAX];
    __shared__ float part[HT];
    __shared__ FoldLds FA, FB;           // the decoder's first conv, the encoder's last conv
    const int s = blockIdx.x + s_off;
    const int tid = threadIdx.x;
    const bool enc = s < d.n_enc;
    const int q = s - d.n_enc;
    const QSeg g = qseg(d, q);
    const int dz = d.d_z;
    float* dz_ = v0;   // dJ/dz
    const bool feat = enc && Fd.has_feat && (d.flags & GPI_HEAD_ENC);

    // the folded convs' parameters, input BN coefficients and batch statistics first: their loads are in
    // flight together (the encoder conv's are consumed at the end)
    if (feat) fold_stage_params(Fd.feat, Fd.enc_ctx, P, FB, s);
    if (Fd.has_lat && (d.flags & GPI_HEAD_LATENT)) {
        const gpi_conv_desc& c = Fd.lat;
        fold_stage_params(c, Fd.dec_ctx, P, FA, s);
        if (tid >= 32 && tid < 32 + c.cout) {          // the output's BN-backward coefficients
            const int co = tid - 32;
            int gsz;
            const int gr = fold_group(Fd.dec_ctx, s, gsz);
            const double n = (double)gsz * c.h_out * c.w_out;
            const int64_t st = c.out_stat + co;
            float mean, inv;
            fold_mean_invstd(fold_stat(Fd.dec_ctx, gr, st, 0), fold_stat(Fd.dec_ctx, gr, st, 1), n, Fd.dec_ctx.bn_eps,
                             mean, inv);
            FA.oc[4 * co] = mean;
            FA.oc[4 * co + 1] = inv;
            FA.oc[4 * co + 2] = (float)(fold_stat(Fd.dec_ctx, gr, st, 2) / n);
            FA.oc[4 * co + 3] = (float)(fold_stat(Fd.dec_ctx, gr, st, 3) / n);
        }
    }
    __syncthreads();
    if (feat) fold_input_image(Fd.feat, ws, FB, s, nullptr);

    // latent map: dz = lat_w^T glat
    if (d.flags & GPI_HEAD_LATENT) {
        if (Fd.has_lat) {
            // the decoder's first conv backward: dY = BN-backward of its output's S, weight-gradient
            // slab row, input gradient = the latent image gradient (stored at glat, and into v1)
            const gpi_conv_desc& c = Fd.lat;
            fold_input_image(c, ws, FA, s, nullptr);
            const int HWo = c.h_out * c.w_out;
            for (int e = tid; e < c.cout * HWo; e += HT) {
                const int co = e / HWo, p = e - co * HWo;
                const int64_t o = ((int64_t)s * c.out_ctot + c.out_c0 + co) * HWo + p;
                const float zv = ws[c.out_off + o], sv = ws[c.gout_off + o];
                const float* oc = FA.oc + 4 * co;
                FA.o[e] = FA.ds[co] * ((sv - oc[2] - ((zv - oc[0]) * oc[1]) * oc[3]) * oc[1]);
            }
            __syncthreads();
            fold_backward(c, Fd.dec_ctx, FA, s, v1);
        } else {
            const float* gl = ws + d.glat + (int64_t)s * d.d_lat;
            for (int j = tid; j < d.d_lat; j += HT) v1[j] = gl[j];
        }
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
    if (feat) {
        // the encoder's last conv backward on its (direct, dropout-scaled) output gradient
        const int HWo = Fd.feat.h_out * Fd.feat.w_out;
        for (int e = tid; e < d.d_feat; e += HT) FB.o[e] = v0[e] * FB.ds[e / HWo];
        __syncthreads();
        fold_backward(Fd.feat, Fd.enc_ctx, FB, s, nullptr);
        return;
    }
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

// the folded convs' shapes (gpi.h gpi_head_fold) and their wiring to the head's buffers
bool pow2(int v) { return v >= 2 && (v & (v - 1)) == 0; }

bool fold_conv_ok(const gpi_conv_desc& c) {
    return c.k == 3 && c.pad == 1 && (c.stride == 1 || c.stride == 2) && !c.upsample && c.cin >= 1 &&
           pow2(c.w_in) && pow2(c.h_in) && pow2(c.w_out) && pow2(c.h_out) &&
           c.cin <= FOLD_CIN && c.cout >= 1 && c.cout <= FOLD_COUT && c.h_in <= FOLD_HW && c.w_in <= FOLD_HW &&
           c.h_out * c.stride == c.h_in && c.w_out * c.stride == c.w_in && c.in_off >= 0;
}

bool fold_ok(const gpi_head_desc* d, const gpi_head_fold* f) {
    if (!f) return true;
    if (f->has_feat) {
        const gpi_conv_desc& c = f->feat;
        if (!fold_conv_ok(c) || !c.in_bn || c.gout_mode != 1 || c.epilogue != GPI_EPI_STORE || c.out_off != d->feat ||
            c.out_c0 != 0 || c.out_ctot != c.cout || c.cout * c.h_out * c.w_out != d->d_feat || !f->enc_ctx.stats ||
            !f->enc_ctx.ws || !(d->flags & GPI_HEAD_ENC))
            return false;
    }
    if (f->has_lat) {
        const gpi_conv_desc& c = f->lat;
        if (!fold_conv_ok(c) || c.in_bn || c.stride != 1 || c.gout_mode != 0 || c.epilogue != GPI_EPI_STORE_STATS ||
            c.out_stat < 0 || c.in_off != d->lat || c.in_c0 != 0 || c.in_ctot != c.cin ||
            c.cin * c.h_in * c.w_in != d->d_lat || (c.gin_off >= 0 && (c.gin_off != d->glat || c.gin_accumulate)) ||
            !f->dec_ctx.stats || !f->dec_ctx.ws || !(d->flags & GPI_HEAD_LATENT))
            return false;
    }
    return true;
}

bool head_ok(const gpi_head_desc* d) {
    return d && d->d_z > 0 && d->d_z <= VMAX && d->d_feat <= VMAX && d->d_lat <= VMAX && d->d_x <= VMAX &&
           d->n_enc >= 0 && d->n_q >= 0 && d->n_q2 >= 0 && (d->n_enc + d->n_q + d->n_q2) > 0 && d->terms &&
           (d->n_q2 == 0 || d->terms2);
}

}  // namespace

extern "C" int gpi_head_forward_folded(const gpi_head_desc* d, const gpi_head_fold* f, const float* params, float* ws,
                                       void* stream) {
    if (!head_ok(d) || !params || !ws) return GPI_ERR_ARG;
    if (!fold_ok(d, f)) return GPI_ERR_UNSUPPORTED;
    gpi_head_fold F{};
    if (f) F = *f;
    hipLaunchKernelGGL(head_fwd_kernel, dim3(d->n_enc + d->n_q + d->n_q2), dim3(HT), 0, (hipStream_t)stream, *d, params, ws,
                       F);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_head_forward(const gpi_head_desc* d, const float* params, float* ws, void* stream) {
    return gpi_head_forward_folded(d, nullptr, params, ws, stream);
}

extern "C" int gpi_head_backward_folded(const gpi_head_desc* d, const gpi_head_fold* f, const float* params, float* ws,
                                        double* gacc, void* stream) {
    if (!head_ok(d) || !params || !ws || !gacc) return GPI_ERR_ARG;
    if (!fold_ok(d, f)) return GPI_ERR_UNSUPPORTED;
    const bool pe = d->flags & GPI_HEAD_PART_ENC, pq = d->flags & GPI_HEAD_PART_Q;
    if (pe && pq) return GPI_ERR_ARG;
    const int nq = d->n_q + d->n_q2;
    const int nb = pe ? d->n_enc : (pq ? nq : d->n_enc + nq), s_off = pq ? d->n_enc : 0;
    if (nb == 0) return GPI_OK;
    gpi_head_fold F{};
    if (f) F = *f;
    hipLaunchKernelGGL(head_bwd_kernel, dim3(nb), dim3(HT), 0, (hipStream_t)stream, *d, params, ws, gacc, s_off, F);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_head_backward(const gpi_head_desc* d, const float* params, float* ws, double* gacc,
                                 void* stream) {
    return gpi_head_backward_folded(d, nullptr, params, ws, gacc, stream);
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
