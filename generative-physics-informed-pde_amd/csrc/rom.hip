// Coarse-grained model (ROM) solve for gfx950: one wave64 per sample.
//
// Reference: ROM.__call__ / GetStiffness / _solve_eqs (bottleneck/ROM.py:59-100)
// builds a dense K(x) = M x^T from the FEniCS tensor M, overwrites the
// Dirichlet rows with identity rows and calls a batched dense LU solve;
// ReducedOrderModelOperator (components.py:296-298) then prolongates with the
// dense P1 matrix W.  Here:
//   * K is the closed-form 5-point stencil of the coarse "/" mesh
//     (physics/grid.py), assembled directly into banded LDS storage;
//   * the Dirichlet nodes are eliminated (u_B = F_B, rhs -= K_IB F_B): the
//     SPD interior system has the same solution as the row-replaced one;
//   * banded Cholesky (bandwidth nc-1) in LDS, no pivoting needed (SPD);
//   * mu_y = W u is evaluated from the closed-form P1 interpolation weights;
//   * LOGLIK mode fuses DiagonalGaussianLogLikelihood(Y, mu_y, 2 logsigma_y)
//     and its adjoint: lambda = K_II^{-1} W^T dmu,
//     dJ/dc_pq = -(lambda_p - lambda_q)(u_p - u_q), dJ/dkappa_t = 1/2 sum over
//     its two legs, dJ/dx = dJ/dkappa * exp(x).
#include "common.h"
#include <stdlib.h>

using namespace gpi;

namespace {

// the log effective property of sample row `row` (x rows at d.x_stride), element t: stored, or drawn here
// from q_X (x_draw: the head's fmaf(expf(logsigma), eps, mu), so both hold the same value)
__device__ __forceinline__ float rom_x(const gpi_rom_desc& d, int64_t row, int t) {
    const int64_t o = row * d.x_stride + t;
    if (d.x_draw) return fmaf(expf(d.x_ls[o]), d.x_eps[o], d.x_mu[o]);
    return d.x[o];
}

// Phase stamps of the timing build (make timing; tools/rom_probe.py): thread 0 of workgroup b writes
// the shader clock at phase boundary i to g_rom_phase[b % 256][i].  Compiled out of the product.
#ifdef GPI_PHASE_TIMING
__device__ unsigned long long g_rom_phase[256 * 8];
#define RPHASE(i)                                                                                       \
    do {                                                                                                \
        if (threadIdx.x == 0) g_rom_phase[(blockIdx.x & 255) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define RPHASE(i) \
    do {          \
    } while (0)
#endif

struct RomDims {
    int nc, nn, nT, nI, bw, n, dy, r;
};

__device__ __forceinline__ float kap(const float* k, int nc, int I, int J, int ul) {
    return k[2 * (I + nc * J) + ul];
}

// horizontal edge (I,J)-(I+1,J)
__device__ __forceinline__ float c_h(const float* k, int nc, int I, int J) {
    float c = 0.f;
    if (J < nc) c += kap(k, nc, I, J, 0);
    if (J > 0) c += kap(k, nc, I, J - 1, 1);
    return 0.5f * c;
}
// vertical edge (I,J)-(I,J+1)
__device__ __forceinline__ float c_v(const float* k, int nc, int I, int J) {
    float c = 0.f;
    if (I > 0) c += kap(k, nc, I - 1, J, 0);
    if (I < nc) c += kap(k, nc, I, J, 1);
    return 0.5f * c;
}

__device__ void chol_band(float* L, const RomDims& D) {
    const int w = D.bw + 1;
    const int lane = threadIdx.x, NT = blockDim.x;
    for (int k = 0; k < D.nI; ++k) {
        const float dkk = sqrtf(L[k * w]);
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += NT)
            if (k + t < D.nI) L[(k + t) * w + t] /= dkk;
        if (lane == 0) L[k * w] = dkk;
        __syncthreads();
        const int np = D.bw * (D.bw + 1) / 2;
        for (int e = lane; e < np; e += NT) {
            // decode e -> (t1 >= t2) in [1, bw]
            int t1 = 1, rem = e;
            while (rem >= t1) { rem -= t1; ++t1; }
            const int t2 = rem + 1;
            const int i = k + t1, j = k + t2;
            if (i < D.nI) L[i * w + (t1 - t2)] -= L[i * w + t1] * L[j * w + t2];
        }
        __syncthreads();
    }
}

// solve L L^T x = b in place (b -> x)
__device__ void solve_band(const float* L, float* b, const RomDims& D) {
    const int w = D.bw + 1;
    const int lane = threadIdx.x, NT = blockDim.x;
    for (int k = 0; k < D.nI; ++k) {
        const float yk = b[k] / L[k * w];
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += NT)
            if (k + t < D.nI) b[k + t] -= L[(k + t) * w + t] * yk;
        if (lane == 0) b[k] = yk;
        __syncthreads();
    }
    for (int k = D.nI - 1; k >= 0; --k) {
        const float xk = b[k] / L[k * w];
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += NT)
            if (k - t >= 0) b[k - t] -= L[k * w + t] * xk;
        if (lane == 0) b[k] = xk;
        __syncthreads();
    }
}

// Single-thread banded Cholesky / solves for the common coarse grids (nc = 4, 8): the band
// is only bw + 1 = nc wide, so the factorisation is a chain of nI dependent sqrt / scale /
// rank-1-update steps.  Run by one lane with the active (bw+1) x (bw+1) window in registers
// and the loop fully unrolled (every window index static: the window shift is register
// renaming), it costs ~40 VALU instructions per step instead of three LDS round trips and
// three workgroup barriers (78 -> ~10 us for the 63-unknown system at nc = 8).
// dinv[k] = 1 / L(k,k) is kept for the solves, which run as partially unrolled loops (a full
// unroll lets the scheduler hoist every band load and spill).
template <int NC>
__device__ __forceinline__ void chol_band_seq(float* __restrict__ L, float* __restrict__ dinv) {
    constexpr int W = NC, NI = (NC - 1) * (NC + 1);
    float win[W][W];   // win[a][t] = L(k + a, k + a - t)
#pragma unroll
    for (int a = 0; a < W; ++a)
#pragma unroll
        for (int t = 0; t < W; ++t) win[a][t] = a < NI ? L[a * W + t] : 0.f;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const float dk = sqrtf(win[0][0]);
        const float inv = 1.f / dk;
        win[0][0] = dk;
        dinv[k] = inv;
#pragma unroll
        for (int a = 1; a < W; ++a) win[a][a] *= inv;                       // L(k+a, k)
#pragma unroll
        for (int a = 1; a < W; ++a)
#pragma unroll
            for (int b = 1; b <= a; ++b) win[a][a - b] = fmaf(-win[a][a], win[b][b], win[a][a - b]);
#pragma unroll
        for (int t = 0; t < W; ++t) L[k * W + t] = win[0][t];
#pragma unroll
        for (int a = 0; a + 1 < W; ++a)
#pragma unroll
            for (int t = 0; t < W; ++t) win[a][t] = win[a + 1][t];
#pragma unroll
        for (int t = 0; t < W; ++t) win[W - 1][t] = (k + W < NI) ? L[(k + W) * W + t] : 0.f;
    }
}

// L L^T x = b in place, single lane (see chol_band_seq)
template <int NC>
__device__ __forceinline__ void solve_band_seq(const float* __restrict__ L, const float* __restrict__ dinv,
                                               float* __restrict__ b) {
    constexpr int BW = NC - 1, W = NC, NI = (NC - 1) * (NC + 1);
    float h[BW];   // sliding window of the last BW solution values (h[t-1] = y[k - t])
#pragma unroll
    for (int t = 0; t < BW; ++t) h[t] = 0.f;
#pragma unroll 8
    for (int k = 0; k < NI; ++k) {
        float a = b[k];
#pragma unroll
        for (int t = 1; t <= BW; ++t)
            if (k - t >= 0) a = fmaf(-L[k * W + t], h[t - 1], a);
        a *= dinv[k];
        b[k] = a;
#pragma unroll
        for (int t = BW - 1; t > 0; --t) h[t] = h[t - 1];
        h[0] = a;
    }
#pragma unroll
    for (int t = 0; t < BW; ++t) h[t] = 0.f;        // h[t-1] = x[k + t]
#pragma unroll 8
    for (int k = NI - 1; k >= 0; --k) {
        float a = b[k];
#pragma unroll
        for (int t = 1; t <= BW; ++t)
            if (k + t < NI) a = fmaf(-L[(k + t) * W + t], h[t - 1], a);
        a *= dinv[k];
        b[k] = a;
#pragma unroll
        for (int t = BW - 1; t > 0; --t) h[t] = h[t - 1];
        h[0] = a;
    }
}

__device__ __forceinline__ void interp(int i, int j, int r, int nc, int& n00, int& n10, int& n11, float& w0,
                                       float& w1, float& w2) {
    int I = i / r, J = j / r;
    if (I > nc - 1) I = nc - 1;
    if (J > nc - 1) J = nc - 1;
    const float xi = (float)(i - I * r) / (float)r, eta = (float)(j - J * r) / (float)r;
    n00 = I + (nc + 1) * J;
    n11 = n00 + (nc + 1) + 1;
    if (xi >= eta) { n10 = n00 + 1; w0 = 1.f - xi; w1 = xi - eta; w2 = eta; }
    else { n10 = n00 + (nc + 1); w0 = 1.f - eta; w1 = eta - xi; w2 = xi; }
}

#ifndef GPI_ROM_NT
#define GPI_ROM_NT 256
#endif
constexpr int ROM_NT = GPI_ROM_NT;   // threads per sample
constexpr int ROM_U = 8;         // fine nodes per batch of global loads
#ifndef GPI_ROM_FAST_NT_DEFAULT
#define GPI_ROM_FAST_NT_DEFAULT 512
#endif

__global__ __launch_bounds__(ROM_NT) void rom_kernel(gpi_rom_desc d, RomDims D) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int w = D.bw + 1;
    float* kp = sm;                   // [nT] kappa
    float* L = kp + D.nT;             // [nI * w]
    float* u = L + D.nI * w;          // [nn]
    float* b = u + D.nn;              // [nI]
    float* lam = b + D.nI;            // [nn]
    double* du = (double*)(sm + ((D.nT + D.nI * w + 2 * D.nn + D.nI + 1) & ~1));   // [nn] fp64 W^T dmu
    double* lred = du + D.nn;         // [ROM_NT / 64] per-wave log-likelihood sums
    float* dinv = (float*)(lred + ROM_NT / 64);   // [nI] 1 / L(k,k) (nc = 4, 8 path)
    const int s = blockIdx.x;
    const int tid = threadIdx.x, NT = ROM_NT;
    const int nc = D.nc;
    const float* F = d.F + (int64_t)s * D.nn;
    RPHASE(0);

    bool bad = false;
    for (int t = tid; t < D.nT; t += NT) {
        const float xv = rom_x(d, s, t);
        const float kv = d.input_kappa ? xv : expf(xv) + 1e-8f;
        bad |= !(kv > 1e-12f);
        kp[t] = kv;
    }
    if (bad && d.flag) atomicOr(d.flag, 1);
    for (int e = tid; e < D.nn; e += NT) {
        du[e] = (d.mode == GPI_ROM_BACKWARD && d.duc) ? (double)d.duc[(int64_t)s * D.nn + e] : 0.0;
        lam[e] = 0.f;
    }
    __syncthreads();

    // ---- assemble interior system (banded lower) + rhs
    for (int ii = tid; ii < D.nI; ii += NT) {
        const int J = ii / (nc - 1), I = ii - J * (nc - 1) + 1;
        const int p = I + (nc + 1) * J;
        const float chl = c_h(kp, nc, I - 1, J), chr = c_h(kp, nc, I, J);
        const float cvd = J > 0 ? c_v(kp, nc, I, J - 1) : 0.f;
        const float cvu = J < nc ? c_v(kp, nc, I, J) : 0.f;
        float* row = L + ii * w;
        for (int t = 0; t < w; ++t) row[t] = 0.f;
        row[0] = chl + chr + cvd + cvu;
        if (I - 1 >= 1) row[1] += -chl;
        if (J >= 1) row[D.bw] += -cvd;
        float rhs = F[p];
        if (I - 1 == 0) rhs += chl * F[p - 1];
        if (I + 1 == nc) rhs += chr * F[p + 1];
        b[ii] = rhs;
    }
    __syncthreads();
    RPHASE(1);
    if (nc == 8 || nc == 4) {
        if (tid == 0) {
            if (nc == 8) { chol_band_seq<8>(L, dinv); solve_band_seq<8>(L, dinv, b); }
            else { chol_band_seq<4>(L, dinv); solve_band_seq<4>(L, dinv, b); }
        }
        __syncthreads();
    } else {
        chol_band(L, D);
        solve_band(L, b, D);
    }
    for (int e = tid; e < D.nn; e += NT) {
        const int I = e % (nc + 1), J = e / (nc + 1);
        u[e] = (I == 0 || I == nc) ? F[e] : b[J * (nc - 1) + (I - 1)];
    }
    __syncthreads();
    RPHASE(2);
    if (d.uc) for (int e = tid; e < D.nn; e += NT) d.uc[(int64_t)s * D.nn + e] = u[e];
    if (d.mode == GPI_ROM_FORWARD && !d.mu_y) return;   // coarse solutions only (VO MC predictive)

    // ---- prolongation (+ log-likelihood, + W^T of the output gradient), by coarse square:
    // four threads share square q = (I, J) and its corner values; each takes every fourth
    // fine free node the square owns (interp()'s partition), loads its Y / logsigma / dmu
    // in batches of ROM_U, and accumulates its W^T contributions to the four corners in
    // registers; one fp64 LDS atomic per corner per square at the end.
    const int nf = D.n, r = D.r;
    const float rinv = 1.f / (float)r;
    float Lsum = 0.f;
    const bool want_g = d.mode == GPI_ROM_LOGLIK || (d.mode == GPI_ROM_BACKWARD && d.dmu);
    for (int qb = 0; qb < nc * nc; qb += NT / 4) {
        const int q = qb + (tid >> 2), sub = tid & 3;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};   // corners v0, v1 (+x), v2 (+y), v3 (+x+y)
        int v0 = 0;
        if (q < nc * nc) {
            const int I = q % nc, J = q / nc;
            v0 = I + (nc + 1) * J;
            const float u0 = u[v0], u1 = u[v0 + 1], u2 = u[v0 + nc + 1], u3 = u[v0 + nc + 2];
            const int i0 = I == 0 ? 1 : I * r, i1 = (I + 1) * r - 1;           // free columns (inclusive)
            const int rows = J == nc - 1 ? r + 1 : r;
            const int ncol = i1 - i0 + 1, total = rows * ncol;
            for (int e0 = sub; e0 < total; e0 += 4 * ROM_U) {
                int pp[ROM_U];
                float yv[ROM_U], lv[ROM_U], gv[ROM_U];
#pragma unroll
                for (int k = 0; k < ROM_U; ++k) {
                    const int e = min(e0 + 4 * k, total - 1);
                    const int jj = e / ncol, ii = e - jj * ncol;
                    pp[k] = (J * r + jj) * (nf - 1) + (i0 + ii - 1);
                }
                if (d.mode == GPI_ROM_LOGLIK) {
#pragma unroll
                    for (int k = 0; k < ROM_U; ++k) {
                        yv[k] = d.Y[(int64_t)s * D.dy + pp[k]];
                        lv[k] = d.logsig_y[pp[k]];
                    }
                } else if (want_g) {
#pragma unroll
                    for (int k = 0; k < ROM_U; ++k) gv[k] = d.dmu[(int64_t)s * D.dy + pp[k]];
                }
#pragma unroll
                for (int k = 0; k < ROM_U; ++k) {
                    const int e = e0 + 4 * k;
                    if (e >= total) break;
                    const int jj = e / ncol, ii = e - jj * ncol;
                    const float xi = (float)(i0 + ii - I * r) * rinv, eta = (float)jj * rinv;
                    float w0, w1, w2, w3;
                    if (xi >= eta) { w0 = 1.f - xi; w1 = xi - eta; w2 = 0.f; w3 = eta; }
                    else { w0 = 1.f - eta; w1 = 0.f; w2 = eta - xi; w3 = xi; }
                    const float mu = w0 * u0 + (w1 * u1 + w2 * u2) + w3 * u3;
                    if (d.mu_y) d.mu_y[(int64_t)s * D.dy + pp[k]] = mu;
                    if (!want_g) continue;
                    float g;
                    if (d.mode == GPI_ROM_LOGLIK) {
                        const float ee = expf(-2.f * lv[k]);
                        const float rr = yv[k] - mu;
                        Lsum += -0.5f * (2.f * lv[k] + rr * rr * ee + GPI_LOG2PI);
                        g = -d.loss_scale * rr * ee;
                        const float gl = d.loss_scale * (1.f - rr * rr * ee);
                        if (d.gls_part) d.gls_part[(int64_t)s * D.dy + pp[k]] = gl;
                        else atomicAdd(d.gacc_logsig + pp[k], (double)gl);
                    } else {
                        g = gv[k];
                    }
                    acc[0] += w0 * g;
                    acc[1] += w1 * g;
                    acc[2] += w2 * g;
                    acc[3] += w3 * g;
                }
            }
        }
        if (want_g) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                acc[c] += __shfl_xor(acc[c], 1, 64);
                acc[c] += __shfl_xor(acc[c], 2, 64);
            }
            if (q < nc * nc && sub == 0) {
                atomicAdd(&du[v0], (double)acc[0]);
                atomicAdd(&du[v0 + 1], (double)acc[1]);
                atomicAdd(&du[v0 + nc + 1], (double)acc[2]);
                atomicAdd(&du[v0 + nc + 2], (double)acc[3]);
            }
        }
    }
    if (d.mode == GPI_ROM_LOGLIK) {
        Lsum = wave_sum(Lsum);
        if ((tid & 63) == 0) lred[tid >> 6] = (double)Lsum;
        __syncthreads();
        if (tid == 0 && d.loss_acc) {
            double t = lred[0];
#pragma unroll
            for (int w = 1; w < ROM_NT / 64; ++w) t += lred[w];
            atomicAdd(d.loss_acc + blockIdx.x % GPI_REPLICAS, t);
        }
    }
    if (d.mode == GPI_ROM_FORWARD) return;
    __syncthreads();
    RPHASE(3);

    // ---- adjoint
    for (int ii = tid; ii < D.nI; ii += NT) {
        const int J = ii / (nc - 1), I = ii - J * (nc - 1) + 1;
        b[ii] = (float)du[I + (nc + 1) * J];
    }
    __syncthreads();
    if (nc == 8 || nc == 4) {
        if (tid == 0) {
            if (nc == 8) solve_band_seq<8>(L, dinv, b);
            else solve_band_seq<4>(L, dinv, b);
        }
        __syncthreads();
    } else {
        solve_band(L, b, D);
    }
    RPHASE(4);
    for (int ii = tid; ii < D.nI; ii += NT) {
        const int J = ii / (nc - 1), I = ii - J * (nc - 1) + 1;
        lam[I + (nc + 1) * J] = b[ii];
    }
    __syncthreads();
    // ---- dJ/dx per coarse triangle
    for (int t = tid; t < D.nT; t += NT) {
        const int q = t >> 1, ul = t & 1;
        const int I = q % nc, J = q / nc;
        const int v0 = I + (nc + 1) * J, v1 = v0 + 1, v2 = v0 + (nc + 1), v3 = v2 + 1;
        float dk;
        if (!ul) {   // legs v0-v1 (bottom), v1-v3 (right)
            dk = -(lam[v0] - lam[v1]) * (u[v0] - u[v1]) - (lam[v1] - lam[v3]) * (u[v1] - u[v3]);
        } else {     // legs v2-v3 (top), v0-v2 (left)
            dk = -(lam[v2] - lam[v3]) * (u[v2] - u[v3]) - (lam[v0] - lam[v2]) * (u[v0] - u[v2]);
        }
        const float g = 0.5f * dk * (d.input_kappa ? 1.f : (kp[t] - 1e-8f));
        float* gp = d.gx + (int64_t)s * d.gx_stride + t;
        *gp = (d.gx_accumulate ? *gp : 0.f) + g;
    }
    RPHASE(5);
}

// ---------------------------------------------------------------------------------------------
// rom_kernel_fast<NC> (nc = 4 / 8, one 256-thread workgroup per sample): the same result as
// rom_kernel with the sequential chains cut (r03 phase stamps of rom_kernel at C64: Cholesky + solve
// 83 k cycles, adjoint solve 55 k, prolongation 19 k of 162 k; 72.8 us per launch):
//   * wave 0 factors K = L L^T and forms Z = L^{-1} in ONE pass (chol_inv_wave): the factorisation runs
//     redundantly in every lane and lane j takes the forward substitution of e_j as each row of L
//     becomes final; u = K^{-1} b and the adjoint lambda = K^{-1} W^T dmu are then Z^T (Z v) mat-vecs
//     over the four waves (kinv_apply) instead of sequential triangular sweeps;
//   * the Y / logsigma_y loads of the prolongation are issued at entry (in flight during the
//     factorisation);
//   * d/dlogsigma_y per sample and node goes to a row of gls_part (plain stores) when given, reduced
//     with the decoder slabs, instead of 4095 same-address fp64 atomics per sample.
// (r03 A/B: a wave-parallel factorisation with rotating window rows and ds_bpermute took 23.7 k cycles,
// the redundant form 13.9 k; 64 independent register solves with v_readlane coefficients 17.5 k for the
// sweeps vs 3.7 k for the two Z mat-vecs.)  21.3 us per launch at C64.

constexpr int KINV_P = 65;     // pitch of the Z = L^{-1} image (conflict-free row and column access)

// Z = L^{-1} (K = L L^T) by ONE wave: every lane runs the same banded factorisation (chol_band_seq's
// register window, the pivot by v_rsq instead of IEEE sqrt + division; the values are uniform, the band
// rows come by broadcast LDS reads) and, as row k of L becomes final at step k, lane j takes
// forward-substitution step k of L y = e_j -- the factorisation instructions serve all 64 right-hand
// sides at once (SIMT: an instruction costs the same with one lane active or 64), no LDS or cross-lane
// traffic in the substitution.  Column j of Z goes to z[k][j] (pitch KINV_P).  Then
// K^{-1} v = Z^T (Z v): two parallel triangular mat-vecs per solve.
template <int NC>
__device__ __forceinline__ void chol_inv_wave(const float* __restrict__ L, float* __restrict__ z) {
    constexpr int W = NC, BW = NC - 1, NI = (NC - 1) * (NC + 1);
    const int j = threadIdx.x & 63;
    float win[W][W];   // win[a][t] = L(k + a, k + a - t)
    float nxt[2][W];   // rows k + W, k + W + 1 (prefetched)
#pragma unroll
    for (int a = 0; a < W; ++a)
#pragma unroll
        for (int t = 0; t < W; ++t) win[a][t] = a < NI ? L[a * W + t] : 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < W; ++t) nxt[u][t] = (W + u < NI) ? L[(W + u) * W + t] : 0.f;
    float h[BW];       // h[t-1] = y[k - t] of this lane's right-hand side e_j
#pragma unroll
    for (int t = 0; t < BW; ++t) h[t] = 0.f;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const float inv = __builtin_amdgcn_rsqf(win[0][0]);
        // forward substitution step k (row k of L is final: L(k, k - t) = win[0][t], 1 / L(k,k) = inv)
        float y = j == k ? 1.f : 0.f, y2 = 0.f;
#pragma unroll
        for (int t = 1; t <= BW; ++t) {
            if (k - t < 0) continue;
            if (t & 1) y = fmaf(-win[0][t], h[t - 1], y);
            else y2 = fmaf(-win[0][t], h[t - 1], y2);
        }
        y = (y + y2) * inv;
        z[k * KINV_P + j] = y;
#pragma unroll
        for (int t = BW - 1; t > 0; --t) h[t] = h[t - 1];
        h[0] = y;
        // factorisation step k
#pragma unroll
        for (int a = 1; a < W; ++a) win[a][a] *= inv;                       // L(k+a, k)
#pragma unroll
        for (int a = 1; a < W; ++a)
#pragma unroll
            for (int b = 1; b <= a; ++b) win[a][a - b] = fmaf(-win[a][a], win[b][b], win[a][a - b]);
#pragma unroll
        for (int a = 0; a + 1 < W; ++a)
#pragma unroll
            for (int t = 0; t < W; ++t) win[a][t] = win[a + 1][t];
#pragma unroll
        for (int t = 0; t < W; ++t) {
            win[W - 1][t] = nxt[0][t];
            nxt[0][t] = nxt[1][t];
            nxt[1][t] = (k + W + 2 < NI) ? L[(k + W + 2) * W + t] : 0.f;
        }
    }
}

// out[i] = (Z^T (Z v))_i = (K^{-1} v)_i for i < NI (v, out in LDS; out may alias v; part: NW x 64 + 64
// floats of scratch).  All NT = 64 NW threads call it: wave p sums the terms k = p (mod NW) of every row
// i = lane (fully unrolled, conflict-free: bank (i + k) mod 64), the NW partial sums meet in LDS (pairwise,
// in a fixed order); three barriers.
template <int NW>
__device__ __forceinline__ float part_sum(const float* part, int i) {
    if constexpr (NW == 4) return (part[i] + part[64 + i]) + (part[128 + i] + part[192 + i]);
    else return part_sum<NW / 2>(part, i) + part_sum<NW / 2>(part + 64 * (NW / 2), i);
}

template <int NC, int NT>
__device__ __forceinline__ void kinv_apply(const float* __restrict__ z, const float* v, float* part, float* out) {
    constexpr int NW = NT / 64, NI = (NC - 1) * (NC + 1), NM = (NI + NW - 1) / NW;
    const int i = threadIdx.x & 63, p = threadIdx.x >> 6;
    float a = 0.f;
#pragma unroll
    for (int m = 0; m < NM; ++m) {            // (Z v)_i = sum_{k <= i} Z[i][k] v_k
        const int k = NW * m + p;
        if (k < NI) a = fmaf((k <= i && i < NI) ? z[i * KINV_P + k] : 0.f, v[k], a);
    }
    part[p * 64 + i] = a;
    __syncthreads();
    float* w = part + 64 * NW;                // (Z v), 64 floats
    if (threadIdx.x < 64) w[i] = part_sum<NW>(part, i);
    __syncthreads();
    a = 0.f;
#pragma unroll
    for (int m = 0; m < NM; ++m) {            // (Z^T w)_i = sum_{k >= i} Z[k][i] w_k
        const int k = NW * m + p;
        if (k < NI) a = fmaf((k >= i && i < NI) ? z[k * KINV_P + i] : 0.f, w[k], a);
    }
    part[p * 64 + i] = a;
    __syncthreads();
    if (threadIdx.x < NI) out[i] = part_sum<NW>(part, i);
    __syncthreads();
}

// NT threads per sample (256 / 512 / 1024): SUB = NT / 64 threads share one coarse square of the
// prolongation (nc = 8: 64 squares; nc = 4 uses 16 of them), so a wider workgroup has more waves in flight
// over the 4095 fine nodes; the factorisation stays in wave 0.
template <int NC, int NT>
__global__ __launch_bounds__(NT) void rom_kernel_fast(gpi_rom_desc d, RomDims D) {
    constexpr int W = NC, BW = NC - 1, NI = (NC - 1) * (NC + 1), NN = (NC + 1) * (NC + 1), NT2 = 2 * NC * NC;
    constexpr int SUB = NT / 64, NW = NT / 64;
    constexpr int PF = (SUB >= 8 ? 1 : 3) * ROM_U;   // prefetched fine nodes per thread (a square holds <= (r+1) r)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* kp = sm;                   // [NT2] kappa
    float* L = kp + NT2;              // [NI * W]
    float* u = L + NI * W;            // [NN]
    float* b = u + NN;                // [NI]
    float* lam = b + NI;              // [NN]
    float* dinv = lam + NN;           // [NI]
    float* kinv = dinv + NI;          // [NI][KINV_P]: Z = L^{-1}
    float* part = kinv + NI * KINV_P; // [64 NW + 64] kinv_apply scratch
    double* du = (double*)(sm + ((NT2 + NI * W + 2 * NN + 2 * NI + NI * KINV_P + 64 * NW + 64 + 1) & ~1));   // [NN]
    double* lred = du + NN;           // [NW]
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const float* F = d.F + (int64_t)s * NN;
    const int nf = D.n, r = D.r;
    RPHASE(0);

    // ---- entry: every global read in flight (kappa, F, and this thread's first PF fine nodes)
    const int q0 = tid / SUB, sub = tid & (SUB - 1);
    float ypf[PF], lpf[PF];
    {
        const bool okq = q0 < NC * NC && d.mode == GPI_ROM_LOGLIK;
        const int I = q0 % NC, J = q0 / NC;
        const int i0 = I == 0 ? 1 : I * r, i1 = (I + 1) * r - 1;
        const int rows = J == NC - 1 ? r + 1 : r;
        const int ncol = i1 - i0 + 1, total = rows * ncol;
        const uint32_t mcol = (ncol > 1 ? (uint32_t)(((1ull << 32) + ncol - 1) / ncol) : 0u);   // e / ncol = umulhi(e, mcol), e < 2^16
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int e = sub + SUB * k;
            const bool ok = okq && e < total;
            const int jj = ok ? (mcol ? (int)__umulhi((uint32_t)e, mcol) : e) : 0, ii = ok ? e - jj * ncol : 0;
            const int pp = (J * r + jj) * (nf - 1) + (i0 + ii - 1);
            ypf[k] = ok ? d.Y[(int64_t)s * D.dy + pp] : 0.f;
            lpf[k] = ok ? d.logsig_y[pp] : 0.f;
        }
    }
    bool bad = false;
    for (int t = tid; t < NT2; t += NT) {
        const float xv = rom_x(d, s, t);
        const float kv = d.input_kappa ? xv : expf(xv) + 1e-8f;
        bad |= !(kv > 1e-12f);
        kp[t] = kv;
    }
    if (bad && d.flag) atomicOr(d.flag, 1);
    for (int e = tid; e < NN; e += NT) {
        du[e] = (d.mode == GPI_ROM_BACKWARD && d.duc) ? (double)d.duc[(int64_t)s * NN + e] : 0.0;
        lam[e] = 0.f;
    }
    __syncthreads();
    // ---- assemble the interior system (banded lower) + rhs
    for (int ii = tid; ii < NI; ii += NT) {
        const int J = ii / (NC - 1), I = ii - J * (NC - 1) + 1;
        const int p = I + (NC + 1) * J;
        const float chl = c_h(kp, NC, I - 1, J), chr = c_h(kp, NC, I, J);
        const float cvd = J > 0 ? c_v(kp, NC, I, J - 1) : 0.f;
        const float cvu = J < NC ? c_v(kp, NC, I, J) : 0.f;
        float* row = L + ii * W;
#pragma unroll
        for (int t = 0; t < W; ++t) row[t] = 0.f;
        row[0] = chl + chr + cvd + cvu;
        if (I - 1 >= 1) row[1] += -chl;
        if (J >= 1) row[BW] += -cvd;
        float rhs = F[p];
        if (I - 1 == 0) rhs += chl * F[p - 1];
        if (I + 1 == NC) rhs += chr * F[p + 1];
        b[ii] = rhs;
    }
    __syncthreads();
    RPHASE(1);
    // the prefetched Y / logsigma_y values in registers from here on (issued at entry, they arrived with
    // kappa and F): otherwise the compiler sinks the loads to the prolongation, a round trip there
#pragma unroll
    for (int k = 0; k < PF; ++k) asm volatile("" : : "v"(ypf[k]), "v"(lpf[k]));
    static_assert(NC * NC <= 64, "window per wave");
    // every lane of wave 0: the factorisation (uniform) + forward substitution of e_lane -> Z = L^{-1}
    if (tid < 64) chol_inv_wave<NC>(L, kinv);
    RPHASE(6);
    __syncthreads();
    // interior coarse solution u_I = K^{-1} b = Z^T (Z b), in place of b
    kinv_apply<NC, NT>(kinv, b, part, b);
    RPHASE(2);
    for (int e = tid; e < NN; e += NT) {
        const int I = e % (NC + 1), J = e / (NC + 1);
        u[e] = (I == 0 || I == NC) ? F[e] : b[J * (NC - 1) + (I - 1)];
    }
    __syncthreads();
    if (d.uc) for (int e = tid; e < NN; e += NT) d.uc[(int64_t)s * NN + e] = u[e];

    // ---- prolongation (+ log-likelihood, + W^T of the output gradient), as rom_kernel; the first
    // PF nodes of every thread's square from the entry prefetch
    const float rinv = 1.f / (float)r;
    float Lsum = 0.f;
    const bool want_g = d.mode == GPI_ROM_LOGLIK || (d.mode == GPI_ROM_BACKWARD && d.dmu);
    for (int qb = 0; qb < NC * NC; qb += NT / SUB) {
        const int q = qb + q0;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        int v0 = 0;
        if (q < NC * NC) {
            const int I = q % NC, J = q / NC;
            v0 = I + (NC + 1) * J;
            const float u0 = u[v0], u1 = u[v0 + 1], u2 = u[v0 + NC + 1], u3 = u[v0 + NC + 2];
            const int i0 = I == 0 ? 1 : I * r, i1 = (I + 1) * r - 1;
            const int rows = J == NC - 1 ? r + 1 : r;
            const int ncol = i1 - i0 + 1, total = rows * ncol;
            const uint32_t mcol = (ncol > 1 ? (uint32_t)(((1ull << 32) + ncol - 1) / ncol) : 0u);
            for (int e0 = sub; e0 < total; e0 += SUB * ROM_U) {
                const int bi = (e0 - sub) / (SUB * ROM_U);
                const bool pre = qb == 0 && bi < PF / ROM_U;
                int pp[ROM_U];
                float yv[ROM_U], lv[ROM_U], gv[ROM_U];
#pragma unroll
                for (int k = 0; k < ROM_U; ++k) {
                    const int e = min(e0 + SUB * k, total - 1);
                    const int jj = (mcol ? (int)__umulhi((uint32_t)e, mcol) : e), ii = e - jj * ncol;
                    pp[k] = (J * r + jj) * (nf - 1) + (i0 + ii - 1);
                }
                if (d.mode == GPI_ROM_LOGLIK) {
                    if (pre) {
#pragma unroll
                        for (int k = 0; k < ROM_U; ++k) {
                            if constexpr (PF == ROM_U) {
                                yv[k] = ypf[k];
                                lv[k] = lpf[k];
                            } else {
                                yv[k] = bi == 0 ? ypf[k] : (bi == 1 ? ypf[ROM_U + k] : ypf[2 * ROM_U + k]);
                                lv[k] = bi == 0 ? lpf[k] : (bi == 1 ? lpf[ROM_U + k] : lpf[2 * ROM_U + k]);
                            }
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < ROM_U; ++k) {
                            yv[k] = d.Y[(int64_t)s * D.dy + pp[k]];
                            lv[k] = d.logsig_y[pp[k]];
                        }
                    }
                } else if (want_g) {
#pragma unroll
                    for (int k = 0; k < ROM_U; ++k) gv[k] = d.dmu[(int64_t)s * D.dy + pp[k]];
                }
#pragma unroll
                for (int k = 0; k < ROM_U; ++k) {
                    const int e = e0 + SUB * k;
                    if (e >= total) break;
                    const int jj = (mcol ? (int)__umulhi((uint32_t)e, mcol) : e), ii = e - jj * ncol;
                    const float xi = (float)(i0 + ii - I * r) * rinv, eta = (float)jj * rinv;
                    float w0, w1, w2, w3;
                    if (xi >= eta) { w0 = 1.f - xi; w1 = xi - eta; w2 = 0.f; w3 = eta; }
                    else { w0 = 1.f - eta; w1 = 0.f; w2 = eta - xi; w3 = xi; }
                    const float mu = w0 * u0 + (w1 * u1 + w2 * u2) + w3 * u3;
                    if (d.mu_y) d.mu_y[(int64_t)s * D.dy + pp[k]] = mu;
                    if (!want_g) continue;
                    float g;
                    if (d.mode == GPI_ROM_LOGLIK) {
                        const float ee = expf(-2.f * lv[k]);
                        const float rr = yv[k] - mu;
                        Lsum += -0.5f * (2.f * lv[k] + rr * rr * ee + GPI_LOG2PI);
                        g = -d.loss_scale * rr * ee;
                        const float gl = d.loss_scale * (1.f - rr * rr * ee);
                        if (d.gls_part) d.gls_part[(int64_t)s * D.dy + pp[k]] = gl;
                        else atomicAdd(d.gacc_logsig + pp[k], (double)gl);
                    } else {
                        g = gv[k];
                    }
                    acc[0] += w0 * g;
                    acc[1] += w1 * g;
                    acc[2] += w2 * g;
                    acc[3] += w3 * g;
                }
            }
        }
        if (want_g) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int o = 1; o < SUB; o <<= 1) acc[c] += __shfl_xor(acc[c], o, 64);
            if (q < NC * NC && sub == 0) {
                atomicAdd(&du[v0], (double)acc[0]);
                atomicAdd(&du[v0 + 1], (double)acc[1]);
                atomicAdd(&du[v0 + NC + 1], (double)acc[2]);
                atomicAdd(&du[v0 + NC + 2], (double)acc[3]);
            }
        }
    }
    RPHASE(7);
    if (d.mode == GPI_ROM_LOGLIK) {
        Lsum = wave_sum(Lsum);
        if ((tid & 63) == 0) lred[tid >> 6] = (double)Lsum;
        __syncthreads();
        if (tid == 0 && d.loss_acc) {
            double t = lred[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) t += lred[w];
            atomicAdd(d.loss_acc + blockIdx.x % GPI_REPLICAS, t);
        }
    }
    if (d.mode == GPI_ROM_FORWARD) return;
    __syncthreads();
    RPHASE(3);
    // ---- adjoint lambda = K^{-1} (W^T dmu)_interior = Z^T (Z r)
    for (int ii = tid; ii < NI; ii += NT) {
        const int J = ii / (NC - 1), I = ii - J * (NC - 1) + 1;
        b[ii] = (float)du[I + (NC + 1) * J];
    }
    __syncthreads();
    kinv_apply<NC, NT>(kinv, b, part, b);
    for (int ii = tid; ii < NI; ii += NT) {
        const int J = ii / (NC - 1), I = ii - J * (NC - 1) + 1;
        lam[I + (NC + 1) * J] = b[ii];
    }
    __syncthreads();
    RPHASE(4);
    // ---- dJ/dx per coarse triangle
    for (int t = tid; t < NT2; t += NT) {
        const int q = t >> 1, ul = t & 1;
        const int I = q % NC, J = q / NC;
        const int v0 = I + (NC + 1) * J, v1 = v0 + 1, v2 = v0 + (NC + 1), v3 = v2 + 1;
        float dk;
        if (!ul) dk = -(lam[v0] - lam[v1]) * (u[v0] - u[v1]) - (lam[v1] - lam[v3]) * (u[v1] - u[v3]);
        else dk = -(lam[v2] - lam[v3]) * (u[v2] - u[v3]) - (lam[v0] - lam[v2]) * (u[v0] - u[v2]);
        const float g = 0.5f * dk * (d.input_kappa ? 1.f : (kp[t] - 1e-8f));
        float* gp = d.gx + (int64_t)s * d.gx_stride + t;
        *gp = (d.gx_accumulate ? *gp : 0.f) + g;
    }
    RPHASE(5);
}

template <int NC, int NT>
size_t rom_fast_lds() {
    constexpr int W = NC, NI = (NC - 1) * (NC + 1), NN = (NC + 1) * (NC + 1), NT2 = 2 * NC * NC, NW = NT / 64;
    const size_t fl = ((NT2 + NI * W + 2 * NN + 2 * NI + NI * KINV_P + 64 * NW + 64 + 1) & ~1);
    return sizeof(float) * fl + sizeof(double) * (NN + NW);
}

// Coarse solutions only (FORWARD without mu_y: the VO MC predictive, N_vo x N_mc samples), nc = 4 / 8:
// ONE LANE PER SAMPLE.  rom_kernel runs the banded Cholesky in one lane of a 256-thread workgroup per
// sample; here every lane of a wave64 factors its own sample's system with the same register window
// (chol_band_seq), the forward substitution fused into the factorisation (row k of L is final when
// the window reaches it) and the band rows / right-hand side in LDS interleaved by lane ([entry][64]:
// conflict-free).  Slot 0 of each stored L row holds 1 / L(k,k).
template <int NC>
__global__ __launch_bounds__(64) void rom_lane_kernel(gpi_rom_desc d) {
    constexpr int W = NC, BW = NC - 1, NI = (NC - 1) * (NC + 1), NN = (NC + 1) * (NC + 1);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Ls = sm;                       // [NI * W][64]
    float* Bs = sm + NI * W * 64;         // [NI][64]
    const int lane = threadIdx.x;
    const int s = blockIdx.x * 64 + lane;
    const bool act = s < d.n;
    const int sc = act ? s : 0;
    const float* __restrict__ F = d.F + (int64_t)sc * NN;
    auto kap = [&](int I, int J, int ul) -> float {
        const float v = rom_x(d, sc, 2 * (I + NC * J) + ul);
        return d.input_kappa ? v : expf(v) + 1e-8f;
    };
    auto ch = [&](int I, int J) -> float {        // horizontal edge (I,J)-(I+1,J)
        float c = 0.f;
        if (J < NC) c += kap(I, J, 0);
        if (J > 0) c += kap(I, J - 1, 1);
        return 0.5f * c;
    };
    auto cv = [&](int I, int J) -> float {        // vertical edge (I,J)-(I,J+1)
        float c = 0.f;
        if (I > 0) c += kap(I - 1, J, 0);
        if (I < NC) c += kap(I, J, 1);
        return 0.5f * c;
    };
    bool bad = false;
#pragma unroll
    for (int t = 0; t < 2 * NC * NC; ++t) {
        const float v = rom_x(d, sc, t);
        bad |= !((d.input_kappa ? v : expf(v) + 1e-8f) > 1e-12f);
    }
    if (act && bad && d.flag) atomicOr(d.flag, 1);
    // ---- assemble the interior rows (banded lower) + rhs
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int J = k / (NC - 1), I = k - J * (NC - 1) + 1, p = I + (NC + 1) * J;
        const float chl = ch(I - 1, J), chr = ch(I, J);
        const float cvd = J > 0 ? cv(I, J - 1) : 0.f, cvu = J < NC ? cv(I, J) : 0.f;
#pragma unroll
        for (int t = 0; t < W; ++t) {
            float v = 0.f;
            if (t == 0) v = chl + chr + cvd + cvu;
            if (t == 1 && I - 1 >= 1) v += -chl;
            if (t == BW && J >= 1) v += -cvd;
            Ls[(k * W + t) * 64 + lane] = v;
        }
        float rhs = F[p];
        if (I - 1 == 0) rhs += chl * F[p - 1];
        if (I + 1 == NC) rhs += chr * F[p + 1];
        Bs[k * 64 + lane] = rhs;
    }
    // ---- factorisation + forward substitution (register window, see chol_band_seq)
    float win[W][W];   // win[a][t] = L(k + a, k + a - t)
    float h[BW];       // h[t-1] = y[k - t]
#pragma unroll
    for (int a = 0; a < W; ++a)
#pragma unroll
        for (int t = 0; t < W; ++t) win[a][t] = a < NI ? Ls[(a * W + t) * 64 + lane] : 0.f;
#pragma unroll
    for (int t = 0; t < BW; ++t) h[t] = 0.f;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const float dk = sqrtf(win[0][0]);
        const float inv = 1.f / dk;
#pragma unroll
        for (int a = 1; a < W; ++a) win[a][a] *= inv;                       // L(k+a, k)
#pragma unroll
        for (int a = 1; a < W; ++a)
#pragma unroll
            for (int b = 1; b <= a; ++b) win[a][a - b] = fmaf(-win[a][a], win[b][b], win[a][a - b]);
        float y = Bs[k * 64 + lane];
#pragma unroll
        for (int t = 1; t <= BW; ++t)
            if (k - t >= 0) y = fmaf(-win[0][t], h[t - 1], y);
        y *= inv;
        Bs[k * 64 + lane] = y;
#pragma unroll
        for (int t = BW - 1; t > 0; --t) h[t] = h[t - 1];
        h[0] = y;
        Ls[(k * W) * 64 + lane] = inv;
#pragma unroll
        for (int t = 1; t < W; ++t) Ls[(k * W + t) * 64 + lane] = win[0][t];
#pragma unroll
        for (int a = 0; a + 1 < W; ++a)
#pragma unroll
            for (int t = 0; t < W; ++t) win[a][t] = win[a + 1][t];
#pragma unroll
        for (int t = 0; t < W; ++t) win[W - 1][t] = (k + W < NI) ? Ls[((k + W) * W + t) * 64 + lane] : 0.f;
    }
    // ---- back substitution L^T x = y
#pragma unroll
    for (int t = 0; t < BW; ++t) h[t] = 0.f;        // h[t-1] = x[k + t]
#pragma unroll
    for (int k = NI - 1; k >= 0; --k) {
        float a = Bs[k * 64 + lane];
#pragma unroll
        for (int t = 1; t <= BW; ++t)
            if (k + t < NI) a = fmaf(-Ls[((k + t) * W + t) * 64 + lane], h[t - 1], a);
        a *= Ls[(k * W) * 64 + lane];
        Bs[k * 64 + lane] = a;
#pragma unroll
        for (int t = BW - 1; t > 0; --t) h[t] = h[t - 1];
        h[0] = a;
    }
    if (!act) return;
    float* uc = d.uc + (int64_t)s * NN;
#pragma unroll
    for (int e = 0; e < NN; ++e) {
        const int I = e % (NC + 1), J = e / (NC + 1);
        uc[e] = (I == 0 || I == NC) ? F[e] : Bs[(J * (NC - 1) + (I - 1)) * 64 + lane];
    }
}

}  // namespace

#ifdef GPI_PHASE_TIMING
// timing build only (not declared in gpi.h): copy the ROM phase stamps out and clear them
extern "C" int gpi_debug_rom_stamps(unsigned long long* out) {
    static unsigned long long zeros[256 * 8];
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rom_phase), sizeof(zeros)) != hipSuccess) return GPI_ERR_LAUNCH;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rom_phase), zeros, sizeof(zeros)) != hipSuccess) return GPI_ERR_LAUNCH;
    return GPI_OK;
}
#endif

extern "C" int gpi_rom(const gpi_rom_desc* d, void* stream) {
    if (!d || !d->x || !d->F || d->nc < 2 || d->nc > 12 || d->refine < 1 || d->n < 0) return GPI_ERR_ARG;
    if (d->mode == GPI_ROM_LOGLIK && (!d->Y || !d->logsig_y || (!d->gacc_logsig && !d->gls_part) || !d->gx))
        return GPI_ERR_ARG;
    if (d->mode == GPI_ROM_BACKWARD && ((!d->dmu && !d->duc) || !d->gx)) return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    RomDims D;
    D.nc = d->nc;
    D.nn = (d->nc + 1) * (d->nc + 1);
    D.nT = 2 * d->nc * d->nc;
    D.nI = (d->nc - 1) * (d->nc + 1);
    D.bw = d->nc - 1;
    D.r = d->refine;
    D.n = d->nc * d->refine;
    D.dy = (D.n + 1) * (D.n - 1);
    if (d->mode == GPI_ROM_FORWARD && !d->mu_y && d->uc && (d->nc == 4 || d->nc == 8)) {
        const size_t lds = sizeof(float) * 64 * (D.nI * (D.bw + 1) + D.nI);
        const void* k = d->nc == 8 ? (const void*)rom_lane_kernel<8> : (const void*)rom_lane_kernel<4>;
        if (lds > 64 * 1024 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return GPI_ERR_LAUNCH;
        const dim3 grid((d->n + 63) / 64);
        if (d->nc == 8) hipLaunchKernelGGL(rom_lane_kernel<8>, grid, dim3(64), lds, (hipStream_t)stream, *d);
        else hipLaunchKernelGGL(rom_lane_kernel<4>, grid, dim3(64), lds, (hipStream_t)stream, *d);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    static const bool slow = getenv("GPI_ROM_SLOW") && atoi(getenv("GPI_ROM_SLOW"));   // A/B: the r02 kernel
    if ((d->nc == 8 || d->nc == 4) && !slow) {
        // nc = 8: the workgroup width (GPI_ROM_FAST_NT = 256 / 512 / 1024; r03 A/B in DESIGN.md)
        static const int fnt = getenv("GPI_ROM_FAST_NT") ? atoi(getenv("GPI_ROM_FAST_NT")) : GPI_ROM_FAST_NT_DEFAULT;
        const size_t lds_8_1024 = rom_fast_lds<8, 1024>(), lds_8_512 = rom_fast_lds<8, 512>();
        const size_t lds_8_256 = rom_fast_lds<8, 256>(), lds_4_256 = rom_fast_lds<4, 256>();
        if (d->nc == 8 && fnt == 1024)
            hipLaunchKernelGGL((rom_kernel_fast<8, 1024>), dim3(d->n), dim3(1024), lds_8_1024, (hipStream_t)stream, *d, D);
        else if (d->nc == 8 && fnt == 512)
            hipLaunchKernelGGL((rom_kernel_fast<8, 512>), dim3(d->n), dim3(512), lds_8_512, (hipStream_t)stream, *d, D);
        else if (d->nc == 8)
            hipLaunchKernelGGL((rom_kernel_fast<8, 256>), dim3(d->n), dim3(256), lds_8_256, (hipStream_t)stream, *d, D);
        else
            hipLaunchKernelGGL((rom_kernel_fast<4, 256>), dim3(d->n), dim3(256), lds_4_256, (hipStream_t)stream, *d, D);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    const size_t lds = sizeof(float) * (D.nT + D.nI * (D.bw + 1) + 4 * D.nn + 2 * D.nI + 2 * (ROM_NT / 64) + 4);
    hipLaunchKernelGGL(rom_kernel, dim3(d->n), dim3(ROM_NT), lds, (hipStream_t)stream, *d, D);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
