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

using namespace gpi;

namespace {

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
    const int lane = threadIdx.x;
    for (int k = 0; k < D.nI; ++k) {
        const float dkk = sqrtf(L[k * w]);
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += 64)
            if (k + t < D.nI) L[(k + t) * w + t] /= dkk;
        if (lane == 0) L[k * w] = dkk;
        __syncthreads();
        const int np = D.bw * (D.bw + 1) / 2;
        for (int e = lane; e < np; e += 64) {
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
    const int lane = threadIdx.x;
    for (int k = 0; k < D.nI; ++k) {
        const float yk = b[k] / L[k * w];
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += 64)
            if (k + t < D.nI) b[k + t] -= L[(k + t) * w + t] * yk;
        if (lane == 0) b[k] = yk;
        __syncthreads();
    }
    for (int k = D.nI - 1; k >= 0; --k) {
        const float xk = b[k] / L[k * w];
        __syncthreads();
        for (int t = 1 + lane; t <= D.bw; t += 64)
            if (k - t >= 0) b[k - t] -= L[k * w + t] * xk;
        if (lane == 0) b[k] = xk;
        __syncthreads();
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

__global__ __launch_bounds__(64) void rom_kernel(gpi_rom_desc d, RomDims D) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int w = D.bw + 1;
    float* kp = sm;                   // [nT] kappa
    float* L = kp + D.nT;             // [nI * w]
    float* u = L + D.nI * w;          // [nn]
    float* b = u + D.nn;              // [nI]
    float* lam = b + D.nI;            // [nn]
    double* du = (double*)(sm + ((D.nT + D.nI * w + 2 * D.nn + D.nI + 1) & ~1));   // [nn] fp64 W^T dmu
    const int s = blockIdx.x;
    const int lane = threadIdx.x;
    const int nc = D.nc;
    const float* x = d.x + (int64_t)s * d.x_stride;
    const float* F = d.F + (int64_t)s * D.nn;

    bool bad = false;
    for (int t = lane; t < D.nT; t += 64) {
        const float kv = d.input_kappa ? x[t] : expf(x[t]) + 1e-8f;
        bad |= !(kv > 1e-12f);
        kp[t] = kv;
    }
    if (bad && d.flag) atomicOr(d.flag, 1);
    for (int e = lane; e < D.nn; e += 64) {
        du[e] = (d.mode == GPI_ROM_BACKWARD && d.duc) ? (double)d.duc[(int64_t)s * D.nn + e] : 0.0;
        lam[e] = 0.f;
    }
    __syncthreads();

    // ---- assemble interior system (banded lower) + rhs
    for (int ii = lane; ii < D.nI; ii += 64) {
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
    chol_band(L, D);
    solve_band(L, b, D);
    for (int e = lane; e < D.nn; e += 64) {
        const int I = e % (nc + 1), J = e / (nc + 1);
        u[e] = (I == 0 || I == nc) ? F[e] : b[J * (nc - 1) + (I - 1)];
    }
    __syncthreads();
    if (d.uc) for (int e = lane; e < D.nn; e += 64) d.uc[(int64_t)s * D.nn + e] = u[e];

    // ---- prolongation (+ log-likelihood)
    const int nf = D.n;
    float Lsum = 0.f;
    for (int p = lane; p < D.dy; p += 64) {
        const int j = p / (nf - 1), i = p - j * (nf - 1) + 1;
        int n00, n10, n11;
        float w0, w1, w2;
        interp(i, j, D.r, nc, n00, n10, n11, w0, w1, w2);
        const float mu = w0 * u[n00] + w1 * u[n10] + w2 * u[n11];
        if (d.mu_y) d.mu_y[(int64_t)s * D.dy + p] = mu;
        if (d.mode == GPI_ROM_FORWARD) continue;
        float g;
        if (d.mode == GPI_ROM_LOGLIK) {
            const float ls = d.logsig_y[p];
            const float e = expf(-2.f * ls);
            const float rr = d.Y[(int64_t)s * D.dy + p] - mu;
            Lsum += -0.5f * (2.f * ls + rr * rr * e + GPI_LOG2PI);
            g = -d.loss_scale * rr * e;
            atomicAdd(d.gacc_logsig + p, (double)(d.loss_scale * (1.f - rr * rr * e)));
        } else {
            if (!d.dmu) continue;
            g = d.dmu[(int64_t)s * D.dy + p];
        }
        atomicAdd(&du[n00], (double)(w0 * g));
        atomicAdd(&du[n10], (double)(w1 * g));
        atomicAdd(&du[n11], (double)(w2 * g));
    }
    if (d.mode == GPI_ROM_LOGLIK) {
        Lsum = wave_sum(Lsum);
        if (lane == 0 && d.loss_acc) atomicAdd(d.loss_acc + blockIdx.x % GPI_REPLICAS, (double)Lsum);
    }
    if (d.mode == GPI_ROM_FORWARD) return;
    __syncthreads();

    // ---- adjoint
    for (int ii = lane; ii < D.nI; ii += 64) {
        const int J = ii / (nc - 1), I = ii - J * (nc - 1) + 1;
        b[ii] = (float)du[I + (nc + 1) * J];
    }
    __syncthreads();
    solve_band(L, b, D);
    for (int ii = lane; ii < D.nI; ii += 64) {
        const int J = ii / (nc - 1), I = ii - J * (nc - 1) + 1;
        lam[I + (nc + 1) * J] = b[ii];
    }
    __syncthreads();
    // ---- dJ/dx per coarse triangle
    for (int t = lane; t < D.nT; t += 64) {
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
}

}  // namespace

extern "C" int gpi_rom(const gpi_rom_desc* d, void* stream) {
    if (!d || !d->x || !d->F || d->nc < 2 || d->nc > 12 || d->refine < 1 || d->n < 0) return GPI_ERR_ARG;
    if (d->mode == GPI_ROM_LOGLIK && (!d->Y || !d->logsig_y || !d->gacc_logsig || !d->gx)) return GPI_ERR_ARG;
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
    const size_t lds = sizeof(float) * (D.nT + D.nI * (D.bw + 1) + 4 * D.nn + D.nI + 8);
    hipLaunchKernelGGL(rom_kernel, dim3(d->n), dim3(64), lds, (hipStream_t)stream, *d, D);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
