// Virtual observables (bottleneck/VirtualObservables.py) for gfx950.
//
// Reference: per VO sample, FEniCS assembles K_ff / f_eff once
// (QuerryPoint._assemble_system, VirtualObservables.py:57-59), the CGR sampler
// forms W^T K_ff and W^T f_eff densely with numpy (:61-69,297-321), the flux
// sampler runs one FEniCS facet assembly per coarse cell (flux.py:81-158); the
// MC predictive runs the ROM once per VO sample in a Python loop
// (generative.py:198-207) and the conditioning is a torch fp64 Cholesky per
// VO sample in another Python loop (VirtualObservables.py:642-669,891-898).
// Here every step is one batched launch over all VO samples:
//   vo_query_columns / vo_query_flux  Gamma, alpha from the closed-form P1 stencil
//                                     (one thread per fine free node = Gamma column)
//   vo_moments_kernel                 MC mean / std of W u_s + sigma eps from the
//                                     coarse ROM solutions (no [n_mc, d_y] sample matrix)
//   vo_lambda_kernel                  Lambda = Gamma C Gamma^T + diag(v), 32x32 fp64 tiles
//   vo_chol_kernel                    Cholesky + (Gamma g - alpha) + solve, one workgroup per sample
//   vo_linv_kernel                    L^-1 (into lam's upper triangle)
//   vo_columns_kernel                 posterior mean / variance per column (|L^-1 Gamma_i|^2, blocked GEMM)
//   vo_precision_kernel               beta / mean VO variances (deterministic row reductions)
#include "common.h"

using namespace gpi;

namespace {

// ---------------------------------------------------------------- fine grid helpers
struct FineGrid {
    int n, nc, r, dy, nn_c, nT_c;
};

__device__ __forceinline__ double kcell(const double* lk, int n, int i, int j, int ul) {
    return exp(lk[2 * (i + n * j) + ul]);
}
// conductance of the horizontal edge (i,j)-(i+1,j): the lower-right triangle of square (i,j)
// and the upper-left triangle of square (i,j-1) (P1 on right triangles: -1/2 kappa per leg)
__device__ __forceinline__ double ch_(const double* lk, int n, int i, int j) {
    double c = 0.0;
    if (j < n) c += kcell(lk, n, i, j, 0);
    if (j > 0) c += kcell(lk, n, i, j - 1, 1);
    return 0.5 * c;
}
// vertical edge (i,j)-(i,j+1): upper-left of square (i,j), lower-right of square (i-1,j)
__device__ __forceinline__ double cv_(const double* lk, int n, int i, int j) {
    double c = 0.0;
    if (i < n) c += kcell(lk, n, i, j, 1);
    if (i > 0) c += kcell(lk, n, i - 1, j, 0);
    return 0.5 * c;
}

// P1 prolongation weights of fine node (i,j) onto the coarse "/" mesh (components.py:42-60)
__device__ __forceinline__ void interp_w(int i, int j, int r, int nc, int (&k)[3], double (&w)[3]) {
    int I = i / r, J = j / r;
    if (I > nc - 1) I = nc - 1;
    if (J > nc - 1) J = nc - 1;
    const double xi = (double)(i - I * r) / (double)r, eta = (double)(j - J * r) / (double)r;
    const int n00 = I + (nc + 1) * J;
    k[0] = n00;
    k[2] = n00 + (nc + 1) + 1;
    if (xi >= eta) { k[1] = n00 + 1; w[0] = 1.0 - xi; w[1] = xi - eta; w[2] = eta; }
    else { k[1] = n00 + (nc + 1); w[0] = 1.0 - eta; w[1] = eta - xi; w[2] = xi; }
}

__device__ __forceinline__ double bc_value(const double* u, int i, int j, int n) {
    const double y = (double)j / (double)n;
    return i == 0 ? u[0] * (1.0 - y) + u[1] * y : u[2] * (1.0 - y) + u[3] * y;
}

constexpr int NZ = 16;   // nonzeros of one CGR column: 5 stencil nodes x 3 coarse weights

struct SparseCol {
    int k[NZ];
    double v[NZ];
    int n;
    __device__ void add(int kk, double vv) {
        for (int t = 0; t < n; ++t)
            if (k[t] == kk) { v[t] += vv; return; }
        if (n < NZ) { k[n] = kk; v[n] = vv; ++n; }
    }
};

// Gamma column of fine free node p (all rows; flux rows zero here, added by vo_query_flux)
// and, in workgroup 0 of each field, alpha.
__global__ __launch_bounds__(256) void vo_query_columns(gpi_vo_query_desc d, FineGrid G, int m) {
    extern __shared__ __attribute__((aligned(16))) double sacc[];   // [nn_c]
    const int f = blockIdx.y;
    const int n = G.n, nc = G.nc, r = G.r;
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    double* gam = d.gamma + (int64_t)f * m * G.dy;
    const bool cgr = d.flags & GPI_VO_CGR;
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < G.dy) {
        const int jj = p / (n - 1), ii = p - jj * (n - 1) + 1;
        SparseCol col;
        col.n = 0;
        if (cgr) {
            const double chl = ch_(lk, n, ii - 1, jj), chr = ch_(lk, n, ii, jj);
            const double cvd = jj > 0 ? cv_(lk, n, ii, jj - 1) : 0.0;
            const double cvu = jj < n ? cv_(lk, n, ii, jj) : 0.0;
            // column i of K_ff: K[j, i] for the free nodes j of the 5-point star
            const int ni[5] = {ii, ii - 1, ii + 1, ii, ii};
            const int nj[5] = {jj, jj, jj, jj - 1, jj + 1};
            const double kv[5] = {chl + chr + cvd + cvu, -chl, -chr, -cvd, -cvu};
            for (int t = 0; t < 5; ++t) {
                const int a = ni[t], b = nj[t];
                if (a < 1 || a > n - 1 || b < 0 || b > n) continue;
                if (t >= 3 && kv[t] == 0.0) continue;
                int kk[3];
                double w[3];
                interp_w(a, b, r, nc, kk, w);
                for (int c = 0; c < 3; ++c)
                    if (w[c] != 0.0) col.add(kk[c], w[c] * kv[t]);
            }
        }
        for (int row = 0; row < m; ++row) {
            double v = 0.0;
            for (int t = 0; t < col.n; ++t) v = col.k[t] == row ? col.v[t] : v;
            gam[(int64_t)row * G.dy + p] = v;
        }
    }
    if (blockIdx.x != 0) return;
    // alpha: W^T f_eff, f_eff[j] = sum over the Dirichlet neighbours c of j of c_jc g_c (zero source)
    const int m_cgr = cgr ? G.nn_c : 0;
    for (int e = threadIdx.x; e < G.nn_c; e += 256) sacc[e] = 0.0;
    __syncthreads();
    if (cgr) {
        const double* u = d.bc + 4 * f;
        for (int e = threadIdx.x; e < 2 * (n + 1); e += 256) {
            const int side = e / (n + 1), jj = e - side * (n + 1);
            const int ii = side == 0 ? 1 : n - 1;
            const int ic = side == 0 ? 0 : n;
            const double c = ch_(lk, n, side == 0 ? 0 : n - 1, jj);
            double fe = c * bc_value(u, ic, jj, n);
            if (n == 2) {   // a single interior column touches both sides
                if (side == 1) continue;
                fe += ch_(lk, n, n - 1, jj) * bc_value(u, n, jj, n);
            }
            int kk[3];
            double w[3];
            interp_w(ii, jj, r, nc, kk, w);
            for (int t = 0; t < 3; ++t)
                if (w[t] != 0.0) atomicAdd(&sacc[kk[t]], w[t] * fe);
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < m; e += 256) d.alpha[(int64_t)f * m + e] = e < m_cgr ? sacc[e] : 0.0;
}

// Flux rows: one thread per (field, coarse triangle k) owns row k and walks the 3r fine
// facets of its edges.  Per facet of fine square (i,j), corners u0=(i,j), u1=(i+1,j),
// u2=(i,j+1), u3=(i+1,j+1), |e| kappa grad(u).n_out on the fine triangle inside k:
//   lower-right (cells 2q): bottom k(u1-u3), right k(u1-u0), diagonal k(u0-2u1+u3)
//   upper-left  (2q+1)    : left k(u2-u3),  top k(u2-u0),   diagonal k(u0-2u2+u3)
// Edges on y=0 / y=1 are interior-facet (dS) measures over boundary facets in the
// reference and contribute nothing; x=0 / x=1 edges are ds, all others dS with the
// '+' side inside coarse cell k (flux.py:24-31,123-126).  Constrained fine nodes are
// dropped (Gamma_reduced keeps the free columns, alpha = 0: flux.py:151-156).
__device__ __forceinline__ void flux_add(double* row, int n, int i, int j, int dy, double coef) {
    if (i < 1 || i > n - 1 || coef == 0.0) return;
    row[(int64_t)(j * (n - 1) + i - 1)] += coef;
    (void)dy;
}

__global__ __launch_bounds__(64) void vo_query_flux(gpi_vo_query_desc d, FineGrid G, int m, int row0) {
    const int f = blockIdx.y;
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= G.nT_c) return;
    const int n = G.n, nc = G.nc, r = G.r;
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    double* row = d.gamma + ((int64_t)f * m + row0 + k) * G.dy;
    const int Q = k >> 1, ul = k & 1;
    const int I = Q % nc, J = Q / nc;
    for (int e = 0; e < 3; ++e) {
        if (ul == 0 && e == 0 && J == 0) continue;            // bottom edge on y = 0
        if (ul == 1 && e == 1 && J == nc - 1) continue;       // top edge on y = 1
        for (int t = 0; t < r; ++t) {
            int i, j;
            if (ul == 0) {
                if (e == 0) { i = I * r + t; j = J * r; }
                else if (e == 1) { i = (I + 1) * r - 1; j = J * r + t; }
                else { i = I * r + t; j = J * r + t; }
            } else {
                if (e == 0) { i = I * r; j = J * r + t; }
                else if (e == 1) { i = I * r + t; j = (J + 1) * r - 1; }
                else { i = I * r + t; j = J * r + t; }
            }
            const double kap = kcell(lk, n, i, j, ul);
            double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
            if (ul == 0) {
                if (e == 0) { c1 = kap; c3 = -kap; }
                else if (e == 1) { c1 = kap; c0 = -kap; }
                else { c0 = kap; c1 = -2.0 * kap; c3 = kap; }
            } else {
                if (e == 0) { c2 = kap; c3 = -kap; }
                else if (e == 1) { c2 = kap; c0 = -kap; }
                else { c0 = kap; c2 = -2.0 * kap; c3 = kap; }
            }
            flux_add(row, n, i, j, G.dy, c0);
            flux_add(row, n, i + 1, j, G.dy, c1);
            flux_add(row, n, i, j + 1, G.dy, c2);
            flux_add(row, n, i + 1, j + 1, G.dy, c3);
        }
    }
}


// ---------------------------------------------------------------- Galerkin rows from test functions
__device__ __forceinline__ double test_value(const gpi_vo_galerkin_desc& d, int f, int a, int p, int n,
                                             uint64_t base, double cx, double cy) {
    const int dy = (n + 1) * (n - 1);
    if (d.V) return d.V[((int64_t)f * d.m_aux + a) * dy + p];
    if (d.kind == GPI_VO_TEST_GAUSS) {
        const uint4_ q = philox(base + (uint64_t)(((int64_t)f * d.m_aux + a) * dy + p), d.sub, d.seed);
        const double u0 = ((double)q.x + 1.0) * 2.3283064365386963e-10;   // (0, 1]
        const double u1 = (double)q.y * 2.3283064365386963e-10;
        return sqrt(-2.0 * log(u0)) * cos(6.283185307179586 * u1);
    }
    const int jj = p / (n - 1), ii = p - jj * (n - 1) + 1;
    const double x = (double)ii / n - cx, y = (double)jj / n - cy;
    return exp(-(x * x + y * y) / (d.length * d.length));
}

__device__ __forceinline__ void rbf_center(const gpi_vo_galerkin_desc& d, int f, int a, uint64_t base, double& cx,
                                           double& cy) {
    if (d.centers) {
        cx = d.centers[((int64_t)f * d.m_aux + a) * 2];
        cy = d.centers[((int64_t)f * d.m_aux + a) * 2 + 1];
    } else {
        // a separate counter range (above every Gaussian counter) for the centres
        const uint4_ q = philox(base + ((uint64_t)1 << 62) + (uint64_t)((int64_t)f * d.m_aux + a), d.sub, d.seed);
        cx = (double)q.x * 2.3283064365386963e-10;
        cy = (double)q.y * 2.3283064365386963e-10;
    }
}

__global__ __launch_bounds__(256) void vo_galerkin_kernel(gpi_vo_galerkin_desc d) {
    __shared__ double red[4];
    const int a = blockIdx.y, f = blockIdx.z;
    const int n = d.n_fine, dy = (n + 1) * (n - 1);
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    const uint64_t base = d.offset ? *d.offset : 0;
    double cx = 0.0, cy = 0.0;
    if (d.kind == GPI_VO_TEST_RBF) rbf_center(d, f, a, base, cx, cy);
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < dy) {
        const int jj = p / (n - 1), ii = p - jj * (n - 1) + 1;
        const double chl = ch_(lk, n, ii - 1, jj), chr = ch_(lk, n, ii, jj);
        const double cvd = jj > 0 ? cv_(lk, n, ii, jj - 1) : 0.0;
        const double cvu = jj < n ? cv_(lk, n, ii, jj) : 0.0;
        double g = (chl + chr + cvd + cvu) * test_value(d, f, a, p, n, base, cx, cy);
        if (ii > 1) g -= chl * test_value(d, f, a, p - 1, n, base, cx, cy);
        if (ii < n - 1) g -= chr * test_value(d, f, a, p + 1, n, base, cx, cy);
        if (jj > 0) g -= cvd * test_value(d, f, a, p - (n - 1), n, base, cx, cy);
        if (jj < n) g -= cvu * test_value(d, f, a, p + (n - 1), n, base, cx, cy);
        d.gamma[((int64_t)f * d.m + d.row0 + a) * dy + p] = g;
    }
    if (blockIdx.x != 0) return;
    // alpha = V_a . f_eff: only the free nodes next to x = 0 / x = 1 carry f_eff
    const double* u = d.bc + 4 * f;
    double s = 0.0;
    for (int e = threadIdx.x; e < 2 * (n + 1); e += 256) {
        const int side = e / (n + 1), jj = e - side * (n + 1);
        if (n == 2 && side == 1) continue;
        const int ii = side == 0 ? 1 : n - 1;
        double fe = ch_(lk, n, side == 0 ? 0 : n - 1, jj) * bc_value(u, side == 0 ? 0 : n, jj, n);
        if (n == 2) fe += ch_(lk, n, n - 1, jj) * bc_value(u, n, jj, n);
        s += fe * test_value(d, f, a, jj * (n - 1) + ii - 1, n, base, cx, cy);
    }
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) d.alpha[(int64_t)f * d.m + d.row0 + a] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------- MC predictive moments
constexpr int MOM_CH = 64;   // MC samples staged in LDS per chunk

__device__ __forceinline__ float normal_at(uint64_t ctr, uint64_t sub, uint64_t seed) {
    const uint4_ q = philox(ctr, sub, seed);
    const float u0 = u01(q.x), u1 = u01(q.y);
    return sqrtf(-2.f * logf(u0)) * cosf(6.2831853071795864f * u1);
}

__global__ __launch_bounds__(256) void vo_moments_kernel(gpi_vo_moments_desc d, FineGrid G) {
    extern __shared__ __attribute__((aligned(16))) float su[];   // [MOM_CH][nn_c]
    const int j = blockIdx.y;
    const int n = G.n, nn = G.nn_c;
    const int p = blockIdx.x * 256 + threadIdx.x;
    const bool act = p < G.dy;
    int kk[3] = {0, 0, 0};
    float w[3] = {0.f, 0.f, 0.f};
    float sig = 0.f;
    if (act) {
        const int jj = p / (n - 1), ii = p - jj * (n - 1) + 1;
        double wd[3];
        interp_w(ii, jj, G.r, G.nc, kk, wd);
        for (int t = 0; t < 3; ++t) w[t] = (float)wd[t];
        if (d.logsig_y) sig = expf(d.logsig_y[p]);
    }
    const uint64_t base = d.offset ? *d.offset : 0;
    const int64_t row0 = (int64_t)j * d.n_mc;
    // one pass (each draw made once): fp64 sums of y - K and (y - K)^2, shifted by the first sample K
    double s1 = 0.0, s2 = 0.0, K = 0.0;
    for (int s0 = 0; s0 < d.n_mc; s0 += MOM_CH) {
        const int ns = min(MOM_CH, d.n_mc - s0);
        __syncthreads();
        for (int e = threadIdx.x; e < ns * nn; e += 256) su[e] = d.uc[(row0 + s0) * nn + e];
        __syncthreads();
        if (!act) continue;
        for (int s = 0; s < ns; ++s) {
            const float* us = su + s * nn;
            float y = w[0] * us[kk[0]] + w[1] * us[kk[1]] + w[2] * us[kk[2]];
            if (d.logsig_y) {
                const int64_t rr = row0 + s0 + s;
                const float e = d.eps ? d.eps[rr * G.dy + p]
                                      : normal_at(base + (uint64_t)(rr * G.dy + p), d.sub, d.seed);
                y = fmaf(sig, e, y);
            }
            if (s0 + s == 0) K = (double)y;
            const double t = (double)y - K;
            s1 += t;
            s2 = fma(t, t, s2);
        }
    }
    const double mean = K + s1 / (double)d.n_mc;
    const double ssd = fmax(s2 - s1 * (s1 / (double)d.n_mc), 0.0);
    if (!act) return;
    const float sd = (float)sqrt(ssd / (double)(d.n_mc - 1));
    const int64_t o = (int64_t)j * G.dy + p;
    d.mean[o] = (float)mean;
    if (d.std) d.std[o] = sd;
    if (d.prec) d.prec[o] = 1.f / (sd * sd);
}

// ---------------------------------------------------------------- conditioning
constexpr int LT = 32;   // Lambda tile

// Lambda[a][b] = sum_i Gamma[a][i] cov_i Gamma[b][i] (+ vo_var on the diagonal), lower tiles
// (ta >= tb) computed and mirrored.  cov_i = 1 / (double) prec_i, formed once per k-step by 32
// threads (not per tile element).  The next k-step's Gamma tiles are loaded into registers while
// the current one is multiplied (one global round trip per k-step hidden behind the FMAs).
__global__ __launch_bounds__(256) void vo_lambda_kernel(gpi_vo_condition_desc d) {
    __shared__ double As[LT][LT + 1], Bs[LT][LT + 1], cv[LT];
    const int j = blockIdx.y;
    int t = blockIdx.x, ta = 0;
    while (t > ta) { t -= ta + 1; ++ta; }
    const int tb = t;
    const int m = d.m, dy = d.d_y;
    const double* gam = d.gamma + (int64_t)j * m * dy;
    const float* prec = d.prec + (int64_t)j * dy;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    // this thread's 4 elements of each 32 x 32 tile: rows rr = (tid >> 5) + 8 u, column cc = tid & 31
    const int cc = threadIdx.x & 31, r0 = threadIdx.x >> 5;
    double pa[4], pb[4], pc = 0.0;
    auto fetch = [&](int k0) {
        const int i = k0 + cc;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int a = ta * LT + r0 + 8 * u, b = tb * LT + r0 + 8 * u;
            pa[u] = (i < dy && a < m) ? gam[(int64_t)a * dy + i] : 0.0;
            pb[u] = (i < dy && b < m) ? gam[(int64_t)b * dy + i] : 0.0;
        }
        pc = (threadIdx.x < LT && k0 + (int)threadIdx.x < dy) ? (double)prec[k0 + threadIdx.x] : 1.0;
    };
    fetch(0);
    for (int k0 = 0; k0 < dy; k0 += LT) {
        if (threadIdx.x < LT) cv[threadIdx.x] = 1.0 / pc;
#pragma unroll
        for (int u = 0; u < 4; ++u) Bs[r0 + 8 * u][cc] = pb[u];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) As[r0 + 8 * u][cc] = pa[u] * cv[cc];
        if (k0 + LT < dy) fetch(k0 + LT);      // next tiles in flight during the FMAs below
        __syncthreads();
#pragma unroll 8
        for (int c = 0; c < LT; ++c) {
            const double a0 = As[ty][c], a1 = As[ty + 16][c];
            const double b0 = Bs[tx][c], b1 = Bs[tx + 16][c];
            acc[0][0] = fma(a0, b0, acc[0][0]);
            acc[0][1] = fma(a0, b1, acc[0][1]);
            acc[1][0] = fma(a1, b0, acc[1][0]);
            acc[1][1] = fma(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
    double* lam = d.lam + (int64_t)j * m * m;
    for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 2; ++v) {
            const int a = ta * LT + ty + 16 * u, b = tb * LT + tx + 16 * v;
            if (a >= m || b >= m || b > a) continue;
            double val = acc[u][v];
            if (a == b) val += d.vo_var[a];
            lam[(int64_t)a * m + b] = val;
            lam[(int64_t)b * m + a] = val;
        }
}

// In-place lower Cholesky of one m x m matrix A (row-major) by the 256 threads of the block.
__device__ void chol_block(double* A, int m, bool& bad) {
    const int tid = threadIdx.x;
    for (int k = 0; k < m; ++k) {
        const double akk = A[k * m + k];
        if (!(akk > 0.0)) bad = true;
        const double dk = sqrt(akk);
        __syncthreads();
        for (int i = k + 1 + tid; i < m; i += 256) A[i * m + k] /= dk;
        if (tid == 0) A[k * m + k] = dk;
        __syncthreads();
        for (int i = k + 1 + (tid >> 4); i < m; i += 16) {
            const double lik = A[i * m + k];
            for (int jj = k + 1 + (tid & 15); jj <= i; jj += 16) A[i * m + jj] -= lik * A[jj * m + k];
        }
        __syncthreads();
    }
}

// Blocked right-looking Cholesky of the global-memory Lambda (m <= 256): per 16-column panel the
// diagonal block is factored in LDS, the rows below solve against it (one thread per row, panel in
// LDS) and the trailing lower triangle takes ONE rank-16 update (instead of 16 rank-1 sweeps over
// global memory).
constexpr int CP_W = 16, CP_R = 256;
__device__ void chol_panel(double* A, int m, bool& bad) {
    __shared__ double D[CP_W][CP_W + 1];
    __shared__ double P[CP_R][CP_W + 1];
    const int tid = threadIdx.x;
    for (int K0 = 0; K0 < m; K0 += CP_W) {
        const int w = min(CP_W, m - K0), R0 = K0 + w, R = m - R0;
        for (int e = tid; e < CP_W * CP_W; e += 256) {
            const int r = e / CP_W, c = e - r * CP_W;
            D[r][c] = (r < w && c <= r) ? A[(int64_t)(K0 + r) * m + K0 + c] : 0.0;
        }
        for (int e = tid; e < R * CP_W; e += 256) {
            const int r = e / CP_W, c = e - r * CP_W;
            P[r][c] = c < w ? A[(int64_t)(R0 + r) * m + K0 + c] : 0.0;
        }
        __syncthreads();
        if (tid < 64) {                             // diagonal block: wave 0, lane r holds row r, no barriers
            const int r = tid & (CP_W - 1);
            double row[CP_W];
#pragma unroll
            for (int c = 0; c < CP_W; ++c) row[c] = D[r][c];
#pragma unroll
            for (int k = 0; k < CP_W; ++k) {
                if (k < w) {
                    const double akk = __shfl(row[k], k, 64);
                    if (!(akk > 0.0)) bad = true;
                    const double dk = sqrt(akk);
                    if (r == k) row[k] = dk;
                    else if (r > k) row[k] /= dk;
#pragma unroll
                    for (int c = k + 1; c < CP_W; ++c) {
                        const double lc = __shfl(row[k], c, 64);
                        if (r >= c && r > k) row[c] = fma(-row[k], lc, row[c]);
                    }
                }
            }
            if (tid < CP_W)
#pragma unroll
                for (int c = 0; c < CP_W; ++c) D[r][c] = row[c];
        }
        __syncthreads();
        if (tid < R) {                              // panel rows: x L11^T = a
            for (int c = 0; c < w; ++c) {
                double a = P[tid][c];
                for (int k = 0; k < c; ++k) a -= P[tid][k] * D[c][k];
                P[tid][c] = a / D[c][c];
            }
        }
        __syncthreads();
        for (int e = tid; e < CP_W * CP_W; e += 256) {
            const int r = e / CP_W, c = e - r * CP_W;
            if (r < w && c <= r) A[(int64_t)(K0 + r) * m + K0 + c] = D[r][c];
        }
        for (int e = tid; e < R * CP_W; e += 256) {
            const int r = e / CP_W, c = e - r * CP_W;
            if (c < w) A[(int64_t)(R0 + r) * m + K0 + c] = P[r][c];
        }
        const int ntri = R * (R + 1) / 2;           // trailing update over the lower triangle, flattened
        for (int e = tid; e < ntri; e += 256) {
            int i = (int)((sqrtf(8.f * (float)e + 1.f) - 1.f) * 0.5f);
            while (i * (i + 1) / 2 > e) --i;
            while ((i + 1) * (i + 2) / 2 <= e) ++i;
            const int jj = e - i * (i + 1) / 2;
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < CP_W; ++c) s = fma(P[i][c], P[jj][c], s);
            A[(int64_t)(R0 + i) * m + R0 + jj] -= s;
        }
        __syncthreads();
    }
}

template <bool LDS>
__global__ __launch_bounds__(256) void vo_chol_kernel(gpi_vo_condition_desc d) {
    extern __shared__ __attribute__((aligned(16))) double sm[];   // [m] rhs (+ [m*m] matrix if LDS)
    const int j = blockIdx.x;
    const int m = d.m, dy = d.d_y;
    double* lam = d.lam + (int64_t)j * m * m;
    double* b = sm;
    double* A = LDS ? sm + m : lam;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (LDS) {
        for (int e = tid; e < m * m; e += 256) A[e] = lam[e];
        __syncthreads();
    }
    bool bad = false;
    if constexpr (LDS) chol_block(A, m, bad);
    else if (m <= CP_R) chol_panel(A, m, bad);
    else chol_block(A, m, bad);
    if (bad && d.flag && tid == 0) atomicOr(d.flag, 1);
    if (!LDS) return;       // large m: b by vo_rhs_kernel, solves by vo_solvec_kernel
    // b = Gamma g - alpha (column-sparse path: already in solvec, vo_rhs_sparse_kernel)
    if (d.sparse) {
        for (int a = tid; a < m; a += 256) b[a] = d.solvec[(int64_t)j * m + a];
    } else {
        const double* gam = d.gamma + (int64_t)j * m * dy;
        const float* g = d.g + (int64_t)j * dy;
        for (int a = wid; a < m; a += 4) {
            double s = 0.0;
            for (int i = lane; i < dy; i += 64) s = fma(gam[(int64_t)a * dy + i], (double)g[i], s);
            s = wave_sum_d(s);
            if (lane == 0) b[a] = s - d.alpha[(int64_t)j * m + a];
        }
    }
    __syncthreads();
    // L z = b, L^T x = z
    for (int k = 0; k < m; ++k) {
        const double zk = b[k] / A[k * m + k];
        __syncthreads();
        for (int i = k + 1 + tid; i < m; i += 256) b[i] -= A[i * m + k] * zk;
        if (tid == 0) b[k] = zk;
        __syncthreads();
    }
    for (int k = m - 1; k >= 0; --k) {
        const double xk = b[k] / A[k * m + k];
        __syncthreads();
        for (int i = tid; i < k; i += 256) b[i] -= A[k * m + i] * xk;
        if (tid == 0) b[k] = xk;
        __syncthreads();
    }
    for (int e = tid; e < m; e += 256) d.solvec[(int64_t)j * m + e] = b[e];
    if (LDS)
        for (int e = tid; e < m * m; e += 256) lam[e] = A[e];
}

// L^{-1} per sample, stored transposed in the strict upper triangle of lam (lam[c*m + a] =
// (L^{-1})_{ac}, a > c; the diagonal is 1 / L_aa, the lower triangle keeps L).  One thread per
// column c (forward substitution over the rows below it).
__global__ __launch_bounds__(256) void vo_linv_kernel(gpi_vo_condition_desc d) {
    const int j = blockIdx.x, m = d.m;
    double* lam = d.lam + (int64_t)j * m * m;
    for (int c = threadIdx.x; c < m; c += blockDim.x) {
        double* x = lam + (int64_t)c * m;            // x[a] = (L^{-1})_{ac} for a > c
        const double xc = 1.0 / lam[(int64_t)c * m + c];
        for (int a = c + 1; a < m; ++a) {
            const double* La = lam + (int64_t)a * m;
            double s = La[c] * xc;
            for (int b = c + 1; b < a; ++b) s = fma(La[b], x[b], s);
            x[a] = -s / La[a];
        }
    }
}

// The same, one wave per column c (m <= 256): column-oriented forward substitution of L x = e_c
// with x in registers (lane holds x[lane + 64k]); per row b one broadcast of x[b] and an axpy of
// L's column b over the rows below.  Reciprocal diagonal in LDS.
__global__ __launch_bounds__(256) void vo_linv_wave_kernel(gpi_vo_condition_desc d) {
    __shared__ double dinv[256];
    const int j = blockIdx.y, m = d.m;
    double* lam = d.lam + (int64_t)j * m * m;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int a = threadIdx.x; a < m; a += blockDim.x) dinv[a] = 1.0 / lam[(int64_t)a * m + a];
    __syncthreads();
    const int c = blockIdx.x * 4 + w;
    if (c >= m) return;
    double x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = (lane + 64 * k == c) ? 1.0 : 0.0;
    for (int b = c; b < m; ++b) {
        const int kb = b >> 6;
        const double own = kb == 0 ? x[0] : kb == 1 ? x[1] : kb == 2 ? x[2] : x[3];
        const double xb = __shfl(own, b & 63, 64) * dinv[b];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int a = lane + 64 * k;
            if (a == b) x[k] = xb;
            else if (a > b && a < m) x[k] = fma(-lam[(int64_t)a * m + b], xb, x[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int a = lane + 64 * k;
        if (a > c && a < m) lam[(int64_t)c * m + a] = x[k];
    }
}

// The same by 32 x 32 blocks (m <= 256), one workgroup per (block column jb, sample): block row ib of
// column block jb of L^-1 is X_ib = L_ib,ib^-1 (delta_ib,jb I - sum_{kb=jb}^{ib-1} L_ib,kb X_kb): the sum as
// LDS tile products, the triangular solve per column inside one wave (thread (tc, tr) = (tid / 8, tid % 8)
// keeps rows tr + 8u of column tc in registers; the owner of row k hands x_k to the column's 8 lanes by a
// shuffle, no barrier).  The finished blocks stay in LDS for the block rows below and are written
// transposed into lam's strict upper triangle (only the lower triangle is read here, so workgroups never
// race).
constexpr int TI = 32;
__global__ __launch_bounds__(256) void vo_linv_block_kernel(gpi_vo_condition_desc d) {
    extern __shared__ double xs[];                       // [nb - jb][TI][TI + 1]
    __shared__ double Ls[TI][TI + 1];
    const int jb = blockIdx.x, j = blockIdx.y, m = d.m, nb = (m + TI - 1) / TI;
    double* lam = d.lam + (int64_t)j * m * m;
    const int tid = threadIdx.x, lane = tid & 63;
    const int tc = tid >> 3, tr = tid & 7;               // compute layout
    const int lc = tid & 31, lr = tid >> 5;              // tile-load layout (rows of 32 contiguous)
    for (int ib = jb; ib < nb; ++ib) {
        double* Xi = xs + (ib - jb) * TI * (TI + 1);
        double acc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = (ib == jb && tr + 8 * u == tc && ib * TI + tc < m) ? 1.0 : 0.0;
        for (int kb = jb; kb < ib; ++kb) {
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int a = ib * TI + lr + 8 * u, b = kb * TI + lc;
                Ls[lr + 8 * u][lc] = (a < m && b < m) ? lam[(int64_t)a * m + b] : 0.0;
            }
            __syncthreads();
            const double* Xk = xs + (kb - jb) * TI * (TI + 1);
#pragma unroll 8
            for (int c = 0; c < TI; ++c) {
                const double xv = Xk[c * (TI + 1) + tc];
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] = fma(-Ls[tr + 8 * u][c], xv, acc[u]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {                    // diagonal block (identity on rows past m)
            const int r = lr + 8 * u, a = ib * TI + r, b = ib * TI + lc;
            Ls[r][lc] = (a < m && b < m) ? (lc <= r ? lam[(int64_t)a * m + b] : 0.0) : (r == lc ? 1.0 : 0.0);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < TI; ++k) {
            const double cand = acc[k >> 3] / Ls[k][k];
            const double xk = __shfl(cand, (lane & ~7) | (k & 7), 64);
            if (tr == (k & 7)) acc[k >> 3] = xk;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (tr + 8 * u > k) acc[u] = fma(-Ls[tr + 8 * u][k], xk, acc[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) Xi[(tr + 8 * u) * (TI + 1) + tc] = acc[u];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {                    // lam[c m + a] = X[a][c], a > c (rows fastest)
            const int r = lc, cl = lr + 8 * u, a = ib * TI + r, c = jb * TI + cl;
            if (a < m && c < m && a > c) lam[(int64_t)c * m + a] = Xi[r * (TI + 1) + cl];
        }
    }
}

// b = Gamma g - alpha into solvec (large-m path; one workgroup per (row a, VO sample j)): the two
// triangular sweeps would be 2 m barrier-separated steps over global memory, so vo_solvec_kernel
// applies L^-T L^-1 to it once L^-1 exists.
__global__ __launch_bounds__(256) void vo_rhs_kernel(gpi_vo_condition_desc d) {
    __shared__ double red[4];
    const int a = blockIdx.x, j = blockIdx.y, m = d.m, dy = d.d_y;
    const double* row = d.gamma + ((int64_t)j * m + a) * dy;
    const float* g = d.g + (int64_t)j * dy;
    double s = 0.0;
    for (int i = threadIdx.x; i < dy; i += 256) s = fma(row[i], (double)g[i], s);
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
        d.solvec[(int64_t)j * m + a] = (red[0] + red[1]) + (red[2] + red[3]) - d.alpha[(int64_t)j * m + a];
}

// solvec = Lambda^{-1} b = L^-T (L^-1 b) from the L^-1 in lam's upper triangle (large-m path).
constexpr int VS_MAXM = 1024;
__global__ __launch_bounds__(256) void vo_solvec_kernel(gpi_vo_condition_desc d) {
    __shared__ double bs[VS_MAXM], ts[VS_MAXM];
    const int j = blockIdx.x, m = d.m;
    const double* lam = d.lam + (int64_t)j * m * m;
    double* sv = d.solvec + (int64_t)j * m;
    for (int a = threadIdx.x; a < m; a += blockDim.x) bs[a] = sv[a];
    __syncthreads();
    for (int a = threadIdx.x; a < m; a += blockDim.x) {          // t = L^-1 b
        double s = bs[a] / lam[(int64_t)a * m + a];
        for (int c = 0; c < a; ++c) s = fma(lam[(int64_t)c * m + a], bs[c], s);
        ts[a] = s;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < m; c += blockDim.x) {          // solvec = L^-T t
        double s = ts[c] / lam[(int64_t)c * m + c];
        for (int a = c + 1; a < m; ++a) s = fma(lam[(int64_t)c * m + a], ts[a], s);
        sv[c] = s;
    }
}

// Posterior per column i of Gamma (fp64): q = L^{-1} Gamma_i as a blocked lower-triangular GEMM
// Q = L^{-1} Gamma over a 64-column tile (64 x 32 L^{-1} blocks and 32 x 64 Gamma blocks in LDS,
// fp64 MFMA 16x16x4 per wave), only |q|^2 kept;  mean_i = g_i - cov_i Gamma_i . solvec,
// vars_i = cov_i - cov_i^2 |q|^2.
constexpr int VC_BA = 64, VC_BK = 32, VC_BN = 64;
__global__ __launch_bounds__(256) void vo_columns_kernel(gpi_vo_condition_desc d) {
    __shared__ double Ls[VC_BA][VC_BK + 1];
    __shared__ double Gs[VC_BK][VC_BN];
    __shared__ double red[16][VC_BN];
    const int j = blockIdx.y;
    const int m = d.m, dy = d.d_y;
    const int tid = threadIdx.x;
    const int i0 = blockIdx.x * VC_BN;
    const double* gam = d.gamma + (int64_t)j * m * dy;
    const double* lam = d.lam + (int64_t)j * m * m;
    const double* sv = d.solvec + (int64_t)j * m;
    // Gamma_i . solvec: 4 partial sums per column
    {
        const int col = tid & 63, part = tid >> 6;
        const int i = i0 + col;
        double s = 0.0;
        if (i < dy)
            for (int a = part; a < m; a += 4) s = fma(gam[(int64_t)a * dy + i], sv[a], s);
        red[part][col] = s;
    }
    __syncthreads();
    double smv = 0.0;
    if (tid < VC_BN) smv = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    __syncthreads();
    // v_mfma_f64_16x16x4_f64: wave w owns rows [16w, 16w + 16) of the 64-row block and the four 16-column
    // sub-blocks; A[l&15][k=l>>4], B[k=l>>4][l&15], D col = l&15, row = (l>>4) + 4 reg.
    typedef double f64x4 __attribute__((ext_vector_type(4)));
    const int lane = tid & 63, w = tid >> 6;
    double qp[4] = {0.0, 0.0, 0.0, 0.0};          // per 16-column sub-block, this lane's column
    for (int A0 = 0; A0 < m; A0 += VC_BA) {
        f64x4 acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
        const int bend = min(A0 + VC_BA, m);
        for (int B0 = 0; B0 < bend; B0 += VC_BK) {
            for (int e = tid; e < VC_BA * VC_BK; e += 256) {
                const int ra = e & (VC_BA - 1), rb = e / VC_BA;
                const int a = A0 + ra, b = B0 + rb;
                double v = 0.0;
                if (a < m && b < m) {
                    if (a > b) v = lam[(int64_t)b * m + a];
                    else if (a == b) v = 1.0 / lam[(int64_t)a * m + a];
                }
                Ls[ra][rb] = v;
            }
            for (int e = tid; e < VC_BK * VC_BN; e += 256) {
                const int rb = e / VC_BN, col = e & (VC_BN - 1);
                const int b = B0 + rb, i = i0 + col;
                Gs[rb][col] = (b < m && i < dy) ? gam[(int64_t)b * dy + i] : 0.0;
            }
            __syncthreads();
#pragma unroll
            for (int k0 = 0; k0 < VC_BK; k0 += 4) {
                const double av = Ls[16 * w + (lane & 15)][k0 + (lane >> 4)];
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const double bv = Gs[k0 + (lane >> 4)][16 * cb + (lane & 15)];
                    acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[cb], 0, 0, 0);
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) qp[cb] = fma(acc[cb][r], acc[cb][r], qp[cb]);
    }
    // sum the four row groups of the wave (lanes l, l^16, l^32, l^48), then the four waves
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        qp[cb] += __shfl_xor(qp[cb], 16, 64);
        qp[cb] += __shfl_xor(qp[cb], 32, 64);
    }
    if (lane < 16)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) red[w][16 * cb + lane] = qp[cb];
    __syncthreads();
    if (tid >= VC_BN) return;
    const int i = i0 + tid;
    if (i >= dy) return;
    const double qn = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    const int64_t o = (int64_t)j * dy + i;
    const double cov = 1.0 / (double)d.prec[o];
    const double mean = (double)d.g[o] - cov * smv;
    const double var = cov - cov * cov * qn;
    d.mean[o] = mean;
    d.vars[o] = var;
    if (d.mean32) d.mean32[o] = (float)mean;
    if (d.logsig32) d.logsig32[o] = 0.5f * logf((float)var);
}

// ---------------------------------------------------------------- column-sparse conditioning
// With gpi_vo_sparse (CGR / flux rows: <= VS_R nonzeros per column, the same rows in every sample):
//   Lambda      one thread per (pair (a, b), sample): sum over the columns holding both rows
//   b           one wave per (row a, sample) over the row's nonzeros
//   Lambda^-1   U U^T with U = L^-T (upper triangle of lam after vo_linv), 32 x 32 tiles
//   columns     one thread per (column i, sample): Gamma_i . solvec and Gamma_i^T Lambda^-1 Gamma_i
//               from the column's <= VS_R slots (|L^-1 Gamma_i|^2 without forming L^-1 Gamma_i)
// Every sum runs in a fixed order (reproducible).
constexpr int VS_R = 16;

// nz[a, i] = 1 if gamma[j, a, i] != 0 for some sample j (16 loads in flight per thread)
__global__ __launch_bounds__(256) void vo_nz_kernel(const double* gamma, int n, int m, int dy, uint8_t* nz) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)m * dy) return;
    const int64_t plane = (int64_t)m * dy;
    bool any = false;
    for (int j0 = 0; j0 < n && !any; j0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (j0 + u < n) ? gamma[(int64_t)(j0 + u) * plane + e] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) any = any || (v[u] != 0.0);
    }
    nz[e] = any ? 1 : 0;
}

__global__ __launch_bounds__(256) void vo_pattern_kernel(const uint8_t* nz, int m, int dy, int r, int32_t* rows,
                                                         int32_t* count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= dy) return;
    int c = 0;
    for (int a = 0; a < m; ++a)
        if (nz[(int64_t)a * dy + i]) {
            if (c < r) rows[(int64_t)i * r + c] = a;
            ++c;
        }
    for (int s = c; s < r; ++s) rows[(int64_t)i * r + s] = -1;
    count[i] = c;
}

__global__ __launch_bounds__(256) void vo_sparse_values_kernel(const double* gamma, int n, int m, int dy,
                                                               gpi_vo_sparse sp) {
    const int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
    if (i >= dy) return;
    const double* gj = gamma + (int64_t)j * m * dy;
    double* out = const_cast<double*>(sp.vals) + ((int64_t)j * dy + i) * sp.r;
    for (int s = 0; s < sp.r; ++s) {
        const int a = sp.rows[(int64_t)i * sp.r + s];
        out[s] = a >= 0 ? gj[(int64_t)a * dy + i] : 0.0;
    }
}

__global__ __launch_bounds__(256) void vo_lambda_sparse_kernel(gpi_vo_condition_desc d, gpi_vo_sparse sp) {
    const int p = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
    if (p >= sp.n_pairs) return;
    const int m = d.m, r = sp.r, rr = r * r;
    const double* v = sp.vals + (int64_t)j * d.d_y * r;
    const float* prec = d.prec + (int64_t)j * d.d_y;
    double acc = 0.0;
    const int e1 = sp.pair_ptr[p + 1];
    for (int e = sp.pair_ptr[p]; e < e1; ++e) {
        const int src = sp.pair_src[e];
        const int i = src / rr, st = src - i * rr, s = st / r, t = st - s * r;
        acc = fma(v[i * r + s] / (double)prec[i], v[i * r + t], acc);
    }
    const int ab = sp.pair_ab[p], a = ab / m, b = ab - a * m;
    if (a == b) acc += d.vo_var[a];
    double* lam = d.lam + (int64_t)j * m * m;
    lam[(int64_t)a * m + b] = acc;
    lam[(int64_t)b * m + a] = acc;
}

// b = Gamma g - alpha into solvec, one wave per (row a, sample j)
__global__ __launch_bounds__(256) void vo_rhs_sparse_kernel(gpi_vo_condition_desc d, gpi_vo_sparse sp) {
    const int lane = threadIdx.x & 63, a = blockIdx.x * 4 + (threadIdx.x >> 6), j = blockIdx.y;
    if (a >= d.m) return;                                  // wave-uniform
    const double* v = sp.vals + (int64_t)j * d.d_y * sp.r;
    const float* g = d.g + (int64_t)j * d.d_y;
    double s = 0.0;
    const int e1 = sp.row_ptr[a + 1];
    for (int e = sp.row_ptr[a] + lane; e < e1; e += 64) {
        const int src = sp.row_src[e];
        s = fma(v[src], (double)g[src / sp.r], s);
    }
    s = wave_sum_d(s);
    if (lane == 0) d.solvec[(int64_t)j * d.m + a] = s - d.alpha[(int64_t)j * d.m + a];
}

// Lambda^-1 = L^-T L^-1 = U U^T, U[a][c] = (L^-1)_{ca}: lam[a m + c] for c > a, 1 / lam[a m + a] at c = a;
// lower 32 x 32 tiles (ta >= tb) computed and mirrored; the c-loop starts at row tile ta (U is upper).
__global__ __launch_bounds__(256) void vo_inv_kernel(gpi_vo_condition_desc d, gpi_vo_sparse sp) {
    __shared__ double As[LT][LT + 1], Bs[LT][LT + 1];
    const int j = blockIdx.y;
    int t = blockIdx.x, ta = 0;
    while (t > ta) { t -= ta + 1; ++ta; }
    const int tb = t, m = d.m;
    const double* lam = d.lam + (int64_t)j * m * m;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int cc = threadIdx.x & 31, r0 = threadIdx.x >> 5;
    auto U = [&](int a, int c) -> double {
        if (a >= m || c >= m || c < a) return 0.0;
        const double x = lam[(int64_t)a * m + c];
        return c == a ? 1.0 / x : x;
    };
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    for (int c0 = ta * LT; c0 < m; c0 += LT) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            As[r0 + 8 * u][cc] = U(ta * LT + r0 + 8 * u, c0 + cc);
            Bs[r0 + 8 * u][cc] = U(tb * LT + r0 + 8 * u, c0 + cc);
        }
        __syncthreads();
#pragma unroll 8
        for (int c = 0; c < LT; ++c) {
            const double a0 = As[ty][c], a1 = As[ty + 16][c];
            const double b0 = Bs[tx][c], b1 = Bs[tx + 16][c];
            acc[0][0] = fma(a0, b0, acc[0][0]);
            acc[0][1] = fma(a0, b1, acc[0][1]);
            acc[1][0] = fma(a1, b0, acc[1][0]);
            acc[1][1] = fma(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
    double* inv = sp.inv + (int64_t)j * m * m;
    for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 2; ++v) {
            const int a = ta * LT + ty + 16 * u, b = tb * LT + tx + 16 * v;
            if (a >= m || b >= m || b > a) continue;
            inv[(int64_t)a * m + b] = acc[u][v];
            inv[(int64_t)b * m + a] = acc[u][v];
        }
}

// Posterior of column i of sample j from its slots: mean_i = g_i - cov_i Gamma_i . solvec,
// vars_i = cov_i - cov_i^2 Gamma_i^T Lambda^-1 Gamma_i.
__global__ __launch_bounds__(256) void vo_columns_sparse_kernel(gpi_vo_condition_desc d, gpi_vo_sparse sp) {
    const int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
    if (i >= d.d_y) return;
    const int m = d.m, r = sp.r;
    int rw[VS_R];
    double v[VS_R];
#pragma unroll
    for (int s = 0; s < VS_R; ++s) {
        rw[s] = s < r ? sp.rows[(int64_t)i * r + s] : -1;
        v[s] = rw[s] >= 0 ? sp.vals[((int64_t)j * d.d_y + i) * r + s] : 0.0;
    }
    const double* inv = sp.inv + (int64_t)j * m * m;
    const double* sv = d.solvec + (int64_t)j * m;
    double smv = 0.0, qn = 0.0;
#pragma unroll
    for (int s = 0; s < VS_R; ++s) {
        if (rw[s] < 0) continue;
        const double* ia = inv + (int64_t)rw[s] * m;
        smv = fma(v[s], sv[rw[s]], smv);
        double off = 0.0;
#pragma unroll
        for (int t = 0; t < s; ++t)
            if (rw[t] >= 0) off = fma(v[t], ia[rw[t]], off);
        qn = fma(v[s], fma(2.0, off, v[s] * ia[rw[s]]), qn);
    }
    const int64_t o = (int64_t)j * d.d_y + i;
    const double cov = 1.0 / (double)d.prec[o];
    const double mean = (double)d.g[o] - cov * smv;
    const double var = cov - cov * cov * qn;
    d.mean[o] = mean;
    d.vars[o] = var;
    if (d.mean32) d.mean32[o] = (float)mean;
    if (d.logsig32) d.logsig32[o] = 0.5f * logf((float)var);
}

// ---------------------------------------------------------------- precision
// One workgroup per (row a, VO sample j): its term (Gamma_j mean_j - alpha_j)_a^2 + (Gamma_j^2 vars_j)_a
// into terms[a, j]; vo_precision_final sums them over j in order (reproducible) into beta / vo_var.
__global__ __launch_bounds__(256) void vo_precision_kernel(gpi_vo_precision_desc d) {
    __shared__ double red[2][4];
    const int a = blockIdx.x, j = blockIdx.y;
    const int m = d.m, dy = d.d_y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const double* row = d.gamma + ((int64_t)j * m + a) * dy;
    const double* mu = d.mean + (int64_t)j * dy;
    const double* va = d.vars + (int64_t)j * dy;
    double s1 = 0.0, s2 = 0.0;
    for (int i = tid; i < dy; i += 256) {
        const double gv = row[i];
        s1 = fma(gv, mu[i], s1);
        s2 = fma(gv * gv, va[i], s2);
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (lane == 0) { red[0][wid] = s1; red[1][wid] = s2; }
    __syncthreads();
    if (tid == 0) {
        const double r1 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]) - d.alpha[(int64_t)j * m + a];
        const double r2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        d.terms[(int64_t)a * d.n + j] = r1 * r1 + r2;
    }
}

// The same terms from the column-sparse view: one wave per (row a, sample j) over the row's nonzeros.
__global__ __launch_bounds__(256) void vo_precision_sparse_kernel(gpi_vo_precision_desc d, gpi_vo_sparse sp) {
    const int lane = threadIdx.x & 63, a = blockIdx.x, j = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (j >= d.n) return;                                  // wave-uniform
    const double* v = sp.vals + (int64_t)j * d.d_y * sp.r;
    const double* mu = d.mean + (int64_t)j * d.d_y;
    const double* va = d.vars + (int64_t)j * d.d_y;
    double s1 = 0.0, s2 = 0.0;
    const int e1 = sp.row_ptr[a + 1];
    for (int e = sp.row_ptr[a] + lane; e < e1; e += 64) {
        const int src = sp.row_src[e], i = src / sp.r;
        const double gv = v[src];
        s1 = fma(gv, mu[i], s1);
        s2 = fma(gv * gv, va[i], s2);
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (lane == 0) {
        const double r1 = s1 - d.alpha[(int64_t)j * d.m + a];
        d.terms[(int64_t)a * d.n + j] = r1 * r1 + s2;
    }
}

__global__ __launch_bounds__(256) void vo_precision_final(gpi_vo_precision_desc d) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= d.m) return;
    double sum = 0.0;
    for (int j = 0; j < d.n; ++j) sum += d.terms[(int64_t)a * d.n + j];
    const double beta = 0.5 * sum + d.beta0;
    d.beta[a] = beta;
    d.vo_var[a] = (d.infinite && d.infinite[a]) ? 0.0 : beta / (0.5 * (double)d.n + d.alpha0 + 1.0);
}

// ---------------------------------------------------------------- reparametrised rows
__global__ __launch_bounds__(256) void gauss_sample_kernel(float* out, const float* mean, const float* ls,
                                                           int64_t total, int32_t dim, int32_t rep,
                                                           const float* eps, uint64_t seed,
                                                           const uint64_t* offset, uint64_t sub) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int64_t r = e / dim;
    const int t = (int)(e - r * dim);
    const int64_t src = (r / rep) * dim + t;
    const float z = eps ? eps[e] : normal_at((offset ? *offset : 0) + (uint64_t)e, sub, seed);
    out[e] = fmaf(expf(ls[src]), z, mean[src]);
}


// ---------------------------------------------------------------- predictive (Analysis)
constexpr int GPT = 128;   // threads per predictive row

__global__ __launch_bounds__(GPT) void gp_sample_kernel(gpi_gp_sample_desc d) {
    __shared__ float zs[512];
    const int r = blockIdx.x;
    const int j = r / d.rep;
    const uint64_t base = d.offset ? *d.offset : 0;
    for (int k = threadIdx.x; k < d.d_z; k += GPT) {
        const int64_t e = (int64_t)r * d.d_z + k;
        const float ez = d.eps_z ? d.eps_z[e] : normal_at(base + (uint64_t)e, d.sub, d.seed);
        zs[k] = fmaf(expf(d.qz_ls[(int64_t)j * d.d_z + k]), ez, d.qz_mu[(int64_t)j * d.d_z + k]);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < d.d_x; t += GPT) {
        float a = d.gp_b[t];
        const float* w = d.gp_w + (int64_t)t * d.d_z;
        for (int k = 0; k < d.d_z; ++k) a = fmaf(w[k], zs[k], a);
        if (d.gp_ls) {
            const int64_t e = (int64_t)r * d.d_x + t;
            const float ex = d.eps_x ? d.eps_x[e] : normal_at(base + (uint64_t)e, d.sub + 1, d.seed);
            a = fmaf(expf(d.gp_ls[t]), ex, a);
        }
        d.x[(int64_t)r * d.d_x + t] = a;
    }
}

// per sample: relative error and log score (one workgroup per sample)
__global__ __launch_bounds__(256) void scores_rows_kernel(const float* Y, const float* mean, const float* std,
                                                          int d_y, double* out) {
    __shared__ double red[3][4];
    const int n = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    double se = 0.0, sy = 0.0, ls = 0.0;
    for (int p = tid; p < d_y; p += 256) {
        const int64_t o = (int64_t)n * d_y + p;
        const double y = Y[o], mu = mean[o], sd = std[o];
        const double r = y - mu;
        se += r * r;
        sy += y * y;
        ls += -log(sd) - 0.5 * r * r / (sd * sd) - 0.91893853320467274;
    }
    se = wave_sum_d(se);
    sy = wave_sum_d(sy);
    ls = wave_sum_d(ls);
    if (lane == 0) { red[0][wid] = se; red[1][wid] = sy; red[2][wid] = ls; }
    __syncthreads();
    if (tid == 0) {
        const double a = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        const double b = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        const double c = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
        atomicAdd(out + 0, sqrt(a) / sqrt(b));
        atomicAdd(out + 1, c / (double)d_y);
    }
}

// per output p: 1 - sum_n (Y - mean)^2 / sum_n (Y - Ybar)^2 (one thread per output)
__global__ __launch_bounds__(256) void scores_cols_kernel(const float* Y, const float* mean, int n, int d_y,
                                                          double* out) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (p < d_y) {
        double yb = 0.0;
        for (int k = 0; k < n; ++k) yb += (double)Y[(int64_t)k * d_y + p];
        yb /= (double)n;
        double num = 0.0, den = 0.0;
        for (int k = 0; k < n; ++k) {
            const double y = Y[(int64_t)k * d_y + p];
            const double r = y - (double)mean[(int64_t)k * d_y + p], c = y - yb;
            num += r * r;
            den += c * c;
        }
        v = 1.0 - num / den;
    }
    v = wave_sum_d(v);
    if ((threadIdx.x & 63) == 0) atomicAdd(out + 2, v);
}

bool grid_of(int n_fine, int nc, FineGrid& G) {
    if (n_fine < 2 || nc < 1 || n_fine % nc) return false;
    G.n = n_fine;
    G.nc = nc;
    G.r = n_fine / nc;
    G.dy = (n_fine + 1) * (n_fine - 1);
    G.nn_c = (nc + 1) * (nc + 1);
    G.nT_c = 2 * nc * nc;
    return true;
}

}  // namespace

extern "C" int gpi_vo_rows(int32_t n_fine, int32_t nc, int32_t flags) {
    FineGrid G;
    if (!grid_of(n_fine, nc, G) || !(flags & (GPI_VO_CGR | GPI_VO_FLUX)) || (flags & ~(GPI_VO_CGR | GPI_VO_FLUX)))
        return GPI_ERR_ARG;
    return ((flags & GPI_VO_CGR) ? G.nn_c : 0) + ((flags & GPI_VO_FLUX) ? G.nT_c : 0);
}

extern "C" int gpi_vo_query(const gpi_vo_query_desc* d, void* stream) {
    if (!d || !d->logkappa || !d->bc || !d->gamma || !d->alpha || d->n < 0) return GPI_ERR_ARG;
    const int m = gpi_vo_rows(d->n_fine, d->nc, d->flags);
    if (m < 0) return m;
    if (d->n == 0) return GPI_OK;
    FineGrid G;
    grid_of(d->n_fine, d->nc, G);
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(vo_query_columns, dim3((G.dy + 255) / 256, d->n), dim3(256), sizeof(double) * G.nn_c, st, *d,
                       G, m);
    GPI_CHECK_LAUNCH();
    if (d->flags & GPI_VO_FLUX) {
        const int row0 = (d->flags & GPI_VO_CGR) ? G.nn_c : 0;
        hipLaunchKernelGGL(vo_query_flux, dim3((G.nT_c + 63) / 64, d->n), dim3(64), 0, st, *d, G, m, row0);
        GPI_CHECK_LAUNCH();
    }
    return GPI_OK;
}

extern "C" int gpi_vo_moments(const gpi_vo_moments_desc* d, void* stream) {
    FineGrid G;
    if (!d || !d->uc || !d->mean || d->n < 0 || d->n_mc < 2 || d->refine < 1) return GPI_ERR_ARG;
    if (!grid_of(d->nc * d->refine, d->nc, G)) return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    const size_t lds = sizeof(float) * MOM_CH * G.nn_c;
    if (lds > 64 * 1024) return GPI_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(vo_moments_kernel, dim3((G.dy + 255) / 256, d->n), dim3(256), lds, (hipStream_t)stream, *d,
                       G);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

static bool sparse_ok(const gpi_vo_sparse& sp, int m) {
    return sp.r >= 1 && sp.r <= VS_R && sp.n_pairs >= m && sp.rows && sp.vals && sp.pair_ptr && sp.pair_ab &&
           sp.pair_src && sp.row_ptr && sp.row_src;
}

extern "C" int gpi_vo_condition(const gpi_vo_condition_desc* d, void* stream) {
    if (!d || !d->alpha || !d->g || !d->prec || !d->vo_var || !d->lam || !d->solvec || !d->mean || !d->vars ||
        d->n < 0 || d->m < 1 || d->d_y < 1 || (!d->gamma && !d->sparse))
        return GPI_ERR_ARG;
    if (d->sparse && (!sparse_ok(*d->sparse, d->m) || !d->sparse->inv)) return GPI_ERR_ARG;
    if (d->m > VS_MAXM) return GPI_ERR_UNSUPPORTED;
    if (d->n == 0) return GPI_OK;
    const hipStream_t st = (hipStream_t)stream;
    const int T = (d->m + LT - 1) / LT;
    const size_t lds_small = sizeof(double) * ((size_t)d->m * d->m + d->m);
    if (d->sparse) {
        const gpi_vo_sparse sp = *d->sparse;
        if (hipMemsetAsync(d->lam, 0, sizeof(double) * (size_t)d->n * d->m * d->m, st) != hipSuccess)
            return GPI_ERR_LAUNCH;
        hipLaunchKernelGGL(vo_lambda_sparse_kernel, dim3((sp.n_pairs + 255) / 256, d->n), dim3(256), 0, st, *d, sp);
        GPI_CHECK_LAUNCH();
        hipLaunchKernelGGL(vo_rhs_sparse_kernel, dim3((d->m + 3) / 4, d->n), dim3(256), 0, st, *d, sp);
        GPI_CHECK_LAUNCH();
        if (lds_small <= 64 * 1024)
            hipLaunchKernelGGL(vo_chol_kernel<true>, dim3(d->n), dim3(256), lds_small, st, *d);
        else
            hipLaunchKernelGGL(vo_chol_kernel<false>, dim3(d->n), dim3(256), sizeof(double) * d->m, st, *d);
    } else {
        hipLaunchKernelGGL(vo_lambda_kernel, dim3(T * (T + 1) / 2, d->n), dim3(256), 0, st, *d);
        GPI_CHECK_LAUNCH();
        if (lds_small <= 64 * 1024) {
            hipLaunchKernelGGL(vo_chol_kernel<true>, dim3(d->n), dim3(256), lds_small, st, *d);
        } else {
            hipLaunchKernelGGL(vo_rhs_kernel, dim3(d->m, d->n), dim3(256), 0, st, *d);
            GPI_CHECK_LAUNCH();
            hipLaunchKernelGGL(vo_chol_kernel<false>, dim3(d->n), dim3(256), sizeof(double) * d->m, st, *d);
        }
    }
    GPI_CHECK_LAUNCH();
    if (d->m <= 256) {
        const int nb = (d->m + TI - 1) / TI;
        hipLaunchKernelGGL(vo_linv_block_kernel, dim3(nb, d->n), dim3(256), sizeof(double) * nb * TI * (TI + 1), st,
                           *d);
    } else {
        hipLaunchKernelGGL(vo_linv_kernel, dim3(d->n), dim3(256), 0, st, *d);
    }
    GPI_CHECK_LAUNCH();
    if (lds_small > 64 * 1024) hipLaunchKernelGGL(vo_solvec_kernel, dim3(d->n), dim3(256), 0, st, *d);
    GPI_CHECK_LAUNCH();
    if (d->sparse) {
        const gpi_vo_sparse sp = *d->sparse;
        hipLaunchKernelGGL(vo_inv_kernel, dim3(T * (T + 1) / 2, d->n), dim3(256), 0, st, *d, sp);
        GPI_CHECK_LAUNCH();
        hipLaunchKernelGGL(vo_columns_sparse_kernel, dim3((d->d_y + 255) / 256, d->n), dim3(256), 0, st, *d, sp);
    } else {
        hipLaunchKernelGGL(vo_columns_kernel, dim3((d->d_y + VC_BN - 1) / VC_BN, d->n), dim3(256), 0, st, *d);
    }
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_vo_pattern(const double* gamma, int32_t n, int32_t m, int32_t d_y, int32_t r, int32_t* rows,
                              int32_t* count, uint8_t* work, void* stream) {
    if (!gamma || !rows || !count || !work || n < 1 || m < 1 || d_y < 1 || r < 1) return GPI_ERR_ARG;
    const hipStream_t st = (hipStream_t)stream;
    const int64_t md = (int64_t)m * d_y;
    hipLaunchKernelGGL(vo_nz_kernel, dim3((unsigned)((md + 255) / 256)), dim3(256), 0, st, gamma, n, m, d_y, work);
    GPI_CHECK_LAUNCH();
    hipLaunchKernelGGL(vo_pattern_kernel, dim3((d_y + 255) / 256), dim3(256), 0, st, work, m, d_y, r, rows, count);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_vo_sparse_values(const double* gamma, int32_t n, int32_t m, int32_t d_y, const gpi_vo_sparse* sp,
                                    void* stream) {
    if (!gamma || !sp || !sp->rows || !sp->vals || sp->r < 1 || n < 0 || m < 1 || d_y < 1) return GPI_ERR_ARG;
    if (n == 0) return GPI_OK;
    hipLaunchKernelGGL(vo_sparse_values_kernel, dim3((d_y + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, gamma,
                       n, m, d_y, *sp);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_vo_precision(const gpi_vo_precision_desc* d, void* stream) {
    if (!d || (!d->gamma && !d->sparse) || !d->alpha || !d->mean || !d->vars || !d->beta || !d->vo_var || d->n < 0 ||
        d->m < 1 || d->d_y < 1 || (d->n > 0 && !d->terms))
        return GPI_ERR_ARG;
    if (d->sparse && !sparse_ok(*d->sparse, d->m)) return GPI_ERR_ARG;
    const hipStream_t st = (hipStream_t)stream;
    if (d->n > 0) {
        if (d->sparse)
            hipLaunchKernelGGL(vo_precision_sparse_kernel, dim3(d->m, (d->n + 3) / 4), dim3(256), 0, st, *d,
                               *d->sparse);
        else
            hipLaunchKernelGGL(vo_precision_kernel, dim3(d->m, d->n), dim3(256), 0, st, *d);
        GPI_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(vo_precision_final, dim3((d->m + 255) / 256), dim3(256), 0, st, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_gauss_sample(float* out, const float* mean, const float* logsigma, int64_t rows, int32_t dim,
                                int32_t rep, const float* eps, uint64_t seed, const uint64_t* offset, uint64_t sub,
                                void* stream) {
    if (!out || !mean || !logsigma || rows < 0 || dim < 1 || rep < 1) return GPI_ERR_ARG;
    const int64_t total = rows * dim;
    if (total == 0) return GPI_OK;
    hipLaunchKernelGGL(gauss_sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, out, mean, logsigma, total, dim, rep, eps, seed, offset, sub);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_gp_sample(const gpi_gp_sample_desc* d, void* stream) {
    if (!d || !d->qz_mu || !d->qz_ls || !d->gp_w || !d->gp_b || !d->x || d->rows < 0 || d->rep < 1 || d->d_z < 1 ||
        d->d_z > 512 || d->d_x < 1)
        return GPI_ERR_ARG;
    if (d->rows == 0) return GPI_OK;
    hipLaunchKernelGGL(gp_sample_kernel, dim3(d->rows), dim3(GPT), 0, (hipStream_t)stream, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_predictive_scores(const float* Y, const float* mean, const float* std, int32_t n, int32_t d_y,
                                     double* out, void* stream) {
    if (!Y || !mean || !std || !out || n < 1 || d_y < 1) return GPI_ERR_ARG;
    const hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, 3 * sizeof(double), st) != hipSuccess) return GPI_ERR_LAUNCH;
    hipLaunchKernelGGL(scores_rows_kernel, dim3(n), dim3(256), 0, st, Y, mean, std, d_y, out);
    GPI_CHECK_LAUNCH();
    hipLaunchKernelGGL(scores_cols_kernel, dim3((d_y + 255) / 256), dim3(256), 0, st, Y, mean, n, d_y, out);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_vo_galerkin(const gpi_vo_galerkin_desc* d, void* stream) {
    if (!d || !d->logkappa || !d->bc || !d->gamma || !d->alpha || d->n < 0 || d->n_fine < 2 || d->m_aux < 1 ||
        d->row0 < 0 || d->row0 + d->m_aux > d->m || (d->kind != GPI_VO_TEST_GAUSS && d->kind != GPI_VO_TEST_RBF) ||
        (d->kind == GPI_VO_TEST_RBF && !d->V && !(d->length > 0.0)))
        return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    const int dy = (d->n_fine + 1) * (d->n_fine - 1);
    hipLaunchKernelGGL(vo_galerkin_kernel, dim3((dy + 255) / 256, d->m_aux, d->n), dim3(256), 0, (hipStream_t)stream,
                       *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
