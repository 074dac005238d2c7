// Fine-grid coarse-grained residual (CGR) as a matrix-free 5-point stencil.
//
// Reference: CoarseGrainedResidualSampler builds, once per VO sample,
//   Gamma = W^T K_ff(kappa),  alpha = W^T f_eff   (VirtualObservables.py:57-69,297-321)
// with FEniCS assembly + scipy slicing (physics/LinearElliptic.py:137-159),
// and update_vo_precision evaluates Gamma y - alpha (VirtualObservables.py:990).
// Since f_eff = -K_fc g (zero source), Gamma y - alpha = W^T [K yhat]_free with
// yhat = y on free nodes and the Dirichlet data g on x=0 / x=1; K is the
// 5-point stencil with edge conductances c = (kappa_a + kappa_b)/2 of the two
// pixels sharing the edge (kappa/2 on boundary edges).  One workgroup per
// field; exp(logkappa) staged in LDS; coarse sums accumulated in fp64 LDS.
//
// Flux residual (FluxConstrainSampler, VirtualObservables.py:323-349 +
// FluxConstraintReducedOrderModel, bottleneck/flux.py:81-158): r_fc = Gamma_fc y with
// alpha_fc = 0 (flux.py:153 quirk); row k = outward flux of kappa grad(u) over the
// fine facets on the boundary of coarse triangle k (edges on y=0 / y=1 excluded: dS
// over boundary facets), u = y on free nodes and 0 on the Dirichlet nodes (the reduced
// Gamma keeps free columns only).  Same closed forms as vo.hip's vo_query_flux.
#include "common.h"

using namespace gpi;

namespace {

__device__ __forceinline__ float bcval(const float* u, int i, int j, int n) {
    const float y = (float)j / (float)n;
    return i == 0 ? (u[0] * (1.f - y) + u[1] * y) : (u[2] * (1.f - y) + u[3] * y);
}

__global__ __launch_bounds__(256) void cgr_kernel(gpi_residual_desc d) {
    extern __shared__ __attribute__((aligned(16))) double smd[];
    const int n = d.n_fine, nc = d.nc, nn = (nc + 1) * (nc + 1);
    const int r = n / nc;
    double* acc = smd;                                  // [nn]
    float* kp = (float*)(smd + nn + 2 * nc * nc);       // [n*n] kappa by square (i + n j)
    const int f = blockIdx.x;
    const float* lk = d.logkappa + (int64_t)f * n * n;
    const float* y = d.y + (int64_t)f * (n + 1) * (n - 1);
    const float* u = d.bc + 4 * f;
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const int row = e / n, col = e - row * n;      // image pixel (row 0 = top)
        kp[col + n * (n - 1 - row)] = expf(lk[e]);
    }
    for (int e = threadIdx.x; e < nn; e += 256) acc[e] = 0.0;
    __syncthreads();
    const int dy = (n + 1) * (n - 1);
    for (int p = threadIdx.x; p < dy; p += 256) {
        const int j = p / (n - 1), i = p - j * (n - 1) + 1;
        const float yc = y[p];
        auto yhat = [&](int ii, int jj) -> float {
            if (ii == 0 || ii == n) return bcval(u, ii, jj, n);
            return y[jj * (n - 1) + ii - 1];
        };
        auto K = [&](int ii, int jj) -> float { return kp[ii + n * jj]; };
        // horizontal neighbours (i-1, j), (i+1, j)
        float ch_l = 0.f, ch_r = 0.f, cv_d = 0.f, cv_u = 0.f;
        if (j < n) { ch_l += K(i - 1, j); ch_r += K(i, j); }
        if (j > 0) { ch_l += K(i - 1, j - 1); ch_r += K(i, j - 1); }
        if (j > 0) { cv_d = K(i - 1, j - 1) + K(i, j - 1); }
        if (j < n) { cv_u = K(i - 1, j) + K(i, j); }
        float Ky = 0.5f * (ch_l * (yc - yhat(i - 1, j)) + ch_r * (yc - yhat(i + 1, j)));
        if (j > 0) Ky += 0.5f * cv_d * (yc - yhat(i, j - 1));
        if (j < n) Ky += 0.5f * cv_u * (yc - yhat(i, j + 1));
        // restriction W^T: closed-form P1 weights
        int I = i / r, J = j / r;
        if (I > nc - 1) I = nc - 1;
        if (J > nc - 1) J = nc - 1;
        const float xi = (float)(i - I * r) / (float)r, eta = (float)(j - J * r) / (float)r;
        const int n00 = I + (nc + 1) * J, n11 = n00 + (nc + 1) + 1;
        int n10;
        float w0, w1, w2;
        if (xi >= eta) { n10 = n00 + 1; w0 = 1.f - xi; w1 = xi - eta; w2 = eta; }
        else { n10 = n00 + (nc + 1); w0 = 1.f - eta; w1 = eta - xi; w2 = xi; }
        if (w0 != 0.f) atomicAdd(&acc[n00], (double)(w0 * Ky));
        if (w1 != 0.f) atomicAdd(&acc[n10], (double)(w1 * Ky));
        if (w2 != 0.f) atomicAdd(&acc[n11], (double)(w2 * Ky));
    }
    __syncthreads();
    if (d.r)
        for (int e = threadIdx.x; e < nn; e += 256) d.r[(int64_t)f * nn + e] = (float)acc[e];
    if (!d.r_flux) return;
    // ---- flux rows: one task per (coarse triangle, edge), r facets each
    const int nT = 2 * nc * nc;
    double* racc = acc + nn;                            // [nT]
    for (int e = threadIdx.x; e < nT; e += 256) racc[e] = 0.0;
    __syncthreads();
    auto uf = [&](int ii, int jj) -> float {            // free value, 0 on Dirichlet nodes
        return (ii < 1 || ii > n - 1) ? 0.f : y[jj * (n - 1) + ii - 1];
    };
    for (int task = threadIdx.x; task < 3 * nT; task += 256) {
        const int k = task / 3, e = task - 3 * k;
        const int Q = k >> 1, ul = k & 1;
        const int I = Q % nc, J = Q / nc;
        if (ul == 0 && e == 0 && J == 0) continue;          // bottom edge on y = 0
        if (ul == 1 && e == 1 && J == nc - 1) continue;     // top edge on y = 1
        float s = 0.f;
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
            const float u0 = uf(i, j), u1 = uf(i + 1, j), u2 = uf(i, j + 1), u3 = uf(i + 1, j + 1);
            float v;
            if (ul == 0) v = e == 0 ? u1 - u3 : (e == 1 ? u1 - u0 : u0 - 2.f * u1 + u3);
            else v = e == 0 ? u2 - u3 : (e == 1 ? u2 - u0 : u0 - 2.f * u2 + u3);
            s = fmaf(kp[i + n * j], v, s);
        }
        atomicAdd(&racc[k], (double)s);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nT; e += 256) d.r_flux[(int64_t)f * nT + e] = (float)racc[e];
}

}  // namespace

extern "C" int gpi_cgr_residual(const gpi_residual_desc* d, void* stream) {
    if (!d || !d->logkappa || !d->y || !d->bc || (!d->r && !d->r_flux) || d->nc < 1 || d->n_fine < 2 || d->n < 0)
        return GPI_ERR_ARG;
    if (d->n_fine % d->nc) return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    const int nn = (d->nc + 1) * (d->nc + 1);
    const size_t lds = sizeof(double) * (nn + 2 * d->nc * d->nc) + sizeof(float) * d->n_fine * d->n_fine;
    if (lds > 160 * 1024) return GPI_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(cgr_kernel, dim3(d->n), dim3(256), lds, (hipStream_t)stream, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
