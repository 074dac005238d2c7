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
// field (layout in cgr_kernel); coarse sums accumulated in fp64 LDS.
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

// One workgroup per field, one wave per coarse row band J (fine rows J r .. J r + r - 1, plus the
// top row j = n in the last band); lanes run over the fine columns in chunks of 64 (coalesced y /
// log kappa loads, re-reads of neighbours served by L1/L2), each lane keeps the W^T-restricted
// contributions of its nodes to the four corners of its coarse square in registers over the
// band's rows, then groups of G = min(r, 64) lanes (one coarse square per group when r is a power
// of two; G = 1 otherwise) reduce by shuffles and one lane adds 4 fp64 values per square into
// LDS.  No field-sized LDS staging: every grid size runs (256^2 included).
constexpr int CGR_MAXW = 8;      // waves per workgroup (bands beyond loop)
constexpr int CGR_MAXM = 8;      // 64-column chunks per row (n <= 512)

// FLUX: the flux rows in the same pass -- pixel (i, j) of the band adds kappa_ij * (u-differences
// of its corners) to the rows of its coarse square's two triangles when it lies on one of their
// edges (the per-task sums of the reference's facet loops, flux.py:99-158), so the field is read once.
template <int MM, bool FLUX>   // MM: 64-column chunks per row, ceil(n / 64)
__global__ __launch_bounds__(64 * CGR_MAXW) void cgr_kernel(gpi_residual_desc d, int G) {
    extern __shared__ __attribute__((aligned(16))) double smd[];
    const int n = d.n_fine, nc = d.nc, nn = (nc + 1) * (nc + 1);
    const int r = n / nc;
    const float rinv = 1.f / (float)r;
    double* acc = smd;                                  // [nn]
    double* racc = smd + nn;                            // [2 nc^2]
    const int f = blockIdx.x;
    const float* lk = d.logkappa + (int64_t)f * n * n;
    const float* y = d.y + (int64_t)f * (n + 1) * (n - 1);
    const float* u = d.bc + 4 * f;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int e = threadIdx.x; e < nn + 2 * nc * nc; e += blockDim.x) smd[e] = 0.0;
    __syncthreads();
    // kappa of square (a, b) (b counted from the bottom; image row 0 = top)
    auto K = [&](int a, int b) -> float { return expf(lk[(n - 1 - b) * n + a]); };
    auto yhat = [&](int ii, int jj) -> float {
        if (ii == 0 || ii == n) return bcval(u, ii, jj, n);
        return y[jj * (n - 1) + ii - 1];
    };
    for (int J = wave; J < nc; J += nw) {
        float c[MM][4];
        // carried across the band's rows: kappa of the squares below the row (kd*), y of the rows
        // below (yd), at (yc) and above (yu): per node 2 kappa loads (+ exp) and 3 y loads
        float kdl[MM], kdr[MM], yd[MM], yc[MM], yu[MM];
        float flr[MM], ful[MM];        // flux rows of the square's lower-right / upper-left triangle
        const int j0 = J * r, j1 = J == nc - 1 ? n : (J + 1) * r - 1;
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            c[m][0] = c[m][1] = c[m][2] = c[m][3] = 0.f;
            flr[m] = ful[m] = 0.f;
            const int i = 64 * m + lane;
            const bool act = i >= 1 && i <= n - 1;
            kdl[m] = (act && j0 > 0) ? K(i - 1, j0 - 1) : 0.f;
            kdr[m] = (i < n && j0 > 0) ? K(i, j0 - 1) : 0.f;
            yc[m] = act ? y[j0 * (n - 1) + i - 1] : 0.f;
            yd[m] = (act && j0 > 0) ? y[(j0 - 1) * (n - 1) + i - 1] : 0.f;
        }
#pragma unroll 2
        for (int j = j0; j <= j1; ++j) {
            const float eta = (float)(j - j0) * rinv;
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                const int i = 64 * m + lane;
                const bool act = i >= 1 && i <= n - 1;
                const bool pix = i < n && j < n;              // pixel (i, j) (FLUX; i = 0 included)
                const float kul = (act && j < n) ? K(i - 1, j) : 0.f;
                const float kur = ((FLUX ? pix : act) && j < n) ? K(i, j) : 0.f;
                yu[m] = (act && j < n) ? y[(j + 1) * (n - 1) + i - 1] : 0.f;
                const bool rf = i + 1 <= n - 1;                // right neighbour is a free node
                const float yR = (FLUX ? (i < n && rf) : (act && rf)) ? y[j * (n - 1) + i] : 0.f;
                const float yl = act ? yhat(i - 1, j) : 0.f;
                const float yr = act ? (rf ? yR : bcval(u, n, j, n)) : 0.f;
                const float ycm = yc[m], ydm = yd[m];
                float Ky = (kul + kdl[m]) * (ycm - yl) + (kur + kdr[m]) * (ycm - yr);
                if (j > 0) Ky += (kdl[m] + kdr[m]) * (ycm - ydm);
                if (j < n) Ky += (kul + kur) * (ycm - yu[m]);
                Ky = act ? 0.5f * Ky : 0.f;
                int I = i / r;
                if (I > nc - 1) I = nc - 1;
                const float xi = (float)(i - I * r) * rinv;
                if (xi >= eta) {
                    c[m][0] += (1.f - xi) * Ky; c[m][1] += (xi - eta) * Ky; c[m][3] += eta * Ky;
                } else {
                    c[m][0] += (1.f - eta) * Ky; c[m][2] += (eta - xi) * Ky; c[m][3] += xi * Ky;
                }
                if (FLUX && pix) {
                    const float u0 = act ? ycm : 0.f, u1 = yR, u2 = act ? yu[m] : 0.f;
                    const float u3 = rf ? y[(j + 1) * (n - 1) + i] : 0.f;
                    const int tr = i - (i / r) * r, tj = j - j0;
                    float vl = 0.f, vu = 0.f;
                    if (tj == 0 && J > 0) vl += u1 - u3;             // bottom edge (not on y = 0)
                    if (tr == r - 1) vl += u1 - u0;                  // right edge
                    if (tr == 0) vu += u2 - u3;                      // left edge
                    if (tj == r - 1 && J < nc - 1) vu += u2 - u0;    // top edge (not on y = 1)
                    if (tr == tj) { vl += u0 - 2.f * u1 + u3; vu += u0 - 2.f * u2 + u3; }   // diagonal
                    flr[m] = fmaf(kur, vl, flr[m]);
                    ful[m] = fmaf(kur, vu, ful[m]);
                }
                kdl[m] = kul; kdr[m] = kur;
                yd[m] = ycm; yc[m] = yu[m];
            }
        }
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            for (int o = 1; o < G; o <<= 1)
#pragma unroll
                for (int k = 0; k < 4; ++k) c[m][k] += __shfl_xor(c[m][k], o, 64);
            if (FLUX)
                for (int o = 1; o < G; o <<= 1) {
                    flr[m] += __shfl_xor(flr[m], o, 64);
                    ful[m] += __shfl_xor(ful[m], o, 64);
                }
            const int i = 64 * m + lane;
            if ((lane % G) == 0 && i < n) {
                int I = i / r;
                if (I > nc - 1) I = nc - 1;
                const int v0 = I + (nc + 1) * J;
                atomicAdd(&acc[v0], (double)c[m][0]);
                atomicAdd(&acc[v0 + 1], (double)c[m][1]);
                atomicAdd(&acc[v0 + nc + 1], (double)c[m][2]);
                atomicAdd(&acc[v0 + nc + 2], (double)c[m][3]);
                if (FLUX) {
                    const int q = I + nc * J;
                    atomicAdd(&racc[2 * q], (double)flr[m]);
                    atomicAdd(&racc[2 * q + 1], (double)ful[m]);
                }
            }
        }
    }
    __syncthreads();
    if (d.r)
        for (int e = threadIdx.x; e < nn; e += blockDim.x) d.r[(int64_t)f * nn + e] = (float)acc[e];
    if (!FLUX) return;
    const int nT = 2 * nc * nc;
    for (int e = threadIdx.x; e < nT; e += blockDim.x) d.r_flux[(int64_t)f * nT + e] = (float)racc[e];
}

template <int MM>
void launch_cgr(const gpi_residual_desc& d, int G, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
    if (d.r_flux) hipLaunchKernelGGL((cgr_kernel<MM, true>), grid, block, lds, st, d, G);
    else hipLaunchKernelGGL((cgr_kernel<MM, false>), grid, block, lds, st, d, G);
}

}  // namespace

extern "C" int gpi_cgr_residual(const gpi_residual_desc* d, void* stream) {
    if (!d || !d->logkappa || !d->y || !d->bc || (!d->r && !d->r_flux) || d->nc < 1 || d->n_fine < 2 || d->n < 0)
        return GPI_ERR_ARG;
    if (d->n_fine % d->nc) return GPI_ERR_ARG;
    if (d->n_fine > 64 * CGR_MAXM) return GPI_ERR_UNSUPPORTED;
    if (d->n == 0) return GPI_OK;
    const int nn = (d->nc + 1) * (d->nc + 1);
    const size_t lds = sizeof(double) * (nn + 2 * d->nc * d->nc);
    if (lds > 160 * 1024) return GPI_ERR_UNSUPPORTED;
    const int r = d->n_fine / d->nc;
    const int G = (r & (r - 1)) == 0 ? (r < 64 ? r : 64) : 1;   // lanes per coarse square (see cgr_kernel)
    const int waves = d->nc < CGR_MAXW ? d->nc : CGR_MAXW;
    const int M = (d->n_fine + 63) / 64;
    const dim3 grid(d->n), block(64 * waves);
    const hipStream_t st = (hipStream_t)stream;
    if (M == 1) launch_cgr<1>(*d, G, grid, block, lds, st);
    else if (M == 2) launch_cgr<2>(*d, G, grid, block, lds, st);
    else if (M <= 4) launch_cgr<4>(*d, G, grid, block, lds, st);
    else launch_cgr<8>(*d, G, grid, block, lds, st);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
