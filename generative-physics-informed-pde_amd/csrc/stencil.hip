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
#include <stdlib.h>
#include <type_traits>

using namespace gpi;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// Streaming form (16-B aligned fields, n % 16 == 0, 16 <= n <= 256, r = n / nc a power of two >= 4: 32^2 ...
// 256^2 at nc = 8).  One workgroup of NT = 4 n threads per field walks the field bottom-up in chunks of CR = 16
// node rows.  Every thread loads ONE float4 of log kappa and ONE float4 of y per chunk, DEPTH chunks ahead of
// the one it consumes, takes exp once per pixel and scatters both into LDS rows: three chunk slots of 16 rows,
// pitch n + 4, column i of a row at 1 + i.  y rows carry yhat: the Dirichlet data of columns 0 and n are written
// next to the free values, so the stencil needs no boundary branch; the pad columns (-1, n + 1, n + 2) stay
// zero.  After one barrier per chunk, thread (ro, q) computes the 4 nodes i0 = 4q .. 4q + 3 of node row
// j = 16 s - 1 + ro from 16-B LDS reads (3 y rows, 2 kappa rows), restricts them with W^T -- the four are in one
// coarse square, r % 4 == 0; the P1 weights by min / max, no branch -- and adds the square's four corner sums
// (after a shuffle over the r / 4 threads of the square's row) into fp64 LDS accumulators.  The arithmetic per
// node is cgr_kernel's (same products, same order).  Chunk s + 1 is written into the slot of chunk s - 2,
// which no thread reads after the barrier of chunk s: one barrier per chunk.
constexpr int CGRS_CR = 16;        // node rows per chunk
#ifndef GPI_CGR_DEPTH
#define GPI_CGR_DEPTH 2            // chunks in flight ahead of the one computed
#endif
__host__ __device__ inline int cgrs_pitch(int n) { return n + 4; }
template <int DEPTH, bool FLUX, int NS>   // NS > 0: the chunk count n / 16 + 1 at compile time (loop fully
                                         // unrolled: exact wait counts, every chunk's loads DEPTH chunks ahead)
__global__ __launch_bounds__(1024) void cgr_stream_kernel(gpi_residual_desc d, int lr) {
    extern __shared__ __attribute__((aligned(16))) double smd[];
    const int n = d.n_fine, nc = d.nc, nn = (nc + 1) * (nc + 1), nT = 2 * nc * nc;
    const int r = 1 << lr;
    const float rinv = 1.f / (float)r;
    const int NT = blockDim.x, tid = threadIdx.x;
    const int PT = cgrs_pitch(n), SLOT = CGRS_CR * PT;
    double* acc = smd;                                   // [nn]
    double* racc = smd + nn;                             // [nT]
    float* kr = (float*)(smd + ((nn + nT + 1) & ~1));    // kappa rows [3 slots][16][PT] (16-B aligned)
    float* yr = kr + 3 * SLOT;                           // y rows, the same layout
    const int f = blockIdx.x;
    const int ny = (n + 1) * (n - 1);                    // y values per field
    const float* lk = d.logkappa + (int64_t)f * n * n;
    const int64_t ybase = (int64_t)f * ny;
    const int64_t ytotal = (int64_t)d.n * ny;
    const float u0b = d.bc[4 * f], u1b = d.bc[4 * f + 1], u2b = d.bc[4 * f + 2], u3b = d.bc[4 * f + 3];
    for (int e = tid; e < nn + nT; e += NT) smd[e] = 0.0;
    for (int e = tid; e < (6 * SLOT + PT) / 4; e += NT) reinterpret_cast<f32x4*>(kr)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();                                     // (the pads stay zero; chunk stores come after)
    const int nsteps = NS > 0 ? NS : n / CGRS_CR + 1;   // chunk s: kappa pixel rows / y node rows [16 s, 16 s + 16)
    const int npr = n >> 2;                              // threads per row (4 columns each)
    const int ro = tid / npr, q = tid - ro * npr;
    // (branch-free: every thread issues all loads of every chunk -- clamped to a valid address where the
    // chunk has no such data -- so the compiler's wait counts stay exact and the prefetch stays in flight)
    // y: thread (ro, q) loads the free values 4 q .. 4 q + 3 (columns 4 q + 1 .. 4 q + 4) of node row 16 s + ro by
    // four dword loads (rows of n - 1 floats are not 16-B aligned); the last one of q = n / 4 - 1 is column n,
    // whose Dirichlet value it writes instead
    const int64_t ylast = ytotal - 1;
    auto load_chunk = [&](int s, f32x4& kv, f32x4& yv) {
        const int b0 = s * CGRS_CR;
        // pixel rows [b0, b0 + 16) = image rows [n - b0 - 16, n - b0): one contiguous run
        const int kro = b0 < n ? n - b0 - CGRS_CR : 0;
        kv = *(const f32x4*)(lk + kro * n + 4 * tid);
        const int jj = min(b0 + ro, n);
        const int64_t g = ybase + (int64_t)jj * (n - 1) + 4 * q;
#pragma unroll
        for (int k = 0; k < 4; ++k) yv[k] = d.y[min(g + k, ylast)];
    };
    // LDS position of column i (-1 .. n + 2) of node / pixel row j (>= 0); zrow: a zero row
    auto rowpos = [&](int j) -> int { return ((j >> 4) % 3) * SLOT + (j & 15) * PT + 1; };
    const int zrow = 6 * SLOT + 1;
    const float fn = (float)n;
    auto bcv = [&](int i, int j) -> float {
        const float t = (float)j / fn;
        return i == 0 ? (u0b * (1.f - t) + u1b * t) : (u2b * (1.f - t) + u3b * t);
    };
    constexpr float LOG2E = 1.4426950408889634f;
    auto store_chunk = [&](int s, const f32x4& kv, const f32x4& yv) {
        const int b0 = s * CGRS_CR;
        if (b0 < n) {
            const int q4 = tid / npr;
            const int pb = b0 + CGRS_CR - 1 - q4;                       // pixel row (from the bottom) of image row
            const int a = 4 * (tid - q4 * npr);                         // n - b0 - 16 + q4
            float* p = kr + rowpos(pb) + a;
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k] = __builtin_amdgcn_exp2f(kv[k] * LOG2E);
        }
        const int jj = b0 + ro;
        if (jj <= n) {
            float* p = yr + rowpos(jj) + 4 * q + 1;                     // column 4 q + 1 (8-B aligned)
            f32x4 v = yv;
            if (q == npr - 1) v[3] = bcv(n, jj);
            *(f32x2*)p = f32x2{v[0], v[1]};
            *(f32x2*)(p + 2) = f32x2{v[2], v[3]};
            if (q == 0) p[-1] = bcv(0, jj);
        }
    };
    f32x4 kb[DEPTH], yb[DEPTH];
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) load_chunk(u, kb[u], yb[u]);
    const int i0 = 4 * q;
    const int I = i0 >> lr;                              // < nc (i0 + 3 < n)
    const int tr0 = i0 - (I << lr);
    const int lanes_sq = r >> 2;                         // threads of one square's row (consecutive lanes)
#pragma unroll
    for (int s0 = 0; s0 < (NS > 0 ? NS : nsteps); s0 += DEPTH) {
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) {
            const int s = s0 + u;
            if (s < nsteps) store_chunk(s, kb[u], yb[u]);     // (uniform)
            load_chunk(s + DEPTH, kb[u], yb[u]);              // (past the last chunk: clamped, unused)
            __syncthreads();
            // node rows of this chunk: [16 s - 1, 16 s + 15) (the last chunk: [n - 1, n])
            const int j = s * CGRS_CR - 1 + ro;
            const bool rowok = s < nsteps && j >= 0 && j <= n && (s < nsteps - 1 || ro < 2);
            float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, flr = 0.f, ful = 0.f;
            int J = 0;
            if (rowok) {
                J = min(j >> lr, nc - 1);
                const int tj = j - J * r;
                const float eta = (float)tj * rinv;
                // row windows (columns i0 - 1 .. i0 + 6): yhat of rows j - 1, j, j + 1; kappa of pixel rows j - 1, j;
                // rows outside the field (y row -1 / n + 1, kappa row -1 / n) read the zero row
                const bool jdn = j > 0, jup = j < n;
                const int pc = rowpos(j) + i0 - 1;
                const int pd = (jdn ? rowpos(j - 1) : zrow) + i0 - 1, pu = (jup ? rowpos(j + 1) : zrow) + i0 - 1;
                const int pk = (jup ? rowpos(j) : zrow) + i0 - 1;
                const f32x4 yc0 = *(const f32x4*)(yr + pc), yd0 = *(const f32x4*)(yr + pd), yu0 = *(const f32x4*)(yr + pu);
                const f32x4 yc1 = *(const f32x4*)(yr + pc + 4), yd1 = *(const f32x4*)(yr + pd + 4),
                            yu1 = *(const f32x4*)(yr + pu + 4);
                const f32x4 kc0 = *(const f32x4*)(kr + pk), kd0 = *(const f32x4*)(kr + pd);
                const float kc4 = kr[pk + 4], kd4 = kr[pd + 4];
                const float yc[6] = {yc0[0], yc0[1], yc0[2], yc0[3], yc1[0], yc1[1]};
                const float yd[4] = {yd0[1], yd0[2], yd0[3], yd1[0]};
                const float yu[5] = {yu0[1], yu0[2], yu0[3], yu1[0], yu1[1]};
                const float kc[5] = {kc0[0], kc0[1], kc0[2], kc0[3], kc4};
                const float kd[5] = {kd0[0], kd0[1], kd0[2], kd0[3], kd4};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int i = i0 + t;
                    const bool act = t > 0 || i0 > 0;                   // i >= 1 (i <= n - 1 always)
                    const float kul = act ? kc[t] : 0.f, kur = kc[t + 1];
                    const float kdl = act ? kd[t] : 0.f, kdr = kd[t + 1];
                    const float ycm = act ? yc[t + 1] : 0.f, ydm = act ? yd[t] : 0.f, yum = act ? yu[t] : 0.f;
                    const float yl = act ? yc[t] : 0.f;                 // yhat(i - 1, j)
                    const float yrr = act ? yc[t + 2] : 0.f;            // yhat(i + 1, j)
                    // (rows outside the field: zero conductances, the terms add +-0)
                    float Ky = (kul + kdl) * (ycm - yl) + (kur + kdr) * (ycm - yrr);
                    Ky += (kdl + kdr) * (ycm - ydm);
                    Ky += (kul + kur) * (ycm - yum);
                    Ky = act ? 0.5f * Ky : 0.f;
                    const float xi = (float)(tr0 + t) * rinv;
                    c0 += (1.f - fmaxf(xi, eta)) * Ky;
                    c1 += fmaxf(xi - eta, 0.f) * Ky;
                    c2 += fmaxf(eta - xi, 0.f) * Ky;
                    c3 += fminf(xi, eta) * Ky;
                    if (FLUX && jup) {
                        const bool rf = i + 1 <= n - 1;
                        const float u0 = ycm, u1 = rf ? yc[t + 2] : 0.f, u2 = yum;
                        const float u3 = rf ? yu[t + 1] : 0.f;
                        const int tr = tr0 + t;
                        float vl = 0.f, vu = 0.f;
                        if (tj == 0 && J > 0) vl += u1 - u3;             // bottom edge (not on y = 0)
                        if (tr == r - 1) vl += u1 - u0;                  // right edge
                        if (tr == 0) vu += u2 - u3;                      // left edge
                        if (tj == r - 1 && J < nc - 1) vu += u2 - u0;    // top edge (not on y = 1)
                        if (tr == tj) { vl += u0 - 2.f * u1 + u3; vu += u0 - 2.f * u2 + u3; }   // diagonal
                        flr = fmaf(kur, vl, flr);
                        ful = fmaf(kur, vu, ful);
                    }
                }
            }
            // the r / 4 threads of one square's row are consecutive lanes (npr | 64 or 64 | npr)
            for (int o = 1; o < lanes_sq; o <<= 1) {
                c0 += __shfl_xor(c0, o, 64);
                c1 += __shfl_xor(c1, o, 64);
                c2 += __shfl_xor(c2, o, 64);
                c3 += __shfl_xor(c3, o, 64);
                if (FLUX) {
                    flr += __shfl_xor(flr, o, 64);
                    ful += __shfl_xor(ful, o, 64);
                }
            }
            if (rowok && (q & (lanes_sq - 1)) == 0) {
                const int v0 = I + (nc + 1) * J;
                atomicAdd(&acc[v0], (double)c0);
                atomicAdd(&acc[v0 + 1], (double)c1);
                atomicAdd(&acc[v0 + nc + 1], (double)c2);
                atomicAdd(&acc[v0 + nc + 2], (double)c3);
                if (FLUX && j < n) {
                    const int qq = I + nc * J;
                    atomicAdd(&racc[2 * qq], (double)flr);
                    atomicAdd(&racc[2 * qq + 1], (double)ful);
                }
            }
        }
    }
    __syncthreads();
    if (d.r)
        for (int e = tid; e < nn; e += NT) d.r[(int64_t)f * nn + e] = (float)acc[e];
    if (!FLUX) return;
    for (int e = tid; e < nT; e += NT) d.r_flux[(int64_t)f * nT + e] = (float)racc[e];
}

// Band form without barriers (nc <= 16 bands of r = n / nc rows, 64 * MM >= n columns): one wave per coarse
// row band, lane = column (MM columns per lane, 64 apart), rows in order with the band's rows loaded
// PF rows ahead into registers (the loop is unrolled: R rows, + 1 in the top band, at compile time), one exp
// per pixel, the row neighbours (kappa of pixel i - 1, yhat of nodes i -+ 1) by DPP wave shifts (the lane
// crossing a 64-column chunk edge takes its neighbour's value by readlane), the W^T-restricted contributions
// of a lane's nodes -- all in one coarse square over the band -- accumulated in registers over the band
// and reduced once at its end (shuffles over the square's r lanes, 4 fp64 LDS adds per square).  The
// arithmetic per node is cgr_kernel's.
__device__ __forceinline__ float dpp_shr1(float v, float in0) {      // lane l <- lane l - 1; lane 0 <- in0
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(in0), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_shl1(float v, float in63) {     // lane l <- lane l + 1; lane 63 <- in63
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(in63), __float_as_int(v), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_shr1_z(float v) {              // lane l <- lane l - 1; lane 0 <- 0
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lane_of(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// f(0), f(1), ..., f(N - 1) with compile-time arguments (a fully unrolled loop whatever the body's size)
template <int I, int N>
struct StaticFor {
    template <typename F>
    __device__ __forceinline__ static void run(F& f) {
        f(std::integral_constant<int, I>{});
        StaticFor<I + 1, N>::run(f);
    }
};
template <int N>
struct StaticFor<N, N> {
    template <typename F>
    __device__ __forceinline__ static void run(F&) {}
};
template <int N, typename F>
__device__ __forceinline__ void static_for(F& f) { StaticFor<0, N>::run(f); }

// FLUX, band rows r <= this: the edge terms as per-lane sums and the diagonal term at the band's end from five
// loads per lane; above, every term per row (the end loads hit r rows per square, uncoalesced, and the extra
// sums cost registers: both slower at r = 16 / 32, r05r)
#ifndef GPI_CGR_DIAG_END_R
#define GPI_CGR_DIAG_END_R 8
#endif
#ifndef GPI_CGR_PF
#define GPI_CGR_PF 4               // band rows loaded ahead (x columns per lane: 4 measured ahead of 8, r05f)
#endif
template <int R, int MM, bool FLUX>
__global__ __launch_bounds__(512) void cgr_band_kernel(gpi_residual_desc d) {
    extern __shared__ __attribute__((aligned(16))) double smd[];
    constexpr int PF0 = GPI_CGR_PF / MM > 2 ? GPI_CGR_PF / MM : 2;        // ~ the same bytes in flight per wave for any MM
    constexpr int PF = PF0 < R + 1 ? PF0 : R + 1;
    const int nc = d.nc, n = nc * R, nn = (nc + 1) * (nc + 1), nT = 2 * nc * nc;
    constexpr float rinv = 1.f / (float)R;
    double* acc = smd;
    double* racc = smd + nn;
    const int f = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int J = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // one wave per band (blockDim = 64 nc)
    const float* lk = d.logkappa + (int64_t)f * n * n;
    const float* y = d.y + (int64_t)f * (n + 1) * (n - 1);
    const float u0b = d.bc[4 * f], u1b = d.bc[4 * f + 1], u2b = d.bc[4 * f + 2], u3b = d.bc[4 * f + 3];
    for (int e = threadIdx.x; e < nn + nT; e += blockDim.x) smd[e] = 0.0;
    __syncthreads();
    const float rfn = 1.f / (float)n;
    const int j0 = J * R;
    const bool top = J == nc - 1;                                  // the top band also owns node row n
    // raw loads of band row jr (node row j = j0 + jr): kappa pixel row j (log), y node row j + 1; clamped
    // row addresses (branch-free: exact wait counts); the y lanes off the free columns (0, n and past n) read
    // past the buffer's end, i.e. 0, so no per-row lane masks (kappa of the lanes >= n is finite and only
    // reaches the non-free lanes, whose sums are dropped at the band's end)
    // buffer loads: the row in the (scalar) soffset, the column in a per-lane voffset fixed for the band, so
    // no per-row 64-bit addresses are held in registers across the unrolled rows
    const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)lk, (short)0, 4 * n * n, 0x00020000);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 4 * (n + 1) * (n - 1), 0x00020000);
    int vk[MM], vy[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        const int i = 64 * m + lane;
        vk[m] = 4 * min(i, n - 1);
        vy[m] = (i >= 1 && i <= n - 1) ? 4 * (i - 1) : 0x7ffffff0;   // out of range: the load returns 0
    }
    auto load_k = [&](int j, int m) -> float {
        const int jj = min(max(j, 0), n - 1);
        return __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rk, vk[m], 4 * (n - 1 - jj) * n, 0));
    };
    auto load_y = [&](int j, int m) -> float {
        const int jj = min(max(j, 0), n);
        return __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, vy[m], 4 * jj * (n - 1), 0));
    };
    float kraw[PF][MM], yraw[PF][MM];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            kraw[p][m] = load_k(j0 + p, m);
            yraw[p][m] = load_y(j0 + p + 1, m);
        }
    // carried rows: kappa of pixel row j - 1 (kd, and kdl = kd of pixel i - 1), y of rows j - 1 (yd) and j
    // (yc, free values only: 0 at the Dirichlet columns)
    float kd[MM], kdl[MM], yd[MM], yc[MM], kdd[MM];
    // per lane over the band: S = sum Ky, E = sum eta Ky, C1 = sum max(xi - eta, 0) Ky (Ky without its factor
    // 1/2); the four W^T weights of a node (1 - max(xi, eta), max(xi - eta, 0), max(eta - xi, 0), min(xi, eta))
    // follow from these and xi at the band's end (max(xi, eta) = eta + P, min(xi, eta) = eta - Q, Q = P - xi + eta)
    float c[MM][4], flr[MM], ful[MM];
    // FLUX, per lane over the band: fe1 = sum kur (u1 - u0) (the right-edge term), fe2 = sum kur (u2 - u3)
    // (left edge), and in flr / ful the bottom / top edge terms (band rows 0 / r - 1); the edge sums enter on
    // the edge lanes at the band's end, with the diagonal term (row tr = the lane's column in its square), whose
    // five operands are loaded there (L2 hits: the band has just streamed them)
    float fe1[MM], fe2[MM];
    constexpr bool DEND = R <= GPI_CGR_DIAG_END_R;
    {
        float kp[MM];
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            const int i = 64 * m + lane;
            const float k = expf(load_k(j0 - 1, m));
            kp[m] = (j0 > 0 && i < n) ? k : 0.f;
            const float a = load_y(j0 - 1, m), b = load_y(j0, m);
            yd[m] = j0 > 0 ? a : 0.f;
            yc[m] = b;
            c[m][0] = c[m][1] = c[m][2] = c[m][3] = 0.f;
            flr[m] = ful[m] = fe1[m] = fe2[m] = 0.f;
        }
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            kd[m] = kp[m];
            kdl[m] = dpp_shr1(kp[m], m > 0 ? lane_of(kp[m > 0 ? m - 1 : 0], 63) : 0.f);
            kdd[m] = kdl[m] + kd[m];
        }
    }
    // the Dirichlet data (x = 0: u0 + (u1 - u0) t, x = 1: u2 + (u3 - u2) t at t = j / n), linear in the band row
    // jr: per lane dA + dB jr on columns 0 and n (0 elsewhere), added to the free values; bra + brb jr the
    // right neighbour of the last chunk's lane 63 when 64 MM = n
    float dA[MM], dB[MM];
    const float dl = (u1b - u0b) * rfn, dr = (u3b - u2b) * rfn;
    const float bra = fmaf(dr, (float)j0, u2b), brb = dr;
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        const int i = 64 * m + lane;
        dA[m] = i == 0 ? fmaf(dl, (float)j0, u0b) : (i == n ? bra : 0.f);
        dB[m] = i == 0 ? dl : (i == n ? dr : 0.f);
    }
    auto row = [&](auto jr_c) {
        constexpr int jr = decltype(jr_c)::value;
        // (j and eta pass through an empty asm at the row's start, so the row's divisions, weights and
        // Dirichlet data are computed here, not hoisted to the kernel's top for every row at once)
        int j = j0 + jr;
        asm volatile("" : "+s"(j));
        const int p = jr % PF;
        float eta = (float)jr * rinv;
        asm volatile("" : "+v"(eta));
        float ku[MM], yu[MM], yhc[MM];
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            // kappa(i, j) = kur and y(i, j + 1) (free values); none above node row n (the top band's row R)
            ku[m] = jr == R ? 0.f : __builtin_amdgcn_exp2f(kraw[p][m] * 1.4426950408889634f);
            yu[m] = jr == R ? 0.f : yraw[p][m];
            // yhat of row j: the Dirichlet data at columns 0 and n
            yhc[m] = fmaf(dB[m], (float)jr, dA[m]) + yc[m];
        }
        const float br = fmaf(brb, (float)jr, bra);
        // the next row's loads into the freed slot
        if (jr + PF <= R) {
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                kraw[p][m] = load_k(j + PF, m);
                yraw[p][m] = load_y(j + PF + 1, m);
            }
        }
        // (keeps the scheduler from hoisting every row's loads to the top: PF rows in flight, not R)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            const int i = 64 * m + lane;
            // neighbours across the 64-column chunk edges
            const float yr_in = m < MM - 1 ? lane_of(yhc[m < MM - 1 ? m + 1 : 0], 0) : (64 * MM == n ? br : 0.f);
            // (the wave shifts run unconditionally: a DPP move under a lane condition became a branch; the
            // first chunk's take 0 at lane 0 by the DPP bound control, no extra move)
            const float sk = m > 0 ? dpp_shr1(ku[m], lane_of(ku[m > 0 ? m - 1 : 0], 63)) : dpp_shr1_z(ku[m]);
            const float sl = m > 0 ? dpp_shr1(yhc[m], lane_of(yhc[m > 0 ? m - 1 : 0], 63)) : dpp_shr1_z(yhc[m]);
            const float sr = dpp_shl1(yhc[m], yr_in);
            // no lane masks inside: every operand is finite, the rows below 0 / above n have kappa 0 (their
            // terms vanish), and the lanes off the free columns are zeroed once at the band's end
            const float kul = sk, kur = ku[m], kdlm = kdl[m], kdr = kd[m];
            const float ycm = yc[m], yl = sl, yrr = sr, ydm = yd[m], yum = yu[m];
            const float a = kul + kdlm, b = kur + kdr, dd = kul + kur, cc = kdd[m];
            // 2 Ky = (a + b + cc + dd) ycm - a yl - b yr - cc yd - dd yu, a + b + cc + dd = 2 (cc + dd)
            const float s4 = fmaf(a, yl, fmaf(b, yrr, fmaf(cc, ydm, dd * yum)));
            const float Ky = fmaf(2.f * (cc + dd), ycm, -s4);
            int I = i / R;
            if (I > nc - 1) I = nc - 1;
            const float xi = (float)(i - I * R) * rinv;
            c[m][0] += Ky;
            c[m][1] = fmaf(eta, Ky, c[m][1]);
            c[m][2] = fmaf(fmaxf(xi - eta, 0.f), Ky, c[m][2]);
            // u1 = y(i + 1, j), u3 = y(i + 1, j + 1): free values of the right neighbour (0 at column n)
            float u1 = 0.f, u3 = 0.f;
            if (FLUX) {
                const float y1_in = m < MM - 1 ? lane_of(yc[m < MM - 1 ? m + 1 : 0], 0) : 0.f;
                const float y3_in = m < MM - 1 ? lane_of(yu[m < MM - 1 ? m + 1 : 0], 0) : 0.f;
                u1 = dpp_shl1(yc[m], y1_in);
                u3 = dpp_shl1(yu[m], y3_in);
            }
            if (FLUX && DEND && jr < R) {      // (lanes >= n: their square's sums are never stored)
                const float u0 = ycm, u2 = yum;
                fe1[m] = fmaf(kur, u1 - u0, fe1[m]);            // right edge (tr = r - 1 lanes)
                fe2[m] = fmaf(kur, u2 - u3, fe2[m]);            // left edge (tr = 0 lanes)
                if (jr == 0 && J > 0) flr[m] = kur * (u1 - u3);          // bottom edge (not on y = 0)
                if (jr == R - 1 && J < nc - 1) ful[m] = fmaf(kur, u2 - u0, ful[m]);   // top edge (not on y = 1)
            }
            if (FLUX && !DEND && jr < R) {
                // r >= 16: every term per row (the edge sums as extra accumulators measured slower at r = 32)
                const float u0 = ycm, u2 = yum;
                const int tr = i - (i / R) * R;
                float vl = 0.f, vu = 0.f;
                if (jr == 0 && J > 0) vl += u1 - u3;             // bottom edge (not on y = 0)
                if (tr == R - 1) vl += u1 - u0;                  // right edge
                if (tr == 0) vu += u2 - u3;                      // left edge
                if (jr == R - 1 && J < nc - 1) vu += u2 - u0;    // top edge (not on y = 1)
                if (tr == jr) { vl += u0 - 2.f * u1 + u3; vu += u0 - 2.f * u2 + u3; }   // diagonal
                flr[m] = fmaf(kur, vl, flr[m]);
                ful[m] = fmaf(kur, vu, ful[m]);
            }
        }
        // (the accumulators pass through an empty asm at the row's end: the row's arithmetic runs here,
        // not sunk to the band's end with every row's operands held live until then)
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            asm volatile("" : "+v"(c[m][0]), "+v"(c[m][1]), "+v"(c[m][2]));
            if (FLUX) asm volatile("" : "+v"(flr[m]), "+v"(ful[m]));
            if (FLUX && DEND) asm volatile("" : "+v"(fe1[m]), "+v"(fe2[m]));
        }
        // carry: row j becomes the row below
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            kdl[m] = m > 0 ? dpp_shr1(ku[m], lane_of(ku[m > 0 ? m - 1 : 0], 63)) : dpp_shr1_z(ku[m]);   // (= sk: CSE)
            kd[m] = ku[m];
            kdd[m] = kdl[m] + kd[m];                                  // (= dd: CSE)
            yd[m] = yc[m];
            yc[m] = yu[m];
        }
    };
    static_for<R>(row);
    if (top) row(std::integral_constant<int, R>{});                // node row n (uniform branch)
    // the r lanes of one coarse square (r a power of two <= 64: one group of consecutive lanes; otherwise
    // lane by lane)
    constexpr int G = (R & (R - 1)) == 0 ? (R < 64 ? R : 64) : 1;
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        {
            const int i = 64 * m + lane;
            int I = i / R;
            if (I > nc - 1) I = nc - 1;
            const float xi = (float)(i - I * R) * rinv;
            const float h = (i >= 1 && i <= n - 1) ? 0.5f : 0.f;     // Ky's 1/2; the free columns only
            const float S = h * c[m][0], E = h * c[m][1], C1 = h * c[m][2];
            const float C2 = C1 - xi * S + E;
            c[m][0] = S - E - C1;
            c[m][1] = C1;
            c[m][2] = C2;
            c[m][3] = E - C2;
            if (FLUX && DEND) {
                const int tr = i - (i / R) * R;
                if (tr == R - 1) flr[m] += fe1[m];
                if (tr == 0) ful[m] += fe2[m];
                // the diagonal node (i, j0 + tr) of the lane's square: kappa(i, jd), y(i | i + 1, jd | jd + 1)
                const int jd = j0 + tr;
                {
                const int vy1 = (i + 1 >= 1 && i + 1 <= n - 1) ? 4 * i : 0x7ffffff0;
                const float kdg = __builtin_amdgcn_exp2f(
                    __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rk, vk[m] + 4 * (n - 1 - jd) * n, 0, 0)) *
                    1.4426950408889634f);
                // (per-lane rows: the row offset joins the VGPR offset, added as uint32 so that the sentinel of a
                // non-free column wraps to an out-of-range offset -- the load returns 0 -- without signed overflow)
                const uint32_t o0 = 4u * (uint32_t)jd * (uint32_t)(n - 1), o1 = o0 + 4u * (uint32_t)(n - 1);
                const uint32_t va = (uint32_t)vy[m], vb = (uint32_t)vy1;
                const float u0 = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, (int)(va + o0), 0, 0));
                const float u1 = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, (int)(vb + o0), 0, 0));
                const float u2 = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, (int)(va + o1), 0, 0));
                const float u3 = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, (int)(vb + o1), 0, 0));
                flr[m] = fmaf(kdg, u0 - 2.f * u1 + u3, flr[m]);
                ful[m] = fmaf(kdg, u0 - 2.f * u2 + u3, ful[m]);
                }
            }
        }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) c[m][k] += __shfl_xor(c[m][k], o, 64);
            if (FLUX) {
                flr[m] += __shfl_xor(flr[m], o, 64);
                ful[m] += __shfl_xor(ful[m], o, 64);
            }
        }
        const int i = 64 * m + lane;
        if ((lane % G) == 0 && i < n) {
            int I = i / R;
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
    __syncthreads();
    if (d.r)
        for (int e = threadIdx.x; e < nn; e += blockDim.x) d.r[(int64_t)f * nn + e] = (float)acc[e];
    if (!FLUX) return;
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
    // form: d->form (GPI_CGR_*); GPI_CGR_AUTO takes the first that applies of the barrier-free band form
    // (cgr_band_kernel, its (r, columns) instantiations), the streaming form (cgr_stream_kernel, aligned fields,
    // n <= 256) and the general band kernel (cgr_kernel<M>, any grid).  GPI_CGR_FORM (A/B runs) changes AUTO's
    // first choice: 2 band (default), 1 streaming, 0 general.
    if (d->form < GPI_CGR_AUTO || d->form > GPI_CGR_GENERAL) return GPI_ERR_ARG;
    static const int env_form = [] { const char* v = getenv("GPI_CGR_FORM"); return v && *v ? atoi(v) : 2; }();
    const bool auto_ = d->form == GPI_CGR_AUTO;
    if (d->form == GPI_CGR_BAND || (auto_ && env_form >= 2)) {
        const int n = d->n_fine, MM = (n + 63) / 64;
        bool done = false;
        if (d->nc <= 8) {
            const dim3 grid(d->n), block(64 * d->nc);
            const hipStream_t st = (hipStream_t)stream;
            const bool fl = d->r_flux != nullptr;
            done = true;
#define GPI_CGR_BAND_LAUNCH(RR, M)                                                                             \
    if (fl) hipLaunchKernelGGL((cgr_band_kernel<RR, M, true>), grid, block, lds, st, *d);              \
    else hipLaunchKernelGGL((cgr_band_kernel<RR, M, false>), grid, block, lds, st, *d);
            if (r == 4 && MM == 1) { GPI_CGR_BAND_LAUNCH(4, 1) }
            else if (r == 8 && MM == 1) { GPI_CGR_BAND_LAUNCH(8, 1) }
            else if (r == 16 && MM == 1) { GPI_CGR_BAND_LAUNCH(16, 1) }
            else if (r == 16 && MM == 2) { GPI_CGR_BAND_LAUNCH(16, 2) }
            else if (r == 32 && MM == 4) { GPI_CGR_BAND_LAUNCH(32, 4) }
            else done = false;
#undef GPI_CGR_BAND_LAUNCH
        }
        if (done) {
            GPI_CHECK_LAUNCH();
            return GPI_OK;
        }
        if (d->form == GPI_CGR_BAND) return GPI_ERR_UNSUPPORTED;
    }
    if (d->form == GPI_CGR_STREAM || (auto_ && env_form >= 1)) {
        const int n = d->n_fine;
        const bool ok = n % CGRS_CR == 0 && n >= CGRS_CR && n <= 256 && r >= 4 && (r & (r - 1)) == 0 &&
                        ((uintptr_t)d->logkappa & 15) == 0 && ((uintptr_t)d->y & 15) == 0;
        int lr = 0;
        while ((1 << lr) < r) ++lr;
        const int nd = (nn + 2 * d->nc * d->nc + 1) & ~1;
        const size_t lds2 = sizeof(double) * nd + sizeof(float) * (6 * CGRS_CR + 1) * cgrs_pitch(n);
        if (ok && lds2 <= 160 * 1024) {
            const dim3 grid(d->n), block(4 * n);
            const hipStream_t st = (hipStream_t)stream;
            const bool fl = d->r_flux != nullptr;
            auto go = [&](auto ns_c) -> int {
                constexpr int NS = decltype(ns_c)::value;
                const void* k = fl ? (const void*)cgr_stream_kernel<GPI_CGR_DEPTH, true, NS>
                                   : (const void*)cgr_stream_kernel<GPI_CGR_DEPTH, false, NS>;
                if (lds2 > 64 * 1024 &&
                    hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2) != hipSuccess)
                    return GPI_ERR_LAUNCH;
                if (fl) hipLaunchKernelGGL((cgr_stream_kernel<GPI_CGR_DEPTH, true, NS>), grid, block, lds2, st, *d, lr);
                else hipLaunchKernelGGL((cgr_stream_kernel<GPI_CGR_DEPTH, false, NS>), grid, block, lds2, st, *d, lr);
                return GPI_OK;
            };
            int rc;
            switch (n) {
                case 32: rc = go(std::integral_constant<int, 3>{}); break;
                case 64: rc = go(std::integral_constant<int, 5>{}); break;
                case 128: rc = go(std::integral_constant<int, 9>{}); break;
                case 256: rc = go(std::integral_constant<int, 17>{}); break;
                default: rc = go(std::integral_constant<int, 0>{}); break;
            }
            if (rc != GPI_OK) return rc;
            GPI_CHECK_LAUNCH();
            return GPI_OK;
        }
        if (d->form == GPI_CGR_STREAM) return GPI_ERR_UNSUPPORTED;
    }
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
