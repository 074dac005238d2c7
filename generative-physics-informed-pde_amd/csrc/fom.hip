// FOM data generation on the device: labels Y and log-conductivity fields.
//
// Reference: DataLoader.assemble (utils/data.py:72-103) solves, per sample, the FEniCS system
// a = kappa grad u . grad v dx with the NDP boundary data (physics/LinearElliptic.py:85-101, PETSc LU)
// for Y on the fine free nodes; NormalRandomFieldSampler (physics/RandomField.py:162-209) draws the
// log-conductivity images from a dense squared-exponential covariance factor.
//
// gpi_fom_solve: the Dirichlet-reduced operator K_ff is the 5-point stencil of physics/grid.py
// (edge conductance c = (kappa_a + kappa_b) / 2 of the two triangles having the edge as a leg), SPD.
// One workgroup of 1024 threads per sample runs Jacobi-preconditioned CG in the Chronopoulos-Gear
// form, so that every iteration has ONE fused block reduction ((r,u), (Au,u), (r,r)) and one more
// barrier (the preconditioned residual u is read by the neighbours' stencil).  Up to 64^2 every
// vector lives in registers and u in LDS (fom_pcg_reg_kernel); larger grids keep the vectors in the
// caller's workspace (fom_pcg_kernel).
//
// gpi_random_field: separable restatement x = mean + sigma L_y (S o G) L_x^T of the KL sampler (the SE
// kernel on a tensor grid is C_y (x) C_x), two batched fp64 products with 16-row panels in LDS.
#include <stdlib.h>

#include "common.h"

using namespace gpi;

namespace {

constexpr int FT = 1024;   // threads per FOM workgroup
constexpr int FW = FT / 64;

struct FomGeom {
    int n, dy, ne_h, ne_v;
    int64_t ws;
};

__device__ __forceinline__ double bcv(const double* u, int side_right, int j, int n) {
    const double y = (double)j / (double)n;
    return side_right ? u[2] * (1.0 - y) + u[3] * y : u[0] * (1.0 - y) + u[1] * y;
}

__device__ __forceinline__ double kc(const double* lk, int n, int i, int j, int ul) {
    return exp(lk[2 * (i + n * j) + ul]);
}

// four fused wave + block sums; every thread receives the totals (fixed summation order)
__device__ __forceinline__ void block_sum4(double (&v)[4], double* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = wave_sum_d(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) red[wv * 4 + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double s = 0.0;
        for (int w = 0; w < FW; ++w) s += red[w * 4 + k];
        v[k] = s;
    }
}

__global__ __launch_bounds__(FT) void fom_pcg_kernel(gpi_fom_desc d, FomGeom G) {
    __shared__ double red[FW * 4];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = G.n, nm = n - 1, dy = G.dy;
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    const double* ub = d.bc + 4 * f;
    double* W = d.work + (int64_t)f * G.ws;
    double* ch = W;                 // [(n+1) n]: edge (i,j)-(i+1,j) at j n + i
    double* cv = ch + G.ne_h;       // [n (n+1)]: edge (i,j)-(i,j+1) at j (n+1) + i
    double* dinv = cv + G.ne_v;     // [dy]
    double* r = dinv + dy;
    double* pd = r + dy;
    double* s = pd + dy;
    double* u = s + dy;
    double* w = u + dy;
    double* x = d.y + (int64_t)f * dy;

    // ---- conductances: horizontal edges are legs of T_lr(i,j) / T_ul(i,j-1), vertical ones of
    // T_ul(i,j) / T_lr(i-1,j) (P1 element matrix kappa/2 [[2,-1,-1],[-1,1,0],[-1,0,1]])
    for (int e = tid; e < G.ne_h; e += FT) {
        const int j = e / n, i = e - j * n;
        double c = 0.0;
        if (j < n) c += kc(lk, n, i, j, 0);
        if (j > 0) c += kc(lk, n, i, j - 1, 1);
        ch[e] = 0.5 * c;
    }
    for (int e = tid; e < G.ne_v; e += FT) {
        const int j = e / (n + 1), i = e - j * (n + 1);
        double c = 0.0;
        if (i < n) c += kc(lk, n, i, j, 1);
        if (i > 0) c += kc(lk, n, i - 1, j, 0);
        cv[e] = 0.5 * c;
    }
    __syncthreads();

    struct Star {
        int i, j;
        double cl, cr, cd, cu;
    };
    auto star = [&](int p) {
        Star t;
        t.j = p / nm;
        t.i = p - t.j * nm + 1;
        t.cl = ch[t.j * n + t.i - 1];
        t.cr = ch[t.j * n + t.i];
        t.cd = t.j > 0 ? cv[(t.j - 1) * (n + 1) + t.i] : 0.0;
        t.cu = t.j < n ? cv[t.j * (n + 1) + t.i] : 0.0;
        return t;
    };
    // (K_ff v)_p with v = 0 on the Dirichlet columns
    auto apply = [&](const double* v, int p, const Star& t) {
        double a = (t.cl + t.cr + t.cd + t.cu) * v[p];
        if (t.i > 1) a -= t.cl * v[p - 1];
        if (t.i < nm) a -= t.cr * v[p + 1];
        if (t.j > 0) a -= t.cd * v[p - nm];
        if (t.j < n) a -= t.cu * v[p + nm];
        return a;
    };
    // f_eff = -K_fc g: the Dirichlet neighbours of the first / last free column
    auto rhs = [&](const Star& t) {
        double b = 0.0;
        if (t.i == 1) b += t.cl * bcv(ub, 0, t.j, n);
        if (t.i == nm) b += t.cr * bcv(ub, 1, t.j, n);
        return b;
    };

    const bool warm = d.flags & GPI_FOM_WARM;
    for (int p = tid; p < dy; p += FT) {
        const Star t = star(p);
        dinv[p] = 1.0 / (t.cl + t.cr + t.cd + t.cu);
        if (!warm) {
            const double gl = bcv(ub, 0, t.j, n), gr = bcv(ub, 1, t.j, n);
            x[p] = gl + (gr - gl) * ((double)t.i / (double)n);
        }
    }
    __syncthreads();
    double bb = 0.0;
    for (int p = tid; p < dy; p += FT) {
        const Star t = star(p);
        const double b = rhs(t);
        bb += b * b;
        const double rv = b - apply(x, p, t);
        r[p] = rv;
        u[p] = dinv[p] * rv;
    }
    __syncthreads();
    double v4[4] = {0.0, 0.0, 0.0, bb};
    for (int p = tid; p < dy; p += FT) {
        const Star t = star(p);
        const double wv = apply(u, p, t), rv = r[p], uv = u[p];
        w[p] = wv;
        v4[0] += rv * uv;
        v4[1] += wv * uv;
        v4[2] += rv * rv;
    }
    block_sum4(v4, red);
    const double tol2 = d.rtol * d.rtol * v4[3];
    double gam = v4[0], alpha = v4[0] / v4[1], beta = 0.0;
    bool conv = v4[2] <= tol2;
    int it = 0;
    while (!conv && it < d.max_iter) {
        for (int p = tid; p < dy; p += FT) {
            const double pv = it == 0 ? u[p] : u[p] + beta * pd[p];
            const double sv = it == 0 ? w[p] : w[p] + beta * s[p];
            pd[p] = pv;
            s[p] = sv;
            x[p] += alpha * pv;
            const double rv = r[p] - alpha * sv;
            r[p] = rv;
            u[p] = dinv[p] * rv;
        }
        __syncthreads();
        double q[4] = {0.0, 0.0, 0.0, 0.0};
        for (int p = tid; p < dy; p += FT) {
            const Star t = star(p);
            const double wv = apply(u, p, t), rv = r[p], uv = u[p];
            w[p] = wv;
            q[0] += rv * uv;
            q[1] += wv * uv;
            q[2] += rv * rv;
        }
        block_sum4(q, red);
        ++it;
        conv = q[2] <= tol2;
        if (!conv) {
            beta = q[0] / gam;
            alpha = q[0] / (q[1] - beta * q[0] / alpha);
            gam = q[0];
        }
    }
    if (tid == 0) {
        if (d.iters) d.iters[f] = it;
        if (!conv && d.flag) atomicAdd(d.flag, 1);
    }
}

// Register-resident variant for grids whose free nodes fit NPT per thread (n <= 64 at NPT = 4): the
// iteration vectors x, r, p, s, w live in registers; the stencil operand u, the conductances and the
// Jacobi scaling in LDS -- no global traffic inside the iteration.  Same algorithm, same per-thread
// node order and reduction order as fom_pcg_kernel.
template <int NPT>
__global__ __launch_bounds__(FT) void fom_pcg_reg_kernel(gpi_fom_desc d, FomGeom G) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ double red[FW * 4];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = G.n, nm = n - 1, dy = G.dy;
    double* us = sm;                    // [dy] preconditioned residual (stencil operand)
    double* dinv = us + dy;             // [dy]
    double* ch = dinv + dy;             // [(n+1) n]
    double* cv = ch + G.ne_h;           // [n (n+1)]
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    const double* ub = d.bc + 4 * f;
    double* x = d.y + (int64_t)f * dy;
    for (int e = tid; e < G.ne_h; e += FT) {
        const int j = e / n, i = e - j * n;
        double c = 0.0;
        if (j < n) c += kc(lk, n, i, j, 0);
        if (j > 0) c += kc(lk, n, i, j - 1, 1);
        ch[e] = 0.5 * c;
    }
    for (int e = tid; e < G.ne_v; e += FT) {
        const int j = e / (n + 1), i = e - j * (n + 1);
        double c = 0.0;
        if (i < n) c += kc(lk, n, i, j, 1);
        if (i > 0) c += kc(lk, n, i - 1, j, 0);
        cv[e] = 0.5 * c;
    }
    __syncthreads();
    double X[NPT], R[NPT], Pd[NPT], Sv[NPT], Wv[NPT];
    int IJ[NPT];                        // i | j << 16
    const bool warm = d.flags & GPI_FOM_WARM;
    auto valid = [&](int k) { return tid + k * FT < dy; };
    auto node = [&](int k) { return tid + k * FT; };
    // (K_ff v)_p with v from LDS (Dirichlet columns zero); vp = v at p itself
    auto apply = [&](int k, double vp) {
        const int p = node(k), i = IJ[k] & 0xffff, j = IJ[k] >> 16;
        const double cl = ch[j * n + i - 1], cr = ch[j * n + i];
        const double cd = j > 0 ? cv[(j - 1) * (n + 1) + i] : 0.0, cu = j < n ? cv[j * (n + 1) + i] : 0.0;
        double a = (cl + cr + cd + cu) * vp;
        if (i > 1) a -= cl * us[p - 1];
        if (i < nm) a -= cr * us[p + 1];
        if (j > 0) a -= cd * us[p - nm];
        if (j < n) a -= cu * us[p + nm];
        return a;
    };
    double bb = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int p = valid(k) ? node(k) : 0;
        const int j = p / nm, i = p - j * nm + 1;
        IJ[k] = i | (j << 16);
        Pd[k] = Sv[k] = Wv[k] = R[k] = 0.0;
        X[k] = 0.0;
        if (!valid(k)) continue;
        const double cl = ch[j * n + i - 1], cr = ch[j * n + i];
        const double cd = j > 0 ? cv[(j - 1) * (n + 1) + i] : 0.0, cu = j < n ? cv[j * (n + 1) + i] : 0.0;
        dinv[p] = 1.0 / (cl + cr + cd + cu);
        const double gl = bcv(ub, 0, j, n), gr = bcv(ub, 1, j, n);
        X[k] = warm ? x[p] : gl + (gr - gl) * ((double)i / (double)n);
        const double b = (i == 1 ? cl * gl : 0.0) + (i == nm ? cr * gr : 0.0);
        R[k] = b;                       // b; A x0 subtracted below
        bb += b * b;
        us[p] = X[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k)
        if (valid(k)) R[k] -= apply(k, X[k]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k)
        if (valid(k)) us[node(k)] = dinv[node(k)] * R[k];
    __syncthreads();
    double v4[4] = {0.0, 0.0, 0.0, bb};
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        if (!valid(k)) continue;
        const double u = us[node(k)];
        Wv[k] = apply(k, u);
        v4[0] += R[k] * u;
        v4[1] += Wv[k] * u;
        v4[2] += R[k] * R[k];
    }
    block_sum4(v4, red);
    const double tol2 = d.rtol * d.rtol * v4[3];
    double gam = v4[0], alpha = v4[0] / v4[1], beta = 0.0;
    bool conv = v4[2] <= tol2;
    int it = 0;
    while (!conv && it < d.max_iter) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            if (!valid(k)) continue;
            const int p = node(k);
            const double u = us[p];
            Pd[k] = it == 0 ? u : u + beta * Pd[k];
            Sv[k] = it == 0 ? Wv[k] : Wv[k] + beta * Sv[k];
            X[k] += alpha * Pd[k];
            R[k] -= alpha * Sv[k];
        }
        __syncthreads();                // every u read before it is overwritten
#pragma unroll
        for (int k = 0; k < NPT; ++k)
            if (valid(k)) us[node(k)] = dinv[node(k)] * R[k];
        __syncthreads();
        double q[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            if (!valid(k)) continue;
            const double u = us[node(k)];
            Wv[k] = apply(k, u);
            q[0] += R[k] * u;
            q[1] += Wv[k] * u;
            q[2] += R[k] * R[k];
        }
        block_sum4(q, red);
        ++it;
        conv = q[2] <= tol2;
        if (!conv) {
            beta = q[0] / gam;
            alpha = q[0] / (q[1] - beta * q[0] / alpha);
            gam = q[0];
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k)
        if (valid(k)) x[node(k)] = X[k];
    if (tid == 0) {
        if (d.iters) d.iters[f] = it;
        if (!conv && d.flag) atomicAdd(d.flag, 1);
    }
}

// ---------------------------------------------------------------- multigrid-preconditioned CG
// The same operator and right-hand side, CG preconditioned by one geometric-multigrid V(1,1) cycle:
// levels n, n / 2, ..., MG_COARSE (n a power of two), vertex-centred coarsening (coarse node (I, J) = fine
// node (2I, 2J); the Dirichlet columns stay columns 0 and n_l on every level), bilinear prolongation P,
// restriction R = P^T, coarse operators by rediscretisation: a coarse edge's conductance is the series
// (harmonic) conductance of its two fine half-edges, summed over the fine edges of its band with weights
// 1/2, 1, 1/2 (exact for constant kappa, the half-conductance Neumann rows included).  Red-black
// Gauss-Seidel smoothing, red then black going down and black then red coming up, a palindromic sweep
// sequence on the coarsest level: the cycle is a symmetric positive definite preconditioner, so the
// iteration stays CG (iteration counts ~ independent of n instead of growing with it).  One workgroup
// per sample, every level in the caller's workspace (the coarse levels stay in L2).
constexpr int MG_COARSE = 4;       // coarsest level: squares per side
constexpr int MG_CSWEEPS = 8;      // red-black sweep pairs each way on the coarsest level

struct MgLev {
    int n;            // squares per side
    double* ch;       // [(n+1) n]: edge (i,j)-(i+1,j) at j n + i
    double* cv;       // [n (n+1)]: edge (i,j)-(i,j+1) at j (n+1) + i
    double* e;        // [dy] correction (level 0: z)
    double* b;        // [dy] right-hand side (level 0: the CG residual r)
    double* t;        // [dy] residual of the smoothed correction (level 0: q)
};

__device__ __forceinline__ int64_t mg_dy(int n) { return (int64_t)(n + 1) * (n - 1); }

// doubles per sample: level 0 conductances + r, p, q, z; levels >= 1 conductances + e, b, t
__host__ __device__ inline int64_t mg_workspace(int n) {
    int64_t w = 2 * (int64_t)n * (n + 1) + 4 * (int64_t)(n + 1) * (n - 1);
    for (int m = n / 2; m >= MG_COARSE; m /= 2) w += 2 * (int64_t)m * (m + 1) + 3 * (int64_t)(m + 1) * (m - 1);
    return w;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v = wave_sum_d(v);
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < FW; ++w) s += red[w];
    __syncthreads();                  // red reusable
    return s;
}

__global__ __launch_bounds__(FT) void fom_mgcg_kernel(gpi_fom_desc d, FomGeom G, int nlev) {
    __shared__ double red[FW];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = G.n, nm = n - 1;
    const int64_t dy = G.dy;
    const double* lk = d.logkappa + (int64_t)f * 2 * n * n;
    const double* ub = d.bc + 4 * f;
    double* W = d.work + (int64_t)f * G.ws;
    double* x = d.y + (int64_t)f * dy;
    __shared__ MgLev lev[12];          // (in LDS: a private array indexed by level would live in scratch)
    if (tid == 0) {
        double* q = W;
        int m = n;
        for (int l = 0; l < nlev; ++l, m /= 2) {
            lev[l].n = m;
            lev[l].ch = q;
            lev[l].cv = q + (int64_t)m * (m + 1);
            q += 2 * (int64_t)m * (m + 1);
            lev[l].e = q;
            lev[l].b = q + mg_dy(m);
            lev[l].t = q + 2 * mg_dy(m);
            q += 3 * mg_dy(m);
            if (l == 0) q += mg_dy(m);      // level 0: e = z, b = r, t = q, and p after them
        }
    }
    __syncthreads();
    double* z = lev[0].e;
    double* r = lev[0].b;
    double* qv = lev[0].t;
    double* pv = lev[0].t + dy;

    // ---- fine conductances (as fom_pcg_kernel), then every coarser level's from the one below
    {
        double* ch = lev[0].ch;
        double* cv = lev[0].cv;
        for (int e = tid; e < (n + 1) * n; e += FT) {
            const int j = e / n, i = e - j * n;
            double c = 0.0;
            if (j < n) c += kc(lk, n, i, j, 0);
            if (j > 0) c += kc(lk, n, i, j - 1, 1);
            ch[e] = 0.5 * c;
        }
        for (int e = tid; e < n * (n + 1); e += FT) {
            const int j = e / (n + 1), i = e - j * (n + 1);
            double c = 0.0;
            if (i < n) c += kc(lk, n, i, j, 1);
            if (i > 0) c += kc(lk, n, i - 1, j, 0);
            cv[e] = 0.5 * c;
        }
    }
    __syncthreads();
    for (int l = 1; l < nlev; ++l) {
        const MgLev& F = lev[l - 1];
        const MgLev& Cl = lev[l];
        const int nf = F.n, ncl = Cl.n;
        for (int e = tid; e < (ncl + 1) * ncl; e += FT) {
            const int J = e / ncl, I = e - J * ncl;
            double c = 0.0;
            for (int rr = 2 * J - 1; rr <= 2 * J + 1; ++rr) {
                if (rr < 0 || rr > nf) continue;
                const double a = F.ch[rr * nf + 2 * I], bq = F.ch[rr * nf + 2 * I + 1];
                c += (rr == 2 * J ? 1.0 : 0.5) * (a * bq / (a + bq));
            }
            Cl.ch[e] = c;
        }
        for (int e = tid; e < ncl * (ncl + 1); e += FT) {
            const int J = e / (ncl + 1), I = e - J * (ncl + 1);
            double c = 0.0;
            for (int ss = 2 * I - 1; ss <= 2 * I + 1; ++ss) {
                if (ss < 0 || ss > nf) continue;
                const double a = F.cv[2 * J * (nf + 1) + ss], bq = F.cv[(2 * J + 1) * (nf + 1) + ss];
                c += (ss == 2 * I ? 1.0 : 0.5) * (a * bq / (a + bq));
            }
            Cl.cv[e] = c;
        }
        __syncthreads();
    }

    // ---- level helpers: node p = j (m - 1) + i - 1 of the free nodes i in [1, m - 1], j in [0, m]
    auto nb_sum = [&](const MgLev& L, const double* v, int p, int i, int j, double& dg) {
        const int m = L.n, mm = m - 1;
        const double cl = L.ch[j * m + i - 1], cr = L.ch[j * m + i];
        const double cd = j > 0 ? L.cv[(j - 1) * (m + 1) + i] : 0.0, cu = j < m ? L.cv[j * (m + 1) + i] : 0.0;
        dg = cl + cr + cd + cu;
        double s = 0.0;
        if (i > 1) s += cl * v[p - 1];
        if (i < mm) s += cr * v[p + 1];
        if (j > 0) s += cd * v[p - mm];
        if (j < m) s += cu * v[p + mm];
        return s;
    };
    // one red-black half sweep of A e = b (zero: e = 0 before it, so the colour's neighbours are 0 and
    // the other colour is zeroed in the same pass)
    // (every pass below handles MGU nodes per thread and trip, their loads issued before any store: the
    // passes are latency-bound, one workgroup per sample)
    constexpr int MGU = 4;
    auto half = [&](const MgLev& L, int colour, bool zero) {
        const int m = L.n, mm = m - 1;
        if (zero) {
            const int64_t ny = mg_dy(m);
            for (int64_t p0 = tid; p0 < ny; p0 += MGU * FT) {
                double dg[MGU], bv[MGU];
                bool red[MGU];
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    red[u] = false;
                    if (p >= ny) continue;
                    const int j = (int)(p / mm), i = (int)(p - (int64_t)j * mm) + 1;
                    red[u] = ((i + j) & 1) == colour;
                    const double cl = L.ch[j * m + i - 1], cr = L.ch[j * m + i];
                    const double cd = j > 0 ? L.cv[(j - 1) * (m + 1) + i] : 0.0, cu = j < m ? L.cv[j * (m + 1) + i] : 0.0;
                    dg[u] = cl + cr + cd + cu;
                    bv[u] = L.b[p];
                }
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    if (p < ny) L.e[p] = red[u] ? bv[u] / dg[u] : 0.0;
                }
            }
        } else {
            // the colour's nodes only: row j holds them at i = i0(j) + 2 k, k < m / 2
            const int hr = m / 2;
            const int64_t nq = (int64_t)(m + 1) * hr;
            for (int64_t q0 = tid; q0 < nq; q0 += MGU * FT) {
                double val[MGU];
                int64_t pp[MGU];
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t q = q0 + (int64_t)u * FT;
                    pp[u] = -1;
                    if (q >= nq) continue;
                    const int j = (int)(q / hr), k = (int)(q - (int64_t)j * hr);
                    const int i = (((1 + j) & 1) == colour ? 1 : 2) + 2 * k;
                    if (i > mm) continue;
                    const int64_t p = (int64_t)j * mm + i - 1;
                    pp[u] = p;
                    const double cl = L.ch[j * m + i - 1], cr = L.ch[j * m + i];
                    const double cd = j > 0 ? L.cv[(j - 1) * (m + 1) + i] : 0.0, cu = j < m ? L.cv[j * (m + 1) + i] : 0.0;
                    double sum = L.b[p];
                    if (i > 1) sum += cl * L.e[p - 1];
                    if (i < mm) sum += cr * L.e[p + 1];
                    if (j > 0) sum += cd * L.e[p - mm];
                    if (j < m) sum += cu * L.e[p + mm];
                    val[u] = sum / (cl + cr + cd + cu);
                }
#pragma unroll
                for (int u = 0; u < MGU; ++u)
                    if (pp[u] >= 0) L.e[pp[u]] = val[u];
            }
        }
        __syncthreads();
    };
    auto vcycle = [&]() {
        for (int l = 0; l + 1 < nlev; ++l) {
            const MgLev& L = lev[l];
            half(L, 0, true);
            half(L, 1, false);
            const int m = L.n, mm = m - 1;
            const int64_t ny = mg_dy(m);
            for (int64_t p0 = tid; p0 < ny; p0 += MGU * FT) {        // t = b - A e
                double tv[MGU];
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    if (p >= ny) continue;
                    const int j = (int)(p / mm), i = (int)(p - (int64_t)j * mm) + 1;
                    double dg;
                    const double s = nb_sum(L, L.e, (int)p, i, j, dg);
                    tv[u] = L.b[p] - (dg * L.e[p] - s);
                }
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    if (p < ny) L.t[p] = tv[u];
                }
            }
            __syncthreads();
            const MgLev& Cl = lev[l + 1];
            const int mc = Cl.n, mcm = mc - 1;
            const int64_t nyc = mg_dy(mc);
            for (int64_t pc = tid; pc < nyc; pc += FT) {              // b_c = P^T t
                const int J = (int)(pc / mcm), I = (int)(pc - (int64_t)J * mcm) + 1;
                double s = 0.0;
                for (int bj = -1; bj <= 1; ++bj) {
                    const int j = 2 * J + bj;
                    if (j < 0 || j > m) continue;
                    const double wy = bj == 0 ? 1.0 : 0.5;
                    for (int ai = -1; ai <= 1; ++ai) {
                        const int i = 2 * I + ai;       // in [1, m - 1]: I in [1, mc - 1]
                        s += wy * (ai == 0 ? 1.0 : 0.5) * L.t[(int64_t)j * mm + i - 1];
                    }
                }
                Cl.b[pc] = s;
            }
            __syncthreads();
        }
        {
            const MgLev& Lc = lev[nlev - 1];
            half(Lc, 0, true);
            half(Lc, 1, false);
            for (int k = 1; k < MG_CSWEEPS; ++k) {
                half(Lc, 0, false);
                half(Lc, 1, false);
            }
            for (int k = 0; k < MG_CSWEEPS; ++k) {
                half(Lc, 1, false);
                half(Lc, 0, false);
            }
        }
        for (int l = nlev - 2; l >= 0; --l) {
            const MgLev& L = lev[l];
            const MgLev& Cl = lev[l + 1];
            const int m = L.n, mm = m - 1, mc = Cl.n, mcm = mc - 1;
            const int64_t ny = mg_dy(m);
            for (int64_t p0 = tid; p0 < ny; p0 += MGU * FT) {        // e += P e_c
                double nv[MGU];
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    if (p >= ny) continue;
                    const int j = (int)(p / mm), i = (int)(p - (int64_t)j * mm) + 1;
                    double s = 0.0;
                    const int I0 = i >> 1, J0 = j >> 1;
                    const int ni = (i & 1) ? 2 : 1, nj = (j & 1) ? 2 : 1;
                    const double wx = ni == 2 ? 0.5 : 1.0, wyv = nj == 2 ? 0.5 : 1.0;
                    for (int b2 = 0; b2 < nj; ++b2)
                        for (int a2 = 0; a2 < ni; ++a2) {
                            const int I = I0 + a2, J = J0 + b2;
                            if (I < 1 || I > mcm) continue;            // Dirichlet columns: 0
                            s += wx * wyv * Cl.e[(int64_t)J * mcm + I - 1];
                        }
                    nv[u] = L.e[p] + s;
                }
#pragma unroll
                for (int u = 0; u < MGU; ++u) {
                    const int64_t p = p0 + (int64_t)u * FT;
                    if (p < ny) L.e[p] = nv[u];
                }
            }
            __syncthreads();
            half(L, 1, false);
            half(L, 0, false);
        }
    };

    // ---- CG: r = b - A x, z = M r, p = z
    const bool warm = d.flags & GPI_FOM_WARM;
    for (int64_t p = tid; p < dy; p += FT) {
        const int j = (int)(p / nm), i = (int)(p - (int64_t)j * nm) + 1;
        if (!warm) {
            const double gl = bcv(ub, 0, j, n), gr = bcv(ub, 1, j, n);
            x[p] = gl + (gr - gl) * ((double)i / (double)n);
        }
    }
    __syncthreads();
    double bb = 0.0;
    for (int64_t p = tid; p < dy; p += FT) {
        const int j = (int)(p / nm), i = (int)(p - (int64_t)j * nm) + 1;
        double dg;
        const double s = nb_sum(lev[0], x, (int)p, i, j, dg);
        const double b = (i == 1 ? lev[0].ch[j * n] * bcv(ub, 0, j, n) : 0.0) +
                         (i == nm ? lev[0].ch[j * n + nm] * bcv(ub, 1, j, n) : 0.0);
        bb += b * b;
        r[p] = b - (dg * x[p] - s);
    }
    __syncthreads();
    const double tol2 = d.rtol * d.rtol * block_sum_d(bb, red);
    vcycle();
    double rz = 0.0, rr = 0.0;
    for (int64_t p = tid; p < dy; p += FT) {
        rz += r[p] * z[p];
        rr += r[p] * r[p];
        pv[p] = z[p];
    }
    rz = block_sum_d(rz, red);
    rr = block_sum_d(rr, red);
    bool conv = rr <= tol2;
    int it = 0;
    while (!conv && it < d.max_iter) {
        double pq = 0.0;
        for (int64_t p0 = tid; p0 < dy; p0 += MGU * FT) {
            double qq[MGU];
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p >= dy) continue;
                const int j = (int)(p / nm), i = (int)(p - (int64_t)j * nm) + 1;
                double dg;
                const double s = nb_sum(lev[0], pv, (int)p, i, j, dg);
                const double pp = pv[p];
                qq[u] = dg * pp - s;
                pq += pp * qq[u];
            }
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p < dy) qv[p] = qq[u];
            }
        }
        const double alpha = rz / block_sum_d(pq, red);
        double r2 = 0.0;
        for (int64_t p0 = tid; p0 < dy; p0 += MGU * FT) {
            double xv[MGU], rv[MGU];
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p >= dy) continue;
                xv[u] = x[p] + alpha * pv[p];
                rv[u] = r[p] - alpha * qv[p];
                r2 += rv[u] * rv[u];
            }
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p < dy) {
                    x[p] = xv[u];
                    r[p] = rv[u];
                }
            }
        }
        r2 = block_sum_d(r2, red);
        ++it;
        conv = r2 <= tol2;
        if (conv) break;
        vcycle();
        double rz2 = 0.0;
        for (int64_t p0 = tid; p0 < dy; p0 += MGU * FT) {
            double a[MGU], c[MGU];
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                a[u] = p < dy ? r[p] : 0.0;
                c[u] = p < dy ? z[p] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < MGU; ++u) rz2 += a[u] * c[u];
        }
        rz2 = block_sum_d(rz2, red);
        const double beta = rz2 / rz;
        rz = rz2;
        for (int64_t p0 = tid; p0 < dy; p0 += MGU * FT) {
            double nv[MGU];
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p < dy) nv[u] = z[p] + beta * pv[p];
            }
#pragma unroll
            for (int u = 0; u < MGU; ++u) {
                const int64_t p = p0 + (int64_t)u * FT;
                if (p < dy) pv[p] = nv[u];
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (d.iters) d.iters[f] = it;
        if (!conv && d.flag) atomicAdd(d.flag, 1);
    }
}

// ---------------------------------------------------------------- random field
constexpr int RB = 16;   // output rows per workgroup

__device__ __forceinline__ double u01d(uint32_t v) {   // (0, 1]
    return ((double)v + 1.0) * 2.3283064365386963e-10;
}

// work[b] = (S o G_b) L_x^T: panel of RB rows of G (given or Philox) in LDS, L_x^T streamed (coalesced in c)
__global__ __launch_bounds__(256) void rf_rows_kernel(gpi_random_field_desc d) {
    extern __shared__ __attribute__((aligned(16))) double gp[];   // [RB][px]
    const int b = blockIdx.y, r0 = blockIdx.x * RB, px = d.px, py = d.py;
    const int64_t P = (int64_t)py * px, q4 = (P + 3) / 4;
    const int nr = min(RB, py - r0);
    for (int e = threadIdx.x; e < RB * px; e += 256) {
        const int64_t g = (int64_t)r0 * px + e;
        double v = 0.0;
        if (e >= nr * px) {
        } else if (d.gamma) {
            v = d.gamma[(int64_t)b * P + g];
        } else {
            const uint4_ h = philox((uint64_t)b * q4 + (uint64_t)(g >> 2), d.sub, d.seed);
            const int k = (int)(g & 3);
            const double ua = u01d(k < 2 ? h.x : h.z), ub = u01d(k < 2 ? h.y : h.w);
            const double rad = sqrt(-2.0 * log(ua)), th = 6.283185307179586 * ub;
            v = (k & 1) ? rad * sin(th) : rad * cos(th);
        }
        if (d.scale && e < nr * px) v *= d.scale[g];
        gp[e] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < px; c += 256) {
        double acc[RB];
#pragma unroll
        for (int t = 0; t < RB; ++t) acc[t] = 0.0;
        for (int k = 0; k < px; ++k) {
            const double l = d.lxt[(int64_t)k * px + c];
#pragma unroll
            for (int t = 0; t < RB; ++t) acc[t] = fma(gp[t * px + k], l, acc[t]);
        }
        for (int t = 0; t < nr; ++t) d.work[(int64_t)b * P + (int64_t)(r0 + t) * px + c] = acc[t];
    }
}

// x[b] = mean + sigma L_y work[b]: panel of RB rows of L_y in LDS, work[b] streamed (coalesced in c)
__global__ __launch_bounds__(256) void rf_cols_kernel(gpi_random_field_desc d) {
    extern __shared__ __attribute__((aligned(16))) double lp[];   // [RB][py]
    const int b = blockIdx.y, r0 = blockIdx.x * RB, px = d.px, py = d.py;
    const int64_t P = (int64_t)py * px;
    const int nr = min(RB, py - r0);
    for (int e = threadIdx.x; e < RB * py; e += 256) {
        const int t = e / py, k = e - t * py;
        lp[e] = t < nr ? d.ly[(int64_t)(r0 + t) * py + k] : 0.0;
    }
    __syncthreads();
    const double* T = d.work + (int64_t)b * P;
    for (int c = threadIdx.x; c < px; c += 256) {
        double acc[RB];
#pragma unroll
        for (int t = 0; t < RB; ++t) acc[t] = 0.0;
        for (int k = 0; k < py; ++k) {
            const double v = T[(int64_t)k * px + c];
#pragma unroll
            for (int t = 0; t < RB; ++t) acc[t] = fma(lp[t * py + k], v, acc[t]);
        }
        for (int t = 0; t < nr; ++t) d.x[(int64_t)b * P + (int64_t)(r0 + t) * px + c] = d.mean + d.stddev * acc[t];
    }
}

}  // namespace

extern "C" int64_t gpi_fom_workspace(int32_t n_fine) {
    if (n_fine < 2) return -1;
    const int64_t n = n_fine, dy = (n + 1) * (n - 1);
    const int64_t pcg = 2 * n * (n + 1) + 6 * dy;
    const int64_t mg = (n_fine & (n_fine - 1)) == 0 && n_fine >= 2 * MG_COARSE ? mg_workspace(n_fine) : 0;
    return pcg > mg ? pcg : mg;
}

extern "C" int gpi_fom_solve(const gpi_fom_desc* d, void* stream) {
    if (!d || !d->logkappa || !d->bc || !d->y || !d->work || d->n < 0 || d->n_fine < 2 || d->max_iter < 0 ||
        !(d->rtol >= 0.0))
        return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    FomGeom G;
    G.n = d->n_fine;
    G.dy = (d->n_fine + 1) * (d->n_fine - 1);
    G.ne_h = (d->n_fine + 1) * d->n_fine;
    G.ne_v = d->n_fine * (d->n_fine + 1);
    G.ws = gpi_fom_workspace(d->n_fine);
    const size_t lds = sizeof(double) * (2 * (size_t)G.dy + G.ne_h + G.ne_v);
    static bool attr = false;
    if (!attr) {
        attr = true;
        if (hipFuncSetAttribute((const void*)fom_pcg_reg_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                150 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)fom_pcg_reg_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                150 * 1024) != hipSuccess)
            return GPI_ERR_LAUNCH;
    }
    // multigrid-preconditioned CG for power-of-two grids of >= GPI_FOM_MG_MIN (default 64) squares per side (0: off;
    // r05w: 64^2 164 k vs 112 k labels/s, 128^2 55 k vs 2.9 k, 256^2 7.5 k vs 196 -- 15 iterations instead of 400-1600;
    // at 32^2 the register-resident Jacobi form is as fast: 330 k vs 325 k)
    // (read per call: a data-generation call, not a per-step one)
    const int mg_min = [] { const char* v = getenv("GPI_FOM_MG_MIN"); return v && *v ? atoi(v) : 64; }();
    const int nf = d->n_fine;
    if (mg_min > 0 && nf >= mg_min && (nf & (nf - 1)) == 0 && nf >= 2 * MG_COARSE) {
        int nlev = 0;
        for (int m = nf; m >= MG_COARSE; m /= 2) ++nlev;
        if (nlev > 12) return GPI_ERR_UNSUPPORTED;
        hipLaunchKernelGGL(fom_mgcg_kernel, dim3(d->n), dim3(FT), 0, (hipStream_t)stream, *d, G, nlev);
        GPI_CHECK_LAUNCH();
        return GPI_OK;
    }
    if (G.dy <= FT && lds <= 150 * 1024) {
        hipLaunchKernelGGL(fom_pcg_reg_kernel<1>, dim3(d->n), dim3(FT), lds, (hipStream_t)stream, *d, G);
    } else if (G.dy <= 4 * FT && lds <= 150 * 1024) {
        hipLaunchKernelGGL(fom_pcg_reg_kernel<4>, dim3(d->n), dim3(FT), lds, (hipStream_t)stream, *d, G);
    } else {
        hipLaunchKernelGGL(fom_pcg_kernel, dim3(d->n), dim3(FT), 0, (hipStream_t)stream, *d, G);
    }
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

extern "C" int gpi_random_field(const gpi_random_field_desc* d, void* stream) {
    if (!d || !d->ly || !d->lxt || !d->work || !d->x || d->n < 0 || d->py < 1 || d->px < 1 || !(d->stddev > 0.0))
        return GPI_ERR_ARG;
    if (d->n == 0) return GPI_OK;
    const size_t lds_r = sizeof(double) * RB * d->px, lds_c = sizeof(double) * RB * d->py;
    if (lds_r > 64 * 1024 || lds_c > 64 * 1024) return GPI_ERR_UNSUPPORTED;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((d->py + RB - 1) / RB, d->n);
    hipLaunchKernelGGL(rf_rows_kernel, grid, dim3(256), lds_r, st, *d);
    GPI_CHECK_LAUNCH();
    hipLaunchKernelGGL(rf_cols_kernel, grid, dim3(256), lds_c, st, *d);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
