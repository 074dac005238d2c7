// DenseNet codec convolutions for gfx950 (wave64, 256-thread workgroups).
//
// Forward (one launch per conv of bottleneck/codec.py):
//   out = conv(act(in)),  act = relu(BN_train(.)) | identity
//   - the input tile + halo of every input channel is staged in LDS already
//     activated (BN scale/shift from the fp64 batch sums of the producer's
//     epilogue, ReLU, zero padding applied AFTER the activation), with the
//     nearest x2 upsample folded into the addressing;
//   - weights are wave-uniform (scalar loads);
//   - epilogue: raw store + per-channel sum/sum^2 (fp32 block reduction,
//     fp64 atomics) for the consumer's train-mode BN, or the fused Gaussian
//     log-likelihood of the decoder output.
// Backward (one launch per conv, reverse order):
//   - g_out = BN-backward of the accumulated S buffer of the output
//     (S = sum over BN consumers c of gamma_c dL/d(bn_c); the per-channel
//     means of S and S*xhat were accumulated by the consumers) or a direct
//     gradient;
//   - weight gradient partial per workgroup (deterministic slab, reduced by
//     gpi_wgrad_reduce), input gradient by gather over owned input pixels,
//     ReLU mask, S_in += gamma * dbn and the per-channel dgamma/dbeta/S sums.
#include "common.h"

using namespace gpi;

namespace {

struct ConvGeom {
    int spb, th, tw, tiles_y, tiles_x, nblocks;
    int rh, rw;   // activated input region per (sample, channel)
    int gh, gw;   // output-gradient region per (sample, channel)
};

__host__ __device__ inline int fdiv2(int x) { return x >= 0 ? x / 2 : -((-x + 1) / 2); }
__host__ __device__ inline int cdiv2(int x) { return -fdiv2(-x); }

// input region needed by output positions [o0, o0 + t)
__host__ __device__ inline void in_region(int k, int s, int up, int pad, int o0, int t, int& i0, int& len) {
    if (up) {
        int a = o0 - pad, b = o0 + t - 1 - pad + k - 1;
        i0 = fdiv2(a);
        len = fdiv2(b) - i0 + 1;
    } else {
        i0 = o0 * s - pad;
        len = (t - 1) * s + k;
    }
}

// output-gradient region needed by the input pixels owned by the tile
__host__ __device__ inline void g_region(int k, int s, int pad, int o0, int t, int& g0, int& len) {
    if (s == 2) {
        g0 = cdiv2(2 * o0 + pad - k + 1);
        len = fdiv2(2 * o0 + 2 * t - 1 + pad) - g0 + 1;
    } else {
        g0 = o0 + pad - (k - 1);
        len = t + k - 1;
    }
}

// input pixels whose gradient this output tile owns (a partition of the input)
__host__ __device__ inline void owned(int s, int up, int o0, int t, int& p0, int& len) {
    if (up) { p0 = o0 / 2; len = t / 2; }
    else if (s == 2) { p0 = 2 * o0; len = 2 * t; }
    else { p0 = o0; len = t; }
}

int gcd_i(int a, int b) {
    while (b) { int t = a % b; a = b; b = t; }
    return a;
}

bool conv_geom(const gpi_conv_desc& d, const gpi_groups& g, ConvGeom& G) {
    if (g.n_groups < 1 || g.n_groups > GPI_MAX_GROUPS) return false;
    if (d.cin < 1 || d.cin > GPI_MAX_CIN || d.cout < 1 || d.cout > GPI_MAX_COUT) return false;
    if (d.k != 1 && d.k != 3 && d.k != 5 && d.k != 7) return false;
    if (d.upsample) {
        if (d.stride != 1 || d.h_out != 2 * d.h_in || d.w_out != 2 * d.w_in || d.pad != d.k / 2) return false;
    } else if (d.stride == 2) {
        if (d.h_in != 2 * d.h_out || d.w_in != 2 * d.w_out) return false;
    } else if (d.stride == 1) {
        if (d.h_in != d.h_out || d.w_in != d.w_out || d.pad != d.k / 2) return false;
    } else {
        return false;
    }
    const int plane = d.h_out * d.w_out;
    int B = g.start[g.n_groups] - g.start[0];
    if (g.start[0] != 0 || B <= 0) return false;
    if (plane >= 256) {
        G.tw = d.w_out >= 16 ? 16 : d.w_out;
        G.th = 256 / G.tw;
        if (G.th > d.h_out) G.th = d.h_out;
        G.spb = 1;
    } else {
        G.th = d.h_out;
        G.tw = d.w_out;
        int spb = 256 / plane;
        int gg = 0;
        for (int k = 0; k < g.n_groups; ++k) gg = gcd_i(gg, g.start[k + 1] - g.start[k]);
        while (spb > 1 && (gg % spb)) --spb;
        G.spb = spb;
    }
    if ((d.upsample && (G.th & 1)) || (d.upsample && (G.tw & 1))) return false;
    G.tiles_y = (d.h_out + G.th - 1) / G.th;
    G.tiles_x = (d.w_out + G.tw - 1) / G.tw;
    if (d.h_out % G.th || d.w_out % G.tw) return false;
    G.nblocks = (B / G.spb) * G.tiles_y * G.tiles_x;
    int i0;
    in_region(d.k, d.stride, d.upsample, d.pad, 0, G.th, i0, G.rh);
    in_region(d.k, d.stride, d.upsample, d.pad, 0, G.tw, i0, G.rw);
    if (d.upsample) { G.rh += 1; G.rw += 1; }   // parity-independent bound
    int g0;
    g_region(d.k, d.stride, d.pad, 0, G.th, g0, G.gh);
    g_region(d.k, d.stride, d.pad, 0, G.tw, g0, G.gw);
    return true;
}

// Sum the GPI_REPLICAS copies of the stat records [stat0, stat0 + nch) of group grp into
// dst[4 * nch] (LDS, fp64: sum, sumsq, ssum, sxsum).  Caller syncs before and after.
__device__ __forceinline__ void gather_stats(const gpi_codec_ctx& c, int64_t stat0, int nch, int grp, double* dst) {
    const int n = nch * GPI_REPLICAS;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const int ch = e / GPI_REPLICAS, r = e - ch * GPI_REPLICAS;
        const gpi_stat st = c.stats[((int64_t)r * c.n_stats + stat0 + ch) * GPI_MAX_GROUPS + grp];
        atomicAdd(&dst[4 * ch + 0], st.sum);
        atomicAdd(&dst[4 * ch + 1], st.sumsq);
        atomicAdd(&dst[4 * ch + 2], st.ssum);
        atomicAdd(&dst[4 * ch + 3], st.sxsum);
    }
}

__device__ __forceinline__ gpi_stat* stat_slot(const gpi_codec_ctx& c, int64_t stat, int grp) {
    const int r = blockIdx.x % GPI_REPLICAS;
    return c.stats + ((int64_t)r * c.n_stats + stat) * GPI_MAX_GROUPS + grp;
}

__device__ __forceinline__ void mean_invstd(const double* s4, double n, float eps, float& mean, float& invstd) {
    const double m = s4[0] / n;
    double var = s4[1] / n - m * m;
    if (var < 0.0) var = 0.0;
    mean = (float)m;
    invstd = (float)(1.0 / sqrt(var + (double)eps));
}

constexpr int HDR_D = 4 * (GPI_MAX_CIN + GPI_MAX_COUT);   // fp64 gathered stats
constexpr int HDR = 2 * HDR_D + 2 * GPI_MAX_CIN + 96;      // floats: stats, scale/shift, reduction scratch

template <int K, int S, int UP, int CP>
__global__ __launch_bounds__(256) void conv_fwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    double* gst = (double*)smem;
    float* sc = smem + 2 * HDR_D;
    float* sh = sc + GPI_MAX_CIN;
    float* scratch = sh + GPI_MAX_CIN;         // 2*CP*4 floats
    float* red = scratch + 2 * CP * 4;         // 2*CP floats
    float* tile = smem + HDR;

    const int tid = threadIdx.x;
    const int tiles = G.tiles_y * G.tiles_x;
    const int sb = blockIdx.x / tiles, tt = blockIdx.x - sb * tiles;
    const int oy0 = (tt / G.tiles_x) * G.th, ox0 = (tt % G.tiles_x) * G.tw;
    const int s0 = sb * G.spb;
    const int grp = group_of(c.groups, s0);
    const int gsz = c.groups.start[grp + 1] - c.groups.start[grp];
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;

    if (d.in_bn) {
        for (int e = tid; e < 4 * d.cin; e += 256) gst[e] = 0.0;
        __syncthreads();
        gather_stats(c, d.in_stat, d.cin, grp, gst);
        __syncthreads();
        if (tid < d.cin) {
            float mean, inv;
            mean_invstd(gst + 4 * tid, (double)gsz * HWi, c.bn_eps, mean, inv);
            const float gam = c.params[d.gamma_off + tid], bet = c.params[d.beta_off + tid];
            sc[tid] = gam * inv;
            sh[tid] = bet - mean * gam * inv;
        }
        __syncthreads();
    }

    int iy0, rh_, ix0, rw_;
    in_region(K, S, UP, d.pad, oy0, G.th, iy0, rh_);
    in_region(K, S, UP, d.pad, ox0, G.tw, ix0, rw_);
    const int rh = G.rh, rw = G.rw;
    const int plane_r = rh * rw;
    const int per_s = d.cin * plane_r;
    const int total = G.spb * per_s;
    for (int e = tid; e < total; e += 256) {
        const int s = e / per_s;
        int r = e - s * per_s;
        const int ci = r / plane_r;
        r -= ci * plane_r;
        const int ry = r / rw, rx = r - ry * rw;
        const int iy = iy0 + ry, ix = ix0 + rx;
        float v = 0.f;
        if (ry < rh_ && rx < rw_ && iy >= 0 && iy < d.h_in && ix >= 0 && ix < d.w_in) {
            const int gs = s0 + s;
            const float* src;
            if (d.in_off >= 0) src = c.ws + d.in_off + (int64_t)gs * d.in_ctot * HWi;
            else src = c.ext_in + (int64_t)(c.ext_idx ? c.ext_idx[gs] : gs) * c.ext_stride;
            const float x = src[(int64_t)(d.in_c0 + ci) * HWi + iy * d.w_in + ix];
            v = d.in_bn ? fmaxf(fmaf(x, sc[ci], sh[ci]), 0.f) : x;
        }
        tile[e] = v;
    }
    __syncthreads();

    const int tp = G.th * G.tw;
    const int s = tid / tp;
    const int pr = tid - s * tp;
    const int ty = pr / G.tw, tx = pr - ty * G.tw;
    const int oy = oy0 + ty, ox = ox0 + tx;
    const bool active = (s < G.spb) && oy < d.h_out && ox < d.w_out;
    float acc[CP];
#pragma unroll
    for (int co = 0; co < CP; ++co) acc[co] = 0.f;
    if (active) {
        const float* tb = tile + s * per_s;
        const float* wp = c.params + d.w_off;
        for (int ci = 0; ci < d.cin; ++ci) {
            const float* tci = tb + ci * plane_r;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int ry = UP ? (fdiv2(oy - d.pad + ky) - iy0) : (ty * S + ky);
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int rx = UP ? (fdiv2(ox - d.pad + kx) - ix0) : (tx * S + kx);
                    const float v = tci[ry * rw + rx];
#pragma unroll
                    for (int co = 0; co < CP; ++co)
                        if (co < d.cout) acc[co] = fmaf(wp[((co * d.cin + ci) * K + ky) * K + kx], v, acc[co]);
                }
            }
        }
    }

    const int gs = s0 + s;
    if (d.epilogue == GPI_EPI_GAUSS_LOSS) {
        float L = 0.f;
        if (active) {
            const float mu = acc[0], ls = acc[1];
            int row = gs - c.groups.start[grp];
            if (c.tgt_idx[grp]) row = c.tgt_idx[grp][row];
            const float t = c.tgt[grp][(int64_t)row * HWo + oy * d.w_out + ox];
            const float e = expf(-2.f * ls);
            const float r = t - mu;
            L = -0.5f * (2.f * ls + r * r * e + GPI_LOG2PI);
            const float scl = c.loss_scale[grp];
            float* go = c.ws + d.gout_off + (int64_t)gs * 2 * HWo + oy * d.w_out + ox;
            go[0] = -scl * r * e;
            go[HWo] = scl * (1.f - r * r * e);
            if (d.out_off >= 0) {
                float* o = c.ws + d.out_off + (int64_t)gs * d.out_ctot * HWo + (int64_t)d.out_c0 * HWo + oy * d.w_out + ox;
                o[0] = mu;
                o[HWo] = ls;
            }
        }
        float v[1] = {L};
        block_sum<1>(v, scratch, red);
        __syncthreads();
        if (tid == 0) atomicAdd(c.loss_acc + grp * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, (double)red[0]);
        return;
    }

    if (active) {
        float* o = c.ws + d.out_off + (int64_t)gs * d.out_ctot * HWo + (int64_t)d.out_c0 * HWo + oy * d.w_out + ox;
#pragma unroll
        for (int co = 0; co < CP; ++co)
            if (co < d.cout) o[(int64_t)co * HWo] = acc[co];
    }
    if (d.epilogue == GPI_EPI_STORE_STATS) {
        float v[2 * CP];
#pragma unroll
        for (int co = 0; co < CP; ++co) {
            const float a = (active && co < d.cout) ? acc[co] : 0.f;
            v[2 * co] = a;
            v[2 * co + 1] = a * a;
        }
        block_sum<2 * CP>(v, scratch, red);
        __syncthreads();
        if (tid < 2 * d.cout) {
            gpi_stat* st = stat_slot(c, d.out_stat + (tid >> 1), grp);
            atomicAdd((tid & 1) ? &st->sumsq : &st->sum, (double)red[tid]);
        }
    }
}

template <int K, int S, int UP, int CP>
__global__ __launch_bounds__(256) void conv_bwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // header
    double* csum = (double*)smem;                // [MAX_CIN][2] fp64 per-channel BN-backward sums
    double* gst = csum + 2 * GPI_MAX_CIN;        // [MAX_CIN + MAX_COUT][4] gathered stats
    float* i_mean = smem + 4 * GPI_MAX_CIN + 2 * HDR_D;   // [MAX_CIN]
    float* i_inv = i_mean + GPI_MAX_CIN;
    float* i_gam = i_inv + GPI_MAX_CIN;
    float* i_bet = i_gam + GPI_MAX_CIN;
    float* o_coef = i_bet + GPI_MAX_CIN;         // [COUT][4]: mean, inv, mS, mSx
    float* wl = o_coef + 4 * GPI_MAX_COUT;       // weights [cout*cin*K*K]
    const int nw = d.cout * d.cin * K * K;
    float* gl = wl + ((nw + 3) & ~3);
    const int gplane = G.gh * G.gw;
    float* al = gl + G.spb * d.cout * gplane;
    const int plane_r = G.rh * G.rw;
    const int per_s = d.cin * plane_r;
    float* wred = al + G.spb * per_s;            // [parts][CP][nthr_j]

    const int tid = threadIdx.x;
    const int tiles = G.tiles_y * G.tiles_x;
    const int sb = blockIdx.x / tiles, tt = blockIdx.x - sb * tiles;
    const int oy0 = (tt / G.tiles_x) * G.th, ox0 = (tt % G.tiles_x) * G.tw;
    const int s0 = sb * G.spb;
    const int grp = group_of(c.groups, s0);
    const int gsz = c.groups.start[grp + 1] - c.groups.start[grp];
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;

    for (int e = tid; e < HDR_D; e += 256) gst[e] = 0.0;
    if (tid < 2 * GPI_MAX_CIN) csum[tid] = 0.0;
    __syncthreads();
    if (d.in_bn) gather_stats(c, d.in_stat, d.cin, grp, gst);
    if (d.gout_mode == 0) gather_stats(c, d.out_stat, d.cout, grp, gst + 4 * GPI_MAX_CIN);
    __syncthreads();
    if (tid < d.cin && d.in_bn) {
        float mean, inv;
        mean_invstd(gst + 4 * tid, (double)gsz * HWi, c.bn_eps, mean, inv);
        i_mean[tid] = mean;
        i_inv[tid] = inv;
        i_gam[tid] = c.params[d.gamma_off + tid];
        i_bet[tid] = c.params[d.beta_off + tid];
    }
    if (d.gout_mode == 0 && tid < d.cout) {
        const double* st = gst + 4 * (GPI_MAX_CIN + tid);
        const double n = (double)gsz * HWo;
        float mean, inv;
        mean_invstd(st, n, c.bn_eps, mean, inv);
        o_coef[4 * tid] = mean;
        o_coef[4 * tid + 1] = inv;
        o_coef[4 * tid + 2] = (float)(st[2] / n);
        o_coef[4 * tid + 3] = (float)(st[3] / n);
    }
    for (int e = tid; e < nw; e += 256) wl[e] = c.params[d.w_off + e];
    __syncthreads();

    // ---- output gradient region
    int gy0, gh_, gx0, gw_;
    g_region(K, S, d.pad, oy0, G.th, gy0, gh_);
    g_region(K, S, d.pad, ox0, G.tw, gx0, gw_);
    {
        const int per = d.cout * gplane;
        const int total = G.spb * per;
        for (int e = tid; e < total; e += 256) {
            const int s = e / per;
            int r = e - s * per;
            const int co = r / gplane;
            r -= co * gplane;
            const int ry = r / G.gw, rx = r - ry * G.gw;
            const int oy = gy0 + ry, ox = gx0 + rx;
            float g = 0.f;
            if (oy >= 0 && oy < d.h_out && ox >= 0 && ox < d.w_out) {
                const int gs = s0 + s;
                const int64_t idx = ((int64_t)gs * d.out_ctot + d.out_c0 + co) * HWo + oy * d.w_out + ox;
                const float sv = c.ws[d.gout_off + idx];
                if (d.gout_mode == 0) {
                    const float z = c.ws[d.out_off + idx];
                    const float inv = o_coef[4 * co + 1];
                    const float xh = (z - o_coef[4 * co]) * inv;
                    g = (sv - o_coef[4 * co + 2] - xh * o_coef[4 * co + 3]) * inv;
                } else {
                    g = sv;
                }
            }
            gl[e] = g;
        }
    }
    // ---- activated input region
    int iy0, rh_, ix0, rw_;
    in_region(K, S, UP, d.pad, oy0, G.th, iy0, rh_);
    in_region(K, S, UP, d.pad, ox0, G.tw, ix0, rw_);
    {
        const int total = G.spb * per_s;
        for (int e = tid; e < total; e += 256) {
            const int s = e / per_s;
            int r = e - s * per_s;
            const int ci = r / plane_r;
            r -= ci * plane_r;
            const int ry = r / G.rw, rx = r - ry * G.rw;
            const int iy = iy0 + ry, ix = ix0 + rx;
            float v = 0.f;
            if (ry < rh_ && rx < rw_ && iy >= 0 && iy < d.h_in && ix >= 0 && ix < d.w_in) {
                const int gs = s0 + s;
                const float* src;
                if (d.in_off >= 0) src = c.ws + d.in_off + (int64_t)gs * d.in_ctot * HWi;
                else src = c.ext_in + (int64_t)(c.ext_idx ? c.ext_idx[gs] : gs) * c.ext_stride;
                const float x = src[(int64_t)(d.in_c0 + ci) * HWi + iy * d.w_in + ix];
                v = d.in_bn ? fmaxf(fmaf(x - i_mean[ci], i_inv[ci] * i_gam[ci], i_bet[ci]), 0.f) : x;
            }
            al[e] = v;
        }
    }
    __syncthreads();

    // ---- weight gradient partial: dW[co][j] = sum_pixels g[co][o] * a[j-window of o]
    {
        const int J = d.cin * K * K;
        const int nthr_j = J < 256 ? J : 256;
        const int parts = 256 / nthr_j;
        const int part = tid / nthr_j, jl = tid - part * nthr_j;
        const int R = G.spb * G.th;          // (sample, row) pairs
        for (int jb = 0; jb < J; jb += nthr_j) {
            const int j = jb + jl;
            float acc[CP];
#pragma unroll
            for (int co = 0; co < CP; ++co) acc[co] = 0.f;
            if (part < parts && j < J) {
                const int ci = j / (K * K);
                const int kk = j - ci * K * K;
                const int ky = kk / K, kx = kk - ky * K;
                const int rb = part * R / parts, re = (part + 1) * R / parts;
                for (int rr = rb; rr < re; ++rr) {
                    const int s = rr / G.th;
                    const int ty = rr - s * G.th;
                    const int oy = oy0 + ty;
                    const int ry = UP ? (fdiv2(oy - d.pad + ky) - iy0) : (ty * S + ky);
                    const float* arow = al + s * per_s + ci * plane_r + ry * G.rw;
                    const float* grow = gl + s * d.cout * gplane + (oy - gy0) * G.gw + (ox0 - gx0);
                    for (int tx = 0; tx < G.tw; ++tx) {
                        const int rx = UP ? (fdiv2(ox0 + tx - d.pad + kx) - ix0) : (tx * S + kx);
                        const float a = arow[rx];
#pragma unroll
                        for (int co = 0; co < CP; ++co)
                            if (co < d.cout) acc[co] = fmaf(grow[co * gplane + tx], a, acc[co]);
                    }
                }
            }
            if (parts > 1) {
                if (part < parts) {
#pragma unroll
                    for (int co = 0; co < CP; ++co) wred[(part * CP + co) * nthr_j + jl] = acc[co];
                }
                __syncthreads();
                if (part == 0) {
                    for (int p = 1; p < parts; ++p)
#pragma unroll
                        for (int co = 0; co < CP; ++co) acc[co] += wred[(p * CP + co) * nthr_j + jl];
                }
                __syncthreads();
            }
            if (part == 0 && j < J) {
                float* wp = c.wpart + d.wpart_off + (int64_t)blockIdx.x * (d.cout * J + (d.in_bn ? 2 * d.cin : 0));
#pragma unroll
                for (int co = 0; co < CP; ++co)
                    if (co < d.cout) wp[co * J + j] = acc[co];
            }
        }
    }

    // ---- input gradient (gather) over owned input pixels
    if (d.gin_off >= 0) {
        int py0, ph, px0, pw;
        owned(S, UP, oy0, G.th, py0, ph);
        owned(S, UP, ox0, G.tw, px0, pw);
        const int pp = ph * pw;
        const int per = d.cin * pp;
        const int total = G.spb * per;
        int cur_ci = -1;
        float sd = 0.f, sdx = 0.f;
        for (int e = tid; e < total; e += 256) {
            const int s = e / per;
            int r = e - s * per;
            const int ci = r / pp;
            r -= ci * pp;
            const int qy = r / pw, qx = r - qy * pw;
            const int py = py0 + qy, px = px0 + qx;
            float da = 0.f;
            for (int co = 0; co < d.cout; ++co) {
                const float* gc = gl + (s * d.cout + co) * gplane;
                const float* wc = wl + (co * d.cin + ci) * K * K;
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        const float w = wc[ky * K + kx];
                        if (UP) {
#pragma unroll
                            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                                for (int dx = 0; dx < 2; ++dx) {
                                    const int oy = 2 * py + dy + d.pad - ky, ox = 2 * px + dx + d.pad - kx;
                                    da = fmaf(w, gc[(oy - gy0) * G.gw + (ox - gx0)], da);
                                }
                        } else if (S == 2) {
                            const int oy2 = py + d.pad - ky, ox2 = px + d.pad - kx;
                            if (!(oy2 & 1) && !(ox2 & 1))
                                da = fmaf(w, gc[((oy2 >> 1) - gy0) * G.gw + ((ox2 >> 1) - gx0)], da);
                        } else {
                            const int oy = py + d.pad - ky, ox = px + d.pad - kx;
                            da = fmaf(w, gc[(oy - gy0) * G.gw + (ox - gx0)], da);
                        }
                    }
                }
            }
            const int gs = s0 + s;
            const int64_t idx = ((int64_t)gs * d.in_ctot + d.in_c0 + ci) * HWi + py * d.w_in + px;
            float* gp = c.ws + d.gin_off + idx;
            if (d.in_bn) {
                const float x = c.ws[d.in_off + idx];
                const float xh = (x - i_mean[ci]) * i_inv[ci];
                const float bn = fmaf(i_gam[ci], xh, i_bet[ci]);
                const float dbn = bn > 0.f ? da : 0.f;
                const float prev = d.gin_accumulate ? *gp : 0.f;
                *gp = prev + i_gam[ci] * dbn;
                if (ci != cur_ci) {
                    if (cur_ci >= 0) {
                        atomicAdd(&csum[2 * cur_ci], (double)sd);
                        atomicAdd(&csum[2 * cur_ci + 1], (double)sdx);
                    }
                    cur_ci = ci;
                    sd = 0.f;
                    sdx = 0.f;
                }
                sd += dbn;
                sdx += dbn * xh;
            } else {
                const float prev = d.gin_accumulate ? *gp : 0.f;
                *gp = prev + da;
            }
        }
        if (d.in_bn && cur_ci >= 0) {
            atomicAdd(&csum[2 * cur_ci], (double)sd);
            atomicAdd(&csum[2 * cur_ci + 1], (double)sdx);
        }
    }
    if (d.in_bn) {
        // dbeta / dgamma partials go to this workgroup's slab row (reduced by gpi_wgrad_reduce);
        // the S statistics of the input channels to a replica slot (summed by the producer's backward)
        __syncthreads();
        if (tid < d.cin) {
            const double s_d = csum[2 * tid], s_dx = csum[2 * tid + 1];
            const int J = d.cin * K * K;
            float* row = c.wpart + d.wpart_off + (int64_t)blockIdx.x * (d.cout * J + 2 * d.cin) + d.cout * J;
            row[tid] = (float)s_dx;            // dgamma
            row[d.cin + tid] = (float)s_d;     // dbeta
            if (d.gin_off >= 0) {
                gpi_stat* st = stat_slot(c, d.in_stat + tid, grp);
                const double gam = i_gam[tid];
                atomicAdd(&st->ssum, gam * s_d);
                atomicAdd(&st->sxsum, gam * s_dx);
            }
        }
    }
}

size_t fwd_lds(const gpi_conv_desc& d, const ConvGeom& G) {
    return sizeof(float) * ((size_t)HDR + (size_t)G.spb * d.cin * G.rh * G.rw);
}

size_t bwd_lds(const gpi_conv_desc& d, const ConvGeom& G, int cp) {
    const int nw = d.cout * d.cin * d.k * d.k;
    size_t f = 8 * GPI_MAX_CIN + 2 * HDR_D + 4 * GPI_MAX_COUT + ((nw + 3) & ~3) + (size_t)G.spb * d.cout * G.gh * G.gw +
               (size_t)G.spb * d.cin * G.rh * G.rw + (size_t)cp * 256;
    return f * sizeof(float);
}

typedef void (*conv_kernel_t)(gpi_conv_desc, gpi_codec_ctx, ConvGeom);

template <int K, int S, int UP>
conv_kernel_t pick(int cp, bool fwd) {
    if (cp == 2) return fwd ? conv_fwd_kernel<K, S, UP, 2> : conv_bwd_kernel<K, S, UP, 2>;
    if (cp == 4) return fwd ? conv_fwd_kernel<K, S, UP, 4> : conv_bwd_kernel<K, S, UP, 4>;
    return fwd ? conv_fwd_kernel<K, S, UP, 8> : conv_bwd_kernel<K, S, UP, 8>;
}

conv_kernel_t select_kernel(const gpi_conv_desc& d, int cp, bool fwd) {
    const int key = d.k * 100 + d.stride * 10 + d.upsample;
    switch (key) {
        case 110: return pick<1, 1, 0>(cp, fwd);
        case 310: return pick<3, 1, 0>(cp, fwd);
        case 311: return pick<3, 1, 1>(cp, fwd);
        case 320: return pick<3, 2, 0>(cp, fwd);
        case 510: return pick<5, 1, 0>(cp, fwd);
        case 511: return pick<5, 1, 1>(cp, fwd);
        case 720: return pick<7, 2, 0>(cp, fwd);
        case 710: return pick<7, 1, 0>(cp, fwd);
        case 520: return pick<5, 2, 0>(cp, fwd);
        case 120: return pick<1, 2, 0>(cp, fwd);
        default: return nullptr;
    }
}

int cp_of(int cout) { return cout <= 2 ? 2 : (cout <= 4 ? 4 : 8); }

int launch(const gpi_conv_desc& d, const gpi_codec_ctx& c, hipStream_t st, bool fwd) {
    ConvGeom G;
    if (!conv_geom(d, c.groups, G)) return GPI_ERR_UNSUPPORTED;
    if (d.epilogue == GPI_EPI_GAUSS_LOSS && d.cout != 2) return GPI_ERR_ARG;
    if (!fwd && d.in_bn && d.in_off < 0) return GPI_ERR_ARG;
    const int cp = cp_of(d.cout);
    conv_kernel_t k = select_kernel(d, cp, fwd);
    if (!k) return GPI_ERR_UNSUPPORTED;
    const size_t lds = fwd ? fwd_lds(d, G) : bwd_lds(d, G, cp);
    if (lds > 160 * 1024) return GPI_ERR_UNSUPPORTED;
    if (lds > 64 * 1024) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return GPI_ERR_LAUNCH;
    }
    hipLaunchKernelGGL(k, dim3(G.nblocks), dim3(256), lds, st, d, c, G);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

// Slab reduction: workgroup (item, weight chunk of <= 256, row chunk of RROWS).
// Thread (w, p) sums rows p, p + P, ... of its row chunk for weight w
// (coalesced: consecutive w read consecutive floats of a slab row), the P
// partials meet in LDS, one fp64 atomic per weight per workgroup.
constexpr int RROWS = 64;

struct ReduceArgs {
    gpi_reduce_item it[GPI_MAX_REDUCE_ITEMS];
    int32_t first_block[GPI_MAX_REDUCE_ITEMS + 1];
    int32_t wchunks[GPI_MAX_REDUCE_ITEMS];
    int32_t n;
};

__global__ __launch_bounds__(256) void wgrad_reduce(ReduceArgs a, const float* __restrict__ wpart, double* gacc) {
    __shared__ float red[256];
    int k = 0;
    while (k + 1 < a.n && (int)blockIdx.x >= a.first_block[k + 1]) ++k;
    const gpi_reduce_item it = a.it[k];
    const int local = blockIdx.x - a.first_block[k];
    const int wc = local % a.wchunks[k], rc = local / a.wchunks[k];
    const int w0 = wc * 256;
    const int nw = min(256, it.numel - w0);
    const int P = 256 / nw;
    const int tid = threadIdx.x;
    const int w = tid % nw, p = tid / nw;
    const int r0 = rc * RROWS, r1 = min(it.blocks, r0 + RROWS);
    float s = 0.f;
    if (p < P) {
        const float* base = wpart + it.part_off + w0 + w;
#pragma unroll 4
        for (int r = r0 + p; r < r1; r += P) s += base[(int64_t)r * it.row_stride];
    }
    red[tid] = s;
    __syncthreads();
    if (tid < nw) {
        double t = 0.0;
        for (int q = 0; q < P; ++q) t += (double)red[q * nw + tid];
        atomicAdd(gacc + it.w_off + w0 + tid, t);
    }
}

}  // namespace

extern "C" int gpi_conv_blocks(const gpi_conv_desc* op, const gpi_groups* groups, int32_t* blocks) {
    if (!op || !groups || !blocks) return GPI_ERR_ARG;
    ConvGeom G;
    if (!conv_geom(*op, *groups, G)) return GPI_ERR_UNSUPPORTED;
    *blocks = G.nblocks;
    return GPI_OK;
}

extern "C" int gpi_conv_forward(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, (hipStream_t)stream, true);
}

extern "C" int gpi_conv_backward(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, (hipStream_t)stream, false);
}

extern "C" int gpi_codec_forward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream) {
    if (!ops || !ctx || n_ops < 0) return GPI_ERR_ARG;
    for (int i = 0; i < n_ops; ++i) {
        int r = launch(ops[i], *ctx, (hipStream_t)stream, true);
        if (r != GPI_OK) return r;
    }
    return GPI_OK;
}

extern "C" int gpi_codec_backward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream) {
    if (!ops || !ctx || n_ops < 0) return GPI_ERR_ARG;
    for (int i = n_ops - 1; i >= 0; --i) {
        int r = launch(ops[i], *ctx, (hipStream_t)stream, false);
        if (r != GPI_OK) return r;
    }
    return GPI_OK;
}

extern "C" int gpi_wgrad_reduce(const gpi_reduce_item* items, int n_items, const float* wpart, double* gacc,
                                void* stream) {
    if (!items || n_items < 0 || n_items > GPI_MAX_REDUCE_ITEMS || !wpart || !gacc) return GPI_ERR_ARG;
    for (int k = 0; k < n_items; ++k)
        if (items[k].row_stride < items[k].numel || items[k].numel <= 0) return GPI_ERR_ARG;
    if (n_items == 0) return GPI_OK;
    ReduceArgs a;
    a.n = n_items;
    int nb = 0;
    for (int k = 0; k < n_items; ++k) {
        a.it[k] = items[k];
        a.first_block[k] = nb;
        a.wchunks[k] = (items[k].numel + 255) / 256;
        nb += a.wchunks[k] * ((items[k].blocks + RROWS - 1) / RROWS);
    }
    a.first_block[n_items] = nb;
    hipLaunchKernelGGL(wgrad_reduce, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, wpart, gacc);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
