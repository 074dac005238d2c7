// DenseNet codec convolutions for gfx950 (wave64, 256-thread workgroups).
//
// Forward (one launch per conv of bottleneck/codec.py):
//   out = conv(act(in)),  act = relu(BN_train(.)) | identity
//   - the input tile + halo of every input channel is staged in LDS already
//     activated (BN scale/shift from the replicated fp64 batch sums written by
//     the producer's epilogue, ReLU, zero padding applied AFTER the
//     activation), nearest x2 upsampling folded into the addressing;
//   - global loads are issued in batches of 8 per thread before any use, so a
//     workgroup pays a few memory round trips, not one per element;
//   - weights are staged transposed ([ci][tap][co]) so one LDS vector read
//     broadcasts the taps of all output channels;
//   - epilogue: raw store + per-channel sum / sum^2 (block reduction, fp64
//     atomics into one of GPI_REPLICAS slots) for the consumer's train-mode BN,
//     or the fused Gaussian log-likelihood of the decoder output.
// Backward (one launch per conv, reverse order):
//   - g_out = BN-backward of the accumulated S buffer of the output
//     (S = sum over BN consumers c of gamma_c dL/d(bn_c); the per-channel means
//     of S and S * xhat come from the consumers' replicated sums) or a direct
//     gradient;
//   - weight-gradient partial per workgroup (slab row, reduced by
//     gpi_wgrad_reduce together with the dgamma/dbeta partials);
//   - input gradient by gather: one thread per owned input pixel computes all
//     input channels at once (weights staged [co][tap][ci]), then the ReLU mask,
//     S_in (+)= gamma * dbn with all its global loads in flight together.
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
    if (d.upsample && ((G.th & 1) || (G.tw & 1))) return false;
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
// dst[4 * nch] (LDS, fp64: sum, sumsq, ssum, sxsum).  Caller zeroes dst and syncs around.
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

// Fill dst[0, total) (LDS) with f(q, ry, rx), q = e / plane, (ry, rx) the position in the
// rh x rw plane.  Eight elements per thread are loaded before any is stored, so their
// global loads are in flight together.
constexpr int FILL_U = 8;
template <typename F>
__device__ __forceinline__ void fill(float* dst, int total, int plane, int rw, F f) {
    for (int e0 = threadIdx.x; e0 < total; e0 += FILL_U * 256) {
        float v[FILL_U];
#pragma unroll
        for (int u = 0; u < FILL_U; ++u) {
            const int e = e0 + u * 256;
            v[u] = 0.f;
            if (e < total) {
                const int q = e / plane, pos = e - q * plane;
                const int ry = pos / rw;
                v[u] = f(q, ry, pos - ry * rw);
            }
        }
#pragma unroll
        for (int u = 0; u < FILL_U; ++u) {
            const int e = e0 + u * 256;
            if (e < total) dst[e] = v[u];
        }
    }
}

template <int CP>
__device__ __forceinline__ void fma_vec(float (&acc)[CP], const float* w, float v) {
    if constexpr (CP % 4 == 0) {
#pragma unroll
        for (int q = 0; q < CP / 4; ++q) {
            const float4 w4 = reinterpret_cast<const float4*>(w)[q];
            acc[4 * q + 0] = fmaf(w4.x, v, acc[4 * q + 0]);
            acc[4 * q + 1] = fmaf(w4.y, v, acc[4 * q + 1]);
            acc[4 * q + 2] = fmaf(w4.z, v, acc[4 * q + 2]);
            acc[4 * q + 3] = fmaf(w4.w, v, acc[4 * q + 3]);
        }
    } else {
#pragma unroll
        for (int q = 0; q < CP / 2; ++q) {
            const float2 w2 = reinterpret_cast<const float2*>(w)[q];
            acc[2 * q + 0] = fmaf(w2.x, v, acc[2 * q + 0]);
            acc[2 * q + 1] = fmaf(w2.y, v, acc[2 * q + 1]);
        }
    }
}

struct TileIdx {
    int sb, oy0, ox0, s0, grp, gsz;
};

__device__ __forceinline__ TileIdx tile_of(const ConvGeom& G, const gpi_groups& g) {
    TileIdx t;
    const int tiles = G.tiles_y * G.tiles_x;
    t.sb = blockIdx.x / tiles;
    const int tt = blockIdx.x - t.sb * tiles;
    t.oy0 = (tt / G.tiles_x) * G.th;
    t.ox0 = (tt % G.tiles_x) * G.tw;
    t.s0 = t.sb * G.spb;
    t.grp = group_of(g, t.s0);
    t.gsz = g.start[t.grp + 1] - g.start[t.grp];
    return t;
}

// ---------------------------------------------------------------------------------- forward
constexpr int FWD_HDR = 8 * GPI_MAX_CIN + 2 * GPI_MAX_CIN + 64 + 16;   // gst (fp64) | sc | sh | scratch | red

template <int K, int S, int UP, int CP>
__global__ __launch_bounds__(256) void conv_fwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    constexpr int KK = K * K;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    double* gst = (double*)smem;
    float* sc = smem + 8 * GPI_MAX_CIN;
    float* sh = sc + GPI_MAX_CIN;
    float* scratch = sh + GPI_MAX_CIN;   // 2*CP*4 <= 64
    float* red = scratch + 64;           // 2*CP <= 16
    float* wT = smem + FWD_HDR;          // [cin][KK][CP]
    float* tile = wT + ((d.cin * KK * CP + 3) & ~3);

    const int tid = threadIdx.x;
    const TileIdx T = tile_of(G, c.groups);
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;

    if (d.in_bn) {
        for (int e = tid; e < 4 * d.cin; e += 256) gst[e] = 0.0;
        __syncthreads();
        gather_stats(c, d.in_stat, d.cin, T.grp, gst);
    }
    for (int e = tid; e < d.cin * KK * CP; e += 256) {
        const int co = e % CP, r = e / CP;
        wT[e] = co < d.cout ? c.params[d.w_off + (int64_t)co * d.cin * KK + r] : 0.f;
    }
    __syncthreads();
    if (d.in_bn && tid < d.cin) {
        float mean, inv;
        mean_invstd(gst + 4 * tid, (double)T.gsz * HWi, c.bn_eps, mean, inv);
        const float gam = c.params[d.gamma_off + tid], bet = c.params[d.beta_off + tid];
        sc[tid] = gam * inv;
        sh[tid] = bet - mean * gam * inv;
    }
    __syncthreads();

    int iy0, rh_, ix0, rw_;
    in_region(K, S, UP, d.pad, T.oy0, G.th, iy0, rh_);
    in_region(K, S, UP, d.pad, T.ox0, G.tw, ix0, rw_);
    const int rw = G.rw;
    const int plane_r = G.rh * rw;
    const int per_s = d.cin * plane_r;
    const float* inb = d.in_off >= 0 ? c.ws + d.in_off : nullptr;
    fill(tile, G.spb * per_s, plane_r, rw, [&](int q, int ry, int rx) -> float {
        const int s = q / d.cin, ci = q - s * d.cin;
        const int iy = iy0 + ry, ix = ix0 + rx;
        if (ry >= rh_ || rx >= rw_ || iy < 0 || iy >= d.h_in || ix < 0 || ix >= d.w_in) return 0.f;
        const int gs = T.s0 + s;
        const float* src = inb ? inb + (int64_t)gs * d.in_ctot * HWi
                               : c.ext_in + (int64_t)(c.ext_idx ? c.ext_idx[gs] : gs) * c.ext_stride;
        const float x = src[(int64_t)(d.in_c0 + ci) * HWi + iy * d.w_in + ix];
        return d.in_bn ? fmaxf(fmaf(x, sc[ci], sh[ci]), 0.f) : x;
    });
    __syncthreads();

    const int tp = G.th * G.tw;
    const int s = tid / tp;
    const int pr = tid - s * tp;
    const int ty = pr / G.tw, tx = pr - ty * G.tw;
    const int oy = T.oy0 + ty, ox = T.ox0 + tx;
    const bool active = (s < G.spb) && oy < d.h_out && ox < d.w_out;
    float acc[CP];
#pragma unroll
    for (int co = 0; co < CP; ++co) acc[co] = 0.f;
    if (active) {
        const float* tb = tile + s * per_s;
        for (int ci = 0; ci < d.cin; ++ci) {
            const float* tci = tb + ci * plane_r;
            const float* wci = wT + ci * KK * CP;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int ry = UP ? (fdiv2(oy - d.pad + ky) - iy0) : (ty * S + ky);
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int rx = UP ? (fdiv2(ox - d.pad + kx) - ix0) : (tx * S + kx);
                    fma_vec<CP>(acc, wci + (ky * K + kx) * CP, tci[ry * rw + rx]);
                }
            }
        }
    }

    const int gs = T.s0 + s;
    if (d.epilogue == GPI_EPI_GAUSS_LOSS) {
        float L = 0.f;
        if (active) {
            const float mu = acc[0], ls = acc[1];
            int row = gs - c.groups.start[T.grp];
            if (c.tgt_idx[T.grp]) row = c.tgt_idx[T.grp][row];
            const float t = c.tgt[T.grp][(int64_t)row * HWo + oy * d.w_out + ox];
            const float e = expf(-2.f * ls);
            const float r = t - mu;
            L = -0.5f * (2.f * ls + r * r * e + GPI_LOG2PI);
            const float scl = c.loss_scale[T.grp];
            float* go = c.ws + d.gout_off + (int64_t)gs * 2 * HWo + oy * d.w_out + ox;
            go[0] = -scl * r * e;
            go[HWo] = scl * (1.f - r * r * e);
            if (d.out_off >= 0) {
                float* o = c.ws + d.out_off + (int64_t)gs * d.out_ctot * HWo + (int64_t)d.out_c0 * HWo +
                           oy * d.w_out + ox;
                o[0] = mu;
                o[HWo] = ls;
            }
        }
        float v[1] = {L};
        block_sum<1>(v, scratch, red);
        __syncthreads();
        if (tid == 0) atomicAdd(c.loss_acc + T.grp * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, (double)red[0]);
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
            gpi_stat* st = stat_slot(c, d.out_stat + (tid >> 1), T.grp);
            atomicAdd((tid & 1) ? &st->sumsq : &st->sum, (double)red[tid]);
        }
    }
}

// ---------------------------------------------------------------------------------- backward
// header floats: csum fp64 [2*MAX_CIN] | gst fp64 [4*(MAX_CIN+MAX_COUT)] | i_sc i_sh i_mean i_inv i_gam [MAX_CIN] | o_coef [4*MAX_COUT]
constexpr int BWD_HDR = 4 * GPI_MAX_CIN + 8 * (GPI_MAX_CIN + GPI_MAX_COUT) + 5 * GPI_MAX_CIN + 4 * GPI_MAX_COUT;

template <int K, int S, int UP, int CP, int CINP>
__global__ __launch_bounds__(256) void conv_bwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    constexpr int KK = K * K;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    double* csum = (double*)smem;
    double* gst = csum + 2 * GPI_MAX_CIN;
    float* i_sc = smem + 4 * GPI_MAX_CIN + 8 * (GPI_MAX_CIN + GPI_MAX_COUT);
    float* i_sh = i_sc + GPI_MAX_CIN;
    float* i_mean = i_sh + GPI_MAX_CIN;
    float* i_inv = i_mean + GPI_MAX_CIN;
    float* i_gam = i_inv + GPI_MAX_CIN;
    float* o_coef = i_gam + GPI_MAX_CIN;              // [MAX_COUT][4]: mean, inv, mS, mSx
    float* wD = smem + BWD_HDR;                       // [cout][KK][CINP]
    float* gl = wD + d.cout * KK * CINP;
    const int gplane = G.gh * G.gw;
    float* al = gl + ((G.spb * d.cout * gplane + 3) & ~3);
    const int plane_r = G.rh * G.rw;
    const int per_s = d.cin * plane_r;
    float* wred = al + ((G.spb * per_s + 3) & ~3);    // [parts][CP][nthr_j]

    const int tid = threadIdx.x;
    const TileIdx T = tile_of(G, c.groups);
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;

    for (int e = tid; e < 2 * GPI_MAX_CIN + 4 * (GPI_MAX_CIN + GPI_MAX_COUT); e += 256) csum[e] = 0.0;
    __syncthreads();
    if (d.in_bn) gather_stats(c, d.in_stat, d.cin, T.grp, gst);
    if (d.gout_mode == 0) gather_stats(c, d.out_stat, d.cout, T.grp, gst + 4 * GPI_MAX_CIN);
    for (int e = tid; e < d.cout * KK * CINP; e += 256) {
        const int ci = e % CINP, r = e / CINP;
        const int co = r / KK, t = r - co * KK;
        wD[e] = ci < d.cin ? c.params[d.w_off + ((int64_t)co * d.cin + ci) * KK + t] : 0.f;
    }
    __syncthreads();
    if (tid < d.cin && d.in_bn) {
        float mean, inv;
        mean_invstd(gst + 4 * tid, (double)T.gsz * HWi, c.bn_eps, mean, inv);
        const float gam = c.params[d.gamma_off + tid], bet = c.params[d.beta_off + tid];
        i_mean[tid] = mean;
        i_inv[tid] = inv;
        i_gam[tid] = gam;
        i_sc[tid] = gam * inv;
        i_sh[tid] = bet - mean * gam * inv;
    }
    if (d.gout_mode == 0 && tid < d.cout) {
        const double* st = gst + 4 * (GPI_MAX_CIN + tid);
        const double n = (double)T.gsz * HWo;
        float mean, inv;
        mean_invstd(st, n, c.bn_eps, mean, inv);
        o_coef[4 * tid] = mean;
        o_coef[4 * tid + 1] = inv;
        o_coef[4 * tid + 2] = (float)(st[2] / n);
        o_coef[4 * tid + 3] = (float)(st[3] / n);
    }
    __syncthreads();

    // ---- output-gradient region
    int gy0, gh_, gx0, gw_;
    g_region(K, S, d.pad, T.oy0, G.th, gy0, gh_);
    g_region(K, S, d.pad, T.ox0, G.tw, gx0, gw_);
    fill(gl, G.spb * d.cout * gplane, gplane, G.gw, [&](int q, int ry, int rx) -> float {
        const int s = q / d.cout, co = q - s * d.cout;
        const int oy = gy0 + ry, ox = gx0 + rx;
        if (oy < 0 || oy >= d.h_out || ox < 0 || ox >= d.w_out) return 0.f;
        const int64_t idx = ((int64_t)(T.s0 + s) * d.out_ctot + d.out_c0 + co) * HWo + oy * d.w_out + ox;
        const float sv = c.ws[d.gout_off + idx];
        if (d.gout_mode != 0) return sv;
        const float z = c.ws[d.out_off + idx];
        const float inv = o_coef[4 * co + 1];
        const float xh = (z - o_coef[4 * co]) * inv;
        return (sv - o_coef[4 * co + 2] - xh * o_coef[4 * co + 3]) * inv;
    });
    // ---- activated input region (same activation as the forward)
    int iy0, rh_, ix0, rw_;
    in_region(K, S, UP, d.pad, T.oy0, G.th, iy0, rh_);
    in_region(K, S, UP, d.pad, T.ox0, G.tw, ix0, rw_);
    const float* inb = d.in_off >= 0 ? c.ws + d.in_off : nullptr;
    fill(al, G.spb * per_s, plane_r, G.rw, [&](int q, int ry, int rx) -> float {
        const int s = q / d.cin, ci = q - s * d.cin;
        const int iy = iy0 + ry, ix = ix0 + rx;
        if (ry >= rh_ || rx >= rw_ || iy < 0 || iy >= d.h_in || ix < 0 || ix >= d.w_in) return 0.f;
        const int gs = T.s0 + s;
        const float* src = inb ? inb + (int64_t)gs * d.in_ctot * HWi
                               : c.ext_in + (int64_t)(c.ext_idx ? c.ext_idx[gs] : gs) * c.ext_stride;
        const float x = src[(int64_t)(d.in_c0 + ci) * HWi + iy * d.w_in + ix];
        return d.in_bn ? fmaxf(fmaf(x, i_sc[ci], i_sh[ci]), 0.f) : x;
    });
    __syncthreads();

    // ---- weight gradient partial: dW[co][j] = sum_pixels g[co][o] * a[j-window of o]
    const int J = d.cin * KK;
    const int rowlen = d.cout * J + (d.in_bn ? 2 * d.cin : 0);
    {
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
                const int ci = j / KK;
                const int kk = j - ci * KK;
                const int ky = kk / K, kx = kk - ky * K;
                const int rb = part * R / parts, re = (part + 1) * R / parts;
                for (int rr = rb; rr < re; ++rr) {
                    const int s = rr / G.th;
                    const int ty = rr - s * G.th;
                    const int oy = T.oy0 + ty;
                    const int ry = UP ? (fdiv2(oy - d.pad + ky) - iy0) : (ty * S + ky);
                    const float* arow = al + s * per_s + ci * plane_r + ry * G.rw;
                    const float* grow = gl + s * d.cout * gplane + (oy - gy0) * G.gw + (T.ox0 - gx0);
                    for (int tx = 0; tx < G.tw; ++tx) {
                        const int rx = UP ? (fdiv2(T.ox0 + tx - d.pad + kx) - ix0) : (tx * S + kx);
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
                float* wp = c.wpart + d.wpart_off + (int64_t)blockIdx.x * rowlen;
#pragma unroll
                for (int co = 0; co < CP; ++co)
                    if (co < d.cout) wp[co * J + j] = acc[co];
            }
        }
    }

    // ---- input gradient: one thread per owned input pixel, all input channels at once
    float sd[CINP], sdx[CINP];
#pragma unroll
    for (int ci = 0; ci < CINP; ++ci) { sd[ci] = 0.f; sdx[ci] = 0.f; }
    if (d.gin_off >= 0) {
        int py0, ph, px0, pw;
        owned(S, UP, T.oy0, G.th, py0, ph);
        owned(S, UP, T.ox0, G.tw, px0, pw);
        const int pp = ph * pw;
        const int total = G.spb * pp;
        for (int e = tid; e < total; e += 256) {
            const int s = e / pp;
            const int r = e - s * pp;
            const int qy = r / pw, qx = r - qy * pw;
            const int py = py0 + qy, px = px0 + qx;
            float da[CINP];
#pragma unroll
            for (int ci = 0; ci < CINP; ++ci) da[ci] = 0.f;
            for (int co = 0; co < d.cout; ++co) {
                const float* gc = gl + (s * d.cout + co) * gplane;
                const float* wco = wD + co * KK * CINP;
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        float g;
                        if (UP) {
                            const int oy = 2 * py + d.pad - ky - gy0, ox = 2 * px + d.pad - kx - gx0;
                            g = gc[oy * G.gw + ox] + gc[oy * G.gw + ox + 1] + gc[(oy + 1) * G.gw + ox] +
                                gc[(oy + 1) * G.gw + ox + 1];
                        } else if (S == 2) {
                            const int oy2 = py + d.pad - ky, ox2 = px + d.pad - kx;
                            if ((oy2 & 1) || (ox2 & 1)) continue;
                            g = gc[((oy2 >> 1) - gy0) * G.gw + ((ox2 >> 1) - gx0)];
                        } else {
                            g = gc[(py + d.pad - ky - gy0) * G.gw + (px + d.pad - kx - gx0)];
                        }
                        fma_vec<CINP>(da, wco + (ky * K + kx) * CINP, g);
                    }
                }
            }
            const int gs = T.s0 + s;
            const int64_t idx0 = ((int64_t)gs * d.in_ctot + d.in_c0) * HWi + py * d.w_in + px;
            float* gp = c.ws + d.gin_off + idx0;
            if (d.in_bn) {
                const float* xp = c.ws + d.in_off + idx0;
                float xv[CINP], pv[CINP];
#pragma unroll
                for (int ci = 0; ci < CINP; ++ci) {
                    xv[ci] = 0.f;
                    pv[ci] = 0.f;
                    if (ci < d.cin) {
                        xv[ci] = xp[(int64_t)ci * HWi];
                        if (d.gin_accumulate) pv[ci] = gp[(int64_t)ci * HWi];
                    }
                }
#pragma unroll
                for (int ci = 0; ci < CINP; ++ci) {
                    if (ci < d.cin) {
                        const float bnv = fmaf(xv[ci], i_sc[ci], i_sh[ci]);
                        const float xh = (xv[ci] - i_mean[ci]) * i_inv[ci];
                        const float dbn = bnv > 0.f ? da[ci] : 0.f;
                        gp[(int64_t)ci * HWi] = pv[ci] + i_gam[ci] * dbn;
                        sd[ci] += dbn;
                        sdx[ci] += dbn * xh;
                    }
                }
            } else {
                float pv[CINP];
#pragma unroll
                for (int ci = 0; ci < CINP; ++ci)
                    pv[ci] = (ci < d.cin && d.gin_accumulate) ? gp[(int64_t)ci * HWi] : 0.f;
#pragma unroll
                for (int ci = 0; ci < CINP; ++ci)
                    if (ci < d.cin) gp[(int64_t)ci * HWi] = pv[ci] + da[ci];
            }
        }
    }
    if (d.in_bn) {
        // per-channel sums -> csum (fp64 LDS), then slab row (dgamma, dbeta) and the S statistics
        const int lane = tid & 63;
#pragma unroll
        for (int ci = 0; ci < CINP; ++ci) {
            if (ci < d.cin) {
                const float a = wave_sum(sd[ci]), b = wave_sum(sdx[ci]);
                if (lane == 0) {
                    atomicAdd(&csum[2 * ci], (double)a);
                    atomicAdd(&csum[2 * ci + 1], (double)b);
                }
            }
        }
        __syncthreads();
        if (tid < d.cin) {
            const double s_d = csum[2 * tid], s_dx = csum[2 * tid + 1];
            float* row = c.wpart + d.wpart_off + (int64_t)blockIdx.x * rowlen + d.cout * J;
            row[tid] = (float)s_dx;            // dgamma
            row[d.cin + tid] = (float)s_d;     // dbeta
            if (d.gin_off >= 0) {
                gpi_stat* st = stat_slot(c, d.in_stat + tid, T.grp);
                const double gam = i_gam[tid];
                atomicAdd(&st->ssum, gam * s_d);
                atomicAdd(&st->sxsum, gam * s_dx);
            }
        }
    }
}

size_t fwd_lds(const gpi_conv_desc& d, const ConvGeom& G, int cp) {
    return sizeof(float) * ((size_t)FWD_HDR + ((d.cin * d.k * d.k * cp + 3) & ~3) +
                            (size_t)G.spb * d.cin * G.rh * G.rw);
}

size_t bwd_lds(const gpi_conv_desc& d, const ConvGeom& G, int cp, int cinp) {
    size_t f = BWD_HDR + (size_t)d.cout * d.k * d.k * cinp + (((size_t)G.spb * d.cout * G.gh * G.gw + 3) & ~3) +
               (((size_t)G.spb * d.cin * G.rh * G.rw + 3) & ~3) + (size_t)cp * 256;
    return f * sizeof(float);
}

typedef void (*conv_kernel_t)(gpi_conv_desc, gpi_codec_ctx, ConvGeom);

template <int K, int S, int UP, int CP>
conv_kernel_t pick_cinp(int cinp, bool fwd) {
    if (fwd) return conv_fwd_kernel<K, S, UP, CP>;
    return cinp == 8 ? conv_bwd_kernel<K, S, UP, CP, 8> : conv_bwd_kernel<K, S, UP, CP, 16>;
}

template <int K, int S, int UP>
conv_kernel_t pick(int cp, int cinp, bool fwd) {
    if (cp == 2) return pick_cinp<K, S, UP, 2>(cinp, fwd);
    if (cp == 4) return pick_cinp<K, S, UP, 4>(cinp, fwd);
    return pick_cinp<K, S, UP, 8>(cinp, fwd);
}

conv_kernel_t select_kernel(const gpi_conv_desc& d, int cp, int cinp, bool fwd) {
    const int key = d.k * 100 + d.stride * 10 + d.upsample;
    switch (key) {
        case 110: return pick<1, 1, 0>(cp, cinp, fwd);
        case 310: return pick<3, 1, 0>(cp, cinp, fwd);
        case 311: return pick<3, 1, 1>(cp, cinp, fwd);
        case 320: return pick<3, 2, 0>(cp, cinp, fwd);
        case 510: return pick<5, 1, 0>(cp, cinp, fwd);
        case 720: return pick<7, 2, 0>(cp, cinp, fwd);
        default: return nullptr;
    }
}

int cp_of(int cout) { return cout <= 2 ? 2 : (cout <= 4 ? 4 : 8); }

int launch(const gpi_conv_desc& d, const gpi_codec_ctx& c, hipStream_t st, bool fwd) {
    ConvGeom G;
    if (!conv_geom(d, c.groups, G)) return GPI_ERR_UNSUPPORTED;
    if (d.epilogue == GPI_EPI_GAUSS_LOSS && d.cout != 2) return GPI_ERR_ARG;
    if (!fwd && d.in_bn && d.in_off < 0) return GPI_ERR_ARG;
    if (!fwd && d.cin > 16) return GPI_ERR_UNSUPPORTED;
    const int cp = cp_of(d.cout);
    const int cinp = d.cin <= 8 ? 8 : 16;
    conv_kernel_t k = select_kernel(d, cp, cinp, fwd);
    if (!k) return GPI_ERR_UNSUPPORTED;
    const size_t lds = fwd ? fwd_lds(d, G, cp) : bwd_lds(d, G, cp, cinp);
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
