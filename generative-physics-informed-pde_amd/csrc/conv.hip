// DenseNet codec convolutions for gfx950 (wave64, 256-thread workgroups).
//
// Every launch is one conv of bottleneck/codec.py.  A workgroup owns one tile:
// `th` whole output rows of ONE sample, so every (channel, tile) operand is a
// single contiguous run of global memory whose cache lines are used whole.
// Operands live in LDS as row images with a zero halo of HALO columns on each
// side (pitch = width + 2 HALO), filled by 16-byte LDS-DMA (global_load_lds);
// halo chunks and rows outside the plane read a zero page.  A workgroup runs
// in four phases so that it pays ONE global round trip before it computes:
//   1. issue every global read at once: the LDS images (input, output
//      gradient, BN-backward operand), the weights, the 16 replicas of the BN
//      batch sums and the input-gradient operands (registers);
//   2. BN coefficients from the fp64 sums (train mode, biased variance);
//   3. activation transforms in LDS, in place (BN + ReLU of the input image,
//      padding untouched so it stays zero AFTER the activation; BN-backward of
//      the output gradient);
//   4. compute, epilogue.
// Forward (VALU, one output pixel per thread): out = conv(act(in)); epilogue
// stores + per-channel sum / sum^2 into one of GPI_REPLICAS fp64 slots (the
// consumer's train-mode BN) or the fused Gaussian log-likelihood of the decoder
// output.  Backward (MFMA): weight-gradient partial per workgroup (slab row,
// reduced by gpi_wgrad_reduce with the dgamma/dbeta partials) and the input
// gradient with the ReLU mask and S_in (+)= gamma * dbn.
#include "common.h"
#include <stdlib.h>
#include <stdio.h>
#include <algorithm>
#include <string.h>
#include <string>
#include <utility>
#include <vector>
#include <atomic>
#include <mutex>

using namespace gpi;

// Contraction per expression only (C's FP_CONTRACT on): hipcc's default lets the backend fuse a multiply and
// an add across statements wherever the schedule puts them together, so the generic kernels and the
// compile-time shape instantiations (fold_shape) rounded a few products differently (1-ulp differences in
// the decoder's half tiles, r06); with contraction fixed by the source both compute the same bits.
#pragma clang fp contract(on)

namespace {

constexpr int HALO = 4;   // zero halo columns on each side of an LDS row image

// 256 zero bytes in device memory: the source of LDS-DMA padding lanes and of
// the stat loads of unused lanes.
__device__ __attribute__((aligned(256))) float g_zero_page[64];

// q = e / d without a division: e * d < 2^32 (checked on the host).
struct Div {
    uint32_t m, one;
};

Div mkdiv(int d) {
    Div v;
    v.one = d == 1;
    v.m = d == 1 ? 0u : (uint32_t)(((1ull << 32) + (uint64_t)d - 1) / (uint64_t)d);
    return v;
}

__device__ __forceinline__ int dq(int e, Div v) { return v.one ? e : (int)__umulhi((uint32_t)e, v.m); }

// Phase stamps of the timing build (make timing): thread 0 of workgroup b writes the
// shader clock at phase boundary i to g_phase[b % 4096][i], the 100 MHz real-time
// clock at entry / exit to g_rt[b % 4096][0 / 1].  Compiled out of the product.
#ifdef GPI_PHASE_TIMING
// (hidden visibility: the stamps address the arrays PC-relative -- as default-visibility symbols of a -fPIC
// library each stamp loaded the address from the GOT first, one scalar-load round trip per stamp that
// inflated every measured phase by ~0.5-1 k cycles, r06)
__device__ __attribute__((visibility("hidden"))) unsigned long long g_phase[4096 * 16];
__device__ __attribute__((visibility("hidden"))) unsigned long long g_rt[4096 * 2];
#define PHASE(i)                                                                                     \
    do {                                                                                             \
        if (threadIdx.x == 0) g_phase[(blockIdx.x & 4095) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// slot 15 of g_phase: where the workgroup ran (HW_ID: cu [11:8], sh [12], se [15:13]; XCC_ID << 32)
#define RTSTAMP(i)                                                                                 \
    do {                                                                                           \
        if (threadIdx.x == 0) {                                                                    \
            g_rt[(blockIdx.x & 4095) * 2 + (i)] = __builtin_amdgcn_s_memrealtime();                \
            if ((i) == 0)                                                                          \
                g_phase[(blockIdx.x & 4095) * 16 + 15] =                                           \
                    (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                \
                    ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);        \
        }                                                                                          \
    } while (0)
#else
#define PHASE(i) \
    do {         \
    } while (0)
#define RTSTAMP(i) \
    do {           \
    } while (0)
#endif

__host__ __device__ inline int fdiv2(int x) { return x >= 0 ? x / 2 : -((-x + 1) / 2); }
__host__ __device__ inline int cdiv2(int x) { return -fdiv2(-x); }
__host__ __device__ inline int pad256(int n) { return (n + 255) & ~255; }

// forward statistics epilogue: each wave's sums as fp64 atomics of its own (1) or the workgroup's sum through LDS (0)
#ifndef GPI_FWD_WAVE_ATOMICS
#define GPI_FWD_WAVE_ATOMICS 0
#endif
// forward (one pixel per thread): the per-channel weight offset forced into a VGPR (1) or left to the compiler (0)
#ifndef GPI_FWD_WVGPR
#define GPI_FWD_WVGPR 1
#endif

// Tile geometry: tile t of sample b covers output rows [t*th, (t+1)*th), all columns.
struct ConvGeom {
    int th, tiles, nblocks;
    int rh, P;      // input image: rows [iy0, iy0 + rh), pitch P = w_in + 2H
    int gh, PG;     // output-gradient image: rows [gy0, gy0 + gh), pitch PG = w_out + 2H
    int ph;         // owned input rows (backward)
    const float* zero;   // the zero page (kernel argument: no per-use address reload)
    int zreg;       // backward: the BN-backward operand z of the output in registers (<= ZREG chunks / thread)
    int npx;        // forward: horizontally adjacent output pixels per thread (1, 2, 4)
    int cg;         // forward, tiles of <= 128 pixels: input-channel groups computing partial sums in parallel
                    // (256 / pixels threads per pixel instead of one busy wave), summed through LDS
    int fuse;       // backward: the fused output-conv launch (forward + loss + backward, gpi_conv_loss_fused)
    int vsum;       // backward, single-channel stride-2 input conv (weight gradient only, vwg): the four waves'
                    // partial slab rows summed in LDS into one row per tile (vsum_op)
    int vshift;     // ... its weight gradient in the column-shift form (vwg, cout <= 8; GPI_VWG_SHIFT)
    int ucls;       // backward, 3x3 upsampling conv: weight-gradient columns (ci, row offset) per output-row parity
                    // (GPI_UP_ROWCLS; only where it saves a column block: 6 <= cin <= 8)
    int lsum;       // backward (MFMA weight gradient): the four waves' partial slab rows summed in LDS at the
                    // end into ONE row per tile (accumulators held in registers through the input gradient)
    int split;      // backward: 2 workgroups per tile, input gradient (blockIdx < nblocks) and weight gradient
                    // (the rest) in parallel on otherwise idle CUs (launches well under one round)
    int xcd;        // XCD-aware block order: the blocks the dispatcher deals to one XCD (b, b + 8, ...) take
                    // consecutive tiles (adjacent rows of one sample; with split, the two roles of a tile next
                    // to each other), so the halo rows two tiles share are read from HBM once into that
                    // XCD's L2 instead of once per XCD.  0: tile = blockIdx.x (xcd_mode)
    int grid;       // launched workgroups (xcd remap)
    // backward (GPI_HALF_TILES): tiles [nfull, nblocks) are half-height tiles (htiles per sample, geometry ha)
    // of samples [half_b, B).  A batch whose tile count is no multiple of the 256 CUs (the decoder's 288
    // samples: 1152 tiles) left half the CUs one workgroup more than the rest, and a launch lasts as long as
    // its busiest CUs (fused output conv: last exits 32.0 us on 5-workgroup CUs, 27.8 us on 4-workgroup
    // ones, tools/phase_probe.py); with the samples past the first 1024 tiles split into half tiles, every
    // CU gets four full tiles and one half (0.5679-0.5683 vs 0.5723-0.5730 ms per step, r04v)
    int nfull, half_b, htiles;
    struct Alt {
        int th, rh, gh, ph, zreg, in_sq, in_sr, in_sc, g_sq, g_sr, g_sc;
        Div d_in4, d_g4, d_tp;
    } ha;
    int alt;        // fused output conv: half the workgroups run the input gradient (VALU) before the weight
                    // gradient (MFMA), so a CU's co-resident workgroups overlap the two pipes (fuse_alt)
    uint32_t* sig;             // cross-stream hand-off (gpi_*_sig): workgroup 0 increments *sig at entry, i.e.
    const int64_t* sig_epoch;  // once every earlier kernel of the stream has completed (gpi_stream_signal)
    int in_sq, in_sr, in_sc;   // 256 chunks of the input image = (planes, rows, chunks)
    int g_sq, g_sr, g_sc;      // ... of the output-gradient image
    Div d_in4, d_P4, d_g4, d_PG4, d_cin, d_cout, d_win, d_tp, d_wout, d_w2;
#ifdef GPI_PHASE_TIMING
    int dbg;   // GPI_DBG_SKIP of the timing build (never the product): 1 skip wgrad, 2 dgrad, 4 loss atomics,
              // 8 return after the operand loads, 16 return at entry, 32 forward returns after its loads,
              // 64 forward skips its compute loop, 128 forward skips its statistics epilogue
#endif
};

// Work-skip switches exist only in the timing build (make timing); the product library always
// does all of the work.
#ifdef GPI_PHASE_TIMING
#define SKIP(G, bit) (((G).dbg & (bit)) != 0)
#else
#define SKIP(G, bit) false
#endif

// first input row and row count of the input image of output rows [o0, o0 + t)
__host__ __device__ inline void in_rows(int k, int s, int up, int pad, int o0, int t, int& i0, int& len) {
    if (up) {
        i0 = fdiv2(o0 - pad);
        len = fdiv2(o0 + t - 1 - pad + k - 1) - i0 + 1;
    } else {
        i0 = o0 * s - pad;
        len = (t - 1) * s + k;
    }
}

// output-gradient rows needed by the input rows owned by the tile (and by its own rows)
__host__ __device__ inline void g_rows(int k, int s, int pad, int o0, int t, int& g0, int& len) {
    if (s == 2) {
        g0 = cdiv2(2 * o0 + pad - k + 1);
        len = fdiv2(2 * o0 + 2 * t - 1 + pad) - g0 + 1;
    } else {
        g0 = o0 + pad - (k - 1);
        len = t + k - 1;
    }
}

// input rows whose gradient the tile owns (a partition of the input rows)
__host__ __device__ inline void owned_rows(int s, int up, int o0, int t, int& p0, int& len) {
    if (up) { p0 = o0 / 2; len = t / 2; }
    else if (s == 2) { p0 = 2 * o0; len = 2 * t; }
    else { p0 = o0; len = t; }
}

// Chunks (16 B) of the output's raw z image a backward thread holds in registers instead of LDS.
constexpr int ZREG = 3;

// Tiles: the forward computes one output pixel per thread (<= 256 per tile); the MFMA
// backward takes taller tiles (fewer halo rows and per-tile fixed costs per pixel).
int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}


bool conv_geom(const gpi_conv_desc& d, const gpi_groups& g, ConvGeom& G, bool fwd, bool fuse = false) {
    if (g.n_groups < 1 || g.n_groups > GPI_MAX_GROUPS) return false;
    if (d.cin < 1 || d.cin > GPI_MAX_CIN || d.cout < 1 || d.cout > GPI_MAX_COUT) return false;
    if (d.k != 1 && d.k != 3 && d.k != 5 && d.k != 7) return false;
    if (d.pad > HALO || (d.w_in & 3) || (d.w_out & 3) || d.w_out > 256) return false;
    if (d.upsample) {
        if (d.stride != 1 || d.h_out != 2 * d.h_in || d.w_out != 2 * d.w_in || d.pad != d.k / 2) return false;
    } else if (d.stride == 2) {
        if (d.h_in != 2 * d.h_out || d.w_in != 2 * d.w_out || d.pad != d.k / 2) return false;
    } else if (d.stride == 1) {
        if (d.h_in != d.h_out || d.w_in != d.w_out || d.pad != d.k / 2) return false;
    } else {
        return false;
    }
    const int B = g.start[g.n_groups] - g.start[0];
    if (g.start[0] != 0 || B <= 0) return false;
    // output pixels per tile (taller backward tiles only pay on planes >= 64 wide: measured);
    // GPI_TILE_FWD / GPI_TILE_BWD / GPI_TILE_S2 override the targets (tuning runs only)
    // Stride 2: the single-channel input conv (no input gradient) takes larger tiles, the backward of
    // the transition convs 4 output rows (more workgroups for the parity-class input gradient).
    // Forward: 1024-pixel tiles on planes >= 64 wide, 8 rows on 32-wide planes, 512 px below, halved
    // while the input row image exceeds 28 KB of LDS.
    // Backward: 8 output rows below 64 wide, 512 px on 64-wide planes; the upsampling convs 16 rows on
    // 32- and 64-wide planes, 1024 px on wider ones (per-operator sweeps with bench.py --kprof).
    static const int t_fwd = env_int("GPI_TILE_FWD", 512), t_fwd64 = env_int("GPI_TILE_FWD64", 1024),
                     t_bwd = env_int("GPI_TILE_BWD", 512), t_s2 = env_int("GPI_TILE_S2", 128),
                     t_s2brows = env_int("GPI_TILE_S2BROWS", 4), t_s2c1 = env_int("GPI_TILE_S2C1", 512),
                     t_bwdup = env_int("GPI_TILE_BWDUP", 1024), t_bwdrows = env_int("GPI_TILE_BWDROWS", 8),
                     t_fwdrows = env_int("GPI_TILE_FWDROWS", 8), t_fuse = env_int("GPI_TILE_FUSE", 1024);
    // Round 4 per-operator sweep with half tiles (profiles/r04z_tile_sweep.txt): 16-row tiles for the upsampling
    // forward on 32-wide planes (TransUp2.conv2 13.8 -> 11.2 us), the upsampling backward below 32 wide
    // (TransUp1.conv2 11.6 -> 10.2) and the 3x3 backward of <= 8 input channels on 32-wide planes (EncBlock1.dl1
    // 20.3 -> 19.0, DecBlock3.dl1 21.5 -> 20.9; with 10 channels the LDS image halves the resident workgroups:
    // LastTransUp.conv1 23.9 -> 32.5); 512-px tiles for the single-channel input conv (forward 11.0 -> 10.3 us;
    // the backward, with the column-shift weight gradient, 0.5535 vs 0.5554 ms/step: profiles/r04z_ab_s2c1.txt)
    static const int t_fwdup32 = env_int("GPI_TILE_FWDUP32", 16), t_bwdups = env_int("GPI_TILE_BWDUPS", 16),
                     t_bwd32k3 = env_int("GPI_TILE_BWD32K3", 16), t_s2c1f = env_int("GPI_TILE_S2C1F", 512),
                     t_fwdwide = env_int("GPI_TILE_FWDWIDE", 8);   // the 3x3 forward of >= 10 channels, 32 wide
    const int target =
        d.stride == 2 ? (d.cin == 1 ? (fwd ? t_s2c1f : t_s2c1) : (fwd ? t_s2 : t_s2brows * d.w_out))
        : fwd ? (d.w_out >= 64 ? t_fwd64
                               : (d.w_out >= 32 ? (d.upsample && d.w_out == 32 ? t_fwdup32
                                                   : (d.k == 3 && d.cin >= 10 && d.w_out == 32 ? t_fwdwide : t_fwdrows)) * d.w_out
                                                : t_fwd))
              : (d.upsample ? (d.w_out >= 32 ? t_bwdup / 64 * min(d.w_out, 64) : t_bwdups * d.w_out)
                            : (d.w_out >= 64 ? t_bwd
                                             : (d.w_out == 32 && d.k == 3 && d.cin <= 8 ? t_bwd32k3 : t_bwdrows) * d.w_out));
    // the backward of the loss-epilogue output conv (fused with its forward, K - 1 extra forward rows
    // per tile): 1024 px (r02 A/B: 16 rows 9 us per step faster than 8).  Keyed on the op, not on the
    // fusion, so gpi_conv_blocks' slab rows fit both launch forms.
    const bool loss_bwd = !fwd && (d.epilogue == GPI_EPI_GAUSS_LOSS || d.epilogue == GPI_EPI_GAUSS_EXP_LOSS);
    G.th = (loss_bwd ? t_fuse : target) / d.w_out;
    if (G.th < 1) G.th = 1;
    if (G.th > d.h_out) G.th = d.h_out;
    if (fwd && d.stride == 1 && !d.upsample) {
        for (;;) {
            int y0, rh;
            in_rows(d.k, 1, 0, d.pad, 0, G.th, y0, rh);
            const int half = G.th / 2;
            if (4 * d.cin * rh * (d.w_in + 2 * HALO) <= 28 * 1024 || half < 1 || d.h_out % half) break;
            G.th = half;
        }
    }
    if (d.upsample && G.th < 2) G.th = 2;   // upsampled tiles pair output rows (256-wide planes)
    while (d.h_out % G.th) --G.th;
    if (d.upsample && (G.th & 1)) return false;
    G.tiles = d.h_out / G.th;
    G.nblocks = B * G.tiles;
    int i0;
    in_rows(d.k, d.stride, d.upsample, d.pad, 0, G.th, i0, G.rh);
    if (d.upsample) G.rh += 1;   // parity-independent bound
    if (fuse) G.rh += d.k - 1;   // fused output conv: the forward's input rows above and below
    G.P = d.w_in + 2 * HALO;
    g_rows(d.k, d.stride, d.pad, 0, G.th, i0, G.gh);
    G.PG = d.w_out + 2 * HALO;
    owned_rows(d.stride, d.upsample, 0, G.th, i0, G.ph);
    // exactness of the magic divisions: largest dividend * divisor < 2^32
    const uint64_t lim = 1ull << 32;
    const uint64_t in4 = (uint64_t)G.rh * G.P / 4, g4 = (uint64_t)G.gh * G.PG / 4;
    const uint64_t ein = in4 * d.cin, eg = g4 * d.cout, eo = (uint64_t)G.ph * d.w_in;
    if (ein * in4 >= lim || in4 * (G.P / 4) >= lim || eg * g4 >= lim || g4 * (G.PG / 4) >= lim ||
        eo * d.w_in >= lim || 256ull * G.th * d.w_out >= lim)
        return false;
    G.zero = nullptr;   // set by launch()
    // forward: NPX adjacent output pixels per thread when the tile has >= 256 * NPX pixels (input row
    // window and weight reads shared by the NPX pixels); GPI_FWD_NPX caps it (tuning runs only)
    static const int npx_cap = env_int("GPI_FWD_NPX", 4);
    G.npx = 1;
    if (fwd) {
        const int tp = G.th * d.w_out;
        while (2 * G.npx <= npx_cap && tp >= 256 * 2 * G.npx && d.w_out % (2 * G.npx) == 0) G.npx *= 2;
    }
    G.cg = 1;
    if (fwd && G.npx == 1 && d.epilogue != GPI_EPI_GAUSS_LOSS && d.epilogue != GPI_EPI_GAUSS_EXP_LOSS) {
        // (kept on: without channel groups the C64 step is 1.9 us faster in the graph -- 0.5544 / 0.5552 / 0.5547
        // vs 0.5561 / 0.5567 / 0.5571 ms interleaved, profiles/r04z_ab_fwd_cg.txt -- but the one-chain channel
        // sum moves the 256^2 codec forward to 1.08e-5 of the fp64 oracle, over the 1e-5 bar, against 6.5e-6
        // with the groups: profiles/r04z_fwd_err_cg.txt)
        static const int cg_on = env_int("GPI_FWD_CG", 1);
        const int tp = G.th * d.w_out;
        if (cg_on && tp <= 128 && 256 % tp == 0 && !d.upsample && d.k <= 3) G.cg = std::min(256 / tp, d.cin);
    }
    // the BN-backward operand image in registers when it is small: LDS = gradient + input images only
    // (one more resident workgroup per CU on the 32x32 / 64x64 decoder planes)
    G.zreg = (!fwd && d.gout_mode == 0 && (int64_t)d.cout * G.gh * (G.PG / 4) <= (int64_t)ZREG * 256) ? 1 : 0;
    G.split = 0;   // decided by launch() from the LDS footprint
    G.fuse = fuse ? 1 : 0;
    G.lsum = 0;     // decided by launch() / gpi_conv_blocks from the LDS footprint (lsum_op)
    G.vsum = 0;     // decided by launch() / gpi_conv_blocks (vsum_op)
    {
        static const int vshift = env_int("GPI_VWG_SHIFT", 1);
        G.vshift = (!fwd && vshift && d.k == 7 && d.stride == 2 && d.cin == 1 && d.cout <= 8) ? 1 : 0;
        static const int ucls = env_int("GPI_UP_ROWCLS", 1);
        G.ucls = (!fwd && ucls && d.upsample && d.k == 3 && d.pad == 1 && (2 * d.cin + 15) / 16 < (3 * d.cin + 15) / 16)
                     ? 1 : 0;
    }
    G.xcd = 0;      // set by launch() (xcd_mode)
    G.alt = 0;
    G.grid = 0;     // set by launch()
    G.sig = nullptr;
    G.sig_epoch = nullptr;
#ifdef GPI_PHASE_TIMING
    static const int dbg = env_int("GPI_DBG_SKIP", 0);
    G.dbg = dbg;
#endif
    {
        const int P4 = G.P / 4, pl = G.rh * P4, Q4 = G.PG / 4, gl = G.gh * Q4;
        G.in_sq = 256 / pl;
        G.in_sr = (256 % pl) / P4;
        G.in_sc = (256 % pl) % P4;
        G.g_sq = 256 / gl;
        G.g_sr = (256 % gl) / Q4;
        G.g_sc = (256 % gl) % Q4;
    }
    G.d_in4 = mkdiv((int)in4);
    G.d_P4 = mkdiv(G.P / 4);
    G.d_g4 = mkdiv((int)g4);
    G.d_PG4 = mkdiv(G.PG / 4);
    G.d_cin = mkdiv(d.cin);
    G.d_cout = mkdiv(d.cout);
    G.d_win = mkdiv(d.w_in);
    G.d_tp = mkdiv(G.th * d.w_out);
    G.d_wout = mkdiv(d.w_out);
    G.d_w2 = mkdiv(d.w_in >= 2 ? d.w_in / 2 : 1);
    G.nfull = G.nblocks;
    G.half_b = B;
    G.htiles = 0;
    G.ha = ConvGeom::Alt{G.th, G.rh, G.gh, G.ph, G.zreg, G.in_sq, G.in_sr, G.in_sc, G.g_sq, G.g_sr, G.g_sc,
                         G.d_in4, G.d_g4, G.d_tp};
    // half tiles for the samples past the largest multiple of 256 tiles (GPI_HALF_TILES: 0 off, 1 the loss
    // op's backward only, 2 every backward launch)
    static const int half_tiles = env_int("GPI_HALF_TILES", 2);
    const int tot = B * G.tiles, base = tot & ~255;
    static const int half_fwd = env_int("GPI_HALF_FWD", 1);
    // (only launches of at most five tiles per CU, one round of resident workgroups: with several rounds
    // the dispatcher evens the CUs out itself, and the half tiles' extra rows and longer prologue cost --
    // the c128 step 1.616 vs 1.558 ms with every launch split)
    if (half_tiles && (fwd ? half_fwd && half_tiles > 1 && G.cg == 1 : (half_tiles > 1 || loss_bwd)) &&
        (G.th & 1) == 0 && base > 0 && tot != base && tot <= 5 * 256 && base % G.tiles == 0) {
        ConvGeom::Alt& a = G.ha;
        a.th = G.th / 2;
        int y0;
        in_rows(d.k, d.stride, d.upsample, d.pad, 0, a.th, y0, a.rh);
        if (d.upsample) a.rh += 1;
        if (fuse) a.rh += d.k - 1;
        g_rows(d.k, d.stride, d.pad, 0, a.th, y0, a.gh);
        owned_rows(d.stride, d.upsample, 0, a.th, y0, a.ph);
        a.zreg = (!fwd && d.gout_mode == 0 && (int64_t)d.cout * a.gh * (G.PG / 4) <= (int64_t)ZREG * 256) ? 1 : 0;
        const int P4 = G.P / 4, pl = a.rh * P4, Q4 = G.PG / 4, gq = a.gh * Q4;
        a.in_sq = 256 / pl;
        a.in_sr = (256 % pl) / P4;
        a.in_sc = (256 % pl) % P4;
        a.g_sq = 256 / gq;
        a.g_sr = (256 % gq) / Q4;
        a.g_sc = (256 % gq) % Q4;
        a.d_in4 = mkdiv(pl);
        a.d_g4 = mkdiv(gq);
        a.d_tp = mkdiv(a.th * d.w_out);
        const bool ok = d.gin_off < 0 || (((a.ph * d.w_in) & 15) == 0 && (d.stride != 2 || (a.ph & 1) == 0));
        if (!ok) a = ConvGeom::Alt{G.th, G.rh, G.gh, G.ph, G.zreg, G.in_sq, G.in_sr, G.in_sc, G.g_sq, G.g_sr, G.g_sc,
                                   G.d_in4, G.d_g4, G.d_tp};
        else {
        G.half_b = base / G.tiles;
        G.nfull = base;
        G.htiles = 2 * G.tiles;
        G.nblocks = base + (B - G.half_b) * G.htiles;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------------- compile-time shapes
// Every conv launch of the C64 step has a fixed shape: the kernel variant, the B-independent fields of the
// descriptor and the whole tile geometry (ConvGeom less the batch-dependent block counts).  conv_shapes.h
// (written by tools/gen_conv_shapes.py from the launches one step makes) lists them; a launch whose shape
// equals an entry runs the instantiation with SHP = that entry, which overwrites its by-value descriptor
// and geometry with the entry's constants at entry (fold_shape): the address arithmetic, the staging
// loops' trip counts and carries, the magic divisions and the variant branches fold to constants, and the
// argument block no longer needs SGPRs (40 v_writelane spills and ~1200 instructions
// before the first barrier of conv_bwd_kernel<3,1,0>).  Any other launch -- another grid, batch, tile
// override -- takes the generic instantiation (SHP = -1); GPI_CONV_SHAPES=0 forces it (A/B, tests).
#define SHAPE_D(X) X(k) X(stride) X(pad) X(upsample) X(cin) X(cout) X(h_in) X(w_in) X(h_out) X(w_out) \
    X(in_bn) X(gout_mode) X(epilogue) X(gin_accumulate)
#define SHAPE_G(X) X(th) X(tiles) X(rh) X(P) X(gh) X(PG) X(ph) X(zreg) X(npx) X(cg) X(fuse) X(vsum) X(vshift) \
    X(ucls) X(lsum) X(split) X(xcd) X(alt) X(in_sq) X(in_sr) X(in_sc) X(g_sq) X(g_sr) X(g_sc)
#define SHAPE_GD(X) X(d_in4) X(d_P4) X(d_g4) X(d_PG4) X(d_cin) X(d_cout) X(d_win) X(d_tp) X(d_wout) X(d_w2)
#define SHAPE_A(X) X(th) X(rh) X(gh) X(ph) X(zreg) X(in_sq) X(in_sr) X(in_sc) X(g_sq) X(g_sr) X(g_sc)
#define SHAPE_AD(X) X(d_in4) X(d_g4) X(d_tp)

struct ShapeC {
    // kernel variant: template arguments of the instantiation, and the signs of the offsets that switch work
    int fwd, fusek, half, exf, v3, cp, npxk, upk, has_gin, drop, wout, ext_in;
#define F(n) int D_##n;
    SHAPE_D(F)
#undef F
#define F(n) int G_##n;
    SHAPE_G(F)
#undef F
#define F(n) int M_##n, O_##n;
    SHAPE_GD(F)
#undef F
#define F(n) int A_##n;
    SHAPE_A(F)
#undef F
#define F(n) int AM_##n, AO_##n;
    SHAPE_AD(F)
#undef F
};

// (GPI_SHAPES_FILE: another table, for A/B builds of other tile rules -- tools/shape_variant.sh)
#if defined(GPI_SHAPES_FILE)
#include GPI_SHAPES_FILE
#elif __has_include("conv_shapes.h")
#include "conv_shapes.h"
#endif
#ifndef GPI_CONV_SHAPE_LIST
#define GPI_CONV_SHAPE_LIST
#define GPI_CONV_SHAPE_COUNT 0
#endif
constexpr ShapeC kShapes[GPI_CONV_SHAPE_COUNT + 1] = {GPI_CONV_SHAPE_LIST ShapeC{}};   // (+ a zero sentinel)
constexpr int kNumShapes = GPI_CONV_SHAPE_COUNT;
// Translation units of the shape instantiations: entries [kBounds[p], kBounds[p + 1]) are instantiated by this file
// compiled with GPI_CONV_SHAPE_PART = p (part 0: the bench workload's shapes, with the launch code; parts 1-3: the
// other configurations' shapes, each part its own object so they compile in parallel)
#ifndef GPI_CONV_SHAPE_BOUNDS
#define GPI_CONV_SHAPE_BOUNDS {0, GPI_CONV_SHAPE_COUNT, GPI_CONV_SHAPE_COUNT, GPI_CONV_SHAPE_COUNT, GPI_CONV_SHAPE_COUNT}
#endif
constexpr int kBounds[5] = GPI_CONV_SHAPE_BOUNDS;
#ifndef GPI_CONV_SHAPE_PART
#define GPI_CONV_SHAPE_PART 0
#endif

// the fused output conv's shape instantiation: which field groups it folds (bit 0 descriptor, 1 geometry,
// 2 magic divisors); 0: none, the launch keeps the generic kernel.  Its 5-wave budget is at 95 VGPRs already:
// with the descriptor folded as well the loss phase unrolls and spills (173 registers; 2-11 for the single
// groups under hipcc's default contraction), geometry + divisors fit (92 VGPRs) and cut the prologue from
// 1448 to 933 instructions (620 -> 371 VALU)
#ifndef GPI_FUSE_FOLD
#define GPI_FUSE_FOLD 6
#endif

// the launch's descriptor and geometry with the entry's constants (SHP >= 0; the host matched every field)
template <int SHP>
__device__ __forceinline__ void fold_shape(gpi_conv_desc& d, ConvGeom& G) {
    if constexpr (SHP >= 0) {
        constexpr ShapeC s = kShapes[SHP];
        constexpr int fm = s.fusek ? GPI_FUSE_FOLD : 7;
        if constexpr (fm & 1) {
#define F(n) d.n = s.D_##n;
        SHAPE_D(F)
#undef F
        }
        if constexpr (fm & 2) {
#define F(n) G.n = s.G_##n;
        SHAPE_G(F)
#undef F
#define F(n) G.ha.n = s.A_##n;
        SHAPE_A(F)
#undef F
        }
        if constexpr (fm & 4) {
#define F(n) G.n = Div{(uint32_t)s.M_##n, (uint32_t)s.O_##n};
        SHAPE_GD(F)
#undef F
#define F(n) G.ha.n = Div{(uint32_t)s.AM_##n, (uint32_t)s.AO_##n};
        SHAPE_AD(F)
#undef F
        }
        if constexpr (s.has_gin) __builtin_assume(d.gin_off >= 0); else d.gin_off = -1;
        if constexpr (s.drop) __builtin_assume(d.drop_off >= 0); else d.drop_off = -1;
        if constexpr (s.wout) __builtin_assume(d.wpart_off >= 0); else d.wpart_off = -1;
        if constexpr (s.ext_in) d.in_off = -1; else __builtin_assume(d.in_off >= 0);
        // without half tiles every tile is a full one (the grid holds nblocks tiles, or 2 nblocks split roles)
        if constexpr (!s.half) G.nfull = 0x7fffffff;
    }
}

__device__ __forceinline__ void glds4(const float* g, float* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 4, 0, 0);
}

__device__ __forceinline__ void glds16(const float* g, float* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// dst[e] = *src(e) for e in [0, total) by 4-byte LDS-DMA; src(e) == nullptr reads the
// zero page.  dst is padded to a multiple of 256 floats (whole waves write).
template <typename Src>
__device__ __forceinline__ void stage(float* dst, int total, const float* zero, Src src) {
    const int wb = threadIdx.x & ~63;
    for (int e0 = 0; e0 < total; e0 += 256) {
        if (e0 + wb < total) {
            const int e = e0 + (int)threadIdx.x;
            const float* p = e < total ? src(e) : nullptr;
            glds4(p ? p : zero, dst + e0 + wb);
        }
    }
}

// Chunk (16 B) e of a row image of planes of nr rows x P4 chunks decomposed as
// (plane q, row r, chunk c4), advanced by 256 chunks per step with constant carries
// (sq, sr, sc) = decomposition of 256, so a loop pays no division per chunk.
// GPI_STAGE_SEL: the row-image staging loops take each chunk's source by a select of the computed plane address
// and the zero page (0: the compiler's branchy form, A/B)
#ifndef GPI_STAGE_SEL
#define GPI_STAGE_SEL 1
#endif
struct ChunkIter {
    int q, r, c4;
    __device__ __forceinline__ void init(int e, int plane4, int P4, Div d_q4, Div d_p4) {
        q = dq(e, d_q4);
        const int rem = e - q * plane4;
        r = dq(rem, d_p4);
        c4 = rem - r * P4;
    }
    __device__ __forceinline__ void step(int sq, int sr, int sc, int P4, int nr) {
        c4 += sc;
        if (c4 >= P4) { c4 -= P4; ++r; }
        r += sr;
        if (r >= nr) { r -= nr; ++q; }
        q += sq;
    }
};

// Extra zero chunks staged after every row image: the maskless MFMA loops read up to a
// few floats past an image's last row.
constexpr int IMG_MARGIN4 = 16;
__host__ __device__ inline int img_floats(int nq, int nr, int P) { return pad256(4 * (nq * nr * (P / 4) + IMG_MARGIN4)); }

// Row image of nq planes (plane q at plane(q), an h x w plane): rows [r0, r0 + nr),
// LDS pitch P = w + 2 HALO.  16-byte LDS-DMA; halo chunks, rows outside [0, h) and the
// IMG_MARGIN4 tail chunks read the zero page.
template <typename Plane>
__device__ __forceinline__ void stage_img(float* dst, int nq, int nr, int P, Div d_q4, Div d_p4, int sq, int sr,
                                          int sc, int r0, int h, int w, const float* zero, Plane plane) {
    const int P4 = P >> 2, plane4 = nr * P4, total = nq * plane4 + IMG_MARGIN4;
    const int wb = threadIdx.x & ~63;
    const int c4lo = HALO / 4, c4hi = HALO / 4 + w / 4;
    ChunkIter it;
    it.init(threadIdx.x, plane4, P4, d_q4, d_p4);
    for (int e0 = 0; e0 < total; e0 += 256) {
        if (e0 + wb < total) {
            const int row = r0 + it.r;
            const bool ok = it.q < nq && row >= 0 && row < h && it.c4 >= c4lo && it.c4 < c4hi;
#if GPI_STAGE_SEL
            // the chunk's plane address computed for every lane (never dereferenced where !ok), then ONE select:
            // without the empty asm the compiler sank the address arithmetic under three exec-masked branches
            // (the bounds tests), ≈ 10 SALU + branch issue per chunk in the staging loops of every conv launch
            const float* pv = plane(it.q) + row * w + 4 * (it.c4 - c4lo);
            asm volatile("" : "+v"(pv));
            const float* p = ok ? pv : zero;
#else
            const float* p = ok ? plane(it.q) + row * w + 4 * (it.c4 - c4lo) : zero;
#endif
            glds16(p, dst + 4 * (e0 + wb));
        }
        it.step(sq, sr, sc, P4, nr);
    }
}

// Sums of the GPI_REPLICAS copies of the stat records of channels [0, na) of stat
// a and [0, nb) of stat b (group grp) into LDS: threads 8 * ch + 4 * h + k own field
// k of channel ch, replicas [16 h, 16 h + 16), all loads in flight at once; the two
// halves meet by a lane exchange.  na + nb <= 32.
constexpr int STAT_HALF = GPI_REPLICAS / 2;
struct StatLoad {
    double v[STAT_HALF];
    double* out;
};

__device__ __forceinline__ void stat_issue(const gpi_stat* stats, int64_t n_stats, int grp, int64_t sa, int na,
                                           double* da, int64_t sb, int nb, double* db, const float* zero, StatLoad& L) {
    const int t = threadIdx.x, k = t & 3, h = (t >> 2) & 1, ch = t >> 3;
    const double* p = (const double*)zero;
    int64_t step = 0;
    L.out = nullptr;
    // layout [GPI_REPLICAS][group][stat]: consecutive channels of one replica share cache lines
    const int64_t rstride = n_stats * GPI_MAX_GROUPS * 4;   // doubles per replica
    const gpi_stat* sg = stats + (int64_t)grp * n_stats;
    if (ch < na) {
        p = &sg[sa + ch].sum + k + h * STAT_HALF * rstride;
        step = rstride;
        L.out = da + 4 * ch + k;
    } else if (ch - na < nb) {
        p = &sg[sb + ch - na].sum + k + h * STAT_HALF * rstride;
        step = rstride;
        L.out = db + 4 * (ch - na) + k;
    }
    const auto g = (const __attribute__((address_space(1))) double*)p;
#pragma unroll
    for (int r = 0; r < STAT_HALF; ++r) L.v[r] = g[r * step];
}

__device__ __forceinline__ void stat_finish(StatLoad& L) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < STAT_HALF; r += 2) {
        s0 += L.v[r];
        s1 += L.v[r + 1];
    }
    double s = s0 + s1;
    s += __shfl_xor(s, 4, 64);
    if (L.out && !(threadIdx.x & 4)) *L.out = s;
}

__device__ __forceinline__ gpi_stat* stat_slot(const gpi_codec_ctx& c, int64_t stat, int grp) {
    const int r = blockIdx.x % GPI_REPLICAS;
    return c.stats + ((int64_t)r * GPI_MAX_GROUPS + grp) * c.n_stats + stat;
}

// BN coefficients: every rounding spelled out (explicit FMAs, no compiler contraction choice), so a
// host can reproduce the kernels' ReLU decisions bit for bit (tests/gpu_masks.py)
__device__ __forceinline__ void mean_invstd(const double* s4, double n, float eps, float& mean, float& invstd) {
    const double m = s4[0] / n;
    double var = fma(-m, m, s4[1] / n);
    if (var < 0.0) var = 0.0;
    mean = (float)m;
    invstd = (float)(1.0 / sqrt(var + (double)eps));
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

// Keep a kernel argument in a register from kernel entry on: the compiler cannot
// rematerialise the value of an opaque asm, so it never re-reads the (large, by-value)
// argument block with a dependent s_load + s_waitcnt in the middle of a phase.
template <typename T>
__device__ __forceinline__ T pin(T v) {
    asm volatile("" : "+s"(v));
    return v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Every 64-byte line of the kernel-argument segment, touched by ONE batch of scalar loads at entry.
// The compiler issues argument loads lazily, next to their first use, and the large by-value
// descriptors (~0.5 KB) made that 3 to 4 dependent round trips to the argument segment before a
// tile's operand loads were even issued (tools/prologue_waits.sh).  With every line in the scalar
// cache after this one round trip, the later lazy loads hit it.
template <int NBYTES>
__device__ __forceinline__ void touch_kernargs() {
    const __attribute__((address_space(4))) uint32_t* ka =
        (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
    constexpr int NL = (NBYTES + 63) / 64;
    uint32_t x[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) x[i] = ka[16 * i];      // all lines in flight, one wait below
#pragma unroll
    for (int i = 0; i < NL; ++i) asm volatile("" : : "s"(x[i]));
}
constexpr int CONV_KARG_BYTES = (int)(sizeof(gpi_conv_desc) + sizeof(gpi_codec_ctx) + sizeof(ConvGeom) + 16);

// the launch's hand-off signal (G.sig): one relaxed agent-scope atomic increment by workgroup 0 at entry,
// fire and forget -- the kernels before this one on its stream have completed and released their writes
// by the time it starts (the counter protocol of gpi_stream_signal)
__device__ __forceinline__ void entry_signal(const ConvGeom& G) {
    if (G.sig && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_add(G.sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Global-address-space views of (pinned, hence generic) pointers: ordinary loads and
// stores through them stay global_load / global_store.  A flat access could alias LDS,
// so the compiler would drain every outstanding LDS-DMA (vmcnt(0)) in front of it.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* as_gld(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* as_gst(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

struct TileIdx {
    int b, oy0, grp, gsz;
};

// logical block of this workgroup: identity, or (G.xcd) the blocks of dispatcher XCD slot x = b % 8
// numbered consecutively -- XCD x holds logical blocks [x q + min(x, r), ...) for grid = 8 q + r.
// A bijection on [0, grid) for any grid; placement affects speed only, never the result.
__device__ __forceinline__ int logical_block(const ConvGeom& G) {
    const int b = blockIdx.x;
    if (!G.xcd) return b;
    const int q = G.grid >> 3, r = G.grid & 7, x = b & 7;
    return x * q + min(x, r) + (b >> 3);
}

__device__ __forceinline__ TileIdx tile_of(const ConvGeom& G, const gpi_groups& g, int tile = -1) {
    if (tile < 0) tile = logical_block(G);
    TileIdx t;
    if (tile < G.nfull) {
        t.b = tile / G.tiles;
        t.oy0 = (tile - t.b * G.tiles) * G.th;
    } else {                         // half-height tiles (GPI_HALF_TILES)
        const int u = tile - G.nfull, q = u / G.htiles;
        t.b = G.half_b + q;
        t.oy0 = (u - q * G.htiles) * G.ha.th;
    }
    t.grp = group_of(g, t.b);
    t.gsz = karg_sel(g.start, t.grp + 1) - karg_sel(g.start, t.grp);
    return t;
}

// Base of input channel in_c0 of the tile's sample (global).  ext input: one
// dependent index load (the encoder's first conv only).
__device__ __forceinline__ const float* input_base(const gpi_conv_desc& d, const gpi_codec_ctx& c, int b) {
    const int HWi = d.h_in * d.w_in;
    if (d.in_off >= 0) return c.ws + d.in_off + ((int64_t)b * d.in_ctot + d.in_c0) * HWi;
    return c.ext_in + (int64_t)(c.ext_idx ? c.ext_idx[b] : b) * c.ext_stride + (int64_t)d.in_c0 * HWi;
}

// In-place BN + ReLU of an input row image (16-byte chunks); halo chunks and rows
// outside the plane keep their zeros.
__device__ __forceinline__ void activate_img(float* img, const ConvGeom& G, const gpi_conv_desc& d, int iy0,
                                             const float* sc, const float* sh) {
    const int P4 = G.P >> 2, plane4 = G.rh * P4, total = d.cin * plane4;
    const int c4lo = HALO / 4, c4hi = HALO / 4 + d.w_in / 4;
    float4* im4 = reinterpret_cast<float4*>(img);
    ChunkIter it;
    it.init(threadIdx.x, plane4, P4, G.d_in4, G.d_P4);
    for (int e0 = threadIdx.x; e0 < total; e0 += 512) {
        float4 v[2];
        bool ok[2];
        int ci[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = iy0 + it.r;
            ok[u] = e0 + 256 * u < total && row >= 0 && row < d.h_in && it.c4 >= c4lo && it.c4 < c4hi;
            ci[u] = it.q;
            if (ok[u]) v[u] = im4[e0 + 256 * u];
            it.step(G.in_sq, G.in_sr, G.in_sc, P4, G.rh);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (ok[u]) {
                const float a = sc[ci[u]], b = sh[ci[u]];
                float4 o;
                o.x = fmaxf(fmaf(v[u].x, a, b), 0.f);
                o.y = fmaxf(fmaf(v[u].y, a, b), 0.f);
                o.z = fmaxf(fmaf(v[u].z, a, b), 0.f);
                o.w = fmaxf(fmaf(v[u].w, a, b), 0.f);
                im4[e0 + 256 * u] = o;
            }
        }
    }
}

// win[t] = p[t], t < NW, where p - OFF is 16-byte aligned (OFF in 0..3): whole 16-B LDS reads.
// A wave's lanes take 4-pixel groups of consecutive rows; single-dword window reads of such a
// layout hit 16 distinct banks 4 ways (rows 8 banks apart, lanes 4 apart), 16-B reads of 16 lanes
// cover all 64 banks once.  Reads up to 4 * ceil((OFF + NW) / 4) floats from p - OFF (callers keep
// that inside the row pitch).
template <int NW, int OFF>
__device__ __forceinline__ void lds_window(const float* p, float (&win)[NW]) {
    constexpr int NCH = (OFF + NW + 3) / 4;
    const float4* q = reinterpret_cast<const float4*>(p - OFF);
    float buf[4 * NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const float4 v = q[c];
        buf[4 * c] = v.x;
        buf[4 * c + 1] = v.y;
        buf[4 * c + 2] = v.z;
        buf[4 * c + 3] = v.w;
    }
#pragma unroll
    for (int t = 0; t < NW; ++t) win[t] = buf[OFF + t];
}

// Activation / gradient stores of the conv epilogues: write-through (sc1) stores, which leave no dirty
// line in the XCD's L2 for the kernel-end release to write back (the next launch reads them from memory
// either way: other XCDs' L2s never see this one's lines).  C64 step 0.6267 vs 0.6346 ms with plain
// stores (r02 A/B, 3 x 300 replays each; 0.630 vs 0.633 on a second box); GPI_PLAIN_STORES builds the
// plain form for A/B runs.  The weight-gradient slab partials (scattered dwords) stay plain: write-through
// measured slower there (0.636-0.652 ms).
#ifndef GPI_PLAIN_STORES
// relaxed agent-scope atomic stores lower to global_store_dword[x2] sc1 (the compiler schedules and
// allocates them like ordinary stores)
// (global address space: a generic pointer would make them flat stores, which also count against the LDS
// counter and are ordered against LDS traffic)
__device__ __forceinline__ void st2(float* p, f32x2 v) {
    __hip_atomic_store((__attribute__((address_space(1))) uint64_t*)p, __builtin_bit_cast(uint64_t, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4(float* p, f32x4 v) {
    // no 16-byte atomic store exists to lower it from; as two 8-byte halves it measured slower.
    // The s_nop: a store of more than 8 data bytes reads its data VGPRs after issue, and a VALU write to them
    // right behind it is a hazard the compiler's hazard recognizer does not see through inline asm -- the
    // compile-time shape instantiations scheduled such a write there and stored clobbered values (r06)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v));
}
__device__ __forceinline__ void st1(float* p, float v) {
    __hip_atomic_store((__attribute__((address_space(1))) float*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#else
__device__ __forceinline__ void st4(float* p, f32x4 v) { *as_gst((f32x4*)p) = v; }
__device__ __forceinline__ void st2(float* p, f32x2 v) { *as_gst((f32x2*)p) = v; }
__device__ __forceinline__ void st1(float* p, float v) { *as_gst(p) = v; }
#endif

// NPX consecutive floats of one output row (16-B / 8-B aligned: x0 is a multiple of NPX, planes are
// multiples of 4 floats, buffers 16-B aligned -- aligned_ok)
template <int NPX>
__device__ __forceinline__ void store_px(float* p, const float (&v)[NPX]) {
    if constexpr (NPX == 4) {
        st4(p, f32x4{v[0], v[1], v[2], v[3]});
    } else if constexpr (NPX == 2) {
        st2(p, f32x2{v[0], v[1]});
    } else {
#pragma unroll
        for (int q = 0; q < NPX; ++q) st1(p + q, v[q]);
    }
}

// ---------------------------------------------------------------------------------- forward
// header floats: gst fp64 [4*MAX_CIN] | sc | sh [MAX_CIN] | scratch [64] | red [16] | dropout scales [8]
constexpr int FWD_HDR = 8 * GPI_MAX_CIN + 2 * GPI_MAX_CIN + 64 + 16 + 8;

template <int K, int S, int UP, int CP, int NPX, bool HALF = false, int SHP = -1>
// (the channel-group instantiation NPX == 0 runs one workgroup per CU: no occupancy target)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NPX == 0 ? 1 : 5))) void conv_fwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    fold_shape<SHP>(d, G);
    touch_kernargs<CONV_KARG_BYTES>();
    entry_signal(G);
    if (SKIP(G, 16)) return;
    // the tile's geometry: the launch's, or the half-height one (HALF instantiation, GPI_HALF_TILES)
    ConvGeom Gt_;
    if constexpr (HALF) {
        Gt_ = G;
        if (logical_block(G) >= G.nfull) {
            const ConvGeom::Alt& a = G.ha;
            Gt_.th = a.th; Gt_.rh = a.rh; Gt_.in_sq = a.in_sq; Gt_.in_sr = a.in_sr; Gt_.in_sc = a.in_sc;
            Gt_.d_in4 = a.d_in4; Gt_.d_tp = a.d_tp;
        }
    }
    const ConvGeom& Gt = HALF ? Gt_ : G;
    constexpr int KK = K * K;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    double* gst = (double*)smem;
    float* sc = smem + 8 * GPI_MAX_CIN;
    float* sh = sc + GPI_MAX_CIN;
    float* scratch = sh + GPI_MAX_CIN;   // 2*CP*4 <= 64
    float* red = scratch + 64;           // 2*CP <= 16
    float* dsl = red + 16;               // [CP] Dropout2d scales of this sample's output channels
    float* wT = smem + pad256(FWD_HDR);  // [cin][KK][CP]
    const int nw = d.cin * KK * CP;
    float* img = wT + pad256(nw);        // [cin][rh][P] + zero margin

    const int tid = threadIdx.x;
    RTSTAMP(0);
    PHASE(0);
    float* const ws = pin(c.ws);
    const float* const params = pin(c.params);
    const float* const zero = pin(Gt.zero);
    const int64_t w_off = pin(d.w_off);
    const TileIdx T = tile_of(Gt, c.groups);
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;
    const float* ib = input_base(d, c, T.b);
    // Dropout2d after this conv: the sample's output-channel scales (0 or 1/(1-p)) into LDS (read by
    // the epilogue after the barriers below; no registers held across the compute)
    const bool drop = d.drop_off >= 0;
    PHASE(1);

    // ---- phase 1: every global read of the tile in flight together
    stage(wT, nw, zero, [&](int e) -> const float* {
        const int co = e % CP, r = e / CP;
        return co < d.cout ? params + w_off + (int64_t)co * d.cin * KK + r : nullptr;
    });
    int iy0, rh_;
    in_rows(K, S, UP, d.pad, T.oy0, Gt.th, iy0, rh_);
    stage_img(img, d.cin, Gt.rh, Gt.P, Gt.d_in4, Gt.d_P4, Gt.in_sq, Gt.in_sr, Gt.in_sc, iy0, d.h_in, d.w_in, zero,
              [&](int q) -> const float* { return ib + (int64_t)q * HWi; });
    // (issued after the DMA; stored to LDS only after the stat loads are issued and waited for -- an
    // LDS store of it right here would drain every outstanding DMA first: one more round trip)
    float dsv = 1.f;
    if (drop && tid >= 64 && tid < 64 + d.cout) dsv = *as_gld(ws + d.drop_off + (int64_t)T.b * d.cout + (tid - 64));
    if (d.in_bn) {
        float gam = 0.f, bet = 0.f;
        if (tid < d.cin) {
            gam = *as_gld(params + d.gamma_off + tid);
            bet = *as_gld(params + d.beta_off + tid);
        }
        StatLoad L;
        stat_issue(c.stats, c.n_stats, T.grp, d.in_stat, d.cin, gst, 0, 0, nullptr, zero, L);
        stat_finish(L);
        __syncthreads();
        if (SKIP(G, 8) || SKIP(G, 32)) return;
        PHASE(2);
        // ---- phase 2: BN coefficients
        if (tid < d.cin) {
            float mean, inv;
            mean_invstd(gst + 4 * tid, (double)T.gsz * HWi, c.bn_eps, mean, inv);
            sc[tid] = gam * inv;
            sh[tid] = fmaf(-(mean * gam), inv, bet);   // explicit FMA (bn_coefs): no contraction choice
        }
        __syncthreads();
        // ---- phase 3: BN + ReLU in LDS
        activate_img(img, Gt, d, iy0, sc, sh);
    }
    if (drop && tid >= 64 && tid < 64 + d.cout) dsl[tid - 64] = dsv;
    __syncthreads();
    PHASE(4);

    // ---- phase 4: compute.  NPX == 1: one output pixel per thread and pass (two passes only for the
    // 256-wide upsampled planes, whose tiles pair output rows).  NPX > 1: NPX horizontally adjacent
    // pixels per thread; per (ci, ky) the thread reads the input row window the NPX x K taps cover
    // once into registers, and every weight vector read serves NPX pixels.
    const int tp = Gt.th * d.w_out;
    float Lv = 0.f;
    float vst[2 * CP];
#pragma unroll
    for (int q = 0; q < 2 * CP; ++q) vst[q] = 0.f;
    const bool gauss = d.epilogue == GPI_EPI_GAUSS_LOSS || d.epilogue == GPI_EPI_GAUSS_EXP_LOSS;
    if constexpr (NPX > 1) {
        constexpr int PADK = K / 2;   // launch() checks pad == k / 2
        // window column of tap kx of pixel p (x0 is a multiple of NPX, even, for the upsampling offsets)
        constexpr int NW = UP ? ((NPX - 1 + K - 1 + (PADK & 1)) >> 1) + 1 : (NPX - 1) * S + K;
        const int ng = tp / NPX;
        for (int gbase = 0; gbase < ng; gbase += 256) {
            const int g = gbase + tid;
            const bool active = g < ng;
            const int ty = dq(g * NPX, Gt.d_wout), x0 = g * NPX - ty * d.w_out;
            const int oy = T.oy0 + ty;
            float acc[NPX][CP];
#pragma unroll
            for (int p = 0; p < NPX; ++p)
#pragma unroll
                for (int co = 0; co < CP; ++co) acc[p][co] = 0.f;
            if (active && !SKIP(G, 64)) {
                const int plane = Gt.rh * Gt.P;
                const int cb = UP ? fdiv2(x0 - PADK) + HALO : x0 * S - PADK + HALO;
                for (int ci = 0; ci < d.cin; ++ci) {
                    const float* tci = img + ci * plane + cb;
                    const float* wci = wT + ci * KK * CP;
#pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        const int ry = UP ? (fdiv2(oy - PADK + ky) - iy0) : (ty * S + ky);
                        const float* trow = tci + ry * Gt.P;
                        float win[NW];
                        if constexpr (!UP && (NPX * S) % 4 == 0) {
                            // x0 * S is a multiple of 4: the window starts (HALO - K/2) mod 4 past a 16-B boundary
                            lds_window<NW, (HALO - PADK) & 3>(trow, win);
                        } else {
#pragma unroll
                            for (int t = 0; t < NW; ++t) win[t] = trow[t];
                        }
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            float wv[CP];
                            const float* wp = wci + (ky * K + kx) * CP;
                            if constexpr (CP % 4 == 0) {
#pragma unroll
                                for (int q = 0; q < CP / 4; ++q) {
                                    const float4 w4 = reinterpret_cast<const float4*>(wp)[q];
                                    wv[4 * q] = w4.x;
                                    wv[4 * q + 1] = w4.y;
                                    wv[4 * q + 2] = w4.z;
                                    wv[4 * q + 3] = w4.w;
                                }
                            } else {
#pragma unroll
                                for (int q = 0; q < CP / 2; ++q) {
                                    const float2 w2 = reinterpret_cast<const float2*>(wp)[q];
                                    wv[2 * q] = w2.x;
                                    wv[2 * q + 1] = w2.y;
                                }
                            }
#pragma unroll
                            for (int p = 0; p < NPX; ++p) {
                                const float v = win[UP ? ((p + kx + (PADK & 1)) >> 1) : p * S + kx];
#pragma unroll
                                for (int co = 0; co < CP; ++co) acc[p][co] = fmaf(wv[co], v, acc[p][co]);
                            }
                        }
                    }
                }
            }
            if (drop) {
#pragma unroll
                for (int co = 0; co < CP; ++co) {
                    const float ds = co < d.cout ? dsl[co] : 1.f;
#pragma unroll
                    for (int p = 0; p < NPX; ++p) acc[p][co] *= ds;
                }
            }
            const int64_t pix0 = (int64_t)oy * d.w_out + x0;
            if (gauss) {
                if (active) {
                    int row = T.b - karg_sel(c.groups.start, T.grp);
                    if (const int32_t* ti = karg_sel(c.tgt_idx, T.grp)) row = ti[row];
                    const float* tg = karg_sel(c.tgt, T.grp) + (int64_t)row * HWo + pix0;
                    const bool ex = d.epilogue == GPI_EPI_GAUSS_EXP_LOSS;
                    const float scl = karg_sel(c.loss_scale, T.grp);
                    float g0[NPX], g1[NPX];
#pragma unroll
                    for (int p = 0; p < NPX; ++p) {
                        const float tgt = tg[p];
                        const float mu = acc[p][0], ls = acc[p][1];
                        const float e = expf(-2.f * ls);
                        const float emu = ex ? expf(mu) : 1.f;
                        const float r = ex ? expf(tgt) - emu : tgt - mu;
                        Lv += -0.5f * (2.f * ls + r * r * e + GPI_LOG2PI);
                        g0[p] = -scl * r * e * emu;
                        g1[p] = scl * (1.f - r * r * e);
                    }
                    float* go = ws + d.gout_off + (int64_t)T.b * 2 * HWo + pix0;
                    store_px<NPX>(go, g0);
                    store_px<NPX>(go + HWo, g1);
                    if (d.out_off >= 0) {
                        float m0[NPX], m1[NPX];
#pragma unroll
                        for (int p = 0; p < NPX; ++p) {
                            m0[p] = acc[p][0];
                            m1[p] = acc[p][1];
                        }
                        float* o = ws + d.out_off + ((int64_t)T.b * d.out_ctot + d.out_c0) * HWo + pix0;
                        store_px<NPX>(o, m0);
                        store_px<NPX>(o + HWo, m1);
                    }
                }
                continue;
            }
            if (active) {
                float* o = ws + d.out_off + ((int64_t)T.b * d.out_ctot + d.out_c0) * HWo + pix0;
#pragma unroll
                for (int co = 0; co < CP; ++co) {
                    if (co < d.cout) {
                        float v[NPX];
#pragma unroll
                        for (int p = 0; p < NPX; ++p) v[p] = acc[p][co];
                        store_px<NPX>(o + (int64_t)co * HWo, v);
                    }
                }
            }
            if (d.epilogue == GPI_EPI_STORE_STATS) {
#pragma unroll
                for (int co = 0; co < CP; ++co) {
#pragma unroll
                    for (int p = 0; p < NPX; ++p) {
                        const float a = (active && co < d.cout) ? acc[p][co] : 0.f;
                        vst[2 * co] += a;
                        vst[2 * co + 1] += a * a;
                    }
                }
            }
        }
    } else {
        // NPX == 0: the channel-group instantiation (Gt.cg > 1), otherwise one group (folds away)
        const int cg = NPX == 0 ? Gt.cg : 1;
        for (int pbase = 0; pbase < tp; pbase += 256) {
            // cg > 1 (tp <= 128, one pass): thread = (channel group, pixel)
            const int grp = NPX == 0 ? dq(tid, Gt.d_tp) : 0;
            const int pix = NPX == 0 ? tid - grp * tp : pbase + tid;
            const int ty = dq(pix, Gt.d_wout), tx = pix - ty * d.w_out;
            const int oy = T.oy0 + ty, ox = tx;
            bool active = pix < tp && grp < cg;
            float tgt = 0.f;
            if (gauss && active) {
                int row = T.b - karg_sel(c.groups.start, T.grp);
                if (const int32_t* ti = karg_sel(c.tgt_idx, T.grp)) row = ti[row];
                tgt = karg_sel(c.tgt, T.grp)[(int64_t)row * HWo + oy * d.w_out + ox];
            }
            PHASE(5);
            float acc[CP];
    #pragma unroll
            for (int co = 0; co < CP; ++co) acc[co] = 0.f;
            if (active && !SKIP(G, 64)) {
                const int plane = Gt.rh * Gt.P;
                for (int ci = grp; ci < d.cin; ci += cg) {
                    const float* tci = img + ci * plane;
                    // the weight offset held in a VGPR: the uniform LDS reads then take one VGPR base with
                    // immediate offsets (as an SGPR address every read needed its own v_mov of the address)
                    int wofs = pad256(FWD_HDR) + ci * KK * CP;      // wT = smem + pad256(FWD_HDR)
                    if (GPI_FWD_WVGPR) asm volatile("" : "+v"(wofs));
                    const float* wci = smem + wofs;
    #pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        const int ry = UP ? (fdiv2(oy - d.pad + ky) - iy0) : (ty * S + ky);
                        const float* trow = tci + ry * Gt.P;
    #pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            const int col = UP ? fdiv2(ox - d.pad + kx) + HALO : ox * S - d.pad + kx + HALO;
                            fma_vec<CP>(acc, wci + (ky * K + kx) * CP, trow[col]);
                        }
                    }
                }
            }
            if (NPX == 0 && cg > 1) {
                // channel-group partials [grp - 1][pix][CP] after the image; group 0 sums them in group order
                float* part = img + img_floats(d.cin, Gt.rh, Gt.P);
                if (active && grp > 0) {
    #pragma unroll
                    for (int co = 0; co < CP; ++co) part[((grp - 1) * tp + pix) * CP + co] = acc[co];
                }
                __syncthreads();
                if (active && grp == 0) {
                    for (int g = 1; g < cg; ++g) {
    #pragma unroll
                        for (int co = 0; co < CP; ++co) acc[co] += part[((g - 1) * tp + pix) * CP + co];
                    }
                }
                active = active && grp == 0;
            }
            PHASE(6);
            if (drop) {
    #pragma unroll
                for (int co = 0; co < CP; ++co)
                    if (co < d.cout) acc[co] *= dsl[co];
            }
            if (gauss) {
                if (active) {
                    const float mu = acc[0], ls = acc[1];
                    const float e = expf(-2.f * ls);
                    // log-property Gaussian (default) or the exponentiated field's (d mean: chain factor exp(mu))
                    const bool ex = d.epilogue == GPI_EPI_GAUSS_EXP_LOSS;
                    const float emu = ex ? expf(mu) : 1.f;
                    const float r = ex ? expf(tgt) - emu : tgt - mu;
                    Lv += -0.5f * (2.f * ls + r * r * e + GPI_LOG2PI);
                    const float scl = karg_sel(c.loss_scale, T.grp);
                    auto go = as_gst(ws + d.gout_off + (int64_t)T.b * 2 * HWo + oy * d.w_out + ox);
                    go[0] = -scl * r * e * emu;
                    go[HWo] = scl * (1.f - r * r * e);
                    if (d.out_off >= 0) {
                        auto o = as_gst(ws + d.out_off + (int64_t)T.b * d.out_ctot * HWo + (int64_t)d.out_c0 * HWo +
                                     oy * d.w_out + ox);
                        o[0] = mu;
                        o[HWo] = ls;
                    }
                }
                continue;
            }
            if (active) {
                float* o = ws + d.out_off + ((int64_t)T.b * d.out_ctot + d.out_c0) * HWo + oy * d.w_out + ox;
    #pragma unroll
                for (int co = 0; co < CP; ++co)
                    if (co < d.cout) st1(o + (int64_t)co * HWo, acc[co]);
            }
            if (d.epilogue == GPI_EPI_STORE_STATS) {
    #pragma unroll
                for (int co = 0; co < CP; ++co) {
                    const float a = (active && co < d.cout) ? acc[co] : 0.f;
                    vst[2 * co] += a;
                    vst[2 * co + 1] += a * a;
                }
            }
        }
    }

    if (d.epilogue == GPI_EPI_GAUSS_LOSS || d.epilogue == GPI_EPI_GAUSS_EXP_LOSS) {
        float v[1] = {Lv};
        block_sum<1>(v, scratch, red);      // thread 0 wrote red[0] itself: no barrier before reading it
        if (tid == 0 && !SKIP(G, 4)) atomicAdd(c.loss_acc + T.grp * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS, (double)red[0]);
        PHASE(7);
        RTSTAMP(1);
        return;
    }
    if (d.epilogue == GPI_EPI_STORE_STATS && !SKIP(G, 128)) {
#if GPI_FWD_WAVE_ATOMICS
        // per-wave sums straight to the fp64 replicas (no LDS stage, no barrier): 4 atomics per (channel, stat)
        // per workgroup instead of 1, the wave's own replica (4 blockIdx + wave)
        wave_sums(vst);
        const int lane = tid & 63;
        if (lane < 2 * d.cout && !SKIP(G, 4)) {
            float v = vst[0];
#pragma unroll
            for (int q = 1; q < 2 * CP; ++q) v = lane == q ? vst[q] : v;
            gpi_stat* st = c.stats + ((int64_t)((4 * blockIdx.x + (tid >> 6)) % GPI_REPLICAS) * GPI_MAX_GROUPS + T.grp) *
                                         c.n_stats + d.out_stat + (lane >> 1);
            atomicAdd((lane & 1) ? &st->sumsq : &st->sum, (double)v);
        }
#else
        block_sum<2 * CP>(vst, scratch, red);   // thread t < 2 CP wrote red[t] itself: no barrier
        if (tid < 2 * d.cout && !SKIP(G, 4)) {
            gpi_stat* st = stat_slot(c, d.out_stat + (tid >> 1), T.grp);
            atomicAdd((tid & 1) ? &st->sumsq : &st->sum, (double)red[tid]);
        }
#endif
    }
    PHASE(7);
    RTSTAMP(1);
}

// ---------------------------------------------------------------------------------- backward
// MFMA (v_mfma_f32_16x16x4_f32, exact f32 fmaf chains) for both contractions:
//  * weight gradient by the column-shift form
//      dW[(co,kx)][(ci,ky)] = sum_{ty,x} g[co][ty][ox(x, kx)] * a[ci][row(ty,ky)][col(x)]
//    (x runs over the virtual input columns of an output row: rows M = cout*K,
//    columns N = cin*K), the reduction split over the four waves by output row
//    and summed in LDS in a fixed order;
//  * input gradient as [owned pixels] x [cin] with reduction over (co, ky, kx):
//    A = the output-gradient window of the pixel (LDS), B = W (LDS, [co*KK+tap][16]).
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// header floats, sized by the launch's channel counts: gst fp64 [4*(cin+cout)] | i_sc i_sh i_mean i_inv i_gam [cin]
// | o_coef [4*cout] | o_drop [cout], padded to 64 floats (LDS is the residency limit of the large backward
// launches: <= 31 KB gives 5 workgroups per CU, measured tools/bench_dispatch.hip)
__host__ __device__ inline int pad64(int n) { return (n + 63) & ~63; }
__host__ __device__ inline int bwd_hdr(int cin, int cout) { return pad64(8 * (cin + cout) + 5 * cin + 5 * cout); }
// ops whose backward takes the VALU input gradient with SGPR weights (the decoder's 5x5 output conv)
__host__ __device__ inline bool vop_op(const gpi_conv_desc& d) {
    return d.k == 5 && d.stride == 1 && !d.upsample && d.gin_off >= 0 && d.cin <= 4 && d.cout <= 2;
}
__host__ __device__ inline int bwd_rowlen(const gpi_conv_desc& d) {
    return d.cout * d.cin * d.k * d.k + (d.in_bn ? 2 * d.cin : 0);
}
// LDS of such an op between the header and the gradient image: [fuse: target rows] | channel-sum scratch
// (256) + SLAB_ROWS weight-gradient partial rows
__host__ __device__ inline int vop_mid_floats(int gh, int w_out, int rowlen, bool fuse);
template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

template <int V>
struct IntC {
    static constexpr int value = V;
};

// GPI_IG_PRE: the MFMA input gradient's accumulated S_in operands of the second pixel round (tiles of > 256
// owned pixels) are loaded in phase 1 with the first round's, instead of at the round's start (a global
// round trip inside the compute phase)
#ifndef GPI_IG_PRE
#define GPI_IG_PRE 0
#endif
// GPI_S2_IG_SERIAL: the stride-2 input gradient's reduction one MFMA step at a time (table read -> gathered
// gradient read -> MFMA, the form before r05; A/B only).  Default: four steps' operands in flight per MFMA group
// GPI_IG_PAIR: the stride-1 / upsampling MFMA input gradient by pixel-block pairs (m, m + 4) sharing the
// offset-table and weight reads (A/B)
#ifndef GPI_IG_PAIR
#define GPI_IG_PAIR 0
#endif
#ifndef GPI_S2_IG_SERIAL
#define GPI_S2_IG_SERIAL 0
#endif
// GPI_VDG3: the input gradient of the 3x3 / stride-1 backwards on the VALU (v_pk_fma_f32 over input-channel
// pairs, the weights by broadcast LDS reads, as the fused output conv's) instead of the MFMA gather form
// (16 x 16 x 4 blocks, N = cin padded to 16, two dependent LDS reads per step).  Measured r05 (phase probe,
// tools/phase_probe.py): EncBlock1.dl1.bwd phase 6 18.3 k -> 13.8 k cycles, DecBlock3.dl1 23.1 k -> 20.2 k,
// launch time -1.0 / -1.3 us (kprof), but the step 0.5591-0.5608 vs 0.5538-0.5544 ms with it off
// (profiles/r05i_ab_vdg3.txt): off by default; cin 10 (LastTransUp.conv1) was slower still (weight reads)
#ifndef GPI_VDG3
#define GPI_VDG3 0
#endif
// occupancy target (waves per SIMD) of the 1x1 / 3x3 / 7x7 backward instantiations (no C64 backward launch
// holds more than 5 workgroups per CU; 4 / 5 / 6 measured alike, r04r)
#ifndef GPI_BWD_WAVES
#define GPI_BWD_WAVES 6
#endif
// ... of the 3x3 / stride-1 instantiation with the VALU input gradient (its per-thread channel sums and
// accumulators: 12 spilled VGPRs at 5 waves, none at 4; its launches hold <= 5 workgroups per CU)
#ifndef GPI_BWD3_WAVES
#define GPI_BWD3_WAVES 4
#endif
// per-wave input-channel sums [2][4 waves][32] (256 floats) alias the offset table (>= 256 floats)
constexpr int SLAB_ROWS = 4;    // partial-slab rows per workgroup: one per wave (no cross-wave dW reduction;
                                // vop ops: summed in LDS, one row per workgroup)
// [WB: input-gradient weights, <= 200 floats | WF (fuse): forward weights, later the channel-sum scratch (256) |
//  SLAB_ROWS weight-gradient partial rows]
__host__ __device__ inline int vop_mid_floats(int gh, int w_out, int rowlen, bool fuse) {
    return pad256(512 + SLAB_ROWS * rowlen);
}

// FUSE (the decoder's output conv, Gaussian-loss epilogue, no dropout): the launch computes its own
// forward first -- output rows [oy0 - K/2, oy0 + th + K/2) from an input image K/2 rows taller on each
// side, the log-likelihood of its owned rows and the loss gradient straight into the LDS gradient
// image -- then runs the backward on it: no output-gradient round trip through HBM, one launch less.
#ifndef GPI_FUSE_WAVES
#define GPI_FUSE_WAVES 5
#endif
// ... of its compile-time shape instantiation (geometry folded: 80 VGPRs fit 6 waves without spills, where the
// generic kernel spills 14-15)
#ifndef GPI_FUSE_SHP_WAVES
#define GPI_FUSE_SHP_WAVES 5
#endif
// fused output conv forward: which of the K weight-pair taps come by broadcast LDS read (one ds_read_b64 of
// the (co 0, co 1) pair) instead of two v_readlane (GPI_FUSE_WLDS = how many; the odd taps first).  The
// launch: 30.29 / 30.52 us with every pair by readlane, 29.63 / 29.55 with 4 of 5 by LDS, 29.40 / 29.44 with
// all 5 (r03 A/B): the forward phase was VALU-issue bound, the LDS pipe has room for the broadcast reads
#ifndef GPI_FUSE_WLDS
#define GPI_FUSE_WLDS 5
#endif
// the VALU input gradient (vop ops): weight channel pairs by broadcast LDS read (1) or v_readlane (0)
#ifndef GPI_VDG_WLDS
#define GPI_VDG_WLDS 1
#endif
__host__ __device__ constexpr bool fuse_wlds(int ky) {
    return GPI_FUSE_WLDS <= 0 ? false : (GPI_FUSE_WLDS >= 5 ? true : (ky & 1 ? (ky / 2) < GPI_FUSE_WLDS : (ky / 2) < GPI_FUSE_WLDS - 2));
}

template <int K, int S, int UP, bool FUSE = false, bool HALF = false, bool V3 = false, bool EXF = false, int SHP = -1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K == 5 ? (FUSE ? (SHP >= 0 ? GPI_FUSE_SHP_WAVES : GPI_FUSE_WAVES) : 4) : (V3 ? GPI_BWD3_WAVES : GPI_BWD_WAVES)))) void conv_bwd_kernel(gpi_conv_desc d, gpi_codec_ctx c, ConvGeom G) {
    fold_shape<SHP>(d, G);
    touch_kernargs<CONV_KARG_BYTES>();
    entry_signal(G);
    if (SKIP(G, 16)) return;
    // the tile's geometry: the launch's, or the half-height one of the tiles past nfull (GPI_HALF_TILES)
    ConvGeom Gt_;
    if constexpr (HALF) {
        const int lb0 = logical_block(G);
        const bool wgr0 = G.split && (G.xcd ? (lb0 & 1) != 0 : lb0 >= G.nblocks);
        const int tile0 = !G.split ? lb0 : (G.xcd ? lb0 >> 1 : (wgr0 ? lb0 - G.nblocks : lb0));
        // (HALF: the instantiation for launches with half tiles -- the per-tile geometry copy costs the
        // prologue ~130 instructions and 7 more argument-load waits, which the launches without half tiles,
        // e.g. the encoder's, do not pay)
        Gt_ = G;
        if (tile0 >= G.nfull) {
            const ConvGeom::Alt& a = G.ha;
            Gt_.th = a.th; Gt_.rh = a.rh; Gt_.gh = a.gh; Gt_.ph = a.ph; Gt_.zreg = a.zreg;
            Gt_.in_sq = a.in_sq; Gt_.in_sr = a.in_sr; Gt_.in_sc = a.in_sc;
            Gt_.g_sq = a.g_sq; Gt_.g_sr = a.g_sr; Gt_.g_sc = a.g_sc;
            Gt_.d_in4 = a.d_in4; Gt_.d_g4 = a.d_g4; Gt_.d_tp = a.d_tp;
        }
    }
    const ConvGeom& Gt = HALF ? Gt_ : G;
    constexpr int KK = K * K;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    double* gst = (double*)smem;                      // [cin][4] input stats, then [cout][4] output stats
    float* i_sc = smem + 8 * (d.cin + d.cout);
    float* i_sh = i_sc + d.cin;
    float* i_mean = i_sh + d.cin;
    float* i_inv = i_mean + d.cin;
    float* i_gam = i_inv + d.cin;
    float* o_coef = i_gam + d.cin;                    // [cout][4]: mean, inv, mS, mSx
    float* o_drop = o_coef + 4 * d.cout;              // [cout] Dropout2d scales of the output channels
    const bool has_gin = d.gin_off >= 0;
    const bool obn = d.gout_mode == 0;
    const int KD = d.cout * KK;                       // input-gradient reduction length
    const int KD4 = (KD + 3) & ~3;
    // vop: the VALU input gradient (5x5, stride 1, cin <= 4; always with FUSE) takes its weights from
    // SGPRs, so there is no wD / offset table; that LDS region (`mid`) holds instead [FUSE: the Gaussian
    // target rows of the tile, [gh][w_out], staged with the operand images] and, once those are dead,
    // the channel-sum scratch (256) and the four waves' weight-gradient partial rows, summed in LDS
    // into ONE slab row per tile (a quarter of the slab bytes, one coalesced store)
    const bool vop = FUSE || (K == 5 && S == 1 && !UP && has_gin && d.cin <= 4 && d.cout <= 2);
    // v3: the VALU input gradient of a 3x3 / stride-1 op (GPI_VDG3; tiles of >= 256 owned pixels, cin <= 12):
    // weights staged as WB3[((co K + ky) K + kx) CIV3 + ci], CIV3 = cin rounded up to 4, in wD's place
    // (V3: an instantiation of its own -- its accumulators and prefetched operands need a 4-wave VGPR budget,
    // which the MFMA form's launches of up to 5 workgroups per CU must not pay; picked by v3_op on the host)
    const bool v3 = V3 && K == 3 && S == 1 && !UP && !FUSE && has_gin && d.cin <= 8 && Gt.ph * d.w_in >= 256;
    const int CIV3 = (d.cin + 3) & ~3;
    const int J = d.cin * KK;
    const int rowlen = d.cout * J + (d.in_bn ? 2 * d.cin : 0);
    float* wD = smem + bwd_hdr(d.cin, d.cout);        // [KD4][16]: W[co][ci][tap] at (co*KK + tap)*16 + ci, zero padded
    const int nwd = (has_gin && !vop) ? KD4 * 16 : 0;
    float* const mid = wD;
    const int nmid = vop ? vop_mid_floats(Gt.gh, d.w_out, rowlen, FUSE) : 0;
    // S1 / UP: [KD4] output-gradient offset of reduction index k; S2: per parity class of the input
    // pixel [4][2][KD4]: (output-gradient offset, weight row) of the class's k-th valid tap
    int* ktab = (int*)(wD + pad256(nwd) + nmid);
    float* gl = (float*)ktab + ((has_gin && !vop) ? pad256((S == 2 ? 8 : 1) * KD4) : 0);   // [cout][gh][PG]
    const int gplane = Gt.gh * Gt.PG;
    const int gimg = img_floats(d.cout, Gt.gh, Gt.PG);
    const bool zreg = Gt.zreg != 0;
    float* gz = gl + gimg;                            // raw z of the output (BN-backward only, LDS form)
    float* al = gz + ((obn && !zreg) ? gimg : 0);     // [cin][rh][P]
    // FUSE: the image starts K/2 rows above the backward's first input row; alb is the backward's view
    float* const alb = FUSE ? al + (K / 2) * Gt.P : al;
    // reduction scratch: aliases gz (dead after phase 3) when it is large enough -- 8 KB less LDS
    // per workgroup, one more resident workgroup per CU on the 32x32 planes
    // channel-sum scratch: the offset table's space, dead after the input gradient (in_bn implies has_gin);
    // FUSE: the target image's (>= 256 floats, dead after the loss phase)
    float* red = vop ? mid + 256 : (float*)ktab;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, kq = lane >> 4, l16 = lane & 15;
    RTSTAMP(0);
    PHASE(0);
    float* const ws = pin(c.ws);
    const float* const params = pin(c.params);
    const float* const zero = pin(Gt.zero);
    const int64_t w_off = pin(d.w_off), gout_off = pin(d.gout_off), out_off = pin(d.out_off);
    const int64_t gin_off = pin(d.gin_off);
    // split launches: workgroups [0, nblocks) compute the input gradient (+ BN-backward sums, dgamma /
    // dbeta), [nblocks, 2 nblocks) the weight gradient of the same tiles
    // (xcd order: logical blocks 2t / 2t + 1 are tile t's two roles, on one XCD)
    const int lb = logical_block(G);
    const bool wg_role = Gt.split && (Gt.xcd ? (lb & 1) != 0 : lb >= Gt.nblocks);
    const bool dg_role = !wg_role;
    // wpart_off < 0: input gradient only (no weight / gamma / beta gradient, no slab row): callers that
    // discard the shared-weight gradients (the PredictionEnsemble's decoder passes)
    const bool wout = d.wpart_off >= 0;
    const bool do_wgrad = (!Gt.split || wg_role) && wout;
    const int tile = !Gt.split ? lb : (Gt.xcd ? lb >> 1 : (wg_role ? lb - Gt.nblocks : lb));
    const TileIdx T = tile_of(Gt, c.groups, tile);
    const int HWi = d.h_in * d.w_in, HWo = d.h_out * d.w_out;
    const float* ib = input_base(d, c, T.b);
    PHASE(1);

    // ---- phase 1: every global read in flight together
    // (LDS stores first: an LDS store behind an outstanding LDS-DMA waits for that DMA)
    if constexpr (FUSE) {
        // the gradient image is computed in phase 3': zero halo columns, out-of-plane rows and margin
        float4* g4 = reinterpret_cast<float4*>(gl);
        for (int e = tid; e < gimg / 4; e += 256) g4[e] = float4{0.f, 0.f, 0.f, 0.f};
    }
    const int CIV = d.cin <= 2 ? 2 : 4;      // vop: input channels per weight vector (zero padded)
    if (vop) {
        // weights W[co][ci][ky][kx] transposed for the packed (v_pk_fma_f32) loops: input gradient
        // WB[((co K + ky) K + kx) CIV + ci]; FUSE forward WF[((ci K + kx) K + ky) 2 + co]
        stage(mid, d.cout * KK * CIV, zero, [&](int e) -> const float* {
            const int ci = e % CIV, t = e / CIV, co = t / KK, tap = t - co * KK;
            return ci < d.cin ? params + w_off + ((int64_t)co * d.cin + ci) * KK + tap : nullptr;
        });
        if (FUSE)
            stage(mid + 256, d.cin * KK * 2, zero, [&](int e) -> const float* {
                const int co = e & 1, t = e >> 1, ci = t / KK, r = t - ci * KK, kx = r / K, ky = r - kx * K;
                return params + w_off + ((int64_t)co * d.cin + ci) * KK + ky * K + kx;
            });
    }
    if (has_gin && dg_role && v3)
        stage(wD, d.cout * KK * CIV3, zero, [&](int e) -> const float* {
            const int t = e / CIV3, ci = e - t * CIV3, co = t / KK, tap = t - co * KK;
            return ci < d.cin ? params + w_off + ((int64_t)co * d.cin + ci) * KK + tap : nullptr;
        });
    else if (has_gin && dg_role && !vop)
        stage(wD, nwd, zero, [&](int e) -> const float* {
            const int ci = e & 15, k = e >> 4;
            const int co = k / KK, t = k - co * KK;
            return ci < d.cin && k < KD ? params + w_off + ((int64_t)co * d.cin + ci) * KK + t : nullptr;
        });
    PHASE(12);
    int gy0, gh_;
    g_rows(K, S, d.pad, T.oy0, Gt.th, gy0, gh_);
    const int64_t gbase = ((int64_t)T.b * d.out_ctot + d.out_c0) * HWo;
    // FUSE: the Gaussian target of this thread's first forward item (column x, RPF rows), loaded with the
    // operand images into registers (one global round trip less inside the loss phase)
    constexpr int RPF = 5;                    // FUSE: vertically adjacent output pixels per forward item
    float tv0[FUSE ? RPF : 1];
    const float* tg = zero;
    if constexpr (FUSE) {
        int trow0 = T.b - karg_sel(c.groups.start, T.grp);
        if (const int32_t* ti = karg_sel(c.tgt_idx, T.grp)) trow0 = ti[trow0];
        tg = karg_sel(c.tgt, T.grp) + (int64_t)trow0 * HWo;
        const int nitem = ((Gt.gh + RPF - 1) / RPF) * d.w_out;
        const int rg = dq(tid, Gt.d_wout), x = tid - rg * d.w_out;
#pragma unroll
        for (int p = 0; p < RPF; ++p) {
            const int oy = gy0 + rg * RPF + p;
            const bool ok = tid < nitem && rg * RPF + p < Gt.gh && oy >= 0 && oy < d.h_out;
            tv0[p] = *as_gld(ok ? tg + oy * d.w_out + x : zero);
        }
    } else {
        stage_img(gl, d.cout, Gt.gh, Gt.PG, Gt.d_g4, Gt.d_PG4, Gt.g_sq, Gt.g_sr, Gt.g_sc, gy0, d.h_out, d.w_out, zero,
                  [&](int q) -> const float* { return ws + gout_off + gbase + (int64_t)q * HWo; });
    }
    PHASE(13);
    f32x4 zr[ZREG];           // zreg: this thread's chunks tid + 256 u of the z image
    if (obn && zreg) {
        const int P4 = Gt.PG >> 2, plane4 = Gt.gh * P4, total = d.cout * plane4;
        const int c4lo = HALO / 4, c4hi = HALO / 4 + d.w_out / 4;
        ChunkIter it;
        it.init(tid, plane4, P4, Gt.d_g4, Gt.d_PG4);
#pragma unroll
        for (int u = 0; u < ZREG; ++u) {
            const int row = gy0 + it.r;
            const bool ok = tid + 256 * u < total && row >= 0 && row < d.h_out && it.c4 >= c4lo && it.c4 < c4hi;
            const float* src = ok ? ws + out_off + gbase + (int64_t)it.q * HWo + row * d.w_out + 4 * (it.c4 - c4lo)
                                  : zero;
            zr[u] = *as_gld((const f32x4*)src);
            it.step(Gt.g_sq, Gt.g_sr, Gt.g_sc, P4, Gt.gh);
        }
    } else if (obn) {
        stage_img(gz, d.cout, Gt.gh, Gt.PG, Gt.d_g4, Gt.d_PG4, Gt.g_sq, Gt.g_sr, Gt.g_sc, gy0, d.h_out, d.w_out, zero,
                  [&](int q) -> const float* { return ws + out_off + gbase + (int64_t)q * HWo; });
    }
    PHASE(14);
    int iy0, rh_;
    in_rows(K, S, UP, d.pad, T.oy0, Gt.th, iy0, rh_);
    const int iyA = FUSE ? iy0 - K / 2 : iy0;        // first row of the LDS input image
    stage_img(al, d.cin, Gt.rh, Gt.P, Gt.d_in4, Gt.d_P4, Gt.in_sq, Gt.in_sr, Gt.in_sc, iyA, d.h_in, d.w_in, zero,
              [&](int q) -> const float* { return ib + (int64_t)q * HWi; });
    PHASE(8);
    // input-gradient epilogue operand (previous S_in, when accumulating) of this wave's first
    // four pixel blocks: lane (kq, l16) owns channel l16 at the 4 consecutive pixels
    // 16 m + 4 kq + [0, 4).  The input itself is read back from the LDS image.
    int py0, ph_;
    owned_rows(S, UP, T.oy0, Gt.th, py0, ph_);
    // cin <= 4 at stride 1: the input gradient runs on the VALU (phase 4b'), the MFMA form would
    // leave >= 3/4 of its N = 16 columns empty
    // (FUSE: always the VALU input gradient -- launch() checks cin <= 4 -- so the MFMA input-gradient
    // path and its operand registers compile away)
    const bool vdg = vop && dg_role;     // (launch() never splits a vop op: dg_role holds)
    const int nmblk = (!FUSE && has_gin && dg_role && !vdg && !v3 && !SKIP(G, 2)) ? (Gt.ph * d.w_in) >> 4 : 0;
    const int ci_l = min(l16, d.cin - 1);
    const bool cok = l16 < d.cin;
    const int64_t ibase = ((int64_t)T.b * d.in_ctot + d.in_c0 + ci_l) * HWi + (int64_t)py0 * d.w_in;
    f32x4 pv4[4];
#if GPI_IG_PRE
    f32x4 pv4b[4];            // round 1's operands, loaded with round 0's in phase 1 (GPI_IG_PRE)
#endif
    auto own_load = [&](int round, f32x4 (&dst)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int m = wv + 4 * (4 * round + u);
            const bool ok = m < nmblk && cok;
            const int64_t o = ibase + 16 * m + 4 * kq;
            if (d.gin_accumulate) dst[u] = *as_gld((const f32x4*)(ok ? ws + gin_off + o : zero));
            else dst[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // v3: the previous S_in of this thread's first item (Q = 2 pixels of channels < cin), with the operand loads
    float pv3[8][2];
    if (v3 && dg_role && d.gin_accumulate && !SKIP(G, 2)) {
        const int Q = Gt.ph * d.w_in >= 512 ? 2 : 1;
        const int gq = tid;
        const int qy = dq(Q * gq, Gt.d_win), px0 = Q * gq - qy * d.w_in;
        const bool iok = gq < (Gt.ph * d.w_in) / Q;
        const int64_t gb_in = ((int64_t)T.b * d.in_ctot + d.in_c0) * HWi + (int64_t)(py0 + qy) * d.w_in + px0;
#pragma unroll
        for (int ci = 0; ci < 8; ++ci) {
            const bool ok = iok && ci < d.cin;
            const float* pp = ok ? ws + gin_off + gb_in + (int64_t)ci * HWi : zero;
            pv3[ci][0] = *as_gld(pp);
            pv3[ci][1] = *as_gld(ok && Q == 2 ? pp + 1 : zero);
        }
    }
    if (nmblk > 0 && S != 2) {
        own_load(0, pv4);
#if GPI_IG_PRE
        if (nmblk > 16) own_load(1, pv4b);
#endif
    }
    PHASE(9);
    float gam = 0.f, bet = 0.f;
    if (d.in_bn && tid < d.cin) {
        gam = *as_gld(params + d.gamma_off + tid);
        bet = *as_gld(params + d.beta_off + tid);
    }
    const bool drop = d.drop_off >= 0;
    // the dropout scale goes to LDS after the stat loads (an LDS store of it here would drain every
    // outstanding DMA before the stat loads are even issued)
    float odv = 1.f;
    if (drop && tid >= 128 && tid < 128 + d.cout) odv = *as_gld(ws + d.drop_off + (int64_t)T.b * d.cout + (tid - 128));
    {
        StatLoad L;
        stat_issue(c.stats, c.n_stats, T.grp, d.in_stat, d.in_bn ? d.cin : 0, gst, d.out_stat, obn ? d.cout : 0,
                   gst + 4 * d.cin, zero, L);
        PHASE(10);
        stat_finish(L);
        PHASE(11);
    }
    if (tid >= 128 && tid < 128 + d.cout) o_drop[tid - 128] = odv;
    __syncthreads();
    if (SKIP(G, 8)) return;
    PHASE(2);

    // ---- phase 2: coefficients
    if (tid < d.cin && d.in_bn) {
        float mean, inv;
        mean_invstd(gst + 4 * tid, (double)T.gsz * HWi, c.bn_eps, mean, inv);
        i_mean[tid] = mean;
        i_inv[tid] = inv;
        i_gam[tid] = gam;
        i_sc[tid] = gam * inv;
        i_sh[tid] = fmaf(-(mean * gam), inv, bet);
    }
    if (obn && tid >= 64 && tid < 64 + d.cout) {
        const int co = tid - 64;
        const double* st = gst + 4 * (d.cin + co);
        const double n = (double)T.gsz * HWo;
        float mean, inv;
        mean_invstd(st, n, c.bn_eps, mean, inv);
        o_coef[4 * co] = mean;
        o_coef[4 * co + 1] = inv;
        o_coef[4 * co + 2] = (float)(st[2] / n);
        o_coef[4 * co + 3] = (float)(st[3] / n);
    }
    __syncthreads();
    PHASE(3);

    // ---- phase 3: activations in LDS; offset table of the input-gradient reduction
    if (d.in_bn) activate_img(al, Gt, d, iyA, i_sc, i_sh);
    if (has_gin && dg_role && S == 2) {
        // input pixel (py, px) = (py0 + 2a + ry, 2b + rx) receives output (oy, ox) through tap (ky, kx)
        // iff 2 oy = py + pad - ky, 2 ox = px + pad - kx: the valid taps depend on the parity class
        // (ry, rx) only.  Class table entry k: A = gl offset (co, dy = (ry + pad - ky) / 2,
        // dx = (rx + pad - kx) / 2) relative to (a, b); B = weight row co * KK + ky * K + kx.
        for (int e = tid; e < 4 * KD4; e += 256) {
            const int cls = e / KD4, k = e - cls * KD4;
            const int ry = cls >> 1, rx = cls & 1;
            const int ky0 = (ry + d.pad) & 1, kx0 = (rx + d.pad) & 1;
            const int nky = (K - ky0 + 1) >> 1, nkx = (K - kx0 + 1) >> 1;
            int oa = 0, ob = 0;
            if (k < d.cout * nky * nkx) {
                const int co = k / (nky * nkx), r = k - co * nky * nkx, jy = r / nkx, jx = r - jy * nkx;
                const int ky = ky0 + 2 * jy, kx = kx0 + 2 * jx;
                oa = co * gplane + ((ry + d.pad - ky) >> 1) * Gt.PG + ((rx + d.pad - kx) >> 1);
                ob = co * KK + ky * K + kx;
            }
            // (interleaved (A, 16 B) pairs: one ds_read_b64 per reduction step)
            ktab[cls * 2 * KD4 + 2 * k] = oa;
            ktab[cls * 2 * KD4 + 2 * k + 1] = 16 * ob;
        }
    }
    if (has_gin && dg_role && S != 2 && !vop && !v3) {
        // A operand of reduction index k = (co, ky, kx) for owned pixel (qy, px):
        // gl[(S1) qy*PG + px | (UP) 2 qy*PG + 2 px] + ktab[k]
        const int ry0 = (UP ? 2 * py0 : py0) + d.pad - gy0;
        for (int k = tid; k < KD4; k += 256) {
            int o = 0;
            if (k < KD) {
                const int co = k / KK, tap = k - co * KK, ky = tap / K, kx = tap - ky * K;
                o = co * gplane + (ry0 - ky) * Gt.PG + d.pad - kx + HALO;
            }
            ktab[k] = o;
        }
    }
    if (obn && zreg) {
        // BN-backward of the output gradient with z from registers: chunk tid + 256 u
        const int P4 = Gt.PG >> 2, plane4 = Gt.gh * P4, total = d.cout * plane4;
        const int c4lo = HALO / 4, c4hi = HALO / 4 + d.w_out / 4;
        float4* g4 = reinterpret_cast<float4*>(gl);
        ChunkIter it;
        it.init(tid, plane4, P4, Gt.d_g4, Gt.d_PG4);
#pragma unroll
        for (int u = 0; u < ZREG; ++u) {
            const int e = tid + 256 * u;
            const int row = gy0 + it.r;
            if (e < total && row >= 0 && row < d.h_out && it.c4 >= c4lo && it.c4 < c4hi) {
                const float* oc = o_coef + 4 * it.q;
                const float m = oc[0], inv = oc[1], mS = oc[2], mSx = oc[3];
                const float ds = o_drop[it.q];
                const float4 sv = g4[e];
                const f32x4 zv = zr[u];
                float4 o;
                o.x = ds * ((sv.x - mS - ((zv[0] - m) * inv) * mSx) * inv);
                o.y = ds * ((sv.y - mS - ((zv[1] - m) * inv) * mSx) * inv);
                o.z = ds * ((sv.z - mS - ((zv[2] - m) * inv) * mSx) * inv);
                o.w = ds * ((sv.w - mS - ((zv[3] - m) * inv) * mSx) * inv);
                g4[e] = o;
            }
            it.step(Gt.g_sq, Gt.g_sr, Gt.g_sc, P4, Gt.gh);
        }
    } else if (obn) {
        const int P4 = Gt.PG >> 2, plane4 = Gt.gh * P4, total = d.cout * plane4;
        const int c4lo = HALO / 4, c4hi = HALO / 4 + d.w_out / 4;
        float4* g4 = reinterpret_cast<float4*>(gl);
        const float4* z4 = reinterpret_cast<const float4*>(gz);
        ChunkIter it;
        it.init(tid, plane4, P4, Gt.d_g4, Gt.d_PG4);
        for (int e0 = tid; e0 < total; e0 += 512) {
            float4 sv[2], zv[2];
            bool ok[2];
            int co[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int row = gy0 + it.r;
                ok[u] = e0 + 256 * u < total && row >= 0 && row < d.h_out && it.c4 >= c4lo && it.c4 < c4hi;
                co[u] = it.q;
                if (ok[u]) {
                    sv[u] = g4[e0 + 256 * u];
                    zv[u] = z4[e0 + 256 * u];
                }
                it.step(Gt.g_sq, Gt.g_sr, Gt.g_sc, P4, Gt.gh);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (ok[u]) {
                    const float* oc = o_coef + 4 * co[u];
                    const float m = oc[0], inv = oc[1], mS = oc[2], mSx = oc[3];
                    const float ds = o_drop[co[u]];     // d(dropped output)/d(conv output)
                    float4 o;
                    o.x = ds * ((sv[u].x - mS - ((zv[u].x - m) * inv) * mSx) * inv);
                    o.y = ds * ((sv[u].y - mS - ((zv[u].y - m) * inv) * mSx) * inv);
                    o.z = ds * ((sv[u].z - mS - ((zv[u].z - m) * inv) * mSx) * inv);
                    o.w = ds * ((sv[u].w - mS - ((zv[u].w - m) * inv) * mSx) * inv);
                    g4[e0 + 256 * u] = o;
                }
            }
        }
    }
    if (!obn && drop) {
        // direct output gradient: scale by the dropout mask (halo / margin zeros stay zero)
        const int plane4 = Gt.gh * (Gt.PG >> 2), total = d.cout * plane4;
        float4* g4 = reinterpret_cast<float4*>(gl);
        for (int e = tid; e < total; e += 256) {
            const float ds = o_drop[dq(e, Gt.d_g4)];
            float4 v = g4[e];
            v.x *= ds;
            v.y *= ds;
            v.z *= ds;
            v.w *= ds;
            g4[e] = v;
        }
    }
    __syncthreads();
    if constexpr (FUSE) {
        // ---- phase 3': forward of output rows gy0 + [0, gh), the Gaussian log-likelihood of the owned
        // rows, d(-logL)/d(mu, logsigma) into the gradient image.  (mu, logsigma) of a pixel is one packed
        // pair: every tap is ONE v_pk_fma_f32 with the (co 0, co 1) weight pair of the tap, read from
        // LDS (WF, uniform address: a broadcast read) -- no scalar loads in the loop, whose lgkmcnt
        // waits used to drain the LDS reads as well (r03: 22.5 k cycles per workgroup for this phase)
        constexpr int PADK = K / 2;
        float Lv = 0.f;
        // the exp-field loss is an instantiation of its own (EXF; launch() picks it from d.epilogue): as a
        // runtime flag its two extra exps per pixel ran as selects in the log-field form as well
        constexpr bool ex = EXF;
        const float scl = karg_sel(c.loss_scale, T.grp);
        // RPF vertically adjacent pixels of one column per thread: items (column, row group) fill the
        // 256 lanes exactly on 64-wide planes (20 rows = 4 groups x 64 columns with 16-row tiles).  Per
        // (ci, kx) the column's RPF + K - 1 input values are read once (lanes on consecutive columns: one
        // 256-B LDS row per read, no bank conflicts) and serve the RPF x K taps.  The weights: a tap's
        // (co 0, co 1) pair by one broadcast ds_read_b64 (fuse_wlds, the default for every tap) or, for
        // taps left to the VALU, by two v_readlane from wr[] (lane l holds WF[64 j + l])
        const int nrg = (Gt.gh + RPF - 1) / RPF, nitem = nrg * d.w_out;
        auto fwd_items = [&](auto ci_c) {
            constexpr int CIN = decltype(ci_c)::value;
            constexpr int NWR = (CIN * KK * 2 + 63) / 64;
            float wr[NWR];
#pragma unroll
            for (int j = 0; j < NWR; ++j) wr[j] = mid[256 + 64 * j + lane];
            for (int it = tid; it < nitem; it += 256) {
                const int rg = dq(it, Gt.d_wout), x = it - rg * d.w_out;
                const int j0 = rg * RPF;
                float tv[RPF];
#pragma unroll
                for (int p = 0; p < RPF; ++p) {
                    const int oy = gy0 + j0 + p;
                    const bool ok = j0 + p < Gt.gh && oy >= 0 && oy < d.h_out;
                    tv[p] = it == tid ? tv0[p] : (ok ? as_gld(tg)[oy * d.w_out + x] : 0.f);
                }
                f32x2 acc[RPF];
#pragma unroll
                for (int p = 0; p < RPF; ++p) acc[p] = f32x2{0.f, 0.f};
#pragma unroll
                for (int ci = 0; ci < CIN; ++ci) {
                    if (ci >= d.cin) break;
                    const float* acol = al + ci * Gt.rh * Gt.P + HALO + x - PADK;
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        float v[RPF + K - 1];
#pragma unroll
                        for (int r = 0; r < RPF + K - 1; ++r) v[r] = acol[min(j0 + r, Gt.rh - 1) * Gt.P + kx];
                        f32x2 w[K];
#pragma unroll
                        for (int ky = 0; ky < K; ++ky) {
                            const int i = ((ci * K + kx) * K + ky) * 2;
                            if (fuse_wlds(ky)) {
                                // (co 0, co 1) pair by one broadcast LDS read: the LDS pipe takes part of
                                // the weight traffic off the VALU (GPI_FUSE_WLDS taps of K)
                                w[ky] = *reinterpret_cast<const f32x2*>(mid + 256 + i);
                            } else {
                                w[ky][0] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wr[i >> 6]), i & 63));
                                w[ky][1] = __int_as_float(
                                    __builtin_amdgcn_readlane(__float_as_int(wr[(i + 1) >> 6]), (i + 1) & 63));
                            }
                        }
                        // input row j0 + r feeds pixel p through tap ky = r - p
#pragma unroll
                        for (int r = 0; r < RPF + K - 1; ++r) {
#pragma unroll
                            for (int p = 0; p < RPF; ++p) {
                                const int ky = r - p;
                                if (ky < 0 || ky >= K) continue;
                                acc[p] = __builtin_elementwise_fma(w[ky], f32x2{v[r], v[r]}, acc[p]);
                            }
                        }
                    }
                }
#pragma unroll
                for (int p = 0; p < RPF; ++p) {
                    const int j = j0 + p, oy = gy0 + j;
                    if (j >= Gt.gh || oy < 0 || oy >= d.h_out) continue;
                    const bool own = j >= PADK && j < PADK + Gt.th;
                    const float mu = acc[p][0], ls = acc[p][1];
                    const float e = expf(-2.f * ls);
                    const float emu = ex ? expf(mu) : 1.f;
                    const float r = ex ? expf(tv[p]) - emu : tv[p] - mu;
                    if (own) Lv += -0.5f * (2.f * ls + r * r * e + GPI_LOG2PI);
                    float* g0 = gl + j * Gt.PG + HALO + x;
                    g0[0] = -scl * r * e * emu;
                    g0[gplane] = scl * (1.f - r * r * e);
                }
            }
        };
        if (d.cin <= 2) fwd_items(IntC<2>{});
        else fwd_items(IntC<4>{});
        // one fp64 atomic per workgroup (per-wave atomics into 16 replicas serialise: 2304 x 4 adds)
        const float lw = wave_sum(Lv);
        if (lane == 0) o_coef[wv] = lw;       // o_coef is unused without an output BN
        __syncthreads();
        if (tid == 0 && !SKIP(G, 4))
            atomicAdd(c.loss_acc + T.grp * GPI_REPLICAS + blockIdx.x % GPI_REPLICAS,
                      (double)((o_coef[0] + o_coef[1]) + (o_coef[2] + o_coef[3])));
    }
    PHASE(4);

    // ---- phase 4a: weight gradient (MFMA, column-shift form) -> slab row.
    // Stride 1 / upsampling: no masks in the loop -- the zero halos and tail margins of the
    // images make every out-of-range read a zero or a finite value multiplied by a zero,
    // and rows i >= M / columns j >= N of the tile (clamped operands) are never stored.
    // this wave's partial-slab row: [dW partial over the wave's output rows | dgamma | dbeta partials]
    // (vop: in LDS, summed below into the tile's one slab row)
    float* slab = vop ? mid + 512 + wv * rowlen : c.wpart + d.wpart_off + ((int64_t)tile * SLAB_ROWS + wv) * rowlen;
    const bool lsum = !vop && Gt.lsum;   // (lsum_op: never with vwg; at most 2 x 2 accumulator blocks)
    f32x4 hold[2][2];                   // lsum: this wave's weight-gradient blocks [mb][column block]
    // single-channel 7x7 / stride-2 input conv: weight gradient with the reduction over the tile's
    // output pixels (M = cout, N = the 49 taps in 4 column blocks, K = pixels), no zero-interleaved
    // stride-2 columns (the column-shift form below would compute ~6x the useful products here)
    // (vop: before the input gradient, its partial rows go to LDS; otherwise after it: the MFMA
    // accumulators are then the last live values and, for lsum, go straight to the LDS row sum)
    auto wgrad_phase = [&]() {
        const bool vwg = K == 7 && S == 2 && !UP && d.cin == 1 && !has_gin && d.cout <= 16 && do_wgrad;
        if constexpr (K == 7 && S == 2 && !UP) {
            if (vwg && !SKIP(G, 1)) {
                constexpr int PADC = K / 2, NB = (KK + 15) / 16;
                float* const wrow = Gt.vsum ? gl + wv * rowlen : slab;
                if (G.vshift) {
                    // column-shift form: taps kx = kx0 + 2 s of a stride-2 row are the taps kx0 of the output
                    // pixel s columns further, so dW[co][ky][kx0 + 2 s] = sum_{ty, x} g[co][ty][x - s] *
                    // in[2 ty + ky][2 x + kx0 - 3] over the tile's rows and x in [0, w_out + 4) (the zero halo
                    // columns of the gradient image supply the out-of-range g).  M = (s, co): 4 cout <= 32 rows
                    // in 2 blocks, N = (ky, kx0): 14 of 16 columns, K = pixels -- 2 MFMAs per 4 pixels against
                    // 4 (M = cout, N = 49 taps in 4 blocks), 57 % of the MFMA products useful against 29 %
                    // for the 6-channel C64 input conv.  Each wave takes whole rows (ty = wv, wv + 4, ...).
                    const int mc = 4 * d.cout;
                    const float* ga[2];
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb) {
                        const int m = 16 * mb + l16;
                        const int s = m < mc ? m / d.cout : 0, co = m < mc ? m - s * d.cout : 0;
                        ga[mb] = gl + co * gplane + (T.oy0 - gy0) * Gt.PG + HALO - s;
                    }
                    const int n = min(l16, 13), ky_b = n >> 1, kx0_b = n & 1;
                    const float* const xb0 = alb + ky_b * Gt.P + HALO + kx0_b - PADC;
                    const int wx4 = (d.w_out >> 2) + 1;
                    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
                    for (int ty = wv; ty < Gt.th; ty += 4) {
                        const float* const g0 = ga[0] + ty * Gt.PG;
                        const float* const g1 = ga[1] + ty * Gt.PG;
                        const float* const xr = xb0 + (2 * ty) * Gt.P;
                        for (int c4 = 0; c4 < wx4; ++c4) {
                            const int x = 4 * c4 + kq;
                            const float a0 = g0[x], a1 = g1[x], b = xr[2 * x];
                            acc[0] = mfma4(a0, b, acc[0]);
                            acc[1] = mfma4(a1, b, acc[1]);
                        }
                    }
                    if (Gt.vsum) __syncthreads();        // every wave is done reading gl
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int m = 16 * mb + 4 * kq + r;
                            const int s = m / d.cout, co = m - s * d.cout, kx = kx0_b + 2 * s;
                            if (m < mc && l16 < 14 && kx < K) wrow[co * J + ky_b * K + kx] = acc[mb][r];
                        }
                    }
                } else {
                const int tp = Gt.th * d.w_out;
                const int co_a = min(l16, d.cout - 1);                  // A row (rows >= cout never stored)
                int tap_off[NB];                                        // B column: tap (ky, kx) of this lane
    #pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    const int j = min(16 * nb + l16, KK - 1), ky = j / K, kx = j - ky * K;
                    tap_off[nb] = ky * Gt.P + kx - PADC;
                }
                f32x4 acc[NB];
    #pragma unroll
                for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
                const float* gco = gl + co_a * gplane + (T.oy0 - gy0) * Gt.PG + HALO;
                for (int ps = wv; 4 * ps < tp; ps += 4) {               // 4 output pixels per step, wave-strided
                    const int px = 4 * ps + kq;
                    const int ty = dq(px, Gt.d_wout), ox = px - ty * d.w_out;
                    const float a = gco[ty * Gt.PG + ox];
                    const float* xb = alb + (ty * S) * Gt.P + HALO + S * ox;
                    float bv[NB];
    #pragma unroll
                    for (int nb = 0; nb < NB; ++nb) bv[nb] = xb[tap_off[nb]];
    #pragma unroll
                    for (int nb = 0; nb < NB; ++nb) acc[nb] = mfma4(a, bv[nb], acc[nb]);
                }
                // Gt.vsum: the four waves' tiles summed in LDS (the gradient image, dead after the loop)
                // into ONE slab row per tile -- a quarter of the slab bytes the reduction reads, on the
                // step's critical path at its end; otherwise each wave stores its own row
                if (Gt.vsum) __syncthreads();        // every wave is done reading gl
    #pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co2 = kq * 4 + r, j2 = 16 * nb + l16;
                        if (co2 < d.cout && j2 < KK) wrow[co2 * J + j2] = acc[nb][r];
                    }
                }
                }
                if (Gt.vsum) {
                    __syncthreads();
                    float* srow = c.wpart + d.wpart_off + (int64_t)tile * rowlen;
                    for (int e = tid; e < d.cout * J; e += 256) {
                        const float* r = gl + e;
                        srow[e] = (r[0] + r[rowlen]) + (r[2 * rowlen] + r[3 * rowlen]);
                    }
                }
            }
        }
        {
            // ucls (3x3 upsampling, pad 1): the output rows of one parity py read input rows i + py - 1 and
            // i + py only (i = oy / 2), so the columns are (ci, row offset r) -- 2 cin instead of 3 cin, one column
            // block instead of two for 6 channels -- and the wave's partial sum for (ci, r) is the partial of
            // every tap ky that reads that row (py 0: r 0 -> ky 0, r 1 -> ky 1, 2; py 1: r 0 -> ky 0, 1, r 1 ->
            // ky 2).  A wave's rows ty = wv + 4 k all have the parity of T.oy0 + wv.  (UP == 2: launch() picks
            // that instantiation for ConvGeom::ucls)
            const bool ucls = UP == 2 && K == 3 && !lsum;
            const int MI = d.cout * K, NJ = ucls ? 2 * d.cin : d.cin * K;
            const int nmb = (SKIP(G, 1) || vwg || !do_wgrad) ? 0 : (MI + 15) >> 4, nnb = (NJ + 15) >> 4;
            const int XW = UP ? d.w_out + K - 1 : S * (d.w_out - 1) + K;   // virtual input columns
            const int nxs = (XW + 3) >> 2;
            for (int mb = 0; mb < nmb; ++mb) {
                const int i = 16 * mb + l16;
                const int co = min(i / K, d.cout - 1), kx = i - (i / K) * K;
                for (int nb0 = 0; nb0 < nnb; nb0 += 2) {
                    const bool two = nb0 + 1 < nnb;
                    int ci[2], ky[2];
    #pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int j = 16 * (nb0 + u) + l16;
                        ci[u] = min(ucls ? j >> 1 : j / K, d.cin - 1);
                        ky[u] = ucls ? j & 1 : j - (j / K) * K;      // ucls: the row offset r
                    }
                    // the second column block is a compile-time branch around the whole row loop, so the
                    // accumulators stay in the MFMA registers (a runtime branch inside the loop made the
                    // compiler copy them in and out of AGPRs around every MFMA)
                    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                    auto rows = [&](auto two_c) {
                        constexpr bool TWO = decltype(two_c)::value;
                        for (int ty = wv; ty < Gt.th; ty += 4) {
                            const float* grow = gl + (co * Gt.gh + (T.oy0 + ty - gy0)) * Gt.PG + HALO - kx;
                            const float* brow[2];
    #pragma unroll
                            for (int u = 0; u < 2; ++u) {
                                const int oy = T.oy0 + ty;
                                const int ry = !UP ? ty * S + ky[u]
                                                   : (ucls ? (oy >> 1) + (oy & 1) - 1 + ky[u] : fdiv2(oy - d.pad + ky[u])) - iy0;
                                brow[u] = alb + (ci[u] * Gt.rh + ry) * Gt.P + HALO;
                            }
                            // operands of four steps are read before their MFMAs (LDS read -> dependent
                            // MFMA would serialise every step)
                            if constexpr (UP != 0) {
                                // nearest x2 upsampling: virtual columns 2p + pad and 2p + pad + 1 both read
                                // input column p, so their gradient columns are summed first and the
                                // reduction runs over the (half as many) input columns p
                                const int plo = fdiv2(-d.pad), nps = (fdiv2(XW - 1 - d.pad) - plo + 4) >> 2;
                                int ps = 0;
                                for (; ps + 4 <= nps; ps += 4) {
                                    float a[4], b0[4], b1[4];
    #pragma unroll
                                    for (int u = 0; u < 4; ++u) {
                                        const int pc = plo + 4 * (ps + u) + kq;
                                        const int xv = 2 * pc + d.pad;
                                        a[u] = grow[xv] + grow[xv + 1];
                                        b0[u] = brow[0][pc];
                                        if (TWO) b1[u] = brow[1][pc];
                                    }
    #pragma unroll
                                    for (int u = 0; u < 4; ++u) {
                                        acc0 = mfma4(a[u], b0[u], acc0);
                                        if (TWO) acc1 = mfma4(a[u], b1[u], acc1);
                                    }
                                }
                                for (; ps < nps; ++ps) {
                                    const int pc = plo + 4 * ps + kq;
                                    const int xv = 2 * pc + d.pad;
                                    const float a = grow[xv] + grow[xv + 1];
                                    acc0 = mfma4(a, brow[0][pc], acc0);
                                    if (TWO) acc1 = mfma4(a, brow[1][pc], acc1);
                                }
                            } else {
                                auto a_at = [&](int xv) -> float {
                                    if (S == 2) {
                                        const int t2 = xv - kx;
                                        return (t2 & 1) ? 0.f : grow[kx + (t2 >> 1)];
                                    }
                                    return grow[xv];
                                };
                                int xs = 0;
                                for (; xs + 4 <= nxs; xs += 4) {
                                    float a[4], b0[4], b1[4];
    #pragma unroll
                                    for (int u = 0; u < 4; ++u) {
                                        const int xv = 4 * (xs + u) + kq;
                                        a[u] = a_at(xv);
                                        b0[u] = brow[0][xv - d.pad];
                                        if (TWO) b1[u] = brow[1][xv - d.pad];
                                    }
    #pragma unroll
                                    for (int u = 0; u < 4; ++u) {
                                        acc0 = mfma4(a[u], b0[u], acc0);
                                        if (TWO) acc1 = mfma4(a[u], b1[u], acc1);
                                    }
                                }
                                for (; xs < nxs; ++xs) {
                                    const int xv = 4 * xs + kq;
                                    const float a = a_at(xv);
                                    acc0 = mfma4(a, brow[0][xv - d.pad], acc0);
                                    if (TWO) acc1 = mfma4(a, brow[1][xv - d.pad], acc1);
                                }
                            }
                        }
                    };
                    if (two) rows(BoolC<true>{});
                    else rows(BoolC<false>{});
                    const f32x4 acc[2] = {acc0, acc1};
                    if (lsum) {
                        // kept for the LDS sum at the end (mb < 2, nb0 == 0: lsum_op)
                        if (mb == 0) {
                            hold[0][0] = acc0;
                            hold[0][1] = acc1;
                        } else {
                            hold[1][0] = acc0;
                            hold[1][1] = acc1;
                        }
                        continue;
                    }
                    // each wave stores its partial tile into its own slab row (lane (kq, l16) holds rows
                    // 4 kq + r, column l16 of the 16 x 16 block); the slab reduction sums the rows
    #pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        if (u == 1 && !two) break;
                        const int j2 = 16 * (nb0 + u) + l16;
    #pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i2 = 16 * mb + 4 * kq + r;
                            if (i2 < MI && j2 < NJ) {
                                const int co2 = i2 / K, kx2 = i2 - co2 * K;
                                if (ucls) {
                                    const int ci2 = j2 >> 1, rr = j2 & 1, py = (T.oy0 + wv) & 1;
                                    const int kyl = rr ? 1 + py : 0, kyh = rr ? 2 : py;
                                    float* const sp = slab + co2 * J + ci2 * KK + kx2;
                                    sp[kyl * K] = acc[u][r];
                                    if (kyh != kyl) sp[kyh * K] = acc[u][r];
                                } else {
                                    const int ci2 = j2 / K, ky2 = j2 - ci2 * K;
                                    slab[co2 * J + ci2 * KK + ky2 * K + kx2] = acc[u][r];
                                }
                            }
                        }
                    }
                }
            }
        }
    };
    // fuse_alt: which workgroups take the weight gradient last -- blocks of one CU are (roughly) those
    // the XCD's dispatcher deals it 32 apart: bit 8 of the block index alternates among them
    const int bsel = Gt.alt == 1 ? (int)(blockIdx.x >> 8) : Gt.alt == 2 ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    const bool wg_late = FUSE && Gt.alt != 0 && (bsel & 1) != 0;
    if (vop && !wg_late) wgrad_phase();
    PHASE(5);

    // ---- phase 4b: input gradient (MFMA) + BN backward of the input + S_in (+)= gamma * dbn
    float sd = 0.f, sdx = 0.f;   // this lane's channel l16
    if (nmblk > 0) {
        // x-hat of an active (a > 0) input from its activation a = gamma x-hat + beta
        float l_bet = 0.f, l_rgam = 0.f, l_gam = 0.f;
        if (d.in_bn) {
            l_gam = i_gam[ci_l];
            l_bet = i_sh[ci_l] + i_mean[ci_l] * i_sc[ci_l];     // beta
            l_rgam = 1.f / l_gam;
        }
        const float* arow0 = alb + (ci_l * Gt.rh + (py0 - iy0)) * Gt.P + HALO;   // owned row 0 of channel l16
        const int nkd = KD4 >> 2;
#if GPI_IG_PAIR
        bool paired = false;
        f32x4 acc_next = {0.f, 0.f, 0.f, 0.f};
#endif
        for (int round = 0; wv + 16 * round < nmblk; ++round) {
            if (round > 0 && S != 2) {
#if GPI_IG_PRE
                if (round == 1) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) pv4[u] = pv4b[u];
                } else
#endif
                own_load(round, pv4);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = wv + 4 * (4 * round + u);
                if (m < nmblk) {
                    const int i = 16 * m + l16;                   // owned pixel of this lane's A row
                    const int qy = dq(i, Gt.d_win), px = i - qy * d.w_in;
                    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                    if (S == 2) {
                        // parity-class blocks: block m covers 16 consecutive pixels (a, b) of class
                        // cls = m / nbc, i.e. input pixels (py0 + 2a + ry, 2b + rx); only the class's
                        // valid taps enter the reduction (1 / 2 / 2 / 4 of the 9 at K = 3)
                        const int nbc = nmblk >> 2, cls = m / nbc, mb = m - cls * nbc;
                        const int ry = cls >> 1, rx = cls & 1;
                        const int nky = (K - ((ry + d.pad) & 1) + 1) >> 1, nkx = (K - ((rx + d.pad) & 1) + 1) >> 1;
                        // (wave-uniform: m is; readfirstlane keeps the reduction loop's control scalar)
                        const int nk = __builtin_amdgcn_readfirstlane(d.cout * nky * nkx);
                        const int cp = 16 * mb + l16, a2 = dq(cp, Gt.d_w2), b2 = cp - a2 * (d.w_in >> 1);
                        const float* ab = gl + ((py0 >> 1) - gy0 + a2) * Gt.PG + b2 + HALO;
                        const int2* tAB = reinterpret_cast<const int2*>(ktab + cls * 2 * KD4);
                        const int nks = (nk + 3) >> 2;            // (4 nks <= KD4: every table read in range)
#if GPI_S2_IG_SERIAL
                        for (int ks = 0; ks < nks; ++ks) {
                            const int k = 4 * ks + kq;
                            const int2 t = tAB[k];
                            const float a = k < nk ? ab[t.x] : 0.f;
                            acc = mfma4(a, wD[t.y + l16], acc);
                        }
#else
                        // operands of four steps in flight before their MFMAs (the serial form was a chain of two
                        // dependent LDS round trips per MFMA); the padded entries k >= nk hold (0, 0): their
                        // loads stay in range, the select zeroes their A value -- the sums, and their order, are
                        // the serial form's
                        int ks = 0;
                        for (; ks + 4 <= nks; ks += 4) {
                            int2 t[4];
                            float a[4], b[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) t[u] = tAB[4 * (ks + u) + kq];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                a[u] = ab[t[u].x];
                                b[u] = wD[t[u].y + l16];
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) acc = mfma4(4 * (ks + u) + kq < nk ? a[u] : 0.f, b[u], acc);
                        }
                        for (; ks < nks; ++ks) {
                            const int k = 4 * ks + kq;
                            const int2 t = tAB[k];
                            const float a = ab[t.x], b = wD[t.y + l16];
                            acc = mfma4(k < nk ? a : 0.f, b, acc);
                        }
#endif
                    } else {
                        const float* gp0 = gl + (UP ? 2 * (qy * Gt.PG + px) : qy * Gt.PG + px);
                        auto aval = [&](int k) -> float {
                            const float* ga = gp0 + ktab[k];
                            return UP ? (ga[0] + ga[1]) + (ga[Gt.PG] + ga[Gt.PG + 1]) : ga[0];
                        };
#if GPI_IG_PAIR
                        // block pairs (m, m + 4): one offset-table and weight read per step serve both blocks'
                        // gathers and MFMAs (two independent accumulator chains); each block's sum and its
                        // order are the single-block form's
                        if ((u & 1) && paired) {
                            acc = acc_next;
                        } else if (!(u & 1) && m + 4 < nmblk) {
                            const int i1 = i + 64;
                            const int qy1 = dq(i1, Gt.d_win), px1 = i1 - qy1 * d.w_in;
                            const float* gp1 = gl + (UP ? 2 * (qy1 * Gt.PG + px1) : qy1 * Gt.PG + px1);
                            auto at = [&](const float* ga) -> float {
                                return UP ? (ga[0] + ga[1]) + (ga[Gt.PG] + ga[Gt.PG + 1]) : ga[0];
                            };
                            f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
                            int ks = 0;
                            for (; ks + 4 <= nkd; ks += 4) {
                                int o[4];
                                float a0[4], a1[4], b[4];
#pragma unroll
                                for (int v = 0; v < 4; ++v) o[v] = ktab[4 * (ks + v) + kq];
#pragma unroll
                                for (int v = 0; v < 4; ++v) {
                                    a0[v] = at(gp0 + o[v]);
                                    a1[v] = at(gp1 + o[v]);
                                    b[v] = wD[(4 * (ks + v) + kq) * 16 + l16];
                                }
#pragma unroll
                                for (int v = 0; v < 4; ++v) {
                                    acc = mfma4(a0[v], b[v], acc);
                                    acc1 = mfma4(a1[v], b[v], acc1);
                                }
                            }
                            for (; ks < nkd; ++ks) {
                                const int k = 4 * ks + kq;
                                const int o = ktab[k];
                                const float b = wD[k * 16 + l16];
                                acc = mfma4(at(gp0 + o), b, acc);
                                acc1 = mfma4(at(gp1 + o), b, acc1);
                            }
                            acc_next = acc1;
                            paired = true;
                        } else {
                        paired = false;
#endif
                        int ks = 0;
                        for (; ks + 4 <= nkd; ks += 4) {   // operands of four steps before their MFMAs
                            float a[4], b[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int k = 4 * (ks + u) + kq;
                                a[u] = aval(k);
                                b[u] = wD[k * 16 + l16];
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) acc = mfma4(a[u], b[u], acc);
                        }
                        for (; ks < nkd; ++ks) {
                            const int k = 4 * ks + kq;
                            acc = mfma4(aval(k), wD[k * 16 + l16], acc);
                        }
#if GPI_IG_PAIR
                        }
#endif
                    }
                    if (cok && S == 2) {
                        const int nbc = nmblk >> 2, cls = m / nbc, mb = m - cls * nbc;
                        const int ry = cls >> 1, rx = cls & 1;
                        const int cp0 = 16 * mb + 4 * kq, a2 = dq(cp0, Gt.d_w2), b2 = cp0 - a2 * (d.w_in >> 1);
                        const int qy = 2 * a2 + ry;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int px = 2 * (b2 + q) + rx;
                            const int64_t go = ibase + (int64_t)qy * d.w_in + px;
                            const float pa = d.gin_accumulate ? *as_gld(ws + gin_off + go) : 0.f;
                            float o;
                            if (d.in_bn) {
                                const float av = arow0[qy * Gt.P + px];
                                const float dbn = av > 0.f ? acc[q] : 0.f;
                                o = pa + l_gam * dbn;
                                sd += dbn;
                                sdx += dbn * ((av - l_bet) * l_rgam);
                            } else {
                                o = pa + acc[q];
                            }
                            *as_gst(ws + gin_off + go) = o;   // every other pixel: plain (sc1 measured slower)
                        }
                    } else if (cok) {
                        float* gp = ws + gin_off + ibase + 16 * m + 4 * kq;
                        const int i0 = 16 * m + 4 * kq;
                        const int qy0 = dq(i0, Gt.d_win), px0 = i0 - qy0 * d.w_in;
                        const f32x4 av = *(const f32x4*)(arow0 + qy0 * Gt.P + px0);
                        const float pa[4] = {pv4[u][0], pv4[u][1], pv4[u][2], pv4[u][3]};
                        float o[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (d.in_bn) {
                                const float dbn = av[q] > 0.f ? acc[q] : 0.f;
                                o[q] = pa[q] + l_gam * dbn;
                                sd += dbn;
                                sdx += dbn * ((av[q] - l_bet) * l_rgam);
                            } else {
                                o[q] = pa[q] + acc[q];
                            }
                        }
                        st4(gp, f32x4{o[0], o[1], o[2], o[3]});
                    }
                }
            }
        }
    }
#if GPI_VDG3
    // ---- phase 4b (v3): the 3x3 / stride-1 input gradient on the VALU.  Q consecutive pixels of an owned
    // row per thread (2 when the tile has >= 512 owned pixels, else 1), all input channels as packed pairs:
    // per (co, ky) the output-gradient window of the Q pixels (Q + 2 values) from the LDS image, per tap the
    // CIV3 weights by CIV3 / 4 broadcast ds_read_b128, then Q x CIV3 / 2 v_pk_fma_f32.  The previous S_in
    // (accumulating ops) is loaded at the item's start, under the compute.  Epilogue as the MFMA form's: ReLU
    // mask, BN-backward sums, S_in (+)= gamma * dbn; the per-channel sums are wave-summed (DPP) and handed
    // to the MFMA form's reduction as the kq = 0 lanes' values of channel l16.
    if constexpr (K == 3 && S == 1 && !UP && !FUSE) {
        if (v3 && dg_role && !SKIP(G, 2)) {
            auto v3_rows = [&](auto ci_c, auto q_c) {
                constexpr int CI = decltype(ci_c)::value, Q = decltype(q_c)::value, CH = CI / 2;
                float s1[CI], s2[CI];
#pragma unroll
                for (int ci = 0; ci < CI; ++ci) s1[ci] = s2[ci] = 0.f;
                const int npq = (Gt.ph * d.w_in) / Q;
                for (int gq = tid; gq < npq; gq += 256) {
                    const int qy = dq(Q * gq, Gt.d_win), px0 = Q * gq - qy * d.w_in;
                    const int64_t gb_in = ((int64_t)T.b * d.in_ctot + d.in_c0) * HWi + (int64_t)(py0 + qy) * d.w_in + px0;
                    float pv[CI][Q];
                    if (gq == tid) {           // (loaded in phase 1)
#pragma unroll
                        for (int ci = 0; ci < CI; ++ci)
#pragma unroll
                            for (int q = 0; q < Q; ++q) pv[ci][q] = d.gin_accumulate ? pv3[ci][q] : 0.f;
                    } else {
#pragma unroll
                        for (int ci = 0; ci < CI; ++ci) {
                            const bool ok = ci < d.cin && d.gin_accumulate;
                            const float* pp = ok ? ws + gin_off + gb_in + (int64_t)ci * HWi : zero;
#pragma unroll
                            for (int q = 0; q < Q; ++q) pv[ci][q] = as_gld(pp)[ok ? q : 0];
                        }
                    }
                    f32x2 acc2[CH][Q];
#pragma unroll
                    for (int h = 0; h < CH; ++h)
#pragma unroll
                        for (int q = 0; q < Q; ++q) acc2[h][q] = f32x2{0.f, 0.f};
                    for (int co = 0; co < d.cout; ++co) {
#pragma unroll
                        for (int ky = 0; ky < K; ++ky) {
                            const float* grow = gl + co * gplane + (qy + py0 + d.pad - ky - gy0) * Gt.PG + HALO + px0 +
                                                d.pad - (K - 1);
                            float gw[K + Q - 1];
#pragma unroll
                            for (int t = 0; t < K + Q - 1; ++t) gw[t] = grow[t];
                            const float* wrow = wD + (co * K + ky) * K * CI;
#pragma unroll
                            for (int kx = 0; kx < K; ++kx) {
                                f32x4 w4[CI / 4];
#pragma unroll
                                for (int v = 0; v < CI / 4; ++v) w4[v] = *reinterpret_cast<const f32x4*>(wrow + kx * CI + 4 * v);
#pragma unroll
                                for (int q = 0; q < Q; ++q) {
                                    const float gv = gw[q + K - 1 - kx];
#pragma unroll
                                    for (int h = 0; h < CH; ++h) {
                                        const f32x2 w = f32x2{w4[h >> 1][2 * (h & 1)], w4[h >> 1][2 * (h & 1) + 1]};
                                        acc2[h][q] = __builtin_elementwise_fma(w, f32x2{gv, gv}, acc2[h][q]);
                                    }
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) {
                        if (ci >= d.cin) break;
                        const float* ap = alb + (ci * Gt.rh + (py0 - iy0 + qy)) * Gt.P + HALO + px0;
                        // (the channel's BN constants by uniform LDS reads here, not held across the item)
                        const float lg = d.in_bn ? i_gam[ci] : 0.f;
                        const float lb = d.in_bn ? i_sh[ci] + i_mean[ci] * i_sc[ci] : 0.f;
                        const float lr = d.in_bn ? 1.f / lg : 0.f;
                        float o[Q];
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            const float a = acc2[ci >> 1][q][ci & 1];
                            if (d.in_bn) {
                                const float av = ap[q];
                                const float dbn = av > 0.f ? a : 0.f;
                                o[q] = pv[ci][q] + lg * dbn;
                                s1[ci] += dbn;
                                s2[ci] += dbn * ((av - lb) * lr);
                            } else {
                                o[q] = pv[ci][q] + a;
                            }
                        }
                        store_px<Q>(ws + gin_off + gb_in + (int64_t)ci * HWi, o);
                    }
                }
                if (d.in_bn) {
                    // wave sums (DPP) of the 2 CI channel sums; lane l16 of the kq = 0 lanes takes channel l16's
                    float v2[2 * CI];
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) {
                        v2[ci] = s1[ci];
                        v2[CI + ci] = s2[ci];
                    }
                    wave_sums(v2);
                    float a = 0.f, b = 0.f;
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) {
                        a = l16 == ci ? v2[ci] : a;
                        b = l16 == ci ? v2[CI + ci] : b;
                    }
                    sd = kq == 0 ? a : 0.f;
                    sdx = kq == 0 ? b : 0.f;
                }
            };
            const bool q2 = Gt.ph * d.w_in >= 512;
            if (d.cin <= 4) { if (q2) v3_rows(IntC<4>{}, IntC<2>{}); else v3_rows(IntC<4>{}, IntC<1>{}); }
            else if (d.cin <= 8) { if (q2) v3_rows(IntC<8>{}, IntC<2>{}); else v3_rows(IntC<8>{}, IntC<1>{}); }

        }
    }
#endif
    // ---- phase 4b': input gradient on the VALU (cin <= 4, 5x5, stride 1): Q consecutive pixels of an
    // owned row per thread (4 for cin <= 2, 2 otherwise), all (<= 4) input channels at once.  The
    // weights W[co][ci][ky][kx] are wave-uniform: scalar loads from the parameters (constant address
    // space, SGPR operands of the FMAs), no LDS traffic for them; the output-gradient row window of
    // the Q pixels is read from LDS once per (co, ky).
    float vsd[4] = {0.f, 0.f, 0.f, 0.f}, vsdx[4] = {0.f, 0.f, 0.f, 0.f};
    if (vdg && !SKIP(G, 2)) {
        float lg[4], lb[4], lr[4];
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            const int cc = min(ci, d.cin - 1);
            lg[ci] = d.in_bn ? i_gam[cc] : 0.f;
            lb[ci] = d.in_bn ? i_sh[cc] + i_mean[cc] * i_sc[cc] : 0.f;
            lr[ci] = d.in_bn ? 1.f / lg[ci] : 0.f;
        }
        // packed over input-channel pairs: WB[((co K + ky) K + kx) CIV + ci]; lane l holds WB[64 j + l] in
        // wb[j], a tap's channel pair is taken by v_readlane (no LDS traffic for the weights in the loop)
        auto vdg_rows = [&](auto ci_c) {
            constexpr int CI = decltype(ci_c)::value;     // == CIV
            constexpr int CH = CI / 2;
            constexpr int Q = CI == 2 ? 4 : 2;
            constexpr int NWB = (2 * KK * CI + 63) / 64;   // cout <= 2 (vop)
            float wb[NWB];
    #pragma unroll
            for (int j = 0; j < NWB; ++j) wb[j] = mid[64 * j + lane];
            const int npq = (Gt.ph * d.w_in) / Q;
            for (int gq = tid; gq < npq; gq += 256) {
                const int qy = dq(Q * gq, Gt.d_win), px0 = Q * gq - qy * d.w_in;
                const int64_t pix = (int64_t)(py0 + qy) * d.w_in + px0;
                const int64_t gbase_in = ((int64_t)T.b * d.in_ctot + d.in_c0) * HWi + pix;
                f32x2 acc2[CH][Q];
    #pragma unroll
                for (int h = 0; h < CH; ++h)
    #pragma unroll
                    for (int q = 0; q < Q; ++q) acc2[h][q] = f32x2{0.f, 0.f};
    #pragma unroll
                for (int co = 0; co < 2; ++co) {
                    if (co >= d.cout) break;
    #pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        const float* grow = gl + co * gplane + (qy + py0 + d.pad - ky - gy0) * Gt.PG + HALO + px0 +
                                            d.pad - (K - 1);
                        float gw[K + Q - 1];
                        if constexpr (Q == 4) {
                            // px0 multiple of 4: the window starts (HALO + pad - (K - 1)) mod 4 past a 16-B boundary
                            lds_window<K + Q - 1, (HALO + K / 2 - (K - 1)) & 3>(grow, gw);
                        } else {
    #pragma unroll
                            for (int t = 0; t < K + Q - 1; ++t) gw[t] = grow[t];
                        }
    #pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            f32x2 w[CH];
    #pragma unroll
                            for (int h = 0; h < CH; ++h) {
                                const int i = ((co * K + ky) * K + kx) * CI + 2 * h;
                                if (GPI_VDG_WLDS) {
                                    // the channel pair by one broadcast LDS read (as the fused forward's weights)
                                    w[h] = *reinterpret_cast<const f32x2*>(mid + i);
                                } else {
                                    w[h][0] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wb[i >> 6]), i & 63));
                                    w[h][1] = __int_as_float(
                                        __builtin_amdgcn_readlane(__float_as_int(wb[(i + 1) >> 6]), (i + 1) & 63));
                                }
                            }
    #pragma unroll
                            for (int q = 0; q < Q; ++q) {
                                const float gv = gw[q + K - 1 - kx];
    #pragma unroll
                                for (int h = 0; h < CH; ++h)
                                    acc2[h][q] = __builtin_elementwise_fma(w[h], f32x2{gv, gv}, acc2[h][q]);
                            }
                        }
                    }
                }
                float acc[CI][Q];
    #pragma unroll
                for (int ci = 0; ci < CI; ++ci)
    #pragma unroll
                    for (int q = 0; q < Q; ++q) acc[ci][q] = acc2[ci >> 1][q][ci & 1];
    #pragma unroll
                for (int ci = 0; ci < CI; ++ci) {
                    if (ci >= d.cin) break;
                    const float* ap = alb + (ci * Gt.rh + (py0 - iy0 + qy)) * Gt.P + HALO + px0;
                    float av[Q], pv[Q], o[Q];
    #pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        av[q] = ap[q];
                        pv[q] = 0.f;
                    }
                    if (d.gin_accumulate) {
                        auto pp = as_gld(ws + gin_off + gbase_in + (int64_t)ci * HWi);
    #pragma unroll
                        for (int q = 0; q < Q; ++q) pv[q] = pp[q];
                    }
    #pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        if (d.in_bn) {
                            const float dbn = av[q] > 0.f ? acc[ci][q] : 0.f;
                            o[q] = pv[q] + lg[ci] * dbn;
                            vsd[ci] += dbn;
                            vsdx[ci] += dbn * ((av[q] - lb[ci]) * lr[ci]);
                        } else {
                            o[q] = pv[q] + acc[ci][q];
                        }
                    }
                    store_px<Q>(ws + gin_off + gbase_in + (int64_t)ci * HWi, o);
                }
            }
        };
        if (d.cin <= 2) vdg_rows(IntC<2>{});
        else vdg_rows(IntC<4>{});
    }
    if (d.in_bn && dg_role) {
        __syncthreads();          // red aliases the offset table the input-gradient loop read
        if (vdg) {
            // per-thread channel sums: wave sums -> this wave's slab row (dgamma / dbeta partials) and LDS
            float ws8[8] = {vsd[0], vsd[1], vsd[2], vsd[3], vsdx[0], vsdx[1], vsdx[2], vsdx[3]};
            wave_sums(ws8);
#pragma unroll
            for (int ci = 0; ci < 4; ++ci) {
                const float a = ws8[ci], b = ws8[4 + ci];
                if (lane == 0 && ci < d.cin) {
                    red[wv * 32 + ci] = a;
                    red[128 + wv * 32 + ci] = b;
                    slab[d.cout * J + ci] = b;
                    slab[d.cout * J + d.cin + ci] = a;
                }
            }
        } else {
            // lanes 16 apart share a channel: fold them (v3: wave sums already in the kq = 0 lanes)
            if (!v3) {
                sd += __shfl_xor(sd, 16, 64);
                sdx += __shfl_xor(sdx, 16, 64);
                sd += __shfl_xor(sd, 32, 64);
                sdx += __shfl_xor(sdx, 32, 64);
            }
            if (kq == 0) {
                red[wv * 32 + l16] = sd;
                red[128 + wv * 32 + l16] = sdx;
                if (cok && !lsum && wout) {
                    slab[d.cout * J + l16] = sdx;             // dgamma partial of this wave
                    slab[d.cout * J + d.cin + l16] = sd;      // dbeta partial
                }
            }
        }
        __syncthreads();
        if (tid < d.cin) {
            // the four waves in a fixed order: the BN-backward sums of the input statistics
            double s_d = 0.0, s_dx = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                s_d += (double)red[w * 32 + tid];
                s_dx += (double)red[128 + w * 32 + tid];
            }
            gpi_stat* st = stat_slot(c, d.in_stat + tid, T.grp);
            const double gm = i_gam[tid];
            if (!SKIP(G, 4)) {
                atomicAdd(&st->ssum, gm * s_d);
                atomicAdd(&st->sxsum, gm * s_dx);
            }
        }
    }
    if (!vop || wg_late) wgrad_phase();
    PHASE(6);
    if (lsum) {
        // the four waves' partial rows into LDS (the whole region after the header is dead by now; the
        // barrier also orders the channel-sum scratch reads above), summed in a fixed order into the
        // tile's one slab row.  Split launches: each role sums and stores its own columns.
        __syncthreads();
        const int MI = d.cout * K, NJ = d.cin * K;
        const int nmb = (SKIP(G, 1) || !do_wgrad) ? 0 : (MI + 15) >> 4;
        const bool two = NJ > 16;
        float* lrow = wD + wv * rowlen;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            if (mb >= nmb) break;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !two) break;
                const f32x4 a = hold[mb][u];
                const int j2 = 16 * u + l16;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i2 = 16 * mb + 4 * kq + r;
                    if (i2 < MI && j2 < NJ) {
                        const int co2 = i2 / K, kx2 = i2 - co2 * K, ci2 = j2 / K, ky2 = j2 - ci2 * K;
                        lrow[co2 * J + ci2 * KK + ky2 * K + kx2] = a[r];
                    }
                }
            }
        }
        if (d.in_bn && dg_role && kq == 0 && cok) {
            lrow[d.cout * J + l16] = sdx;             // dgamma partial of this wave
            lrow[d.cout * J + d.cin + l16] = sd;      // dbeta partial
        }
        __syncthreads();
        const int c0 = (Gt.split && !do_wgrad) ? d.cout * J : 0;
        const int c1 = !wout ? 0 : ((Gt.split && !dg_role) ? d.cout * J : rowlen);
        float* srow = c.wpart + d.wpart_off + (int64_t)tile * rowlen;
        for (int e = c0 + tid; e < c1; e += 256) {
            const float* r = wD + e;
            srow[e] = (r[0] + r[rowlen]) + (r[2 * rowlen] + r[3 * rowlen]);
        }
    }
    if (vop) {
        // the four waves' partial rows in a fixed order -> the tile's slab row
        __syncthreads();
        float* srow = c.wpart + d.wpart_off + (int64_t)tile * rowlen;
        for (int e = tid; e < (wout ? rowlen : 0); e += 256) {
            const float* r = mid + 512 + e;
            srow[e] = (r[0] + r[rowlen]) + (r[2 * rowlen] + r[3 * rowlen]);
        }
    }
    PHASE(7);
    RTSTAMP(1);
}

size_t fwd_lds(const gpi_conv_desc& d, const ConvGeom& G, int cp) {
    return sizeof(float) * ((size_t)pad256(FWD_HDR) + pad256(d.cin * d.k * d.k * cp) + img_floats(d.cin, G.rh, G.P) +
                            (G.cg > 1 ? (size_t)(G.cg - 1) * G.th * d.w_out * cp : 0));
}

size_t bwd_lds_floats(const gpi_conv_desc& d, int rh, int P, int gh, int PG, int zreg, bool fuse) {
    const int KD4 = (d.cout * d.k * d.k + 3) & ~3;
    const int gimg = img_floats(d.cout, gh, PG);
    const bool zimg = d.gout_mode == 0 && !zreg;             // z image in LDS
    // offset table, at least BWD_RED floats: the channel-sum scratch aliases it (fuse: the target image
    // [gh][w_out] in place of the MFMA input-gradient weights and offset table)
    const size_t mid = vop_op(d) ? vop_mid_floats(gh, d.w_out, bwd_rowlen(d), fuse)
                                 : (d.gin_off >= 0 ? pad256(KD4 * 16) + pad256((d.stride == 2 ? 8 : 1) * KD4) : 0);
    return (size_t)bwd_hdr(d.cin, d.cout) + mid + gimg + (zimg ? gimg : 0) + img_floats(d.cin, rh, P);
}

size_t bwd_lds(const gpi_conv_desc& d, const ConvGeom& G) {
    return sizeof(float) * bwd_lds_floats(d, G.rh, G.P, G.gh, G.PG, G.zreg, G.fuse != 0);
}

// One slab row per tile for the MFMA backward (G.lsum): the weight-gradient accumulators fit the
// kernel's 2 x 2 register blocks (cout K, cin K <= 32), not the single-channel stride-2 input conv's
// own form, and the four partial rows fit the LDS after the header.  On every launch it cost more than the
// stores and the smaller reductions save with the generic kernels -- 0.6315 vs 0.6258 ms/step (r03, 3 x 600
// replays per arm).  Default 2 since r06: only on output planes of <= 16 x 16 pixels (3: <= 8 x 8; 1: every
// launch; 0: off), where the four slab rows per tile are as many bytes as the launch's own operands (PMC:
// TransDown3.conv2.bwd 2.7-3.0x its algorithmic bytes) -- with the shape kernels 0.4384-0.4393 vs 0.4413-0.4419
// ms/step (profiles/r06k_ab_lsum.txt)
bool lsum_op(const gpi_conv_desc& d, const ConvGeom& G) {
    static const int on = env_int("GPI_LSUM", 2);
    if (!on || vop_op(d) || G.fuse) return false;
    if ((on == 2 && d.h_out * d.w_out > 256) || (on == 3 && d.h_out * d.w_out > 64)) return false;
    if (d.k == 7 && d.stride == 2 && !d.upsample && d.cin == 1 && d.gin_off < 0 && d.cout <= 16) return false;
    if (d.cout * d.k > 32 || d.cin * d.k > 32) return false;
    const size_t avail = bwd_lds_floats(d, G.rh, G.P, G.gh, G.PG, G.zreg, false) - bwd_hdr(d.cin, d.cout);
    return avail >= (size_t)4 * bwd_rowlen(d);
}

// One slab row per tile for the single-channel 7x7 stride-2 input conv's weight gradient (the kernel's
// vwg form): the four waves' rows summed in LDS over the dead gradient image, when it holds them.
bool vsum_op(const gpi_conv_desc& d, const ConvGeom& G) {
    static const int on = env_int("GPI_VSUM", 1);
    if (!on || !(d.k == 7 && d.stride == 2 && !d.upsample && d.cin == 1 && d.gin_off < 0 && d.cout <= 16)) return false;
    return (size_t)img_floats(d.cout, G.gh, G.PG) >= (size_t)4 * bwd_rowlen(d);
}

typedef void (*conv_kernel_t)(gpi_conv_desc, gpi_codec_ctx, ConvGeom);

// entries whose instantiation spills at its occupancy target (the folded loops unroll further than the generic
// kernel's): their launches keep the generic kernel (GPI_CONV_SHAPE_NOFOLD in conv_shapes.h, from
// tools/kernel_resources.sh after a build; tools/gen_conv_shapes.py carries the list over)
#ifndef GPI_CONV_SHAPE_NOFOLD
#define GPI_CONV_SHAPE_NOFOLD {-1}
#endif
constexpr int kNoFold[] = GPI_CONV_SHAPE_NOFOLD;
constexpr bool no_fold(int i) {
    for (int v : kNoFold)
        if (v == i) return true;
    return false;
}

template <int I>
conv_kernel_t shape_kernel() {
    constexpr ShapeC s = kShapes[I];
    // (the fused output conv only with GPI_FUSE_FOLD != 0: see there)
    if constexpr ((s.fusek != 0 && GPI_FUSE_FOLD == 0) || no_fold(I)) return nullptr;
    else if constexpr (s.fwd != 0) return conv_fwd_kernel<s.D_k, s.D_stride, s.D_upsample, s.cp, s.npxk, s.half != 0, I>;
    else return conv_bwd_kernel<s.D_k, s.D_stride, s.upk, s.fusek != 0, s.half != 0, s.v3 != 0, s.exf != 0, I>;
}

// kernel of entry LO + i, entries [LO, LO + n) instantiated here
template <int LO, int... I>
conv_kernel_t shape_kernel_at(int i, std::integer_sequence<int, I...>) {
    static const conv_kernel_t t[] = {shape_kernel<LO + I>()..., nullptr};
    return t[i];
}

}  // namespace

// the other parts' tables of kernels (hidden: not part of the library's interface)
namespace gpi_conv_parts {
__attribute__((visibility("hidden"))) void* shape_part1(int i);
__attribute__((visibility("hidden"))) void* shape_part2(int i);
__attribute__((visibility("hidden"))) void* shape_part3(int i);
#if GPI_CONV_SHAPE_PART > 0
#define GPI_PART_FN_(p) shape_part##p
#define GPI_PART_FN(p) GPI_PART_FN_(p)
void* GPI_PART_FN(GPI_CONV_SHAPE_PART)(int i) {
    constexpr int lo = kBounds[GPI_CONV_SHAPE_PART], n = kBounds[GPI_CONV_SHAPE_PART + 1] - lo;
    return (void*)shape_kernel_at<lo>(i, std::make_integer_sequence<int, n>{});
}
#endif
}  // namespace gpi_conv_parts

namespace {
#if GPI_CONV_SHAPE_PART == 0

template <int K, int S, int UP, int NPX, bool HALF>
conv_kernel_t pick_cp_h(int cp) {
    if (cp == 2) return conv_fwd_kernel<K, S, UP, 2, NPX, HALF>;
    if (cp == 4) return conv_fwd_kernel<K, S, UP, 4, NPX, HALF>;
    if (cp == 6) return conv_fwd_kernel<K, S, UP, 6, NPX, HALF>;
    return conv_fwd_kernel<K, S, UP, 8, NPX, HALF>;
}

template <int K, int S, int UP, int NPX>
conv_kernel_t pick_cp(int cp, bool half = false) {
    // (no channel-group instantiation with half tiles: conv_geom keeps those launches whole)
    if constexpr (NPX != 0) {
        if (half) return pick_cp_h<K, S, UP, NPX, true>(cp);
    }
    return pick_cp_h<K, S, UP, NPX, false>(cp);
}

template <int K, int S, int UP>
conv_kernel_t pick(int cp, bool fwd, int npx, bool half, bool ucls = false) {
    if constexpr (UP != 0) {
        // UP = 2: the upsampling backward with the row-parity weight-gradient columns (ConvGeom::ucls), an
        // instantiation of its own: as a runtime branch its index arithmetic spilled 4 registers of every
        // upsampling backward (+1.2-1.6 us per launch)
        if (!fwd && ucls) return half ? conv_bwd_kernel<K, S, 2, false, true> : conv_bwd_kernel<K, S, 2>;
    }
    if constexpr (K == 3 && S == 1 && UP == 0) {
        // (the ucls slot carries v3_op for this shape)
        if (!fwd && ucls) return half ? conv_bwd_kernel<3, 1, 0, false, true, true> : conv_bwd_kernel<3, 1, 0, false, false, true>;
    }
    if (!fwd) return half ? conv_bwd_kernel<K, S, UP, false, true> : conv_bwd_kernel<K, S, UP>;
    if (npx == 4) return pick_cp<K, S, UP, 4>(cp, half);
    if (npx == 2) return pick_cp<K, S, UP, 2>(cp, half);
    if constexpr (!UP && K <= 3) {   // channel-group instantiation: the small-plane codec convs only
        if (npx == 0) return pick_cp<K, S, UP, 0>(cp);
    }
    return pick_cp<K, S, UP, 1>(cp, half);
}

// the backward ops that take the VALU input gradient (GPI_VDG3; the kernel's v3 condition at full tiles)
bool v3_op(const gpi_conv_desc& d, const ConvGeom& G) {
    return GPI_VDG3 && d.k == 3 && d.stride == 1 && !d.upsample && d.gin_off >= 0 && d.cin <= 8 && G.ph * d.w_in >= 256;
}

conv_kernel_t select_kernel(const gpi_conv_desc& d, int cp, bool fwd, int npx, bool half, bool ucls) {
    const int key = d.k * 100 + d.stride * 10 + d.upsample;
    switch (key) {
        case 110: return pick<1, 1, 0>(cp, fwd, npx, half);
        case 310: return pick<3, 1, 0>(cp, fwd, npx, half, ucls);
        case 311: return pick<3, 1, 1>(cp, fwd, npx, half, ucls);
        case 320: return pick<3, 2, 0>(cp, fwd, npx, half);
        case 510: return pick<5, 1, 0>(cp, fwd, npx, half);
        case 720: return pick<7, 2, 0>(cp, fwd, npx, half);
        default: return nullptr;
    }
}

// output channels per thread in the forward (accumulators; weights stored with this stride): the
// 5- and 6-channel 1x1, stride-2 and upsampling convs take 6 (float2 weight reads) instead of padding
// to 8; the 3x3 stride-1 and 7x7 ones measured faster with 8 (float4 reads)
int cp_of(const gpi_conv_desc& d) {
    const int cout = d.cout;
    if (cout <= 2) return 2;
    if (cout <= 4) return 4;
    // GPI_FWD_CP6=1: the 3x3 stride-1 ones with 5-6 outputs on 6 as well (A/B of the rule on the shape kernels)
    static const int cp6 = env_int("GPI_FWD_CP6", 0);
    const bool wide8 = d.k == 7 || (d.k == 3 && d.stride == 1 && !d.upsample && !cp6);
    return (cout <= 6 && !wide8) ? 6 : 8;
}

// Alignment preconditions of the 16-byte operand paths (row images, float4 epilogue).
bool aligned_ok(const gpi_conv_desc& d, const gpi_codec_ctx& c, bool fwd) {
    if (((uintptr_t)c.ws & 15) || (d.in_off >= 0 && (d.in_off & 3))) return false;
    if (d.in_off < 0 && (((uintptr_t)c.ext_in & 15) || (c.ext_stride & 3))) return false;
    if (fwd) return true;
    if (d.cin > 16) return false;
    if (d.in_bn && (d.in_off < 0 || d.gin_off < 0)) return false;
    if ((d.gout_off & 3) || (d.gout_mode == 0 && (d.out_off & 3))) return false;
    if (d.gin_off >= 0 && (d.gin_off & 3)) return false;
    return true;
}

// XCD-aware block order per launch kind (ConvGeom::xcd), GPI_XCD_MODE bits: 1 forward, 2 backward,
// 4 split backward, 8 the fused output conv.  With every kind on, the step's PMC traffic fell 547 ->
// 505 MB (the fused output conv 1.24x -> 1.05x its algorithmic bytes, the 32/64-wide forwards ~1.15x ->
// 1.03x) at unchanged forward and fused launch times, but several backward launches ran 0.6-2.2 us
// slower (step 0.635 vs 0.625 ms, r03x).  Default 9 (forward + fused): 0.6233 / 0.6219 ms vs 0.6232 /
// 0.6228 with the fused conv alone and 0.6277 / 0.6250 with the non-split backwards too (r03y).
bool xcd_mode(bool fwd, bool fuse, bool split, bool half) {
    static const int mode = env_int("GPI_XCD_MODE", 9);
    // (a launch with half tiles keeps the dispatch order: the XCD-consecutive order would put every half
    // tile on the last XCDs -- 0.5714-0.5722 vs 0.5694-0.5709 ms for the fused output conv, r04t)
    return !half && (mode & (fuse ? 8 : fwd ? 1 : split ? 4 : 2)) != 0;
}

// The shape of a planned launch (compile-time shapes above): the kernel variant select_kernel picks, the
// B-independent descriptor fields and the geometry.  Unused bytes stay zero (value-initialised), so two
// shapes compare by their bytes.
ShapeC shape_of(const gpi_conv_desc& d, const ConvGeom& G, bool fwd, bool fuse, int cp, bool exf) {
    ShapeC s{};
    const bool half = G.nfull < G.nblocks;
    s.fwd = fwd;
    s.fusek = fuse;
    s.has_gin = d.gin_off >= 0;
    s.drop = d.drop_off >= 0;
    s.wout = d.wpart_off >= 0;
    s.ext_in = d.in_off < 0;
    if (fuse) {
        s.half = half;
        s.exf = exf;
        s.upk = 0;
    } else if (!fwd) {
        const bool u = G.ucls != 0 || v3_op(d, G);
        s.half = half;
        s.upk = (d.upsample && u) ? 2 : d.upsample;
        s.v3 = d.k == 3 && d.stride == 1 && !d.upsample && u;
    } else {
        // pick(): NPX = 0 (channel groups) only for the stride-1 / stride-2 convs of k <= 3 without upsampling,
        // and its instantiation has no half-tile form
        const int npx = G.cg > 1 ? 0 : G.npx;
        s.npxk = (npx == 0 && !(d.upsample == 0 && d.k <= 3)) ? 1 : npx;
        s.half = s.npxk == 0 ? 0 : half;
        s.cp = cp;
    }
#define F(n) s.D_##n = d.n;
    SHAPE_D(F)
#undef F
#define F(n) s.G_##n = G.n;
    SHAPE_G(F)
#undef F
#define F(n) s.M_##n = (int)G.n.m, s.O_##n = (int)G.n.one;
    SHAPE_GD(F)
#undef F
#define F(n) s.A_##n = G.ha.n;
    SHAPE_A(F)
#undef F
#define F(n) s.AM_##n = (int)G.ha.n.m, s.AO_##n = (int)G.ha.n.one;
    SHAPE_AD(F)
#undef F
    return s;
}

// kernel of table entry i, from the part that instantiates it
conv_kernel_t shape_kernel_any(int i) {
    if (i < 0 || i >= kNumShapes) return nullptr;
    if (i < kBounds[1]) return shape_kernel_at<0>(i, std::make_integer_sequence<int, kBounds[1]>{});
    if (i < kBounds[2]) return (conv_kernel_t)gpi_conv_parts::shape_part1(i - kBounds[1]);
    if (i < kBounds[3]) return (conv_kernel_t)gpi_conv_parts::shape_part2(i - kBounds[2]);
    return (conv_kernel_t)gpi_conv_parts::shape_part3(i - kBounds[3]);
}

// launches planned / planned with a compile-time shape since load (gpi_conv_shape_info); the shapes seen
// while GPI_CONV_SHAPES_RECORD=1 (gpi_conv_shapes_dump, tools/gen_conv_shapes.py)
// (atomic counters and a lock around the recording: launches may come from more than one host thread)
std::atomic<int64_t> g_shape_planned{0}, g_shape_matched{0};
std::vector<ShapeC> g_shapes_seen;
std::mutex g_shapes_mu;

// index of s in kShapes, or -1
int shape_index(const ShapeC& s) {
    for (int i = 0; i < kNumShapes; ++i)
        if (memcmp(&kShapes[i], &s, sizeof(ShapeC)) == 0) return i;
    return -1;
}

// dry: plan only (no device call) -- the shape recording of gpi_conv_shape_plan
int launch(const gpi_conv_desc& d, const gpi_codec_ctx& c, hipStream_t st, bool fwd, bool fuse = false,
           uint32_t* sig = nullptr, const int64_t* sig_epoch = nullptr, bool dry = false) {
    ConvGeom G;
    if (!conv_geom(d, c.groups, G, fwd, fuse)) return GPI_ERR_UNSUPPORTED;
    if (sig && !sig_epoch) return GPI_ERR_ARG;
    G.sig = sig;
    G.sig_epoch = sig_epoch;
    if (fuse && (fwd || d.k != 5 || d.stride != 1 || d.upsample || d.cout != 2 || d.cin > 4 || d.drop_off >= 0 ||
                 d.gout_mode != 1 || d.gin_off < 0 ||
                 (d.epilogue != GPI_EPI_GAUSS_LOSS && d.epilogue != GPI_EPI_GAUSS_EXP_LOSS)))
        return GPI_ERR_UNSUPPORTED;
    if ((d.epilogue == GPI_EPI_GAUSS_LOSS || d.epilogue == GPI_EPI_GAUSS_EXP_LOSS) && d.cout != 2) return GPI_ERR_ARG;
    if (d.in_off < 0 && !c.ext_in) return GPI_ERR_ARG;
    if (!aligned_ok(d, c, fwd)) return GPI_ERR_UNSUPPORTED;
    if (!fwd && d.gin_off >= 0 && ((G.ph * d.w_in) & 15)) return GPI_ERR_UNSUPPORTED;
    if (!fwd && d.gin_off >= 0 && d.stride == 2 && ((d.w_in & 7) || (G.ph & 1))) return GPI_ERR_UNSUPPORTED;
    const int cp = cp_of(d);
    const bool exf = d.epilogue == GPI_EPI_GAUSS_EXP_LOSS;
    conv_kernel_t k = fuse ? (G.nfull < G.nblocks ? (exf ? conv_bwd_kernel<5, 1, 0, true, true, false, true> : conv_bwd_kernel<5, 1, 0, true, true>)
                                                  : (exf ? conv_bwd_kernel<5, 1, 0, true, false, false, true> : conv_bwd_kernel<5, 1, 0, true>))
                           : select_kernel(d, cp, fwd, G.cg > 1 ? 0 : G.npx, G.nfull < G.nblocks,
                                           G.ucls != 0 || (!fwd && v3_op(d, G)));
    if (!k) return GPI_ERR_UNSUPPORTED;
    static const float* zero = nullptr;
    if (!zero && !dry) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_zero_page)) != hipSuccess) return GPI_ERR_LAUNCH;
        zero = (const float*)p;
    }
    G.zero = zero;
    if (!fwd) G.lsum = lsum_op(d, G) ? 1 : 0;
    if (!fwd) G.vsum = vsum_op(d, G) ? 1 : 0;
    const size_t lds = fwd ? fwd_lds(d, G, cp) : bwd_lds(d, G);
    if (lds > 160 * 1024) return GPI_ERR_UNSUPPORTED;
    if (!fwd && d.gin_off >= 0 && !fuse && !vop_op(d)) {
        // resident workgroups per CU: LDS (~160 KB less a per-workgroup reserve, tools/bench_dispatch.hip)
        // and the kernels' occupancy (6 waves per SIMD, 4 for the 5x5 kernel)
        static const int split_env = env_int("GPI_BWD_SPLIT", 1);
        const int per_cu = std::min((int)(160000 / std::max<size_t>(lds, 1)), d.k == 5 ? 4 : 6);
        // split only well under one round: 2 x 576 workgroups measured slower than 576 (r02 A/B)
        G.split = (split_env && d.wpart_off >= 0 && 2 * G.nblocks <= std::min(per_cu, 4) * 256) ? 1 : 0;
    }
    const int grid = G.nblocks * (G.split ? 2 : 1);
    G.grid = grid;
    G.xcd = xcd_mode(fwd, fuse, G.split != 0, G.nfull < G.nblocks) ? 1 : 0;
    // r04l (2 x 400 steps per arm, one box): 1 -> 0.5761 / 0.5759, off 0.5768 / 0.5773, 2 -> 0.5773 / 0.5777,
    // 3 -> 0.5776 / 0.5770 ms per step
    static const int fuse_alt = env_int("GPI_FUSE_ALT", 1);
    G.alt = fuse ? fuse_alt : 0;
    {
        // (GPI_CONV_SHAPES read per launch: a debugging run can compare both forms of one op in one process)
        const int shapes_on = env_int("GPI_CONV_SHAPES", 1);
        static const int record = env_int("GPI_CONV_SHAPES_RECORD", 0);
        const ShapeC s = shape_of(d, G, fwd, fuse, cp, exf);
        g_shape_planned += dry ? 0 : 1;
        const int si = shapes_on ? shape_index(s) : -1;
        const conv_kernel_t ks = si >= 0 ? shape_kernel_any(si) : nullptr;
        if (ks) {
            k = ks;
            g_shape_matched += dry ? 0 : 1;
        }
        if (record || dry) {
            std::lock_guard<std::mutex> lk(g_shapes_mu);
            bool seen = false;
            for (const ShapeC& q : g_shapes_seen) seen = seen || memcmp(&q, &s, sizeof(ShapeC)) == 0;
            if (!seen) g_shapes_seen.push_back(s);
        }
        if (dry) return GPI_OK;
    }
#ifdef GPI_PHASE_TIMING
    static const int dbg_print = env_int("GPI_DBG_PRINT", 0);
    if (dbg_print)
        fprintf(stderr, "conv %s k%d s%d up%d cin%d cout%d in%dx%d out%dx%d th%d blocks %d lds %zu\n",
                fwd ? "fwd" : "bwd", d.k, d.stride, d.upsample, d.cin, d.cout, d.h_in, d.w_in, d.h_out, d.w_out, G.th,
                G.nblocks, lds);
#endif
    if (lds > 64 * 1024) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return GPI_ERR_LAUNCH;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, d, c, G);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

// Slab reduction: workgroup (item, weight chunk of <= 256, row chunk of RROWS).
// Thread (w, p) sums rows p, p + P, ... of its row chunk for weight w
// (coalesced: consecutive w read consecutive floats of a slab row), the P
// partials meet in LDS, one fp64 atomic per weight per workgroup.
#ifndef GPI_RROWS
#define GPI_RROWS 64
#endif
constexpr int RROWS = GPI_RROWS;

struct ReduceArgs {
    gpi_reduce_item it[GPI_MAX_REDUCE_ITEMS];
    int32_t first_block[GPI_MAX_REDUCE_ITEMS + 1];
    int32_t wchunks[GPI_MAX_REDUCE_ITEMS];
    int32_t n;
    int32_t rrows;       // slab rows per workgroup (RROWS, or fewer for a small call: see gpi_wgrad_reduce)
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
    const int r0 = rc * a.rrows, r1 = min(it.blocks, r0 + a.rrows);
    float s = 0.f;
    if (p < P) {
        // 16 slab loads in flight per thread (the reduction is latency-bound, not bandwidth-bound)
        const float* base = wpart + it.part_off + w0 + w;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        int r = r0 + p;
        for (; r + 15 * P < r1; r += 16 * P) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = base[(int64_t)(r + u * P) * it.row_stride];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc[u & 3] += v[u];
        }
        for (; r < r1; r += P) acc[0] += base[(int64_t)r * it.row_stride];
        s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    red[tid] = s;
    __syncthreads();
    if (tid < nw) {
        double t = 0.0;
        for (int q = 0; q < P; ++q) t += (double)red[q * nw + tid];
        atomicAdd(gacc + it.w_off + w0 + tid, t);
    }
}

// One thread per (BN layer, channel): the layer's codec calls in order.
__global__ __launch_bounds__(256) void bn_running_kernel(const gpi_bn_running_item* items, int n_items, int max_ch,
                                                         const gpi_stat* stats, int64_t n_stats, float momentum) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int li = t / max_ch, c = t - li * max_ch;
    if (li >= n_items) return;
    const gpi_bn_running_item it = items[li];
    if (c >= it.channels) return;
    double rm = it.running_mean[c], rv = it.running_var[c];
    for (int k = 0; k < it.n_calls; ++k) {
        double s = 0.0, s2 = 0.0;
        for (int r = 0; r < GPI_REPLICAS; ++r) {
            const gpi_stat& st = stats[((int64_t)r * GPI_MAX_GROUPS + it.group[k]) * n_stats + it.stat + c];
            s += st.sum;
            s2 += st.sumsq;
        }
        const double n = it.count[k];
        const double mean = s / n;
        double var = s2 / n - mean * mean;
        if (var < 0.0) var = 0.0;
        rm = (1.0 - momentum) * rm + momentum * mean;
        rv = (1.0 - momentum) * rv + momentum * (n > 1.0 ? var * n / (n - 1.0) : var);
    }
    it.running_mean[c] = (float)rm;
    it.running_var[c] = (float)rv;
    if (c == 0) *it.num_batches_tracked += it.n_calls;
}

#endif  // GPI_CONV_SHAPE_PART == 0
}  // namespace

#if GPI_CONV_SHAPE_PART == 0
extern "C" int gpi_bn_running_update(const gpi_bn_running_item* items, int n_items, int max_channels,
                                     const gpi_stat* stats, int64_t n_stats, float momentum, void* stream) {
    if (n_items < 0 || max_channels < 1 || (n_items > 0 && (!items || !stats))) return GPI_ERR_ARG;
    if (n_items == 0) return GPI_OK;
    const int threads = n_items * max_channels;
    hipLaunchKernelGGL(bn_running_kernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream, items, n_items,
                       max_channels, stats, n_stats, momentum);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}

#ifdef GPI_PHASE_TIMING
// timing build only (not declared in gpi.h): copy the phase / real-time stamps out and clear them.
extern "C" int gpi_debug_phase_stamps(unsigned long long* phase, unsigned long long* rt) {
    static unsigned long long zeros[4096 * 16];
    if (hipMemcpyFromSymbol(phase, HIP_SYMBOL(g_phase), sizeof(zeros)) != hipSuccess) return GPI_ERR_LAUNCH;
    if (hipMemcpyFromSymbol(rt, HIP_SYMBOL(g_rt), sizeof(unsigned long long) * 4096 * 2) != hipSuccess)
        return GPI_ERR_LAUNCH;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), zeros, sizeof(zeros)) != hipSuccess) return GPI_ERR_LAUNCH;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rt), zeros, sizeof(unsigned long long) * 4096 * 2) != hipSuccess)
        return GPI_ERR_LAUNCH;
    return GPI_OK;
}
#endif

extern "C" int gpi_conv_blocks(const gpi_conv_desc* op, const gpi_groups* groups, int32_t* blocks) {
    if (!op || !groups || !blocks) return GPI_ERR_ARG;
    ConvGeom G;
    if (!conv_geom(*op, *groups, G, false)) return GPI_ERR_UNSUPPORTED;   // backward tiling
    // one slab row per wave, or per workgroup (vop ops; lsum: the rows summed in LDS)
    *blocks = G.nblocks * ((vop_op(*op) || lsum_op(*op, G) || vsum_op(*op, G)) ? 1 : SLAB_ROWS);
    return GPI_OK;
}

extern "C" int gpi_conv_launch_info(const gpi_conv_desc* op, const gpi_groups* groups, int fwd, int32_t* info) {
    if (!op || !groups || !info) return GPI_ERR_ARG;
    ConvGeom G;
    if (!conv_geom(*op, *groups, G, fwd != 0)) return GPI_ERR_UNSUPPORTED;
    const int cp = cp_of(*op);
    info[0] = G.th;
    info[1] = G.nblocks;
    info[2] = (int32_t)(fwd ? fwd_lds(*op, G, cp) : bwd_lds(*op, G));
    info[3] = cp;
    info[4] = G.npx;
    info[5] = G.P;
    info[6] = G.PG;
    return GPI_OK;
}

extern "C" int gpi_conv_shape_info(int64_t* info) {
    if (!info) return GPI_ERR_ARG;
    info[0] = kNumShapes;
    info[1] = g_shape_planned;
    info[2] = g_shape_matched;
    {
        std::lock_guard<std::mutex> lk(g_shapes_mu);
        info[3] = (int64_t)g_shapes_seen.size();
    }
    return GPI_OK;
}

extern "C" int gpi_conv_shape_plan(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, int fwd, int fuse) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, nullptr, fwd != 0, fuse != 0, nullptr, nullptr, true);
}

extern "C" int gpi_conv_shapes_dump(char* buf, int64_t len) {
    if (!buf || len <= 0) return GPI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_shapes_mu);
    std::string out = "#define GPI_CONV_SHAPE_COUNT " + std::to_string(g_shapes_seen.size()) + "\n#define GPI_CONV_SHAPE_LIST";
    for (const ShapeC& s : g_shapes_seen) {
        const int* f = reinterpret_cast<const int*>(&s);
        out += " \\\n    {";
        for (size_t i = 0; i < sizeof(ShapeC) / sizeof(int); ++i) out += (i ? "," : "") + std::to_string(f[i]);
        out += "},";
    }
    out += "\n";
    if ((int64_t)out.size() + 1 > len) return GPI_ERR_ARG;
    memcpy(buf, out.c_str(), out.size() + 1);
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

extern "C" int gpi_conv_loss_fused(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, (hipStream_t)stream, false, true);
}

extern "C" int gpi_conv_forward_sig(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, uint32_t* flag,
                                    const int64_t* epoch, void* stream) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, (hipStream_t)stream, true, false, flag, epoch);
}

extern "C" int gpi_conv_backward_sig(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, uint32_t* flag,
                                     const int64_t* epoch, void* stream) {
    if (!op || !ctx) return GPI_ERR_ARG;
    return launch(*op, *ctx, (hipStream_t)stream, false, false, flag, epoch);
}

extern "C" int gpi_codec_forward_sig(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, uint32_t* flag,
                                     const int64_t* epoch, void* stream) {
    if (!ops || !ctx || n_ops < 0) return GPI_ERR_ARG;
    for (int i = 0; i < n_ops; ++i) {
        int r = launch(ops[i], *ctx, (hipStream_t)stream, true, false, i == 0 ? flag : nullptr, epoch);
        if (r != GPI_OK) return r;
    }
    return GPI_OK;
}

extern "C" int gpi_codec_backward_sig(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, uint32_t* flag,
                                      const int64_t* epoch, void* stream) {
    if (!ops || !ctx || n_ops < 0) return GPI_ERR_ARG;
    for (int i = n_ops - 1; i >= 0; --i) {
        int r = launch(ops[i], *ctx, (hipStream_t)stream, false, false, i == n_ops - 1 ? flag : nullptr, epoch);
        if (r != GPI_OK) return r;
    }
    return GPI_OK;
}

extern "C" int gpi_codec_forward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream) {
    return gpi_codec_forward_sig(ops, n_ops, ctx, nullptr, nullptr, stream);
}

extern "C" int gpi_codec_backward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream) {
    return gpi_codec_backward_sig(ops, n_ops, ctx, nullptr, nullptr, stream);
}

extern "C" int gpi_wgrad_reduce(const gpi_reduce_item* items, int n_items, const float* wpart, double* gacc,
                                void* stream) {
    if (!items || n_items < 0 || n_items > GPI_MAX_REDUCE_ITEMS || !wpart || !gacc) return GPI_ERR_ARG;
    for (int k = 0; k < n_items; ++k)
        if (items[k].row_stride < items[k].numel || items[k].numel <= 0) return GPI_ERR_ARG;
    if (n_items == 0) return GPI_OK;
    ReduceArgs a;
    a.n = n_items;
    // a call of few workgroups (the input conv's slabs alone, at the step's tail) takes fewer rows per
    // workgroup, so every thread's loads are ONE round trip: RROWS / 4 below 128 workgroups
    // (GPI_RROWS_SMALL overrides)
    static const int rr_small = env_int("GPI_RROWS_SMALL", RROWS / 4);
    for (int pass = 0; pass < 2; ++pass) {
        a.rrows = pass == 0 ? RROWS : std::max(1, rr_small);
        int nb = 0;
        for (int k = 0; k < n_items; ++k) {
            a.it[k] = items[k];
            a.first_block[k] = nb;
            a.wchunks[k] = (items[k].numel + 255) / 256;
            nb += a.wchunks[k] * ((items[k].blocks + a.rrows - 1) / a.rrows);
        }
        a.first_block[n_items] = nb;
        if (nb >= 128) break;
    }
    const int nb = a.first_block[n_items];
    hipLaunchKernelGGL(wgrad_reduce, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, wpart, gacc);
    GPI_CHECK_LAUNCH();
    return GPI_OK;
}
#endif  // GPI_CONV_SHAPE_PART == 0
