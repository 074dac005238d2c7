/*
 * gpi.h -- C ABI of libgpi_hip.so, the MI355X (gfx950) kernels behind the
 * physics-informed ELBO training step of pkmtum/generative-physics-informed-pde.
 *
 * The reference has no native layer of its own: its hot path is PyTorch
 * (cuDNN/cuBLAS/torch.solve) plus FEniCS assembly at setup.  These entry
 * points replace exactly the third-party kernels on that path
 * (SURVEY.md section 2.2); each one cites the reference code it stands in for.
 *
 * Conventions
 *   - The caller owns every buffer.  Device pointers / element offsets in,
 *     results out; the library never allocates and never synchronises the
 *     host, so every call is safe inside hipStreamBeginCapture.
 *   - Calls are stream-ordered on the hipStream_t passed as `stream`
 *     (NULL = the legacy default stream).
 *   - Every entry point returns int: GPI_OK (0) or a negative error code;
 *     nothing throws across the ABI.  gpi_error_string() names the code.
 *   - fp32 storage and arithmetic; statistics, loss sums and parameter
 *     gradients are accumulated in fp64.
 *   - Offsets in the descriptors are element offsets into the buffers named
 *     by the context (params / workspace / gradient accumulator).
 */
#ifndef GPI_H
#define GPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPI_OK 0
#define GPI_ERR_ARG (-1)
#define GPI_ERR_LAUNCH (-2)
#define GPI_ERR_UNSUPPORTED (-3)

#define GPI_MAX_GROUPS 4
#define GPI_MAX_CIN 32
#define GPI_MAX_COUT 8
#define GPI_MAX_REDUCE_ITEMS 48
#define GPI_MAX_GEMM_ITEMS 12
/* Cross-workgroup scalar sums (BN statistics, loss / ELBO terms) are spread
 * over GPI_REPLICAS copies indexed by workgroup % GPI_REPLICAS so that
 * thousands of workgroups never serialise on one fp64 atomic address; the
 * reader sums the replicas. */
#ifndef GPI_REPLICAS
#define GPI_REPLICAS 16
#endif
/* workgroups of the fused step epilogue + Adam launch (grid-stride): well under one resident round of
 * 256-thread workgroups on 256 CUs, so its cross-stream wait cannot starve the signalling stream */
#ifndef GPI_EPILOGUE_MAX_WG
#define GPI_EPILOGUE_MAX_WG 512
#endif

/* Conv epilogues */
#define GPI_EPI_STORE 0        /* store raw output */
#define GPI_EPI_STORE_STATS 1  /* store raw output + per-channel fp64 sum / sum^2 (train-mode BN) */
#define GPI_EPI_GAUSS_LOSS 2   /* cout == 2: (mean, logsigma) -> Gaussian log-lik vs target, writes d(-elbo)/d(out) */
#define GPI_EPI_GAUSS_EXP_LOSS 3  /* as GAUSS_LOSS on the exponentiated field: N(exp(target); exp(mean), sigma^2)
                                     (generative.py:238-239, reconstruct_log_eff_property = False) */

/* Per-channel BatchNorm statistics record, one per (channel, group). */
typedef struct gpi_stat {
    double sum;     /* sum x           (forward)  */
    double sumsq;   /* sum x^2         (forward)  */
    double ssum;    /* sum S           (backward: S = sum_c gamma_c dL/d(bn_c)) */
    double sxsum;   /* sum S * xhat    (backward) */
} gpi_stat;

/* Samples of one codec call are split into BN-statistics groups: the
 * reference calls the decoder once per batch (unsupervised, supervised, ...)
 * and train-mode BatchNorm normalises each call with its own batch
 * statistics (bottleneck/codec.py:164-294; nothing calls .eval()).  One
 * launch here serves all groups. */
typedef struct gpi_groups {
    int32_t n_groups;
    int32_t start[GPI_MAX_GROUPS + 1];   /* group g = samples [start[g], start[g+1]) */
} gpi_groups;

/* One convolution of the DenseNet codec with its fused neighbours:
 *   out = conv(act(in)),  act = relu(batchnorm_train(.)) or identity,
 * nearest x2 upsampling folded into the addressing, dense-block concat
 * never materialised (channel offsets into a shared block buffer).
 * Replaces nn.Conv2d / nn.BatchNorm2d / ReLU / UpsamplingNearest2d /
 * torch.cat of bottleneck/codec.py:150-298, Encoder.py:151, Decoder.py:217. */
typedef struct gpi_conv_desc {
    int32_t cin, cout, k, stride, pad, upsample;
    int32_t h_in, w_in, h_out, w_out;
    /* input: raw (pre-BN) features; in_off < 0 selects ctx->ext_in */
    int64_t in_off;
    int32_t in_ctot, in_c0;
    int32_t in_bn;                 /* 1: relu(BN) applied on the fly */
    int32_t gin_accumulate;        /* backward: 0 overwrite gin, 1 add */
    int64_t gamma_off, beta_off;   /* param offsets of the input BN affine */
    int64_t in_stat;               /* stat index of input channel in_c0 */
    int64_t w_off;                 /* param offset, weight [cout][cin][k][k] */
    /* output */
    int64_t out_off;
    int32_t out_ctot, out_c0;
    int64_t out_stat;              /* stat index of output channel out_c0, or -1 */
    int32_t epilogue;              /* GPI_EPI_* */
    int32_t gout_mode;             /* backward: 0 = BN-backward of the S buffer, 1 = direct gradient */
    int64_t gout_off;              /* S buffer (mode 0) / gradient buffer (mode 1), output layout */
    int64_t gin_off;               /* S buffer / gradient of the input (input layout), or -1 */
    int64_t wpart_off;             /* partial slab, one row per workgroup:
                                      [cout*cin*k*k dW][cin dgamma][cin dbeta] (BN part only if in_bn) */
    int64_t drop_off;              /* Dropout2d after this conv (codec.py:177-178,218-282): workspace
                                      floats [B][cout], the per-(sample, channel) scale 0 or 1/(1-p)
                                      applied to the output (forward) and to its gradient
                                      (backward); -1: no dropout */
} gpi_conv_desc;

/* Per-call pointers shared by all codec operators. */
typedef struct gpi_codec_ctx {
    const float* params;           /* flat fp32 parameters */
    float* ws;                     /* workspace (activations, S / gradient buffers) */
    gpi_stat* stats;               /* BN statistics records [GPI_REPLICAS][GPI_MAX_GROUPS][stat] */
    double* gacc;                  /* fp64 gradient accumulator, parallel to params */
    float* wpart;                  /* weight-gradient partial slabs */
    const float* ext_in;           /* external input (e.g. the unlabeled image pool) */
    const int32_t* ext_idx;        /* row of ext_in for each sample (NULL: identity) */
    int64_t ext_stride;            /* floats per ext_in row */
    const float* tgt[GPI_MAX_GROUPS];      /* Gaussian-loss targets per group */
    const int32_t* tgt_idx[GPI_MAX_GROUPS];/* target row per sample of the group (NULL: identity) */
    float loss_scale[GPI_MAX_GROUPS];      /* d(-elbo)/d(logL): 1, or 1/batch when normalize */
    double* loss_acc;              /* [GPI_MAX_GROUPS][GPI_REPLICAS] Gaussian log-likelihood sums */
    int64_t n_stats;               /* stat records per replica */
    float bn_eps;                  /* 1e-5 (torch default) */
    gpi_groups groups;
} gpi_codec_ctx;

/* Slab reduction item: gacc[w_off + i] += sum_b wpart[part_off + b*row_stride + i], i < numel. */
typedef struct gpi_reduce_item {
    int64_t part_off, w_off;
    int32_t blocks, numel;
    int32_t row_stride, _pad;      /* floats between consecutive slab rows */
} gpi_reduce_item;

/* Dense (per-sample) part of the ELBO: encoder FC / ReLU / split heads
 * (Encoder.py:175-182, codec.py:495-504), reparametrisation
 * (bottleneck/utils.py:216-219, components.py:167-172), KL
 * (bottleneck/utils.py:246-248), the decoder latent map (Decoder.py:213),
 * and the effective-property map with its Gaussian log-likelihood
 * (components.py:201-256, generative.py:469-470).
 * Samples [0, n_enc) take the amortised-encoder path, samples
 * [n_enc, n_enc + n_q) the per-sample variational path (and
 * [n_enc + n_q, + n_q2) a second variational segment, see n_q2). */
#define GPI_HEAD_ENC      0x01  /* feat -> FC -> relu -> (mu, logsigma) for encoder samples */
#define GPI_HEAD_REPARAM  0x02  /* z = mu + exp(logsigma) eps, KL (encoder samples) */
#define GPI_HEAD_QZ       0x04  /* z from q_z params, KL (q samples) */
#define GPI_HEAD_LATENT   0x08  /* lat = latent_map(z) for all samples */
#define GPI_HEAD_GP       0x10  /* gp(z), X-sample from q_X, log-lik + entropy (q samples) */
#define GPI_HEAD_LOCKX    0x20  /* with GPI_HEAD_GP: X~ = gp(z) itself, no q_X / log-lik / entropy
                                 * (independent_X = False: _elbo_supervised_lockX generative.py:429-459,
                                 * _elbo_virtual_observables_lockX :300-339) */
/* launch subsets (gpi_head_backward): only the encoder samples / only the variational ones, so the
 * two halves can run on different streams (the variational half needs the ROM adjoint) */
#define GPI_HEAD_PART_ENC 0x100
#define GPI_HEAD_PART_Q   0x200
/* the per-sample VALU form of the dense layers instead of the batched MFMA form (A/B and parity tests;
 * the MFMA form is the default wherever its width / alignment preconditions hold) */
#define GPI_HEAD_VALU     0x400

typedef struct gpi_head_desc {
    int32_t flags;
    int32_t n_enc, n_q;
    int32_t d_feat, d_z, d_lat, d_x;
    int32_t _pad;
    /* parameter offsets (-1 if absent) */
    int64_t fc_w, fc_b, mu_w, mu_b, ls_w, ls_b;
    int64_t lat_w, lat_b;
    int64_t gp_w, gp_b, gp_ls;
    int64_t qz_mu, qz_ls, qx_mu, qx_ls;
    /* workspace offsets */
    int64_t feat, gfeat, hpre;       /* [n_enc, d_feat] */
    int64_t zmu, zls, eps_z, z, gz;  /* [n_enc + n_q, d_z] */
    int64_t lat, glat;               /* [n_enc + n_q, d_lat] */
    int64_t eps_x, xs, mux, gxs, gmux; /* [n_q, d_x] */
    int64_t dzmu, dzls;              /* [n_enc + n_q, d_z] backward deltas */
    int64_t dhpre;                   /* [n_enc, d_feat] backward delta */
    float kl_scale_enc, kl_scale_q, lx_scale, _fpad;
    /* fp64 term accumulators (terms[0..]): KL_enc, KL_q, logL_X, entropy */
    double* terms;                   /* [4][GPI_REPLICAS] */
    /* Second per-sample variational segment: samples [n_enc + n_q, n_enc + n_q + n_q2), e.g. the
     * virtual-observable term (generative.py:341-392) next to the supervised one, with its own
     * q_z / q_X rows, flags (GPI_HEAD_QZ [| GPI_HEAD_GP]; GP off = VO hold-off), scales and
     * term slots.  Workspace rows eps_x / xs / mux / gxs / gmux run over both segments. */
    int32_t n_q2, flags2;
    int64_t qz_mu2, qz_ls2, qx_mu2, qx_ls2;
    float kl_scale_q2, lx_scale2;
    double* terms2;                  /* [3][GPI_REPLICAS]: KL_q, logL_X, entropy of segment 2 */
} gpi_head_desc;

/* Batched outer-product GEMM for shared dense-layer gradients:
 *   gacc[c_off + m*N + n] += sum_s A[s*lda + m] * B[s*ldb + n]
 *   gacc[bias_off + m]    += sum_s A[s*lda + m]       (bias_off >= 0)   */
typedef struct gpi_gemm_item {
    int64_t a_off, b_off, c_off, bias_off;
    int32_t S, M, N, lda, ldb, flags;   /* flags bit 0: ReLU applied to B; bit 1 (item 0): the scalar
                                         * VALU tile form instead of MFMA (A/B and parity tests) */
} gpi_gemm_item;

/* Coarse-grained model (ROM) on the nc x nc "/" mesh: K(kappa) from the
 * closed-form 5-point stencil, Dirichlet nodes eliminated (the SPD interior
 * system equals ROM.py's row-replaced system), banded Cholesky per sample,
 * P1 prolongation to the fine free nodes, optional fused Gaussian
 * log-likelihood and its adjoint.
 * Replaces ROM.__call__/GetStiffness/_solve_eqs (bottleneck/ROM.py:59-100),
 * ReducedOrderModelOperator.forward (components.py:296-302) and
 * DiagonalGaussianLogLikelihood(Y, mu_y, 2 logsigma_y) (generative.py:473). */
#define GPI_ROM_FORWARD 0   /* mu_y = W solve(K(exp(x)+1e-8), F) */
#define GPI_ROM_LOGLIK  1   /* forward + log-lik + backward to x and logsigma_y */
#define GPI_ROM_BACKWARD 2  /* given d(mu_y): backward to x */

typedef struct gpi_rom_desc {
    int32_t nc, refine, n, mode;
    int32_t input_kappa;       /* 1: x holds kappa itself (ROM.__call__), 0: log effective property */
    int32_t x_draw;            /* 1: x is drawn here, x = x_mu + exp(x_ls) x_eps element-wise (the q_X sample of
                                  components.py:167-172, the same fmaf as the head's), rows at x_stride */
    const float* x;            /* [n, 2 nc^2] log effective property */
    int64_t x_stride;
    const float* F;            /* [n, (nc+1)^2] F_ROM_BC */
    float* mu_y;               /* [n, d_y] out (optional) */
    const float* Y;            /* [n, d_y] targets (LOGLIK) */
    const float* logsig_y;     /* [d_y] (LOGLIK) */
    float loss_scale;          /* d(-elbo)/d(logL_y) */
    int32_t gx_accumulate;
    const float* dmu;          /* [n, d_y] upstream gradient (BACKWARD), or NULL */
    const float* duc;          /* [n, (nc+1)^2] upstream gradient w.r.t. the coarse solution (BACKWARD), or NULL */
    float* gx;                 /* [n, 2 nc^2] d/dx out */
    int64_t gx_stride;
    double* gacc_logsig;       /* fp64 accumulator for d/d logsigma_y (LOGLIK) */
    double* loss_acc;          /* [GPI_REPLICAS] sum log-lik (LOGLIK) */
    int32_t* flag;             /* set to 1 if any kappa <= 1e-12 (ROM.py:74-76), checked lazily */
    float* uc;                 /* optional [n, (nc+1)^2] coarse solution */
    float* gls_part;           /* optional [n, d_y] (LOGLIK): per-sample d/d logsigma_y contributions written with
                                  plain stores instead of the fp64 atomics into gacc_logsig (32 x 4095 same-address
                                  atomics per C64 step); the caller reduces the n rows (gpi_wgrad_reduce item) */
    const float* x_mu;         /* x_draw: [n, 2 nc^2] q_X means, log-sigmas and noise */
    const float* x_ls;
    const float* x_eps;
} gpi_rom_desc;

/* Coarse-grained residual on the fine grid (VirtualObservables CGR query,
 * VirtualObservables.py:57-69,297-321 + physics/LinearElliptic.py:137-159):
 *   r = W^T [K_f(kappa) yhat]_free  (= Gamma y - alpha),
 * kappa = exp(logkappa image) per pixel, yhat = y on free nodes and the NDP
 * Dirichlet data u0..u3 on x=0 / x=1.  Matrix-free 5-point stencil, flux rows (r_flux) in the
 * same pass; any n_fine <= 512 with n_fine % nc == 0 (GPI_ERR_UNSUPPORTED above). */
/* kernel form of gpi_cgr_residual (gpi_residual_desc.form; every form computes the same residual):
 * AUTO the first that applies of BAND (cgr_band_kernel: one wave per coarse row band, no barrier; nc <= 8 and
 * r in {4, 8, 16, 32} at n_fine / 64 columns per lane in {1, 2, 4}), STREAM (cgr_stream_kernel: 16-row chunks
 * through LDS rings; 16-byte aligned fields, n_fine a multiple of 16 up to 256, r a power of two >= 4) and
 * GENERAL (cgr_kernel: any grid); an explicit form that does not apply returns GPI_ERR_UNSUPPORTED. */
#define GPI_CGR_AUTO    0
#define GPI_CGR_BAND    1
#define GPI_CGR_STREAM  2
#define GPI_CGR_GENERAL 3

typedef struct gpi_residual_desc {
    int32_t n_fine, nc, n, form;
    const float* logkappa;     /* [n, n_fine, n_fine] image (row 0 = top) */
    const float* y;            /* [n, d_y] fine free values */
    const float* bc;           /* [n, 4] u0..u3 */
    float* r;                  /* [n, (nc+1)^2] CGR residual */
    float* r_flux;             /* [n, 2 nc^2] flux residual Gamma_fc y (alpha_fc = 0), or NULL;
                                  bottleneck/flux.py:81-158, rows as GPI_VO_FLUX */
} gpi_residual_desc;

/* ------------------------------------------------------------------------
 * Virtual observables (bottleneck/VirtualObservables.py).
 *
 * Query rows of one VO sample (LinearQuerry.Gamma / .alpha, fp64 as the
 * reference asserts at VirtualObservables.py:396-407), rows in the order the
 * reference concatenates its samplers (QuerryEnsemble.FromQuerryPointEnsemble,
 * VirtualObservables.py:519-539):
 *   GPI_VO_CGR   (nc+1)^2 rows: CoarseGrainedResidualSampler, Gamma = W^T K_ff,
 *                alpha = W^T f_eff (VirtualObservables.py:57-69,297-321);
 *   GPI_VO_FLUX  2 nc^2 rows: FluxConstrainSampler / FluxConstraintReducedOrderModel,
 *                Gamma[k, free i] = d/du_i of the outward flux of kappa grad u over the
 *                boundary of coarse triangle k (top/bottom domain edges excluded),
 *                alpha = 0 (bottleneck/flux.py:81-158, incl. the alpha quirk at :153).
 * Conductivity per DG0 cell of the fine mesh (QuerryPoint.x = X_DG, cell 2q the
 * lower-right and 2q+1 the upper-left triangle of fine square q = i + n j). */
#define GPI_VO_CGR  0x1
#define GPI_VO_FLUX 0x2

typedef struct gpi_vo_query_desc {
    int32_t n_fine, nc, n, flags;
    const double* logkappa;    /* [n, 2 n_fine^2] log conductivity per DG0 cell (X_DG) */
    const double* bc;          /* [n, 4] NDP boundary values u0..u3 */
    double* gamma;             /* [n, m, d_y] out (every entry written), m = gpi_vo_rows(...) */
    double* alpha;             /* [n, m] out */
} gpi_vo_query_desc;

/* Galerkin query rows from test functions V on the fine free nodes
 * (QuerryPoint.construct_querry_weak_galerkin, VirtualObservables.py:61-69):
 *   Gamma[row0 + a] = V_a^T K_ff  (= K_ff V_a, K symmetric),  alpha[row0 + a] = V_a^T f_eff,
 * with V given, or drawn per (sample, a) as
 *   GPI_VO_TEST_GAUSS  V ~ N(0, 1) i.i.d.       (GaussianSketchingSampler, :230-258)
 *   GPI_VO_TEST_RBF    V_j = exp(-|x_j - r0|^2 / l^2), r0 ~ U(0,1)^2 per row
 *                      (RadialBasisFunctionSampler + fawkes FastRadialBasisFunction, :172-228)
 * from Philox (counter *offset + ((sample * m_aux + a) * d_y + j), stream sub) or `centers`. */
#define GPI_VO_TEST_GAUSS 0
#define GPI_VO_TEST_RBF   1

typedef struct gpi_vo_galerkin_desc {
    int32_t n_fine, n, m_aux, kind;
    const double* logkappa;    /* [n, 2 n_fine^2] */
    const double* bc;          /* [n, 4] */
    const double* V;           /* optional [n, m_aux, d_y] test functions */
    const double* centers;     /* optional [n, m_aux, 2] RBF centres */
    double length;             /* RBF length scale l */
    uint64_t seed;
    const uint64_t* offset;
    uint64_t sub;
    double* gamma;             /* [n, m, d_y]: rows row0 .. row0 + m_aux - 1 written */
    double* alpha;             /* [n, m] */
    int32_t m, row0;
} gpi_vo_galerkin_desc;

/* MC predictive moments of the ROM (GenerativeModel.update_virtual_observables,
 * generative.py:198-207): for VO sample j and its n_mc coarse solutions u_s
 * (gpi_rom FORWARD with uc), y_s = W u_s + exp(logsig_y) eps_s
 * (ReducedOrderModelOperator.propagate_samples, components.py:304-311);
 * mean = torch.mean(y_s), std = torch.std(y_s) (unbiased), prec = 1 / std^2 (fp32). */
typedef struct gpi_vo_moments_desc {
    int32_t nc, refine, n, n_mc;
    const float* uc;           /* [n * n_mc, (nc+1)^2] */
    const float* logsig_y;     /* [d_y] or NULL (no observation noise) */
    const float* eps;          /* optional injected noise [n * n_mc, d_y]; NULL: device Philox */
    uint64_t seed;
    const uint64_t* offset;    /* device Philox offset (may be NULL = 0) */
    uint64_t sub;
    float* mean;               /* [n, d_y] out */
    float* std;                /* [n, d_y] out (optional) */
    float* prec;               /* [n, d_y] out (optional) */
} gpi_vo_moments_desc;

/* Column-sparse view of Gamma [n, m, d_y] (optional, for gpi_vo_condition / gpi_vo_precision).
 * The CGR and flux rows (VirtualObservables.py:297-321, flux.py:81-158) give every column i (a fine
 * node) <= ~11 nonzero rows, the same rows in every sample; with this view Lambda, Gamma g - alpha,
 * the column posteriors and the precision terms cost O(nnz) instead of O(m d_y) (the dense path reads
 * all of Gamma, 0.9 GB at 64^2 x 128 VO samples, in each of them).  Built once per Gamma:
 * gpi_vo_pattern (rows / counts), the caller's index lists (gpi/vo.py SparsePlan), then
 * gpi_vo_sparse_values.  Empty slots: rows = -1, vals = 0. */
typedef struct gpi_vo_sparse {
    int32_t r;                 /* slots per column */
    int32_t n_pairs;           /* Lambda entries (a >= b) that receive a contribution (all diagonals included) */
    const int32_t* rows;       /* [d_y, r] row of slot s of column i, ascending, -1 = empty */
    const double* vals;        /* [n, d_y, r] Gamma[j, rows[i, s], i] */
    const int32_t* pair_ptr;   /* [n_pairs + 1] contribution ranges */
    const int32_t* pair_ab;    /* [n_pairs] a * m + b, a >= b */
    const int32_t* pair_src;   /* [pair_ptr[n_pairs]] (i * r + s) * r + t: column i, slots s >= t */
    const int32_t* row_ptr;    /* [m + 1] */
    const int32_t* row_src;    /* [row_ptr[m]] i * r + s: the nonzeros of row a, ascending i */
    double* inv;               /* workspace [n, m, m]: Lambda^{-1} (gpi_vo_condition only) */
} gpi_vo_sparse;

/* Gaussian conditioning of every VO sample (VirtualObservable.update,
 * VirtualObservables.py:642-669): prior N(g, diag(1/prec)), observation
 * Gamma y = alpha + N(0, diag(vo_var)):
 *   Lambda = Gamma C Gamma^T + diag(vo_var), L = chol(Lambda),
 *   mean = g - C Gamma^T Lambda^{-1} (Gamma g - alpha),
 *   vars = diag(C) - diag(C)^2 |L^{-1} Gamma_i|^2   (= cov - postcov_diag_subtractor).
 * fp64 throughout (prior casts as the reference: g, prec -> double). */
typedef struct gpi_vo_condition_desc {
    int32_t n, m, d_y, _pad;
    const double* gamma;       /* [n, m, d_y] */
    const double* alpha;       /* [n, m] */
    const float* g;            /* [n, d_y] prior mean */
    const float* prec;         /* [n, d_y] prior precision */
    const double* vo_var;      /* [m] */
    double* lam;               /* workspace [n, m, m] (L in the lower triangle, L^-T above it on return) */
    double* solvec;            /* workspace [n, m] */
    double* mean;              /* [n, d_y] out */
    double* vars;              /* [n, d_y] out */
    float* mean32;             /* optional [n, d_y] out: (float) mean  (ensemble .mean, model dtype) */
    float* logsig32;           /* optional [n, d_y] out: 0.5 log((float) vars)  (ensemble .logsigma) */
    int32_t* flag;             /* optional: set to 1 if a Lambda is not positive definite
                                  (torch.cholesky raises there; checked lazily by the caller) */
    const gpi_vo_sparse* sparse; /* optional column-sparse view of gamma (then gamma itself is not read) */
} gpi_vo_condition_desc;

/* VO precision update (VirtualObservablesEnsemble.update_vo_precision,
 * VirtualObservables.py:971-998 + _get_mean_vo_variances :960-964):
 *   beta = 0.5 sum_j [(Gamma_j mean_j - alpha_j)^2 + Gamma_j^2 vars_j] + beta0,
 *   vo_var = beta / (0.5 n + alpha0 + 1), 0 on rows with infinite precision. */
typedef struct gpi_vo_precision_desc {
    int32_t n, m, d_y, _pad;
    const double* gamma;       /* [n, m, d_y] */
    const double* alpha;       /* [n, m] */
    const double* mean;        /* [n, d_y] */
    const double* vars;        /* [n, d_y] */
    const int32_t* infinite;   /* [m] 1 = infinite precision row */
    double alpha0, beta0;
    double* beta;              /* [m] out (prec_beta) */
    double* vo_var;            /* [m] out (mean VO variances) */
    double* terms;             /* [m, n] workspace: per-(row, VO sample) terms, summed over samples in a
                                  fixed order (bitwise reproducible beta / vo_var) */
    const gpi_vo_sparse* sparse; /* optional column-sparse view of gamma (then gamma itself is not read) */
} gpi_vo_precision_desc;

/* Predictive effective properties (Analysis.sample_predictive_y's first two stages,
 * components.py:472-478 + EffectivePropertyMap.propagate_samples :238-249): for row r,
 * j = r / rep,  z = qz_mu[j] + exp(qz_ls[j]) eps_z,  x = gp_w z + gp_b (+ exp(gp_ls) eps_x when
 * gp_ls != NULL, independent_X).  Normals from Philox (counter *offset + r * dim + t; streams
 * sub, sub + 1) unless eps_z / eps_x are given.  Parameters are plain device pointers. */
typedef struct gpi_gp_sample_desc {
    int32_t rows, rep, d_z, d_x;
    const float* qz_mu;        /* [rows / rep, d_z] */
    const float* qz_ls;
    const float* gp_w;         /* [d_x, d_z] */
    const float* gp_b;         /* [d_x] */
    const float* gp_ls;        /* [d_x] or NULL */
    const float* eps_z;        /* optional [rows, d_z] */
    const float* eps_x;        /* optional [rows, d_x] */
    uint64_t seed;
    const uint64_t* offset;
    uint64_t sub;
    float* x;                  /* [rows, d_x] out */
} gpi_gp_sample_desc;

/* Predictive scores of Analysis.eval_all_y (components.py:493-524): per sample n
 *   relerr_n   = |mean_n - Y_n| / |Y_n|                             (bottleneck/utils.py relative_error)
 *   logscore_n = mean_p [-log std - (Y - mean)^2 / (2 std^2) - log(2 pi) / 2]
 * and per output p (lamp/utils.py:5-20, global_average = False)
 *   r2_p = 1 - sum_n (Y - mean)^2 / sum_n (Y - Ybar_p)^2.
 * out[0] = sum_n relerr_n, out[1] = sum_n logscore_n, out[2] = sum_p r2_p (fp64; caller divides). */
int gpi_predictive_scores(const float* Y, const float* mean, const float* std, int32_t n, int32_t d_y,
                          double* out, void* stream);

/* Flat Adam (torch.optim.Adam semantics, no weight decay / amsgrad),
 * training.py:254,417.  step and lr are read from device memory so the
 * update can be replayed from a captured graph. */
typedef struct gpi_adam_desc {
    float* p; const float* g; float* m; float* v;
    int64_t n;
    const float* lr;           /* device scalar */
    const int64_t* step;       /* device scalar: step number after increment */
    float beta1, beta2, eps, _pad;
    uint64_t* rng_offset;      /* optional: device RNG offset advanced by rng_advance after the update */
    uint64_t rng_advance;      /*           (replaces a separate gpi_rng_advance launch) */
    /* optional: a cross-stream wait's error word (gpi_stream_wait / the fused epilogue's wait_err).  While
     * it is non-zero the update leaves p, m and v untouched (a timed-out hand-off means the gradient may be
     * incomplete; the word is sticky, the host raises on it); counters and the RNG offset still advance. */
    uint32_t* wait_err;
    /* optional (data-parallel steps): the all-reduced error slot of gpi_step_epilogue_desc.err_slot; non-zero
     * -> some rank's hand-off timed out: this rank skips the update too and sets its own *wait_err, so every
     * rank keeps identical parameters and raises. */
    const float* skip_if;
} gpi_adam_desc;

/* ---------------------------------------------------------------- API */
int gpi_version(void);
/* GPI_REPLICAS of this build (bindings size their statistics / term buffers by it). */
int gpi_replicas(void);
/* sha1 (40 hex digits) of the sources this library was built from: the csrc .hip files in name order, then
 * csrc/common.h and include/gpi.h, concatenated (bindings refuse a library older than its sources). */
const char* gpi_source_sha(void);
/* sizeof of every struct above, in declaration order (ABI self-check); returns the count. */
int gpi_struct_sizes(int64_t* out, int n);
const char* gpi_error_string(int code);

/* BatchNorm2d running statistics (train mode, codec.py BatchNorm2d layers, momentum 0.1): for every
 * item (one BN layer: `channels` stat records from `stat`), and for each of its codec calls in call
 * order (group g[k], element count count[k] = samples * H * W):
 *   running_mean = (1 - m) running_mean + m mean,  running_var = (1 - m) running_var + m var * n / (n - 1),
 *   num_batches_tracked += n_calls
 * from the fp64 batch sums the forward kernels accumulated (before the step epilogue clears them). */
typedef struct gpi_bn_running_item {
    int64_t stat;
    int32_t channels, n_calls;
    int32_t group[GPI_MAX_GROUPS];
    double count[GPI_MAX_GROUPS];
    float* running_mean;
    float* running_var;
    int64_t* num_batches_tracked;
} gpi_bn_running_item;
/* items: device array of n_items records (persistent, graph-capture safe). */
int gpi_bn_running_update(const gpi_bn_running_item* items, int n_items, int max_channels, const gpi_stat* stats,
                          int64_t n_stats, float momentum, void* stream);

/* SyncBN exchange of one BN seam (the fp64 BN sums of stat slots [stat0, stat0 + n), fields f0 and f0 + 1, of
 * every BN group; ElboEngine.set_sync_bn, codec.py:164-173 at the union batch).  One 64-thread launch:
 *   GPI_BNX_FOLD    msg[g][c][f] = the GPI_REPLICAS copies summed in replica order (the caller all-reduces msg,
 *                   e.g. over RCCL, then runs UNFOLD);
 *   GPI_BNX_UNFOLD  replica 0 = msg * scale[g], the other replicas 0;
 *   GPI_BNX_PEER    the one-shot peer all-reduce: FOLD into this rank's exchange buffer (slot seq & 1 of its two
 *                   message slots), publish seq in its flag word, wait for every rank's flag to reach seq, sum
 *                   the ranks' messages in rank order from their buffers (IPC-mapped: gpi_peer_alloc /
 *                   gpi_peer_open), then UNFOLD -- no collective library, no host, graph-capturable.  *seq is
 *                   this rank's exchange counter (every rank runs the same sequence of exchanges); a wait of
 *                   more than ~10 s sets *err and the launch returns (the sums are then garbage, nothing hangs).
 * n <= 8 channels (GPI_MAX_COUT).  The sum over the ranks of FOLD messages in rank order equals the RCCL path's
 * for 2 ranks bit for bit (a + b), to rounding for more. */
#define GPI_MAX_RANKS 16
#define GPI_BNX_MSG 64            /* doubles per message: GPI_MAX_GROUPS x GPI_MAX_COUT x 2 */
#define GPI_BNX_FOLD   0
#define GPI_BNX_UNFOLD 1
#define GPI_BNX_PEER   2
typedef struct gpi_bn_exchange_desc {
    gpi_stat* stats;
    int64_t n_stats;
    int32_t stat0, n, f0, mode;
    const double* scale;               /* [GPI_MAX_GROUPS] n_rank / N_global per BN group */
    double* msg;                       /* FOLD / UNFOLD: [GPI_BNX_MSG] */
    int32_t rank, world;
    double* peer_buf[GPI_MAX_RANKS];   /* PEER: each rank's exchange buffer, [2][GPI_BNX_MSG] doubles */
    uint32_t* peer_flag[GPI_MAX_RANKS];/* PEER: each rank's flag word */
    uint32_t* seq;                     /* PEER: this rank's exchange counter (device) */
    uint32_t* err;                     /* PEER: wait timeout (sticky, like gpi_adam_desc.wait_err) */
} gpi_bn_exchange_desc;
int gpi_bn_exchange(const gpi_bn_exchange_desc* d, void* stream);
/* Exchange buffers shared between the ranks' processes: gpi_peer_alloc allocates `bytes` of device memory (zeroed)
 * and writes its IPC handle (64 bytes) to ipc_handle; gpi_peer_open maps another process's buffer from its handle;
 * gpi_peer_close frees (own != 0) or unmaps it. */
int gpi_peer_alloc(int64_t bytes, void** ptr, void* ipc_handle);
int gpi_peer_open(const void* ipc_handle, void** ptr);
int gpi_peer_close(void* ptr, int own);

/* Partial-slab rows a conv backward launch writes: 4 per workgroup (one per wave). */
int gpi_conv_blocks(const gpi_conv_desc* op, const gpi_groups* groups, int32_t* blocks);
/* Launch geometry of one conv pass (fwd != 0: forward) for tuning / profiling tools:
 * info[0] output rows per tile, info[1] workgroups, info[2] LDS bytes per workgroup,
 * info[3] output channels per forward thread, info[4] adjacent output pixels per forward thread
 * (1 for the backward), info[5] / info[6] LDS row pitch (floats) of the input / output-gradient
 * images.  info holds >= 7 entries.  No device work. */
int gpi_conv_launch_info(const gpi_conv_desc* op, const gpi_groups* groups, int fwd, int32_t* info);
/* Compile-time conv shapes (csrc/conv_shapes.h): a launch whose shape -- kernel variant, batch-independent
 * descriptor fields, tile geometry -- equals a built-in entry runs an instantiation with those values as
 * constants (GPI_CONV_SHAPES=0: never).  info[0] built-in entries, info[1] conv launches planned since
 * load, info[2] of them on a built-in shape, info[3] distinct shapes recorded (GPI_CONV_SHAPES_RECORD=1).
 * gpi_conv_shapes_dump writes the recorded shapes as the text of conv_shapes.h (tools/gen_conv_shapes.py);
 * GPI_ERR_ARG when len is too small.  No device work. */
int gpi_conv_shape_info(int64_t* info);
/* Plan one conv launch (fwd / fuse as gpi_conv_forward / _backward / _loss_fused) and record its shape
 * without any device call (host-side shape generation). */
int gpi_conv_shape_plan(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, int fwd, int fuse);
int gpi_conv_shapes_dump(char* buf, int64_t len);
int gpi_conv_forward(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream);
int gpi_conv_backward(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream);
/* Forward AND backward of the decoder's output conv (Decoder.py:288-305 last_decoding conv3, 5x5,
 * cout = 2) with its Gaussian-loss epilogue (generative.py:232-239, bottleneck/utils.py:231-243) in one
 * launch: adds the log-likelihood to ctx->loss_acc and writes the weight-gradient slab rows and the
 * input's S / BN-backward sums exactly as gpi_conv_forward followed by gpi_conv_backward would (the
 * output gradient never leaves LDS).  op: k = 5, stride 1, no upsampling, cin <= 4, cout = 2,
 * epilogue GPI_EPI_GAUSS_LOSS / GPI_EPI_GAUSS_EXP_LOSS, gout_mode 1, no dropout; out_off is ignored. */
int gpi_conv_loss_fused(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, void* stream);
/* Run a codec program: ops in order (forward) / reverse order (backward). */
int gpi_codec_forward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream);
int gpi_codec_backward(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, void* stream);
/* The same launches with a cross-stream hand-off signal folded into the FIRST kernel launched (ops[0]
 * forward, ops[n_ops-1] backward): its workgroup 0 increments *flag at entry, which is what
 * gpi_stream_signal on this stream right before the call would do (see gpi_stream_wait), without a
 * launch of its own.  flag NULL: no signal (epoch: the wait's counter, checked non-NULL). */
int gpi_conv_forward_sig(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, uint32_t* flag, const int64_t* epoch,
                         void* stream);
int gpi_conv_backward_sig(const gpi_conv_desc* op, const gpi_codec_ctx* ctx, uint32_t* flag, const int64_t* epoch,
                          void* stream);
int gpi_codec_forward_sig(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, uint32_t* flag,
                          const int64_t* epoch, void* stream);
int gpi_codec_backward_sig(const gpi_conv_desc* ops, int n_ops, const gpi_codec_ctx* ctx, uint32_t* flag,
                           const int64_t* epoch, void* stream);
int gpi_wgrad_reduce(const gpi_reduce_item* items, int n_items, const float* wpart, double* gacc, void* stream);

int gpi_head_forward(const gpi_head_desc* d, const float* params, float* ws, void* stream);
int gpi_head_backward(const gpi_head_desc* d, const float* params, float* ws, double* gacc, void* stream);

int gpi_outer_gemm(const gpi_gemm_item* items, int n_items, const float* ws, double* gacc, void* stream);

int gpi_rom(const gpi_rom_desc* d, void* stream);
int gpi_cgr_residual(const gpi_residual_desc* d, void* stream);

/* Virtual observables: rows per VO sample for a flag set (or a negative error). */
int gpi_vo_rows(int32_t n_fine, int32_t nc, int32_t flags);
int gpi_vo_query(const gpi_vo_query_desc* d, void* stream);
int gpi_vo_galerkin(const gpi_vo_galerkin_desc* d, void* stream);
int gpi_vo_moments(const gpi_vo_moments_desc* d, void* stream);
int gpi_vo_condition(const gpi_vo_condition_desc* d, void* stream);
/* Column pattern of gamma [n, m, d_y]: rows[i, s] = the s-th row a (ascending) with gamma[j, a, i] != 0
 * for some j (s < r; -1 beyond), count[i] = the number of such rows (may exceed r: the caller then
 * keeps the dense path).  work: [m, d_y] bytes. */
int gpi_vo_pattern(const double* gamma, int32_t n, int32_t m, int32_t d_y, int32_t r, int32_t* rows, int32_t* count,
                   uint8_t* work, void* stream);
/* sp->vals[j, i, s] = gamma[j, sp->rows[i, s], i] (0 on empty slots); only sp->r, rows, vals are used. */
int gpi_vo_sparse_values(const double* gamma, int32_t n, int32_t m, int32_t d_y, const gpi_vo_sparse* sp,
                         void* stream);
int gpi_vo_precision(const gpi_vo_precision_desc* d, void* stream);
/* Reparametrised Gaussian rows (bottleneck/utils.py:216-219, components.py:174-180):
 * out[r, t] = mean[r / rep, t] + exp(logsigma[r / rep, t]) * N(0,1), normals from
 * Philox counter (*offset + r * dim + t) in stream `sub` (or eps[r, t] if eps != NULL). */
int gpi_gp_sample(const gpi_gp_sample_desc* d, void* stream);
int gpi_gauss_sample(float* out, const float* mean, const float* logsigma, int64_t rows, int32_t dim, int32_t rep,
                     const float* eps, uint64_t seed, const uint64_t* offset, uint64_t sub, void* stream);

/* Gradient finalisation: grad[i] = (accumulate ? grad[i] : 0) + (float) gacc[i];
 * also increments the device step counter (if non-NULL) for gpi_adam. */
#define GPI_FINALIZE_ACCUMULATE 1   /* grad += gacc (torch .grad accumulation) instead of grad = gacc */
#define GPI_FINALIZE_ZERO       2   /* zero gacc after reading it (the next step needs no separate fill) */
int gpi_grad_finalize(double* gacc, float* grad, int64_t n, int flags, int64_t* step, void* stream);

/* End-of-step epilogue of the fused training step (one launch instead of four): gradient
 * finalisation as gpi_grad_finalize, then the per-step scratch (BN statistics + ELBO term
 * accumulators) is zeroed for the next step after its first n_terms doubles were saved to
 * terms_dst (the value of the step just run), and the next step's random-subset indices
 * (drawn during this step's backward, off the critical path) are moved into place. */
typedef struct gpi_step_epilogue_desc {
    double* gacc;
    float* grad;
    int64_t n;
    int32_t flags;             /* GPI_FINALIZE_* */
    int32_t n_terms;
    int64_t* step;
    double* scratch;
    int64_t n_scratch;
    double* terms_dst;         /* [n_terms] */
    const int32_t* idx_src;
    int32_t* idx_dst;
    int64_t n_idx;
    /* optional Dropout2d draw folded into the epilogue (exactly gpi_dropout_masks(drop_out, drop_n,
     * drop_p, drop_seed, drop_offset, drop_sub)): the fused step draws the next step's encoder masks
     * here, after the encoder backward that reads the current ones, without a launch of its own */
    float* drop_out;
    int64_t drop_n;            /* 0: no draw */
    float drop_p;
    int32_t _pad2;
    uint64_t drop_seed;
    const uint64_t* drop_offset;
    uint64_t drop_sub;
    /* optional cross-stream wait folded into the epilogue (gpi_step_epilogue_adam only): every
     * workgroup waits until *wait_flag >= *step + 1 (the Adam step counter; see gpi_stream_wait) and
     * acquires before it reads the gradient accumulator -- the join with another stream's final
     * reductions without a wait launch; a timeout sets *wait_err, and while *wait_err is set the launch
     * skips the parameter / moment update (gpi_adam_desc.wait_err).  NULL: no wait.  The launch is a
     * grid-stride loop over at most GPI_EPILOGUE_MAX_WG workgroups, so the waiting workgroups never
     * hold every CU slot the signalling stream's remaining kernels need. */
    const uint32_t* wait_flag;
    uint32_t* wait_err;
    /* data-parallel steps (gpi_step_epilogue, before the gradient all-reduce): grad[err_slot] = 1 when
     * *wait_err is set -- a flat-buffer slot inside the all-reduced shared prefix that holds no parameter,
     * so after the SUM every rank sees whether ANY rank's hand-off timed out (gpi_adam_desc.skip_if).
     * -1: none. */
    int64_t err_slot;
} gpi_step_epilogue_desc;
int gpi_step_epilogue(const gpi_step_epilogue_desc* d, void* stream);
int gpi_adam(const gpi_adam_desc* d, void* stream);
/* gpi_step_epilogue followed by gpi_adam in ONE launch (single-process steps: nothing runs between the
 * gradient delivery and the update).  Requires d->flags == GPI_FINALIZE_ZERO, d->step == NULL (Adam's
 * a->step is the counter: read by every workgroup, incremented once), a->g == d->grad, a->n == d->n,
 * and a shared RNG offset (d->drop_offset == a->rng_offset when both are set).  done: a device
 * uint32 arrival counter, zero before the first call (the launch leaves it zero). */
int gpi_step_epilogue_adam(const gpi_step_epilogue_desc* d, const gpi_adam_desc* a, uint32_t* done, void* stream);

/* Cross-stream hand-off by a device counter instead of an event edge between two streams (in a captured
 * step each such edge costs the waiting hardware queue ~5 us of idle): gpi_stream_signal increments
 * *flag once every earlier kernel of its stream has completed; gpi_stream_wait, launched on another
 * stream, returns once *flag >= *epoch + 1, so the kernels after it see everything the signalling
 * stream wrote before the signal.  Protocol: one signal per flag per step, epoch = the step counter
 * (a device counter that advances only after the step's last hand-off), flags and counter saved /
 * restored together.  A wait that does not see its signal within ~1 s sets *err (if not NULL) and
 * returns.  Both are single-workgroup kernels; safe inside stream capture.  The *_sig launches below
 * fold the signal into a conv launch. */
int gpi_stream_signal(uint32_t* flag, const int64_t* epoch, void* stream);
int gpi_stream_wait(const uint32_t* flag, const int64_t* epoch, uint32_t* err, void* stream);
/* Waits until the device counter *a reaches *b (read once at entry): a stream's step gate on another
 * stream's step counter (the side stream of a step waits for the main stream's previous step to have
 * ended); timeout as gpi_stream_wait. */
int gpi_stream_wait_ge(const int64_t* a, const int64_t* b, uint32_t* err, void* stream);
/* The hand-offs need the waiting and the signalling stream on DIFFERENT hardware queues: on a shared queue
 * a wait enqueued ahead of its signal blocks the queue until it times out (HIP maps streams to its
 * GPU_MAX_HW_QUEUES queues round-robin, so a process with many streams shares them).  Probe of a stream
 * pair: launch gpi_queue_probe on stream A, then gpi_stream_signal(flag) on stream B; *seen = 1 iff the
 * signal arrived while the probe spun (~40 ms bound), i.e. B's kernels run past a spinning kernel of A.
 * *flag must be 0 before the pair is launched. */
int gpi_queue_probe(const uint32_t* flag, uint32_t* seen, void* stream);

/* Device Philox4x32-10 normals: out[i] = N(0,1) for counter (*offset + i);
 * offset is a device uint64 advanced by gpi_rng_advance (graph-replay safe). */
/* Several Philox draws of one step in ONE launch (the fused step's next-step draws on its side stream: the
 * decoder's Dropout2d scales, the random subset, the reparametrisation noise), each item bit-identical to its
 * own entry point's launch with the same seed / offset / sub: GPI_DRAW_RANDN = gpi_randn(out, n, ...),
 * GPI_DRAW_DROPOUT = gpi_dropout_masks(out, n, p, ...), GPI_DRAW_SUBSET = gpi_random_subset(out, n, k, ...)
 * (pool n <= 16384; at most one subset item).  Workgroups are dealt to the items by block ranges. */
#define GPI_MAX_DRAWS 6
#define GPI_DRAW_RANDN   0
#define GPI_DRAW_DROPOUT 1
#define GPI_DRAW_SUBSET  2
typedef struct gpi_draw_item {
    int32_t kind;
    float p;                   /* dropout probability (GPI_DRAW_DROPOUT) */
    void* out;                 /* float* (randn, dropout) or int32_t* (subset) */
    int64_t n;                 /* values (randn, dropout) or pool size (subset) */
    int64_t k;                 /* subset size */
    uint64_t sub;              /* Philox sub stream */
    uint64_t seed;             /* Philox key (the subset's: the seed shared by every rank) */
} gpi_draw_item;
int gpi_draws(const gpi_draw_item* items, int n_items, const uint64_t* offset, void* stream);
int gpi_randn(float* out, int64_t n, uint64_t seed, const uint64_t* offset, uint64_t sub, void* stream);
int gpi_rng_advance(uint64_t* offset, uint64_t by, void* stream);
/* Dropout2d channel scales (nn.Dropout2d train mode, codec.py:177-178): out[i] = 0 with
 * probability p, else 1/(1-p), for Philox counter (*offset + i/4); 0 <= p < 1. */
int gpi_dropout_masks(float* out, int64_t n, float p, uint64_t seed, const uint64_t* offset, uint64_t sub,
                      void* stream);
/* Uniform random subset (randperm(n)[:k] semantics, utils/data.py:444). */
int gpi_random_subset(int32_t* out, int32_t n, int32_t k, uint64_t seed, const uint64_t* offset, uint64_t sub, void* stream);
/* The same subset for ANY pool size n (torch.randperm(N)[:k] of utils/data.py:441-445 accepts any N;
 * gpi_random_subset keeps all n keys in one workgroup's LDS and refuses n > 16384): a 16-bit
 * histogram of the keys selects the candidates that can be among the first k, which are then ranked.
 * Bit-identical order to gpi_random_subset.  workspace: caller-owned device memory of at least
 * gpi_random_subset_workspace(n) bytes, 16-byte aligned (no state kept between calls). */
int gpi_random_subset_workspace(int32_t n, int64_t* bytes);
int gpi_random_subset_ws(int32_t* out, int32_t n, int32_t k, uint64_t seed, const uint64_t* offset, uint64_t sub,
                         void* workspace, int64_t ws_bytes, void* stream);

/* ---- FOM data generation (setup side; reference utils/data.py:72-103 DataLoader.assemble ->
 * physics/LinearElliptic.py:85-101 solve, one PETSc LU per sample).  Batched conjugate gradients on the
 * matrix-free 5-point stencil of the NDP problem, one workgroup per sample, fp64 throughout: preconditioned
 * by one geometric-multigrid V(1,1) cycle on power-of-two grids from GPI_FOM_MG_MIN (env, default 64; 0 off),
 * by Jacobi in the Chronopoulos-Gear form (one fused reduction per iteration) otherwise.  Stops at the same
 * recurrence-residual criterion either way. */
#define GPI_FOM_WARM 1   /* y holds the initial guess (default: linear interpolation of the BCs in x) */
typedef struct gpi_fom_desc {
    int32_t n_fine;            /* squares per side */
    int32_t n;                 /* samples */
    int32_t flags;             /* GPI_FOM_* */
    int32_t max_iter;
    const double* logkappa;    /* [n, 2 n_fine^2] DG0 log-conductivity (X_DG layout, cells 2q / 2q+1, q = i + n_fine j) */
    const double* bc;          /* [n, 4] NDP u0..u3 */
    double rtol;               /* stop at ||b - A y|| <= rtol ||b|| (recurrence residual) */
    double* y;                 /* [n, d_y] free-node solution */
    double* work;              /* [n, gpi_fom_workspace(n_fine)] caller-owned scratch */
    int32_t* iters;            /* [n] iterations used, or NULL */
    int32_t* flag;             /* [1] += samples not converged within max_iter, or NULL */
} gpi_fom_desc;
int64_t gpi_fom_workspace(int32_t n_fine);   /* doubles per sample */
int gpi_fom_solve(const gpi_fom_desc* d, void* stream);

/* Separable Gaussian random field (physics/RandomField.py:162-209 on the tensor grid of pixel
 * centres): the squared-exponential covariance is sigma^2 C_y (x) C_x, whose eigenpairs are products
 * of the 1-D ones, so the reference's KL sampler (eigh of the dense C + 1e-12 I, optional truncation)
 * is x[b] = mean + stddev * L_y (S o G_b) L_x^T with L = the 1-D eigenvectors and S[i,j] =
 * sqrt(sigma^2 lambda_i mu_j + 1e-12) on the retained modes, 0 elsewhere.  G_b ~ N(0, I) given, or
 * drawn with Philox(seed, counter b * ceil(py px / 4) + q, sub): 4 fp64 Box-Muller normals per counter. */
typedef struct gpi_random_field_desc {
    int32_t py, px;
    int32_t n;
    int32_t pad0;
    double mean, stddev;
    const double* ly;          /* [py, py] */
    const double* lxt;         /* [px, px] = L_x^T */
    const double* scale;       /* [py, px] S, or NULL (all ones) */
    const double* gamma;       /* [n, py, px] or NULL */
    uint64_t seed, sub;
    double* work;              /* [n, py, px] scratch ((S o G) L_x^T) */
    double* x;                 /* [n, py, px] */
} gpi_random_field_desc;
int gpi_random_field(const gpi_random_field_desc* d, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPI_H */
