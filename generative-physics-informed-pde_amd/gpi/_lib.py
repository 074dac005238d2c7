"""ctypes binding of libgpi_hip.so (include/gpi.h).

The library is loaded after ``torch`` so that both share torch's HIP runtime
(libamdhip64.so.7 is matched by soname).  There is no fallback: if the
library is missing, or a kernel is requested without a GPU, the call raises.
"""
import ctypes as C
import os

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libgpi_hip.so')
if os.environ.get('GPI_LIB_VARIANT'):               # tools: A/B builds of the same sources (libgpi_hip_<v>.so)
    LIB_PATH = os.path.join(HERE, 'libgpi_hip_%s.so' % os.environ['GPI_LIB_VARIANT'])
if os.environ.get('GPI_PHASE_TIMING') == '1':      # tools/phase_probe.py: the stamped build of the same kernels
    LIB_PATH = os.path.join(HERE, 'libgpi_hip_timing%s.so' % (
        ('_' + os.environ['GPI_LIB_VARIANT']) if os.environ.get('GPI_LIB_VARIANT') else ''))

GPI_MAX_GROUPS = 4
GPI_MAX_CIN = 32
GPI_MAX_COUT = 8
GPI_MAX_REDUCE_ITEMS = 48
GPI_MAX_GEMM_ITEMS = 12
# statistic / term replicas of the library build (16; a variant build's value by GPI_REPLICAS, checked at load)
GPI_REPLICAS = int(os.environ.get('GPI_REPLICAS', '16'))
FINALIZE_ACCUMULATE = 1
FINALIZE_ZERO = 2

EPI_STORE, EPI_STORE_STATS, EPI_GAUSS_LOSS, EPI_GAUSS_EXP_LOSS = 0, 1, 2, 3
HEAD_ENC, HEAD_REPARAM, HEAD_QZ, HEAD_LATENT, HEAD_GP, HEAD_LOCKX = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
HEAD_PART_ENC, HEAD_PART_Q, HEAD_VALU = 0x100, 0x200, 0x400
ROM_FORWARD, ROM_LOGLIK, ROM_BACKWARD = 0, 1, 2
VO_CGR, VO_FLUX = 0x1, 0x2
FOM_WARM = 1
VO_TEST_GAUSS, VO_TEST_RBF = 0, 1

i32, i64, f32, u64 = C.c_int32, C.c_int64, C.c_float, C.c_uint64
vp = C.c_void_p


class Stat(C.Structure):
    _fields_ = [('sum', C.c_double), ('sumsq', C.c_double), ('ssum', C.c_double), ('sxsum', C.c_double)]


class Groups(C.Structure):
    _fields_ = [('n_groups', i32), ('start', i32 * (GPI_MAX_GROUPS + 1))]


class ConvDesc(C.Structure):
    _fields_ = [('cin', i32), ('cout', i32), ('k', i32), ('stride', i32), ('pad', i32), ('upsample', i32),
                ('h_in', i32), ('w_in', i32), ('h_out', i32), ('w_out', i32),
                ('in_off', i64), ('in_ctot', i32), ('in_c0', i32), ('in_bn', i32), ('gin_accumulate', i32),
                ('gamma_off', i64), ('beta_off', i64), ('in_stat', i64), ('w_off', i64),
                ('out_off', i64), ('out_ctot', i32), ('out_c0', i32), ('out_stat', i64),
                ('epilogue', i32), ('gout_mode', i32), ('gout_off', i64), ('gin_off', i64), ('wpart_off', i64),
                ('drop_off', i64)]

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if 'drop_off' not in k:
            self.drop_off = -1


class BnRunningItem(C.Structure):
    _fields_ = [('stat', i64), ('channels', i32), ('n_calls', i32), ('group', i32 * GPI_MAX_GROUPS),
                ('count', C.c_double * GPI_MAX_GROUPS), ('running_mean', vp), ('running_var', vp),
                ('num_batches_tracked', vp)]


class CodecCtx(C.Structure):
    _fields_ = [('params', vp), ('ws', vp), ('stats', vp), ('gacc', vp), ('wpart', vp),
                ('ext_in', vp), ('ext_idx', vp), ('ext_stride', i64),
                ('tgt', vp * GPI_MAX_GROUPS), ('tgt_idx', vp * GPI_MAX_GROUPS),
                ('loss_scale', f32 * GPI_MAX_GROUPS), ('loss_acc', vp), ('n_stats', i64), ('bn_eps', f32),
                ('groups', Groups)]


class ReduceItem(C.Structure):
    _fields_ = [('part_off', i64), ('w_off', i64), ('blocks', i32), ('numel', i32), ('row_stride', i32),
                ('_pad', i32)]


class HeadDesc(C.Structure):
    _fields_ = [('flags', i32), ('n_enc', i32), ('n_q', i32), ('d_feat', i32), ('d_z', i32), ('d_lat', i32),
                ('d_x', i32), ('_pad', i32)] + \
               [(n, i64) for n in ('fc_w', 'fc_b', 'mu_w', 'mu_b', 'ls_w', 'ls_b', 'lat_w', 'lat_b', 'gp_w', 'gp_b',
                                   'gp_ls', 'qz_mu', 'qz_ls', 'qx_mu', 'qx_ls', 'feat', 'gfeat', 'hpre', 'zmu',
                                   'zls', 'eps_z', 'z', 'gz', 'lat', 'glat', 'eps_x', 'xs', 'mux', 'gxs', 'gmux',
                                   'dzmu', 'dzls', 'dhpre')] + \
               [('kl_scale_enc', f32), ('kl_scale_q', f32), ('lx_scale', f32), ('_fpad', f32), ('terms', vp),
                ('n_q2', i32), ('flags2', i32), ('qz_mu2', i64), ('qz_ls2', i64), ('qx_mu2', i64), ('qx_ls2', i64),
                ('kl_scale_q2', f32), ('lx_scale2', f32), ('terms2', vp)]


class GemmItem(C.Structure):
    _fields_ = [('a_off', i64), ('b_off', i64), ('c_off', i64), ('bias_off', i64),
                ('S', i32), ('M', i32), ('N', i32), ('lda', i32), ('ldb', i32), ('flags', i32)]


class RomDesc(C.Structure):
    _fields_ = [('nc', i32), ('refine', i32), ('n', i32), ('mode', i32), ('input_kappa', i32), ('x_draw', i32),
                ('x', vp), ('x_stride', i64), ('F', vp), ('mu_y', vp), ('Y', vp), ('logsig_y', vp),
                ('loss_scale', f32), ('gx_accumulate', i32), ('dmu', vp), ('duc', vp), ('gx', vp), ('gx_stride', i64),
                ('gacc_logsig', vp), ('loss_acc', vp), ('flag', vp), ('uc', vp), ('gls_part', vp),
                ('x_mu', vp), ('x_ls', vp), ('x_eps', vp)]


CGR_AUTO, CGR_BAND, CGR_STREAM, CGR_GENERAL = 0, 1, 2, 3


class ResidualDesc(C.Structure):
    _fields_ = [('n_fine', i32), ('nc', i32), ('n', i32), ('form', i32),
                ('logkappa', vp), ('y', vp), ('bc', vp), ('r', vp), ('r_flux', vp)]


class AdamDesc(C.Structure):
    _fields_ = [('p', vp), ('g', vp), ('m', vp), ('v', vp), ('n', i64), ('lr', vp), ('step', vp),
                ('beta1', f32), ('beta2', f32), ('eps', f32), ('_pad', f32), ('rng_offset', vp),
                ('rng_advance', C.c_uint64), ('wait_err', vp), ('skip_if', vp)]


class VoQueryDesc(C.Structure):
    _fields_ = [('n_fine', i32), ('nc', i32), ('n', i32), ('flags', i32),
                ('logkappa', vp), ('bc', vp), ('gamma', vp), ('alpha', vp)]


class VoMomentsDesc(C.Structure):
    _fields_ = [('nc', i32), ('refine', i32), ('n', i32), ('n_mc', i32),
                ('uc', vp), ('logsig_y', vp), ('eps', vp), ('seed', u64), ('offset', vp), ('sub', u64),
                ('mean', vp), ('std', vp), ('prec', vp)]


class VoConditionDesc(C.Structure):
    _fields_ = [('n', i32), ('m', i32), ('d_y', i32), ('_pad', i32),
                ('gamma', vp), ('alpha', vp), ('g', vp), ('prec', vp), ('vo_var', vp), ('lam', vp), ('solvec', vp),
                ('mean', vp), ('vars', vp), ('mean32', vp), ('logsig32', vp), ('flag', vp), ('sparse', vp)]


class VoPrecisionDesc(C.Structure):
    _fields_ = [('n', i32), ('m', i32), ('d_y', i32), ('_pad', i32),
                ('gamma', vp), ('alpha', vp), ('mean', vp), ('vars', vp), ('infinite', vp),
                ('alpha0', C.c_double), ('beta0', C.c_double), ('beta', vp), ('vo_var', vp), ('terms', vp),
                ('sparse', vp)]


class VoSparse(C.Structure):
    _fields_ = [('r', i32), ('n_pairs', i32), ('rows', vp), ('vals', vp), ('pair_ptr', vp), ('pair_ab', vp),
                ('pair_src', vp), ('row_ptr', vp), ('row_src', vp), ('inv', vp)]


class GpSampleDesc(C.Structure):
    _fields_ = [('rows', i32), ('rep', i32), ('d_z', i32), ('d_x', i32),
                ('qz_mu', vp), ('qz_ls', vp), ('gp_w', vp), ('gp_b', vp), ('gp_ls', vp), ('eps_z', vp), ('eps_x', vp),
                ('seed', u64), ('offset', vp), ('sub', u64), ('x', vp)]


class VoGalerkinDesc(C.Structure):
    _fields_ = [('n_fine', i32), ('n', i32), ('m_aux', i32), ('kind', i32),
                ('logkappa', vp), ('bc', vp), ('V', vp), ('centers', vp), ('length', C.c_double),
                ('seed', u64), ('offset', vp), ('sub', u64), ('gamma', vp), ('alpha', vp), ('m', i32), ('row0', i32)]


class StepEpilogueDesc(C.Structure):
    _fields_ = [('gacc', vp), ('grad', vp), ('n', i64), ('flags', i32), ('n_terms', i32), ('step', vp),
                ('scratch', vp), ('n_scratch', i64), ('terms_dst', vp), ('idx_src', vp), ('idx_dst', vp),
                ('n_idx', i64), ('drop_out', vp), ('drop_n', i64), ('drop_p', f32), ('_pad2', i32),
                ('drop_seed', u64), ('drop_offset', vp), ('drop_sub', u64), ('wait_flag', vp), ('wait_err', vp),
                ('err_slot', i64)]

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if 'err_slot' not in k:
            self.err_slot = -1


class FomDesc(C.Structure):
    _fields_ = [('n_fine', i32), ('n', i32), ('flags', i32), ('max_iter', i32), ('logkappa', vp), ('bc', vp),
                ('rtol', C.c_double), ('y', vp), ('work', vp), ('iters', vp), ('flag', vp)]


class RandomFieldDesc(C.Structure):
    _fields_ = [('py', i32), ('px', i32), ('n', i32), ('pad0', i32), ('mean', C.c_double), ('stddev', C.c_double),
                ('ly', vp), ('lxt', vp), ('scale', vp), ('gamma', vp), ('seed', u64), ('sub', u64), ('work', vp), ('x', vp)]


GPI_MAX_DRAWS = 6
DRAW_RANDN, DRAW_DROPOUT, DRAW_SUBSET = 0, 1, 2


class DrawItem(C.Structure):
    _fields_ = [('kind', i32), ('p', f32), ('out', vp), ('n', i64), ('k', i64), ('sub', u64), ('seed', u64)]


GPI_MAX_RANKS = 16
GPI_BNX_MSG = 64
BNX_FOLD, BNX_UNFOLD, BNX_PEER = 0, 1, 2


class BnExchangeDesc(C.Structure):
    _fields_ = [('stats', vp), ('n_stats', i64), ('stat0', i32), ('n', i32), ('f0', i32), ('mode', i32),
                ('scale', vp), ('msg', vp), ('rank', i32), ('world', i32),
                ('peer_buf', vp * GPI_MAX_RANKS), ('peer_flag', vp * GPI_MAX_RANKS), ('seq', vp), ('err', vp)]


STRUCTS = [Stat, Groups, ConvDesc, CodecCtx, ReduceItem, HeadDesc, GemmItem, RomDesc, ResidualDesc, AdamDesc,
           VoQueryDesc, VoMomentsDesc, VoConditionDesc, VoPrecisionDesc, GpSampleDesc,
           VoGalerkinDesc, StepEpilogueDesc, FomDesc, RandomFieldDesc, VoSparse, DrawItem, BnExchangeDesc]

# name -> (restype, argtypes)
SIGNATURES = {
    'gpi_version': (C.c_int, []),
    'gpi_replicas': (C.c_int, []),
    'gpi_source_sha': (C.c_char_p, []),
    'gpi_conv_shape_info': (C.c_int, [C.c_void_p]),
    'gpi_conv_shapes_dump': (C.c_int, [C.c_char_p, C.c_int64]),
    'gpi_conv_shape_plan': (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    'gpi_struct_sizes': (C.c_int, [C.POINTER(i64), C.c_int]),
    'gpi_error_string': (C.c_char_p, [C.c_int]),
    'gpi_conv_blocks': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(Groups), C.POINTER(i32)]),
    'gpi_bn_running_update': (C.c_int, [vp, C.c_int, C.c_int, vp, i64, f32, vp]),
    'gpi_conv_loss_fused': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(CodecCtx), vp]),
    'gpi_conv_launch_info': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(Groups), C.c_int, C.POINTER(i32)]),
    'gpi_conv_forward': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(CodecCtx), vp]),
    'gpi_conv_backward': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(CodecCtx), vp]),
    'gpi_codec_forward': (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.POINTER(CodecCtx), vp]),
    'gpi_codec_backward': (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.POINTER(CodecCtx), vp]),
    'gpi_conv_forward_sig': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(CodecCtx), vp, vp, vp]),
    'gpi_conv_backward_sig': (C.c_int, [C.POINTER(ConvDesc), C.POINTER(CodecCtx), vp, vp, vp]),
    'gpi_codec_forward_sig': (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.POINTER(CodecCtx), vp, vp, vp]),
    'gpi_codec_backward_sig': (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.POINTER(CodecCtx), vp, vp, vp]),
    'gpi_wgrad_reduce': (C.c_int, [C.POINTER(ReduceItem), C.c_int, vp, vp, vp]),
    'gpi_head_forward': (C.c_int, [C.POINTER(HeadDesc), vp, vp, vp]),
    'gpi_head_backward': (C.c_int, [C.POINTER(HeadDesc), vp, vp, vp, vp]),
    'gpi_outer_gemm': (C.c_int, [C.POINTER(GemmItem), C.c_int, vp, vp, vp]),
    'gpi_rom': (C.c_int, [C.POINTER(RomDesc), vp]),
    'gpi_cgr_residual': (C.c_int, [C.POINTER(ResidualDesc), vp]),
    'gpi_grad_finalize': (C.c_int, [vp, vp, i64, C.c_int, vp, vp]),
    'gpi_adam': (C.c_int, [C.POINTER(AdamDesc), vp]),
    'gpi_step_epilogue': (C.c_int, [C.POINTER(StepEpilogueDesc), vp]),
    'gpi_step_epilogue_adam': (C.c_int, [C.POINTER(StepEpilogueDesc), C.POINTER(AdamDesc), vp, vp]),
    'gpi_fom_workspace': (i64, [i32]),
    'gpi_fom_solve': (C.c_int, [C.POINTER(FomDesc), vp]),
    'gpi_random_field': (C.c_int, [C.POINTER(RandomFieldDesc), vp]),
    'gpi_randn': (C.c_int, [vp, i64, u64, vp, u64, vp]),
    'gpi_draws': (C.c_int, [vp, C.c_int, vp, vp]),
    'gpi_bn_exchange': (C.c_int, [C.POINTER(BnExchangeDesc), vp]),
    'gpi_peer_alloc': (C.c_int, [i64, C.POINTER(vp), vp]),
    'gpi_peer_open': (C.c_int, [vp, C.POINTER(vp)]),
    'gpi_peer_close': (C.c_int, [vp, C.c_int]),
    'gpi_dropout_masks': (C.c_int, [vp, i64, f32, u64, vp, u64, vp]),
    'gpi_rng_advance': (C.c_int, [vp, u64, vp]),
    'gpi_stream_signal': (C.c_int, [vp, vp, vp]),
    'gpi_stream_wait': (C.c_int, [vp, vp, vp, vp]),
    'gpi_stream_wait_ge': (C.c_int, [vp, vp, vp, vp]),
    'gpi_queue_probe': (C.c_int, [vp, vp, vp]),
    'gpi_random_subset': (C.c_int, [vp, i32, i32, u64, vp, u64, vp]),
    'gpi_random_subset_workspace': (C.c_int, [i32, C.POINTER(i64)]),
    'gpi_random_subset_ws': (C.c_int, [vp, i32, i32, u64, vp, u64, vp, i64, vp]),
    'gpi_vo_rows': (C.c_int, [i32, i32, i32]),
    'gpi_vo_query': (C.c_int, [C.POINTER(VoQueryDesc), vp]),
    'gpi_vo_moments': (C.c_int, [C.POINTER(VoMomentsDesc), vp]),
    'gpi_vo_galerkin': (C.c_int, [C.POINTER(VoGalerkinDesc), vp]),
    'gpi_vo_condition': (C.c_int, [C.POINTER(VoConditionDesc), vp]),
    'gpi_vo_precision': (C.c_int, [C.POINTER(VoPrecisionDesc), vp]),
    'gpi_vo_pattern': (C.c_int, [vp, i32, i32, i32, i32, vp, vp, vp, vp]),
    'gpi_vo_sparse_values': (C.c_int, [vp, i32, i32, i32, C.POINTER(VoSparse), vp]),
    'gpi_gauss_sample': (C.c_int, [vp, vp, vp, i64, i32, i32, vp, u64, vp, u64, vp]),
    'gpi_gp_sample': (C.c_int, [C.POINTER(GpSampleDesc), vp]),
    'gpi_predictive_scores': (C.c_int, [vp, vp, vp, i32, i32, vp, vp]),
}

_LIB = None
SRC_DIR = os.path.join(os.path.dirname(HERE), 'csrc')
INCLUDE_H = os.path.join(os.path.dirname(os.path.dirname(HERE)), 'include', 'gpi.h')


def source_sha():
    """sha1 of the library's sources as csrc/Makefile computes it (csrc/*.hip in name order, csrc/common.h,
    include/gpi.h, concatenated); None when the sources are not next to the package."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(SRC_DIR, '*.hip')), key=os.path.basename)
    files += [os.path.join(SRC_DIR, 'common.h'), os.path.join(SRC_DIR, 'conv_shapes.h'), INCLUDE_H]
    if not all(os.path.exists(f) for f in files):
        return None
    h = hashlib.sha1()
    for f in files:
        with open(f, 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


def check_source_sha(L, path=None):
    """Refuse a library built from other sources than the ones next to it (a stale build would run
    silently otherwise).  GPI_ALLOW_STALE_LIB=1 overrides (A/B builds of earlier sources)."""
    want = source_sha()
    got = L.gpi_source_sha().decode()
    if want is not None and got != want and os.environ.get('GPI_ALLOW_STALE_LIB') != '1':
        raise NativeError('stale native library %s: built from sources sha1 %s, the sources here are %s; '
                          'rebuild (make -C csrc) or set GPI_ALLOW_STALE_LIB=1' % (path or LIB_PATH, got, want))
    return got


class NativeError(RuntimeError):
    pass


def lib():
    """Load (once) and return the native library.  Raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError('libgpi_hip.so not built (%s); run __graft_entry__.build() / make -C csrc' % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        stale_ok = os.environ.get('GPI_ALLOW_STALE_LIB') == '1'
        # the source check first: a library built before an entry point existed (gpi_source_sha included)
        # is a stale build, reported as one, not as an undefined symbol
        if hasattr(L, 'gpi_source_sha'):
            L.gpi_source_sha.restype, L.gpi_source_sha.argtypes = SIGNATURES['gpi_source_sha']
            check_source_sha(L)
        elif not stale_ok:
            raise NativeError('stale native library %s: built before gpi_source_sha existed; rebuild (make -C csrc) '
                              'or set GPI_ALLOW_STALE_LIB=1' % LIB_PATH)
        missing = [name for name in SIGNATURES if not hasattr(L, name)]
        if missing:
            raise NativeError('stale native library %s: no %s; rebuild (make -C csrc)' % (LIB_PATH, ', '.join(missing)))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        sizes = (i64 * 64)()
        k = L.gpi_struct_sizes(sizes, 64)
        if k != len(STRUCTS):
            raise NativeError('ABI mismatch: %d structs in the library, %d in the binding' % (k, len(STRUCTS)))
        for s, cls in zip(sizes[:k], STRUCTS):
            if s != C.sizeof(cls):
                raise NativeError('ABI mismatch for %s: C %d bytes, ctypes %d' % (cls.__name__, s, C.sizeof(cls)))
        if L.gpi_replicas() != GPI_REPLICAS:
            raise NativeError('ABI mismatch: the library keeps %d statistic replicas, the binding %d (GPI_REPLICAS)'
                              % (L.gpi_replicas(), GPI_REPLICAS))
        _LIB = L
    return _LIB


def check(rc, what):
    if rc != 0:
        msg = lib().gpi_error_string(rc).decode()
        raise NativeError('%s failed: %s (%d)' % (what, msg, rc))


def require_device(t):
    if not isinstance(t, torch.Tensor) or t.device.type != 'cuda':
        raise NativeError('the HIP path needs tensors on a ROCm GPU (got %s); there is no CPU fallback'
                          % (t.device if isinstance(t, torch.Tensor) else type(t)))


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def stream_handle(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
