"""Execution engines: the ELBO training step and the standalone codec / ROM
operators, each a fixed sequence of libgpi_hip.so launches over
pre-planned workspaces.  No host synchronisation anywhere on the path.

ElboEngine = GenerativeModel.elbo (generative.py:247-287) for the armortized
unsupervised term (generative.py:546-585) + the supervised freeX term
(generative.py:461-500) + the virtual-observable freeX term
(generative.py:341-392, hold-off variant included), or their lockX variants
(independent_X = False: X~ = gp(z), generative.py:300-339,429-459), and its backward:

  forward   encoder program (B_u)            conv.hip  (11 launches at C64)
            dense head (all samples)          head.hip  (1)
            decoder program (B_u + N_s + N_vo, one BN group per term, fused Gaussian loss)  (12)
            ROM solve + log-lik + adjoint     rom.hip   (1 per labeled / VO term)
  backward  decoder program (reverse), dense head, encoder program (reverse),
            weight-gradient slab reduction, outer-product GEMMs, finalize.
"""
import ctypes as C
import os
import math

import torch

from . import _lib as L
from .plan import Arena, encoder_program, decoder_program

ENT_CONST = 0.5 * (math.log(2 * math.pi) + 1)
N_TERMS = 16
R = L.GPI_REPLICAS
# term slots in the fp64 scratch
T_LX0 = 0          # decoder Gaussian log-lik per group (0..3)
T_KL_ENC, T_KL_Q, T_LOGL_X, T_ENT = 4, 5, 6, 7           # head terms (supervised segment)
T_KL_Q2, T_LOGL_X2, T_ENT2 = 8, 9, 10                   # head terms (VO segment)
T_LOGL_Y, T_LOGL_Y2 = 11, 12                            # ROM log-lik (supervised, VO)


def groups_struct(sizes):
    g = L.Groups()
    g.n_groups = len(sizes)
    s = 0
    g.start[0] = 0
    for i, n in enumerate(sizes):
        s += n
        g.start[i + 1] = s
    for i in range(len(sizes) + 1, L.GPI_MAX_GROUPS + 1):
        g.start[i] = s
    return g


class Workspace(object):
    def __init__(self):
        self.ws = Arena()
        self.stats = Arena(align=1)
        self.parts = Arena()
        self.t_ws = None

    def alloc(self, n):
        return self.ws.alloc(n)

    def materialize(self, device):
        self.t_ws = torch.zeros(max(self.ws.size, 64), dtype=torch.float32, device=device)
        self.n_stats = max(self.stats.size, 1)
        self.t_scr = torch.zeros(N_TERMS * R + R * self.n_stats * L.GPI_MAX_GROUPS * 4 + 4, dtype=torch.float64,
                                 device=device)
        self.t_parts = torch.zeros(max(self.parts.size, 64), dtype=torch.float32, device=device)
        self.t_flag = torch.zeros(4, dtype=torch.int32, device=device)

    def view(self, off, *shape):
        n = 1
        for s in shape:
            n *= s
        return self.t_ws[off:off + n].view(*shape)

    def fptr(self, off):
        return C.c_void_p(self.t_ws.data_ptr() + 4 * off)

    @property
    def terms(self):
        """[N_TERMS] term sums (replica copies folded)."""
        return self.t_scr[:N_TERMS * R].view(N_TERMS, R).sum(1)

    def term_ptr(self, k):
        """Term slot k: GPI_REPLICAS consecutive fp64 accumulators."""
        return C.c_void_p(self.t_scr.data_ptr() + 8 * k * R)

    @property
    def stats_ptr(self):
        return C.c_void_p(self.t_scr.data_ptr() + 8 * N_TERMS * R)

    def zero_scratch(self):
        self.t_scr.zero_()


def make_ctx(ws, flat, group_sizes):
    c = L.CodecCtx()
    c.params = flat.P.data_ptr()
    c.ws = ws.t_ws.data_ptr()
    c.stats = ws.stats_ptr.value
    c.gacc = flat.gacc.data_ptr()
    c.wpart = ws.t_parts.data_ptr()
    c.ext_in = None
    c.ext_idx = None
    c.ext_stride = 0
    c.loss_acc = ws.term_ptr(T_LX0).value
    c.n_stats = ws.n_stats
    c.bn_eps = 1e-5
    c.groups = groups_struct(group_sizes)
    for g in range(L.GPI_MAX_GROUPS):
        c.loss_scale[g] = 1.0
    return c


def _lib():
    return L.lib()


def run_reduce(items, ws, flat, st):
    """gpi_wgrad_reduce over a Python list of ReduceItem, in launches of <= GPI_MAX_REDUCE_ITEMS."""
    for k in range(0, len(items), L.GPI_MAX_REDUCE_ITEMS):
        part = items[k:k + L.GPI_MAX_REDUCE_ITEMS]
        arr = (L.ReduceItem * len(part))(*part)
        _run(_lib().gpi_wgrad_reduce, arr, len(part), C.c_void_p(ws.t_parts.data_ptr()),
             C.c_void_p(flat.gacc.data_ptr()), st, what='wgrad reduce')


def _run(fn, *args, what=None):
    L.check(fn(*args), what or fn.__name__)


def dropout_views(ws, progs):
    out = {}
    for key, prog, B in progs:
        if prog is None or prog.drop_numel == 0:
            continue
        out[key] = {name: ws.view(off, B, cout) for name, off, cout in prog.drop_ops()}
    return out


def draw_dropout(ws, progs, stream, seed, offset_ptr=None, sub=20, only=None):
    """Dropout2d scales of the programs (Philox sub id sub + position); only: the positions to draw."""
    for k, prog in enumerate(progs):
        if prog is None or prog.drop_numel == 0 or (only is not None and k not in only):
            continue
        _run(_lib().gpi_dropout_masks, ws.fptr(prog.drop_off), prog.drop_numel, prog.drop_rate, seed,
             offset_ptr, sub + k, stream, what='dropout masks')


class BnRunning(object):
    """BatchNorm2d running statistics of a set of codec programs (train mode, momentum 0.1):
    the reference updates running_mean / running_var / num_batches_tracked at every codec call;
    here one tiny launch per step folds every call's fp64 batch sums (gpi_bn_running_update)."""

    def __init__(self, entries, ws, device):
        """entries: [(program, module owning the BN layers, [(group, samples), ...] in call order)]."""
        items = []
        self.buffers = []
        max_ch = 1
        for prog, module, calls in entries:
            if prog is None or module is None or not calls:
                continue
            for op in prog.ops:
                if op.bn is None:
                    continue
                bn = module.get_submodule(op.bn)
                if bn.running_mean is None or bn.running_mean.device != device:
                    continue
                it = L.BnRunningItem()
                it.stat, it.channels, it.n_calls = op.desc.in_stat, op.cin, len(calls)
                for k, (g, n) in enumerate(calls):
                    it.group[k] = g
                    it.count[k] = float(n * op.src.H * op.src.W)
                it.running_mean, it.running_var = bn.running_mean.data_ptr(), bn.running_var.data_ptr()
                it.num_batches_tracked = bn.num_batches_tracked.data_ptr()
                items.append(it)
                self.buffers += [bn.running_mean, bn.running_var, bn.num_batches_tracked]
                max_ch = max(max_ch, op.cin)
        self.n = len(items)
        self.max_ch = max_ch
        self.ws = ws
        if self.n:
            arr = (L.BnRunningItem * self.n)(*items)
            raw = bytes(arr)
            self.dev = torch.tensor(list(raw), dtype=torch.uint8, device=device)

    def launch(self, stream, momentum=0.1):
        if self.n:
            _run(_lib().gpi_bn_running_update, C.c_void_p(self.dev.data_ptr()), self.n, self.max_ch,
                 self.ws.stats_ptr, self.ws.n_stats, momentum, stream, what='bn running stats')


def inject_dropout(views, masks):
    """Copy given channel scales {'enc' / 'dec': {conv name: [B, cout]}} into the engine's views."""
    for key, d in masks.items():
        for name, m in d.items():
            views[key][name].copy_(m)


class ElboEngine(object):
    """Fused armortized-unsupervised + supervised-freeX (+ virtual-observable freeX) ELBO of a
    GenerativeModel.  N_vo > 0 adds the VO term (its own decoder BN group, q_z['vo'] / q_X['vo']
    rows as the head's second variational segment, a second ROM launch against targets sampled
    from the VO posterior); vo_holdoff keeps only its logL_x - KL part (generative.py:349-364)."""

    def __init__(self, model, B_u, N_s, normalize=False, N_vo=0, vo_holdoff=False, q_unsup=None,
                 running_modules=None, shared_grads=True):
        """q_unsup: q_z['unsupervised'] for the non-armortized unsupervised term (no encoder,
        GenerativeModel.elbo_unsupervised generative.py:515-544): its rows replace the encoder
        heads; the term's KL is the reference's KLD of q_z['supervised'] (sic, :525).
        shared_grads=False: gradients of the per-sample variational rows only -- the codec backward
        computes input gradients without weight / BN-affine gradients (no slab rows, no slab
        reductions) and the dense weight GEMM is skipped (the PredictionEnsemble, whose Adam updates
        its q_z rows only while the reference discards the decoder gradients it also forms)."""
        self.shared_grads = bool(shared_grads)
        self.model = model
        self.q_unsup = q_unsup
        self.armortized = q_unsup is None
        flat = model._flat
        self.flat = flat
        dev = flat.P.device
        self.B_u, self.N_s, self.N_vo = int(B_u), int(N_s), int(N_vo)
        self.vo_holdoff = bool(vo_holdoff) and self.N_vo > 0
        self.N_q = self.N_s + self.N_vo
        self.B = self.B_u + self.N_q
        self.normalize = bool(normalize)
        # q samples whose X~ enters the ROM / gp likelihood (hold-off VO samples do not)
        self.N_x = self.N_s + (self.N_vo if not self.vo_holdoff else 0)
        enc, dec, gp, g = model.encoder, model.f, model.gp, model.g
        # lockX (independent_X = False): X~ = gp(z), no q_X rows, no q_X noise, no logL_X / entropy
        self.lockx = not gp.independent_X
        self.N_ex = 0 if self.lockx else self.N_x
        self.enc, self.dec = enc, dec
        ws = Workspace()
        self.ws = ws
        offE = (lambda n: flat.offset(enc.get_parameter(n))) if enc is not None else None
        offD = lambda n: flat.offset(dec.get_parameter(n))
        dz = dec.dim_latent
        self.dz = dz
        # ---- encoder program
        if self.B_u > 0 and self.armortized:
            ec = enc.native_config()
            self.ep = encoder_program(**ec)
            self.enc_descs = self.ep.layout(self.B_u, ws.ws, ws.stats, ws.parts, groups_struct([self.B_u]), offE)
            d_feat = self.ep.d_feat
        else:
            self.ep = None
            d_feat = 1
        # ---- decoder program (groups: unsup, sup, vo)
        dc = dec.native_config()
        # the decoder likelihood of generative.py:232-239: log-property Gaussian (default) or the
        # exponentiated field's (reconstruct_log_eff_property = False)
        log_field = getattr(model, 'config', {}).get('reconstruct_log_eff_property', True)
        self.dp = decoder_program(final_epilogue=L.EPI_GAUSS_LOSS if log_field else L.EPI_GAUSS_EXP_LOSS, **dc)
        self.dec_sizes = [n for n in (self.B_u, self.N_s, self.N_vo) if n > 0]
        self.g_sup = (1 if self.B_u > 0 else 0) if self.N_s > 0 else None
        self.g_vo = ((self.B_u > 0) + (self.N_s > 0)) if self.N_vo > 0 else None
        self.dec_descs = self.dp.layout(self.B, ws.ws, ws.stats, ws.parts, groups_struct(self.dec_sizes), offD)
        # codec launch ranges: the encoder's ops [0, n_enc_conv), the decoder's [dec0, ...)
        self.n_enc_conv = len(self.enc_descs) if self.ep is not None else 0
        self.dec0 = 0
        # the loss epilogue consumes (mu, logsigma) in registers: nobody reads the output image (9.4 MB of
        # writes per step at C64)
        self.dec_descs[len(self.dec_descs) - 1].out_off = -1
        if not self.shared_grads:
            for d in self.dec_descs:
                d.wpart_off = -1          # input gradients only
        # the output conv's forward and backward run as ONE launch at the end of the forward
        # (gpi_conv_loss_fused: the loss gradient stays in LDS); GPI_FUSE_OUT=0 keeps them apart (A/B only)
        self.n_dec_sep = len(self.dec_descs) - (1 if os.environ.get('GPI_FUSE_OUT', '1') != '0' else 0)
        # ---- dense head buffers
        d_lat = self.dp.input.per_sample
        d_x = g.dim_effective_property if self.N_q > 0 else 1
        self.d_x = d_x
        self.d_y = g.dim_out
        hb = {}
        for name, n in (('hpre', self.B_u * d_feat), ('dhpre', self.B_u * d_feat),
                        ('zmu', self.B * dz), ('zls', self.B * dz), ('eps_z', self.B * dz), ('z', self.B * dz),
                        ('gz', self.B * dz), ('dzmu', self.B * dz), ('dzls', self.B * dz),
                        ('eps_x', self.N_q * d_x), ('xs', self.N_q * d_x), ('mux', self.N_q * d_x),
                        ('gxs', self.N_q * d_x), ('gmux', self.N_q * d_x),
                        ('y_vo', (self.N_vo if not self.vo_holdoff else 0) * self.d_y)):
            hb[name] = ws.alloc(max(n, 1))
        self.hb = hb
        # ROM log-likelihood: per-sample d/dlogsigma_y rows (plain stores), reduced into gacc with the
        # decoder slabs (gpi_rom gls_part) -- instead of n x d_y same-address fp64 atomics
        self.gls_off = {}
        for key, n in (('sup', self.N_s), ('vo', 0 if self.vo_holdoff else self.N_vo)):
            if n > 0:
                self.gls_off[key] = ws.parts.alloc(n * self.d_y)
        ws.materialize(dev)
        P = lambda mod, n: flat.offset(mod.get_parameter(n))
        h = L.HeadDesc()
        h.flags = L.HEAD_LATENT
        if self.B_u > 0:
            h.flags |= (L.HEAD_ENC if self.armortized else 0) | L.HEAD_REPARAM
        gpf = L.HEAD_GP | (L.HEAD_LOCKX if self.lockx else 0)
        if self.N_s > 0:
            h.flags |= L.HEAD_QZ | gpf
        h.n_enc, h.n_q, h.n_q2 = self.B_u, self.N_s, self.N_vo
        if self.N_vo > 0:
            h.flags2 = L.HEAD_QZ | (0 if self.vo_holdoff else gpf)
        h.d_feat, h.d_z, h.d_lat, h.d_x = d_feat, dz, d_lat, d_x
        if self.B_u > 0 and self.armortized:
            h.fc_w, h.fc_b = P(enc, 'features.FC.weight'), P(enc, 'features.FC.bias')
            h.mu_w, h.mu_b = P(enc, 'features.SplitDense.fc_mean.weight'), P(enc, 'features.SplitDense.fc_mean.bias')
            h.ls_w, h.ls_b = P(enc, 'features.SplitDense.fc_logvar.weight'), P(enc, 'features.SplitDense.fc_logvar.bias')
            h.feat, h.gfeat = self.ep.output.off, self.ep.output.s_off
        else:
            h.fc_w = h.fc_b = h.mu_w = h.mu_b = h.ls_w = h.ls_b = -1
            h.feat = h.gfeat = 0
        h.lat_w, h.lat_b = P(dec, 'latent_map.weight'), P(dec, 'latent_map.bias')
        h.gp_w = h.gp_b = h.gp_ls = h.qz_mu = h.qz_ls = h.qx_mu = h.qx_ls = -1
        h.qz_mu2 = h.qz_ls2 = h.qx_mu2 = h.qx_ls2 = -1
        if self.N_x > 0:
            h.gp_w, h.gp_b = P(gp, 'fc.weight'), P(gp, 'fc.bias')
            if not self.lockx:
                h.gp_ls = P(gp, 'logsigmas_X')
        if self.N_s > 0:
            qz = model.q_z['supervised']
            h.qz_mu, h.qz_ls = flat.offset(qz._mean), flat.offset(qz._logsigma)
            if not self.lockx:
                qx = model.q_X['supervised']
                h.qx_mu, h.qx_ls = flat.offset(qx._mean), flat.offset(qx._logsigma)
        if self.N_vo > 0:
            qz = model.q_z['vo']
            h.qz_mu2, h.qz_ls2 = flat.offset(qz._mean), flat.offset(qz._logsigma)
            if not self.vo_holdoff and not self.lockx:
                qx = model.q_X['vo']
                h.qx_mu2, h.qx_ls2 = flat.offset(qx._mean), flat.offset(qx._logsigma)
        for k, v in hb.items():
            setattr(h, k, v)
        h.lat, h.glat = self.dp.input.off, self.dp.input.s_off
        su = 1.0 / self.B_u if (self.normalize and self.B_u) else 1.0
        ss = 1.0 / self.N_s if (self.normalize and self.N_s) else 1.0
        sv = 1.0 / self.N_vo if (self.normalize and self.N_vo) else 1.0
        self.su, self.ss, self.sv = su, ss, sv
        h.kl_scale_enc, h.kl_scale_q, h.lx_scale = su, ss, ss
        if not self.armortized and self.B_u > 0:
            if self.N_s == 0:
                raise KeyError("elbo_unsupervised takes the KL of q_z['supervised'] (generative.py:525)")
            # the unsupervised term's KL is q_z['supervised']'s: no KL gradient on q_z['unsupervised'],
            # a second one (scale su) on the supervised rows
            h.kl_scale_enc = 0.0
            h.kl_scale_q = ss + su
        h.kl_scale_q2, h.lx_scale2 = sv, sv
        h.terms = ws.term_ptr(T_KL_ENC).value
        h.terms2 = ws.term_ptr(T_KL_Q2).value
        self.head = h
        # ---- contexts
        if self.ep is not None:
            self.ectx = make_ctx(ws, flat, [self.B_u])
            self.ectx.ext_stride = self.ep.input.per_sample
        self.dctx = make_ctx(ws, flat, self.dec_sizes)
        for gi, scale in enumerate([su] * (self.B_u > 0) + [ss] * (self.N_s > 0) + [sv] * (self.N_vo > 0)):
            self.dctx.loss_scale[gi] = scale
        # ---- gradient reductions
        self.reduce_enc = self.ep.reduce_items(offE) if self.ep is not None else []
        # slab-reduction items of the encoder's input conv (the first op; no input BN: one item)
        # (counted per op: 1 for the weight, +1 or +2 for an input BN whose gamma / beta are (not)
        # adjacent; a miscount would leave one of its items to the side stream while the main
        # stream's input-conv backward still writes that slab)
        self.n_reduce_in = self.ep.reduce_counts(offE)[0] if self.ep is not None else 0
        self.reduce_dec = self.dp.reduce_items(offD)
        self.reduce_items = self.reduce_enc + self.reduce_dec
        gi = []
        B = self.B

        def gemm(a, b, S, M, N, lda, ldb, c, bias, flags=0):
            it = L.GemmItem()
            it.a_off, it.b_off, it.c_off, it.bias_off = a, b, c, bias
            it.S, it.M, it.N, it.lda, it.ldb, it.flags = S, M, N, lda, ldb, flags
            gi.append(it)

        gemm(self.dp.input.s_off, hb['z'], B, d_lat, dz, d_lat, dz, h.lat_w, h.lat_b)
        if self.N_x > 0:
            gemm(hb['gmux'], hb['z'] + self.B_u * dz, self.N_x, d_x, dz, d_x, dz, h.gp_w, h.gp_b)
        if self.B_u > 0 and self.armortized:
            gemm(hb['dzmu'], hb['hpre'], self.B_u, dz, d_feat, dz, d_feat, h.mu_w, h.mu_b, 1)
            gemm(hb['dzls'], hb['hpre'], self.B_u, dz, d_feat, dz, d_feat, h.ls_w, h.ls_b, 1)
            gemm(hb['dhpre'], h.feat, self.B_u, d_feat, d_feat, d_feat, d_feat, h.fc_w, h.fc_b)
        if not self.shared_grads:
            gi = []
        self.gemm_items = (L.GemmItem * len(gi))(*gi)
        # ---- ROM (one launch per labeled / VO term; both on the side stream)
        def rom_desc(row0, n, scale, slot):
            r = L.RomDesc()
            rom = g.rom
            r.nc, r.refine, r.n, r.mode = rom.nc, rom.refine, n, L.ROM_LOGLIK
            r.x = ws.fptr(hb['xs'] + row0 * d_x).value
            r.x_stride = d_x
            r.logsig_y = flat.P.data_ptr() + 4 * flat.offset(g.logsigmas_y)
            r.loss_scale = scale
            r.gx_accumulate = 0
            if self.rom_draw:
                # the ROM draws its X~ rows from q_X itself (no wait on the head forward's xs)
                qx = model.q_X['supervised' if slot == T_LOGL_Y else 'vo']
                r.x_draw = 1
                r.x_mu = flat.P.data_ptr() + 4 * flat.offset(qx._mean)
                r.x_ls = flat.P.data_ptr() + 4 * flat.offset(qx._logsigma)
                r.x_eps = ws.fptr(hb['eps_x'] + row0 * d_x).value
            r.gx = ws.fptr(hb['gxs'] + row0 * d_x).value
            r.gx_stride = d_x
            r.gacc_logsig = flat.gacc.data_ptr() + 8 * flat.offset(g.logsigmas_y)
            r.loss_acc = ws.term_ptr(slot).value
            r.flag = ws.t_flag.data_ptr()
            r.mu_y = None
            r.uc = None
            r.dmu = None
            key = 'sup' if slot == T_LOGL_Y else 'vo'
            r.gls_part = ws.t_parts.data_ptr() + 4 * self.gls_off[key]
            it = L.ReduceItem()
            it.part_off, it.w_off, it.numel, it.row_stride, it.blocks = (self.gls_off[key], flat.offset(g.logsigmas_y),
                                                                         self.d_y, self.d_y, n)
            self.rom_reduce.append(it)
            return r

        self.rom_reduce = []
        # GPI_ROM_EARLY=1 (free q_X only): the fused step's ROM runs at the very start of the step on
        # the side stream, its inputs drawn from q_X in the kernel, concurrently with the encoder
        self.rom_draw = os.environ.get('GPI_ROM_EARLY', '0') == '1' and not self.lockx
        self.roms = []
        self.rom = self.rom_vo = None
        if self.N_s > 0:
            self.rom = rom_desc(0, self.N_s, ss, T_LOGL_Y)
            self.roms.append(self.rom)
        if self.N_vo > 0 and not self.vo_holdoff:
            self.rom_vo = rom_desc(self.N_s, self.N_vo, sv, T_LOGL_Y2)
            self.rom_vo.Y = ws.fptr(hb['y_vo']).value
            self.roms.append(self.rom_vo)
        # the ROMs' d/dlogsigma_y rows are reduced with the decoder slabs (after the ROMs on the side stream)
        self.reduce_dec = (self.reduce_dec if self.shared_grads else []) + self.rom_reduce
        self.reduce_items = self.reduce_enc + self.reduce_dec
        self._fixed = (self.B_u, self.N_s, self.N_vo)
        self._side = None
        self._pending_join = False
        # BN running statistics: encoder once, decoder once per term in the reference's call order
        # (unsupervised, supervised, vo: generative.py:247-287)
        run_mods = running_modules or {}
        self.running = BnRunning([(self.ep, run_mods.get('enc', enc), [(0, self.B_u)]),
                                  (self.dp, run_mods.get('dec', dec), list(enumerate(self.dec_sizes)))], ws, dev)
        self._running_pending = False
        # encoder slab reduction: all on the main stream after the input conv's backward ('main'), or
        # split ('split': the input conv's slabs on the main stream, the rest on the side stream
        # concurrently with the input conv's backward)
        self.enc_reduce = os.environ.get('GPI_ENC_REDUCE', 'split')
        # ROM launches enqueued before the decoder forward (capture order) instead of after it
        self.rom_first = False
        # where the fused step's ROM forks to the side stream: after the head forward ('forward') or
        # with the backward's side work ('backward'; GPI_ROM_AT)
        # (A/Bs within the boxes' +-1 % noise: 'backward' 0.6308 / 0.6286 vs 0.6370 / 0.6332 ms on one box,
        # 0.6277 / 0.6274 / 0.6316 / 0.6342 / 0.6485 vs 'forward' 0.6240 / 0.6255 / 0.6303 / 0.6255 / 0.6336 on
        # two others, r03: kept 'forward')
        self.rom_at = os.environ.get('GPI_ROM_AT', 'forward')
        self._rom_deferred = False
        self.rom_early_launched = False
        self._pending_sig = None       # hand-off flag the next main-stream codec call signals
        # callable(side stream handle) launched on the side stream ahead of the ROM (fused step)
        self.side_pre = None
        # SyncBN (set_sync_bn): None = replica-BN, per-rank batch statistics
        self.bn_sync = None
        self.bn_world = 1
        # cross-stream hand-offs: graph events (None) or device flags (set_flag_handoff)
        self.handoff = None
        self.side_done = None
        self._rejoin_pending = False

    # ------------------------------------------------------------------
    def set_flag_handoff(self, flags, epoch, err=None, side_done=None):
        """Hand the side stream its work by device flags (gpi_stream_signal / gpi_stream_wait) instead of
        event edges between the streams: flags = int32 device tensor (>= 4 words), epoch = the step
        counter (int64 device tensor, constant within a step), err = an int32 word the waits set on a
        timeout.  The side stream forks from the main stream once at the start of the forward; after
        the step's last kernel the caller joins it back with rejoin() (stream-capture legality: the
        events there sit at the graph's end, not between kernels of the main chain).
        side_done (int64 device counter): the streams are not joined by events at all -- the side
        stream's step starts with a wait until the step counter has reached side_done (the main stream's
        previous step has ended) and ends by incrementing it, so each stream can be captured as a
        graph of its own (FusedElboStep graph_mode 'streams')."""
        self.handoff = (flags, epoch, err)
        self.side_done = side_done

    def _signal(self, k, st):
        f, e, _ = self.handoff
        _run(_lib().gpi_stream_signal, C.c_void_p(f.data_ptr() + 4 * k), C.c_void_p(e.data_ptr()), st,
             what='stream signal')

    def _sig_args(self, k):
        """(flag, epoch) pointers of hand-off flag k for the *_sig launches (signal folded into a conv)."""
        f, e, _ = self.handoff
        return C.c_void_p(f.data_ptr() + 4 * k), C.c_void_p(e.data_ptr())

    def _wait(self, k, st):
        f, e, err = self.handoff
        _run(_lib().gpi_stream_wait, C.c_void_p(f.data_ptr() + 4 * k), C.c_void_p(e.data_ptr()),
             C.c_void_p(err.data_ptr()) if err is not None else None, st, what='stream wait')

    def rejoin(self):
        """Main stream waits for the side stream's end (flag hand-off mode; a no-op otherwise)."""
        if self._rejoin_pending:
            torch.cuda.current_stream().wait_event(self._ev_join2)
            self._rejoin_pending = False

    def _head_forward(self, st):
        _run(_lib().gpi_head_forward, C.byref(self.head), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), st, what='head forward')

    def _head_backward(self, hd, st):
        _run(_lib().gpi_head_backward, C.byref(hd), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), C.c_void_p(self.flat.gacc.data_ptr()), st, what='head backward')

    def eps_z(self):
        return self.ws.view(self.hb['eps_z'], self.B, self.dz)

    @property
    def has_dropout(self):
        return any(p is not None and p.drop_numel > 0 for p in (self.ep, self.dp))

    def dropout_views(self):
        """{'enc': {conv name: [B_u, cout]}, 'dec': {conv name: [B, cout]}}: the Dropout2d channel
        scales (0 or 1/(1-p)) the next forward uses."""
        return dropout_views(self.ws, (('enc', self.ep, self.B_u), ('dec', self.dp, self.B)))

    def draw_dropout(self, stream, seed, offset_ptr=None, sub=20, codecs=('enc', 'dec')):
        """Fresh Dropout2d scales for every dropout conv of the codecs (device Philox; the encoder's
        stream is sub, the decoder's sub + 1 whichever are drawn)."""
        draw_dropout(self.ws, (self.ep, self.dp), stream, seed, offset_ptr, sub,
                     only=[k for k, c in enumerate(('enc', 'dec')) if c in codecs])

    def eps_x(self):
        """[N_ex, d_x] q_X noise (supervised rows, then VO rows unless held off; none in lockX)."""
        return self.ws.view(self.hb['eps_x'], self.N_ex, self.d_x)

    def y_vo(self):
        """[N_vo, d_y] VO targets y ~ N(VO.mean, VO.var) of this step (generative.py:356)."""
        return self.ws.view(self.hb['y_vo'], self.N_vo if not self.vo_holdoff else 0, self.d_y)

    def bind(self, X_u=None, u_index=None, X_s=None, Y=None, F=None, X_vo=None, F_vo=None):
        """Point the launch descriptors at this step's data tensors.  The engine keeps them alive
        until the next bind: the backward reads X_u again (the input conv's weight gradient), so a
        caller's temporary (e.g. a random-subset gather) must not return to the allocator between
        the forward and the backward."""
        self._bound = (X_u, u_index, X_s, Y, F, X_vo, F_vo)
        if self.B_u > 0:
            L.require_device(X_u)
            assert X_u.dtype == torch.float32 and X_u.is_contiguous()
            if self.armortized:
                self.ectx.ext_in = X_u.data_ptr()
                self.ectx.ext_idx = u_index.data_ptr() if u_index is not None else None
            else:
                assert X_u.shape[0] == self.B_u and u_index is None
            self.dctx.tgt[0] = X_u.data_ptr()
            self.dctx.tgt_idx[0] = u_index.data_ptr() if u_index is not None else None
        if self.N_s > 0:
            gs = 1 if self.B_u > 0 else 0
            for t in (X_s, Y, F):
                L.require_device(t)
                assert t.dtype == torch.float32 and t.is_contiguous()
            self.dctx.tgt[gs] = X_s.data_ptr()
            self.dctx.tgt_idx[gs] = None
            self.rom.Y = Y.data_ptr()
            self.rom.F = F.data_ptr()
        if self.N_vo > 0:
            for t in (X_vo,) + ((F_vo,) if not self.vo_holdoff else ()):
                L.require_device(t)
                assert t.dtype == torch.float32 and t.is_contiguous()
            assert X_vo.shape[0] == self.N_vo
            self.dctx.tgt[self.g_vo] = X_vo.data_ptr()
            self.dctx.tgt_idx[self.g_vo] = None
            if not self.vo_holdoff:
                assert F_vo.shape[0] == self.N_vo
                self.rom_vo.F = F_vo.data_ptr()

    def forward(self, stream=None, compute_value=True, zero_gacc=True, zero_scratch=True, running='now'):
        """Launch the forward; returns the 0-d ELBO tensor (no host sync).  zero_gacc / zero_scratch
        False when the previous step's epilogue already cleared the accumulator / the statistics
        and term scratch (gpi_step_epilogue).  running: BN running-statistics update 'now' (end of
        the forward), 'defer' (on the side stream during backward) or None."""
        st = stream if stream is not None else L.stream_handle()
        if self.handoff is not None:
            # the side stream's one fork of the step, before any of its kernels: its flag waits then
            # follow this step's signals only (never the previous step's); side_done: by the step counter
            self._side_stream()
            if self.side_done is not None:
                _, e, err = self.handoff
                _run(_lib().gpi_stream_wait_ge, C.c_void_p(e.data_ptr()), C.c_void_p(self.side_done.data_ptr()),
                     C.c_void_p(err.data_ptr()) if err is not None else None, C.c_void_p(self._side.cuda_stream),
                     what='side step gate')
            else:
                self._ev_start.record(torch.cuda.current_stream())
                self._side.wait_event(self._ev_start)
        # early ROM: after the side gate (the previous step's update and epilogue -- q_X, eps_x, the
        # cleared term scratch -- are complete); needs the gate and a scratch this forward does not clear
        early = (self.rom_draw and bool(self.roms) and self.side_done is not None and not zero_scratch
                 and not (self.rom_at == 'backward' and not compute_value))
        self.rom_early_launched = early
        if early:
            self.rom_side(C.c_void_p(self._side.cuda_stream))
            self._ev_join.record(self._side)
            self._pending_join = True
        self.forward_a(st, zero_gacc, zero_scratch)
        # rom_at 'backward': the ROM follows the backward's fork on the side stream (ahead of the
        # variational samples' head backward that needs it) -- one cross-stream dependency less per
        # step; only when the value is not read right after the forward
        self._rom_deferred = bool(self.roms) and self.rom_at == 'backward' and not compute_value
        if self.roms and not self._rom_deferred and not early:
            # the ROM solve only feeds the head backward: run it on a side stream,
            # concurrently with the decoder (fork here, join in backward / value).  The decoder
            # is enqueued first so that, in a captured graph, the main chain is the fork's first
            # branch and keeps its hardware queue (each cross-queue dependency costs ~10 us).
            main = torch.cuda.current_stream()
            self._side_stream()
            if self.handoff is not None:
                self._pending_sig = 0          # folded into forward_b's first decoder conv
            else:
                self._ev_fork.record(main)
            if self.rom_first:
                self._launch_roms()
        self.forward_b(st)
        if self.roms and not self.rom_first and not self._rom_deferred and not early:
            self._launch_roms()
        if running == 'now':
            self.running.launch(st)
        self._running_pending = running == 'defer'
        if compute_value:
            self._join()
            return self.elbo_value()
        return None

    # The step's pieces, per stream, between its cross-stream dependencies (forward / backward
    # compose them with events; FusedElboStep's segment capture records each as its own
    # single-stream graph).
    def forward_a(self, st, zero_gacc=True, zero_scratch=True):
        """Main stream, up to the ROM fork: scratch / accumulator reset, encoder forward, head forward."""
        lib = _lib()
        if zero_scratch:
            self.ws.zero_scratch()
        if zero_gacc:
            self.flat.gacc.zero_()
        if self.ep is not None:
            self._codec_forward(self.enc_descs, 0, self.n_enc_conv, self.ectx, st, 'encoder forward')
        if not self.armortized and self.B_u > 0:
            # q_z['unsupervised'] rows as the "encoder" outputs of the head's first segment
            # (torch copies on the current stream, which the launches use)
            self.ws.view(self.hb['zmu'], self.B_u, self.dz).copy_(self.q_unsup._mean.detach())
            self.ws.view(self.hb['zls'], self.B_u, self.dz).copy_(self.q_unsup._logsigma.detach())
        assert lib is not None
        self._head_forward(st)

    def forward_b(self, st):
        """Main stream: decoder forward and its fused output conv (forward + loss + backward)."""
        lib = _lib()
        sig, self._pending_sig = self._pending_sig, None
        self._codec_forward(self.dec_descs, self.dec0, self.n_dec_sep, self.dctx, st, 'decoder forward', sig=sig)
        if self.n_dec_sep < len(self.dec_descs):
            _run(lib.gpi_conv_loss_fused, C.byref(self.dec_descs[self.n_dec_sep]), C.byref(self.dctx), st,
                 what='decoder output conv (forward + loss + backward)')

    def rom_side(self, sst):
        """Side stream: the ROM solves (after the head forward)."""
        if self.side_pre is not None:
            self.side_pre(sst)
        for r in self.roms:
            _run(_lib().gpi_rom, C.byref(r), sst, what='rom')

    def backward_a(self, st, split):
        """Main stream: decoder backward and the head backward (encoder samples only when split:
        the variational samples' need the ROM adjoint and follow it on the side stream)."""
        self._codec_backward(self.dec_descs, self.dec0, self.n_dec_sep, self.dctx, st, 'decoder backward')
        if split:
            hd = L.HeadDesc.from_buffer_copy(self.head)
            hd.flags |= L.HEAD_PART_ENC
            self._head_backward(hd, st)
        else:
            self._head_backward(self.head, st)
        if not self.armortized and self.B_u > 0:
            # d/dmu, d/dlogsigma of q_z['unsupervised'] (written by the head for its first segment)
            n = self.B_u * self.dz
            for src, q in (('dzmu', self.q_unsup._mean), ('dzls', self.q_unsup._logsigma)):
                o = self.flat.offset(q)
                self.flat.gacc[o:o + n].add_(self.ws.view(self.hb[src], n).double())

    def backward_b(self, st, sig=None):
        """Main stream: every encoder conv's backward but the input conv's (reverse order); sig: hand-off
        flag its first launch signals."""
        if self.ep is not None and self.n_enc_conv > 1:
            self._codec_backward(self.enc_descs, 1, self.n_enc_conv, self.ectx, st, 'encoder backward', sig=sig)
        elif sig is not None:
            self._signal(sig, st)

    def backward_c(self, st, enc_split, sig=None):
        """Main stream: the input conv's backward (weight gradient only) and the encoder slab
        reduction (its own slabs only when enc_split: the side stream reduces the rest); sig: hand-off
        flag the input conv's launch signals."""
        if self.ep is None:
            return
        if self.bn_sync is not None and self.enc_descs[0].gout_mode == 0:
            self._sync_stats(self.enc_descs[0].out_stat, self.enc_descs[0].cout, 2, 'enc')
        if sig is not None:
            _run(_lib().gpi_conv_backward_sig, C.byref(self.enc_descs[0]), C.byref(self.ectx), *self._sig_args(sig),
                 st, what='In_conv backward')
        else:
            _run(_lib().gpi_conv_backward, C.byref(self.enc_descs[0]), C.byref(self.ectx), st,
                 what='In_conv backward')
        run_reduce(self.reduce_enc[:self.n_reduce_in] if enc_split else self.reduce_enc, self.ws, self.flat, st)

    def backward_side_a(self, sst, split, side_extra=None):
        """Side stream, after the decoder backward: the variational samples' head backward (split),
        the decoder slab reduction, the deferred BN running statistics, the dense weight GEMM and
        side_extra."""
        lib = _lib()
        if self._rom_deferred:
            self.rom_side(sst)
            self._rom_deferred = False
        if split:
            hq = L.HeadDesc.from_buffer_copy(self.head)
            hq.flags |= L.HEAD_PART_Q
            self._head_backward(hq, sst)
        run_reduce(self.reduce_dec, self.ws, self.flat, sst)
        if self._running_pending:
            self.running.launch(sst)
            self._running_pending = False
        if len(self.gemm_items):
            _run(lib.gpi_outer_gemm, self.gemm_items, len(self.gemm_items), C.c_void_p(self.ws.t_ws.data_ptr()),
                 C.c_void_p(self.flat.gacc.data_ptr()), sst, what='outer gemm')
        if side_extra is not None:
            side_extra(sst)

    def backward_side_b(self, sst):
        """Side stream, after backward_b: the encoder slab reduction but the input conv's."""
        run_reduce(self.reduce_enc[self.n_reduce_in:], self.ws, self.flat, sst)

    # ------------------------------------------------------------------ SyncBN (optional)
    def set_sync_bn(self, allreduce, world, exchange=None):
        """SyncBN mode (the exact-parity alternative to replica-BN): every BN
        layer normalises over the union of the ranks' batches of its codec call, as the reference does
        over its one process's batch (codec.py:164-173 in train mode).  allreduce(t): in-place SUM
        over the ranks.  After each producing conv the fp64 channel sums {sum x, sum x^2} of its output
        are all-reduced (forward), and before each conv whose output feeds a BN the BN-backward sums
        {sum S, sum S x-hat} of that output (backward) -- once per channel and phase.  The kernels
        divide a sum by their own per-rank count n_r of the codec call's BN group, so the all-reduced
        sum is scaled by n_r / N (N = the group's count over all ranks, all-reduced once here): the
        global means for any per-rank batch sizes.  Every rank must run the same BN groups (a term
        with samples on some ranks only is refused).  The codec launches then go one by one (host
        hook between them); running_var's Bessel factor keeps the per-rank count (N/(N-1) for
        N = per-rank samples x pixels, >= 16384 here: a <1e-4 relative difference in the running
        buffer only).  exchange: a gpi.peer.PeerExchange -- every seam in ONE launch through the ranks'
        IPC-mapped buffers (gpi_bn_exchange GPI_BNX_PEER) instead of fold / allreduce / unfold."""
        # per-group sample counts: the encoder call (group 0), then the decoder's groups in order, and
        # the term presence flags (B_u, N_s, N_vo > 0), all summed over the ranks in ONE collective
        enc_n = [self.B_u if self.ep is not None else 0]
        local = enc_n + list(self.dec_sizes) + [0] * (L.GPI_MAX_GROUPS - len(self.dec_sizes))
        present = [float(n > 0) for n in (self.B_u, self.N_s, self.N_vo)]
        t = torch.tensor([float(n) for n in local] + present, dtype=torch.float64, device=self.flat.P.device)
        allreduce(t)
        tot = t.cpu().tolist()
        if any(abs(p * world - s) > 0.5 for p, s in zip(present, tot[len(local):])):
            raise ValueError('SyncBN: every rank must run the same ELBO terms (B_u / N_s / N_vo > 0 on all or '
                             'none of the ranks); got %s of %d ranks' % (tot[len(local):], world))
        fac = [(n / g if g > 0 else 0.0) for n, g in zip(local, tot[:len(local)])]
        dev = self.flat.P.device
        # scale per (program, group): [GPI_MAX_GROUPS] for the encoder's and the decoder's stat slots
        self.bn_scale = {'enc': torch.tensor([fac[0]] + [0.0] * (L.GPI_MAX_GROUPS - 1), dtype=torch.float64,
                                             device=dev).view(-1, 1, 1),
                         'dec': torch.tensor(fac[1:1 + L.GPI_MAX_GROUPS], dtype=torch.float64,
                                             device=dev).view(-1, 1, 1)}
        self.bn_global_counts = {'enc': tot[0], 'dec': tot[1:1 + len(self.dec_sizes)]}
        self.bn_sync = allreduce
        self.bn_world = int(world)
        self.bn_exchange = exchange
        self._bnx_msg = torch.zeros(L.GPI_BNX_MSG, dtype=torch.float64, device=dev)

    def _stats_view(self):
        R, G = L.GPI_REPLICAS, L.GPI_MAX_GROUPS
        o = N_TERMS * R
        return self.ws.t_scr[o:o + R * G * self.ws.n_stats * 4].view(R, G, self.ws.n_stats, 4)

    def _sync_stats(self, stat0, n, f0, kind):
        """All-reduce the replica-folded sums of stat slots [stat0, stat0 + n), fields f0, f0 + 1, scaled
        per BN group by n_rank / N_global (set_sync_bn), back into replica 0: gpi_bn_exchange FOLD, the
        collective on the [groups, n, 2] message, UNFOLD -- or the one-shot peer form (one launch)."""
        lib = _lib()
        d = L.BnExchangeDesc(stats=self.ws.stats_ptr.value, n_stats=self.ws.n_stats, stat0=stat0, n=n, f0=f0,
                             scale=self.bn_scale[kind].data_ptr(), msg=self._bnx_msg.data_ptr())
        st = L.stream_handle()
        if self.bn_exchange is not None:
            self.bn_exchange.fill(d)
            _run(lib.gpi_bn_exchange, C.byref(d), st, what='SyncBN peer exchange')
            return
        d.mode = L.BNX_FOLD
        _run(lib.gpi_bn_exchange, C.byref(d), st, what='SyncBN fold')
        self.bn_sync(self._bnx_msg[:L.GPI_MAX_GROUPS * n * 2])
        d.mode = L.BNX_UNFOLD
        _run(lib.gpi_bn_exchange, C.byref(d), st, what='SyncBN unfold')

    def _codec_kind(self, descs):
        return 'enc' if self.ep is not None and descs is self.enc_descs else 'dec'

    def _codec_forward(self, descs, i0, i1, ctx, st, what, sig=None):
        """descs[i0] .. descs[i1 - 1]; sig: hand-off flag the first launch signals (gpi_codec_forward_sig)."""
        lib = _lib()
        sa = self._sig_args(sig) if sig is not None else (None, None)
        if i1 <= i0:
            if sig is not None:
                self._signal(sig, st)
            return
        if self.bn_sync is None:
            ptr = C.cast(C.byref(descs, i0 * C.sizeof(L.ConvDesc)), C.POINTER(L.ConvDesc))
            _run(lib.gpi_codec_forward_sig, ptr, i1 - i0, C.byref(ctx), *sa, st, what=what)
            return
        kind = self._codec_kind(descs)
        for i in range(i0, i1):
            d = descs[i]
            _run(lib.gpi_conv_forward_sig, C.byref(d), C.byref(ctx), *(sa if i == i0 else (None, None)), st,
                 what=what)
            if d.epilogue == L.EPI_STORE_STATS and d.out_stat >= 0:
                self._sync_stats(d.out_stat, d.cout, 0, kind)

    def _codec_backward(self, descs, i0, i1, ctx, st, what, sig=None):
        """descs[i1 - 1] down to descs[i0] (gpi_codec_backward's order); sig: hand-off flag the first
        launch signals."""
        lib = _lib()
        sa = self._sig_args(sig) if sig is not None else (None, None)
        if i1 <= i0:
            if sig is not None:
                self._signal(sig, st)
            return
        if self.bn_sync is None:
            ptr = C.cast(C.byref(descs, i0 * C.sizeof(L.ConvDesc)), C.POINTER(L.ConvDesc))
            _run(lib.gpi_codec_backward_sig, ptr, i1 - i0, C.byref(ctx), *sa, st, what=what)
            return
        kind = self._codec_kind(descs)
        for i in range(i1 - 1, i0 - 1, -1):
            d = descs[i]
            if d.gout_mode == 0:          # its output feeds a BN: that BN's backward sums are complete
                self._sync_stats(d.out_stat, d.cout, 2, kind)
            _run(lib.gpi_conv_backward_sig, C.byref(d), C.byref(ctx), *(sa if i == i1 - 1 else (None, None)), st,
                 what=what)

    def _launch_roms(self):
        if self.handoff is not None:
            self._wait(0, C.c_void_p(self._side.cuda_stream))
        else:
            self._side.wait_event(self._ev_fork)
        self.rom_side(C.c_void_p(self._side.cuda_stream))
        self._ev_join.record(self._side)
        self._pending_join = True

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=torch.cuda.current_stream().device)
            self._ev_fork, self._ev_join = torch.cuda.Event(), torch.cuda.Event()
            self._ev_fork2, self._ev_join2 = torch.cuda.Event(), torch.cuda.Event()
            self._ev_enc = torch.cuda.Event()
            self._ev_start = torch.cuda.Event()
        return self._side

    def _join(self):
        if self._pending_join:
            torch.cuda.current_stream().wait_event(self._ev_join)
            self._pending_join = False

    def _check_rom_written(self):
        if self._rom_deferred:
            # GPI_ROM_AT=backward with compute_value=False: the ROM (and its log-likelihood terms) runs
            # with the backward's side work, so the terms are not written until backward() is enqueued
            raise RuntimeError('ElboEngine: the ROM log-likelihood is deferred to the backward '
                               '(rom_at="backward"); read the ELBO terms after backward()')

    def elbo_value(self, terms=None):
        """0-d ELBO from the term accumulators (or from a saved copy ``terms`` [N_TERMS * R])."""
        if terms is None:
            self._check_rom_written()
        t = self.ws.terms if terms is None else terms.view(N_TERMS, R).sum(1)
        su, ss, sv = self.su, self.ss, self.sv
        val = t.new_zeros(())
        if self.B_u > 0:
            val = val + su * (t[T_LX0] - (t[T_KL_ENC] if self.armortized else t[T_KL_Q]))
        if self.N_s > 0:
            v = t[T_LX0 + self.g_sup] + t[T_LOGL_Y] - t[T_KL_Q]
            if not self.lockx:
                v = v + t[T_LOGL_X] + t[T_ENT] + self.N_s * ENT_CONST
            val = val + ss * v
        if self.N_vo > 0:
            v = t[T_LX0 + self.g_vo] - t[T_KL_Q2]
            if not self.vo_holdoff:
                v = v + t[T_LOGL_Y2]
                if not self.lockx:
                    v = v + t[T_LOGL_X2] + t[T_ENT2] + self.N_vo * ENT_CONST
            val = val + sv * v
        return val.to(torch.float32)

    def terms(self):
        """Dictionary of the individual ELBO terms (host sync)."""
        self._check_rom_written()
        t = self.ws.terms.cpu()
        out = {}
        gi = 0
        if self.B_u > 0:
            if self.armortized:
                out['ARM_unsupervised_logL_x'] = float(t[T_LX0])
                out['ARM_unsupervised_DKL_z'] = float(t[T_KL_ENC])
            else:
                out['unsupervised_logL_x'] = float(t[T_LX0])
                out['unsupervised_DKL_z'] = float(t[T_KL_Q])
            gi = 1
        if self.N_s > 0:
            out['supervised_logL_x'] = float(t[T_LX0 + gi])
            out['supervised_logL_y'] = float(t[T_LOGL_Y])
            out['supervised_DKL_z'] = float(t[T_KL_Q])
            if not self.lockx:
                out['supervised_logL_X'] = float(t[T_LOGL_X])
                out['supervised_entropy_X'] = float(t[T_ENT]) + self.N_s * ENT_CONST
        if self.N_vo > 0:
            out['vo_logL_x'] = float(t[T_LX0 + self.g_vo])
            out['vo_DKL'] = float(t[T_KL_Q2])
            if not self.vo_holdoff:
                out['vo_logL_y'] = float(t[T_LOGL_Y2])
                if not self.lockx:
                    out['vo_logL_X'] = float(t[T_LOGL_X2])
                    out['vo_entropy'] = float(t[T_ENT2]) + self.N_vo * ENT_CONST
        return out

    def backward(self, stream=None, side_extra=None, main_wait=True):
        """Gradients of -ELBO into flat.gacc (fp64).  side_extra(side_stream_handle) is launched on
        the side stream after the decoder's reductions, concurrently with the encoder backward (the
        fused step draws the next step's subset, noise and decoder dropout masks there; nothing it
        writes may be read by the encoder backward).  main_wait=False (flag hand-off only): the main
        stream does not wait for the side stream's end here -- the caller's next launch does
        (gpi_step_epilogue_adam wait_flag)."""
        st = stream if stream is not None else L.stream_handle()
        main = torch.cuda.current_stream()
        side = self._side_stream()
        # With the ROM still pending on the side stream, only the encoder samples' head backward
        # runs on the main stream; the variational samples' (which need the ROM adjoint) follow
        # the ROM on the side stream, so the main chain never waits for the ROM.
        split = self._pending_join or self._rom_deferred
        flags = self.handoff is not None
        sst = C.c_void_p(side.cuda_stream)
        self.backward_a(st, split)
        # the decoder's slab reduction and the dense weight gradients depend only on what is
        # done by now: run them on the side stream, concurrently with the encoder backward
        # (enqueued after it, so the encoder stays on the main chain's queue in a graph)
        if not flags:
            self._ev_fork2.record(main)
        n_enc = len(self.enc_descs) if self.ep is not None else 0
        enc_split = n_enc and self.enc_reduce == 'split'
        if n_enc:
            # flags: the encoder backward's first conv signals flag 1 (the head backward is done), the
            # input conv's backward flag 2 (the rest of the encoder backward is done)
            self.backward_b(st, sig=1 if flags else None)
            if enc_split and not flags:
                self._ev_enc.record(main)
            self.backward_c(st, enc_split, sig=2 if (flags and enc_split) else None)
        elif flags:
            self._signal(1, st)
        # (captured ahead of the encoder backward instead, the side branch took the launch stream
        # and the main chain the pooled one: 0.7526 vs 0.6289 ms per step, r03)
        if flags:
            self._wait(1, sst)
        else:
            side.wait_event(self._ev_fork2)
        self.backward_side_a(sst, split, side_extra)
        if split:
            self._pending_join = False          # joined below with the rest of the side work
        if enc_split:
            if flags:
                self._wait(2, sst)
            else:
                side.wait_event(self._ev_enc)
            self.backward_side_b(sst)
        if flags:
            # the side's end by flag on the main chain (a wait launch, or folded into the caller's
            # epilogue: main_wait False); the event join (capture legality) after the step's last
            # kernel: rejoin()
            self._signal(3, sst)
            if main_wait:
                self._wait(3, st)
            if self.side_done is not None:
                _run(_lib().gpi_rng_advance, C.c_void_p(self.side_done.data_ptr()), 1, sst, what='side step done')
            else:
                self._ev_join2.record(side)
                self._rejoin_pending = True
        else:
            self._ev_join2.record(side)
            main.wait_event(self._ev_join2)

    def finalize(self, out, accumulate=False, step=None, stream=None, zero_acc=False):
        st = stream if stream is not None else L.stream_handle()
        flags = (L.FINALIZE_ACCUMULATE if accumulate else 0) | (L.FINALIZE_ZERO if zero_acc else 0)
        _run(_lib().gpi_grad_finalize, C.c_void_p(self.flat.gacc.data_ptr()), C.c_void_p(out.data_ptr()),
             self.flat.numel, flags, C.c_void_p(step.data_ptr()) if step is not None else None, st,
             what='grad finalize')

    def check_flag(self):
        """Lazy replacement of ROM.py:75's per-step host sync."""
        if int(self.ws.t_flag[0].item()) != 0:
            raise ValueError('At least one of the conductivity values supplied to the ROM was smaller than 1e-12')


# ==========================================================================
# standalone operators (CNNEncoder.forward, CNNDecoder.forward, ROM, CGR)
# ==========================================================================
class EncoderEngine(object):
    """CNNEncoder.forward (Encoder.py:191-196): x -> (mean, logsigma) and its backward."""

    def __init__(self, enc, flat, B):
        self.flat, self.B = flat, int(B)
        ws = Workspace()
        self.ws = ws
        off = lambda n: flat.offset(enc.get_parameter(n))
        self.p = encoder_program(**enc.native_config())
        self.descs = self.p.layout(self.B, ws.ws, ws.stats, ws.parts, groups_struct([self.B]), off)
        d_feat, dz = self.p.d_feat, enc.latent_dim
        self.dz = dz
        hb = {k: ws.alloc(self.B * n) for k, n in (('hpre', d_feat), ('dhpre', d_feat), ('zmu', dz), ('zls', dz),
                                                    ('eps_z', dz), ('z', dz), ('gz', dz), ('dzmu', dz),
                                                    ('dzls', dz))}
        hb.update({k: 0 for k in ('eps_x', 'xs', 'mux', 'gxs', 'gmux')})
        ws.materialize(flat.P.device)
        h = L.HeadDesc()
        h.flags = L.HEAD_ENC
        h.n_enc, h.n_q, h.d_feat, h.d_z, h.d_lat, h.d_x = self.B, 0, d_feat, dz, 1, 1
        h.fc_w, h.fc_b = off('features.FC.weight'), off('features.FC.bias')
        h.mu_w, h.mu_b = off('features.SplitDense.fc_mean.weight'), off('features.SplitDense.fc_mean.bias')
        h.ls_w, h.ls_b = off('features.SplitDense.fc_logvar.weight'), off('features.SplitDense.fc_logvar.bias')
        h.lat_w = h.lat_b = h.gp_w = h.gp_b = h.gp_ls = h.qz_mu = h.qz_ls = h.qx_mu = h.qx_ls = -1
        for k, v in hb.items():
            setattr(h, k, v)
        h.feat, h.gfeat = self.p.output.off, self.p.output.s_off
        h.lat = h.glat = 0
        h.kl_scale_enc = h.kl_scale_q = h.lx_scale = 1.0
        h.terms = ws.term_ptr(T_KL_ENC).value
        self.head, self.hb = h, hb
        self.ctx = make_ctx(ws, flat, [self.B])
        self.ctx.ext_stride = self.p.input.per_sample
        items = self.p.reduce_items(off)
        self.reduce_items = items
        gi = []
        for a, c, b in ((hb['dzmu'], h.mu_w, h.mu_b), (hb['dzls'], h.ls_w, h.ls_b)):
            it = L.GemmItem(a_off=a, b_off=hb['hpre'], c_off=c, bias_off=b, S=self.B, M=dz, N=d_feat, lda=dz,
                            ldb=d_feat, flags=1)
            gi.append(it)
        gi.append(L.GemmItem(a_off=hb['dhpre'], b_off=h.feat, c_off=h.fc_w, bias_off=h.fc_b, S=self.B, M=d_feat,
                             N=d_feat, lda=d_feat, ldb=d_feat, flags=0))
        self.gemm_items = (L.GemmItem * len(gi))(*gi)
        self.running = BnRunning([(self.p, enc, [(0, self.B)])], ws, flat.P.device)

    def forward(self, x, dropout=None, seed=0):
        """dropout: optional injected channel scales {conv name: [B, cout]} (else drawn, seed)."""
        L.require_device(x)
        x = x.contiguous().float()
        self._x = x
        self.ctx.ext_in = x.data_ptr()
        self.ctx.ext_idx = None
        lib, st = _lib(), L.stream_handle()
        if self.p.drop_numel:
            if dropout is not None:
                inject_dropout(dropout_views(self.ws, (('enc', self.p, self.B),)), {'enc': dropout})
            else:
                draw_dropout(self.ws, (self.p,), st, seed)
        self.ws.zero_scratch()
        _run(lib.gpi_codec_forward, self.descs, len(self.descs), C.byref(self.ctx), st, what='encoder forward')
        self.running.launch(st)
        _run(lib.gpi_head_forward, C.byref(self.head), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), st, what='head forward')
        return (self.ws.view(self.hb['zmu'], self.B, self.dz).clone(),
                self.ws.view(self.hb['zls'], self.B, self.dz).clone())

    def backward(self, dmu, dls):
        lib, st = _lib(), L.stream_handle()
        self.ws.view(self.hb['gz'], self.B, self.dz).copy_(dmu)
        self.ws.view(self.hb['dzls'], self.B, self.dz).copy_(dls)
        self.flat.gacc.zero_()
        _run(lib.gpi_head_backward, C.byref(self.head), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), C.c_void_p(self.flat.gacc.data_ptr()), st, what='head backward')
        _run(lib.gpi_codec_backward, self.descs, len(self.descs), C.byref(self.ctx), st, what='encoder backward')
        run_reduce(self.reduce_items, self.ws, self.flat, st)
        _run(lib.gpi_outer_gemm, self.gemm_items, len(self.gemm_items), C.c_void_p(self.ws.t_ws.data_ptr()),
             C.c_void_p(self.flat.gacc.data_ptr()), st, what='outer gemm')


class DecoderEngine(object):
    """CNNDecoder.forward (Decoder.py:288-305): z -> (mean, logsigma) [B, H, W] and its backward."""

    def __init__(self, dec, flat, B):
        self.flat, self.B = flat, int(B)
        ws = Workspace()
        self.ws = ws
        off = lambda n: flat.offset(dec.get_parameter(n))
        self.p = decoder_program(final_epilogue=None, **dec.native_config())
        self.descs = self.p.layout(self.B, ws.ws, ws.stats, ws.parts, groups_struct([self.B]), off)
        dz = dec.dim_latent
        self.dz = dz
        d_lat = self.p.input.per_sample
        hb = {k: ws.alloc(self.B * dz) for k in ('zmu', 'zls', 'eps_z', 'z', 'gz', 'dzmu', 'dzls')}
        hb.update({k: 0 for k in ('hpre', 'dhpre', 'eps_x', 'xs', 'mux', 'gxs', 'gmux')})
        ws.materialize(flat.P.device)
        h = L.HeadDesc()
        h.flags = L.HEAD_LATENT
        h.n_enc, h.n_q, h.d_feat, h.d_z, h.d_lat, h.d_x = self.B, 0, 1, dz, d_lat, 1
        h.fc_w = h.fc_b = h.mu_w = h.mu_b = h.ls_w = h.ls_b = -1
        h.gp_w = h.gp_b = h.gp_ls = h.qz_mu = h.qz_ls = h.qx_mu = h.qx_ls = -1
        h.lat_w, h.lat_b = off('latent_map.weight'), off('latent_map.bias')
        for k, v in hb.items():
            setattr(h, k, v)
        h.feat = h.gfeat = 0
        h.lat, h.glat = self.p.input.off, self.p.input.s_off
        h.kl_scale_enc = h.kl_scale_q = h.lx_scale = 1.0
        h.terms = ws.term_ptr(T_KL_ENC).value
        self.head, self.hb = h, hb
        self.ctx = make_ctx(ws, flat, [self.B])
        items = self.p.reduce_items(off)
        self.reduce_items = items
        self.gemm_items = (L.GemmItem * 1)(L.GemmItem(a_off=h.glat, b_off=hb['z'], c_off=h.lat_w, bias_off=h.lat_b,
                                                      S=self.B, M=d_lat, N=dz, lda=d_lat, ldb=dz, flags=0))
        o = self.p.output
        self.out_shape = (self.B, o.C, o.H, o.W)
        self.running = BnRunning([(self.p, dec, [(0, self.B)])], ws, flat.P.device)

    def forward(self, z, dropout=None, seed=0):
        """dropout: optional injected channel scales {conv name: [B, cout]} (else drawn, seed)."""
        L.require_device(z)
        lib, st = _lib(), L.stream_handle()
        self.ws.view(self.hb['z'], self.B, self.dz).copy_(z)
        if self.p.drop_numel:
            if dropout is not None:
                inject_dropout(dropout_views(self.ws, (('dec', self.p, self.B),)), {'dec': dropout})
            else:
                draw_dropout(self.ws, (self.p,), st, seed)
        self.ws.zero_scratch()
        _run(lib.gpi_head_forward, C.byref(self.head), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), st, what='latent map')
        _run(lib.gpi_codec_forward, self.descs, len(self.descs), C.byref(self.ctx), st, what='decoder forward')
        self.running.launch(st)
        return self.ws.view(self.p.output.off, *self.out_shape).clone()

    def backward(self, dout):
        lib, st = _lib(), L.stream_handle()
        self.ws.view(self.p.output.s_off, *self.out_shape).copy_(dout)
        self.flat.gacc.zero_()
        _run(lib.gpi_codec_backward, self.descs, len(self.descs), C.byref(self.ctx), st, what='decoder backward')
        _run(lib.gpi_head_backward, C.byref(self.head), C.c_void_p(self.flat.P.data_ptr()),
             C.c_void_p(self.ws.t_ws.data_ptr()), C.c_void_p(self.flat.gacc.data_ptr()), st, what='latent map bwd')
        run_reduce(self.reduce_items, self.ws, self.flat, st)
        _run(lib.gpi_outer_gemm, self.gemm_items, len(self.gemm_items), C.c_void_p(self.ws.t_ws.data_ptr()),
             C.c_void_p(self.flat.gacc.data_ptr()), st, what='outer gemm')
        return self.ws.view(self.hb['dzmu'], self.B, self.dz).clone()


def ROM_NN(nc):
    """Number of coarse nodes of the nc x nc ROM mesh."""
    return (nc + 1) ** 2


def rom_call(nc, refine, x, F, input_kappa, mode, mu_y=None, uc=None, dmu=None, duc=None, gx=None, Y=None,
             logsig_y=None, gacc_logsig=None, loss_acc=None, flag=None, loss_scale=1.0, gx_accumulate=False,
             gls_part=None):
    """Thin launcher of gpi_rom for the standalone ROM / ReducedOrderModelOperator."""
    for t in (x, F):
        L.require_device(t)
    r = L.RomDesc()
    r.nc, r.refine, r.n, r.mode, r.input_kappa = nc, refine, x.shape[0], mode, 1 if input_kappa else 0
    r.x, r.x_stride, r.F = x.data_ptr(), x.stride(0), F.data_ptr()
    p = lambda t: t.data_ptr() if t is not None else None
    r.mu_y, r.uc, r.dmu, r.duc, r.gx, r.Y, r.logsig_y = p(mu_y), p(uc), p(dmu), p(duc), p(gx), p(Y), p(logsig_y)
    r.gx_stride = gx.stride(0) if gx is not None else 0
    r.gacc_logsig, r.loss_acc, r.flag, r.gls_part = p(gacc_logsig), p(loss_acc), p(flag), p(gls_part)
    r.loss_scale, r.gx_accumulate = loss_scale, 1 if gx_accumulate else 0
    _run(_lib().gpi_rom, C.byref(r), L.stream_handle(), what='rom')


def cgr_residual(logkappa_img, y, bc, nc, flux=False):
    """W^T [K(kappa) yhat]_free for a batch of fields -> [N, (nc+1)^2]; flux=True also returns the
    flux-constraint residual Gamma_fc y [N, 2 nc^2] of the same pass (flux.py:81-158, alpha = 0)."""
    for t in (logkappa_img, y, bc):
        L.require_device(t)
    N, n = logkappa_img.shape[0], logkappa_img.shape[-1]
    r = torch.empty(N, (nc + 1) ** 2, dtype=torch.float32, device=y.device)
    d = L.ResidualDesc()
    lk, yy, bb = logkappa_img.contiguous().float(), y.contiguous().float(), bc.contiguous().float()
    d.n_fine, d.nc, d.n = n, nc, N
    rf = torch.empty(N, 2 * nc * nc, dtype=torch.float32, device=y.device) if flux else None
    d.logkappa, d.y, d.bc, d.r = lk.data_ptr(), yy.data_ptr(), bb.data_ptr(), r.data_ptr()
    d.r_flux = rf.data_ptr() if flux else None
    _run(_lib().gpi_cgr_residual, C.byref(d), L.stream_handle(), what='cgr residual')
    return (r, rf) if flux else r
