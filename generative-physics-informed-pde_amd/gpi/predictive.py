"""Native monitoring / validation paths around the ELBO step.

PredictionEnsembleEngine -- PredictionEnsemble.update (components.py:365-388), the
    decoder-only ELBO of the validation set with its own Adam, called 3x per step by
    training.py:419.  It is the ElboEngine with a single hold-off variational segment
    (q_z sample -> latent map -> decoder with fused Gaussian log-lik -> KL), run on a
    private flat buffer: [shadow copy of the decoder weights | the ensemble's q_z]; the
    shadow is refreshed from the model with one device copy per update, and Adam
    (gpi_adam) updates the q_z rows only.  The decoder weight gradients the reference
    leaves in f.*.grad (cleared by the trainer's next zero_grad) are not delivered -- nor computed:
    the codec backward runs input gradients only (no weight-gradient phases, slab rows or slab
    reductions, no dense weight GEMM).

predictive_y -- Analysis.sample_predictive_y for every sample at once
    (components.py:472-478,493-524): q_z draws -> gp mean (+ exp(logsigma_X) noise)
    (gpi_gp_sample) -> ROM coarse solves (gpi_rom) -> mean / std of W u + exp(logsigma_y)
    eps (gpi_vo_moments), i.e. N * N_mc MC samples in three launches instead of a
    Python loop of N ROM calls; predictive_scores -> relerr / logscore / R^2 sums.
"""
import copy
import ctypes as C
import os

import torch

from . import _lib as L
from . import vo as V
from .engine import ElboEngine, rom_call, ROM_NN
from .flat import FlatParameters


def _p(t):
    return t.data_ptr() if t is not None else None


def host_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# ---------------------------------------------------------------- predictive y
def predictive_y(model, q_mean, q_logsigma, F, N_mc, eps=None, seed=None, return_prec=False):
    """(mean, std) [N, d_y] of the MC predictive y of every row of q (Analysis.eval_all_y).
    eps (optional, injected): (eps_z [N*N_mc, d_z], eps_x [N*N_mc, d_x], eps_y [N*N_mc, d_y])."""
    for t in (q_mean, q_logsigma, F):
        L.require_device(t)
    gp, g = model.gp, model.g
    N, dz = q_mean.shape
    dx = g.dim_effective_property
    rom = g.rom
    rows = N * int(N_mc)
    dev = q_mean.device
    seed = host_seed() if seed is None else seed
    x = torch.empty(rows, dx, dtype=torch.float32, device=dev)
    w, b = gp.fc.weight.detach().contiguous(), gp.fc.bias.detach().contiguous()
    assert w.shape == (dx, dz)
    ls = gp.logsigmas_X.detach().contiguous() if gp.independent_X else None
    d = L.GpSampleDesc(rows=rows, rep=int(N_mc), d_z=dz, d_x=dx, qz_mu=_p(q_mean.detach().contiguous()),
                       qz_ls=_p(q_logsigma.detach().contiguous()), gp_w=_p(w), gp_b=_p(b), gp_ls=_p(ls),
                       eps_z=_p(eps[0]) if eps is not None else None, eps_x=_p(eps[1]) if eps is not None else None,
                       seed=seed, offset=None, sub=21, x=_p(x))
    keep = (q_mean, q_logsigma, w, b, ls)
    L.check(L.lib().gpi_gp_sample(C.byref(d), L.stream_handle()), 'gp sample')
    F_mc = F.float().repeat_interleave(int(N_mc), 0).contiguous()
    uc = torch.empty(rows, ROM_NN(rom.nc), dtype=torch.float32, device=dev)
    rom_call(rom.nc, rom.refine, x, F_mc, False, L.ROM_FORWARD, uc=uc)
    mean, std, prec = V.vo_moments(uc, rom.nc, rom.refine, N, int(N_mc), logsig_y=g.logsigmas_y.detach().contiguous(),
                                   eps=eps[2] if eps is not None else None, seed=seed, sub=23)
    del keep
    return (mean, std, prec) if return_prec else (mean, std)


def predictive_scores(Y, mean, std):
    """(mean relerr, mean logscore, R^2) -- Analysis.eval_all_y's three numbers (host sync)."""
    for t in (Y, mean, std):
        L.require_device(t)
        assert t.dtype == torch.float32 and t.is_contiguous()
    N, dy = Y.shape
    out = torch.empty(3, dtype=torch.float64, device=Y.device)
    L.check(L.lib().gpi_predictive_scores(_p(Y), _p(mean), _p(std), N, dy, _p(out), L.stream_handle()),
            'predictive scores')
    o = out.cpu()
    return float(o[0]) / N, float(o[1]) / N, float(o[2]) / dy


# ---------------------------------------------------------------- prediction ensemble
class _EngineModel(object):
    """The attributes ElboEngine reads from a GenerativeModel."""

    def __init__(self, f, gp, g, q_z, flat, config):
        self.f, self.gp, self.g = f, gp, g
        self.config = dict(config)       # decoder likelihood choice (components.py:361)
        self.encoder = None
        self.q_z = {'vo': q_z}
        self.q_X = {'vo': None}
        self._flat = flat


class PredictionEnsembleEngine(object):

    def __init__(self, model, q_z, X, lr_source, betas=(0.9, 0.999), eps=1e-8, running_stage=False):
        """running_stage: the decoder calls' BN running statistics go to the shadow decoder's buffers
        (zeroed: an EMA staging area that ConcurrentPredictionEnsemble folds into model.f) instead of
        straight into model.f's."""
        L.require_device(X)
        self.model = model
        self.q_z = q_z
        self.X = X.detach().contiguous().float()
        self.N = self.X.shape[0]
        self.shadow = copy.deepcopy(model.f)
        self._src = [p for _, p in model.f.named_parameters()]
        named = [('f.' + n, p) for n, p in self.shadow.named_parameters()] + \
                [('q.' + n, p) for n, p in q_z.named_parameters()]
        dev = X.device
        self.flat = FlatParameters(named, dev)
        self.q_off = min(self.flat.offset(q_z._mean), self.flat.offset(q_z._logsigma))
        self.n_dec = self.q_off                       # the shadow decoder's span (parameters + alignment padding)
        self.q_n = self.flat.numel - self.q_off
        assert self.q_n == max(self.flat.offset(q_z._mean), self.flat.offset(q_z._logsigma)) - self.q_off + \
            q_z._mean.numel()
        em = _EngineModel(self.shadow, model.gp, model.g, q_z, self.flat, getattr(model, 'config', {}))
        # the PE's decoder calls are the model's decoder's in the reference (components.py:371): its BN
        # running statistics are model.f's
        # q_z rows' gradients only (the decoder weight gradients the reference forms here are discarded);
        # GPI_PE_SHARED_GRADS=1 computes them anyway (A/B and the parity test's reference form)
        self.running_stage = bool(running_stage)
        if self.running_stage:
            with torch.no_grad():
                for b in self.shadow.buffers():
                    b.zero_()
        self.engine = ElboEngine(em, 0, 0, N_vo=self.N, vo_holdoff=True,
                                 running_modules={'dec': self.shadow if self.running_stage else model.f},
                                 shared_grads=os.environ.get('GPI_PE_SHARED_GRADS', '0') == '1')
        self.engine.bind(X_vo=self.X)
        self.m = torch.zeros(self.q_n, dtype=torch.float32, device=dev)
        self.v = torch.zeros_like(self.m)
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr = torch.zeros(1, dtype=torch.float32, device=dev)
        self._lr_host = None
        self._lr_source = lr_source
        P, G = self.flat.P, self.flat.G
        self.adam = L.AdamDesc(p=P.data_ptr() + 4 * self.q_off, g=G.data_ptr() + 4 * self.q_off, m=self.m.data_ptr(),
                               v=self.v.data_ptr(), n=self.q_n, lr=self.lr.data_ptr(), step=self.step_ctr.data_ptr(),
                               beta1=betas[0], beta2=betas[1], eps=eps)
        self.seed = host_seed()
        self.rng_off = torch.zeros(1, dtype=torch.int64, device=dev)
        self.adam.rng_offset = self.rng_off.data_ptr()
        dp = self.engine.dp
        self.adam.rng_advance = max((self.N * self.engine.dz + 3) // 4 + 1, (dp.drop_numel + 3) // 4 + 1)
        # gradient delivery of the q rows (fp64 accumulator -> G, accumulator zeroed) fused with their Adam
        self.epi = L.StepEpilogueDesc(gacc=self.flat.gacc.data_ptr() + 8 * self.q_off, grad=G.data_ptr() + 4 * self.q_off,
                                      n=self.q_n, flags=L.FINALIZE_ZERO)
        self.done_ctr = torch.zeros(1, dtype=torch.int32, device=dev)

    def _sync_decoder(self):
        src_flat = getattr(self.model.f, '_gpi_flat', None)
        if src_flat is not None and all(src_flat.owns(p) for p in self._src):
            o = src_flat.offset(self._src[0])
            # one copy when the decoder's parameters sit in the model's flat buffer with the same relative
            # offsets (alignment padding included) as in the shadow's
            if all(src_flat.offset(p) - o == self.flat.offset(d) for p, d in zip(self._src, self.shadow.parameters())):
                self.flat.P[:self.n_dec].copy_(src_flat.P[o:o + self.n_dec])
                return
        with torch.no_grad():
            for d, s in zip(self.shadow.parameters(), self._src):
                d.copy_(s)

    def _sync_lr(self):
        self._set_lr(float(self._lr_source()))

    def _set_lr(self, lr):
        if lr != self._lr_host:
            self.lr.fill_(lr)
            self._lr_host = lr

    def update(self, eps=None, sync=True, sync_lr=True):
        """One PredictionEnsemble iteration; returns (elbo, logL, KLD) device scalars (no host sync).
        sync=False skips refreshing the shadow decoder (the model has not changed since the last
        update: the later iterations of one PredictionEnsemble.update(numIter) call)."""
        lib, st = L.lib(), L.stream_handle()
        if sync:
            self._sync_decoder()
        if sync_lr:
            self._sync_lr()
        ez = self.engine.eps_z()
        if eps is not None:
            ez.copy_(eps)
        else:
            L.check(lib.gpi_randn(L.ptr(ez), ez.numel(), self.seed, L.ptr(self.rng_off), 5, st), 'randn pe')
        if self.engine.has_dropout:     # the reference calls the decoder in train mode (components.py:371)
            self.engine.draw_dropout(st, self.seed, L.ptr(self.rng_off), 6)
        self.engine.forward(st, compute_value=False, running='defer')
        t = self.engine.ws.terms
        from .engine import T_LX0, T_KL_Q2
        logL, kld = t[T_LX0].float(), t[T_KL_Q2].float()
        self.engine.backward(st)
        if self.engine.shared_grads:
            self.engine.finalize(self.flat.G, step=self.step_ctr, stream=st, zero_acc=True)
            L.check(lib.gpi_adam(C.byref(self.adam), st), 'pe adam')
        else:
            # only the q rows carry gradients: their delivery and Adam in one launch
            L.check(lib.gpi_step_epilogue_adam(C.byref(self.epi), C.byref(self.adam), L.ptr(self.done_ctr), st),
                    'pe gradient + adam')
        return logL - kld, logL, kld


class ConcurrentPredictionEnsemble(object):
    """The notebook loop's PredictionEnsemble.update(numIter) (training.py:419) on its own stream,
    concurrently with the NEXT training step.

    The reference's iteration n runs training step n (theta_n -> theta_{n+1}) and then the PE group
    PE(n): numIter iterations on theta_{n+1}.  The PE reads the decoder only through its shadow copy
    and writes only its own q_z rows; step n+1 reads theta_{n+1} and writes theta_{n+2} in its final
    Adam.  So once the shadow holds theta_{n+1}, PE(n) and step n+1 are independent:

        for n: cpe.before_step(); step.step(); cpe.after_step(); [cpe.catch_up(); monitor]; schedulers
        cpe.catch_up()

    before_step() (main stream) waits for the PE group in flight and folds its BN running statistics
    into model.f, refreshes the shadow with the current parameters when a PE group is owed and records
    an event; after_step() replays that group (PE(n-1), on theta_n) on the side stream behind the event,
    concurrently with the step just enqueued.  catch_up() runs every owed group on the main stream
    (before reading q_z: the reference's monitoring at iteration n follows PE(n)).  Parameters and q_z
    take exactly the sequential schedule's values (the same launches on the same inputs); the PE's
    learning rate is the one the reference's PE(n) sees (read at after_step of iteration n, before that
    iteration's scheduler steps).  The BN running buffers of model.f (never read by the training
    computation: the reference has no eval mode) receive each PE group's exponential-average updates
    one training step later than in the reference: the PE's calls update a zeroed staging copy (the
    shadow's buffers), folded in as running = (1 - m)^k running + staged, num_batches_tracked += k."""

    def __init__(self, engine, n_iter=3, momentum=0.1):
        if not engine.running_stage:
            raise ValueError('ConcurrentPredictionEnsemble needs PredictionEnsembleEngine(running_stage=True)')
        self.e = engine
        self.n_iter = int(n_iter)
        self.momentum = float(momentum)
        self.stream = torch.cuda.Stream()
        self.ev_a, self.ev_b = torch.cuda.Event(), torch.cuda.Event()
        stage = dict(engine.shadow.named_buffers())
        dst = dict(engine.model.f.named_buffers())
        names = [n for n in stage if n.endswith('running_mean') or n.endswith('running_var')]
        self._fl_dst = [dst[n] for n in names]
        self._fl_stage = [stage[n] for n in names]
        nb = [n for n in stage if n.endswith('num_batches_tracked')]
        self._nb_dst = [dst[n] for n in nb]
        self._nb_stage = [stage[n] for n in nb]
        self.graph = None
        self.in_flight = False       # a PE group launched on the side stream, not yet waited for
        self.steps = 0               # training steps enqueued
        self.groups = 0              # PE groups enqueued: PE(j) for j < groups
        self._launch = False
        self._lr_next = None         # learning rate of the next owed group (host value)

    def _group(self):
        for i in range(self.n_iter):
            self.e.update(sync=False, sync_lr=False)

    def capture(self):
        """The group captured as a HIP graph (after one warm-up group on the side stream; the PE state
        it changes is restored).  Call before training starts."""
        e = self.e
        state = [e.flat.P, e.m, e.v, e.step_ctr, e.rng_off] + self._fl_stage + self._nb_stage
        torch.cuda.synchronize()
        saved = [t.clone() for t in state]
        with torch.cuda.stream(self.stream):
            self._group()
        torch.cuda.synchronize()
        for t, v in zip(state, saved):
            t.copy_(v)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._group()
        torch.cuda.synchronize()

    def _fold(self):
        if self._fl_dst:
            torch._foreach_mul_(self._fl_dst, (1.0 - self.momentum) ** self.n_iter)
            torch._foreach_add_(self._fl_dst, self._fl_stage)
            torch._foreach_zero_(self._fl_stage)
        if self._nb_dst:
            torch._foreach_add_(self._nb_dst, self._nb_stage)
            torch._foreach_zero_(self._nb_stage)

    def _wait(self):
        if self.in_flight:
            torch.cuda.current_stream().wait_event(self.ev_b)
            self._fold()
            self.in_flight = False

    def _refresh(self):
        self.e._sync_decoder()
        if self._lr_next is not None:
            self.e._set_lr(self._lr_next)

    def before_step(self):
        self._wait()
        self._launch = self.groups < self.steps
        if self._launch:
            self._refresh()
            self.ev_a.record(torch.cuda.current_stream())

    def after_step(self):
        self.steps += 1
        if self._launch:
            self.stream.wait_event(self.ev_a)
            with torch.cuda.stream(self.stream):
                if self.graph is not None:
                    self.graph.replay()
                else:
                    self._group()
            self.ev_b.record(self.stream)
            self.in_flight = True
            self.groups += 1
            self._launch = False
        self._lr_next = float(self.e._lr_source())

    def catch_up(self):
        """Main stream: every owed PE group done (and folded): q_z is the reference's after PE(steps-1)."""
        self._wait()
        while self.groups < self.steps:
            self._refresh()
            if self.graph is not None:
                self.graph.replay()
            else:
                self._group()
            self._fold()
            self.groups += 1
