"""GenerativeModel (reference bottleneck/generative.py:10-644) on the native ELBO engine.

Same constructor, registration API, ``elbo(...)`` signature and return value
(a 0-d autograd tensor whose ``backward()`` fills every parameter's ``.grad``)
as the reference, so training.py's loop (zero_grad -> elbo -> backward ->
Adam.step) runs unchanged.  The armortized-unsupervised and supervised
(independent_X) terms run as ONE fused native step (gpi/engine.py); the
per-term methods are kept for callers that use them individually.
"""
import copy

import numpy as np
import torch

import lamp.modules
from bottleneck.components import VariationalApproximation
from bottleneck.utils import DiagonalGaussianLogLikelihood
from gpi.engine import ElboEngine
from gpi.flat import FlatParameters
from gpi.native import anchor, set_flat, engine_for
from gpi import _lib as L
from gpi import vo as gvo
from gpi.engine import rom_call, ROM_NN
from gpi.predictive import predictive_y

SHARED_PREFIXES = ('f.', 'g.', 'gp.', 'encoder.')


class _ElboFunction(torch.autograd.Function):

    @staticmethod
    def forward(ctx, a, engine):
        ctx.engine = engine
        return engine.forward()

    @staticmethod
    def backward(ctx, grad_out):
        e = ctx.engine
        e.backward()
        tmp = torch.empty_like(e.flat.G)
        e.finalize(tmp, zero_acc=True)      # every finalize leaves the fp64 accumulator zeroed
        tmp.mul_(-grad_out)                 # engine gradients are d(-elbo)/dtheta
        e.flat.deliver(tmp)
        return None, None


class GenerativeModel(lamp.modules.BaseModule):

    def __init__(self, f, g, gp, writer=None, *, dtype, device):
        super().__init__()
        self.writer = writer
        self.f = f
        self.g = g
        self.gp = gp
        self.encoder = None
        self.q_z = torch.nn.ModuleDict()
        self.q_X = torch.nn.ModuleDict()
        self._dtype = dtype
        self._device = device
        self._datasets = dict()
        self.VO = None
        self.disable_elbo_vo = False
        self.disable_elbo_supervised = False
        self.disable_elbo_unsupervised = False
        self.manual_logging = False
        self.manual_log = {'elbo_supervised': [], 'elbo_unsupervised': [], 'elbo_vo': []}
        self._independent_X = gp.independent_X
        self.config = {'reconstruct_log_eff_property': True}
        self._tensorboard_logging_interval = 1
        self.preprocess_y_fct = None
        self._flat = None

    # ------------------------------------------------------------ plumbing
    def set(self, ckey, value):
        if ckey not in self.config:
            raise KeyError('{} is not a valid property for the generative model'.format(ckey))
        self.config[ckey] = value

    @property
    def tensorboard_logging_interval(self):
        return self._tensorboard_logging_interval

    @tensorboard_logging_interval.setter
    def tensorboard_logging_interval(self, value):
        assert isinstance(value, int) and value > 0
        self._tensorboard_logging_interval = value

    def _add_scalar(self, tag, value, global_step):
        if self.writer is not None and np.mod(global_step, self._tensorboard_logging_interval) == 0:
            self.writer.add_scalar(tag, value, global_step=global_step)

    @property
    def datasets(self):
        return self._datasets

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    @property
    def dim_effective_property(self):
        return self.g.dim_effective_property

    @property
    def dim_y(self):
        return self.g.dim_out

    @property
    def dim_latent(self):
        return self.f.dim_latent

    def register_encoder(self, encoder):
        self.encoder = encoder

    def init_by_encoder(self, encoder):
        for qz in self.q_z.values():
            qz.init_by_encoder(encoder)

    def get_encoder_decoder_states(self):
        if self.encoder is None:
            raise RuntimeError('Encoder is not set - cannot return encoder state')
        return self.encoder.state(), self.f.state()

    def set_encoder_decoder_states(self, results):
        if self.encoder is None:
            raise Exception('The encoder is not set')
        self.encoder.load(results.encoder_state)
        self.f.load(results.decoder_state)

    # ------------------------------------------------------------ datasets
    def register_supervised_data(self, dataset):
        X = dataset.get('X')
        self.q_z['supervised'] = VariationalApproximation(self.dim_latent, X.shape[0], X=X)
        if self._independent_X:
            self.q_X['supervised'] = VariationalApproximation(self.dim_effective_property, X.shape[0], X=X)
        self._datasets['supervised'] = dataset
        self._flat = None

    def register_unsupervised_data(self, dataset, create_variational_approximation=True):
        if create_variational_approximation:
            X = dataset.get('X')
            self.q_z['unsupervised'] = VariationalApproximation(self.dim_latent, X.shape[0], X=X)
        self._datasets['unsupervised'] = dataset
        self._flat = None

    def register_virtual_observables(self, dataset, VO):
        X = dataset.get('X')
        self.q_z['vo'] = VariationalApproximation(self.dim_latent, X.shape[0], X=X)
        if self._independent_X:
            self.q_X['vo'] = VariationalApproximation(self.dim_effective_property, X.shape[0], X=X)
        self.VO = VO
        self._datasets['vo'] = dataset
        self._flat = None

    def register_datasets(self, datasets, VO=None, create_unsupervised_variational_approximation=True):
        if datasets.get('supervised'):
            self.register_supervised_data(datasets['supervised'])
        if datasets.get('unsupervised'):
            self.register_unsupervised_data(datasets['unsupervised'],
                                            create_variational_approximation=create_unsupervised_variational_approximation)
        if datasets.get('vo'):
            if VO is None:
                raise ValueError('If datasets contains vo, need to pass virtual ensemble')
            self.register_virtual_observables(datasets['vo'], VO)

    # ------------------------------------------------------------ native
    def native_flat(self):
        """Flatten every parameter into one device buffer (shared first, per-sample q last)."""
        params = list(self.named_parameters())
        if self._flat is None or not all(self._flat.owns(p) for _, p in params) or \
                len(params) != len(self._flat.params):
            dev = params[0][1].device
            self._flat = FlatParameters(params, dev, shared_prefixes=SHARED_PREFIXES, err_slot=True)
            set_flat(self, self._flat)
        return self._flat

    def _elbo_engine(self, B_u, N_s, normalize, N_vo=0, vo_holdoff=False, q_unsup=None):
        flat = self.native_flat()
        return engine_for(self, ('elbo', B_u, N_s, N_vo, bool(vo_holdoff), bool(normalize), id(flat),
                                 q_unsup is not None, bool(self.config['reconstruct_log_eff_property'])),
                          lambda: ElboEngine(self, B_u, N_s, normalize=normalize, N_vo=N_vo, vo_holdoff=vo_holdoff,
                                             q_unsup=q_unsup))

    @staticmethod
    def _host_seed():
        # Philox seed from torch's CPU generator: torch.manual_seed reproducibility, no device sync
        return int(torch.randint(0, 2 ** 62, (1,)).item())

    def _run_engine(self, engine, X_u=None, X_s=None, Y=None, F=None, eps=None, X_vo=None, F_vo=None, dropout=None):
        """eps (optional, injected noise): (eps_z [B, d_z], eps_X [N_s + N_vo, n_T] (None in lockX)
        [, eps_y [N_vo, d_y]]).  dropout (optional, injected Dropout2d channel scales):
        {'enc': {conv name: [B_u, cout]}, 'dec': {conv name: [B, cout]}} -- otherwise drawn on the
        device for every call, as nn.Dropout2d does in train mode."""
        if engine.has_dropout:
            if dropout is not None:
                from gpi.engine import inject_dropout
                inject_dropout(engine.dropout_views(), dropout)
            else:
                engine.draw_dropout(L.stream_handle(), self._host_seed())
        if eps is None:
            engine.eps_z().normal_()
            if engine.N_ex > 0:
                engine.eps_x().normal_()
        else:
            engine.eps_z().copy_(eps[0])
            if engine.N_ex > 0:
                engine.eps_x().copy_(eps[1])
        if engine.N_vo > 0 and not engine.vo_holdoff:
            # y ~ reparametrize(VO.mean, VO.logsigma) (generative.py:356)
            if self.VO is None or self.VO.mean is None:
                raise RuntimeError('the virtual observables have no posterior yet: call update_virtual_observables')
            gvo.gauss_sample(engine.y_vo(), self.VO.mean, self.VO.logsigma,
                             eps=eps[2] if (eps is not None and len(eps) > 2) else None, seed=self._host_seed(),
                             sub=11)
        engine.bind(X_u=X_u, X_s=X_s, Y=Y, F=F, X_vo=X_vo, F_vo=F_vo)
        return _ElboFunction.apply(anchor(self, engine.flat.P.device), engine)

    def _log_terms(self, engine, step, prefix_map=None):
        if self.writer is None or np.mod(step, self._tensorboard_logging_interval) != 0:
            return
        for k, v in engine.terms().items():
            self.writer.add_scalar('objective/' + k, v, global_step=step)

    # ------------------------------------------------------------ virtual observables
    @torch.no_grad()
    def update_virtual_observables(self, N_monte_carlo, Y_mean=None, Y_std=None, return_mean_stddev=False, step=None,
                                   Resample=True, eps=None):
        """generative.py:182-222 on the native path.  The per-VO-sample Python loop of MC ROM
        solves becomes three launches over all N_vo * N_mc samples: q_X['vo'] draws
        (gpi_gauss_sample), coarse ROM solves (gpi_rom FORWARD, coarse solutions only) and the
        moments of y = W u + exp(logsigma_y) eps (gpi_vo_moments); VO.update then runs the batched
        precision / conditioning kernels.  ``eps`` optionally injects (eps_X [N_vo * N_mc, n_T],
        eps_y [N_vo * N_mc, d_y])."""
        if step is None:
            raise ValueError('We now require a step parameter to be passed to update VOs')
        if (Y_mean is None or Y_std is None) and not self._independent_X:
            # lockX (generative.py:202-204): y = g(gp(z)) with z ~ q_z['vo'] -- gpi_gp_sample without
            # the logsigma_X noise, coarse solves, moments.  eps = (eps_Z [N_vo * N_mc, d_z], eps_y)
            ds = self._datasets['vo']
            if int(N_monte_carlo) > 2048:
                raise RuntimeError('Batchsize will lead to memory issues')
            qz = self.q_z['vo']
            Y_mean, Y_std, PREC = predictive_y(self, qz.mean.detach(), qz.logsigma.detach(),
                                               ds.get('F_ROM_BC').detach(), int(N_monte_carlo),
                                               eps=(eps[0], None, eps[1]) if eps is not None else None,
                                               seed=self._host_seed(), return_prec=True)
        elif Y_mean is None or Y_std is None:
            ds = self._datasets['vo']
            N, N_mc = ds.N, int(N_monte_carlo)
            if N_mc > 2048:
                raise RuntimeError('Batchsize will lead to memory issues')
            F = ds.get('F_ROM_BC').detach()
            L.require_device(F)
            qx = self.q_X['vo']
            rom = self.g.rom
            dx = qx.dim
            xs = torch.empty(N * N_mc, dx, dtype=torch.float32, device=F.device)
            gvo.gauss_sample(xs, qx.mean.detach().contiguous(), qx.logsigma.detach().contiguous(), rep=N_mc,
                             eps=eps[0] if eps is not None else None, seed=self._host_seed(), sub=12)
            key = (F.data_ptr(), N_mc)
            if getattr(self, '_vo_F_mc_key', None) != key:
                self._vo_F_mc = F.float().repeat_interleave(N_mc, 0).contiguous()
                self._vo_F_mc_key = key
            uc = torch.empty(N * N_mc, ROM_NN(rom.nc), dtype=torch.float32, device=F.device)
            rom_call(rom.nc, rom.refine, xs, self._vo_F_mc, False, L.ROM_FORWARD, uc=uc)
            Y_mean, Y_std, PREC = gvo.vo_moments(uc, rom.nc, rom.refine, N, N_mc,
                                                 logsig_y=self.g.logsigmas_y.detach().contiguous(),
                                                 eps=eps[1] if eps is not None else None, seed=self._host_seed())
        else:
            PREC = 1 / (Y_std ** 2)
        if Resample:
            self.VO.resample()
        self.VO.update(Y_mean, PREC, step, writer=self.writer)
        if step is not None and self.writer is not None:
            Yv = self._datasets['vo'].get('Y').detach()
            err = torch.mean(torch.sqrt(torch.sum((self.VO.mean - Yv) ** 2, 1)) / torch.sqrt(torch.sum(Yv ** 2, 1)))
            self.writer.add_scalar('vo/q_y_mean_rel_err', err.item(), global_step=step)
            self.writer.add_scalar('vo/likelihood', torch.mean(DiagonalGaussianLogLikelihood(
                Yv, self.VO.mean, 2 * self.VO.logsigma)), global_step=step)
        if return_mean_stddev:
            return Y_mean, Y_std

    # ------------------------------------------------------------ ELBO
    def elbo(self, step, vo_holdoff=False, disable_vo=False, armortized_bs=None, normalize=False, l1_penalty=None,
             l2_penalty=None, eps=None, dropout=None):
        """Reference generative.py:247-287.  ``eps`` optionally injects the reparametrisation
        noise as (eps_z [B_u + N_s + N_vo, d_z], eps_X [N_s + N_vo, n_T][, eps_y [N_vo, d_y]]);
        ``dropout`` the Dropout2d channel scales (see _run_engine)."""
        assert not (armortized_bs is not None and self.encoder is None)
        if l1_penalty is not None:
            raise NotImplementedError
        N_vo = 0
        X_vo = F_vo = None
        if self._datasets.get('vo') and not disable_vo and not self.disable_elbo_vo:
            dsv = self._datasets['vo']
            X_vo = dsv.get('X').detach().contiguous()
            F_vo = dsv.get('F_ROM_BC').detach().contiguous()
            N_vo = X_vo.shape[0]
        X_u = None
        B_u = 0
        q_unsup = None
        if self._datasets.get('unsupervised') and not self.disable_elbo_unsupervised and self.encoder is None:
            # elbo_unsupervised (generative.py:515-544): per-sample q_z['unsupervised'] over the whole set
            q_unsup = self.q_z['unsupervised']
            X_u = self._datasets['unsupervised'].get('X').detach().contiguous()
            B_u = X_u.shape[0]
        elif self._datasets.get('unsupervised') and not self.disable_elbo_unsupervised:
            if armortized_bs is None:
                raise ValueError('If armortized learning is used, we need to provide a batch size')
            X_u = self._datasets['unsupervised'].get('X', random_subset=armortized_bs).detach().contiguous()
            B_u = X_u.shape[0]
        N_s = 0
        X_s = Y = F = None
        if self._datasets.get('supervised') and not self.disable_elbo_supervised:
            ds = self._datasets['supervised']
            X_s, Y, F = ds.get('X').detach(), ds.get('Y').detach(), ds.get('F_ROM_BC').detach()
            if self.preprocess_y_fct is not None:
                raise NotImplementedError('preprocess_y_fct is not supported on the native path')
            N_s = X_s.shape[0]
        if B_u == 0 and N_s == 0 and N_vo == 0:
            return 0
        engine = self._elbo_engine(B_u, N_s, normalize, N_vo=N_vo, vo_holdoff=vo_holdoff, q_unsup=q_unsup)
        elbo = self._run_engine(engine, X_u, X_s, Y, F, eps, X_vo=X_vo, F_vo=F_vo, dropout=dropout)
        if l2_penalty is not None:
            pen = sum(torch.norm(p) for p in self.f.parameters())
            if self.encoder is not None:
                pen = pen + sum(torch.norm(p) for p in self.encoder.parameters())
            elbo = elbo - l2_penalty * pen
            self._add_scalar('elbo_l2_penalty', pen, step)
        if self.writer is not None:
            self._log_terms(engine, step)
            self._add_scalar('elbo', elbo, step)
        return elbo

    def elbo_unsupervised_armortized(self, X, step, encoder=None, return_reconstruction=False, normalize=False):
        if self.disable_elbo_unsupervised:
            return 0
        if self.encoder is None:
            raise RuntimeError('Cannot use armortized inference, if encoder has not been registered')
        if 'unsupervised' in self.q_z:
            raise RuntimeError("Cannot use armortized inference, if q_z['unsupervised'] has been registered")
        if return_reconstruction:
            raise NotImplementedError
        engine = self._elbo_engine(X.shape[0], 0, normalize)
        return self._run_engine(engine, X_u=X.detach().contiguous().float())

    def elbo_supervised(self, X, Y, step, normalize=False):
        if self.disable_elbo_supervised:
            return 0
        F = self._datasets['supervised'].get('F_ROM_BC').detach()
        engine = self._elbo_engine(0, X.shape[0], normalize)
        return self._run_engine(engine, X_s=X.detach(), Y=Y.detach(), F=F)

    def random_field_likelihood(self, predict, target):
        if not isinstance(predict, tuple):
            raise NotImplementedError('binary fields are not on the ELBO path')
        if self.config['reconstruct_log_eff_property']:
            return DiagonalGaussianLogLikelihood(target, predict[0], 2 * predict[1])
        return DiagonalGaussianLogLikelihood(torch.exp(target), torch.exp(predict[0]), 2 * predict[1])

    @torch.no_grad()
    def record(self, step):
        if self.writer is None:
            return
        if self._independent_X and 'supervised' in self.q_X:
            self.writer.add_scalar('Monitoring/logEffProp_sup_mean', torch.mean(self.q_X['supervised'].mean), step)
            self.writer.add_scalar('Monitoring/logEffProp_sup_sigma', torch.mean(self.q_X['supervised'].logsigma),
                                   step)
        self.writer.add_scalar('Monitoring/S_avg_precisions', torch.mean(torch.exp(-2 * self.g.logsigmas_y)), step)

    def extract_discriminative_model(self, *, FromLatentEncoding, duplicate, encoder=None):
        if not duplicate:
            raise RuntimeError('We are only able to return duplicates')
        enc = None if FromLatentEncoding else copy.deepcopy(encoder if encoder is not None else self.encoder)
        return DiscriminativeModel(encoder=enc, gp=copy.deepcopy(self.gp.extract_deterministic_map(duplicate=True)),
                                   g=copy.deepcopy(self.g), dim_latent=self.dim_latent)

    def forward(self, X, Y):
        raise NotImplementedError


class DiscriminativeModel(lamp.modules.BaseModule):
    """x -> (encoder) -> gp mean -> ROM (generative.py:605-644)."""

    def __init__(self, encoder, gp, g, dim_latent):
        super().__init__()
        if gp is None or g is None:
            raise ValueError
        self._encoder = encoder
        self._gp = gp
        self._g = g
        self._dim_latent = dim_latent

    def curtail(self):
        self._encoder = None

    def forward(self, x, F):
        if self._encoder is not None:
            x = self._encoder(x)[0]
        return self._g(self._gp(x), F=F)
