"""Variational approximations, effective-property map, ROM operator, W interpolator,
prediction ensemble, predictive analysis (reference bottleneck/components.py:13-654)."""
import copy

import numpy as np
import torch

import lamp.modules
from bottleneck.ROM import ROM
from bottleneck.utils import UnitGaussianKullbackLeiblerDivergence
from gpi.native import RomOperatorFunction


class PhysicsResolutionInterpolator(lamp.modules.BaseModule):
    """W: coarse P1 basis evaluated at the fine free nodes (components.py:13-67).
    Closed-form on the structured mesh (physics/grid.py) instead of FEniCS point location."""

    def __init__(self, physics, mode='ManualInterpolation', only_free_dofs=True, dtype=None, device=None):
        super().__init__()
        W = physics['fom'].grid.prolongation_from(physics['rom'].grid, only_free=only_free_dofs)   # [d_y, n_c]
        self._W = torch.tensor(W.T, dtype=dtype or torch.float64, device=device)                  # [n_c, d_y]

    @property
    def dim_in(self):
        return self._W.shape[0]

    @property
    def dim_out(self):
        return self._W.shape[1]

    def forward(self, x):
        return torch.matmul(x, self._W)


class VariationalApproximation(lamp.modules.BaseModule):
    """Per-sample diagonal Gaussian q (components.py:71-197)."""

    def __init__(self, dim, N, X=None, *, dtype=None, device=None, requires_grad=True):
        super().__init__()
        if X is not None:
            dtype = dtype or X.dtype
            device = device or X.device
        self._logsigma = torch.nn.Parameter(torch.zeros(N, dim, dtype=dtype, device=device),
                                            requires_grad=requires_grad)
        self._mean = torch.nn.Parameter(torch.zeros(N, dim, dtype=dtype, device=device),
                                        requires_grad=requires_grad)
        self._X = X
        self._N = N
        self._dim = dim

    @property
    def N(self):
        return self._N

    @property
    def dim(self):
        return self._dim

    @property
    def dtype(self):
        return self._mean.dtype

    @property
    def device(self):
        return self._mean.device

    @property
    def mean(self):
        return self._mean

    @mean.setter
    def mean(self, value):
        assert tuple(value.shape) == (self._N, self._dim)
        self._mean.data.copy_(value)

    @property
    def logsigma(self):
        return self._logsigma

    @logsigma.setter
    def logsigma(self, value):
        assert tuple(value.shape) == (self._N, self._dim)
        self._logsigma.data.copy_(value)

    def init(self, mean, logsigma):
        self.mean = mean
        self.logsigma = logsigma

    def init_standard_deviation(self, stddev):
        self._logsigma.data.fill_(float(np.log(stddev)))

    def freeze(self):
        self._mean.requires_grad = False
        self._logsigma.requires_grad = False

    def freeze_mean(self):
        self._mean.requires_grad = False

    def unfreeze(self):
        self._mean.requires_grad = True
        self._logsigma.requires_grad = True

    def init_by_encoder(self, encoder):
        with torch.no_grad():
            mu, ls = encoder(self._X.detach())
            self._mean.data.copy_(mu)
            self._logsigma.data.copy_(ls)

    def sample(self, batch_size=1):
        if batch_size != 1:
            raise NotImplementedError
        return self._mean + torch.exp(self._logsigma) * torch.randn_like(self._logsigma)

    def sample_batch_component(self, index, batch_size=1):
        if batch_size > 2048:
            raise RuntimeError('Batchsize will lead to memory issues')
        eps = torch.randn(batch_size, self.dim, dtype=self.dtype, device=self.device)
        return self._mean[index, :] + torch.exp(self._logsigma[index, :]) * eps

    def KLD(self):
        return UnitGaussianKullbackLeiblerDivergence(self._mean, 2 * self._logsigma)

    def entropy(self, sample=None):
        # constant uses N, not N*dim (components.py:196) -- kept for parity
        return torch.sum(self._logsigma) + self.N * 0.5 * (np.log(2 * np.pi) + 1)


class EffectivePropertyMap(lamp.modules.BaseModule):
    """z -> log effective properties (components.py:201-256); 0 hidden layers."""

    def __init__(self, latent_dim, dim_effective_property, num_hidden_layers=0, independent_X=True, *, dtype=None,
                 device=None):
        super().__init__()
        if num_hidden_layers:
            raise NotImplementedError('hidden layers in the effective-property map are not on the ELBO path')
        self.fc = torch.nn.Linear(latent_dim, dim_effective_property)
        if independent_X:
            self.logsigmas_X = torch.nn.Parameter(torch.ones(dim_effective_property))
        self._latent_dim = latent_dim
        self._independent_X = independent_X
        self._to(dtype=dtype, device=device)

    @property
    def independent_X(self):
        return self._independent_X

    @property
    def dim_in(self):
        return self._latent_dim

    def forward(self, z):
        if self._independent_X:
            return self.fc(z), self.logsigmas_X.expand(z.shape[0], -1)
        return self.fc(z)

    def forward_mean(self, z):
        return self.fc(z)

    def propagate_samples(self, z):
        if not self._independent_X:
            return self.forward(z)
        mean, ls = self.forward(z)
        return mean + torch.exp(ls) * torch.randn_like(ls)

    def extract_deterministic_map(self, *, duplicate=True):
        if not duplicate:
            raise NotImplementedError
        return copy.deepcopy(self.fc)


class ReducedOrderModelOperator(lamp.modules.BaseModule):
    """effprop -> (mu_y = W solve(K(exp(effprop)+1e-8), F), logsigma_y) (components.py:260-323)."""

    def __init__(self, rom, W, *, dtype=None, device=None):
        super().__init__()
        self.W = W
        self.rom = rom
        self._dtype = dtype
        self._device = device
        self.logsigmas_y = torch.nn.Parameter(torch.ones(W.shape[0]))
        self._to(dtype=dtype, device=device)

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    @property
    def dim_effective_property(self):
        return self.rom.Vc_dim

    @property
    def dim_in(self):
        return self.dim_effective_property

    @property
    def dim_out(self):
        return self.W.shape[0]

    def forward_mean(self, effprop, F):
        mu, _ = RomOperatorFunction.apply(effprop, F, self.rom.nc, self.rom.refine, False)
        return mu

    def forward(self, effprop, F):
        return self.forward_mean(effprop, F), self.logsigmas_y.repeat(effprop.shape[0], 1)

    def propagate_samples(self, effprops, F):
        mean, ls = self.forward(effprops, F)
        return mean + torch.exp(ls) * torch.randn_like(ls)

    @classmethod
    def FromPhysics(cls, physics, *, dtype=None, device=None):
        W = torch.tensor(physics['W'], dtype=dtype, device=device)          # [d_y, n_c]
        if W.shape[0] < W.shape[1]:
            raise ValueError
        rom = ROM.FromPhysics(physics['rom'], dtype=dtype, device=device)
        return cls(rom, W, dtype=dtype, device=device)


class PredictionEnsemble(object):
    """Validation q_z fitted against the frozen decoder (components.py:326-393).  update() runs the
    native PredictionEnsembleEngine (gpi/predictive.py): decoder-only ELBO + backward + Adam on the
    q_z rows, no host sync unless a writer records the values.  The torch Adam object is kept for
    the scheduler wrapper, which reads and rescales its learning rate."""

    def __init__(self, model, dataset, scheduler_wrapper, lr=1e-2, writer=None):
        self._model = model
        self._dataset = dataset
        X = dataset.get('X')
        self._q_z = VariationalApproximation(model.dim_latent, X.shape[0], X)
        self._optimizer = torch.optim.Adam(self._q_z.parameters(), lr=lr)
        self._scheduler_wrapper = scheduler_wrapper
        self._scheduler_wrapper.register_optimizer(self._optimizer, 'validation')
        self.writer = writer
        self._engine = None

    def set_lr_manually(self, lr):
        raise NotImplementedError

    @property
    def q_z(self):
        return self._q_z

    @property
    def model(self):
        return self._model

    @property
    def dataset(self):
        return self._dataset

    def _native(self):
        if self._engine is None:
            from gpi.predictive import PredictionEnsembleEngine
            self._engine = PredictionEnsembleEngine(self._model, self._q_z, self._dataset.get('X'),
                                                    lambda: self._optimizer.param_groups[0]['lr'])
        return self._engine

    def update(self, numIter=1, record=True, step=None, eps=None):
        """components.py:365-388.  ``eps`` optionally injects the q_z noise per iteration
        (a list of numIter [N, d_z] tensors)."""
        e = self._native()
        for n in range(numIter):
            elbo, logL, KLD = e.update(eps=eps[n] if eps is not None else None, sync=n == 0)
            if n == numIter - 1:
                if record and self.writer is not None:
                    self.writer.add_scalar('PredictionEnsemble/elbo', elbo.item(), global_step=step)
                    self.writer.add_scalar('PredictionEnsemble/logL', logL.item(), global_step=step)
                    self.writer.add_scalar('PredictionEnsemble/KLD', KLD.item(), global_step=step)
                    self.writer.add_scalar('PredictionEnsemble/AvgLatentStddev',
                                           torch.mean(torch.exp(self._q_z.logsigma)), global_step=step)
                # the native engine did this optimizer's steps: tell torch's scheduler hook (as
                # FusedElboStep does), so it does not warn of a scheduler step before any optimizer step
                self._optimizer._opt_called = True
                self._scheduler_wrapper.step('validation', None, None, None, elbo)
        return elbo

    def __repr__(self):
        return 'PredictionEnsemble | Wraps a dataset with {} points for validation purposes'.format(self._dataset.N)


class DataPair(object):
    """A monitored scalar series (components.py:396-424's role): (iteration, value) records, optionally
    mirrored to a tensorboard-style writer under '<label>/<name>'."""

    def __init__(self, writer=None, label='', name=None):
        if writer is not None and name is None:
            raise ValueError('Required to provide a name for the writer')
        self._records = []
        self._writer, self._tag = writer, '%s/%s' % (label, name)

    @property
    def iteration(self):
        return [i for i, _ in self._records]

    @property
    def value(self):
        return [v for _, v in self._records]

    def append(self, iteration, value):
        self._records.append((iteration, value))
        if self._writer is not None:
            self._writer.add_scalar(self._tag, value, global_step=iteration)

    def min(self):
        return min(self.value)

    def max(self):
        return max(self.value)

    def final(self):
        return self._records[-1][1]


class Analysis(object):
    """Predictive evaluation of a q (components.py:427-654).  eval_all_y runs every sample's MC
    predictive at once on the native path (gpi/predictive.py: gp draws, ROM, moments, scores);
    the per-index methods keep the reference's sample-level semantics."""

    def __init__(self, q, model, dataset, identifier=''):
        self._q = q
        self._model = model
        self._dataset = dataset
        self.description = None
        self.data = dict()
        for item in ['relerr_x', 'relerr_y', 'logscore_x', 'logscore_y', 'r2_y']:
            self.data[item] = DataPair(writer=self._model.writer, label=getattr(dataset, 'label', ''), name=item)

    @property
    def dataset(self):
        return self._dataset

    @classmethod
    def FromPredictionEnsemble(cls, pe):
        return cls(pe.q_z, pe.model, pe.dataset)

    @classmethod
    def FromEncoder(cls, model, dataset):
        """q_z of every sample = the encoder's (mean, logsigma) (components.py:443-453), held fixed."""
        with torch.no_grad():
            mean, logsigma = model.encoder(dataset.get('X'))
        q = VariationalApproximation(mean.shape[1], mean.shape[0], dataset.get('X'), dtype=mean.dtype,
                                     device=mean.device, requires_grad=False)
        q.init(mean, logsigma)
        return cls(q, model, dataset)

    @property
    def X(self):
        return self._dataset.get('X')

    @property
    def Y(self):
        return self._dataset.get('Y')

    @property
    def F(self):
        return self._dataset.get('F_ROM_BC')

    @torch.no_grad()
    def sample_predictive_y(self, N_monte_carlo, index):
        Z_samples = self._q.sample_batch_component(index, batch_size=N_monte_carlo)
        X_samples = self._model.gp.propagate_samples(Z_samples)
        return self._model.g.propagate_samples(X_samples, self.F[index, :].unsqueeze(0).expand(
            N_monte_carlo, self.F.shape[1]).contiguous())

    @torch.no_grad()
    def sample_predictive_x(self, N_monte_carlo, index):
        Z_samples = self._q.sample_batch_component(index, batch_size=N_monte_carlo)
        return self._model.f.propagate_samples(Z_samples)

    def eval_all(self, N_monte_carlo, iteration):
        self.relative_error_x(N_monte_carlo, iteration)
        self.eval_all_y(N_monte_carlo, iteration)
        self.predictive_log_probability_x(N_monte_carlo, iteration)

    @torch.no_grad()
    def eval_all_y(self, N_monte_carlo, iteration=None, return_mean_std=False, eps=None):
        """components.py:493-524 for all samples at once; ``eps`` optionally injects
        (eps_z [N*N_mc, d_z], eps_x [N*N_mc, d_x], eps_y [N*N_mc, d_y])."""
        from gpi.predictive import predictive_y, predictive_scores
        Y = self.Y.detach().float().contiguous()
        y_mean, y_std = predictive_y(self._model, self._q.mean, self._q.logsigma, self.F.detach(), N_monte_carlo,
                                     eps=eps)
        relerr_y, logscore_y, r2_y = predictive_scores(Y, y_mean, y_std)
        if iteration is None:
            if return_mean_std:
                # the reference refuses this combination as well (components.py:516-517)
                raise RuntimeError('eval_all_y: return_mean_std=True needs an iteration to record the scores at')
            return logscore_y, r2_y, relerr_y
        self.data['relerr_y'].append(iteration, relerr_y)
        self.data['logscore_y'].append(iteration, logscore_y)
        self.data['r2_y'].append(iteration, r2_y)
        if return_mean_std:
            return y_mean, y_std

    @torch.no_grad()
    def relative_error_y(self, N_monte_carlo, iteration=None, ReturnValue=False):
        relerr = self.eval_all_y(N_monte_carlo)[2]
        if iteration is None:
            return relerr
        self.data['relerr_y'].append(iteration, relerr)
        if ReturnValue:
            return relerr

    @torch.no_grad()
    def predictive_log_probability_y(self, N_monte_carlo, iteration=None):
        logp = self.eval_all_y(N_monte_carlo)[0]
        if iteration is None:
            return logp
        self.data['logscore_y'].append(iteration, logp)

    def _x_moments(self, N_monte_carlo):
        """Per sample: mean and unbiased std over N_monte_carlo decoder draws of the field.  One
        decoder call per sample, as the reference's per-index loop (components.py:472-491):
        train-mode BatchNorm normalises over exactly those N_monte_carlo draws."""
        for index in range(self._q.N):
            draws = self.sample_predictive_x(N_monte_carlo, index).reshape(N_monte_carlo, -1)
            yield index, draws.mean(0), draws.std(0)

    def _record(self, key, value, iteration, ReturnValue=True):
        if iteration is None:
            return value
        self.data[key].append(iteration, value)
        return value if ReturnValue else None

    @torch.no_grad()
    def relative_error_x(self, N_monte_carlo, iteration=None, ReturnValue=False):
        """Mean over samples of ||E[x] - x|| / ||x|| (components.py:526-546)."""
        X = self.X.reshape(self._q.N, -1)
        err = [float(torch.linalg.vector_norm(m - X[i]) / torch.linalg.vector_norm(X[i]))
               for i, m, _ in self._x_moments(N_monte_carlo)]
        return self._record('relerr_x', float(np.mean(err)), iteration, ReturnValue)

    @torch.no_grad()
    def predictive_log_probability_x(self, N_monte_carlo, iteration=None):
        """Mean over samples and pixels of the Gaussian log-density of x under the MC moments
        (components.py:548-570)."""
        X = self.X.reshape(self._q.N, -1)
        half_log2pi = 0.5 * float(np.log(2 * np.pi))
        lp = [float(torch.mean(-torch.log(sd) - 0.5 * ((X[i] - m) / sd) ** 2 - half_log2pi))
              for i, m, sd in self._x_moments(N_monte_carlo)]
        return self._record('logscore_x', float(np.mean(lp)), iteration, ReturnValue=False)
