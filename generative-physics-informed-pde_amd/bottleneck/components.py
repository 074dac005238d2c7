"""Variational approximations, effective-property map, ROM operator, W interpolator,
prediction ensemble (reference bottleneck/components.py:13-393)."""
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
    """Validation q_z fitted against the frozen decoder (components.py:326-393)."""

    def __init__(self, model, dataset, scheduler_wrapper, lr=1e-2, writer=None):
        self._model = model
        self._dataset = dataset
        X = dataset.get('X')
        self._q_z = VariationalApproximation(model.dim_latent, X.shape[0], X)
        self._optimizer = torch.optim.Adam(self._q_z.parameters(), lr=lr)
        self._scheduler_wrapper = scheduler_wrapper
        self._scheduler_wrapper.register_optimizer(self._optimizer, 'validation')
        self.writer = writer

    @property
    def q_z(self):
        return self._q_z

    @property
    def model(self):
        return self._model

    @property
    def dataset(self):
        return self._dataset

    def _elbo(self, X):
        Z = self._q_z.sample()
        logL = self._model.random_field_likelihood(self._model.f(Z), X)
        return logL, self._q_z.KLD()

    def update(self, numIter=1, record=True, step=None):
        X = self._dataset.get('X')
        for n in range(numIter):
            logL, KLD = self._elbo(X.detach())
            elbo = logL - KLD
            self._optimizer.zero_grad()
            (-elbo).backward()
            self._optimizer.step()
            if n == numIter - 1:
                if record and self.writer is not None:
                    self.writer.add_scalar('PredictionEnsemble/elbo', elbo.item(), global_step=step)
                    self.writer.add_scalar('PredictionEnsemble/logL', logL.item(), global_step=step)
                    self.writer.add_scalar('PredictionEnsemble/KLD', KLD.item(), global_step=step)
                self._scheduler_wrapper.step('validation', None, None, None, elbo)

    def __repr__(self):
        return 'PredictionEnsemble | Wraps a dataset with {} points for validation purposes'.format(self._dataset.N)
