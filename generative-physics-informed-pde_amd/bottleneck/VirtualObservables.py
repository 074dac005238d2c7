"""Virtual observables (reference bottleneck/VirtualObservables.py) on the native path.

Same classes, constructors and call contracts as the reference
(QuerryPointEnsemble.FromDataSet, QuerryEnsemble.FromQuerryPointEnsemble,
VirtualObservablesEnsemble(QPE, QE, dtype, device), .update(G, PREC, step),
.mean / .vars / .logsigma, per-VO .querry.Gamma / .alpha / .mean / .vars).

What changes is where the work runs.  The reference assembles every query
with FEniCS + numpy per VO sample and conditions each VO sample with a torch
fp64 Cholesky in a Python loop.  Here the ensemble keeps ONE batched device
layout -- Gamma [N, m, d_y] and alpha [N, m] (fp64), posterior mean / vars
[N, d_y] (fp64) -- built by gpi_vo_query (csrc/vo.hip) in one launch and
updated by gpi_vo_precision + gpi_vo_condition in one launch set; the
per-sample objects hold views of it.  No host synchronisation, no CPU
fallback (gpi/_lib.py raises without a GPU).

Samplers on the native path, concatenated in the reference's order:
CoarseGrainedResidualSampler (infinite precision), FluxConstrainSampler
(learnable precision), GaussianSketchingSampler and RadialBasisFunctionSampler
(infinite precision, test functions redrawn on the device at every resample).
The energy VOs (host numpy loops in the reference) are not native and raise.
"""
import numpy as np
import torch

from gpi import _lib as L
from gpi import vo as V

ALPHA0 = V.ALPHA0
BETA0 = V.BETA0


def _grid_sizes(physics):
    """(n_fine, nc) of a physics dict {'fom', 'rom', 'W'} or of a fom physics + W."""
    return physics['fom'].grid.n, physics['rom'].grid.n


def _host_seed():
    # device Philox seeded from torch's CPU generator (torch.manual_seed reproducible, no device sync)
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _same_device(a, b):
    a, b = torch.device(a), torch.device(b)
    return a.type == b.type and (a.index is None or b.index is None or a.index == b.index)


# ---------------------------------------------------------------------------
class QuerryPoint(object):
    """One VO location: log-conductivity per DG0 cell ``x`` and its BC (VirtualObservables.py:8-69)."""

    def __init__(self, physics, x, bc):
        assert isinstance(x, np.ndarray)
        assert not isinstance(physics, dict)
        assert physics.dim_in == x.size
        assert x.ndim == 1
        self._physics = physics
        self._x = x
        self._bc = bc
        self._K = None
        self._f = None

    @property
    def physics(self):
        return self._physics

    @property
    def bc(self):
        return self._bc

    @property
    def x(self):
        # log-transformed conductivity (reference naming)
        return self._x

    @property
    def u(self):
        """NDP boundary values u0..u3."""
        return self._bc.u if hasattr(self._bc, 'u') else np.asarray(self._bc, dtype=np.float64)

    @property
    def K(self):
        if self._K is None:
            self._assemble_system()
        return self._K

    @property
    def f(self):
        if self._f is None:
            self._assemble_system()
        return self._f

    @property
    def dim_in(self):
        return self._x.size

    @property
    def dim_out(self):
        return self._physics.dim_out

    def _assemble_system(self):
        # setup-side host assembly (reference: FEniCS), only for construct_querry_weak_galerkin
        self._K, self._f = self._physics.assemble_system(np.exp(self._x), bc=self._bc, only_free_dofs=True)

    def construct_querry_weak_galerkin(self, V_):
        assert V_.shape[0] == self.K.shape[0]
        return V_.T @ self.K, V_.T @ self.f


class QuerryPointEnsemble(object):

    def __init__(self, QPs):
        self._QPs = QPs
        self._dev = {}

    def X(self, dtype, device):
        return torch.tensor(np.stack([qp.x for qp in self._QPs]), dtype=dtype, device=device)

    def device_batch(self, device):
        """(x_dg [N, n_DG] fp64, bc [N, 4] fp64) on ``device`` (cached)."""
        key = str(device)
        if key not in self._dev:
            x = torch.tensor(np.stack([qp.x for qp in self._QPs]), dtype=torch.float64, device=device)
            u = torch.tensor(np.stack([qp.u for qp in self._QPs]), dtype=torch.float64, device=device)
            self._dev[key] = (x.contiguous(), u.contiguous())
        return self._dev[key]

    def __iter__(self):
        yield from self._QPs

    def __getitem__(self, item):
        return self._QPs[item]

    def __len__(self):
        return len(self._QPs)

    @property
    def dim_out(self):
        return self._QPs[0].dim_out

    @property
    def N(self):
        return len(self)

    @classmethod
    def FromDataSet(cls, dataset, physics):
        assert not isinstance(physics, dict)
        X_DG = dataset.get('X_DG')
        BCE = dataset.get('BCE')
        assert X_DG.dtype == torch.double
        return cls([QuerryPoint(physics, X_DG[n, :].detach().cpu().numpy().flatten(), BCE[n])
                    for n in range(dataset.N)])


# ---------------------------------------------------------------------------
class BaseSampler(object):

    def __init__(self, qp):
        self._qp = qp

    @property
    def m(self):
        raise NotImplementedError

    @property
    def qp(self):
        return self._qp

    @property
    def dim(self):
        return self.qp.dim_out

    flags = 0

    def sample(self):
        raise NotImplementedError

    @property
    def precision_mask(self):
        raise NotImplementedError

    @property
    def is_constant(self):
        raise NotImplementedError

    @property
    def fixed_precision(self):
        return np.all(self.precision_mask < 0)

    def __call__(self, *args, **kwargs):
        return self.sample(*args, **kwargs)

    def _native(self, flags, device):
        """Gamma, alpha (device fp64) of this query point for ``flags`` (batch of one)."""
        qp = self._qp
        n = int(round(np.sqrt(qp.dim_in / 2)))
        x = torch.tensor(qp.x, dtype=torch.float64, device=device).view(1, -1)
        u = torch.tensor(qp.u, dtype=torch.float64, device=device).view(1, 4)
        g, a = V.vo_query(x, u, n, self._nc, flags)
        return g[0], a[0]


class CoarseGrainedResidualSampler(BaseSampler):
    """Gamma = W^T K_ff, alpha = W^T f_eff, infinite precision (VirtualObservables.py:297-321)."""

    flags = L.VO_CGR

    def __init__(self, qp, W, device=None):
        super().__init__(qp=qp)
        self._V = W
        self._nc = int(round(np.sqrt(W.shape[1]))) - 1
        self._device = device if device is not None else torch.device('cuda')
        self._cache = None

    @property
    def m(self):
        return (self._nc + 1) ** 2

    @property
    def is_constant(self):
        return True

    @property
    def precision_mask(self):
        return -np.ones(self.m)

    def _sample(self):
        return self._V

    def sample_V(self):
        return self._V

    def sample(self):
        if self._cache is None:
            self._cache = self._native(L.VO_CGR, self._device)
        return self._cache


class FluxConstrainSampler(BaseSampler):
    """Flux rows (FluxConstraintReducedOrderModel, bottleneck/flux.py), learnable precision
    (VirtualObservables.py:323-349)."""

    flags = L.VO_FLUX

    def __init__(self, qp, FluxConstrain, device=None):
        super().__init__(qp=qp)
        if not FluxConstrain.initialized:
            raise RuntimeError('Initialize flux-constrain first')
        self._fc = FluxConstrain
        self._nc = FluxConstrain.nc
        self._device = device if device is not None else torch.device('cuda')
        self._cache = None

    @property
    def m(self):
        return 2 * self._nc * self._nc

    @property
    def is_constant(self):
        return True

    @property
    def precision_mask(self):
        return np.ones(self.m)

    def sample(self):
        if self._cache is None:
            self._cache = self._native(L.VO_FLUX, self._device)
        return self._cache

    def _sample(self):
        raise NotImplementedError


class _TestFunctionSampler(BaseSampler):
    """Galerkin rows V^T K_ff / V^T f_eff from random test functions, redrawn on every resample
    (not constant), infinite precision.  V is drawn on the device (gpi_vo_galerkin)."""

    kind = None

    def __init__(self, qp, N_aux, length=0.0, device=None):
        super().__init__(qp=qp)
        self._N = int(N_aux)
        self._length = float(length)
        self._device = device if device is not None else torch.device('cuda')

    @property
    def m(self):
        return self._N

    @property
    def is_constant(self):
        return False

    @property
    def precision_mask(self):
        return -np.ones(self.m)

    def sample(self):
        qp = self._qp
        n = int(round(np.sqrt(qp.dim_in / 2)))
        x = torch.tensor(qp.x, dtype=torch.float64, device=self._device).view(1, -1)
        u = torch.tensor(qp.u, dtype=torch.float64, device=self._device).view(1, 4)
        dy = (n + 1) * (n - 1)
        g = torch.empty(1, self._N, dy, dtype=torch.float64, device=self._device)
        a = torch.empty(1, self._N, dtype=torch.float64, device=self._device)
        V.vo_galerkin(g, a, 0, self._N, x, u, n, self.kind, length=self._length, seed=_host_seed())
        return g[0], a[0]

    def _sample(self):
        raise NotImplementedError('test functions are drawn on the device and not materialised')


class GaussianSketchingSampler(_TestFunctionSampler):
    """V ~ N(0, 1) on the free nodes (VirtualObservables.py:230-258)."""

    kind = L.VO_TEST_GAUSS

    def __init__(self, qp, N_aux, device=None):
        super().__init__(qp, N_aux, device=device)


class RadialBasisFunctionSampler(_TestFunctionSampler):
    """V = exp(-|x - r0|^2 / l^2) at the free nodes, r0 ~ U(0,1)^2 per test function
    (VirtualObservables.py:172-228, fawkes/Expressions.py:26-31)."""

    kind = L.VO_TEST_RBF

    def __init__(self, qp, l, N_aux, device=None):
        assert l is not None
        super().__init__(qp, N_aux, length=l() if callable(l) else l, device=device)


class ConcatenatedSamplers(BaseSampler):

    def __init__(self, samplers):
        super().__init__(qp=None)
        self._samplers = samplers

    @property
    def qp(self):
        return self._samplers[0].qp

    @property
    def flags(self):
        f = 0
        for s in self._samplers:
            f |= s.flags
        return f

    @property
    def m(self):
        return sum(s.m for s in self._samplers)

    @property
    def is_constant(self):
        return all(s.is_constant for s in self._samplers)

    @property
    def precision_mask(self):
        return np.concatenate([s.precision_mask for s in self._samplers])

    def sample(self):
        cache = [s() for s in self._samplers]
        return torch.cat([c[0] for c in cache], 0), torch.cat([c[1] for c in cache], 0)


# ---------------------------------------------------------------------------
class LinearQuerry(object):
    """Gamma / alpha of one VO sample (VirtualObservables.py:353-448); fp64 device tensors."""

    def __init__(self, querry_point, sampler, dtype, device, Gamma=None, alpha=None, ensemble=None, index=None):
        self._sampler = sampler
        self._querry_point = querry_point
        self._ensemble, self._index = ensemble, index
        self._Gamma = None
        self._GammaTransposed = None
        self._alpha = None
        self._dtype = dtype
        self._device = device
        if Gamma is not None:
            self.Gamma, self.alpha = Gamma, alpha
            self.GammaTransposed = Gamma.t()
        else:
            self.resample(ForceResample=True)

    @property
    def Gamma(self):
        return self._Gamma

    @Gamma.setter
    def Gamma(self, value):
        assert value.dtype == torch.double
        self._Gamma = value

    @property
    def GammaTransposed(self):
        return self._GammaTransposed

    @GammaTransposed.setter
    def GammaTransposed(self, value):
        assert value.dtype == torch.double
        self._GammaTransposed = value

    @property
    def alpha(self):
        return self._alpha

    @alpha.setter
    def alpha(self, value):
        assert value.dtype == torch.double
        self._alpha = value

    @property
    def device(self):
        return self._device

    @property
    def dtype(self):
        return self._dtype

    @property
    def m(self):
        return self.Gamma.shape[0]

    def resample(self, ForceResample=False):
        if self._ensemble is not None:
            # rows live in the ensemble's batched layout: redraw this sample's random rows in place
            if not self._sampler.is_constant:
                self._ensemble._draw_aux(index=self._index)
            return
        if not self._sampler.is_constant or ForceResample:
            Gamma, alpha = self._sampler()
            self.Gamma = torch.as_tensor(Gamma, dtype=torch.double, device=self.device)
            self.alpha = torch.as_tensor(alpha, dtype=torch.double, device=self.device)
            self.GammaTransposed = self.Gamma.t()

    @property
    def dim_out(self):
        return self.Gamma.shape[1]

    @property
    def precision_mask(self):
        return self._sampler.precision_mask

    def add_galerkin_sampler(self, sampler):
        pass

    def add_flux_constraint(self):
        raise NotImplementedError


class QuerryEnsemble(object):
    """All LinearQuerries of the VO dataset; ``gamma`` [N, m, d_y] / ``alpha`` [N, m] is the batched
    device layout the native kernels read (each querry's Gamma is a view of it)."""

    def __init__(self, querries, dtype, device, gamma=None, alpha=None):
        self._querries = querries
        self._dtype = dtype
        self._device = device
        self._gamma = gamma
        self._alpha = alpha
        self._aux = []

    def __len__(self):
        return len(self._querries)

    @property
    def N(self):
        return len(self)

    @property
    def m(self):
        return sum(q.m for q in self._querries)

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    @property
    def precision_mask(self):
        return self._querries[0].precision_mask

    @property
    def gamma(self):
        if self._gamma is None or any(q.Gamma.data_ptr() != self._gamma[n].data_ptr()
                                      for n, q in enumerate(self._querries)):
            self._gamma = torch.stack([q.Gamma for q in self._querries]).contiguous()
            self._alpha = torch.stack([q.alpha for q in self._querries]).contiguous()
            self.generation = getattr(self, 'generation', 0) + 1
        return self._gamma

    @property
    def alpha(self):
        self.gamma
        return self._alpha

    def resample(self, ForceResample=False):
        if self._aux:
            self._draw_aux()
            return
        for q in self:
            q.resample(ForceResample=ForceResample)

    def _draw_aux(self, index=None):
        """Redraw the test-function rows (Gaussian sketch / RBF) of all samples, or of one, on the device."""
        x, u = self._qpe.device_batch(self._device)
        sl = slice(None) if index is None else slice(index, index + 1)
        g, a = self._gamma[sl], self._alpha[sl]
        for row0, m_aux, kind, length in self._aux:
            V.vo_galerkin(g, a, row0, m_aux, x[sl], u[sl], self._n_fine, kind, length=length, seed=_host_seed())

    @property
    def dim_out(self):
        return self._querries[0].dim_out

    def __getitem__(self, item):
        return self._querries[item]

    def __iter__(self):
        yield from self._querries

    @classmethod
    def FromQuerryPointEnsemble(cls, QuerryPointEnsemble, physics, CGR, flux, N_gaussian, N_rbf, l_rbf=None, *,
                                dtype=None, device=None):
        """VirtualObservables.py:498-543: sampler rows CGR, flux, Gaussian sketch, RBF per VO sample,
        assembled for the whole ensemble in one launch per sampler kind."""
        assert isinstance(physics, dict)
        W = physics['W']
        if W is None:
            raise NotImplementedError('need to provide W (as numpy array)')
        assert W.shape[0] > W.shape[1]
        assert dtype is not None
        assert device is not None
        if N_rbf > 0:
            assert l_rbf is not None
        n_fine, nc = _grid_sizes(physics)
        dy = (n_fine + 1) * (n_fine - 1)
        flags = (L.VO_CGR if CGR else 0) | (L.VO_FLUX if flux else 0)
        m0 = V.vo_rows(n_fine, nc, flags) if flags else 0
        m = m0 + N_gaussian + N_rbf
        if m == 0:
            raise ValueError('no sampler selected')
        x, u = QuerryPointEnsemble.device_batch(device)
        N = len(QuerryPointEnsemble)
        gamma = torch.empty(N, m, dy, dtype=torch.float64, device=device)
        alpha = torch.empty(N, m, dtype=torch.float64, device=device)
        if m0:
            g0, a0 = V.vo_query(x, u, n_fine, nc, flags)
            gamma[:, :m0].copy_(g0)
            alpha[:, :m0].copy_(a0)
        aux = []
        if N_gaussian > 0:
            aux.append((m0, N_gaussian, L.VO_TEST_GAUSS, 0.0))
        if N_rbf > 0:
            aux.append((m0 + N_gaussian, N_rbf, L.VO_TEST_RBF, float(l_rbf() if callable(l_rbf) else l_rbf)))
        fluxconstr = None
        if flux:
            from bottleneck.flux import FluxConstraintReducedOrderModel
            fluxconstr = FluxConstraintReducedOrderModel(physics)
            fluxconstr.create_measures()
        ens = cls([], dtype=dtype, device=device, gamma=gamma, alpha=alpha)
        ens._qpe, ens._n_fine, ens._aux = QuerryPointEnsemble, n_fine, aux
        for n, qp in enumerate(QuerryPointEnsemble):
            samplers = []
            if CGR:
                samplers.append(CoarseGrainedResidualSampler(qp=qp, W=W, device=device))
            if flux:
                samplers.append(FluxConstrainSampler(qp, fluxconstr, device=device))
            if N_gaussian > 0:
                samplers.append(GaussianSketchingSampler(qp=qp, N_aux=N_gaussian, device=device))
            if N_rbf > 0:
                samplers.append(RadialBasisFunctionSampler(qp=qp, l=l_rbf, N_aux=N_rbf, device=device))
            sampler = samplers[0] if len(samplers) == 1 else ConcatenatedSamplers(samplers)
            ens._querries.append(LinearQuerry(qp, sampler, dtype=dtype, device=device, Gamma=gamma[n],
                                              alpha=alpha[n], ensemble=ens, index=n))
        if aux:
            ens._draw_aux()
        return ens


# ---------------------------------------------------------------------------
class BaseVirtualObservable(object):

    def __init__(self, querry_point, dtype, device):
        assert isinstance(querry_point, QuerryPoint)
        self._querry_point = querry_point
        self._dtype = dtype
        self._device = device

    @property
    def device(self):
        return self._device

    @property
    def dtype(self):
        return self._dtype

    @property
    def querry_point(self):
        return self._querry_point

    @property
    def m(self):
        raise NotImplementedError

    @property
    def d_y(self):
        return self._querry_point.dim_out

    @property
    def mean(self):
        raise NotImplementedError

    @property
    def vars(self):
        raise NotImplementedError

    def resample(self):
        raise NotImplementedError

    def update_precision(self, *args, **kwargs):
        raise NotImplementedError

    def update(self, *args, **kwargs):
        raise NotImplementedError


class VirtualObservable(BaseVirtualObservable):
    """One VO sample; ``mean`` / ``vars`` are views of the ensemble's batched posterior."""

    def __init__(self, querry, querry_point, dtype, device):
        super().__init__(querry_point, dtype, device)
        assert isinstance(querry, LinearQuerry)
        self._querry = querry
        self._mean = None
        self._vars = None
        self._vo_variances = None

    @property
    def querry(self):
        return self._querry

    @property
    def mean(self):
        return self._mean

    @property
    def vars(self):
        return self._vars

    @property
    def m(self):
        return self._querry.m

    @property
    def vo_variances(self):
        return self._vo_variances

    @vo_variances.setter
    def vo_variances(self, value):
        assert value.dtype == torch.double
        assert _same_device(value.device, self.device)
        self._vo_variances = value

    def resample(self, ForceResample=False):
        self._querry.resample(ForceResample=ForceResample)

    @torch.no_grad()
    def update(self, g, prec, iteration, *, ForceUpdate=False):
        """VirtualObservables.py:642-669 for this sample alone (batch of one native launch)."""
        if not ForceUpdate:
            raise RuntimeError
        q = self._querry
        dy = q.Gamma.shape[1]
        mean = torch.empty(1, dy, dtype=torch.float64, device=q.Gamma.device)
        vars_ = torch.empty_like(mean)
        ws = V.vo_condition(q.Gamma.unsqueeze(0).contiguous(), q.alpha.view(1, -1).contiguous(),
                            g.detach().to(torch.float32).reshape(1, dy).contiguous(),
                            prec.detach().to(torch.float32).reshape(1, dy).contiguous(),
                            self._vo_variances.contiguous(), mean, vars_)
        self._flag = ws.flag
        self._mean = mean[0]
        self._vars = vars_[0]


class BaseVirtualObservablesEnsemble(object):

    def __init__(self, QuerryPointEnsemble, virtual_observables, dtype, device):
        self._QuerryPointEnsemble = QuerryPointEnsemble
        self._dtype, self._device = dtype, device
        self._virtual_observables = virtual_observables
        m_target = self._virtual_observables[0].m
        for vo in virtual_observables:
            assert vo.m == m_target

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    @property
    def X(self):
        return self._QuerryPointEnsemble.X

    def __getitem__(self, item):
        return self._virtual_observables[item]

    def __iter__(self):
        yield from self._virtual_observables

    def __len__(self):
        return len(self._virtual_observables)

    def flush_cache(self):
        pass

    @property
    def M(self):
        return sum(a.m for a in self)

    @property
    def m(self):
        return self._virtual_observables[0].m

    @property
    def dim_out(self):
        return self[0].d_y

    @property
    def N(self):
        return len(self)

    def update_vo_precision(self, iteration):
        raise NotImplementedError

    def resample(self, ForceResample=False):
        for vo in self._virtual_observables:
            vo.resample(ForceResample=ForceResample)


class VirtualObservablesEnsemble(BaseVirtualObservablesEnsemble):
    """VirtualObservables.py:908-998 with batched device state:
    posterior mean / vars [N, d_y] fp64 (+ their model-dtype copies mean32 / logsigma32 that
    the VO ELBO term samples from), prec_beta / mean VO variances [m] fp64."""

    def __init__(self, QuerryPointEnsemble, QuerryEnsemble, dtype, device):
        vos = [VirtualObservable(q, qp, dtype=dtype, device=device)
               for q, qp in zip(QuerryEnsemble, QuerryPointEnsemble)]
        super().__init__(QuerryPointEnsemble, vos, dtype=dtype, device=device)
        self._QuerryEnsemble = QuerryEnsemble
        self._alpha_0 = ALPHA0
        self._beta_0 = BETA0
        self._prec_alpha = 0.5 * self.N + self._alpha_0
        self._prec_beta = torch.ones(self.m, dtype=torch.double, device=self.device)
        self._infinite_precision_mask = None
        self._constant_precision = None
        N, dy = self.N, self.dim_out
        self._mean64 = torch.zeros(N, dy, dtype=torch.float64, device=device)
        self._vars64 = torch.zeros(N, dy, dtype=torch.float64, device=device)
        self._mean32 = torch.zeros(N, dy, dtype=torch.float32, device=device)
        self._logsig32 = torch.zeros(N, dy, dtype=torch.float32, device=device)
        self._has_posterior = False
        self._ws = None
        self.sparse = True          # column-sparse kernels when Gamma's columns allow (CGR / flux rows)
        self._plan = None
        self._plan_key = None
        self._mean_vo_variances = self._get_mean_vo_variances()
        self._set_member_variance_values(self._mean_vo_variances)
        self._precision_initialized = False

    @property
    def fixed_precision(self):
        if self._constant_precision is None:
            self._constant_precision = bool(np.all(np.asarray(self._QuerryEnsemble[0].precision_mask) < 0))
        return self._constant_precision

    @property
    def infinite_precision_mask(self):
        if self._infinite_precision_mask is None:
            self._infinite_precision_mask = torch.tensor(np.asarray(self._QuerryEnsemble[0].precision_mask) < 0,
                                                         dtype=torch.bool, device=self.device)
        return self._infinite_precision_mask

    def _get_mean_vo_variances(self):
        mean_vars = self._prec_beta / (self._prec_alpha + 1)
        mean_vars[self.infinite_precision_mask] = 0
        return mean_vars

    def _set_member_variance_values(self, mean_vo_vars):
        for vo in self:
            vo.vo_variances = mean_vo_vars

    # ------------------------------------------------------------------ posterior
    @property
    def mean(self):
        if not self._has_posterior:
            return None
        return self._mean32.detach() if self.dtype == torch.float32 else self._mean64.to(self.dtype)

    @property
    def vars(self):
        if not self._has_posterior:
            return None
        return self._vars64.to(self.dtype)

    @property
    def logsigma(self):
        if not self._has_posterior:
            return None
        return self._logsig32 if self.dtype == torch.float32 else 0.5 * torch.log(self.vars)

    def _bind_members(self):
        for n, vo in enumerate(self):
            vo._mean = self._mean64[n]
            vo._vars = self._vars64[n]

    # ------------------------------------------------------------------ updates
    def _sparse_plan(self, gamma):
        """SparsePlan of the ensemble's Gamma (``gamma`` = qe.gamma), rebuilt when Gamma is replaced; None when
        disabled or when Gamma has test-function rows (dense, and redrawn in place by resample)."""
        qe = self._QuerryEnsemble
        if not self.sparse or getattr(qe, '_aux', None):
            return None
        key = (gamma.data_ptr(), tuple(gamma.shape), getattr(qe, 'generation', 0))
        if key != self._plan_key:
            self._plan = V.SparsePlan.build(gamma)
            self._plan_key = key
        return self._plan

    def update(self, G, PREC, iteration, writer=None):
        self.update_vo_precision(iteration, writer)
        qe = self._QuerryEnsemble
        gamma = qe.gamma
        alpha = qe._alpha
        if self._ws is None:
            self._ws = V.ConditionWorkspace(self.N, self.m, self.dim_out, gamma.device)
        V.vo_condition(gamma, alpha, G.detach().to(torch.float32).contiguous(),
                       PREC.detach().to(torch.float32).contiguous(), self._mean_vo_variances.contiguous(),
                       self._mean64, self._vars64, self._mean32, self._logsig32, ws=self._ws,
                       sparse=self._sparse_plan(gamma))
        self._has_posterior = True
        self._bind_members()
        self.flush_cache()

    def resample(self, ForceResample=False):
        self._QuerryEnsemble.resample(ForceResample=ForceResample)

    def check_flag(self):
        """Lazy replacement of torch.cholesky's error (host sync)."""
        if self._ws is not None and int(self._ws.flag.item()) != 0:
            raise RuntimeError('cholesky: a VO Lambda matrix is not positive definite')

    @torch.no_grad()
    def update_vo_precision(self, iteration, writer=None):
        if not self._precision_initialized:
            self._precision_initialized = True
            return
        if not self._has_posterior:
            raise RuntimeError
        if not self.fixed_precision:
            qe = self._QuerryEnsemble
            beta = torch.empty(self.m, dtype=torch.float64, device=self.device)
            vo_var = torch.empty_like(beta)
            inf = self.infinite_precision_mask.to(torch.int32).contiguous()
            gamma = qe.gamma
            V.vo_precision(gamma, qe._alpha, self._mean64, self._vars64, inf, beta, vo_var,
                           alpha0=self._alpha_0, beta0=self._beta_0, sparse=self._sparse_plan(gamma))
            self._prec_beta = beta
            self._mean_vo_variances = vo_var
            self._set_member_variance_values(self._mean_vo_variances)
            if writer is not None:
                writer.add_scalar('Monitor/Mean_VO_variances', torch.mean(self._mean_vo_variances),
                                  global_step=iteration)


class EnergyVirtualObservablesEnsemble(BaseVirtualObservablesEnsemble):
    """Energy VOs (VirtualObservables.py:672-793,1001-1037) run numpy loops on the host in the
    reference and are outside the native ELBO path (SURVEY.md section 8 lists the constrain VOs)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError('energy virtual observables are not on the native path')
