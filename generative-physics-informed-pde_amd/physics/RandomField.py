"""Gaussian random fields for log-conductivity images (reference physics/RandomField.py:13-219).

The reference assembles the dense squared-exponential covariance
C = sigma^2 exp(-|r|^2 / 2 l^2) + 1e-12 I over all pixel centres (refusing more
than 8192 pixels, RandomField.py:43-44), takes ``eigh`` and samples
mean + L gamma with L = V sqrt(Lambda) truncated to the leading modes that
explain 99.9 % of the variance ('adaptive'), or L = chol(C) (no truncation)
(RandomField.py:162-209).  On the tensor grid of pixel centres the kernel is
separable, C = sigma^2 C_y (x) C_x + 1e-12 I, so its eigenpairs are
(sigma^2 lambda_i mu_j + 1e-12, v_i (x) w_j) and a sample is

    X = mean + V_y (S o G) V_x^T,   S_ij = sqrt(sigma^2 lambda_i mu_j + 1e-12)

on the retained modes (0 elsewhere), G ~ N(0, I)[py, px]: the reference's
distribution (the Cholesky path samples N(mean, C) as well) at O(n^3) setup
instead of O(n^6), valid at 128^2 and 256^2.  Modes are ranked by eigenvalue
with a stable sort, so a truncation cut inside a group of equal eigenvalues
(lambda_i mu_j = lambda_j mu_i on square grids) keeps the lower flat index;
the reference's dense ``eigh`` keeps an arbitrary vector of that degenerate
eigenspace, so only the retained spectrum is comparable there.
``dense=True`` reproduces the reference's dense assembly for small images.
``sample_device`` draws on the GPU (gpi.fom.random_field, csrc/fom.hip).
"""
import numpy as np

ADAPTIVE_FRACTION = 0.999   # RandomField.py:190-194 (the comparison is hard-coded to 0.999)


class NormalRandomFieldSampler(object):

    def __init__(self, mean, stddev, corrlength, py, px, ly=1.0, lx=1.0, Truncation=None, dense=False):
        if stddev <= 0 or corrlength <= 0:
            raise ValueError
        self._mean, self._stddev, self._corrlength = mean, stddev, corrlength
        self._py, self._px = py, px
        self._truncation = Truncation
        self._dense = dense
        # pixel centres (RandomField.py:64-71; the y grid there starts at pixelwidth_x / 2)
        pwx, pwy = lx / px, ly / py
        self._x = np.linspace(0.5 * pwx, lx - 0.5 * pwx, px)
        self._y = np.linspace(0.5 * pwx, ly - 0.5 * pwy, py)
        self._L = None
        self._Vy = self._Vx = self._S = None
        self._dev = {}

    @classmethod
    def FromImage(cls, py, px, mean, stddev, corrlength, Truncation=None, ly=1, lx=1, dense=False):
        return cls(mean, stddev, corrlength, py, px, ly, lx, Truncation, dense)

    @property
    def dim_out(self):
        return self._py * self._px

    @property
    def dim_in(self):
        """Number of retained modes (RandomField.py:84-88)."""
        self._ensure()
        return self._L.shape[1] if self._dense else int(np.count_nonzero(self._S))

    def _truncation_index(self, eigvals_desc):
        t = self._truncation
        if isinstance(t, str):
            if t.lower() != 'adaptive':
                raise ValueError(t)
            t = ADAPTIVE_FRACTION
        if isinstance(t, float):
            assert 0.9 < t < 0.9999
            ve = np.cumsum(eigvals_desc) / np.sum(eigvals_desc)
            t = int(np.argmax(ve > ADAPTIVE_FRACTION))
        if not isinstance(t, (int, np.integer)) or t >= self.dim_out or t < 1:
            raise ValueError(t)
        return int(t)

    def _corr1d(self, t):
        return np.exp(-0.5 * (t[:, None] - t[None, :]) ** 2 / self._corrlength ** 2)

    def _ensure(self):
        if self._L is None and self._S is None:
            self._assemble()

    def _assemble(self):
        if self._dense:
            if self.dim_out > 8192:
                raise RuntimeError('dense sampler is capped at 8192 pixels (RandomField.py:43-44)')
            X, Y = np.meshgrid(self._x, self._y)
            P = np.stack([X.ravel(), Y.ravel()], 1)
            r2 = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
            C = self._stddev ** 2 * np.exp(-0.5 * r2 / self._corrlength ** 2) + 1e-12 * np.eye(P.shape[0])
            if self._truncation is None:
                self._L = np.linalg.cholesky(C)
            else:
                w, V = np.linalg.eigh(C)
                w, V = w[::-1], V[:, ::-1]
                k = self._truncation_index(w)
                self._L = V[:, :k] * np.sqrt(w[:k])[None, :]
            return
        lam, Vy = np.linalg.eigh(self._corr1d(self._y))
        mu, Vx = np.linalg.eigh(self._corr1d(self._x))
        lam, mu = np.clip(lam, 0.0, None), np.clip(mu, 0.0, None)
        ev = self._stddev ** 2 * lam[:, None] * mu[None, :] + 1e-12
        if self._truncation is None:
            S = np.sqrt(ev)
        else:
            order = np.argsort(-ev.ravel(), kind='stable')
            k = self._truncation_index(ev.ravel()[order])
            S = np.zeros(ev.size)
            S[order[:k]] = np.sqrt(ev.ravel()[order[:k]])
            S = S.reshape(ev.shape)
        self._Vy, self._Vx, self._S = Vy, Vx, S

    def factors(self):
        """(V_y [py, py], V_x [px, px], S [py, px]) of the separable form."""
        if self._dense:
            raise RuntimeError('dense sampler has no separable factors')
        self._ensure()
        return self._Vy, self._Vx, self._S

    def covariance(self):
        """The sampler's covariance over the flattened image (row-major), for tests."""
        self._ensure()
        if self._dense:
            return self._L @ self._L.T
        B = np.kron(self._Vy, self._Vx) * self._S.ravel()[None, :]
        return B @ B.T

    def sample(self, gamma=None, batch_size=None, rng=None):
        """Host draw.  gamma: mode coefficients (dense: [dim_in]; separable: [py, px] mode grid)."""
        rng = rng or np.random
        self._ensure()
        n = 1 if batch_size is None else batch_size
        if self._dense:
            G = rng.normal(size=(n, self._L.shape[1])) if gamma is None else np.asarray(gamma).reshape(n, -1)
            X = (self._mean + G @ self._L.T).reshape(n, self._py, self._px)
        else:
            G = rng.normal(size=(n, self._py, self._px)) if gamma is None else np.asarray(gamma).reshape(
                n, self._py, self._px)
            X = self._mean + np.matmul(np.matmul(self._Vy, G * self._S), self._Vx.T)
        return X[0] if batch_size is None else X

    def sample_device(self, batch_size, seed=0, sub=0, gamma=None, device='cuda'):
        """Device draw of batch_size images [N, py, px] fp64 (Philox(seed, sub) or given gamma)."""
        import torch
        from gpi import fom
        Vy, Vx, S = self.factors()
        key = str(device)
        if key not in self._dev:
            t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=device)
            self._dev[key] = (t(Vy), t(Vx.T), t(S))
        ly, lxt, sc = self._dev[key]
        if gamma is not None:
            gamma = torch.as_tensor(gamma, dtype=torch.float64).reshape(batch_size, self._py, self._px)
        return fom.random_field(batch_size, self._py, self._px, self._mean, 1.0, ly, lxt, scale=sc, gamma=gamma,
                                seed=seed, sub=sub, device=device)
