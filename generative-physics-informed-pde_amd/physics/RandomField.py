"""Gaussian random fields for log-conductivity images (reference physics/RandomField.py:13-219).

The reference assembles the dense squared-exponential covariance over all
pixel centres (refusing more than 8192 pixels, RandomField.py:43-44) and
factorises it (Cholesky or KL truncation at 99.9% variance).  On a tensor
grid the SE kernel is separable, C = sigma^2 C_y (x) C_x, so a sample is
mean + sigma L_y G L_x^T with G ~ N(0, I)[py, px]: the same distribution
(without the 1e-12 jitter / truncation) at O(n^3) instead of O(n^6), valid
at 128^2 and 256^2.  ``dense=True`` reproduces the reference's dense
Cholesky path for small images.
"""
import numpy as np


class NormalRandomFieldSampler(object):

    def __init__(self, mean, stddev, corrlength, py, px, ly=1.0, lx=1.0, Truncation=None, dense=False):
        if stddev <= 0 or corrlength <= 0:
            raise ValueError
        self._mean, self._stddev, self._corrlength = mean, stddev, corrlength
        self._py, self._px = py, px
        self._truncation = Truncation
        self._dense = dense
        # pixel centres (RandomField.py:64-71; the y grid there starts at pixelwidth_x/2 -- identical for square pixels)
        self._x = (np.arange(px) + 0.5) * (lx / px)
        self._y = (np.arange(py) + 0.5) * (ly / py)
        self._Lx = self._Ly = self._L = None

    @classmethod
    def FromImage(cls, py, px, mean, stddev, corrlength, Truncation=None, ly=1, lx=1, dense=False):
        return cls(mean, stddev, corrlength, py, px, ly, lx, Truncation, dense)

    @property
    def dim_out(self):
        return self._py * self._px

    def _factor1d(self, t):
        C = np.exp(-0.5 * (t[:, None] - t[None, :]) ** 2 / self._corrlength ** 2)
        w, V = np.linalg.eigh(C)
        w = np.clip(w, 0.0, None)
        return V * np.sqrt(w)[None, :]

    def _assemble(self):
        if self._dense:
            if self.dim_out > 8192:
                raise RuntimeError('dense sampler is capped at 8192 pixels (RandomField.py:43-44)')
            X, Y = np.meshgrid(self._x, self._y)
            P = np.stack([X.ravel(), Y.ravel()], 1)
            r2 = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
            C = self._stddev ** 2 * np.exp(-0.5 * r2 / self._corrlength ** 2) + 1e-12 * np.eye(P.shape[0])
            self._L = np.linalg.cholesky(C)
        else:
            self._Lx = self._factor1d(self._x)
            self._Ly = self._factor1d(self._y)

    def sample(self, gamma=None, batch_size=None, rng=None):
        rng = rng or np.random
        if self._L is None and self._Lx is None:
            self._assemble()
        n = 1 if batch_size is None else batch_size
        if self._dense:
            G = rng.normal(size=(n, self.dim_out)) if gamma is None else np.asarray(gamma).reshape(n, -1)
            X = (self._mean + G @ self._L.T).reshape(n, self._py, self._px)
        else:
            G = rng.normal(size=(n, self._py, self._px)) if gamma is None else np.asarray(gamma).reshape(
                n, self._py, self._px)
            X = self._mean + self._stddev * np.matmul(np.matmul(self._Ly, G), self._Lx.T)
        return X[0] if batch_size is None else X
