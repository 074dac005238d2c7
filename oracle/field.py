"""Restatement of the reference's Gaussian random-field sampler (physics/RandomField.py:13-219).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  numpy float64, dense: the
covariance over all pixel centres (FromImage :61-71, including the y grid that
starts at pixelwidth_x / 2), the 1e-12 jitter (:176), eigh with the spectrum
flipped to descending order (:178-181), the 'adaptive' truncation at the first
index whose explained variance exceeds 0.999 (:183-194, the comparison is
hard-coded to 0.999) or the Cholesky factor without truncation (:205-207).
"""
import numpy as np


def pixel_centres(py, px, ly=1.0, lx=1.0):
    pwx, pwy = lx / px, ly / py
    x = np.linspace(0 + 0.5 * pwx, lx - 0.5 * pwx, px)
    y = np.linspace(0 + 0.5 * pwx, ly - 0.5 * pwy, py)
    X, Y = np.meshgrid(x, y)
    return np.hstack([X.reshape(-1, 1), Y.reshape(-1, 1)])


def covariance(py, px, stddev, corrlength, ly=1.0, lx=1.0):
    P = pixel_centres(py, px, ly, lx)
    C = np.zeros((P.shape[0], P.shape[0]))
    for i, row in enumerate(P):
        r2 = np.sum(np.square(row - P), 1)
        C[i, :] = stddev ** 2 * np.exp(-0.5 * r2 / corrlength ** 2)
    return C + 1e-12 * np.eye(C.shape[0])


def kl_factor(C, truncation=None):
    """L with samples mean + L gamma (RandomField.py:172-207)."""
    w, V = np.linalg.eigh(C)
    w = np.flip(w, 0)
    V = np.fliplr(V)
    if truncation is None:
        return np.linalg.cholesky(C)
    t = truncation
    if isinstance(t, str):
        assert t.lower() == 'adaptive'
        t = 0.999
    if isinstance(t, float):
        assert 0.9 < t < 0.9999
        ve = np.cumsum(w) / np.sum(w)
        t = int(np.argmax(ve > 0.999))
    if t >= C.shape[0] or t < 1:
        raise ValueError(t)
    return V[:, :t].dot(np.diag(np.sqrt(w[:t])))
