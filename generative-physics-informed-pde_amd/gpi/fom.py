"""Launchers of the FOM data-generation kernels (csrc/fom.hip, include/gpi.h).

``fom_solve`` replaces the per-sample PETSc LU of DataLoader.assemble (utils/data.py:72-103 ->
physics/LinearElliptic.py:85-101) by one batched preconditioned-CG launch; ``random_field`` draws
log-conductivity images with the separable restatement of NormalRandomFieldSampler
(physics/RandomField.py:162-209).  Device tensors in, device tensors out; the only host
synchronisation is the optional convergence check.
"""
import ctypes as C

import torch

from . import _lib as L


def _p(t):
    return t.data_ptr() if t is not None else None


def fom_workspace(n_fine):
    k = L.lib().gpi_fom_workspace(int(n_fine))
    if k < 0:
        L.check(-1, 'gpi_fom_workspace')
    return k


def default_max_iter(n_fine):
    return 50 * int(n_fine) + 200


class FomResult(object):

    def __init__(self, y, iters, flag):
        self.y = y
        self.iters = iters
        self.flag = flag

    def check(self):
        """Host sync: raise if any sample did not reach the tolerance within max_iter."""
        k = int(self.flag.item())
        if k:
            raise L.NativeError('FOM solve: %d sample(s) did not converge' % k)
        return self


def fom_solve(x_dg, bc, n_fine, rtol=1e-13, max_iter=None, y0=None, chunk=1024):
    """Free-node FOM solutions y [N, d_y] (fp64) of -div(exp(x_dg) grad u) = 0 with the NDP data bc [N, 4].

    x_dg [N, 2 n_fine^2] is the DG0 log-conductivity (X_DG layout); y0 an optional initial guess."""
    L.require_device(x_dg)
    L.require_device(bc)
    N = x_dg.shape[0]
    n = int(n_fine)
    assert n >= 2 and x_dg.shape == (N, 2 * n * n) and bc.shape == (N, 4)
    dy = (n + 1) * (n - 1)
    x_dg = x_dg.contiguous().double()
    bc = bc.contiguous().double()
    dev = x_dg.device
    if y0 is not None:
        assert y0.shape == (N, dy)
        y = y0.to(device=dev, dtype=torch.float64).contiguous().clone()
    else:
        y = torch.empty(N, dy, dtype=torch.float64, device=dev)
    iters = torch.zeros(N, dtype=torch.int32, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = fom_workspace(n)
    mi = default_max_iter(n) if max_iter is None else int(max_iter)
    chunk = max(1, min(int(chunk), N)) if N else 1
    work = torch.empty(chunk * ws, dtype=torch.float64, device=dev) if N else None
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        d = L.FomDesc(n_fine=n, n=b - a, flags=L.FOM_WARM if y0 is not None else 0, max_iter=mi,
                      logkappa=_p(x_dg[a:b]), bc=_p(bc[a:b]), rtol=float(rtol), y=_p(y[a:b]), work=_p(work),
                      iters=_p(iters[a:b]), flag=_p(flag))
        L.check(L.lib().gpi_fom_solve(C.byref(d), L.stream_handle()), 'fom solve')
    return FomResult(y, iters, flag)


def random_field(n, py, px, mean, stddev, ly, lxt, scale=None, gamma=None, seed=0, sub=0, device=None):
    """x [n, py, px] fp64 = mean + stddev * ly (scale o G) lxt with G ~ N(0, I) (Philox) or gamma."""
    dev = torch.device(device) if device is not None else ly.device
    ly = ly.to(device=dev, dtype=torch.float64).contiguous()
    lxt = lxt.to(device=dev, dtype=torch.float64).contiguous()
    L.require_device(ly)
    assert ly.shape == (py, py) and lxt.shape == (px, px)
    if scale is not None:
        scale = scale.to(device=dev, dtype=torch.float64).contiguous()
        assert scale.shape == (py, px)
    if gamma is not None:
        gamma = gamma.to(device=dev, dtype=torch.float64).contiguous()
        assert gamma.shape == (n, py, px)
    x = torch.empty(n, py, px, dtype=torch.float64, device=dev)
    work = torch.empty_like(x)
    d = L.RandomFieldDesc(py=py, px=px, n=n, pad0=0, mean=float(mean), stddev=float(stddev), ly=_p(ly), lxt=_p(lxt),
                          scale=_p(scale), gamma=_p(gamma), seed=int(seed), sub=int(sub), work=_p(work), x=_p(x))
    L.check(L.lib().gpi_random_field(C.byref(d), L.stream_handle()), 'random field')
    return x
