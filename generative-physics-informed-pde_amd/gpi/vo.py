"""Launchers of the virtual-observable kernels (csrc/vo.hip, include/gpi.h).

Every function takes device tensors, launches on the current stream and never
synchronises the host; shapes are checked here, before any launch, against
what the kernels assume.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib as L

ALPHA0 = 1e-6    # VirtualObservablesEnsemble._alpha_0 (VirtualObservables.py:919)
BETA0 = 1e-6     # ._beta_0 (:920)


def _p(t):
    return t.data_ptr() if t is not None else None


def _dev(*ts):
    for t in ts:
        if t is not None:
            L.require_device(t)


def vo_rows(n_fine, nc, flags):
    m = L.lib().gpi_vo_rows(int(n_fine), int(nc), int(flags))
    if m < 0:
        L.check(m, 'gpi_vo_rows')
    return m


def vo_query(x_dg, bc, n_fine, nc, flags):
    """Gamma [N, m, d_y], alpha [N, m] (fp64) of the CGR / flux samplers for a batch of
    DG0 log-conductivities x_dg [N, 2 n_fine^2] (fp64) and NDP BCs [N, 4]."""
    _dev(x_dg, bc)
    N = x_dg.shape[0]
    assert x_dg.shape == (N, 2 * n_fine * n_fine) and bc.shape == (N, 4)
    m = vo_rows(n_fine, nc, flags)
    dy = (n_fine + 1) * (n_fine - 1)
    x_dg = x_dg.contiguous().double()
    bc = bc.contiguous().double()
    gamma = torch.empty(N, m, dy, dtype=torch.float64, device=x_dg.device)
    alpha = torch.empty(N, m, dtype=torch.float64, device=x_dg.device)
    d = L.VoQueryDesc(n_fine=n_fine, nc=nc, n=N, flags=flags, logkappa=_p(x_dg), bc=_p(bc), gamma=_p(gamma),
                      alpha=_p(alpha))
    L.check(L.lib().gpi_vo_query(C.byref(d), L.stream_handle()), 'vo query')
    return gamma, alpha


def vo_galerkin(gamma, alpha, row0, m_aux, x_dg, bc, n_fine, kind, V=None, centers=None, length=0.0, seed=0,
                sub=31):
    """Rows row0 .. row0 + m_aux of gamma [N, m, d_y] / alpha [N, m] from test functions: given V
    [N, m_aux, d_y] or drawn on the device (VO_TEST_GAUSS / VO_TEST_RBF)."""
    _dev(gamma, alpha, x_dg, bc, V, centers)
    N, m, dy = gamma.shape
    assert dy == (n_fine + 1) * (n_fine - 1) and alpha.shape == (N, m) and 0 <= row0 and row0 + m_aux <= m
    assert x_dg.shape == (N, 2 * n_fine * n_fine) and bc.shape == (N, 4)
    assert gamma.dtype == torch.float64 and gamma.is_contiguous() and alpha.is_contiguous()
    if V is not None:
        assert V.shape == (N, m_aux, dy) and V.dtype == torch.float64
        V = V.contiguous()
    if centers is not None:
        assert centers.shape == (N, m_aux, 2) and centers.dtype == torch.float64
        centers = centers.contiguous()
    x_dg, bc = x_dg.contiguous().double(), bc.contiguous().double()
    d = L.VoGalerkinDesc(n_fine=n_fine, n=N, m_aux=m_aux, kind=kind, logkappa=_p(x_dg), bc=_p(bc), V=_p(V),
                         centers=_p(centers), length=float(length), seed=seed, offset=None, sub=sub, gamma=_p(gamma),
                         alpha=_p(alpha), m=m, row0=row0)
    L.check(L.lib().gpi_vo_galerkin(C.byref(d), L.stream_handle()), 'vo galerkin')


def vo_moments(uc, nc, refine, n, n_mc, logsig_y=None, eps=None, seed=0, offset=None, sub=7, want_std=True):
    """MC mean / std / precision of y_s = W u_s + exp(logsig_y) eps_s per VO sample
    (generative.py:198-207).  uc [n * n_mc, (nc+1)^2] fp32."""
    _dev(uc, logsig_y, eps, offset)
    nf = nc * refine
    dy = (nf + 1) * (nf - 1)
    assert uc.shape == (n * n_mc, (nc + 1) ** 2) and uc.dtype == torch.float32 and uc.is_contiguous()
    if logsig_y is not None:
        assert logsig_y.numel() == dy and logsig_y.dtype == torch.float32
        logsig_y = logsig_y.contiguous()
    if eps is not None:
        assert eps.shape == (n * n_mc, dy) and eps.dtype == torch.float32
        eps = eps.contiguous()
    mean = torch.empty(n, dy, dtype=torch.float32, device=uc.device)
    std = torch.empty_like(mean) if want_std else None
    prec = torch.empty_like(mean)
    d = L.VoMomentsDesc(nc=nc, refine=refine, n=n, n_mc=n_mc, uc=_p(uc), logsig_y=_p(logsig_y), eps=_p(eps),
                        seed=seed, offset=_p(offset), sub=sub, mean=_p(mean), std=_p(std), prec=_p(prec))
    L.check(L.lib().gpi_vo_moments(C.byref(d), L.stream_handle()), 'vo moments')
    return mean, std, prec


VS_R = 16        # slots per column of the column-sparse view (csrc/vo.hip VS_R)


def sparse_index_lists(rows, m):
    """Index lists of the column-sparse view (include/gpi.h gpi_vo_sparse) from the column pattern
    rows [d_y, r] (ascending row per slot, -1 = empty): the contributions of every column to the
    Lambda entries (a >= b, all diagonals present) grouped by entry, and the nonzeros of every row.
    Host bookkeeping only (once per Gamma); every sum over them runs on the device."""
    rows = np.asarray(rows, dtype=np.int64)
    dy, r = rows.shape
    S, T = np.tril_indices(r)                       # s >= t: rows[i, s] >= rows[i, t]
    a, b = rows[:, S], rows[:, T]
    ok = (a >= 0) & (b >= 0)
    ii = np.broadcast_to(np.arange(dy)[:, None], a.shape)
    key = (a * m + b)[ok]
    src = ((ii * r + S[None, :]) * r + T[None, :])[ok]
    diag = np.arange(m, dtype=np.int64) * (m + 1)
    pair_ab = np.union1d(key, diag)
    pidx = np.searchsorted(pair_ab, key)
    order = np.lexsort((src, pidx))
    pair_src = src[order]
    pair_ptr = np.zeros(len(pair_ab) + 1, dtype=np.int64)
    np.cumsum(np.bincount(pidx, minlength=len(pair_ab)), out=pair_ptr[1:])
    ra = rows.reshape(-1)
    rsrc = np.nonzero(ra >= 0)[0]
    rorder = np.lexsort((rsrc, ra[rsrc]))
    row_src = rsrc[rorder]
    row_ptr = np.zeros(m + 1, dtype=np.int64)
    np.cumsum(np.bincount(ra[rsrc], minlength=m), out=row_ptr[1:])
    i32 = lambda x: np.ascontiguousarray(x, dtype=np.int32)
    return dict(pair_ab=i32(pair_ab), pair_ptr=i32(pair_ptr), pair_src=i32(pair_src), row_ptr=i32(row_ptr),
                row_src=i32(row_src))


class SparsePlan(object):
    """Column-sparse view of a Gamma [N, m, d_y] whose columns have <= VS_R nonzero rows in the union
    over samples (CGR / flux rows); ``build`` returns None for denser Gamma (the dense kernels then run).
    Tied to the values of the Gamma it was built from: rebuild after Gamma changes."""

    @classmethod
    def build(cls, gamma, r_max=VS_R):
        _dev(gamma)
        assert gamma.dtype == torch.float64 and gamma.is_contiguous() and gamma.dim() == 3
        N, m, dy = gamma.shape
        r_max = min(int(r_max), VS_R)
        rows = torch.empty(dy, r_max, dtype=torch.int32, device=gamma.device)
        count = torch.empty(dy, dtype=torch.int32, device=gamma.device)
        work = torch.empty(m, dy, dtype=torch.uint8, device=gamma.device)
        L.check(L.lib().gpi_vo_pattern(_p(gamma), N, m, dy, r_max, _p(rows), _p(count), _p(work),
                                       L.stream_handle()), 'vo pattern')
        cmax = int(count.max().item())
        if cmax > r_max:
            return None
        self = cls()
        self.r = max(cmax, 1)
        rows_h = rows[:, :self.r].cpu().numpy()
        lists = sparse_index_lists(rows_h, m)
        dev = gamma.device
        self.rows = torch.from_numpy(np.ascontiguousarray(rows_h, dtype=np.int32)).to(dev)
        for k, v in lists.items():
            setattr(self, k, torch.from_numpy(v).to(dev))
        self.n_pairs = int(len(lists['pair_ab']))
        self.vals = torch.empty(N, dy, self.r, dtype=torch.float64, device=dev)
        self.inv = torch.empty(N, m, m, dtype=torch.float64, device=dev)
        self.shape = (N, m, dy)
        self.desc = L.VoSparse(r=self.r, n_pairs=self.n_pairs, rows=_p(self.rows), vals=_p(self.vals),
                               pair_ptr=_p(self.pair_ptr), pair_ab=_p(self.pair_ab), pair_src=_p(self.pair_src),
                               row_ptr=_p(self.row_ptr), row_src=_p(self.row_src), inv=_p(self.inv))
        self.refresh(gamma)
        return self

    def refresh(self, gamma):
        """Re-gather the slot values from gamma (same pattern)."""
        assert tuple(gamma.shape) == self.shape and gamma.is_contiguous()
        N, m, dy = self.shape
        L.check(L.lib().gpi_vo_sparse_values(_p(gamma), N, m, dy, C.byref(self.desc), L.stream_handle()),
                'vo sparse values')


class ConditionWorkspace(object):
    def __init__(self, N, m, dy, device):
        self.lam = torch.empty(N, m, m, dtype=torch.float64, device=device)
        self.solvec = torch.empty(N, m, dtype=torch.float64, device=device)
        self.flag = torch.zeros(1, dtype=torch.int32, device=device)


def vo_condition(gamma, alpha, g, prec, vo_var, mean, vars_, mean32=None, logsig32=None, ws=None, sparse=None):
    """VirtualObservable.update for every VO sample (VirtualObservables.py:642-669); ``sparse``: a
    SparsePlan of gamma (column-sparse kernels)."""
    _dev(gamma, alpha, g, prec, vo_var, mean, vars_, mean32, logsig32)
    N, m, dy = gamma.shape
    assert alpha.shape == (N, m) and vo_var.shape == (m,)
    assert g.shape == (N, dy) and prec.shape == (N, dy) and g.dtype == torch.float32 and prec.dtype == torch.float32
    assert mean.shape == (N, dy) and vars_.shape == (N, dy) and mean.dtype == torch.float64
    for t in (gamma, alpha, g, prec, vo_var, mean, vars_, mean32, logsig32):
        assert t is None or t.is_contiguous()
    if ws is None:
        ws = ConditionWorkspace(N, m, dy, gamma.device)
    d = L.VoConditionDesc(n=N, m=m, d_y=dy, gamma=_p(gamma), alpha=_p(alpha), g=_p(g), prec=_p(prec),
                          vo_var=_p(vo_var), lam=_p(ws.lam), solvec=_p(ws.solvec), mean=_p(mean), vars=_p(vars_),
                          mean32=_p(mean32), logsig32=_p(logsig32), flag=_p(ws.flag),
                          sparse=C.addressof(sparse.desc) if sparse is not None else None)
    if sparse is not None:
        assert sparse.shape == (N, m, dy)
    L.check(L.lib().gpi_vo_condition(C.byref(d), L.stream_handle()), 'vo condition')
    return ws


def vo_precision(gamma, alpha, mean, vars_, infinite, beta, vo_var, alpha0=ALPHA0, beta0=BETA0, sparse=None):
    """update_vo_precision + _get_mean_vo_variances (VirtualObservables.py:960-998)."""
    _dev(gamma, alpha, mean, vars_, infinite, beta, vo_var)
    N, m, dy = gamma.shape
    assert mean.shape == (N, dy) and vars_.shape == (N, dy) and infinite.shape == (m,)
    assert infinite.dtype == torch.int32 and beta.shape == (m,) and vo_var.shape == (m,)
    terms = torch.empty(m, max(N, 1), dtype=torch.float64, device=beta.device)
    d = L.VoPrecisionDesc(n=N, m=m, d_y=dy, gamma=_p(gamma), alpha=_p(alpha), mean=_p(mean), vars=_p(vars_),
                          infinite=_p(infinite), alpha0=alpha0, beta0=beta0, beta=_p(beta), vo_var=_p(vo_var),
                          terms=_p(terms), sparse=C.addressof(sparse.desc) if sparse is not None else None)
    if sparse is not None:
        assert sparse.shape == (N, m, dy)
    L.check(L.lib().gpi_vo_precision(C.byref(d), L.stream_handle()), 'vo precision')


def gauss_sample(out, mean, logsigma, rep=1, eps=None, seed=0, offset=None, sub=0, stream=None):
    """out[r] = mean[r // rep] + exp(logsigma[r // rep]) * N(0, 1) (float32 rows)."""
    _dev(out, mean, logsigma, eps, offset)
    rows, dim = out.shape
    assert mean.shape == logsigma.shape and mean.shape[-1] == dim and mean.numel() * rep == out.numel()
    for t in (out, mean, logsigma):
        assert t.dtype == torch.float32 and t.is_contiguous()
    st = stream if stream is not None else L.stream_handle()
    L.check(L.lib().gpi_gauss_sample(_p(out), _p(mean), _p(logsigma), rows, dim, rep, _p(eps), seed, _p(offset), sub,
                                     st), 'gauss sample')
    return out
