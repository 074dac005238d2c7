"""GPU parity of the FOM data-generation row (csrc/fom.hip): batched PCG labels against the
oracle's dense FE solve (oracle/fem.py) and, at 128^2 / 256^2, the oracle's matrix-free FE
residual; the device random-field sampler against the separable formula (explicit normals)
and against the sampler covariance (Philox normals, statistical).
Tolerances: labels 1e-9 absolute (values O(0.5), rtol 1e-13 on the residual); FE residual
1e-10 of ||f_eff||; random field 1e-12 absolute; empirical covariance 6 standard errors."""
import numpy as np
import pytest
import torch

from oracle import fem
from physics.grid import pixel_to_cells
from physics.RandomField import NormalRandomFieldSampler

pytestmark = pytest.mark.gpu


def fields(n, N, seed, l=0.15):
    rng = np.random.default_rng(seed)
    s = NormalRandomFieldSampler.FromImage(n, n, 0.4, 0.8, l, Truncation='adaptive' if n > 32 else None)
    X = s.sample(batch_size=N, rng=rng)
    return pixel_to_cells(X), rng.uniform(-0.5, 0.5, (N, 4))


def solve(xd, U, n, **kw):
    from gpi import fom
    t = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    r = fom.fom_solve(t(xd), t(U), n, **kw)
    return r.y.cpu().numpy(), r.iters.cpu().numpy(), int(r.flag.item())


@pytest.mark.parametrize('n,N', [(2, 3), (3, 4), (8, 8), (32, 8), (64, 2)])
def test_fom_labels_match_oracle(device, n, N):
    xd, U = fields(n, N, n)
    y, iters, flag = solve(xd, U, n)
    assert flag == 0
    mesh = fem.unit_square_mesh(n)
    for k in range(N):
        ref = fem.solve_fom(mesh, np.exp(xd[k]), U[k])
        assert np.abs(y[k] - ref).max() < 1e-9, (n, k, np.abs(y[k] - ref).max(), iters[k])


@pytest.mark.parametrize('n,N', [(8, 4), (32, 6), (64, 3)])
def test_fom_multigrid_labels_match_oracle(device, monkeypatch, n, N):
    """The multigrid-preconditioned CG (fom_mgcg_kernel, the default from 64^2) forced onto every
    power-of-two grid from 8^2 (GPI_FOM_MG_MIN=8): labels vs the oracle's dense FE solve at 1e-9, in a few
    tens of iterations where the Jacobi form needs hundreds (407 on average at 64^2)."""
    monkeypatch.setenv('GPI_FOM_MG_MIN', '8')
    xd, U = fields(n, N, n + 1, l=0.04 if n == 64 else 0.15)
    y, iters, flag = solve(xd, U, n)
    assert flag == 0 and iters.max() <= 40, iters
    mesh = fem.unit_square_mesh(n)
    for k in range(N):
        ref = fem.solve_fom(mesh, np.exp(xd[k]), U[k])
        assert np.abs(y[k] - ref).max() < 1e-9, (n, k, np.abs(y[k] - ref).max(), iters[k])
    U[0] = 0.0                                   # zero data: converged on entry
    y0, it0, flag0 = solve(xd, U, n)
    assert flag0 == 0 and it0[0] == 0 and np.abs(y0[0]).max() == 0.0
    _, it2, flag2 = solve(xd, U, n, max_iter=2)  # iteration cap reported
    assert flag2 == N - 1 and it2.max() == 2


@pytest.mark.parametrize('n,N', [(128, 3), (256, 2)])
def test_fom_large_grid_residual(device, n, N):
    xd, U = fields(n, N, n, l=0.04)
    y, iters, flag = solve(xd, U, n)
    assert flag == 0 and iters.max() <= 40, iters      # multigrid-preconditioned from 64^2
    mesh = fem.unit_square_mesh(n)
    for k in range(N):
        kap = np.exp(xd[k])
        r = fem.fom_residual(mesh, kap, U[k], y[k])
        b = fem.fom_residual(mesh, kap, U[k], np.zeros_like(y[k]))
        assert np.linalg.norm(r) <= 1e-10 * np.linalg.norm(b), (n, k, np.linalg.norm(r) / np.linalg.norm(b))


def test_fom_jacobi_workspace_kernel_residual(device, monkeypatch):
    """The Jacobi-preconditioned workspace kernel (fom_pcg_kernel: grids past the register form, non-powers
    of two, or GPI_FOM_MG_MIN=0) at 128^2: FE residual 1e-10 of ||f_eff||, as the multigrid form's."""
    monkeypatch.setenv('GPI_FOM_MG_MIN', '0')
    n, N = 128, 2
    xd, U = fields(n, N, n + 5, l=0.04)
    y, iters, flag = solve(xd, U, n)
    assert flag == 0 and iters.min() > 100, iters
    mesh = fem.unit_square_mesh(n)
    for k in range(N):
        kap = np.exp(xd[k])
        r = fem.fom_residual(mesh, kap, U[k], y[k])
        b = fem.fom_residual(mesh, kap, U[k], np.zeros_like(y[k]))
        assert np.linalg.norm(r) <= 1e-10 * np.linalg.norm(b), (k, np.linalg.norm(r) / np.linalg.norm(b))


def test_fom_edge_cases(device):
    from gpi import fom
    n, N = 16, 4
    xd, U = fields(n, N, 1)
    U[1] = 0.0                                   # zero data: y = 0 without iterating
    y, iters, flag = solve(xd, U, n)
    assert flag == 0 and iters[1] == 0 and np.abs(y[1]).max() == 0.0
    # warm start from the solution: converged on entry
    t = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    r = fom.fom_solve(t(xd), t(U), n, y0=torch.tensor(y), rtol=1e-8)
    assert int(r.flag.item()) == 0 and r.iters.cpu().numpy().max() == 0
    # iteration cap: every non-trivial sample reports non-convergence
    y2, it2, flag2 = solve(xd, U, n, max_iter=2)
    assert flag2 == N - 1 and it2.max() == 2
    with pytest.raises(Exception):
        fom.FomResult(None, None, torch.ones(1, dtype=torch.int32)).check()
    # chunked launches (workspace reuse) give the same labels
    y3, _, _ = solve(xd, U, n, chunk=3)
    np.testing.assert_array_equal(y3, y)
    # empty batch
    e = fom.fom_solve(torch.zeros(0, 2 * n * n, dtype=torch.float64, device='cuda'),
                      torch.zeros(0, 4, dtype=torch.float64, device='cuda'), n)
    assert e.y.shape == (0, (n + 1) * (n - 1))


def test_fom_labels_zero_the_cgr_residual(device):
    """Cross-kernel property: exact FOM labels satisfy Gamma y = alpha of the CGR sampler."""
    from gpi import vo, _lib as L
    n, nc, N = 32, 4, 4
    xd, U = fields(n, N, 5)
    t = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    y, _, _ = solve(xd, U, n)
    G, a = vo.vo_query(t(xd), t(U), n, nc, L.VO_CGR)
    r = torch.einsum('nmd,nd->nm', G, t(y)) - a
    scale = G.abs().amax() * np.abs(y).max() + a.abs().amax()
    assert float(r.abs().max() / scale) < 1e-10


def test_dataloader_assemble_on_device(device):
    from factories.model import ModelFactory
    from utils.data import DataLoader
    fac = ModelFactory.FromIdentifier('highres32')
    physics = fac._physics()
    rng = np.random.default_rng(2)
    s = NormalRandomFieldSampler.FromImage(32, 32, 0.4, 0.8, 0.15)
    dl = DataLoader.FromSampler(s, 12, rng=rng)
    host = DataLoader(dl.X, dl.BCE).assemble(physics)
    dev = DataLoader(dl.X, dl.BCE).assemble(physics, device='cuda')
    assert np.abs(dev.Y - host.Y).max() < 1e-9
    np.testing.assert_array_equal(dev.F_ROM_BC, host.F_ROM_BC)
    assert dev.fom_iters.min() > 0
    part = DataLoader(dl.X, dl.BCE).assemble(physics, indices=[1, 4], device='cuda')
    assert np.isnan(part.Y[0]).all() and np.abs(part.Y[4] - host.Y[4]).max() < 1e-9


@pytest.mark.parametrize('py,px,l,trunc', [(32, 32, 0.15, None), (20, 36, 0.1, 'adaptive'), (64, 64, 0.04, 'adaptive'),
                                            (128, 128, 0.04, 'adaptive')])
def test_random_field_explicit_normals(device, py, px, l, trunc):
    s = NormalRandomFieldSampler.FromImage(py, px, 0.4, 0.8, l, Truncation=trunc)
    G = np.random.default_rng(7).normal(size=(3, py, px))
    x = s.sample_device(3, gamma=G).cpu().numpy()
    ref = s.sample(gamma=G, batch_size=3)
    assert np.abs(x - ref).max() < 1e-12


def test_random_field_philox_statistics(device):
    s = NormalRandomFieldSampler.FromImage(12, 12, 0.4, 0.8, 0.2, Truncation=None)
    N = 40000
    x = s.sample_device(N, seed=11).cpu().numpy().reshape(N, -1)
    C = s.covariance()
    sd = np.sqrt(np.diag(C))
    assert np.abs(x.mean(0) - 0.4).max() < 6 * sd.max() / np.sqrt(N)
    Ce = np.cov(x.T)
    se = np.sqrt((C ** 2 + np.outer(np.diag(C), np.diag(C))) / N)
    assert np.abs(Ce - C).max() < 6 * se.max()
    a = s.sample_device(4, seed=11).cpu().numpy()
    np.testing.assert_array_equal(a, x[:4].reshape(4, 12, 12))
    b = s.sample_device(4, seed=11, sub=1).cpu().numpy()
    assert np.abs(a - b).max() > 0.1
