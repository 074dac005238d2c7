"""Host side of the FOM data-generation row: the separable
random-field sampler against the dense restatement of the reference's sampler
(oracle/field.py: covariance, KL truncation, Cholesky), the oracle's matrix-free FE
residual against its assembled stiffness, and the data factory's file round trip.
Tolerances: spectra 1e-12 relative, untruncated covariances 1e-12 absolute."""
import os

import numpy as np
import pytest

from oracle import fem, field
from physics.RandomField import NormalRandomFieldSampler
from physics.grid import StructuredGrid, pixel_to_cells


@pytest.mark.parametrize('py,px,l,trunc', [(16, 16, 0.15, 'adaptive'), (24, 24, 0.04, 'adaptive'),
                                            (12, 20, 0.3, None), (32, 32, 0.15, None), (20, 12, 0.1, 'adaptive')])
def test_separable_sampler_matches_dense_reference(py, px, l, trunc):
    s = NormalRandomFieldSampler.FromImage(py, px, 0.4, 0.8, l, Truncation=trunc)
    C = field.covariance(py, px, 0.8, l)
    Lref = field.kl_factor(C, trunc)
    assert s.dim_in == Lref.shape[1]
    Cs = s.covariance()
    ws = np.sort(np.linalg.eigvalsh(Cs))[::-1][:Lref.shape[1]]
    wr = np.sort(np.linalg.eigvalsh(Lref @ Lref.T))[::-1][:Lref.shape[1]]
    np.testing.assert_allclose(ws, wr, rtol=1e-10, atol=1e-12)
    if trunc is None:
        np.testing.assert_allclose(Cs, C, atol=1e-12)


def test_sampler_draw_is_the_separable_formula():
    s = NormalRandomFieldSampler.FromImage(16, 16, 0.4, 0.8, 0.15, Truncation='adaptive')
    G = np.random.default_rng(0).normal(size=(3, 16, 16))
    Vy, Vx, S = s.factors()
    X = s.sample(gamma=G, batch_size=3)
    ref = 0.4 + np.kron(Vy, Vx) @ (S.ravel()[None, :] * G.reshape(3, -1)).T
    np.testing.assert_allclose(X.reshape(3, -1), ref.T, atol=1e-12)


def test_dense_cap_kept():
    s = NormalRandomFieldSampler.FromImage(96, 96, 0.4, 0.8, 0.04, dense=True)
    with pytest.raises(RuntimeError):
        s.sample()


@pytest.mark.parametrize('n', [2, 4, 7])
def test_oracle_matrix_free_residual_pins_assembly(n):
    rng = np.random.default_rng(n)
    mesh = fem.unit_square_mesh(n)
    kap = np.exp(rng.normal(size=2 * n * n))
    u = rng.uniform(-0.5, 0.5, 4)
    K = fem.assemble_stiffness(mesh, kap)
    v = rng.normal(size=mesh.num_vertices)
    np.testing.assert_allclose(fem.apply_stiffness(mesh, kap, v), K @ v, atol=1e-12)
    y = fem.solve_fom(mesh, kap, u)
    assert np.abs(fem.fom_residual(mesh, kap, u, y)).max() < 1e-12
    # the product's host solve (scipy on the stencil) is the same system
    np.testing.assert_allclose(StructuredGrid(n).solve(kap, u), y, atol=1e-12)


def test_data_factory_roundtrip(tmp_path):
    from factories.data import DataFactory
    from utils.data import DataLoader
    with pytest.raises(KeyError):
        DataFactory.FromIdentifier('HighRes')
    f = DataFactory.FromIdentifier('highres32', path=str(tmp_path) + '/', seed=3)
    f._N, f._N_unsupervised = 6, 5
    dl, dlu = f.setup()
    assert dl.X.shape == (6, 32, 32) and dlu.X.shape == (5, 32, 32)
    assert os.path.exists(str(tmp_path) + '/highres32.pt') and os.path.exists(str(tmp_path) + '/highres32.ptu')
    dl2, _ = DataFactory.FromIdentifier('highres32', path=str(tmp_path) + '/').setup()
    np.testing.assert_array_equal(dl2.X, dl.X)
    np.testing.assert_array_equal(dl2.BCE.U, dl.BCE.U)
    with pytest.raises(RuntimeError):
        dlu.assemble({'fom': None, 'rom': None})
    with pytest.raises(ValueError):
        DataFactory(path='cdata')._check_path('cdata')
    with pytest.raises(ValueError):
        DataLoader(dl.X[:1]).save(str(tmp_path) + '/noext')


def test_timer_api():
    from utils.time import Timer, StopWatch
    t = Timer(10)
    with t('solve'):
        pass
    assert 'Days' in t.RRT(step=3) and t.ETA(3).startswith('ETA:') and 'solve' in str(t)
    s = StopWatch()
    s.stop()
    assert s.runtime() >= 0.0
