"""Closed-form stencil physics (product, setup side) vs the generic P1 FEM oracle."""
import numpy as np
import pytest

from oracle import fem
from physics.grid import StructuredGrid, pixel_to_cells


@pytest.mark.parametrize('n', [2, 4, 8])
def test_stiffness_matches_generic_p1(n):
    rng = np.random.default_rng(n)
    g = StructuredGrid(n)
    mesh = fem.unit_square_mesh(n)
    kappa = np.exp(rng.normal(size=2 * n * n))
    K_or = fem.assemble_stiffness(mesh, kappa)
    K_pr = g.stiffness(kappa).toarray()
    np.testing.assert_allclose(K_pr, K_or, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('n', [4, 8])
def test_reduced_system_and_fom(n):
    rng = np.random.default_rng(1 + n)
    g = StructuredGrid(n)
    mesh = fem.unit_square_mesh(n)
    kappa = np.exp(rng.normal(size=2 * n * n))
    u = rng.uniform(-0.5, 0.5, 4)
    K1, f1 = fem.assemble_system(mesh, kappa, u)
    K2, f2 = g.assemble_system(kappa, u)
    np.testing.assert_allclose(K2.toarray(), K1, atol=1e-12)
    np.testing.assert_allclose(f2, f1, atol=1e-12)
    np.testing.assert_allclose(g.solve(kappa, u), fem.solve_fom(mesh, kappa, u), atol=1e-10)


def test_constant_kappa_linear_solution_is_exact():
    # known answer: kappa const, u0=u1=a, u2=u3=b  =>  u = a + (b-a) x
    n = 16
    g = StructuredGrid(n)
    y = g.solve(np.full(2 * n * n, 3.7), [0.2, 0.2, -0.4, -0.4])
    x = g.coords[g.free_dofs, 0]
    np.testing.assert_allclose(y, 0.2 + (-0.6) * x, atol=1e-12)


def test_refinement_reproduces_structured_mesh():
    m = fem.unit_square_mesh(2)
    for _ in range(2):
        m = fem.refine_mesh(m)
    assert fem.same_triangulation(m, fem.unit_square_mesh(8))


@pytest.mark.parametrize('nc,r', [(4, 2), (4, 8), (8, 2)])
def test_prolongation_matches_point_location(nc, r):
    gc, gf = StructuredGrid(nc), StructuredGrid(nc * r)
    W_pr = gf.prolongation_from(gc)
    W_or = fem.prolongation_free(fem.unit_square_mesh(nc), fem.unit_square_mesh(nc * r))
    np.testing.assert_allclose(W_pr, W_or, atol=1e-12)
    np.testing.assert_allclose(W_pr.sum(1), 1.0, atol=1e-12)     # partition of unity


def test_rom_tensor_and_sum_rule():
    g = StructuredGrid(4)
    M = g.rom_tensor()
    M_or = fem.rom_stiffness_tensor(fem.unit_square_mesh(4))
    np.testing.assert_allclose(M, M_or, atol=1e-12)
    np.testing.assert_allclose(M.sum(2), g.stiffness(np.ones(g.num_cells)).toarray(), atol=1e-12)


def test_pixel_mapping():
    img = np.arange(16.0).reshape(4, 4)
    np.testing.assert_array_equal(pixel_to_cells(img), fem.image_to_cells(img))


def test_flux_residual_structured_matches_generic_rows():
    """The vectorised closed-form flux residual (oracle.fem.flux_residual_structured, used by the
    GPU flux tests at 64^2..256^2) equals the generic facet-search rows of oracle.fem.flux_rows
    (flux.py:81-158 restated) on small meshes, per-triangle conductivities that differ inside a
    square included."""
    import numpy as np
    from oracle import fem
    rng = np.random.default_rng(7)
    for nc, r in ((2, 2), (2, 4), (3, 3), (4, 2)):
        n = nc * r
        mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
        kap = np.exp(rng.normal(0.3, 0.8, 2 * n * n))
        G, a = fem.flux_rows(mc, mf, kap)
        free = fem.dirichlet_split(mf)[1]
        y = rng.normal(0, 0.5, free.size)
        ref = G[:, free] @ y - a
        kl = kap[0::2].reshape(n, n)
        ku = kap[1::2].reshape(n, n)
        got = fem.flux_residual_structured(nc, r, kl, ku, y)
        assert np.abs(got - ref).max() <= 1e-12 * max(np.abs(ref).max(), 1.0), (nc, r)
