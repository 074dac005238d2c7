"""GPU parity of the virtual-observable path (csrc/vo.hip, the flux residual in
csrc/stencil.hip, the VO term of the ELBO engine) against the oracle and the
golden fixture made by the reference's own VO classes (vo_elbo_c32.npz).
Tolerances per test: fp64 kernels vs fp64 oracle 1e-9..1e-10 relative; fp32 paths
as the ELBO tests (value 2e-5, gradients 2e-3 of the per-parameter max)."""
import os

import numpy as np
import pytest
import torch

from oracle import fem
from oracle import elbo as oelbo

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


def cuda(a, dtype=torch.float32):
    return torch.tensor(np.asarray(a), dtype=dtype, device='cuda')


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def oracle_query(nc, r, x_dg, u):
    """Oracle Gamma / alpha rows in the reference's sampler order: CGR, then flux (free columns)."""
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(nc * r)
    W = fem.prolongation_free(mc, mf)
    kap = np.exp(x_dg)
    Gc, ac = fem.cgr_query(mf, W, kap, u)
    Gf, af = fem.flux_rows(mc, mf, kap)
    free = fem.dirichlet_split(mf)[1]
    return np.vstack([Gc, Gf[:, free]]), np.concatenate([ac, af])


# ---------------------------------------------------------------- queries
def test_vo_query_matches_reference_fixture(device):
    from gpi import _lib as L
    from gpi.vo import vo_query
    d = load('vo_elbo_c32.npz')
    n, nc = int(d['cfg'][0]), int(d['cfg'][1])
    g, a = vo_query(cuda(d['Xv_dg'], torch.float64), cuda(d['Uv'], torch.float64), n, nc, L.VO_CGR | L.VO_FLUX)
    assert rel(g.cpu(), d['Gamma']) < 1e-12
    assert rel(a.cpu(), d['alpha']) < 1e-12


@pytest.mark.parametrize('nc,r', [(2, 8), (3, 4)])
def test_vo_query_random_cells(device, nc, r):
    """Per-triangle conductivities that differ inside a pixel (the generic DG0 case)."""
    from gpi import _lib as L
    from gpi.vo import vo_query
    rng = np.random.default_rng(nc * 10 + r)
    n = nc * r
    N = 2
    x = rng.normal(0.3, 0.9, (N, 2 * n * n))
    u = rng.uniform(-0.5, 0.5, (N, 4))
    for flags in (L.VO_CGR, L.VO_FLUX, L.VO_CGR | L.VO_FLUX):
        g, a = vo_query(cuda(x, torch.float64), cuda(u, torch.float64), n, nc, flags)
        for i in range(N):
            Go, ao = oracle_query(nc, r, x[i], u[i])
            rows = slice(0, (nc + 1) ** 2) if flags == L.VO_CGR else \
                (slice((nc + 1) ** 2, None) if flags == L.VO_FLUX else slice(None))
            assert rel(g[i].cpu(), Go[rows]) < 1e-12, flags
            assert np.abs(a[i].cpu().numpy() - ao[rows]).max() <= 1e-12 * max(np.abs(ao).max(), 1.0)


def test_flux_residual_fp32(device):
    """gpi_cgr_residual's flux output r_fc = Gamma_fc y (alpha_fc = 0) vs the fp64 oracle rows,
    error normalised by ||Gamma_fc||_F ||y||, tolerance 1e-5; the CGR output of the same launch too."""
    from gpi import _lib as L
    import ctypes as C
    rng = np.random.default_rng(5)
    nc, r, N = 4, 8, 3
    n = nc * r
    imgs = rng.normal(0.4, 0.8, (N, n, n))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    y = rng.normal(0, 0.3, (N, (n + 1) * (n - 1)))
    lk, yy, bb = cuda(imgs), cuda(y), cuda(U)
    rc = torch.empty(N, (nc + 1) ** 2, device='cuda')
    rf = torch.empty(N, 2 * nc * nc, device='cuda')
    dsc = L.ResidualDesc(n_fine=n, nc=nc, n=N, logkappa=lk.data_ptr(), y=yy.data_ptr(), bc=bb.data_ptr(),
                         r=rc.data_ptr(), r_flux=rf.data_ptr())
    L.check(L.lib().gpi_cgr_residual(C.byref(dsc), L.stream_handle()), 'residual')
    for i in range(N):
        Go, ao = oracle_query(nc, r, fem.image_to_cells(imgs[i]), U[i])
        ref = Go @ y[i] - ao
        m0 = (nc + 1) ** 2
        sc_c = np.linalg.norm(Go[:m0]) * np.linalg.norm(y[i]) + np.linalg.norm(ao[:m0])
        sc_f = np.linalg.norm(Go[m0:]) * np.linalg.norm(y[i])
        assert np.abs(rc[i].cpu().numpy() - ref[:m0]).max() / sc_c < 1e-5
        assert np.abs(rf[i].cpu().numpy() - ref[m0:]).max() / sc_f < 1e-5


# ---------------------------------------------------------------- moments / conditioning / precision
def test_vo_moments(device):
    from gpi.vo import vo_moments
    rng = np.random.default_rng(3)
    nc, r, N, Nmc = 4, 8, 3, 70            # 70 > one LDS chunk of 64 samples
    n = nc * r
    dy = (n + 1) * (n - 1)
    uc = rng.normal(0, 0.4, (N * Nmc, (nc + 1) ** 2))
    ls = rng.normal(-2, 0.3, dy)
    eps = rng.normal(size=(N * Nmc, dy))
    mean, std, prec = vo_moments(cuda(uc), nc, r, N, Nmc, logsig_y=cuda(ls), eps=cuda(eps))
    W = fem.prolongation_free(fem.unit_square_mesh(nc), fem.unit_square_mesh(n))
    u32 = uc.astype(np.float32).astype(np.float64)
    y = np.einsum('pk,sk->sp', W, u32) + np.exp(ls.astype(np.float32).astype(np.float64)) * \
        eps.astype(np.float32).astype(np.float64)
    y = y.reshape(N, Nmc, dy)
    assert rel(mean.cpu(), y.mean(1)) < 1e-5
    assert rel(std.cpu(), y.std(1, ddof=1)) < 1e-5
    p = prec.cpu().numpy().astype(np.float64)
    assert np.abs(p * y.std(1, ddof=1) ** 2 - 1).max() < 1e-4
    # without observation noise: std of W u alone
    mean0, std0, _ = vo_moments(cuda(uc), nc, r, N, Nmc)
    y0 = np.einsum('pk,sk->sp', W, u32).reshape(N, Nmc, dy)
    assert rel(std0.cpu(), y0.std(1, ddof=1)) < 1e-5


@pytest.mark.parametrize('sparse', [False, True], ids=['dense', 'sparse'])
@pytest.mark.parametrize('m_kind', ['cgr', 'cgr_flux_c64', 'cgr_flux_nc16'])
def test_vo_condition_vs_oracle(device, m_kind, sparse):
    """Conditioning kernel vs the oracle restatement of VirtualObservable.update on the same
    fp32-rounded prior (the reference casts its fp32 Y_mean / PREC to double).  m = 25 keeps Lambda in
    LDS; m = 209 (CGR + flux at 64x64) takes the global-memory Cholesky and the 107 KB column kernel;
    m = 801 (nc = 16) the one-thread-per-column L^-1.  ``sparse``: the column-sparse kernels
    (SparsePlan of the same Gamma)."""
    from gpi.vo import vo_condition, SparsePlan
    if m_kind == 'cgr':
        d = load('vo_c32.npz')
        G, A = d['Gamma'], d['alpha']
        g = d['g'].astype(np.float32)
        p = d['prec'].astype(np.float32)
        vv = d['vo_var']
    else:
        from gpi import _lib as L
        from gpi.vo import vo_query
        rng = np.random.default_rng(11)
        nc, r, N = (8, 8, 2) if m_kind == 'cgr_flux_c64' else (16, 4, 1)
        n = nc * r
        x = rng.normal(0.4, 0.8, (N, 2 * n * n))
        u = rng.uniform(-0.5, 0.5, (N, 4))
        Gt, At = vo_query(cuda(x, torch.float64), cuda(u, torch.float64), n, nc, L.VO_CGR | L.VO_FLUX)
        G, A = Gt.cpu().numpy(), At.cpu().numpy()
        dy = G.shape[2]
        g = rng.normal(0, 0.3, (N, dy)).astype(np.float32)
        p = (1.0 / rng.uniform(0.01, 0.1, (N, dy)) ** 2).astype(np.float32)
        vv = np.concatenate([np.zeros((nc + 1) ** 2), rng.uniform(0.1, 1.0, 2 * nc * nc)])
    N, m, dy = G.shape
    mean = torch.empty(N, dy, dtype=torch.float64, device='cuda')
    vars_ = torch.empty_like(mean)
    m32 = torch.empty(N, dy, device='cuda')
    l32 = torch.empty(N, dy, device='cuda')
    Gd = cuda(G, torch.float64)
    plan = SparsePlan.build(Gd) if sparse else None
    if sparse:
        assert plan is not None and plan.r <= 16
    ws = vo_condition(Gd, cuda(A, torch.float64), cuda(g), cuda(p), cuda(vv, torch.float64),
                      mean, vars_, m32, l32, sparse=plan)
    assert ws.flag.item() == 0
    for i in range(N):
        mo, vo = oelbo.vo_condition(torch.tensor(G[i]), torch.tensor(A[i]), torch.tensor(g[i]).double(),
                                    torch.tensor(p[i]).double(), torch.tensor(vv))
        assert rel(mean[i].cpu(), mo) < 1e-8
        cov = 1.0 / p[i].astype(np.float64)
        assert np.abs(vars_[i].cpu().numpy() - vo.numpy()).max() / cov.max() < 1e-8
        assert rel(m32[i].cpu(), mo.float()) < 1e-6
        assert rel(l32[i].cpu(), 0.5 * torch.log(vo.float())) < 1e-5
    if m_kind == 'cgr':   # and the reference's own outputs (fp64 prior there)
        assert rel(mean.cpu(), d['mean']) < 1e-5


def test_vo_precision_vs_oracle(device):
    from gpi.vo import vo_precision
    d = load('vo_c32.npz')
    G, A, mu, va = (cuda(d[k], torch.float64) for k in ('Gamma', 'alpha', 'mean', 'vars'))
    m = G.shape[1]
    inf = torch.zeros(m, dtype=torch.int32, device='cuda')
    inf[:5] = 1
    beta = torch.empty(m, dtype=torch.float64, device='cuda')
    vv = torch.empty_like(beta)
    vo_precision(G, A, mu, va, inf, beta, vv)
    beta2, vv2 = torch.empty_like(beta), torch.empty_like(vv)
    vo_precision(G, A, mu, va, inf, beta2, vv2)
    assert torch.equal(beta, beta2) and torch.equal(vv, vv2)       # fixed-order sums: reproducible
    assert rel(beta.cpu(), d['prec_beta']) < 1e-12
    ref = oelbo.vo_mean_variances(torch.tensor(d['prec_beta']), G.shape[0], inf.cpu().bool())
    assert rel(vv.cpu(), ref) < 1e-12
    # column-sparse view of the same Gamma
    from gpi.vo import SparsePlan
    plan = SparsePlan.build(G)
    assert plan is not None
    beta3, vv3 = torch.empty_like(beta), torch.empty_like(vv)
    vo_precision(G, A, mu, va, inf, beta3, vv3, sparse=plan)
    assert rel(beta3.cpu(), d['prec_beta']) < 1e-12
    assert rel(vv3.cpu(), ref) < 1e-12


@pytest.mark.parametrize('nc,r', [(4, 8), (8, 8)])
def test_vo_sparse_pattern(device, nc, r):
    """gpi_vo_pattern / gpi_vo_sparse_values on CGR + flux rows: the slots hold exactly the nonzeros of
    every column (union over samples, ascending rows), and a Gamma with a denser column is refused."""
    from gpi import _lib as L
    from gpi.vo import vo_query, SparsePlan
    rng = np.random.default_rng(5)
    n = nc * r
    N = 3
    x = rng.normal(0.4, 0.8, (N, 2 * n * n))
    u = rng.uniform(-0.5, 0.5, (N, 4))
    G, _ = vo_query(cuda(x, torch.float64), cuda(u, torch.float64), n, nc, L.VO_CGR | L.VO_FLUX)
    plan = SparsePlan.build(G)
    assert plan is not None
    Gh = G.cpu().numpy()
    nz = (Gh != 0).any(0)
    rows = plan.rows.cpu().numpy()
    vals = plan.vals.cpu().numpy()
    assert plan.r == int(nz.sum(0).max())
    for i in range(Gh.shape[2]):
        a = np.nonzero(nz[:, i])[0]
        assert np.array_equal(rows[i, :len(a)], a) and np.all(rows[i, len(a):] == -1)
        np.testing.assert_array_equal(vals[:, i, :len(a)], Gh[:, a, i])
        assert np.all(vals[:, i, len(a):] == 0)
    G2 = G.clone()
    G2[0, :, 7] = 1.0                              # one dense column
    assert SparsePlan.build(G2) is None


# ---------------------------------------------------------------- the model path
class _DS(object):
    def __init__(self, perm=None, **t):
        self.t = t
        self.perm = perm
        self.N = next(iter(t.values())).shape[0]

    def __bool__(self):
        return True

    def get(self, key, random_subset=None):
        if random_subset is None:
            return self.t[key]
        return self.t[key][self.perm[:random_subset]]


def build_vo_model(d, independent_X=True):
    from bottleneck.Encoder import CNNEncoder
    from bottleneck.Decoder import CNNDecoder
    from bottleneck.components import EffectivePropertyMap, ReducedOrderModelOperator
    from bottleneck.ROM import ROM
    from bottleneck.generative import GenerativeModel
    from bottleneck import VirtualObservables as VO
    from physics.grid import StructuredGrid
    from physics.LinearElliptic import LinearEllipticPhysics
    from physics.BoundaryConditions import BoundaryCondition
    n, nc, dz, Nu, bs, Ns, Nvo, Nmc = [int(v) for v in d['cfg']]
    enc = CNNEncoder(n, dz, [1, 1], 4, 4, drop_rate=0)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0.)
    rom = ROM(StructuredGrid(nc), n // nc)
    g = ReducedOrderModelOperator(rom, torch.tensor(d['W']), dtype=torch.float32, device='cuda')
    gp = EffectivePropertyMap(dz, 2 * nc * nc, independent_X=independent_X, dtype=torch.float32, device='cuda')
    model = GenerativeModel(f=dec.cuda(), g=g, gp=gp, dtype=torch.float32, device=torch.device('cuda'))
    model.encoder = enc.cuda()
    perm = torch.tensor(d['perm'], device='cuda')
    physics = {'fom': LinearEllipticPhysics('fom', 'NDP', n), 'rom': LinearEllipticPhysics('rom', 'NDP', nc),
               'W': d['W'].astype(np.float64)}
    QPE = VO.QuerryPointEnsemble([VO.QuerryPoint(physics['fom'], x, BoundaryCondition(u))
                                  for x, u in zip(d['Xv_dg'], d['Uv'])])
    QE = VO.QuerryEnsemble.FromQuerryPointEnsemble(QPE, physics, True, True, 0, 0, dtype=torch.float32,
                                                   device=torch.device('cuda'))
    ens = VO.VirtualObservablesEnsemble(QPE, QE, dtype=torch.float32, device=torch.device('cuda'))
    ds_s = _DS(X=cuda(d['Xs']), Y=cuda(d['Ys']), F_ROM_BC=cuda(d['Fs']))
    ds_u = _DS(perm=perm, X=cuda(d['Xu']))
    ds_v = _DS(X=cuda(d['Xv']), Y=cuda(d['Yv']), F_ROM_BC=cuda(d['Fv']))
    model.register_datasets({'supervised': ds_s, 'unsupervised': ds_u, 'vo': ds_v}, ens,
                            create_unsupervised_variational_approximation=False)
    model.load_state_dict({k[6:]: torch.tensor(v) for k, v in d.items() if k.startswith('state.')})
    model.cuda()
    return model, ens, bs


def _vo_model_parity(d, lockx):
    """update_virtual_observables x2 + elbo (armortized + supervised + VO) + backward, and the hold-off
    variant, on the native path vs
      (1) the fp64 oracle (tests/elbo_ref.py): VO update outputs (MC mean / std, VO posterior mean /
          variances, precision beta) 1e-5 relative per tensor; ELBO value 1e-5; every gradient tensor
          5e-5 per-tensor relative (max|g - ref| / max|ref|, no floor), the oracle taking the kernels'
          ReLU tie decisions for all four codec calls (encoder, decoder u / s / vo groups) with the audit
          of test_gpu_c64;
      (2) the reference's own fp32 run recorded in the fixture (ELBO value 2e-5, per-term values)."""
    from elbo_ref import oracle_vo_updates, oracle_vo_fixture_elbo, tensor_rel, check_grads
    from gpu_masks import engine_relu_masks
    from test_gpu_c64 import check_mask_audit
    from oracle import codec as ocodec
    model, ens, bs = build_vo_model(d, independent_X=not lockx)
    if lockx:
        assert 'supervised' not in model.q_X and 'vo' not in model.q_X
    else:
        assert rel(ens._QuerryEnsemble.gamma.cpu(), d['Gamma']) < 1e-12
    ups, beta = oracle_vo_updates(d, lockx=lockx)
    for it in range(2):
        Ym, Ys = model.update_virtual_observables(int(d['cfg'][7]), return_mean_stddev=True, step=it,
                                                  eps=(cuda(d['upd%d.eps_X' % it]), cuda(d['upd%d.eps_y' % it])))
        u = ups[it]
        errs = dict(Y_mean=tensor_rel(Ym.cpu(), u['Y_mean']), Y_std=tensor_rel(Ys.cpu(), u['Y_std']),
                    vo_var=tensor_rel(ens._mean_vo_variances.cpu(), u['vo_var']) if it else 0.0,
                    mean=tensor_rel(ens.mean.cpu(), u['mean']), vars=tensor_rel(ens.vars.cpu(), u['vars']))
        print('update', it, errs)
        assert max(errs.values()) < 1e-5, (it, errs)
        assert rel(Ym.cpu(), d['upd%d.Y_mean' % it]) < 1e-5
        assert rel(ens.mean.cpu(), d['upd%d.mean' % it]) < 1e-5
    assert tensor_rel(ens._prec_beta.cpu(), beta) < 1e-5
    ens.check_flag()
    vo_mean, vo_vars = ens.mean.cpu().numpy(), ens.vars.cpu().numpy()

    if lockx:
        e = [cuda(d['eps%d' % i]) for i in range(4)]
        eps = (torch.cat([e[0], e[1], e[2]]), None, e[3])
        term_keys = ('vo_logL_y', 'vo_DKL', 'supervised_logL_y')
    else:
        e = [cuda(d['eps%d' % i]) for i in range(6)]
        eps = (torch.cat([e[0], e[1], e[3]]), torch.cat([e[2], e[4]]), e[5])
        term_keys = ('vo_logL_x', 'vo_logL_y', 'vo_DKL', 'vo_logL_X', 'vo_entropy', 'supervised_logL_y')
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps)
    Ns, Nvo = int(d['cfg'][5]), int(d['cfg'][6])
    engine = model._elbo_engine(bs, Ns, False, N_vo=Nvo, vo_holdoff=False)
    assert engine.lockx == lockx
    terms = engine.terms()
    for k in term_keys:
        ref = float(d['term.objective/' + k])
        tol = 1e-4 if k == 'vo_logL_y' else 2e-5      # vo_logL_y sees the kernel-side VO posterior
        assert abs(terms[k] - ref) <= tol * max(abs(ref), 1.0), (k, terms[k], ref)
    assert abs(elbo.item() - float(d['elbo'])) / abs(float(d['elbo'])) < 2e-5
    (-elbo).backward()
    masks = engine_relu_masks(engine)
    assert set(masks) == {'enc', 'dec_u', 'dec_s', 'dec_v'}
    ocodec.MASK_AUDIT.clear()
    val_o, gr_o = oracle_vo_fixture_elbo(d, vo_mean, vo_vars, masks=masks, lockx=lockx)
    check_mask_audit()
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))

    model.zero_grad()
    h = [cuda(d['epsh%d' % i]) for i in range(3 if lockx else 4)]
    eps_h = (torch.cat(h), None) if lockx else (torch.cat([h[0], h[1], h[3]]), h[2])
    elbo_h = model.elbo(step=0, armortized_bs=bs, vo_holdoff=True, eps=eps_h)
    assert abs(elbo_h.item() - float(d['elbo_holdoff'])) / abs(float(d['elbo_holdoff'])) < 2e-5
    (-elbo_h).backward()
    engine = model._elbo_engine(bs, Ns, False, N_vo=Nvo, vo_holdoff=True)
    masks = engine_relu_masks(engine)
    ocodec.MASK_AUDIT.clear()
    val_h, gr_h = oracle_vo_fixture_elbo(d, vo_mean, vo_vars, masks=masks, lockx=lockx, holdoff=True)
    check_mask_audit()
    assert abs(elbo_h.item() - val_h) <= 1e-5 * abs(val_h), (elbo_h.item(), val_h)
    errs = {}
    for k, p in model.named_parameters():
        got = p.grad.cpu().numpy() if p.grad is not None else np.zeros(p.shape, np.float32)
        if k not in gr_h or not np.abs(gr_h[k]).any():
            assert np.abs(got).max() == 0, k          # parameters the hold-off term does not reach
            continue
        errs[k] = tensor_rel(got, gr_h[k])
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))


def test_vo_update_and_vo_elbo_match_reference(device):
    """freeX (the factories' default): see _vo_model_parity."""
    _vo_model_parity(load('vo_elbo_c32.npz'), lockx=False)


def test_vo_update_and_vo_elbo_lockx_match_reference(device):
    """independent_X = False (lockX): X~ = gp(z) in the supervised and VO terms
    (generative.py:300-339,429-459) and the VO predictive y = g(gp(z)), z ~ q_z['vo']
    (generative.py:202-204); see _vo_model_parity."""
    _vo_model_parity(load('vo_elbo_lockx_c32.npz'), lockx=True)


# ---------------------------------------------------------------- random test functions
def test_vo_galerkin_rows_given_test_functions(device):
    """V^T K_ff, V^T f_eff (QuerryPoint.construct_querry_weak_galerkin) for explicit V and for RBF
    centres, vs the oracle's assembled K_ff / f_eff (fp64, 1e-12)."""
    from gpi import _lib as L
    from gpi.vo import vo_galerkin
    rng = np.random.default_rng(21)
    nc, r, N, ma = 4, 8, 2, 3
    n = nc * r
    mf = fem.unit_square_mesh(n)
    dy = (n + 1) * (n - 1)
    x = rng.normal(0.3, 0.9, (N, 2 * n * n))
    u = rng.uniform(-0.5, 0.5, (N, 4))
    Vt = rng.normal(size=(N, ma, dy))
    cen = rng.uniform(0, 1, (N, ma, 2))
    m = 2 * ma + 1
    g = torch.full((N, m, dy), 7.0, dtype=torch.float64, device='cuda')
    a = torch.full((N, m), 7.0, dtype=torch.float64, device='cuda')
    xg, ug = cuda(x, torch.float64), cuda(u, torch.float64)
    vo_galerkin(g, a, 1, ma, xg, ug, n, L.VO_TEST_GAUSS, V=cuda(Vt, torch.float64))
    vo_galerkin(g, a, 1 + ma, ma, xg, ug, n, L.VO_TEST_RBF, centers=cuda(cen, torch.float64), length=0.15)
    free = fem.dirichlet_split(mf)[1]
    P = mf.coords[free]
    for i in range(N):
        K, f = fem.assemble_system(mf, np.exp(x[i]), u[i])
        Vr = np.exp(-((P[None, :, 0] - cen[i, :, 0:1]) ** 2 + (P[None, :, 1] - cen[i, :, 1:2]) ** 2) / 0.15 ** 2)
        Vall = np.concatenate([Vt[i], Vr])
        assert rel(g[i, 1:].cpu(), Vall @ K) < 1e-12
        assert np.abs(a[i, 1:].cpu().numpy() - Vall @ f).max() <= 1e-12 * max(np.abs(Vall @ f).max(), 1.0)
        assert float(g[i, 0, 0]) == 7.0 and float(a[i, 0]) == 7.0          # other rows untouched


def test_vo_galerkin_device_draws(device):
    """Device-drawn test functions: Gaussian V recovered from Gamma = V^T K (K SPD) is N(0,1);
    RBF rows are bounded by the RBF's own row of K (0 < V <= 1); redraws differ."""
    from gpi import _lib as L
    from gpi.vo import vo_galerkin
    rng = np.random.default_rng(22)
    nc, r, N, ma = 4, 8, 2, 8
    n = nc * r
    mf = fem.unit_square_mesh(n)
    dy = (n + 1) * (n - 1)
    x = rng.normal(0.3, 0.9, (N, 2 * n * n))
    u = rng.uniform(-0.5, 0.5, (N, 4))
    xg, ug = cuda(x, torch.float64), cuda(u, torch.float64)
    g = torch.empty(N, ma, dy, dtype=torch.float64, device='cuda')
    a = torch.empty(N, ma, dtype=torch.float64, device='cuda')
    vo_galerkin(g, a, 0, ma, xg, ug, n, L.VO_TEST_GAUSS, seed=5)
    K, _ = fem.assemble_system(mf, np.exp(x[0]), u[0])
    Vrec = np.linalg.solve(K, g[0].cpu().numpy().T).T            # K symmetric
    assert abs(Vrec.mean()) < 0.03 and abs(Vrec.std() - 1) < 0.03
    g2 = g.clone()
    vo_galerkin(g2, a, 0, ma, xg, ug, n, L.VO_TEST_GAUSS, seed=6)
    assert (g2 - g).abs().max().item() > 1.0
    vo_galerkin(g, a, 0, ma, xg, ug, n, L.VO_TEST_RBF, length=0.15, seed=5)
    Vrbf = np.linalg.solve(K, g[0].cpu().numpy().T).T
    assert Vrbf.min() > -1e-9 and Vrbf.max() <= 1 + 1e-9 and Vrbf.max() > 0.3


def test_vo_ensemble_with_random_test_functions(device):
    """QuerryEnsemble with CGR + flux + Gaussian + RBF rows; resample redraws only the random rows,
    and the batched conditioning runs on the full row set."""
    from bottleneck import VirtualObservables as VO
    from physics.LinearElliptic import LinearEllipticPhysics
    from physics.BoundaryConditions import BoundaryCondition
    rng = np.random.default_rng(23)
    nc, r, N = 4, 8, 3
    n = nc * r
    physics = {'fom': LinearEllipticPhysics('fom', 'NDP', n), 'rom': LinearEllipticPhysics('rom', 'NDP', nc)}
    physics['W'] = physics['fom'].grid.prolongation_from(physics['rom'].grid)
    QPE = VO.QuerryPointEnsemble([VO.QuerryPoint(physics['fom'], rng.normal(0.4, 0.8, 2 * n * n),
                                                 BoundaryCondition(rng.uniform(-0.5, 0.5, 4))) for _ in range(N)])
    QE = VO.QuerryEnsemble.FromQuerryPointEnsemble(QPE, physics, True, True, 4, 3, l_rbf=0.15,
                                                   dtype=torch.float32, device=torch.device('cuda'))
    m0 = (nc + 1) ** 2 + 2 * nc * nc
    assert QE.gamma.shape[1] == m0 + 7
    assert (QE.precision_mask < 0).sum() == (nc + 1) ** 2 + 7
    before = QE.gamma.clone()
    ens = VO.VirtualObservablesEnsemble(QPE, QE, dtype=torch.float32, device=torch.device('cuda'))
    ens.resample()
    assert torch.equal(QE.gamma[:, :m0], before[:, :m0])
    assert (QE.gamma[:, m0:] - before[:, m0:]).abs().max().item() > 0
    assert QE[1].Gamma.data_ptr() == QE.gamma[1].data_ptr()
    dy = (n + 1) * (n - 1)
    G = cuda(rng.normal(0, 0.3, (N, dy)))
    P = cuda(1.0 / rng.uniform(0.01, 0.1, (N, dy)) ** 2)
    ens.update(G, P, 0)
    ens.check_flag()
    for i in range(N):
        mo, vo = oelbo.vo_condition(QE.gamma[i].cpu(), QE.alpha[i].cpu(), G[i].cpu().double(), P[i].cpu().double(),
                                    ens._mean_vo_variances.cpu())
        assert rel(ens._mean64[i].cpu(), mo) < 1e-7


@pytest.mark.parametrize('n,N', [(64, 4), (128, 2), (256, 2)])
def test_flux_residual_fused_large_grids(device, n, N):
    """The flux-constraint residual fused into the CGR pass (r_flux of gpi_cgr_residual) at the
    64^2 / 128^2 / 256^2 grids (ROM 8x8, r = 8 / 16 / 32) vs the fp64 oracle's closed-form flux rows
    (oracle.fem.flux_residual_structured, pinned to the generic flux_rows): max error <= 1e-5 of the
    largest entry (random y, no cancellation); the CGR output of the same launch vs the matrix-free
    fp64 FE residual, same bound."""
    from gpi.engine import cgr_residual
    rng = np.random.default_rng(n + 1)
    nc = 8
    r = n // nc
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
    W = fem.prolongation_free(mc, mf)
    imgs = rng.normal(0.4, 0.8, (N, n, n))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    y = rng.normal(0, 0.3, (N, (n + 1) * (n - 1)))
    rc, rf = cgr_residual(cuda(imgs), cuda(y), cuda(U), nc=nc, flux=True)
    rc, rf = rc.cpu().numpy(), rf.cpu().numpy()
    for i in range(N):
        kap = np.exp(fem.image_to_square_kappa(imgs[i].astype(np.float32).astype(np.float64)))
        ref_f = fem.flux_residual_structured(nc, r, kap, kap, y[i].astype(np.float32).astype(np.float64))
        assert np.abs(rf[i] - ref_f).max() / np.abs(ref_f).max() < 1e-5
        ref_c = W.T @ fem.fom_residual(mf, np.exp(fem.image_to_cells(imgs[i])), U[i], y[i])
        assert np.abs(rc[i] - ref_c).max() / np.abs(ref_c).max() < 1e-5
