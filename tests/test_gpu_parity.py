"""GPU parity: the HIP kernels (through the C ABI and the drop-in modules)
against golden fixtures produced by the reference's own modules and against
the oracle.  Tolerances: fp32 kernels vs fp32/fp64 references, stated per test."""
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


# ---------------------------------------------------------------- ROM
def test_rom_operator_forward_backward(device):
    from gpi.native import RomOperatorFunction
    d = load('rom_c32.npz')
    x = cuda(d['effprop']).requires_grad_(True)
    F = cuda(d['F'])
    mu, uc = RomOperatorFunction.apply(x, F, 4, 8, False)
    assert rel(mu.detach().cpu(), d['mu_y']) < 2e-5
    ls = cuda(d['logsigmas_y']).requires_grad_(True)
    Y = cuda(d['Y'])
    L = torch.sum(-0.5 * (2 * ls + (Y - mu) ** 2 * torch.exp(-2 * ls) + 1.8378770664093453))
    (-L).backward()
    assert abs(L.item() - float(d['logL'])) / abs(float(d['logL'])) < 1e-5
    assert rel(x.grad.cpu(), d['grad_effprop']) < 1e-3
    assert rel(ls.grad.cpu(), d['grad_logsigmas_y']) < 1e-4


def test_rom_fused_loglik(device):
    from gpi.engine import rom_call
    from gpi import _lib as L
    d = load('rom_c32.npz')
    x, F, Y, ls = cuda(d['effprop']), cuda(d['F']), cuda(d['Y']), cuda(d['logsigmas_y'])
    gx = torch.zeros_like(x)
    gls = torch.zeros(ls.shape[0], dtype=torch.float64, device='cuda')
    acc = torch.zeros(L.GPI_REPLICAS, dtype=torch.float64, device='cuda')
    flag = torch.zeros(1, dtype=torch.int32, device='cuda')
    rom_call(4, 8, x, F, False, L.ROM_LOGLIK, Y=Y, logsig_y=ls, gx=gx, gacc_logsig=gls, loss_acc=acc, flag=flag)
    assert abs(acc.sum().item() - float(d['logL'])) / abs(float(d['logL'])) < 1e-5
    assert rel(gx.cpu(), d['grad_effprop']) < 1e-3
    assert rel(gls.cpu(), d['grad_logsigmas_y']) < 1e-4
    assert flag.item() == 0


def test_rom_call_matches_reference_semantics(device):
    """ROM.__call__(kappa, F): Dirichlet-row dense solve of the reference (ROM.py:65-100)."""
    from bottleneck.ROM import ROM
    from physics.grid import StructuredGrid
    d = load('rom_c32.npz')
    kap = torch.exp(torch.tensor(d['effprop'], dtype=torch.float64)) + 1e-8
    ref = oelbo.rom_solve(torch.tensor(d['M'], dtype=torch.float64), kap, torch.tensor(d['F'], dtype=torch.float64),
                          torch.tensor(d['bc_dofs']))
    rom = ROM(StructuredGrid(4), 8)
    u = rom(kap.float().cuda(), cuda(d['F']))
    assert rel(u.cpu(), ref) < 2e-5


# ---------------------------------------------------------------- CGR residual
def test_cgr_residual_fp32_match(device):
    """North-star residual check: fp32 kernel vs fp64 Gamma y - alpha, error normalised by
    ||Gamma||_F ||y|| + ||alpha||, tolerance 1e-5."""
    from gpi.engine import cgr_residual
    d = load('vo_c32.npz')
    imgs, U, G, A, y = d['imgs'], d['U'], d['Gamma'], d['alpha'], d['g']
    r = cgr_residual(cuda(imgs), cuda(y), cuda(U), nc=4).cpu().numpy()
    for i in range(imgs.shape[0]):
        ref = G[i] @ y[i] - A[i]
        scale = np.linalg.norm(G[i]) * np.linalg.norm(y[i]) + np.linalg.norm(A[i])
        assert np.abs(r[i] - ref).max() / scale < 1e-5


@pytest.mark.parametrize('nc,r,N', [(8, 8, 3), (4, 4, 5), (2, 16, 2)])
def test_cgr_residual_random_fields(device, nc, r, N):
    from gpi.engine import cgr_residual
    rng = np.random.default_rng(nc * r)
    n = nc * r
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
    W = fem.prolongation_free(mc, mf)
    imgs = rng.normal(0.4, 0.8, (N, n, n))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    y = rng.normal(0, 0.3, (N, W.shape[0]))
    out = cgr_residual(cuda(imgs), cuda(y), cuda(U), nc=nc).cpu().numpy()
    for i in range(N):
        Gm, a = fem.cgr_query(mf, W, np.exp(fem.image_to_cells(imgs[i])), U[i])
        ref = Gm @ y[i] - a
        scale = np.linalg.norm(Gm) * np.linalg.norm(y[i]) + np.linalg.norm(a)
        assert np.abs(out[i] - ref).max() / scale < 1e-5


@pytest.mark.parametrize('n,N', [(128, 2), (256, 1)])
def test_cgr_residual_large_grids(device, n, N):
    """BASELINE configs 4 / 5 grids (ROM 8x8, r = 16 / 32): W^T [K yhat]_free vs the oracle's
    matrix-free fp64 FE residual (oracle.fem.fom_residual); max error <= 1e-5 of the largest
    residual entry (no Gamma is formed at these sizes to normalise by)."""
    from gpi.engine import cgr_residual
    rng = np.random.default_rng(n)
    nc = 8
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
    W = fem.prolongation_free(mc, mf)
    imgs = rng.normal(0.4, 0.8, (N, n, n))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    y = rng.normal(0, 0.3, (N, W.shape[0]))
    out = cgr_residual(cuda(imgs), cuda(y), cuda(U), nc=nc).cpu().numpy()
    for i in range(N):
        ref = W.T @ fem.fom_residual(mf, np.exp(fem.image_to_cells(imgs[i])), U[i], y[i])
        assert np.abs(out[i] - ref).max() / np.abs(ref).max() < 1e-5


_BAND_RM = {(4, 1), (8, 1), (16, 1), (16, 2), (32, 4)}


@pytest.mark.parametrize('n,nc,N', [(64, 8, 7), (128, 8, 3), (256, 8, 1), (64, 16, 3), (48, 3, 3), (60, 5, 3)])
@pytest.mark.parametrize('form', ['band', 'stream', 'general'])
def test_cgr_residual_every_kernel_form(device, n, nc, N, form):
    """Each kernel form of gpi_cgr_residual, selected per call (gpi_residual_desc.form): the barrier-free
    band form (cgr_band_kernel), the streaming form (cgr_stream_kernel, LDS ring chunks) and the general
    band kernel (cgr_kernel<M>), CGR rows vs the oracle's matrix-free fp64 FE residual (W^T (K yhat)_free,
    VirtualObservables.py:57-69,297-302 / physics/LinearElliptic.py:137-159) and flux rows vs its closed-form
    flux rows (bottleneck/flux.py:81-158), max error <= 1e-5 of the largest entry; AUTO (the ELBO / VO path's
    choice) equal to the form it picks.  A form whose preconditions fail returns GPI_ERR_UNSUPPORTED: band
    needs nc <= 8 and (r, n / 64 columns per lane) instantiated, streaming a 16-multiple n <= 256, a power-of-
    two r >= 4 and 16-byte aligned fields.  N (n^2 - 1) is odd at N = 7 / 3 / 1, so y's last float4 is partial
    (the streaming kernel's clamped tail load)."""
    import ctypes as C
    from gpi import _lib as L
    r_ = n // nc
    mm = (n + 63) // 64
    applies = {'band': nc <= 8 and (r_, mm) in _BAND_RM,
               'stream': n % 16 == 0 and 16 <= n <= 256 and r_ >= 4 and (r_ & (r_ - 1)) == 0,
               'general': True}
    auto = next(f for f in ('band', 'stream', 'general') if applies[f])
    code = {'auto': L.CGR_AUTO, 'band': L.CGR_BAND, 'stream': L.CGR_STREAM, 'general': L.CGR_GENERAL}
    rng = np.random.default_rng(1000 * n + nc)
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
    W = fem.prolongation_free(mc, mf)
    imgs = rng.normal(0.4, 0.8, (N, n, n))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    y = rng.normal(0, 0.3, (N, W.shape[0]))
    lk, bc, yy = cuda(imgs), cuda(U), cuda(y)
    assert yy.data_ptr() % 16 == 0 and lk.data_ptr() % 16 == 0

    def run(f):
        rc_ = torch.zeros(N, (nc + 1) ** 2, device='cuda')
        rf_ = torch.zeros(N, 2 * nc * nc, device='cuda')
        d = L.ResidualDesc(n_fine=n, nc=nc, n=N, form=code[f], logkappa=lk.data_ptr(), y=yy.data_ptr(),
                           bc=bc.data_ptr(), r=rc_.data_ptr(), r_flux=rf_.data_ptr())
        ret = L.lib().gpi_cgr_residual(C.byref(d), L.stream_handle())
        torch.cuda.synchronize()
        return ret, rc_.cpu().numpy(), rf_.cpu().numpy()

    ret, rc, rf = run(form)
    if not applies[form]:
        assert ret == -3, (form, n, nc, ret)      # GPI_ERR_UNSUPPORTED, nothing launched
        return
    assert ret == 0, ret
    for i in range(N):
        ref = W.T @ fem.fom_residual(mf, np.exp(fem.image_to_cells(imgs[i])), U[i], y[i])
        assert np.abs(rc[i] - ref).max() / np.abs(ref).max() < 1e-5, (form, i)
        kap = np.exp(fem.image_to_square_kappa(imgs[i].astype(np.float32).astype(np.float64)))
        ref_f = fem.flux_residual_structured(nc, r_, kap, kap, y[i].astype(np.float32).astype(np.float64))
        assert np.abs(rf[i] - ref_f).max() / np.abs(ref_f).max() < 1e-5, (form, i)
    if form == auto:
        ret_a, rca, rfa = run('auto')
        assert ret_a == 0 and np.array_equal(rca, rc) and np.array_equal(rfa, rf)


def test_cgr_residual_vanishes_at_fom_solution(device):
    from gpi.engine import cgr_residual
    rng = np.random.default_rng(0)
    nc, n = 8, 64
    mf = fem.unit_square_mesh(n)
    img = rng.normal(0.4, 0.8, (1, n, n))
    u = rng.uniform(-0.5, 0.5, (1, 4))
    y = fem.solve_fom(mf, np.exp(fem.image_to_cells(img[0])), u[0])[None]
    r = cgr_residual(cuda(img), cuda(y), cuda(u), nc=nc).cpu().numpy()
    assert np.abs(r).max() < 1e-4


# ---------------------------------------------------------------- codec
def _codec(tag):
    from bottleneck.Encoder import CNNEncoder
    from bottleneck.Decoder import CNNDecoder
    d = load('codec_%s.npz' % tag)
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]
    enc = CNNEncoder(imsize, dz, blocks, growth, f_enc, drop_rate=0)
    dec = CNNDecoder(imsize, dz, (latent, latent), 1, f_dec, blocks, False, growth, drop_rate=0.)
    enc.load_state_dict({k[4:]: torch.tensor(v) for k, v in d.items() if k.startswith('enc.') and
                         not k.startswith('enc.grad.')})
    dec.load_state_dict({k[4:]: torch.tensor(v) for k, v in d.items() if k.startswith('dec.') and
                         not k.startswith('dec.grad.')})
    return d, enc.cuda(), dec.cuda()


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_encoder_forward_backward(device, tag):
    d, enc, _ = _codec(tag)
    mu, ls = enc(cuda(d['X']))
    assert rel(mu.detach().cpu(), d['enc_mu']) < 1e-4
    assert rel(ls.detach().cpu(), d['enc_ls']) < 1e-4
    (torch.sum(mu * cuda(d['enc_wm'])) + torch.sum(ls * cuda(d['enc_ws']))).backward()
    for k, p in enc.named_parameters():
        assert rel(p.grad.cpu(), d['enc.grad.' + k]) < 2e-3, k


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_decoder_forward_backward(device, tag):
    d, _, dec = _codec(tag)
    Z = cuda(d['Z']).requires_grad_(True)
    mx, lsx = dec(Z)
    assert rel(mx.detach().cpu(), d['dec_mu']) < 1e-4
    assert rel(lsx.detach().cpu(), d['dec_ls']) < 1e-4
    (torch.sum(mx * cuda(d['dec_vm'])) + torch.sum(lsx * cuda(d['dec_vs']))).backward()
    assert rel(Z.grad.cpu(), d['grad_Z']) < 2e-3
    for k, p in dec.named_parameters():
        assert rel(p.grad.cpu(), d['dec.grad.' + k]) < 2e-3, k


# ---------------------------------------------------------------- full ELBO step
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


def build_golden_model(d, independent_X=True):
    from bottleneck.Encoder import CNNEncoder
    from bottleneck.Decoder import CNNDecoder
    from bottleneck.components import EffectivePropertyMap, ReducedOrderModelOperator
    from bottleneck.ROM import ROM
    from bottleneck.generative import GenerativeModel
    from physics.grid import StructuredGrid
    n, nc, dz, Nu, bs, Ns = [int(v) for v in d['cfg']]
    enc = CNNEncoder(n, dz, [1, 1], 4, 4, drop_rate=0)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0.)
    rom = ROM(StructuredGrid(nc), n // nc)
    g = ReducedOrderModelOperator(rom, torch.tensor(d['W']), dtype=torch.float32, device='cuda')
    gp = EffectivePropertyMap(dz, 2 * nc * nc, independent_X=independent_X, dtype=torch.float32, device='cuda')
    model = GenerativeModel(f=dec.cuda(), g=g, gp=gp, dtype=torch.float32, device=torch.device('cuda'))
    model.encoder = enc.cuda()
    perm = torch.tensor(d['perm'], device='cuda')
    ds_s = _DS(X=cuda(d['Xs']), Y=cuda(d['Y']), F_ROM_BC=cuda(d['F']))
    ds_u = _DS(perm=perm, X=cuda(d['Xu']))
    model.register_datasets({'supervised': ds_s, 'unsupervised': ds_u}, None,
                            create_unsupervised_variational_approximation=False)
    state = {k[6:]: torch.tensor(v) for k, v in d.items() if k.startswith('state.')}
    if not independent_X:     # lockX: no q_X rows, no gp.logsigmas_X
        state = {k: v for k, v in state.items() if not k.startswith('q_X.') and k != 'gp.logsigmas_X'}
    model.load_state_dict(state)
    model.cuda()
    return model, bs


def test_elbo_step_matches_reference(device):
    """GenerativeModel.elbo + backward (generative.py:247-287), injected eps, vs the fp64 oracle with
    the kernels' ReLU tie decisions (value 1e-5, every gradient tensor 5e-5 relative, no floor) and vs
    the reference's own fp32 run (value 2e-5, gradients 2e-3 of the tensor's max)."""
    from elbo_ref import oracle_fixture_elbo, tensor_rel, check_grads
    from gpu_masks import engine_relu_masks
    d = load('elbo_c32.npz')
    model, bs = build_golden_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps)
    assert abs(elbo.item() - float(d['elbo'])) / abs(float(d['elbo'])) < 2e-5
    (-elbo).backward()
    val_o, gr_o = oracle_fixture_elbo(d, masks=engine_relu_masks(model._elbo_engine(bs, int(d['cfg'][5]), False)))
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o)
    print(check_grads({k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()},
                      tol_all=5e-5, frac_tight=1.0))
    for k, p in model.named_parameters():      # the reference's fp32 CPU run carries its own rounding
        ref = d['grad.' + k]
        assert np.abs(p.grad.cpu().numpy() - ref).max() / max(np.abs(ref).max(), 1.0) < 2e-3, k


def test_elbo_nonarmortized_matches_reference(device):
    """GenerativeModel.elbo without an encoder (elbo_unsupervised generative.py:515-544: per-sample
    q_z['unsupervised'] rows over the whole set, the KL of q_z['supervised'] sic) + the supervised
    term, + backward, vs the reference run in elbo_nonarm_c32.npz; same tolerances as the armortized test."""
    from bottleneck.Decoder import CNNDecoder
    from bottleneck.components import EffectivePropertyMap, ReducedOrderModelOperator
    from bottleneck.ROM import ROM
    from bottleneck.generative import GenerativeModel
    from physics.grid import StructuredGrid
    d = load('elbo_nonarm_c32.npz')
    n, nc, dz, Nu, Ns = [int(v) for v in d['cfg']]
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0.)
    g = ReducedOrderModelOperator(ROM(StructuredGrid(nc), n // nc), torch.tensor(d['W']), dtype=torch.float32,
                                  device='cuda')
    gp = EffectivePropertyMap(dz, 2 * nc * nc, dtype=torch.float32, device='cuda')
    model = GenerativeModel(f=dec.cuda(), g=g, gp=gp, dtype=torch.float32, device=torch.device('cuda'))
    model.register_datasets({'supervised': _DS(X=cuda(d['Xs']), Y=cuda(d['Y']), F_ROM_BC=cuda(d['F'])),
                             'unsupervised': _DS(X=cuda(d['Xu']))}, None,
                            create_unsupervised_variational_approximation=True)
    model.load_state_dict({k[6:]: torch.tensor(v) for k, v in d.items() if k.startswith('state.')})
    model.cuda()
    eps = (torch.cat([cuda(d['eps_u']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    elbo = model.elbo(step=0, eps=eps)
    assert abs(elbo.item() - float(d['elbo'])) / abs(float(d['elbo'])) < 2e-5
    (-elbo).backward()
    # fp64 oracle with the kernels' ReLU decisions: value 1e-5, every gradient tensor 5e-5 (no floor)
    from elbo_ref import oracle_nonarm_fixture_elbo, tensor_rel, check_grads
    from gpu_masks import engine_relu_masks
    from test_gpu_c64 import check_mask_audit
    from oracle import codec as ocodec
    engine = model._elbo_engine(Nu, Ns, False, q_unsup=model.q_z['unsupervised'])
    masks = engine_relu_masks(engine)
    assert set(masks) == {'dec_u', 'dec_s'}
    ocodec.MASK_AUDIT.clear()
    val_o, gr_o = oracle_nonarm_fixture_elbo(d, masks=masks)
    check_mask_audit()
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))


def test_elbo_grad_accumulation_semantics(device):
    """zero_grad(set_to_none=False) + two backward passes accumulate like torch.
    Atomic accumulation order is not fixed, so the two passes agree to fp32 rounding only."""
    d = load('elbo_c32.npz')
    model, bs = build_golden_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    (-model.elbo(step=0, armortized_bs=bs, eps=eps)).backward()
    g1 = {k: p.grad.clone() for k, p in model.named_parameters()}
    (-model.elbo(step=0, armortized_bs=bs, eps=eps)).backward()
    for k, p in model.named_parameters():
        torch.testing.assert_close(p.grad, 2 * g1[k], rtol=1e-3, atol=1e-4 * max(1.0, g1[k].abs().max().item()))


# ---------------------------------------------------------------- plumbing kernels
def test_flat_adam_matches_torch(device):
    from gpi import _lib as L
    import ctypes as C
    torch.manual_seed(0)
    p0 = torch.randn(1000, device='cuda')
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-2)
    p = p0.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    lr = torch.tensor([1e-2], device='cuda')
    step = torch.zeros(1, dtype=torch.int64, device='cuda')
    for it in range(5):
        g = torch.randn(1000, device='cuda')
        p_ref.grad = g.clone()
        opt.step()
        step += 1
        dsc = L.AdamDesc(p=p.data_ptr(), g=g.data_ptr(), m=m.data_ptr(), v=v.data_ptr(), n=1000, lr=lr.data_ptr(),
                         step=step.data_ptr(), beta1=0.9, beta2=0.999, eps=1e-8)
        L.check(L.lib().gpi_adam(C.byref(dsc), L.stream_handle()), 'adam')
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)


def test_device_rng(device):
    from gpi import _lib as L
    import ctypes as C
    x = torch.empty(1 << 20, device='cuda')
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    L.check(L.lib().gpi_randn(L.ptr(x), x.numel(), 1234, L.ptr(off), 7, L.stream_handle()), 'randn')
    assert abs(x.mean().item()) < 5e-3 and abs(x.std().item() - 1) < 5e-3
    idx = torch.empty(256, dtype=torch.int32, device='cuda')
    L.check(L.lib().gpi_random_subset(L.ptr(idx), 2048, 256, 99, L.ptr(off), 3, L.stream_handle()), 'subset')
    v = idx.cpu().numpy()
    assert len(set(v.tolist())) == 256 and v.min() >= 0 and v.max() < 2048


@pytest.mark.parametrize('n,k,off', [(1, 1, 0), (7, 3, 5), (1000, 256, 17), (1024, 256, 0), (2048, 2048, 3),
                                      (16384, 16384, 1 << 40), (16384, 64, 9)])
def test_random_subset_exact(device, n, k, off):
    """gpi_random_subset (parallel ranks) = the (Philox key, index) order of the numpy restatement,
    bit for bit, including ties and the maximum pool."""
    from gpi import _lib as L
    from philox_ref import random_subset
    o = torch.tensor([off], dtype=torch.int64, device='cuda')
    idx = torch.full((k,), -1, dtype=torch.int32, device='cuda')
    L.check(L.lib().gpi_random_subset(L.ptr(idx), n, k, 1234567, L.ptr(o), 11, L.stream_handle()), 'subset')
    assert np.array_equal(idx.cpu().numpy(), random_subset(n, k, 1234567, off, 11))


@pytest.mark.parametrize('n,k', [(1024, 256), (2048, 256), (16384, 64), (7, 3)])
def test_step_draws_one_launch_matches_separate_launches(device, n, k):
    """gpi_draws (the fused step's next-step draws in ONE launch: Dropout2d scales, random subset, two noise
    blocks) = gpi_dropout_masks / gpi_random_subset / gpi_randn launched one by one with the same seed,
    offset and sub streams, bit for bit, and the subset = the numpy Philox restatement's."""
    from gpi import _lib as L
    from philox_ref import random_subset
    lib, st = L.lib(), L.stream_handle()
    o = torch.tensor([1 << 33], dtype=torch.int64, device='cuda')
    seed = 97531
    nz, nx, nd = 288 * 64 + 3, 32 * 128, 288 * 23 + 1
    a = dict(idx=torch.full((k,), -1, dtype=torch.int32, device='cuda'), z=torch.full((nz,), 7.0, device='cuda'),
             x=torch.full((nx,), 7.0, device='cuda'), d=torch.full((nd,), 7.0, device='cuda'))
    b = {kk: v.clone() for kk, v in a.items()}
    sseed = 24680                        # the subset's own key (FusedElboStep: the seed shared by the ranks)
    items = [L.DrawItem(kind=L.DRAW_DROPOUT, p=0.2, out=a['d'].data_ptr(), n=nd, sub=5, seed=seed),
             L.DrawItem(kind=L.DRAW_SUBSET, out=a['idx'].data_ptr(), n=n, k=k, sub=1, seed=sseed),
             L.DrawItem(kind=L.DRAW_RANDN, out=a['z'].data_ptr(), n=nz, sub=2, seed=seed),
             L.DrawItem(kind=L.DRAW_RANDN, out=a['x'].data_ptr(), n=nx, sub=3, seed=seed)]
    arr = (L.DrawItem * len(items))(*items)
    L.check(lib.gpi_draws(arr, len(items), L.ptr(o), st), 'draws')
    L.check(lib.gpi_dropout_masks(L.ptr(b['d']), nd, 0.2, seed, L.ptr(o), 5, st), 'masks')
    L.check(lib.gpi_random_subset(L.ptr(b['idx']), n, k, sseed, L.ptr(o), 1, st), 'subset')
    L.check(lib.gpi_randn(L.ptr(b['z']), nz, seed, L.ptr(o), 2, st), 'randn z')
    L.check(lib.gpi_randn(L.ptr(b['x']), nx, seed, L.ptr(o), 3, st), 'randn x')
    torch.cuda.synchronize()
    for kk in a:
        assert torch.equal(a[kk], b[kk]), kk
    assert np.array_equal(a['idx'].cpu().numpy(), random_subset(n, k, sseed, 1 << 33, 1))
    assert set(torch.unique(a['d']).tolist()) <= {0.0, 1.25}


@pytest.mark.parametrize('n,k,off', [(7, 3, 5), (16384, 64, 9), (16385, 256, 0), (65536, 256, 17),
                                      (65536, 65536, 3), (200003, 2048, 1 << 40), (1 << 20, 1024, 5)])
def test_random_subset_any_pool_exact(device, n, k, off):
    """gpi_random_subset_ws: any pool size (the reference's torch.randperm(N)[:k], utils/data.py:441-445,
    has no cap; gpi_random_subset keeps the keys in LDS and stops at 16384) -- the histogram-selected
    candidates ranked -- bit for bit the numpy Philox restatement's (key, index) order, from one element
    past the LDS form's limit to a million, k = n included."""
    import ctypes as C
    from gpi import _lib as L
    from philox_ref import random_subset
    nb = C.c_int64(0)
    L.check(L.lib().gpi_random_subset_workspace(n, C.byref(nb)), 'workspace')
    ws = torch.full((nb.value,), 0xAB, dtype=torch.uint8, device='cuda')      # no zero-init assumed
    o = torch.tensor([off], dtype=torch.int64, device='cuda')
    idx = torch.full((k,), -1, dtype=torch.int32, device='cuda')
    for _ in range(2):                   # a second call on the used workspace gives the same result
        L.check(L.lib().gpi_random_subset_ws(L.ptr(idx), n, k, 1234567, L.ptr(o), 11, L.ptr(ws), nb.value,
                                             L.stream_handle()), 'subset')
        assert np.array_equal(idx.cpu().numpy(), random_subset(n, k, 1234567, off, 11))
        idx.fill_(-1)


# ---------------------------------------------------------------- larger grids (BASELINE configs 4 / 5)
def _codec_case(imsize, blocks, B, seed, dz=64, growth=4, f0=6, masks=True):
    """Per-tensor relative gradient errors (and forward errors) of the native encoder / decoder vs
    the fp64 oracle for one seeded model + input; masks: the oracle takes the kernels' ReLU decisions
    (tests/gpu_masks.py)."""
    from gpu_masks import codec_engine_masks
    from bottleneck.Encoder import CNNEncoder
    from bottleneck.Decoder import CNNDecoder
    from oracle import codec as ocodec
    torch.manual_seed(seed)
    enc = CNNEncoder(imsize, dz, blocks, growth, f0, drop_rate=0)
    dec = CNNDecoder(imsize, dz, (8, 8), 1, f0, blocks, False, growth, drop_rate=0.)
    gen = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for m in list(enc.modules()) + list(dec.modules()):
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(1.0 + 0.3 * torch.randn(m.weight.shape, generator=gen))
                m.bias.copy_(0.2 * torch.randn(m.bias.shape, generator=gen))
    sd_e = {k: v.clone().double() for k, v in enc.state_dict().items()}
    sd_d = {k: v.clone().double() for k, v in dec.state_dict().items()}
    enc, dec = enc.cuda(), dec.cuda()
    X = torch.randn(B, imsize, imsize, generator=gen).double() * 0.8 + 0.4
    wm, ws = torch.randn(B, dz, generator=gen).double(), torch.randn(B, dz, generator=gen).double()
    mu, ls = enc(X.float().cuda())
    mk_e = codec_engine_masks(next(iter(enc._gpi_engines.values())), B) if masks else None
    (torch.sum(mu * wm.float().cuda()) + torch.sum(ls * ws.float().cuda())).backward()
    pe = {k: v.requires_grad_(True) for k, v in sd_e.items() if v.is_floating_point() and 'running' not in k}
    mu_o, ls_o = ocodec.encoder_forward(pe, X, imsize, blocks, growth, f0, masks=mk_e)
    (torch.sum(mu_o * wm) + torch.sum(ls_o * ws)).backward()
    fwd = max(rel(mu.detach().cpu(), mu_o.detach()), rel(ls.detach().cpu(), ls_o.detach()))
    errs = {'enc.' + k: rel(q.grad.cpu(), pe[k].grad) for k, q in enc.named_parameters()}
    Z = torch.randn(B, dz, generator=gen).double()
    vm, vs = torch.randn(B, imsize, imsize, generator=gen).double(), torch.randn(B, imsize, imsize, generator=gen).double()
    Zc = Z.float().cuda().requires_grad_(True)
    mx, lsx = dec(Zc)
    mk_d = codec_engine_masks(next(iter(dec._gpi_engines.values())), B) if masks else None
    (torch.sum(mx * vm.float().cuda()) + torch.sum(lsx * vs.float().cuda())).backward()
    pd = {k: v.requires_grad_(True) for k, v in sd_d.items() if v.is_floating_point() and 'running' not in k}
    Zo = Z.clone().requires_grad_(True)
    mx_o, lsx_o = ocodec.decoder_forward(pd, Zo, 8, blocks, growth, f0, masks=mk_d)
    (torch.sum(mx_o * vm) + torch.sum(lsx_o * vs)).backward()
    fwd = max(fwd, rel(mx.detach().cpu(), mx_o.detach()), rel(lsx.detach().cpu(), lsx_o.detach()))
    errs.update({'dec.' + k: rel(q.grad.cpu(), pd[k].grad) for k, q in dec.named_parameters()})
    errs['dec.Z'] = rel(Zc.grad.cpu(), Zo.grad)
    return fwd, errs


@pytest.mark.parametrize('imsize,blocks,B', [(128, [1, 2, 2, 1], 3), (256, [1, 2, 2, 2, 1], 2)])
def test_codec_large_grids_vs_oracle(device, imsize, blocks, B):
    """Encoder / decoder forward + backward at 128^2 (highres128) and 256^2 (the deeper codec) against
    the fp64 oracle restatement (pinned by the reference fixtures at 32^2 / 64^2), six seeds.

    The oracle takes the kernels' ReLU decisions (tests/gpu_masks.py: the kernels' coefficient
    arithmetic reproduced bit for bit from the stored raw inputs and fp64 batch sums): at these sizes
    the fp64 BN outputs come within ~1e-7 of 0 (below the fp32 forward error), where a different
    branch would move that pixel's share of every upstream gradient.  With the branches fixed, for
    EVERY seed: forward within 1e-5, every gradient tensor within 5e-5 (per-tensor relative, no floor),
    and the mask audit (every adopted decision a tie: |fp64 input| < 1e-4, at most 1e-4 of them)."""
    from test_gpu_c64 import check_mask_audit
    from oracle import codec as ocodec
    for seed in range(6):
        ocodec.MASK_AUDIT.clear()
        fwd, errs = _codec_case(imsize, blocks, B, seed)
        check_mask_audit(max_frac=1e-4)
        assert fwd < 1e-5, (seed, fwd)
        bad = {k: e for k, e in errs.items() if not e < 5e-5}
        assert not bad, (seed, bad)


# ---------------------------------------------------------------- fused training step
@pytest.mark.parametrize('independent_X', [True, False])
def test_fused_step_matches_module_path(device, independent_X):
    """FusedElboStep (graph-capturable step: noise and subset drawn one step ahead, fused epilogue)
    against GenerativeModel.elbo + backward with the same noise / subset and parameters, over two
    steps with the native Adam update in between (training.py:405-417; Adam itself is checked by
    test_flat_adam_matches_torch)."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model, bs = build_golden_model(d, independent_X)
    ref_model = copy.deepcopy(model)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    step = FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=7)
    for it in range(2):
        with torch.no_grad():
            for (k, p), (k2, q) in zip(model.named_parameters(), ref_model.named_parameters()):
                assert k == k2
                q.copy_(p)
        e = step.engine
        eps = (e.eps_z().clone(), e.eps_x().clone() if independent_X else None)
        idx = step.idx.clone().long()
        ref_model._datasets['unsupervised'].perm = idx
        ref_model.zero_grad()
        ref = ref_model.elbo(step=it, armortized_bs=bs, eps=eps)
        (-ref).backward()
        step.forward_backward()
        torch.cuda.synchronize()
        assert abs(step.elbo().item() - ref.item()) <= 1e-5 * abs(ref.item()), (it, step.elbo().item(), ref.item())
        G = step.flat.G
        for k, p in ref_model.named_parameters():
            g = G[step.flat.name_offsets[k]:step.flat.name_offsets[k] + p.numel()].view(p.shape)
            err = (g - p.grad).abs().max().item() / max(p.grad.abs().max().item(), 1.0)
            assert err < 1e-4, (it, k, err)
        assert not torch.equal(step.engine.eps_z(), eps[0])        # next step's noise drawn during this one
        assert len(set(step.idx.tolist())) == bs
        step.update()
        torch.cuda.synchronize()
        # BN running statistics: the fused step updates them as the module path does
        sd, rsd = model.state_dict(), ref_model.state_dict()
        for k in sd:
            if k.endswith(('running_mean', 'running_var', 'num_batches_tracked')):
                torch.testing.assert_close(sd[k], rsd[k], rtol=1e-5, atol=1e-6)
    assert step.step_ctr.item() == 2


@pytest.mark.parametrize('mode', ['single', 'segments', 'streams'])
def test_capture_leaves_training_state_untouched(device, mode):
    """FusedElboStep.capture() warms up on snapshots: parameters, Adam moments, step counter, Philox
    offset and the pre-drawn subset / noise are bit-identical afterwards, and the first replayed step
    is the step an eager loop takes (same ELBO, same parameters after the update) -- in both captured
    forms (one two-stream graph; single-stream segment graphs joined by events)."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model_a, bs = build_golden_model(d)
    model_b = copy.deepcopy(model_a)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    eager = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    import os as _os
    _os.environ['GPI_GRAPH_MODE'] = mode     # read by the constructor ('streams' sets the side step gate)
    try:
        graph = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    finally:
        del _os.environ['GPI_GRAPH_MODE']
    # ('streams' falls back to 'single' when the probe finds the two streams on one hardware queue)
    assert graph.graph_mode == mode or (mode == 'streams' and graph.graph_mode == 'single')
    mode = graph.graph_mode
    before = [t.clone() for t in graph._mutable_state()]
    graph.capture()
    torch.cuda.synchronize()
    for t, b in zip(graph._mutable_state(), before):
        assert torch.equal(t, b)
    for _ in range(3):
        eager.step()
        graph.step()
        torch.cuda.synchronize()
        assert abs(eager.elbo().item() - graph.elbo().item()) <= 1e-6 * abs(eager.elbo().item())
        torch.testing.assert_close(graph.flat.P, eager.flat.P, rtol=1e-6, atol=1e-7)
    assert graph.step_ctr.item() == eager.step_ctr.item() == 3
    assert (graph.segs is not None) == (mode == 'segments')
    assert (graph.g_side is not None) == (mode == 'streams')
    if mode == 'streams':
        graph.check_handoff()
        assert graph.side_done.item() == 3


def test_flag_handoff_matches_event_handoff(device, monkeypatch):
    """The captured step with its side-stream hand-offs as device flags (gpi_stream_signal /
    gpi_stream_wait, the default) leaves exactly what the same step with graph events between the
    streams leaves: parameters, Adam moments, ELBO terms and step counter bit for bit over four
    replays, and no flag wait timed out."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model_a, bs = build_golden_model(d)
    model_b = copy.deepcopy(model_a)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    monkeypatch.setenv('GPI_HANDOFF', 'events')
    ev = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    monkeypatch.setenv('GPI_HANDOFF', 'flags')
    fl = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    assert ev.engine.handoff is None and fl.engine.handoff is not None
    ev.capture()
    fl.capture()
    for _ in range(4):
        ev.step()
        fl.step()
    torch.cuda.synchronize()
    fl.check_handoff()
    for a, b in ((ev.flat.P, fl.flat.P), (ev.m, fl.m), (ev.v, fl.v), (ev.last_terms, fl.last_terms),
                 (ev.step_ctr, fl.step_ctr)):
        assert torch.equal(a, b)
    assert int(fl.handoff_flags[0].item()) == 4        # the tag of the last step (counter 3, + 1)


def test_early_rom_matches_rom_after_head_forward(device, monkeypatch):
    """GPI_ROM_EARLY=1: the captured step's ROM draws X~ = mu + exp(logsigma) eps from q_X in the kernel
    and runs at the start of the step on the side stream (before the encoder) instead of after the
    head forward; the step leaves bit for bit what the default order leaves over four replays."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model_a, bs = build_golden_model(d)
    model_b = copy.deepcopy(model_a)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    monkeypatch.setenv('GPI_GRAPH_MODE', 'streams')
    late = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    monkeypatch.setenv('GPI_ROM_EARLY', '1')
    early = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    if early.graph_mode != 'streams':
        pytest.skip('the stream pair shares a hardware queue here: no side step gate (graph mode single)')
    assert early.engine.rom_draw and not late.engine.rom_draw
    late.capture()
    early.capture()
    assert early.engine.rom_early_launched and not late.engine.rom_early_launched
    for _ in range(4):
        late.step()
        early.step()
    torch.cuda.synchronize()
    early.check_handoff()
    for a, b in ((late.flat.P, early.flat.P), (late.m, early.m), (late.v, early.v),
                 (late.last_terms, early.last_terms), (late.step_ctr, early.step_ctr)):
        assert torch.equal(a, b)


def test_unrolled_graph_matches_single_steps(device):
    """capture(unroll=3) + run(7) (two replays of the 3-step graph pair, then one single step) leaves
    exactly what seven step() replays leave: parameters, Adam moments, counters, subsets, flags."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model_a, bs = build_golden_model(d)
    model_b = copy.deepcopy(model_a)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    one = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    unr = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    one.capture()
    unr.capture(unroll=3)
    if unr.graph_mode != 'streams':
        pytest.skip('the stream pair shares a hardware queue here: no unrolled graphs (graph mode single)')
    assert unr.unroll == 3
    for _ in range(7):
        one.step()
    unr.run(7)
    torch.cuda.synchronize()
    unr.check_handoff()
    for a, b in zip(one._mutable_state(), unr._mutable_state()):
        if a.data_ptr() == one.side_done.data_ptr() and one.graph_mode != 'streams':
            continue            # ('single' keeps no side-stream step counter)
        assert torch.equal(a, b)
    assert int(unr.step_ctr.item()) == 7 and int(unr.side_done.item()) == 7


def test_fused_epilogue_adam_matches_two_launches(device):
    """gpi_step_epilogue_adam (epilogue + Adam in one launch, the single-process default) leaves
    exactly what gpi_step_epilogue followed by gpi_adam leave -- parameters, Adam moments, gradient,
    step counter, Philox offset, terms, subsets and dropout masks, bit for bit, over four captured
    steps (the step is deterministic: its fp64 sums of fp32 terms are exact in any order; both launches
    share the explicit-FMA element update) -- and the arrival counter is back at zero after every launch."""
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model_a, bs = build_golden_model(d)
    model_b = copy.deepcopy(model_a)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    two = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    one = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    two.fuse_adam = False
    assert one.fuse_adam
    two.capture()
    one.capture()
    for _ in range(4):
        two.step()
        one.step()
    torch.cuda.synchronize()
    for a, b in zip(two._mutable_state(), one._mutable_state()):
        assert torch.equal(a, b)
    assert one.step_ctr.item() == 4 and one.done_ctr.item() == 0
    assert one.rng_off.item() == 4 * one.rng_span


def test_lr_schedule_drives_fused_step(device):
    """LearningScheduleWrapper.MultiStepLR (lamp/optimization.py, training.py:452,615) registered on
    FusedElboStep.optimizer changes the learning rate the device Adam uses."""
    from gpi.train import FusedElboStep
    from lamp.optimization import LearningScheduleWrapper
    d = load('elbo_c32.npz')
    model, bs = build_golden_model(d)
    step = FusedElboStep(model, cuda(d['Xu']), bs, cuda(d['Xs']), cuda(d['Y']), cuda(d['F']), lr=1e-2, seed=3)
    sw = LearningScheduleWrapper.MultiStepLR([2, 4], factor=0.1)
    sw.register_optimizer(step.optimizer, 'training')
    step.capture()
    seen = []
    import warnings
    with warnings.catch_warnings():
        warnings.filterwarnings('error', message='.*lr_scheduler.step.*')   # no misleading warning
        for _ in range(6):
            step.step()
            sw.step('training', metric=step.elbo())
            torch.cuda.synchronize()
            seen.append(step.lr.item())
    # the lr in effect during step k (the scheduler steps after it, the fused step picks the new value
    # up when it starts): milestones 2 and 4
    np.testing.assert_allclose(seen, [1e-2, 1e-2, 1e-3, 1e-3, 1e-4, 1e-4], rtol=1e-6)


def test_codec_dropout_matches_reference(device):
    """CNNEncoder / CNNDecoder with drop_rate 0.2 in train mode (codec.py:177-178,218-282) on the native
    codec, with the reference run's Dropout2d masks injected, vs codec_drop_c64.npz."""
    from bottleneck.Encoder import CNNEncoder
    from bottleneck.Decoder import CNNDecoder
    d = load('codec_drop_c64.npz')
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]
    p = float(d['p'])
    enc = CNNEncoder(imsize, dz, blocks, growth, f_enc, drop_rate=p)
    dec = CNNDecoder(imsize, dz, (latent, latent), 1, f_dec, blocks, False, growth, drop_rate=p)
    enc.load_state_dict({k[4:]: torch.tensor(v) for k, v in d.items() if k.startswith('enc.') and
                         not k.startswith('enc.grad.')})
    dec.load_state_dict({k[4:]: torch.tensor(v) for k, v in d.items() if k.startswith('dec.') and
                         not k.startswith('dec.grad.')})
    enc, dec = enc.cuda(), dec.cuda()
    drops = {key: {k[len('drop.%s.' % key):]: cuda(v) for k, v in d.items() if k.startswith('drop.%s.' % key)}
             for key in ('enc', 'dec')}
    object.__setattr__(enc, '_gpi_inject_dropout', drops['enc'])
    mu, ls = enc(cuda(d['X']))
    assert rel(mu.detach().cpu(), d['enc_mu']) < 1e-4
    assert rel(ls.detach().cpu(), d['enc_ls']) < 1e-4
    (torch.sum(mu * cuda(d['enc_wm'])) + torch.sum(ls * cuda(d['enc_ws']))).backward()
    for k, q in enc.named_parameters():
        assert rel(q.grad.cpu(), d['enc.grad.' + k]) < 2e-3, k
    object.__setattr__(dec, '_gpi_inject_dropout', drops['dec'])
    Z = cuda(d['Z']).requires_grad_(True)
    mx, lsx = dec(Z)
    assert rel(mx.detach().cpu(), d['dec_mu']) < 1e-4
    assert rel(lsx.detach().cpu(), d['dec_ls']) < 1e-4
    (torch.sum(mx * cuda(d['dec_vm'])) + torch.sum(lsx * cuda(d['dec_vs']))).backward()
    assert rel(Z.grad.cpu(), d['grad_Z']) < 2e-3
    for k, q in dec.named_parameters():
        assert rel(q.grad.cpu(), d['dec.grad.' + k]) < 2e-3, k
    # without injection the masks are drawn on the device: channel scales 0 or 1/(1-p), about p dropped
    out = [dec(Z)[0] for _ in range(2)]
    assert not torch.equal(out[0], out[1])


def test_dropout_mask_statistics(device):
    """gpi_dropout_masks: values in {0, 1/(1-p)}, drop fraction p."""
    from gpi import _lib as L
    import ctypes as C
    x = torch.empty(1 << 20, device='cuda')
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    L.check(L.lib().gpi_dropout_masks(L.ptr(x), x.numel(), C.c_float(0.2), 5, L.ptr(off), 1, L.stream_handle()), 'm')
    v = x.cpu().numpy()
    assert set(np.unique(v).tolist()) == {0.0, np.float32(1.25)}
    assert abs((v == 0).mean() - 0.2) < 3e-3


def test_bn_running_statistics_match_reference(device):
    """BatchNorm2d running_mean / running_var / num_batches_tracked after two model.elbo calls (train
    mode, momentum 0.1; the decoder's unsupervised and supervised calls update in that order) vs the
    reference run (bn_running_c32.npz)."""
    d = load('bn_running_c32.npz')
    model, bs = build_golden_model(d)
    for call in range(2):
        eps = (torch.cat([cuda(d['eps%d_0' % call]), cuda(d['eps%d_1' % call])]), cuda(d['eps%d_2' % call]))
        model.elbo(step=call, armortized_bs=bs, eps=eps)
    torch.cuda.synchronize()
    sd = model.state_dict()
    n = 0
    for k, v in d.items():
        if not k.startswith('after.'):
            continue
        name = k[6:]
        got = sd[name].cpu().numpy()
        if name.endswith('num_batches_tracked'):
            assert int(got) == int(v), name
        else:
            np.testing.assert_allclose(got, v, rtol=2e-5, atol=2e-6, err_msg=name)
        n += 1
    assert n > 0


def test_fused_output_conv_matches_separate_launches(device, monkeypatch):
    """gpi_conv_loss_fused (the decoder output conv's forward + Gaussian loss + backward in one launch,
    the loss gradient kept in LDS) against the separate forward and backward launches of the same op
    (GPI_FUSE_OUT=0 at engine construction): same ELBO (1e-6, the loss block-sum order differs) and
    the same gradients of every parameter (4e-6 of each tensor's max: the two launch forms sum the weight-
    gradient slab rows and the BN-backward channel sums in different orders, fp32 rounding of sums with
    cancellation -- a BN gamma gradient of ~10^3 from ~10^5 terms measured 1.3e-6 apart (r06); both forms are
    held to the fp64 oracle at 5e-5 per tensor by the ELBO tests)."""
    d = load('elbo_c32.npz')
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    out = {}
    for tag, env in (('fused', '1'), ('separate', '0')):
        monkeypatch.setenv('GPI_FUSE_OUT', env)
        model, bs = build_golden_model(d)
        elbo = model.elbo(step=0, armortized_bs=bs, eps=eps)
        (-elbo).backward()
        eng = model._elbo_engine(bs, int(d['cfg'][5]), False)
        assert eng.n_dec_sep == len(eng.dec_descs) - (1 if env == '1' else 0)
        out[tag] = (elbo.item(), {k: p.grad.detach().cpu().numpy().copy() for k, p in model.named_parameters()})
    (v1, g1), (v0, g0) = out['fused'], out['separate']
    assert abs(v1 - v0) <= 1e-6 * abs(v0), (v1, v0)
    for k in g0:
        assert np.abs(g1[k] - g0[k]).max() <= 4e-6 * max(np.abs(g0[k]).max(), 1e-30), k
