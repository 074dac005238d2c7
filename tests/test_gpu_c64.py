"""GPU parity at the BENCHMARKED configuration (BASELINE config 2: highres codec, ROM 8x8 on
64x64, B_u = 256 armortized + N_s = 32 labeled samples) -- the exact shapes bench.py times.

Checked against (1) the reference's own fp32 CPU run of the same step (elbo_c64.npz, rom_c64.npz,
tests/golden/make_golden.py) and (2) the fp64 oracle on identical inputs (tests/elbo_ref.py).
Tolerances: ELBO value 1e-5 relative to the fp64 oracle (north_star); every gradient tensor
5e-5 relative (r02c: worst 1.4e-5) (max|g - ref| / max|ref|, no floor), median 2e-5.  The oracle takes the kernels'
ReLU decisions (tests/gpu_masks.py): among the ~10^7 activations of a C64 batch a few tens lie
within fp32 rounding of 0, and a different branch there moves every gradient upstream of that
pixel by up to 1e-2 (measured r02b without this); the audit below checks that every decision
the oracle adopts is such a tie (|fp64 input| < 1e-4) and that there are few of them."""
import numpy as np
import pytest
import torch

from elbo_ref import load, physics, state_of, oracle_elbo, oracle_fixture_elbo, tensor_rel, check_grads
from oracle import codec as ocodec
from oracle import elbo as oelbo

pytestmark = pytest.mark.gpu
_ORACLE = {}


def cuda(a, dtype=torch.float32):
    return torch.tensor(np.asarray(a), dtype=dtype, device='cuda')


def check_mask_audit(max_abs=1e-4, max_frac=1e-5):
    """The decisions taken from the kernels differ from the oracle's own sign tests only at ties."""
    n_dis = sum(a[1] for a in ocodec.MASK_AUDIT)
    n_all = sum(a[3] for a in ocodec.MASK_AUDIT)
    worst = max((a[2] for a in ocodec.MASK_AUDIT), default=0.0)
    rep = [a for a in ocodec.MASK_AUDIT if a[1]]
    print('relu ties adopted from the kernels: %d of %d activations, largest |x| %.2e %s' % (n_dis, n_all, worst, rep))
    assert n_all > 0
    assert worst < max_abs, rep
    assert n_dis <= max_frac * n_all, rep
    ocodec.MASK_AUDIT.clear()


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


def highres_model(d, droprate=0.0):
    """ModelFactory('highres') (the bench's model) with the fixture's parameters and data."""
    from factories.model import ModelFactory
    fac = ModelFactory.FromIdentifier('highres')
    fac.set('device', 'cuda')
    fac.set('droprate', droprate)
    physics_, model, _, encoder, _, _ = fac.setup()
    model.encoder = encoder.cuda()
    n, nc, dz, Nu, bs, Ns = [int(v) for v in d['cfg']]
    assert physics_['fom'].grid.n == n and physics_['rom'].grid.n == nc and model.dim_latent == dz
    perm = torch.tensor(d['perm'], device='cuda')
    model.register_datasets({'supervised': _DS(X=cuda(d['Xs']), Y=cuda(d['Y']), F_ROM_BC=cuda(d['F'])),
                             'unsupervised': _DS(perm=perm, X=cuda(d['Xu']))}, None,
                            create_unsupervised_variational_approximation=False)
    model.load_state_dict({k[6:]: torch.tensor(v) for k, v in d.items() if k.startswith('state.')})
    model.cuda()
    return model, bs


# ---------------------------------------------------------------- ROM nc = 8 (register-window Cholesky)
def test_rom_c64_operator(device):
    """nc = 8: the single-lane register-window Cholesky / band solves of rom.hip at the benchmarked
    batch (N = 32) vs the reference run (rom_c64.npz) and the fp64 oracle."""
    from gpi.native import RomOperatorFunction
    d = load('rom_c64.npz')
    nc, r = int(d['nc']), int(d['r'])
    M, W, bc = physics(nc, r)
    x = cuda(d['effprop']).requires_grad_(True)
    mu, uc = RomOperatorFunction.apply(x, cuda(d['F']), nc, r, False)
    e64 = torch.tensor(d['effprop'], dtype=torch.float64, requires_grad=True)
    ls64 = torch.tensor(d['logsigmas_y'], dtype=torch.float64, requires_grad=True)
    mu_o, lso = oelbo.rom_operator(torch.tensor(W), torch.tensor(M), torch.tensor(bc), e64,
                                   torch.tensor(d['F'], dtype=torch.float64), ls64)
    assert tensor_rel(mu.detach().cpu(), mu_o.detach()) < 1e-5
    assert tensor_rel(mu.detach().cpu(), d['mu_y']) < 2e-5
    ls = cuda(d['logsigmas_y']).requires_grad_(True)
    Y = cuda(d['Y'])
    L = torch.sum(-0.5 * (2 * ls + (Y - mu) ** 2 * torch.exp(-2 * ls) + 1.8378770664093453))
    (-L).backward()
    Lo = oelbo.dgll(torch.tensor(d['Y'], dtype=torch.float64), mu_o, 2 * lso)
    (-Lo).backward()
    assert abs(L.item() - Lo.item()) <= 1e-5 * abs(Lo.item())
    assert tensor_rel(x.grad.cpu(), e64.grad) < 1e-4
    assert tensor_rel(ls.grad.cpu(), ls64.grad) < 1e-5
    assert tensor_rel(x.grad.cpu(), d['grad_effprop']) < 1e-3


def test_rom_c64_fused_loglik(device):
    """gpi_rom ROM_LOGLIK (the ELBO engine's launch: solve + W u + log-lik + adjoint) at nc = 8."""
    from gpi.engine import rom_call
    from gpi import _lib as L
    d = load('rom_c64.npz')
    nc, r = int(d['nc']), int(d['r'])
    M, W, bc = physics(nc, r)
    x, F, Y, ls = cuda(d['effprop']), cuda(d['F']), cuda(d['Y']), cuda(d['logsigmas_y'])
    gx = torch.zeros_like(x)
    gls = torch.zeros(ls.shape[0], dtype=torch.float64, device='cuda')
    acc = torch.zeros(L.GPI_REPLICAS, dtype=torch.float64, device='cuda')
    flag = torch.zeros(1, dtype=torch.int32, device='cuda')
    rom_call(nc, r, x, F, False, L.ROM_LOGLIK, Y=Y, logsig_y=ls, gx=gx, gacc_logsig=gls, loss_acc=acc, flag=flag)
    e64 = torch.tensor(d['effprop'], dtype=torch.float64, requires_grad=True)
    ls64 = torch.tensor(d['logsigmas_y'], dtype=torch.float64, requires_grad=True)
    mu_o, lso = oelbo.rom_operator(torch.tensor(W), torch.tensor(M), torch.tensor(bc), e64,
                                   torch.tensor(d['F'], dtype=torch.float64), ls64)
    Lo = oelbo.dgll(torch.tensor(d['Y'], dtype=torch.float64), mu_o, 2 * lso)
    (-Lo).backward()
    assert abs(acc.sum().item() - Lo.item()) <= 1e-5 * abs(Lo.item())
    # gx / gls hold d(-logL)/dx, d(-logL)/dlogsigma_y
    assert tensor_rel(gx.cpu(), e64.grad) < 1e-4
    assert tensor_rel(gls.cpu(), ls64.grad) < 1e-5
    assert flag.item() == 0
    # gls_part: the same contributions as per-sample rows (plain stores; the engine reduces them)
    part = torch.full((x.shape[0], ls.shape[0]), float('nan'), device='cuda')
    gx2 = torch.zeros_like(x)
    acc2 = torch.zeros_like(acc)
    rom_call(nc, r, x, F, False, L.ROM_LOGLIK, Y=Y, logsig_y=ls, gx=gx2, gls_part=part, loss_acc=acc2, flag=flag)
    assert torch.isfinite(part).all()
    assert tensor_rel(part.double().sum(0).cpu(), ls64.grad) < 1e-5
    assert torch.equal(gx2, gx) and torch.equal(acc2, acc)


@pytest.mark.parametrize('nc', [4, 8])
def test_rom_coarse_solutions_lane_per_sample(device, nc):
    """gpi_rom FORWARD without mu_y (the VO MC predictive's coarse solves: rom_lane_kernel, one lane per
    sample, 16 384 samples at the notebook's 128 x 128) vs the workgroup-per-sample kernel (FORWARD with
    mu_y) on the same inputs, and a subset vs the fp64 oracle solve (ROM.py:59-100)."""
    from gpi.engine import rom_call
    from gpi import _lib as L
    r = 8
    M, W, bc = physics(nc, r)
    rng = np.random.default_rng(nc)
    N = 16384 + 37                                   # a ragged last wave
    x = cuda(rng.normal(0.3, 0.7, (N, 2 * nc * nc)))
    F = torch.zeros(N, (nc + 1) ** 2, device='cuda')
    Fh = np.zeros((N, (nc + 1) ** 2), dtype=np.float32)
    bnodes = [e for e in range((nc + 1) ** 2) if e % (nc + 1) in (0, nc)]
    Fh[:, bnodes] = rng.uniform(-0.5, 0.5, (N, len(bnodes)))
    F.copy_(torch.from_numpy(Fh))
    uc_lane = torch.empty(N, (nc + 1) ** 2, device='cuda')
    rom_call(nc, r, x, F, False, L.ROM_FORWARD, uc=uc_lane)
    uc_wg = torch.empty_like(uc_lane)
    mu = torch.empty(N, (nc * r + 1) * (nc * r - 1), device='cuda')
    rom_call(nc, r, x, F, False, L.ROM_FORWARD, mu_y=mu, uc=uc_wg)
    assert tensor_rel(uc_lane.cpu(), uc_wg.cpu().numpy().astype(np.float64)) < 2e-6
    sel = [0, 1, 777, N - 1]
    e64 = torch.tensor(x[sel].cpu().numpy(), dtype=torch.float64)
    u = oelbo.rom_solve(torch.tensor(M), torch.exp(e64) + 1e-8, torch.tensor(Fh[sel], dtype=torch.float64),
                        torch.tensor(bc))
    assert tensor_rel(uc_lane[sel].cpu(), u) < 1e-5


# ---------------------------------------------------------------- the ELBO step at the bench shape
def test_elbo_c64_module_path(device):
    """GenerativeModel.elbo + backward (the drop-in module path) at B_u = 256, N_s = 32 with the
    fixture's injected permutation / noise, vs the fp64 oracle and the reference's fp32 run."""
    from gpu_masks import engine_relu_masks
    d = load('elbo_c64.npz')
    model, bs = highres_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps)
    (-elbo).backward()
    masks = engine_relu_masks(model._elbo_engine(bs, int(d['cfg'][5]), False))
    ocodec.MASK_AUDIT.clear()
    val_o, gr_o = oracle_fixture_elbo(d, masks=masks)
    check_mask_audit()
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    assert abs(elbo.item() - float(d['elbo'])) <= 1e-5 * abs(val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))


def test_head_mfma_matches_valu_form(device):
    """The dense layers of the step (encoder FC -> ReLU -> mu / logsigma heads, reparametrisation, KL,
    decoder latent map, gp map, q_X draw and their backward, Encoder.py:175-182, codec.py:495-504,
    Decoder.py:213, components.py:167-256) on the matrix cores (head_fwd_mfma / head_bwd_mfma /
    outer_gemm_mfma, the default) vs the per-sample VALU kernels (GPI_HEAD_VALU) on the same workspace
    state at the bench shape: every output region and every gradient tensor within 1e-5 of the VALU
    form's (max|d| / max|ref|; both are fp32, the sums differ only in order), the ELBO terms within
    1e-6.  The fp64 oracle checks of the whole step (above and below) run through the MFMA form."""
    import ctypes as C
    from gpi import _lib as L
    d = load('elbo_c64.npz')
    model, bs = highres_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    (-model.elbo(step=0, armortized_bs=bs, eps=eps)).backward()
    e = model._elbo_engine(bs, int(d['cfg'][5]), False)
    lib, st = L.lib(), L.stream_handle()
    P, ws, scr, gacc = e.flat.P, e.ws.t_ws, e.ws.t_scr, e.flat.gacc
    ws0 = ws.clone()

    def run(valu):
        ws.copy_(ws0)
        scr.zero_()
        gacc.zero_()
        hd = L.HeadDesc.from_buffer_copy(e.head)
        if valu:
            hd.flags |= L.HEAD_VALU
        items = (L.GemmItem * len(e.gemm_items))(*[L.GemmItem.from_buffer_copy(it) for it in e.gemm_items])
        if valu:
            items[0].flags |= 2
        L.check(lib.gpi_head_forward(C.byref(hd), L.ptr(P), L.ptr(ws), st), 'head forward')
        L.check(lib.gpi_head_backward(C.byref(hd), L.ptr(P), L.ptr(ws), L.ptr(gacc), st), 'head backward')
        L.check(lib.gpi_outer_gemm(items, len(items), L.ptr(ws), L.ptr(gacc), st), 'outer gemm')
        torch.cuda.synchronize()
        return ws.clone(), e.ws.terms.clone(), gacc.clone()

    wm, tm, gm = run(False)
    wv, tv, gv = run(True)
    B, dz = e.B, e.dz
    h = e.head
    regions = {k: (e.hb[k], n) for k, n in (('hpre', e.B_u * h.d_feat), ('dhpre', e.B_u * h.d_feat),
                                            ('zmu', B * dz), ('zls', B * dz), ('z', B * dz), ('dzmu', B * dz),
                                            ('dzls', B * dz), ('mux', e.N_s * h.d_x), ('xs', e.N_s * h.d_x),
                                            ('gmux', e.N_s * h.d_x))}
    regions['lat'] = (h.lat, B * h.d_lat)
    regions['gfeat'] = (h.gfeat, e.B_u * h.d_feat)
    for k, (o, n) in regions.items():
        a, b = wm[o:o + n].double(), wv[o:o + n].double()
        assert float(b.abs().max()) > 0, k
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()), k
    assert torch.allclose(tm, tv, rtol=1e-6, atol=0), (tm, tv)
    off = e.flat.name_offsets
    n_checked = 0
    for k, p in model.named_parameters():
        a, b = gm[off[k]:off[k] + p.numel()], gv[off[k]:off[k] + p.numel()]
        if float(b.abs().max()) == 0:
            continue
        n_checked += 1
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()), k
    assert n_checked >= 12, n_checked


@pytest.mark.parametrize('droprate', [0.0, 0.2])
def test_fused_step_c64(device, droprate):
    """FusedElboStep -- the graph-captured step bench.py times -- at the benchmarked shape over three
    steps with the native Adam between them.  Every step: the ELBO vs the fp64 oracle on that step's
    parameters, subset and device-drawn noise (1e-5); the gradient vs the module path
    (GenerativeModel.elbo, itself checked against the oracle above) on the same inputs, 1e-5 per
    tensor (same kernels); and vs the fp64 oracle with the kernels' ReLU tie decisions: every
    tensor 5e-5, median 2e-5."""
    from gpu_masks import engine_relu_masks
    import copy
    from gpi.train import FusedElboStep
    d = load('elbo_c64.npz')
    model, bs = highres_model(d, droprate)
    ref_model = copy.deepcopy(model)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    step = FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=11)
    n, nc = int(d['cfg'][0]), int(d['cfg'][1])
    names = [k for k, _ in model.named_parameters()]
    off = step.flat.name_offsets
    for it in range(3):
        e = step.engine
        eps_z_t, eps_x_t = e.eps_z().clone(), e.eps_x().clone()
        # the step's device-drawn Dropout2d scales (highres: p = 0.2, factories/model.py:187)
        drops = {k: {n: v.clone() for n, v in dd.items()} for k, dd in e.dropout_views().items()}
        assert bool(drops) == (droprate > 0)
        for dd in drops.values():
            for v in dd.values():
                u = torch.unique(v)
                assert set(u.tolist()) <= {0.0, 1.0 / (1.0 - droprate)}
        eps_z = eps_z_t.cpu().numpy().astype(np.float64)
        eps_x = eps_x_t.cpu().numpy().astype(np.float64)
        idx_t = step.idx.clone().long()
        idx = idx_t.cpu().numpy()
        with torch.no_grad():
            for (k, p), (k2, q) in zip(model.named_parameters(), ref_model.named_parameters()):
                assert k == k2
                q.copy_(p)
        ref_model._datasets['unsupervised'].perm = idx_t
        ref_model.zero_grad()
        ref = ref_model.elbo(step=it, armortized_bs=bs, eps=(eps_z_t, eps_x_t), dropout=drops or None)
        (-ref).backward()
        st = {k: torch.tensor(p.detach().cpu().numpy(), dtype=torch.float64, requires_grad=True)
              for k, p in ref_model.named_parameters()}
        masks = engine_relu_masks(ref_model._elbo_engine(bs, int(d['cfg'][5]), False))
        step.forward_backward()
        torch.cuda.synchronize()
        if droprate > 0:
            # the next step's masks, drawn during this step (decoder: side stream; encoder: the step
            # epilogue) = gpi_dropout_masks at this step's Philox offset, sub ids 4 (enc) / 5 (dec)
            from gpi import _lib as L
            for k, sub in (('enc', 4), ('dec', 5)):
                prog = e.ep if k == 'enc' else e.dp
                ref_m = torch.empty(prog.drop_numel, dtype=torch.float32, device='cuda')
                L.check(L.lib().gpi_dropout_masks(L.ptr(ref_m), prog.drop_numel, prog.drop_rate, step.seed,
                                                  L.ptr(step.rng_off), sub, L.stream_handle()), 'masks')
                torch.cuda.synchronize()
                got_m = e.ws.view(prog.drop_off, prog.drop_numel)
                assert torch.equal(got_m, ref_m), k
                assert not all(torch.equal(v, drops[k][n]) for n, v in e.dropout_views()[k].items()), k
        ocodec.MASK_AUDIT.clear()
        val = oracle_elbo(st, d['Xu'][idx], d['Xs'], d['Y'], d['F'], eps_z[:bs], eps_z[bs:], eps_x, nc, n // nc,
                          masks=masks, drops={k: {n: v.double().cpu() for n, v in dd.items()}
                                              for k, dd in drops.items()})
        check_mask_audit()
        (-val).backward()
        got = step.elbo().item()
        assert abs(got - val.item()) <= 1e-5 * abs(val.item()), (it, got, val.item())
        assert abs(got - ref.item()) <= 1e-6 * abs(val.item()), (it, got, ref.item())
        G = step.flat.G
        # FusedElboStep's G, the module path's .grad and the oracle's .grad all hold d(-ELBO)/dtheta
        g_of = lambda k: G[off[k]:off[k] + st[k].numel()].cpu().numpy().reshape(st[k].shape)
        errs_mod = {k: tensor_rel(g_of(k), p.grad.cpu().numpy()) for k, p in ref_model.named_parameters()}
        bad = {k: v for k, v in errs_mod.items() if v >= 1e-5}
        assert not bad, (it, bad)
        errs = {k: tensor_rel(g_of(k), st[k].grad.numpy()) for k in names}
        print('step', it)
        print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))
        step.update()
        torch.cuda.synchronize()
    assert step.step_ctr.item() == 3


# ---------------------------------------------------------------- elbo(normalize=True), elbo(l2_penalty=...)
@pytest.mark.parametrize('opt', ['norm', 'l2', 'expf'])
def test_elbo_options(device, opt):
    """normalize=True (every term / its batch size) and l2_penalty (minus penalty * sum of parameter
    norms of f and the encoder), generative.py:247-287, and reconstruct_log_eff_property=False (the
    decoder's Gaussian on exp(x), generative.py:236-239), vs the reference run (value 2e-5) and the fp64
    oracle with the kernels' ReLU decisions (value 1e-5, every gradient tensor 5e-5, mask audit)."""
    import sys
    sys.path.insert(0, __file__.rsplit('/', 1)[0])
    from test_gpu_parity import build_golden_model
    d = load('elbo_opts_c32.npz')
    model, bs = build_golden_model(d)
    if opt == 'expf':        # Gaussian on the exponentiated field: the EPI_GAUSS_EXP_LOSS epilogue
        model.set('reconstruct_log_eff_property', False)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    kw = {'norm': dict(normalize=True), 'l2': dict(l2_penalty=float(d['l2_penalty'])), 'expf': {}}[opt]
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps, **kw)
    (-elbo).backward()
    # the fp64 oracle with the kernels' ReLU decisions (as every ELBO variant since r03): value 1e-5,
    # every gradient tensor 5e-5 per-tensor relative, no floor
    from gpu_masks import engine_relu_masks
    masks = engine_relu_masks(model._elbo_engine(bs, int(d['cfg'][5]), opt == 'norm'))
    ocodec.MASK_AUDIT.clear()
    val_o, gr_o = oracle_fixture_elbo(d, log_field=opt != 'expf', masks=masks, **kw)
    check_mask_audit()
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    assert abs(elbo.item() - float(d[opt + '.elbo'])) <= 2e-5 * abs(val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))


# ---------------------------------------------------------------- scale-up grids (BASELINE configs 4 / 5)
@pytest.mark.parametrize('ident,n,Nu,bs,Ns', [('highres128', 128, 8, 4, 2), ('highres256', 256, 8, 4, 2),
                                               ('highres128', 128, 512, 256, 32), ('highres256', 256, 256, 128, 32)],
                         ids=['c128-small', 'c256-small', 'c128-config4', 'c256-config5'])
def test_fused_step_scaleup_grids(device, ident, n, Nu, bs, Ns):
    """FusedElboStep at 128^2 (highres128: blocks [1,2,2,1]) and 256^2 (highres256: [1,2,2,2,1]), ROM 8x8,
    droprate 0.2 (device-drawn Dropout2d), random-init parameters and synthetic fields: one step's ELBO
    vs the fp64 oracle (1e-5) and every gradient tensor vs the oracle with the kernels' ReLU tie
    decisions and dropout scales (5e-5 per tensor).  Small batches (B_u = 4 of a pool of 8, N_s = 2),
    BASELINE config 4's own shape (128^2, B_u = 256 of 512, N_s = 32: the launch geometry bench.py
    --config c128 times) and config 5's per-GPU shape (256^2, B_u = 128 of 256, N_s = 32: bench.py
    --config c256)."""
    from gpu_masks import engine_relu_masks
    from factories.model import ModelFactory
    from gpi.train import FusedElboStep
    import copy
    torch.manual_seed(3)
    fac = ModelFactory.FromIdentifier(ident)
    fac.set('device', 'cuda')
    physics_, model, _, encoder, _, _ = fac.setup()
    model.encoder = encoder.cuda()
    nc = physics_['rom'].grid.n
    assert physics_['fom'].grid.n == n
    rng = np.random.default_rng(n)
    Xu = rng.normal(0.3, 0.6, (Nu, n, n)).astype(np.float32)
    Xs = rng.normal(0.3, 0.6, (Ns, n, n)).astype(np.float32)
    Y = rng.normal(0.0, 0.3, (Ns, (n + 1) * (n - 1))).astype(np.float32)
    F = np.zeros((Ns, (nc + 1) ** 2), dtype=np.float32)
    bnodes = [e for e in range((nc + 1) ** 2) if e % (nc + 1) in (0, nc)]
    F[:, bnodes] = rng.uniform(-0.5, 0.5, (Ns, len(bnodes)))
    model.register_datasets({'supervised': _DS(X=cuda(Xs), Y=cuda(Y), F_ROM_BC=cuda(F)),
                             'unsupervised': _DS(perm=torch.arange(Nu, device='cuda'), X=cuda(Xu))}, None,
                            create_unsupervised_variational_approximation=False)
    model.cuda()
    ref_model = copy.deepcopy(model)
    step = FusedElboStep(model, cuda(Xu), bs, cuda(Xs), cuda(Y), cuda(F), lr=1e-3, seed=5)
    e = step.engine
    eps_z_t, eps_x_t = e.eps_z().clone(), e.eps_x().clone()
    drops_t = {k: {nm: v.clone() for nm, v in dd.items()} for k, dd in e.dropout_views().items()}
    assert drops_t
    idx_t = step.idx.clone().long()
    st = {k: torch.tensor(p.detach().cpu().numpy(), dtype=torch.float64, requires_grad=True)
          for k, p in model.named_parameters()}
    # the module path on the same inputs gives the kernels' ReLU decisions for the oracle
    ref_model._datasets['unsupervised'].perm = idx_t
    ref = ref_model.elbo(step=0, armortized_bs=bs, eps=(eps_z_t, eps_x_t), dropout=drops_t)
    masks = engine_relu_masks(ref_model._elbo_engine(bs, Ns, False))
    step.forward_backward()
    torch.cuda.synchronize()
    eps_z = eps_z_t.cpu().numpy().astype(np.float64)
    eps_x = eps_x_t.cpu().numpy().astype(np.float64)
    idx = idx_t.cpu().numpy()
    drops = {k: {nm: v.double().cpu() for nm, v in dd.items()} for k, dd in drops_t.items()}
    ocodec.MASK_AUDIT.clear()
    val = oracle_elbo(st, Xu[idx], Xs, Y, F, eps_z[:bs], eps_z[bs:], eps_x, nc, n // nc, masks=masks, drops=drops)
    check_mask_audit()
    (-val).backward()
    got = step.elbo().item()
    assert abs(got - val.item()) <= 1e-5 * abs(val.item()), (got, val.item())
    assert abs(got - ref.item()) <= 1e-6 * abs(val.item()), (got, ref.item())
    G = step.flat.G
    off = step.flat.name_offsets
    errs = {k: tensor_rel(G[off[k]:off[k] + st[k].numel()].cpu().numpy().reshape(st[k].shape), st[k].grad.numpy())
            for k in st}
    print(check_grads(errs, tol_all=5e-5, frac_tight=1.0))


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_codec_module_path_vs_oracle(device, tag):
    """The standalone CNNEncoder / CNNDecoder module path (Encoder.py:191-196, Decoder.py:288-305 on
    the native codec) on the reference fixture's weights and inputs vs the fp64 oracle codec with the
    kernels' ReLU decisions (tests/gpu_masks.py, bit-exact coefficient arithmetic): forward 1e-5 and
    every gradient tensor 5e-5 per-tensor relative (max|d| / max|ref|, no floor), mask audit -- the
    tie-aware form of test_encoder_forward_backward / test_decoder_forward_backward (which compare
    with the reference's own fp32 run)."""
    import sys
    sys.path.insert(0, __file__.rsplit('/', 1)[0])
    from test_gpu_parity import _codec
    from gpu_masks import _program_masks, replica_sums
    from gpi import _lib as L
    from gpi.engine import N_TERMS
    d, enc, dec = _codec(tag)
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]

    def engine_masks(e, B):
        torch.cuda.synchronize()
        ws = e.ws
        R, G = L.GPI_REPLICAS, L.GPI_MAX_GROUPS
        scr = ws.t_scr.cpu().numpy()
        o = N_TERMS * R
        stats = replica_sums(scr[o:o + R * G * ws.n_stats * 4].reshape(R, G, ws.n_stats, 4))
        return _program_masks(e.p, ws.t_ws.cpu().numpy(), stats, e.flat.P.detach().cpu().numpy(),
                              slice(0, B), 0, B), ws

    # ---- encoder
    X = cuda(d['X'])
    mu, ls = enc(X)
    e = next(iter(enc._gpi_engines.values()))
    masks, ws = engine_masks(e, X.shape[0])
    hp = ws.t_ws.cpu().numpy()[e.hb['hpre']:e.hb['hpre'] + X.shape[0] * e.p.d_feat]
    masks['features.FC'] = torch.tensor(hp.reshape(X.shape[0], -1) > 0)
    (torch.sum(mu * cuda(d['enc_wm'])) + torch.sum(ls * cuda(d['enc_ws']))).backward()
    pe = {k[4:]: torch.tensor(v, dtype=torch.float64).requires_grad_(True) for k, v in d.items()
          if k.startswith('enc.') and not k.startswith('enc.grad.') and 'running' not in k and 'num_batches' not in k}
    ocodec.MASK_AUDIT.clear()
    mu_o, ls_o = ocodec.encoder_forward(pe, torch.tensor(d['X'], dtype=torch.float64), imsize, blocks, growth, f_enc,
                                        masks=masks)
    (torch.sum(mu_o * torch.tensor(d['enc_wm'], dtype=torch.float64)) +
     torch.sum(ls_o * torch.tensor(d['enc_ws'], dtype=torch.float64))).backward()
    check_mask_audit(max_frac=1e-4)
    assert tensor_rel(mu.detach().cpu().numpy(), mu_o.detach().numpy()) < 1e-5
    assert tensor_rel(ls.detach().cpu().numpy(), ls_o.detach().numpy()) < 1e-5
    errs = {k: tensor_rel(p.grad.cpu().numpy(), pe[k].grad.numpy()) for k, p in enc.named_parameters()}
    bad = {k: v for k, v in errs.items() if not v < 5e-5}
    assert not bad, bad
    # ---- decoder
    Z = cuda(d['Z']).requires_grad_(True)
    mx, lsx = dec(Z)
    e = next(iter(dec._gpi_engines.values()))
    masks, _ = engine_masks(e, Z.shape[0])
    (torch.sum(mx * cuda(d['dec_vm'])) + torch.sum(lsx * cuda(d['dec_vs']))).backward()
    pd = {k[4:]: torch.tensor(v, dtype=torch.float64).requires_grad_(True) for k, v in d.items()
          if k.startswith('dec.') and not k.startswith('dec.grad.') and 'running' not in k and 'num_batches' not in k}
    Zo = torch.tensor(d['Z'], dtype=torch.float64).requires_grad_(True)
    mx_o, lsx_o = ocodec.decoder_forward(pd, Zo, latent, blocks, growth, f_dec, masks=masks)
    (torch.sum(mx_o * torch.tensor(d['dec_vm'], dtype=torch.float64)) +
     torch.sum(lsx_o * torch.tensor(d['dec_vs'], dtype=torch.float64))).backward()
    check_mask_audit(max_frac=1e-4)
    assert tensor_rel(mx.detach().cpu().numpy(), mx_o.detach().numpy()) < 1e-5
    assert tensor_rel(lsx.detach().cpu().numpy(), lsx_o.detach().numpy()) < 1e-5
    errs = {k: tensor_rel(p.grad.cpu().numpy(), pd[k].grad.numpy()) for k, p in dec.named_parameters()}
    errs['Z'] = tensor_rel(Z.grad.cpu().numpy(), Zo.grad.numpy())
    bad = {k: v for k, v in errs.items() if not v < 5e-5}
    assert not bad, bad

