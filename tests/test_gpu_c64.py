"""GPU parity at the BENCHMARKED configuration (BASELINE config 2: highres codec, ROM 8x8 on
64x64, B_u = 256 armortized + N_s = 32 labeled samples) -- the exact shapes bench.py times.

Checked against (1) the reference's own fp32 CPU run of the same step (elbo_c64.npz, rom_c64.npz,
tests/golden/make_golden.py) and (2) the fp64 oracle on identical inputs (tests/elbo_ref.py).
Tolerances: ELBO value 1e-5 relative to the fp64 oracle (north_star); gradients per tensor
relative (max|g - ref| / max|ref|, no floor) by elbo_ref.check_grads: mask-free tensors 1e-4,
median 2e-5, >= 70 % of tensors 1e-4, all 5e-3 (isolated ReLU near-tie flips, see check_grads)."""
import numpy as np
import pytest
import torch

from elbo_ref import load, physics, state_of, oracle_elbo, oracle_fixture_elbo, tensor_rel, check_grads
from oracle import elbo as oelbo

pytestmark = pytest.mark.gpu
_ORACLE = {}


def cuda(a, dtype=torch.float32):
    return torch.tensor(np.asarray(a), dtype=dtype, device='cuda')


def fixture_oracle(name):
    if name not in _ORACLE:
        _ORACLE[name] = oracle_fixture_elbo(load(name))
    return _ORACLE[name]


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


def highres_model(d):
    """ModelFactory('highres') (the bench's model) with the fixture's parameters and data."""
    from factories.model import ModelFactory
    fac = ModelFactory.FromIdentifier('highres')
    fac.set('device', 'cuda')
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


# ---------------------------------------------------------------- the ELBO step at the bench shape
def test_elbo_c64_module_path(device):
    """GenerativeModel.elbo + backward (the drop-in module path) at B_u = 256, N_s = 32 with the
    fixture's injected permutation / noise, vs the fp64 oracle and the reference's fp32 run."""
    d = load('elbo_c64.npz')
    model, bs = highres_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps)
    (-elbo).backward()
    val_o, gr_o = fixture_oracle('elbo_c64.npz')
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    assert abs(elbo.item() - float(d['elbo'])) <= 1e-5 * abs(val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs))


def test_fused_step_c64(device):
    """FusedElboStep -- the graph-captured step bench.py times -- at the benchmarked shape over
    two steps with the native Adam between them: each step's ELBO and gradient vs the fp64 oracle
    evaluated on that step's parameters, subset and device-drawn noise."""
    from gpi.train import FusedElboStep
    d = load('elbo_c64.npz')
    model, bs = highres_model(d)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    step = FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=11)
    n, nc = int(d['cfg'][0]), int(d['cfg'][1])
    names = [k for k, _ in model.named_parameters()]
    for it in range(2):
        e = step.engine
        eps_z = e.eps_z().cpu().numpy().astype(np.float64)
        eps_x = e.eps_x().cpu().numpy().astype(np.float64)
        idx = step.idx.cpu().numpy().astype(np.int64)
        P = step.flat.P
        st = {k: torch.tensor(P[step.flat.name_offsets[k]:step.flat.name_offsets[k] + p.numel()].view(p.shape)
                              .cpu().numpy(), dtype=torch.float64, requires_grad=True)
              for k, p in model.named_parameters()}
        step.forward_backward()
        torch.cuda.synchronize()
        val = oracle_elbo(st, d['Xu'][idx], d['Xs'], d['Y'], d['F'], eps_z[:bs], eps_z[bs:], eps_x, nc, n // nc)
        (-val).backward()
        got = step.elbo().item()
        assert abs(got - val.item()) <= 1e-5 * abs(val.item()), (it, got, val.item())
        G = step.flat.G
        # FusedElboStep's G and the oracle's .grad both hold d(-ELBO)/dtheta
        errs = {k: tensor_rel(G[step.flat.name_offsets[k]:step.flat.name_offsets[k] + st[k].numel()].cpu().numpy()
                              .reshape(st[k].shape), st[k].grad.numpy()) for k in names}
        print('step', it)
        print(check_grads(errs))
        step.update()
        torch.cuda.synchronize()
    assert step.step_ctr.item() == 2


# ---------------------------------------------------------------- elbo(normalize=True), elbo(l2_penalty=...)
@pytest.mark.parametrize('opt', ['norm', 'l2'])
def test_elbo_options(device, opt):
    """normalize=True (every term / its batch size) and l2_penalty (minus penalty * sum of parameter
    norms of f and the encoder), generative.py:247-287, vs the reference run and the fp64 oracle."""
    import sys
    sys.path.insert(0, __file__.rsplit('/', 1)[0])
    from test_gpu_parity import build_golden_model
    d = load('elbo_opts_c32.npz')
    model, bs = build_golden_model(d)
    eps = (torch.cat([cuda(d['eps_enc']), cuda(d['eps_qz'])]), cuda(d['eps_qX']))
    kw = dict(normalize=True) if opt == 'norm' else dict(l2_penalty=float(d['l2_penalty']))
    elbo = model.elbo(step=0, armortized_bs=bs, eps=eps, **kw)
    (-elbo).backward()
    val_o, gr_o = oracle_fixture_elbo(d, **kw)
    assert abs(elbo.item() - val_o) <= 1e-5 * abs(val_o), (elbo.item(), val_o)
    assert abs(elbo.item() - float(d[opt + '.elbo'])) <= 2e-5 * abs(val_o)
    errs = {k: tensor_rel(p.grad.cpu(), gr_o[k]) for k, p in model.named_parameters()}
    print(check_grads(errs))
