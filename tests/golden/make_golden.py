"""Generate golden fixtures by running the REFERENCE's own torch modules.

Run here (where /root/reference exists), never on the GPU box:

    python tests/golden/make_golden.py

The reference imports FEniCS/DOLFIN/PETSc/prettytable, none of which exist in
this image; they are replaced by inert ``MagicMock`` modules.  Everything
FEniCS would *compute* (M, W, F_ROM_BC, Y, Gamma, alpha) is supplied by the
oracle's generic P1 restatement (oracle/fem.py).  ``torch.solve`` (removed in
torch 2) is shimmed to ``torch.linalg.solve`` (ROM.py:59-62; same math).
Random draws are injected by patching ``torch.randn_like`` / ``torch.randperm``
with queues of pre-drawn tensors, which are saved with the fixtures.

Outputs (small .npz, float32 unless noted) -- inputs, outputs and gradients:
  codec_c32.npz / codec_c64.npz   CNNEncoder / CNNDecoder fwd + bwd
  rom_c32.npz                     ROM solve + ReducedOrderModelOperator bwd
  elbo_c32.npz                    GenerativeModel.elbo (armortized + freeX) + bwd
  elbo_nonarm_c32.npz             GenerativeModel.elbo without an encoder (elbo_unsupervised + freeX) + bwd
  vo_c32.npz                      VirtualObservable.update / precision (fp64)
  vo_elbo_c32.npz                 GenerativeModel.update_virtual_observables (x2, CGR + flux
                                  queries through the reference's own sampler / LinearQuerry /
                                  VirtualObservablesEnsemble classes) + elbo with the VO term + bwd
  vo_elbo_lockx_c32.npz           the same with independent_X=False (lockX: X~ = gp(z))
  pe_analysis_c32.npz             PredictionEnsemble.update (3 iterations, own Adam) and
                                  Analysis.eval_all_y (relerr / logscore / R^2)
  terms.npz                       DGLL / KL known values
"""
import os
import sys
import types
from unittest import mock

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, ROOT)
from oracle import fem  # noqa: E402

for m in ['fenics', 'dolfin', 'petsc4py', 'petsc4py.PETSc', 'prettytable']:
    sys.modules[m] = mock.MagicMock()
sys.path.insert(0, REF)

import bottleneck.utils as R_utils            # noqa: E402
import bottleneck.ROM as R_ROM                # noqa: E402
import bottleneck.components as R_comp        # noqa: E402
import bottleneck.generative as R_gen         # noqa: E402
import bottleneck.VirtualObservables as R_VO  # noqa: E402
import lamp.optimization as R_opt             # noqa: E402
from bottleneck.Encoder import CNNEncoder     # noqa: E402
from bottleneck.Decoder import CNNDecoder     # noqa: E402

R_ROM.ROM._solve_eqs = lambda self, A, B: torch.linalg.solve(A, B)


def sd(module, prefix=''):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def grads(module, prefix='grad.'):
    return {prefix + k: p.grad.detach().cpu().numpy().copy()
            for k, p in module.named_parameters() if p.grad is not None}


def randomize_bn(module, gen):
    with torch.no_grad():
        for m in module.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(1.0 + 0.3 * torch.randn(m.weight.shape, generator=gen))
                m.bias.copy_(0.2 * torch.randn(m.bias.shape, generator=gen))


def random_fields(gen, n_img, n):
    # smooth-ish log-conductivity images (separable SE correlation)
    x = (np.arange(n) + 0.5) / n
    C = np.exp(-0.5 * (x[:, None] - x[None, :]) ** 2 / 0.15 ** 2) + 1e-6 * np.eye(n)
    L = np.linalg.cholesky(C)
    G = gen.normal(size=(n_img, n, n))
    return 0.4 + 0.8 * np.einsum('ij,bjk,lk->bil', L, G, L)


# --------------------------------------------------------------------------
def make_codec(tag, imsize, dz, latent, blocks, growth, f_enc, f_dec, B):
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(1)
    enc = CNNEncoder(imsize, dz, blocks, growth, f_enc, drop_rate=0)
    dec = CNNDecoder(imsize, dz, (latent, latent), 1, f_dec, blocks, False, growth, drop_rate=0.,
                     upsample='nearest', force_single_output=False)
    randomize_bn(enc, gen)
    randomize_bn(dec, gen)
    rng = np.random.default_rng(2)
    X = torch.tensor(random_fields(rng, B, imsize), dtype=torch.float32, requires_grad=True)
    mu, ls = enc(X)
    wm = torch.randn(mu.shape, generator=gen)
    ws = torch.randn(ls.shape, generator=gen)
    (torch.sum(mu * wm) + torch.sum(ls * ws)).backward()
    Z = torch.randn(B, dz, generator=gen).requires_grad_(True)
    mx, lsx = dec(Z)
    vm = torch.randn(mx.shape, generator=gen)
    vs = torch.randn(lsx.shape, generator=gen)
    (torch.sum(mx * vm) + torch.sum(lsx * vs)).backward()
    out = dict(X=X.detach().numpy(), enc_mu=mu.detach().numpy(), enc_ls=ls.detach().numpy(),
               enc_wm=wm.numpy(), enc_ws=ws.numpy(), grad_X=X.grad.numpy(),
               Z=Z.detach().numpy(), dec_mu=mx.detach().numpy(), dec_ls=lsx.detach().numpy(),
               dec_vm=vm.numpy(), dec_vs=vs.numpy(), grad_Z=Z.grad.numpy(),
               cfg=np.array([imsize, dz, latent, growth, f_enc, f_dec] + list(blocks)))
    out.update(sd(enc, 'enc.'))
    out.update(grads(enc, 'enc.grad.'))
    out.update(sd(dec, 'dec.'))
    out.update(grads(dec, 'dec.grad.'))
    np.savez_compressed(os.path.join(HERE, 'codec_%s.npz' % tag), **out)
    print('codec', tag, 'enc params', sum(p.numel() for p in enc.parameters()),
          'dec params', sum(p.numel() for p in dec.parameters()))


def dropout_conv_names(module):
    """{id(nn.Dropout2d): name of the conv whose output it drops} for a reference codec
    (codec.py:177-178: a dense layer's 'dropout' follows its last conv; 'dropoutK' follows 'convK')."""
    out = {}
    for name, m in module.named_modules():
        if isinstance(m, torch.nn.Dropout2d):
            parent, leaf = name.rsplit('.', 1)
            if leaf == 'dropout':
                sub = dict(module.named_modules())[parent]
                conv = 'conv2' if hasattr(sub, 'conv2') else 'conv1'
            else:
                conv = 'conv' + leaf[len('dropout'):]
            out[id(m)] = parent + '.' + conv
    return out


def make_codec_drop(tag, imsize, dz, latent, blocks, growth, f0, B, p=0.2):
    """CNNEncoder / CNNDecoder with drop_rate p in train mode (codec.py:177-178,218-282): every
    nn.Dropout2d is patched to multiply by an injected per-(sample, channel) scale (bernoulli(1-p)/(1-p)),
    recorded as drop.enc.<conv> / drop.dec.<conv> -> codec_drop_<tag>.npz."""
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(31)
    enc = CNNEncoder(imsize, dz, blocks, growth, f0, drop_rate=p)
    dec = CNNDecoder(imsize, dz, (latent, latent), 1, f0, blocks, False, growth, drop_rate=p,
                     upsample='nearest', force_single_output=False)
    randomize_bn(enc, gen)
    randomize_bn(dec, gen)
    masks = {}
    names = {}
    for key, mod in (('enc', enc), ('dec', dec)):
        for i, nm in dropout_conv_names(mod).items():
            names[i] = (key, nm)

    def fake_forward(self, x):
        key, nm = names[id(self)]
        if (key, nm) not in masks:
            masks[(key, nm)] = torch.bernoulli(torch.full(x.shape[:2], 1 - p), generator=gen) / (1 - p)
        return x * masks[(key, nm)][:, :, None, None]

    rng = np.random.default_rng(32)
    X = torch.tensor(random_fields(rng, B, imsize), dtype=torch.float32, requires_grad=True)
    with mock.patch.object(torch.nn.Dropout2d, 'forward', fake_forward):
        mu, ls = enc(X)
        wm = torch.randn(mu.shape, generator=gen)
        ws = torch.randn(ls.shape, generator=gen)
        (torch.sum(mu * wm) + torch.sum(ls * ws)).backward()
        Z = torch.randn(B, dz, generator=gen).requires_grad_(True)
        mx, lsx = dec(Z)
        vm = torch.randn(mx.shape, generator=gen)
        vs = torch.randn(lsx.shape, generator=gen)
        (torch.sum(mx * vm) + torch.sum(lsx * vs)).backward()
    assert len(masks) == len(names), (len(masks), len(names))
    out = dict(X=X.detach().numpy(), enc_mu=mu.detach().numpy(), enc_ls=ls.detach().numpy(),
               enc_wm=wm.numpy(), enc_ws=ws.numpy(), grad_X=X.grad.numpy(),
               Z=Z.detach().numpy(), dec_mu=mx.detach().numpy(), dec_ls=lsx.detach().numpy(),
               dec_vm=vm.numpy(), dec_vs=vs.numpy(), grad_Z=Z.grad.numpy(), p=np.float64(p),
               cfg=np.array([imsize, dz, latent, growth, f0, f0] + list(blocks)))
    for (key, nm), m in masks.items():
        out['drop.%s.%s' % (key, nm)] = m.numpy()
    out.update(sd(enc, 'enc.'))
    out.update(grads(enc, 'enc.grad.'))
    out.update(sd(dec, 'dec.'))
    out.update(grads(dec, 'dec.grad.'))
    np.savez_compressed(os.path.join(HERE, 'codec_drop_%s.npz' % tag), **out)
    print('codec dropout', tag, len(masks), 'dropout layers')


# --------------------------------------------------------------------------
def c32_physics():
    nc, r = 4, 8
    mc = fem.unit_square_mesh(nc)
    mf = fem.unit_square_mesh(nc * r)
    M = fem.rom_stiffness_tensor(mc)
    W = fem.prolongation_free(mc, mf)
    cdofs, fdofs = fem.dirichlet_split(mc)
    return nc, r, mc, mf, M, W, cdofs, fdofs


class _Phys(object):
    def __init__(self, c, f):
        self.constrained_dofs = c
        self.free_dofs = f


def c64_physics():
    """highres (factories/model.py:172-213): ROM 8x8, 3 refinements -> 64x64."""
    nc, r = 8, 8
    mc = fem.unit_square_mesh(nc)
    mf = fem.unit_square_mesh(nc * r)
    M = fem.rom_stiffness_tensor(mc)
    W = fem.prolongation_free(mc, mf)
    cdofs, fdofs = fem.dirichlet_split(mc)
    return nc, r, mc, mf, M, W, cdofs, fdofs


def make_rom(tag='c32'):
    """ROM solve + ReducedOrderModelOperator forward / adjoint (ROM.py:59-100, components.py:296-298).
    c64: nc = 8 (81 coarse nodes), N = 32 = the benchmarked labeled batch."""
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics() if tag == 'c32' else c64_physics()
    rng = np.random.default_rng(3 if tag == 'c32' else 33)
    N = 6 if tag == 'c32' else 32
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32),
                                         dtype=torch.float32, device='cpu')
    with torch.no_grad():
        g.logsigmas_y.copy_(torch.tensor(rng.normal(0.5, 0.3, W.shape[0]), dtype=torch.float32))
    U = rng.uniform(-0.5, 0.5, (N, 4))
    F = torch.tensor(np.stack([fem.f_rom_bc(mc, u) for u in U]), dtype=torch.float32)
    effprop = torch.tensor(rng.normal(0, 0.7, (N, M.shape[2])), dtype=torch.float32, requires_grad=True)
    mu, ls = g(effprop, F)
    Y = torch.tensor(rng.normal(0, 0.3, mu.shape), dtype=torch.float32)
    L = R_utils.DiagonalGaussianLogLikelihood(Y, mu, 2 * ls)
    (-L).backward()
    extra = {}
    if tag != 'c32':
        extra = dict(nc=np.int64(nc), r=np.int64(r))       # M / W are rebuilt from the oracle at test time
    else:
        extra = dict(M=M.astype(np.float32), W=W.astype(np.float32))
    np.savez_compressed(os.path.join(HERE, 'rom_%s.npz' % tag), bc_dofs=cdofs, U=U, F=F.numpy(),
                        effprop=effprop.detach().numpy(),
                        logsigmas_y=g.logsigmas_y.detach().numpy(), mu_y=mu.detach().numpy(),
                        Y=Y.numpy(), logL=L.detach().numpy(), grad_effprop=effprop.grad.numpy(),
                        grad_logsigmas_y=g.logsigmas_y.grad.numpy(), **extra)
    print('rom ok', tag, float(L))


# --------------------------------------------------------------------------
class _DS(object):
    """Minimal stand-in for utils.data.DataSet (utils/data.py:419-445)."""

    def __init__(self, **t):
        self.t = t
        self.N = next(iter(t.values())).shape[0]

    def get(self, key, random_subset=None):
        if random_subset is None:
            return self.t[key]
        perm = torch.randperm(self.N, dtype=torch.long)
        return self.t[key][perm[0:random_subset], ]


def make_elbo():
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics()
    n = nc * r
    rng = np.random.default_rng(4)
    Nu, bs, Ns = 16, 8, 4
    dz = 16
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(5)
    enc = CNNEncoder(n, dz, [1, 1], 4, 4, drop_rate=0)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0., upsample='nearest',
                     force_single_output=False, homoscedastic=False)
    randomize_bn(enc, gen)
    randomize_bn(dec, gen)
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32),
                                         dtype=torch.float32, device='cpu')
    gp = R_comp.EffectivePropertyMap(dz, M.shape[2], num_hidden_layers=0, independent_X=True,
                                     dtype=torch.float32, device='cpu')
    model = R_gen.GenerativeModel(f=dec, g=g, gp=gp, dtype=torch.float32, device='cpu')
    model.encoder = enc

    Xu = torch.tensor(random_fields(rng, Nu, n), dtype=torch.float32)
    Xs_img = random_fields(rng, Ns, n)
    Xs = torch.tensor(Xs_img, dtype=torch.float32)
    U = rng.uniform(-0.5, 0.5, (Ns, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(Xs_img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    ds_sup = _DS(X=Xs, Y=torch.tensor(Y, dtype=torch.float32), F_ROM_BC=torch.tensor(F, dtype=torch.float32))
    ds_uns = _DS(X=Xu)
    model.register_datasets({'supervised': ds_sup, 'unsupervised': ds_uns}, None,
                            create_unsupervised_variational_approximation=False)
    with torch.no_grad():
        for q in (model.q_z['supervised'], model.q_X['supervised']):
            q._mean.copy_(torch.tensor(rng.normal(0, 0.5, q._mean.shape)))
            q._logsigma.copy_(torch.tensor(rng.normal(-1.0, 0.3, q._logsigma.shape)))
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))

    perm = torch.tensor(rng.permutation(Nu), dtype=torch.long)
    eps = [torch.tensor(rng.normal(size=s), dtype=torch.float32)
           for s in [(bs, dz), (Ns, dz), (Ns, M.shape[2])]]
    queue = list(eps)
    real_randn_like = torch.randn_like

    def fake_randn_like(t, *a, **k):
        e = queue.pop(0)
        assert e.shape == t.shape, (e.shape, t.shape)
        return e.to(dtype=t.dtype)

    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    with mock.patch('torch.randperm', lambda N, **k: perm.clone()), \
            mock.patch('torch.randn_like', fake_randn_like):
        elbo = model.elbo(step=0, armortized_bs=bs)
    assert not queue
    (-elbo).backward()
    out = {'state.' + k: v for k, v in state0.items()}
    out.update({'grad.' + k: p.grad.detach().numpy() for k, p in model.named_parameters() if p.grad is not None})
    out.update(Xu=Xu.numpy(), Xs=Xs.numpy(), Y=Y.astype(np.float32), F=F.astype(np.float32), U=U,
               perm=perm.numpy(), eps_enc=eps[0].numpy(), eps_qz=eps[1].numpy(), eps_qX=eps[2].numpy(),
               elbo=np.float64(elbo.item()), M=M.astype(np.float32), W=W.astype(np.float32), bc_dofs=cdofs,
               cfg=np.array([n, nc, dz, Nu, bs, Ns]))
    np.savez_compressed(os.path.join(HERE, 'elbo_c32.npz'), **out)
    print('elbo ok', elbo.item(), 'n params', sum(p.numel() for p in model.parameters()))
    del real_randn_like


def _elbo_model(phys, n, dz, blocks, growth, f0, gen, independent_X=True):
    nc, r, mc, mf, M, W, cdofs, fdofs = phys
    torch.manual_seed(0)
    enc = CNNEncoder(n, dz, blocks, growth, f0, drop_rate=0)
    dec = CNNDecoder(n, dz, (8, 8), 1, f0, blocks, False, growth, drop_rate=0., upsample='nearest',
                     force_single_output=False, homoscedastic=False)
    randomize_bn(enc, gen)
    randomize_bn(dec, gen)
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32), dtype=torch.float32, device='cpu')
    gp = R_comp.EffectivePropertyMap(dz, M.shape[2], num_hidden_layers=0, independent_X=independent_X,
                                     dtype=torch.float32, device='cpu')
    model = R_gen.GenerativeModel(f=dec, g=g, gp=gp, dtype=torch.float32, device='cpu')
    model.encoder = enc
    return model, g


def _elbo_run(model, perm, eps, **kw):
    """One reference model.elbo(...) + backward with injected permutation / noise; returns
    (elbo, grads)."""
    queue = list(eps)

    def fake_randn_like(t, *a, **k):
        e = queue.pop(0)
        assert e.shape == t.shape, (e.shape, t.shape)
        return e.to(dtype=t.dtype)

    model.zero_grad()
    with mock.patch('torch.randperm', lambda N, **k: perm.clone()), mock.patch('torch.randn_like', fake_randn_like):
        elbo = model.elbo(step=0, **kw)
    assert not queue
    (-elbo).backward()
    return elbo, {k: p.grad.detach().numpy().copy() for k, p in model.named_parameters() if p.grad is not None}


def make_elbo_c64():
    """GenerativeModel.elbo (armortized + supervised freeX) + backward at the BENCHMARKED shape:
    highres codec (d_z 64, blocks [1, 2, 1], growth 4, init features 6), ROM 8x8 on 64x64,
    B_u = 256 armortized samples out of a pool of 256 (random order), N_s = 32 labeled
    -> elbo_c64.npz.  ~5 MB: inputs stored in fp32, M / W rebuilt from the oracle by the tests."""
    phys = c64_physics()
    nc, r, mc, mf, M, W, cdofs, fdofs = phys
    n = nc * r
    rng = np.random.default_rng(64)
    Nu, bs, Ns, dz = 256, 256, 32, 64
    gen = torch.Generator().manual_seed(65)
    model, g = _elbo_model(phys, n, dz, [1, 2, 1], 4, 6, gen)
    Xu = torch.tensor(random_fields(rng, Nu, n), dtype=torch.float32)
    Xs_img = random_fields(rng, Ns, n).astype(np.float32)
    U = rng.uniform(-0.5, 0.5, (Ns, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x.astype(np.float64))), u) for x, u in zip(Xs_img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    model.register_datasets({'supervised': _DS(X=torch.tensor(Xs_img), Y=torch.tensor(Y, dtype=torch.float32),
                                               F_ROM_BC=torch.tensor(F, dtype=torch.float32)),
                             'unsupervised': _DS(X=Xu)}, None, create_unsupervised_variational_approximation=False)
    with torch.no_grad():
        for q in (model.q_z['supervised'], model.q_X['supervised']):
            q._mean.copy_(torch.tensor(rng.normal(0, 0.5, q._mean.shape)))
            q._logsigma.copy_(torch.tensor(rng.normal(-1.0, 0.3, q._logsigma.shape)))
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))
    perm = torch.tensor(rng.permutation(Nu), dtype=torch.long)
    eps = [torch.tensor(rng.normal(size=s), dtype=torch.float32) for s in [(bs, dz), (Ns, dz), (Ns, M.shape[2])]]
    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    elbo, gr = _elbo_run(model, perm, eps, armortized_bs=bs)
    out = {'state.' + k: v for k, v in state0.items()}
    out.update({'grad.' + k: v for k, v in gr.items()})
    out.update(Xu=Xu.numpy(), Xs=Xs_img, Y=Y.astype(np.float32), F=F.astype(np.float32), U=U,
               perm=perm.numpy(), eps_enc=eps[0].numpy(), eps_qz=eps[1].numpy(), eps_qX=eps[2].numpy(),
               elbo=np.float64(elbo.item()), bc_dofs=cdofs, cfg=np.array([n, nc, dz, Nu, bs, Ns]))
    np.savez_compressed(os.path.join(HERE, 'elbo_c64.npz'), **out)
    print('elbo c64 ok', elbo.item(), 'n params', sum(p.numel() for p in model.parameters()))


def make_bn_running_c32():
    """BatchNorm2d running statistics (train mode, momentum 0.1): the reference model after two
    model.elbo calls (encoder once, decoder twice -- unsupervised then supervised -- per call) ->
    bn_running_c32.npz (state before, running buffers after, injected noise)."""
    phys = c32_physics()
    nc, r, mc, mf, M, W, cdofs, fdofs = phys
    n = nc * r
    rng = np.random.default_rng(54)
    Nu, bs, Ns, dz = 16, 8, 4, 16
    gen = torch.Generator().manual_seed(55)
    model, g = _elbo_model(phys, n, dz, [1, 1], 4, 4, gen)
    Xu = torch.tensor(random_fields(rng, Nu, n), dtype=torch.float32)
    Xs_img = random_fields(rng, Ns, n)
    U = rng.uniform(-0.5, 0.5, (Ns, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(Xs_img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    model.register_datasets({'supervised': _DS(X=torch.tensor(Xs_img, dtype=torch.float32),
                                               Y=torch.tensor(Y, dtype=torch.float32),
                                               F_ROM_BC=torch.tensor(F, dtype=torch.float32)),
                             'unsupervised': _DS(X=Xu)}, None, create_unsupervised_variational_approximation=False)
    with torch.no_grad():       # non-trivial running buffers to start from
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=gen))
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=gen) + 0.5)
    perm = torch.tensor(rng.permutation(Nu), dtype=torch.long)
    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    out = {'state.' + k: v for k, v in state0.items()}
    for call in range(2):
        eps = [torch.tensor(rng.normal(size=s_), dtype=torch.float32) for s_ in [(bs, dz), (Ns, dz), (Ns, M.shape[2])]]
        _elbo_run(model, perm, eps, armortized_bs=bs)
        for i, e in enumerate(eps):
            out['eps%d_%d' % (call, i)] = e.numpy()
    out.update({'after.' + k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()
                if k.endswith(('running_mean', 'running_var', 'num_batches_tracked'))})
    out.update(Xu=Xu.numpy(), Xs=Xs_img.astype(np.float32), Y=Y.astype(np.float32), F=F.astype(np.float32),
               perm=perm.numpy(), M=M.astype(np.float32), W=W.astype(np.float32), bc_dofs=cdofs,
               cfg=np.array([n, nc, dz, Nu, bs, Ns]))
    np.savez_compressed(os.path.join(HERE, 'bn_running_c32.npz'), **out)
    print('bn running ok')


def make_elbo_options_c32():
    """model.elbo(normalize=True) and model.elbo(l2_penalty=...) (generative.py:247-287: every term
    divided by its batch size; minus l2_penalty * sum of the parameter norms of f and the encoder),
    and model.elbo() with reconstruct_log_eff_property=False ('expf') at the C32 shape of elbo_c32 -> elbo_opts_c32.npz."""
    phys = c32_physics()
    nc, r, mc, mf, M, W, cdofs, fdofs = phys
    n = nc * r
    rng = np.random.default_rng(44)
    Nu, bs, Ns, dz = 16, 8, 4, 16
    gen = torch.Generator().manual_seed(45)
    model, g = _elbo_model(phys, n, dz, [1, 1], 4, 4, gen)
    Xu = torch.tensor(random_fields(rng, Nu, n), dtype=torch.float32)
    Xs_img = random_fields(rng, Ns, n)
    U = rng.uniform(-0.5, 0.5, (Ns, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(Xs_img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    model.register_datasets({'supervised': _DS(X=torch.tensor(Xs_img, dtype=torch.float32),
                                               Y=torch.tensor(Y, dtype=torch.float32),
                                               F_ROM_BC=torch.tensor(F, dtype=torch.float32)),
                             'unsupervised': _DS(X=Xu)}, None, create_unsupervised_variational_approximation=False)
    with torch.no_grad():
        for q in (model.q_z['supervised'], model.q_X['supervised']):
            q._mean.copy_(torch.tensor(rng.normal(0, 0.5, q._mean.shape)))
            q._logsigma.copy_(torch.tensor(rng.normal(-1.0, 0.3, q._logsigma.shape)))
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))
    perm = torch.tensor(rng.permutation(Nu), dtype=torch.long)
    shapes = [(bs, dz), (Ns, dz), (Ns, M.shape[2])]
    eps = [torch.tensor(rng.normal(size=s), dtype=torch.float32) for s in shapes]
    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    out = {'state.' + k: v for k, v in state0.items()}
    class _Writer(object):           # the reference's l2 branch logs unconditionally (generative.py:278)
        def add_scalar(self, k, v, global_step=None):
            pass

    for tag, kw in (('norm', dict(normalize=True)), ('l2', dict(l2_penalty=0.05)), ('expf', dict())):
        model.writer = _Writer() if tag == 'l2' else None
        if tag == 'expf':            # Gaussian on the exponentiated field (generative.py:236-239)
            model.set('reconstruct_log_eff_property', False)
        elbo, gr = _elbo_run(model, perm, eps, armortized_bs=bs, **kw)
        out.update({'%s.grad.%s' % (tag, k): v for k, v in gr.items()})
        out['%s.elbo' % tag] = np.float64(elbo.item())
        print('elbo option', tag, elbo.item())
    out.update(Xu=Xu.numpy(), Xs=Xs_img.astype(np.float32), Y=Y.astype(np.float32), F=F.astype(np.float32), U=U,
               perm=perm.numpy(), eps_enc=eps[0].numpy(), eps_qz=eps[1].numpy(), eps_qX=eps[2].numpy(),
               M=M.astype(np.float32), W=W.astype(np.float32), bc_dofs=cdofs, cfg=np.array([n, nc, dz, Nu, bs, Ns]),
               l2_penalty=np.float64(0.05))
    np.savez_compressed(os.path.join(HERE, 'elbo_opts_c32.npz'), **out)


# --------------------------------------------------------------------------
def make_elbo_nonarmortized():
    """GenerativeModel.elbo without an encoder: elbo_unsupervised (generative.py:515-544, per-sample
    q_z['unsupervised'] over the whole set, KL of q_z['supervised'] sic :525) + the supervised freeX
    term -> elbo_nonarm_c32.npz."""
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics()
    n = nc * r
    rng = np.random.default_rng(14)
    Nu, Ns = 6, 4
    dz = 16
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(15)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0., upsample='nearest',
                     force_single_output=False, homoscedastic=False)
    randomize_bn(dec, gen)
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32),
                                         dtype=torch.float32, device='cpu')
    gp = R_comp.EffectivePropertyMap(dz, M.shape[2], num_hidden_layers=0, independent_X=True,
                                     dtype=torch.float32, device='cpu')
    model = R_gen.GenerativeModel(f=dec, g=g, gp=gp, dtype=torch.float32, device='cpu')
    Xu = torch.tensor(random_fields(rng, Nu, n), dtype=torch.float32)
    Xs_img = random_fields(rng, Ns, n)
    Xs = torch.tensor(Xs_img, dtype=torch.float32)
    U = rng.uniform(-0.5, 0.5, (Ns, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(Xs_img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    ds_sup = _DS(X=Xs, Y=torch.tensor(Y, dtype=torch.float32), F_ROM_BC=torch.tensor(F, dtype=torch.float32))
    model.register_datasets({'supervised': ds_sup, 'unsupervised': _DS(X=Xu)}, None,
                            create_unsupervised_variational_approximation=True)
    with torch.no_grad():
        for q in (model.q_z['unsupervised'], model.q_z['supervised'], model.q_X['supervised']):
            q._mean.copy_(torch.tensor(rng.normal(0, 0.5, q._mean.shape)))
            q._logsigma.copy_(torch.tensor(rng.normal(-1.0, 0.3, q._logsigma.shape)))
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))
    eps = [torch.tensor(rng.normal(size=s_), dtype=torch.float32) for s_ in [(Nu, dz), (Ns, dz), (Ns, M.shape[2])]]
    queue = list(eps)

    def fake_randn_like(t, *a, **k):
        e = queue.pop(0)
        assert e.shape == t.shape, (e.shape, t.shape)
        return e.to(dtype=t.dtype)

    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    with mock.patch('torch.randn_like', fake_randn_like):
        elbo = model.elbo(step=0)
    assert not queue
    (-elbo).backward()
    out = {'state.' + k: v for k, v in state0.items()}
    out.update({'grad.' + k: p.grad.detach().numpy() for k, p in model.named_parameters() if p.grad is not None})
    out.update(Xu=Xu.numpy(), Xs=Xs.numpy(), Y=Y.astype(np.float32), F=F.astype(np.float32), U=U,
               eps_u=eps[0].numpy(), eps_qz=eps[1].numpy(), eps_qX=eps[2].numpy(), elbo=np.float64(elbo.item()),
               M=M.astype(np.float32), W=W.astype(np.float32), bc_dofs=cdofs, cfg=np.array([n, nc, dz, Nu, Ns]))
    np.savez_compressed(os.path.join(HERE, 'elbo_nonarm_c32.npz'), **out)
    print('elbo non-armortized ok', elbo.item())


def make_vo():
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics()
    n = nc * r
    rng = np.random.default_rng(6)
    Nvo = 3
    imgs = random_fields(rng, Nvo, n)
    U = rng.uniform(-0.5, 0.5, (Nvo, 4))
    Gam, alp, G, P = [], [], [], []
    for img, u in zip(imgs, U):
        Gm, a = fem.cgr_query(mf, W, np.exp(fem.image_to_cells(img)), u)
        Gam.append(Gm)
        alp.append(a)
        y = fem.solve_fom(mf, np.exp(fem.image_to_cells(img)), u)
        G.append(y + rng.normal(0, 0.05, y.shape))
        P.append(1.0 / rng.uniform(0.01, 0.05, y.shape) ** 2)

    class _Q(object):
        pass

    means, vars_ = [], []
    vo_var = torch.tensor(rng.uniform(1e-6, 1e-4, Gam[0].shape[0]), dtype=torch.double)
    for Gm, a, g_, p_ in zip(Gam, alp, G, P):
        q = mock.MagicMock()
        q.Gamma = torch.tensor(Gm)
        q.GammaTransposed = torch.tensor(Gm).t()
        q.alpha = torch.tensor(a)
        vo = R_VO.VirtualObservable.__new__(R_VO.VirtualObservable)
        vo._querry = q
        vo._device = torch.device('cpu')
        vo._vo_variances = vo_var
        with mock.patch('torch.cholesky', torch.linalg.cholesky):
            vo.update(torch.tensor(g_), torch.tensor(p_), 0, ForceUpdate=True)
        means.append(vo.mean.numpy())
        vars_.append(vo.vars.numpy())
    beta = 0
    for Gm, a, mu, v in zip(Gam, alp, means, vars_):
        beta = beta + (Gm @ mu - a) ** 2 + (Gm ** 2) @ v
    np.savez_compressed(os.path.join(HERE, 'vo_c32.npz'), imgs=imgs, U=U, Gamma=np.stack(Gam),
                        alpha=np.stack(alp), g=np.stack(G), prec=np.stack(P), vo_var=vo_var.numpy(),
                        mean=np.stack(means), vars=np.stack(vars_), prec_beta=0.5 * beta + 1e-6)
    print('vo ok')


# --------------------------------------------------------------------------
class _FakePhysics(object):
    """What QuerryPoint / CoarseGrainedResidualSampler read from a FEniCS physics object;
    the operators come from the oracle's generic P1 assembly."""

    def __init__(self, mesh):
        self.mesh = mesh
        c, f = fem.dirichlet_split(mesh)
        self.dim_out = f.size
        self.Vc = mock.MagicMock()
        self.Vc.dim.return_value = mesh.num_cells

    def assemble_system(self, x, bc=None, only_free_dofs=True):
        return fem.assemble_system(self.mesh, x, bc.u)


class _FakeBC(object):
    def __init__(self, u):
        self.u = u


class _FakeFlux(object):
    """FluxConstraintReducedOrderModel stand-in: oracle flux rows reduced to the free dofs, alpha = 0."""

    initialized = True

    def __init__(self, mc, mf):
        self.mc, self.mf = mc, mf
        self.free = fem.dirichlet_split(mf)[1]

    def assemble_reduced(self, x, bc):
        G, a = fem.flux_rows(self.mc, self.mf, x)
        return G[:, self.free], a


def make_vo_elbo(lockx=False):
    """lockx: the reference's independent_X=False variants (_elbo_supervised_lockX
    generative.py:429-459, _elbo_virtual_observables_lockX :300-339, the lockX branch of
    update_virtual_observables :202-204) -> vo_elbo_lockx_c32.npz."""
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics()
    n = nc * r
    rng = np.random.default_rng(8)
    Nu, bs, Ns, Nvo, Nmc = 8, 4, 3, 3, 6
    dz = 16
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(9)
    enc = CNNEncoder(n, dz, [1, 1], 4, 4, drop_rate=0)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0., upsample='nearest',
                     force_single_output=False, homoscedastic=False)
    randomize_bn(enc, gen)
    randomize_bn(dec, gen)
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32), dtype=torch.float32,
                                         device='cpu')
    gp = R_comp.EffectivePropertyMap(dz, M.shape[2], num_hidden_layers=0, independent_X=not lockx,
                                     dtype=torch.float32, device='cpu')
    model = R_gen.GenerativeModel(f=dec, g=g, gp=gp, dtype=torch.float32, device='cpu')
    model.encoder = enc

    def labeled(k):
        img = random_fields(rng, k, n)
        U = rng.uniform(-0.5, 0.5, (k, 4))
        Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(img, U)])
        F = np.stack([fem.f_rom_bc(mc, u) for u in U])
        return img, U, Y, F

    Xu = random_fields(rng, Nu, n)
    Xs, Us, Ys, Fs = labeled(Ns)
    Xv, Uv, Yv, Fv = labeled(Nvo)
    t32 = lambda a: torch.tensor(a, dtype=torch.float32)
    ds_sup = _DS(X=t32(Xs), Y=t32(Ys), F_ROM_BC=t32(Fs))
    ds_uns = _DS(X=t32(Xu))
    ds_vo = _DS(X=t32(Xv), Y=t32(Yv), F_ROM_BC=t32(Fv))

    # the reference's own query / ensemble classes over oracle operators
    phys = _FakePhysics(mf)
    QPs = [R_VO.QuerryPoint(phys, fem.image_to_cells(x), _FakeBC(u)) for x, u in zip(Xv, Uv)]
    QPE = R_VO.QuerryPointEnsemble(QPs)
    flux = _FakeFlux(mc, mf)
    querries = []
    for qp in QPs:
        sampler = R_VO.ConcatenatedSamplers([R_VO.CoarseGrainedResidualSampler(qp=qp, W=W),
                                             R_VO.FluxConstrainSampler(qp, flux)])
        querries.append(R_VO.LinearQuerry(qp, sampler, dtype=torch.float32, device='cpu'))
    QE = R_VO.QuerryEnsemble(querries, dtype=torch.float32, device='cpu')
    VO = R_VO.VirtualObservablesEnsemble(QPE, QE, dtype=torch.float32, device=torch.device('cpu'))

    model.register_datasets({'supervised': ds_sup, 'unsupervised': ds_uns, 'vo': ds_vo}, VO,
                            create_unsupervised_variational_approximation=False)
    with torch.no_grad():
        for key in ('supervised', 'vo'):
            for q in (model.q_z[key],) + (() if lockx else (model.q_X[key],)):
                q._mean.copy_(torch.tensor(rng.normal(0, 0.5, q._mean.shape)))
                q._logsigma.copy_(torch.tensor(rng.normal(-1.0, 0.3, q._logsigma.shape)))
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))
    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    dx = M.shape[2]
    dy = W.shape[0]

    # two VO updates (the second one exercises the learnable flux-row precisions)
    upd = []
    for it in range(2):
        ex = rng.normal(size=(Nvo, Nmc, dz if lockx else dx))     # q_z draws (lockX) / q_X draws
        ey = rng.normal(size=(Nvo, Nmc, dy))
        q_randn = [torch.tensor(e, dtype=torch.float32) for e in ex]
        q_like = [torch.tensor(e, dtype=torch.float32) for e in ey]

        def fake_randn(*size, **k):
            e = q_randn.pop(0)
            assert tuple(e.shape) == tuple(size), (e.shape, size)
            return e

        def fake_randn_like(t, *a, **k):
            e = q_like.pop(0)
            assert e.shape == t.shape
            return e

        with mock.patch('torch.randn', fake_randn), mock.patch('torch.randn_like', fake_randn_like), \
                mock.patch('torch.cholesky', torch.linalg.cholesky):
            Ym, Ysd = model.update_virtual_observables(Nmc, return_mean_stddev=True, step=it)
        assert not q_randn and not q_like
        upd.append(dict(eps_X=ex.reshape(Nvo * Nmc, ex.shape[2]), eps_y=ey.reshape(Nvo * Nmc, dy), Y_mean=Ym.numpy(),
                        Y_std=Ysd.numpy(), mean=VO.mean.numpy(), vars=VO.vars.numpy(),
                        vo_var=VO._mean_vo_variances.numpy(), prec_beta=VO._prec_beta.numpy()))

    perm = torch.tensor(rng.permutation(Nu), dtype=torch.long)
    shapes = [(bs, dz), (Ns, dz), (Ns, dx), (Nvo, dz), (Nvo, dx), (Nvo, dy)]
    if lockx:
        shapes = [(bs, dz), (Ns, dz), (Nvo, dz), (Nvo, dy)]
    eps = [torch.tensor(rng.normal(size=sh), dtype=torch.float32) for sh in shapes]
    queue = list(eps)

    def fake_randn_like(t, *a, **k):
        e = queue.pop(0)
        assert e.shape == t.shape, (e.shape, t.shape)
        return e.to(dtype=t.dtype)

    class _Writer(object):
        def __init__(self):
            self.d = {}

        def add_scalar(self, k, v, global_step=None):
            self.d[k] = float(v)

    model.writer = _Writer()
    with mock.patch('torch.randperm', lambda N, **k: perm.clone()), mock.patch('torch.randn_like', fake_randn_like):
        elbo = model.elbo(step=0, armortized_bs=bs)
    assert not queue
    terms_main = dict(model.writer.d)
    model.writer = _Writer()
    (-elbo).backward()
    grads_main = {'grad.' + k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()
                  if p.grad is not None}
    # hold-off variant (generative.py:361-364): only q_z['vo'] is sampled for the VO term
    model.zero_grad()
    eps_h = [torch.tensor(rng.normal(size=sh), dtype=torch.float32) for sh in shapes[:3 if lockx else 4]]
    queue = list(eps_h)
    with mock.patch('torch.randperm', lambda N, **k: perm.clone()), mock.patch('torch.randn_like', fake_randn_like):
        elbo_h = model.elbo(step=0, armortized_bs=bs, vo_holdoff=True)
    assert not queue
    terms_h = dict(model.writer.d)
    model.writer = None
    out = {'state.' + k: v for k, v in state0.items()}
    out.update(grads_main)
    out.update(Xu=Xu.astype(np.float32), Xs=Xs.astype(np.float32), Ys=Ys.astype(np.float32),
               Fs=Fs.astype(np.float32), Us=Us, Xv=Xv.astype(np.float32), Yv=Yv.astype(np.float32),
               Fv=Fv.astype(np.float32), Uv=Uv, Xv_dg=np.stack([qp.x for qp in QPs]), perm=perm.numpy(),
               M=M.astype(np.float32), W=W.astype(np.float32), bc_dofs=cdofs,
               cfg=np.array([n, nc, dz, Nu, bs, Ns, Nvo, Nmc]),
               Gamma=np.stack([q.Gamma.numpy() for q in querries]), alpha=np.stack([q.alpha.numpy() for q in querries]),
               elbo=np.float64(elbo.item()), elbo_holdoff=np.float64(elbo_h.item()))
    for k, v in terms_main.items():
        out['term.' + k] = np.float64(v)
    for k, v in terms_h.items():
        out['termh.' + k] = np.float64(v)
    for i, e in enumerate(eps):
        out['eps%d' % i] = e.numpy()
    for i, e in enumerate(eps_h):
        out['epsh%d' % i] = e.numpy()
    for it, u in enumerate(upd):
        for k, v in u.items():
            out['upd%d.%s' % (it, k)] = v
    (-elbo_h).backward()
    out.update({'gradh.' + k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()
                if p.grad is not None})
    np.savez_compressed(os.path.join(HERE, 'vo_elbo_lockx_c32.npz' if lockx else 'vo_elbo_c32.npz'), **out)
    print('vo elbo ok', 'lockX' if lockx else 'freeX', elbo.item(), elbo_h.item())
    return elbo


def make_pe_analysis():
    nc, r, mc, mf, M, W, cdofs, fdofs = c32_physics()
    n = nc * r
    rng = np.random.default_rng(10)
    Nval, dz, Nmc, iters = 5, 16, 6, 3
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(11)
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0., upsample='nearest',
                     force_single_output=False, homoscedastic=False)
    randomize_bn(dec, gen)
    rom = R_ROM.ROM(_Phys(cdofs, fdofs), torch.tensor(M, dtype=torch.float32), torch.float32, 'cpu')
    g = R_comp.ReducedOrderModelOperator(rom, torch.tensor(W, dtype=torch.float32), dtype=torch.float32,
                                         device='cpu')
    gp = R_comp.EffectivePropertyMap(dz, M.shape[2], num_hidden_layers=0, independent_X=True,
                                     dtype=torch.float32, device='cpu')
    model = R_gen.GenerativeModel(f=dec, g=g, gp=gp, dtype=torch.float32, device='cpu')
    with torch.no_grad():
        g.logsigmas_y.copy_(torch.tensor(rng.normal(-2.0, 0.2, g.logsigmas_y.shape)))
        gp.logsigmas_X.copy_(torch.tensor(rng.normal(-1.0, 0.2, gp.logsigmas_X.shape)))
    img = random_fields(rng, Nval, n)
    U = rng.uniform(-0.5, 0.5, (Nval, 4))
    Y = np.stack([fem.solve_fom(mf, np.exp(fem.image_to_cells(x)), u) for x, u in zip(img, U)])
    F = np.stack([fem.f_rom_bc(mc, u) for u in U])
    t32 = lambda a: torch.tensor(a, dtype=torch.float32)
    ds = _DS(X=t32(img), Y=t32(Y), F_ROM_BC=t32(F))
    ds.label = 'validation'

    class _Writer(object):
        def __init__(self):
            self.d = {}

        def add_scalar(self, k, v, global_step=None):
            self.d[k] = float(v)

    state0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    pe = R_comp.PredictionEnsemble(model, ds, R_opt.LearningScheduleWrapper.Dummy(), lr=1e-2, writer=_Writer())
    eps = [torch.tensor(rng.normal(size=(Nval, dz)), dtype=torch.float32) for _ in range(iters)]
    queue = list(eps)

    def fake_randn_like(t, *a, **k):
        e = queue.pop(0)
        assert e.shape == t.shape, (e.shape, t.shape)
        return e

    with mock.patch('torch.randn_like', fake_randn_like):
        pe.update(numIter=iters, record=True, step=0)
    assert not queue
    pe_terms = dict(pe.writer.d)

    # Analysis.eval_all_y on a spread-out q (the PE's q after 3 steps is still near the prior)
    q = R_comp.VariationalApproximation(dz, Nval, t32(img))
    with torch.no_grad():
        q._mean.copy_(torch.tensor(rng.normal(0, 0.7, q._mean.shape)))
        q._logsigma.copy_(torch.tensor(rng.normal(-1.5, 0.3, q._logsigma.shape)))
    ez = rng.normal(size=(Nval, Nmc, dz))
    ex = rng.normal(size=(Nval, Nmc, M.shape[2]))
    ey = rng.normal(size=(Nval, Nmc, W.shape[0]))
    qr = [torch.tensor(e, dtype=torch.float32) for e in ez]
    ql = []
    for i in range(Nval):
        ql += [torch.tensor(ex[i], dtype=torch.float32), torch.tensor(ey[i], dtype=torch.float32)]

    def fake_randn(*size, **k):
        e = qr.pop(0)
        assert tuple(e.shape) == tuple(size)
        return e

    def fake_randn_like2(t, *a, **k):
        e = ql.pop(0)
        assert e.shape == t.shape
        return e

    an = R_comp.Analysis(q, model, ds)
    with mock.patch('torch.randn', fake_randn), mock.patch('torch.randn_like', fake_randn_like2):
        logscore, r2, relerr = an.eval_all_y(Nmc)
    assert not qr and not ql
    out = {'state.' + k: v for k, v in state0.items()}
    out.update(X=img.astype(np.float32), Y=Y.astype(np.float32), F=F.astype(np.float32), W=W.astype(np.float32),
               cfg=np.array([n, nc, dz, Nval, Nmc, iters]), pe_eps=np.stack([e.numpy() for e in eps]),
               pe_mean=pe.q_z._mean.detach().numpy(), pe_logsigma=pe.q_z._logsigma.detach().numpy(),
               pe_elbo=np.float64(pe_terms['PredictionEnsemble/elbo']),
               pe_logL=np.float64(pe_terms['PredictionEnsemble/logL']),
               pe_KLD=np.float64(pe_terms['PredictionEnsemble/KLD']),
               q_mean=q._mean.detach().numpy(), q_logsigma=q._logsigma.detach().numpy(),
               an_eps_z=ez.reshape(Nval * Nmc, -1), an_eps_x=ex.reshape(Nval * Nmc, -1),
               an_eps_y=ey.reshape(Nval * Nmc, -1), logscore=np.float64(logscore), r2=np.float64(r2),
               relerr=np.float64(relerr))
    np.savez_compressed(os.path.join(HERE, 'pe_analysis_c32.npz'), **out)
    print('pe/analysis ok', pe_terms, logscore, r2, relerr)


def make_terms():
    rng = np.random.default_rng(7)
    t = torch.tensor(rng.normal(size=(5, 7)))
    m = torch.tensor(rng.normal(size=(5, 7)))
    lv = torch.tensor(rng.normal(size=(5, 7)))
    np.savez_compressed(os.path.join(HERE, 'terms.npz'), t=t.numpy(), m=m.numpy(), lv=lv.numpy(),
                        dgll=R_utils.DiagonalGaussianLogLikelihood(t, m, lv).numpy(),
                        kl=R_utils.UnitGaussianKullbackLeiblerDivergence(m, lv).numpy())


ALL = {
    'terms': make_terms,
    'codec_c32': lambda: make_codec('c32', 32, 16, 8, [1, 1], 4, 4, 4, B=8),
    'codec_c64': lambda: make_codec('c64', 64, 64, 8, [1, 2, 1], 4, 6, 6, B=4),
    'codec_drop_c64': lambda: make_codec_drop('c64', 64, 64, 8, [1, 2, 1], 4, 6, B=8),
    'rom_c32': make_rom,
    'rom_c64': lambda: make_rom('c64'),
    'elbo_c32': make_elbo,
    'elbo_c64': make_elbo_c64,
    'elbo_opts_c32': make_elbo_options_c32,
    'bn_running_c32': make_bn_running_c32,
    'elbo_nonarm_c32': make_elbo_nonarmortized,
    'vo_c32': make_vo,
    'vo_elbo_c32': make_vo_elbo,
    'vo_elbo_lockx_c32': lambda: make_vo_elbo(lockx=True),
    'pe_analysis_c32': make_pe_analysis,
}

if __name__ == '__main__':
    # python tests/golden/make_golden.py [fixture ...]   (default: all)
    for name in (sys.argv[1:] or list(ALL)):
        ALL[name]()
