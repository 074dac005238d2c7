"""Pin the CPU oracle against golden fixtures produced by the reference's own
modules (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import codec as ocodec
from oracle import elbo as oelbo

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


def params(d, prefix, dtype=torch.float64, grad=False):
    out = {}
    for k, v in d.items():
        if k.startswith(prefix) and '.grad.' not in k and not k.startswith(prefix + 'grad.'):
            name = k[len(prefix):]
            if name.endswith('running_mean') or name.endswith('running_var') or name.endswith('num_batches_tracked'):
                continue
            out[name] = torch.tensor(v, dtype=dtype, requires_grad=grad)
    return out


def test_terms():
    d = load('terms.npz')
    t, m, lv = (torch.tensor(d[k]) for k in ('t', 'm', 'lv'))
    np.testing.assert_allclose(oelbo.dgll(t, m, lv).item(), d['dgll'], rtol=1e-12)
    np.testing.assert_allclose(oelbo.kl_unit(m, lv).item(), d['kl'], rtol=1e-12)


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_codec(tag):
    d = load('codec_%s.npz' % tag)
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]
    pe = params(d, 'enc.', grad=True)
    X = torch.tensor(d['X'], dtype=torch.float64, requires_grad=True)
    mu, ls = ocodec.encoder_forward(pe, X, imsize, blocks, growth, f_enc)
    np.testing.assert_allclose(mu.detach().numpy(), d['enc_mu'], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ls.detach().numpy(), d['enc_ls'], rtol=1e-4, atol=1e-5)
    (torch.sum(mu * torch.tensor(d['enc_wm'])) + torch.sum(ls * torch.tensor(d['enc_ws']))).backward()
    np.testing.assert_allclose(X.grad.numpy(), d['grad_X'], rtol=1e-3, atol=1e-4)
    for k, p in pe.items():
        np.testing.assert_allclose(p.grad.numpy(), d['enc.grad.' + k], rtol=1e-3, atol=2e-4, err_msg=k)

    pd = params(d, 'dec.', grad=True)
    Z = torch.tensor(d['Z'], dtype=torch.float64, requires_grad=True)
    mx, lsx = ocodec.decoder_forward(pd, Z, latent, blocks, growth, f_dec)
    np.testing.assert_allclose(mx.detach().numpy(), d['dec_mu'], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(lsx.detach().numpy(), d['dec_ls'], rtol=1e-4, atol=1e-5)
    (torch.sum(mx * torch.tensor(d['dec_vm'])) + torch.sum(lsx * torch.tensor(d['dec_vs']))).backward()
    np.testing.assert_allclose(Z.grad.numpy(), d['grad_Z'], rtol=1e-3, atol=1e-4)
    for k, p in pd.items():
        np.testing.assert_allclose(p.grad.numpy(), d['dec.grad.' + k], rtol=1e-3, atol=2e-3, err_msg=k)


def test_rom():
    d = load('rom_c32.npz')
    M = torch.tensor(d['M'], dtype=torch.float64)
    W = torch.tensor(d['W'], dtype=torch.float64)
    e = torch.tensor(d['effprop'], dtype=torch.float64, requires_grad=True)
    ls = torch.tensor(d['logsigmas_y'], dtype=torch.float64, requires_grad=True)
    mu, lsr = oelbo.rom_operator(W, M, torch.tensor(d['bc_dofs']), e, torch.tensor(d['F'], dtype=torch.float64), ls)
    np.testing.assert_allclose(mu.detach().numpy(), d['mu_y'], rtol=1e-4, atol=1e-5)
    L = oelbo.dgll(torch.tensor(d['Y'], dtype=torch.float64), mu, 2 * lsr)
    np.testing.assert_allclose(L.item(), d['logL'], rtol=1e-5)
    (-L).backward()
    np.testing.assert_allclose(e.grad.numpy(), d['grad_effprop'], rtol=2e-3, atol=1e-3)
    np.testing.assert_allclose(ls.grad.numpy(), d['grad_logsigmas_y'], rtol=1e-3, atol=1e-4)


def test_elbo_step():
    d = load('elbo_c32.npz')
    n, nc, dz, Nu, bs, Ns = [int(v) for v in d['cfg']]
    st = {k[len('state.'):]: torch.tensor(v, dtype=torch.float64, requires_grad=True)
          for k, v in d.items() if k.startswith('state.') and not k.endswith(('running_mean', 'running_var', 'num_batches_tracked'))}
    enc_p = {k[len('encoder.'):]: v for k, v in st.items() if k.startswith('encoder.')}
    dec_p = {k[len('f.'):]: v for k, v in st.items() if k.startswith('f.')}
    M = torch.tensor(d['M'], dtype=torch.float64)
    W = torch.tensor(d['W'], dtype=torch.float64)
    bc = torch.tensor(d['bc_dofs'])
    enc = lambda x: ocodec.encoder_forward(enc_p, x, n, [1, 1], 4, 4)
    dec = lambda z: ocodec.decoder_forward(dec_p, z, 8, [1, 1], 4, 4)
    Xu = torch.tensor(d['Xu'], dtype=torch.float64)[torch.tensor(d['perm'][:bs])]
    e1, _ = oelbo.elbo_unsupervised_armortized(enc, dec, Xu, torch.tensor(d['eps_enc'], dtype=torch.float64))
    gp = lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])
    rom = lambda x, F: oelbo.rom_operator(W, M, bc, x, F, st['g.logsigmas_y'])
    e2, _ = oelbo.elbo_supervised_freeX(
        dec, gp, st['gp.logsigmas_X'], rom,
        (st['q_z.supervised._mean'], st['q_z.supervised._logsigma']),
        (st['q_X.supervised._mean'], st['q_X.supervised._logsigma']),
        torch.tensor(d['Xs'], dtype=torch.float64), torch.tensor(d['Y'], dtype=torch.float64),
        torch.tensor(d['F'], dtype=torch.float64),
        torch.tensor(d['eps_qz'], dtype=torch.float64), torch.tensor(d['eps_qX'], dtype=torch.float64))
    elbo = e1 + e2
    np.testing.assert_allclose(elbo.item(), float(d['elbo']), rtol=2e-5)
    (-elbo).backward()
    for k, p in st.items():
        ref = d.get('grad.' + k)
        assert ref is not None, k
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(p.grad.numpy() / scale, ref / scale, atol=2e-4, err_msg=k)


def test_vo_update():
    d = load('vo_c32.npz')
    for i in range(d['Gamma'].shape[0]):
        mean, var = oelbo.vo_condition(torch.tensor(d['Gamma'][i]), torch.tensor(d['alpha'][i]),
                                       torch.tensor(d['g'][i]), torch.tensor(d['prec'][i]),
                                       torch.tensor(d['vo_var']))
        np.testing.assert_allclose(mean.numpy(), d['mean'][i], rtol=1e-9, atol=1e-10)
        np.testing.assert_allclose(var.numpy(), d['vars'][i], rtol=1e-7, atol=1e-12)
    beta = oelbo.vo_precision_beta([torch.tensor(g) for g in d['Gamma']], [torch.tensor(a) for a in d['alpha']],
                                   [torch.tensor(m) for m in d['mean']], [torch.tensor(v) for v in d['vars']])
    np.testing.assert_allclose(beta.numpy(), d['prec_beta'], rtol=1e-9)


def _vo_fixture_state(d):
    st = {k[len('state.'):]: torch.tensor(v, dtype=torch.float64, requires_grad=True)
          for k, v in d.items() if k.startswith('state.') and
          not k.endswith(('running_mean', 'running_var', 'num_batches_tracked'))}
    return st


def test_vo_pipeline_and_vo_elbo():
    """update_virtual_observables x2 (MC predictive, precision update, conditioning) and the ELBO
    with the VO term (generative.py:182-222,341-392), oracle vs the reference's own classes."""
    d = load('vo_elbo_c32.npz')
    n, nc, dz, Nu, bs, Ns, Nvo, Nmc = [int(v) for v in d['cfg']]
    st = _vo_fixture_state(d)
    M = torch.tensor(d['M'], dtype=torch.float64)
    W = torch.tensor(d['W'], dtype=torch.float64)
    bc = torch.tensor(d['bc_dofs'])
    t64 = lambda k: torch.tensor(d[k], dtype=torch.float64)
    G, A = t64('Gamma'), t64('alpha')
    m = G.shape[1]
    assert m == (nc + 1) ** 2 + 2 * nc * nc
    infinite = torch.zeros(m, dtype=torch.bool)
    infinite[:(nc + 1) ** 2] = True                       # CGR rows: infinite precision, flux rows learnable
    vo_var = oelbo.vo_mean_variances(torch.ones(m, dtype=torch.float64), Nvo, infinite)
    with torch.no_grad():
        for it in range(2):
            ex = t64('upd%d.eps_X' % it).view(Nvo, Nmc, -1).float().double()
            ey = t64('upd%d.eps_y' % it).view(Nvo, Nmc, -1).float().double()
            Ym, Ysd = oelbo.vo_predictive(W, M, bc, st['q_X.vo._mean'], st['q_X.vo._logsigma'], t64('Fv'),
                                          st['g.logsigmas_y'], ex, ey)
            np.testing.assert_allclose(Ym.numpy(), d['upd%d.Y_mean' % it], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(Ysd.numpy(), d['upd%d.Y_std' % it], rtol=1e-4, atol=1e-6)
            # the reference conditions on its fp32 Y_mean / 1/Y_std^2
            g32 = torch.tensor(d['upd%d.Y_mean' % it]).double()
            p32 = (1 / torch.tensor(d['upd%d.Y_std' % it]) ** 2).double()
            if it == 1:
                beta = oelbo.vo_precision_beta(list(G), list(A), list(mean_prev), list(vars_prev))
                np.testing.assert_allclose(beta.numpy(), d['upd1.prec_beta'], rtol=1e-9)
                vo_var = oelbo.vo_mean_variances(beta, Nvo, infinite)
            np.testing.assert_allclose(vo_var.numpy(), d['upd%d.vo_var' % it], rtol=1e-9)
            res = [oelbo.vo_condition(G[i], A[i], g32[i], p32[i], vo_var) for i in range(Nvo)]
            mean_prev = torch.stack([r[0] for r in res])
            vars_prev = torch.stack([r[1] for r in res])
            np.testing.assert_allclose(mean_prev.numpy(), d['upd%d.mean' % it], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(vars_prev.numpy(), d['upd%d.vars' % it], rtol=1e-5, atol=1e-9)

    # ELBO: armortized + supervised + VO terms
    enc_p = {k[len('encoder.'):]: v for k, v in st.items() if k.startswith('encoder.')}
    dec_p = {k[len('f.'):]: v for k, v in st.items() if k.startswith('f.')}
    enc = lambda x: ocodec.encoder_forward(enc_p, x, n, [1, 1], 4, 4)
    dec = lambda z: ocodec.decoder_forward(dec_p, z, 8, [1, 1], 4, 4)
    gp = lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])
    rom = lambda x, F: oelbo.rom_operator(W, M, bc, x, F, st['g.logsigmas_y'])
    e = [t64('eps%d' % i) for i in range(6)]
    Xu = t64('Xu')[torch.tensor(d['perm'][:bs])]
    e1, _ = oelbo.elbo_unsupervised_armortized(enc, dec, Xu, e[0])
    qz = lambda key: (st['q_z.%s._mean' % key], st['q_z.%s._logsigma' % key])
    qx = lambda key: (st['q_X.%s._mean' % key], st['q_X.%s._logsigma' % key])
    e2, _ = oelbo.elbo_supervised_freeX(dec, gp, st['gp.logsigmas_X'], rom, qz('supervised'), qx('supervised'),
                                        t64('Xs'), t64('Ys'), t64('Fs'), e[1], e[2])
    # VO targets: reparametrize(VO.mean, VO.logsigma) in fp32 (generative.py:356)
    vmean = torch.tensor(d['upd1.mean'])
    vls = 0.5 * torch.log(torch.tensor(d['upd1.vars']))
    y = (vmean + torch.exp(vls) * torch.tensor(d['eps5'])).double()
    e3, terms = oelbo.elbo_supervised_freeX(dec, gp, st['gp.logsigmas_X'], rom, qz('vo'), qx('vo'), t64('Xv'), y,
                                            t64('Fv'), e[3], e[4])
    np.testing.assert_allclose(terms['logL_y'].item(), d['term.objective/vo_logL_y'], rtol=1e-4)
    np.testing.assert_allclose(terms['logL_x'].item(), d['term.objective/vo_logL_x'], rtol=2e-5)
    elbo = e1 + e2 + e3
    np.testing.assert_allclose(elbo.item(), float(d['elbo']), rtol=2e-5)
    (-elbo).backward()
    for k, p in st.items():
        ref = d.get('grad.' + k)
        if ref is None:
            assert p.grad is None or not p.grad.abs().any(), k
            continue
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(p.grad.numpy() / scale, ref / scale, atol=2e-4, err_msg=k)


def test_vo_pipeline_and_vo_elbo_lockx():
    """independent_X = False: the VO predictive y = g(gp(z)) (generative.py:202-204), conditioning,
    and the lockX supervised / VO ELBO terms (generative.py:300-339,429-459) + gradients, oracle vs the
    reference's own classes (vo_elbo_lockx_c32.npz)."""
    d = load('vo_elbo_lockx_c32.npz')
    n, nc, dz, Nu, bs, Ns, Nvo, Nmc = [int(v) for v in d['cfg']]
    st = _vo_fixture_state(d)
    assert not any(k.startswith('q_X.') or k == 'gp.logsigmas_X' for k in st)
    M = torch.tensor(d['M'], dtype=torch.float64)
    W = torch.tensor(d['W'], dtype=torch.float64)
    bc = torch.tensor(d['bc_dofs'])
    t64 = lambda k: torch.tensor(d[k], dtype=torch.float64)
    G, A = t64('Gamma'), t64('alpha')
    m = G.shape[1]
    infinite = torch.zeros(m, dtype=torch.bool)
    infinite[:(nc + 1) ** 2] = True
    vo_var = oelbo.vo_mean_variances(torch.ones(m, dtype=torch.float64), Nvo, infinite)
    gp = lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])
    with torch.no_grad():
        for it in range(2):
            ez = t64('upd%d.eps_X' % it).view(Nvo, Nmc, -1)
            assert ez.shape[2] == dz
            ey = t64('upd%d.eps_y' % it).view(Nvo, Nmc, -1)
            Ym, Ysd = oelbo.vo_predictive(W, M, bc, st['q_z.vo._mean'], st['q_z.vo._logsigma'], t64('Fv'),
                                          st['g.logsigmas_y'], ez, ey, gp_linear=gp)
            np.testing.assert_allclose(Ym.numpy(), d['upd%d.Y_mean' % it], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(Ysd.numpy(), d['upd%d.Y_std' % it], rtol=1e-4, atol=1e-6)
            g32 = torch.tensor(d['upd%d.Y_mean' % it]).double()
            p32 = (1 / torch.tensor(d['upd%d.Y_std' % it]) ** 2).double()
            if it == 1:
                beta = oelbo.vo_precision_beta(list(G), list(A), list(mean_prev), list(vars_prev))
                np.testing.assert_allclose(beta.numpy(), d['upd1.prec_beta'], rtol=1e-9)
                vo_var = oelbo.vo_mean_variances(beta, Nvo, infinite)
            res = [oelbo.vo_condition(G[i], A[i], g32[i], p32[i], vo_var) for i in range(Nvo)]
            mean_prev = torch.stack([r[0] for r in res])
            vars_prev = torch.stack([r[1] for r in res])
            np.testing.assert_allclose(mean_prev.numpy(), d['upd%d.mean' % it], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(vars_prev.numpy(), d['upd%d.vars' % it], rtol=1e-5, atol=1e-9)

    enc_p = {k[len('encoder.'):]: v for k, v in st.items() if k.startswith('encoder.')}
    dec_p = {k[len('f.'):]: v for k, v in st.items() if k.startswith('f.')}
    enc = lambda x: ocodec.encoder_forward(enc_p, x, n, [1, 1], 4, 4)
    dec = lambda z: ocodec.decoder_forward(dec_p, z, 8, [1, 1], 4, 4)
    rom = lambda x, F: oelbo.rom_operator(W, M, bc, x, F, st['g.logsigmas_y'])
    qz = lambda key: (st['q_z.%s._mean' % key], st['q_z.%s._logsigma' % key])
    e = [t64('eps%d' % i) for i in range(4)]
    e1, _ = oelbo.elbo_unsupervised_armortized(enc, dec, t64('Xu')[torch.tensor(d['perm'][:bs])], e[0])
    e2, t2 = oelbo.elbo_supervised_lockX(dec, gp, rom, qz('supervised'), t64('Xs'), t64('Ys'), t64('Fs'), e[1])
    np.testing.assert_allclose(t2['logL_y'].item(), d['term.objective/supervised_logL_y'], rtol=2e-5)
    y = (torch.tensor(d['upd1.mean']) + torch.sqrt(torch.tensor(d['upd1.vars'])) * torch.tensor(d['eps3'])).double()
    e3, t3 = oelbo.elbo_supervised_lockX(dec, gp, rom, qz('vo'), t64('Xv'), y, t64('Fv'), e[2])
    np.testing.assert_allclose(t3['logL_y'].item(), d['term.objective/vo_logL_y'], rtol=1e-4)
    np.testing.assert_allclose(t3['DKL'].item(), d['term.objective/vo_DKL'], rtol=2e-5)
    elbo = e1 + e2 + e3
    np.testing.assert_allclose(elbo.item(), float(d['elbo']), rtol=2e-5)
    (-elbo).backward()
    for k, p in st.items():
        ref = d.get('grad.' + k)
        if ref is None:
            assert p.grad is None or not p.grad.abs().any(), k
            continue
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(p.grad.numpy() / scale, ref / scale, atol=2e-4, err_msg=k)


def test_elbo_nonarmortized():
    """elbo_unsupervised (generative.py:515-544) + supervised freeX, oracle vs the reference run."""
    d = load('elbo_nonarm_c32.npz')
    n, nc, dz, Nu, Ns = [int(v) for v in d['cfg']]
    st = _vo_fixture_state(d)
    t64 = lambda k: torch.tensor(d[k], dtype=torch.float64)
    dec_p = {k[len('f.'):]: v for k, v in st.items() if k.startswith('f.')}
    dec = lambda z: ocodec.decoder_forward(dec_p, z, 8, [1, 1], 4, 4)
    M, W = t64('M'), t64('W')
    qzs = (st['q_z.supervised._mean'], st['q_z.supervised._logsigma'])
    Zu = oelbo.reparam(st['q_z.unsupervised._mean'], st['q_z.unsupervised._logsigma'], t64('eps_u'))
    mx, lsx = dec(Zu)
    e1 = oelbo.dgll(t64('Xu'), mx, 2 * lsx) - oelbo.kl_unit(qzs[0], 2 * qzs[1])      # KL of q_z['supervised'] (sic)
    e2, _ = oelbo.elbo_supervised_freeX(
        dec, lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias']), st['gp.logsigmas_X'],
        lambda x, F: oelbo.rom_operator(W, M, torch.tensor(d['bc_dofs']), x, F, st['g.logsigmas_y']), qzs,
        (st['q_X.supervised._mean'], st['q_X.supervised._logsigma']), t64('Xs'), t64('Y'), t64('F'), t64('eps_qz'),
        t64('eps_qX'))
    elbo = e1 + e2
    np.testing.assert_allclose(elbo.item(), float(d['elbo']), rtol=2e-5)
    (-elbo).backward()
    for k, p in st.items():
        ref = d.get('grad.' + k)
        if ref is None:
            assert p.grad is None or not p.grad.abs().any(), k
            continue
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(p.grad.numpy() / scale, ref / scale, atol=2e-4, err_msg=k)


# ---------------------------------------------------------------- benchmarked shape (C64) and elbo options
def test_rom_c64():
    """nc = 8 ROM solve + adjoint (the benchmarked labeled path) vs the reference run (rom_c64.npz)."""
    from elbo_ref import physics
    d = load('rom_c64.npz')
    M, W, bc = physics(int(d['nc']), int(d['r']))
    assert np.array_equal(bc, d['bc_dofs'])
    e = torch.tensor(d['effprop'], dtype=torch.float64, requires_grad=True)
    ls = torch.tensor(d['logsigmas_y'], dtype=torch.float64, requires_grad=True)
    mu, lsr = oelbo.rom_operator(torch.tensor(W), torch.tensor(M), torch.tensor(bc), e,
                                 torch.tensor(d['F'], dtype=torch.float64), ls)
    np.testing.assert_allclose(mu.detach().numpy(), d['mu_y'], rtol=1e-4, atol=1e-5)
    L = oelbo.dgll(torch.tensor(d['Y'], dtype=torch.float64), mu, 2 * lsr)
    np.testing.assert_allclose(L.item(), d['logL'], rtol=1e-5)
    (-L).backward()
    from elbo_ref import tensor_rel
    assert tensor_rel(e.grad.numpy(), d['grad_effprop']) < 1e-3
    assert tensor_rel(ls.grad.numpy(), d['grad_logsigmas_y']) < 1e-4


def test_elbo_c64():
    """fp64 oracle of the benchmarked step (highres codec, ROM 8x8, B_u = 256, N_s = 32) vs the
    reference's fp32 CPU run (elbo_c64.npz): value 1e-5; gradients by elbo_ref.check_grads (the reference's
    own fp32 run flips a few near-tie ReLUs of the encoder: ~3e-3 on the tensors upstream of them, ~3e-6
    elsewhere)."""
    from elbo_ref import oracle_fixture_elbo, tensor_rel, check_grads
    d = load('elbo_c64.npz')
    val, gr = oracle_fixture_elbo(d)
    assert abs(val - float(d['elbo'])) <= 1e-5 * abs(float(d['elbo']))
    assert set(gr) == {k[5:] for k in d if k.startswith('grad.')}
    print(check_grads({k: tensor_rel(g, d['grad.' + k]) for k, g in gr.items()}))


@pytest.mark.parametrize('opt', ['norm', 'l2', 'expf'])
def test_elbo_options(opt):
    """elbo(normalize=True), elbo(l2_penalty=0.05) (generative.py:247-287) and the exponentiated-field
    likelihood (reconstruct_log_eff_property=False, generative.py:236-239) vs the reference run."""
    from elbo_ref import oracle_fixture_elbo, tensor_rel
    d = load('elbo_opts_c32.npz')
    kw = {'norm': dict(normalize=True), 'l2': dict(l2_penalty=float(d['l2_penalty'])), 'expf': {}}[opt]
    val, gr = oracle_fixture_elbo(d, log_field=opt != 'expf', **kw)
    assert abs(val - float(d[opt + '.elbo'])) <= 1e-5 * abs(float(d[opt + '.elbo']))
    bad = {k: e for k, e in ((k, tensor_rel(g, d[opt + '.grad.' + k])) for k, g in gr.items()) if e >= 2e-3}
    assert not bad, bad


def test_codec_dropout():
    """Oracle codec with injected Dropout2d scales vs the reference's CNNEncoder / CNNDecoder in train
    mode with drop_rate 0.2 and the same injected masks (codec_drop_c64.npz)."""
    d = load('codec_drop_c64.npz')
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]
    drops = {key: {k[len('drop.%s.' % key):]: torch.tensor(v, dtype=torch.float64) for k, v in d.items()
                   if k.startswith('drop.%s.' % key)} for key in ('enc', 'dec')}
    assert len(drops['enc']) == 10 and len(drops['dec']) == 9
    pe = params(d, 'enc.', grad=True)
    X = torch.tensor(d['X'], dtype=torch.float64, requires_grad=True)
    mu, ls = ocodec.encoder_forward(pe, X, imsize, blocks, growth, f_enc, drops=drops['enc'])
    np.testing.assert_allclose(mu.detach().numpy(), d['enc_mu'], rtol=1e-4, atol=1e-5)
    (torch.sum(mu * torch.tensor(d['enc_wm'])) + torch.sum(ls * torch.tensor(d['enc_ws']))).backward()
    for k, p in pe.items():
        np.testing.assert_allclose(p.grad.numpy(), d['enc.grad.' + k], rtol=1e-3, atol=2e-3, err_msg=k)
    pd = params(d, 'dec.', grad=True)
    Z = torch.tensor(d['Z'], dtype=torch.float64, requires_grad=True)
    mx, lsx = ocodec.decoder_forward(pd, Z, latent, blocks, growth, f_dec, drops=drops['dec'])
    np.testing.assert_allclose(mx.detach().numpy(), d['dec_mu'], rtol=1e-4, atol=1e-5)
    (torch.sum(mx * torch.tensor(d['dec_vm'])) + torch.sum(lsx * torch.tensor(d['dec_vs']))).backward()
    np.testing.assert_allclose(Z.grad.numpy(), d['grad_Z'], rtol=1e-3, atol=1e-4)
    for k, p in pd.items():
        np.testing.assert_allclose(p.grad.numpy(), d['dec.grad.' + k], rtol=1e-3, atol=2e-3, err_msg=k)


# ---------------------------------------------------------------- the GPU tests' fp64 oracle helpers
@pytest.mark.parametrize('lockx', [False, True], ids=['freeX', 'lockX'])
@pytest.mark.parametrize('holdoff', [False, True], ids=['vo', 'holdoff'])
def test_oracle_vo_fixture_elbo_helper(lockx, holdoff):
    """tests/elbo_ref.py oracle_vo_fixture_elbo (what the GPU VO-ELBO tests compare the kernels with)
    reproduces the reference run it restates: value 2e-5, gradients 2e-4 of max(|ref|, 1)."""
    from elbo_ref import oracle_vo_fixture_elbo
    d = load('vo_elbo_lockx_c32.npz' if lockx else 'vo_elbo_c32.npz')
    val, gr = oracle_vo_fixture_elbo(d, d['upd1.mean'], d['upd1.vars'], lockx=lockx, holdoff=holdoff)
    key = 'elbo_holdoff' if holdoff else 'elbo'
    np.testing.assert_allclose(val, float(d[key]), rtol=2e-5)
    pre = 'gradh.' if holdoff else 'grad.'
    for k in {k[len(pre):] for k in d if k.startswith(pre)} | set(gr):
        ref = d.get(pre + k)
        if ref is None:
            assert not np.abs(gr[k]).any(), k
            continue
        got = gr.get(k, np.zeros_like(ref))
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(got / scale, ref / scale, atol=2e-4, err_msg=k)


def test_oracle_nonarm_fixture_elbo_helper():
    from elbo_ref import oracle_nonarm_fixture_elbo
    d = load('elbo_nonarm_c32.npz')
    val, gr = oracle_nonarm_fixture_elbo(d)
    np.testing.assert_allclose(val, float(d['elbo']), rtol=2e-5)
    for k, g in gr.items():
        ref = d['grad.' + k]
        scale = max(np.abs(ref).max(), 1.0)
        np.testing.assert_allclose(g / scale, ref / scale, atol=2e-4, err_msg=k)


@pytest.mark.parametrize('lockx', [False, True], ids=['freeX', 'lockX'])
def test_oracle_vo_updates_helper(lockx):
    """tests/elbo_ref.py oracle_vo_updates (fp64 end to end) vs the reference's fp32 VO updates."""
    from elbo_ref import oracle_vo_updates
    d = load('vo_elbo_lockx_c32.npz' if lockx else 'vo_elbo_c32.npz')
    ups, beta = oracle_vo_updates(d, lockx=lockx)
    rel = lambda a, b: float(np.abs(np.asarray(a) - b).max() / np.abs(b).max())
    for it, u in enumerate(ups):
        assert rel(u['Y_mean'], d['upd%d.Y_mean' % it]) < 1e-5
        assert rel(u['Y_std'], d['upd%d.Y_std' % it]) < 1e-4
        assert rel(u['mean'], d['upd%d.mean' % it]) < 1e-5
        assert rel(u['vars'], d['upd%d.vars' % it]) < 1e-4
    assert rel(beta, d['upd1.prec_beta']) < 1e-4
