"""Test helpers: the fp64 CPU oracle of GenerativeModel.elbo (armortized unsupervised +
supervised freeX, generative.py:247-287,461-500,546-585) on a golden fixture's state,
and the comparison metrics the parity tests use.  Test infrastructure only."""
import os

import numpy as np
import torch

from oracle import codec as ocodec
from oracle import elbo as oelbo
from oracle import fem

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

# codec hyper-parameters of the fixtures (factories/model.py:187-257)
CODEC = {32: dict(blocks=[1, 1], growth=4, f0=4), 64: dict(blocks=[1, 2, 1], growth=4, f0=6),
         128: dict(blocks=[1, 2, 2, 1], growth=4, f0=6), 256: dict(blocks=[1, 2, 2, 2, 1], growth=4, f0=6)}
_PHYS = {}


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


def physics(nc, r):
    """(M [n_c, n_c, n_T], W [d_y, n_c], coarse Dirichlet dofs) from the oracle's P1 restatement."""
    key = (nc, r)
    if key not in _PHYS:
        mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(nc * r)
        _PHYS[key] = (fem.rom_stiffness_tensor(mc), fem.prolongation_free(mc, mf), fem.dirichlet_split(mc)[0])
    return _PHYS[key]


def state_of(d, dtype=torch.float64):
    """Fixture 'state.*' entries (BN running buffers dropped) as leaf tensors that require grad."""
    return {k[6:]: torch.tensor(v, dtype=dtype, requires_grad=True) for k, v in d.items()
            if k.startswith('state.') and not k.endswith(('running_mean', 'running_var', 'num_batches_tracked'))}


def oracle_elbo(st, Xu, Xs, Y, F, eps_enc, eps_qz, eps_qX, nc, r, normalize=False, l2_penalty=None, masks=None,
                drops=None, log_field=True):
    """ELBO of the armortized + supervised-freeX model in fp64 from the parameter dict ``st``
    (reference state_dict names) and fully injected inputs / noise; returns the 0-d ELBO (backward
    fills st[*].grad).  masks: optional {'enc', 'dec_u', 'dec_s'} ReLU decisions of the kernels
    under test (oracle/codec.py, tests/gpu_masks.py).  log_field: reconstruct_log_eff_property.  drops: optional Dropout2d channel scales
    {'enc': {conv: [B_u, C]}, 'dec': {conv: [B_u + N_s, C]}} (decoder rows: unlabeled, then labeled)."""
    mk = masks or {}
    dr = drops or {}
    nu = len(Xu)
    sl = lambda d, a, b: {k: torch.as_tensor(np.asarray(v))[a:b] for k, v in d.items()} if d else None
    dr_enc, dr_u, dr_s = (sl(dr.get('enc'), 0, nu), sl(dr.get('dec'), 0, nu), sl(dr.get('dec'), nu, None))
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    n = nc * r
    cfg = CODEC[n] if n in CODEC else CODEC[64]
    M, W, bc = physics(nc, r)
    M, W, bc = t(M), t(W), torch.as_tensor(bc)
    enc_p = {k[8:]: v for k, v in st.items() if k.startswith('encoder.')}
    dec_p = {k[2:]: v for k, v in st.items() if k.startswith('f.')}
    enc = lambda x: ocodec.encoder_forward(enc_p, x, n, cfg['blocks'], cfg['growth'], cfg['f0'], mk.get('enc'),
                                           dr_enc)
    dec_u = lambda z: ocodec.decoder_forward(dec_p, z, 8, cfg['blocks'], cfg['growth'], cfg['f0'], mk.get('dec_u'),
                                             dr_u)
    dec = lambda z: ocodec.decoder_forward(dec_p, z, 8, cfg['blocks'], cfg['growth'], cfg['f0'], mk.get('dec_s'),
                                           dr_s)
    e1, _ = oelbo.elbo_unsupervised_armortized(enc, dec_u, t(Xu), t(eps_enc), log_field)
    gp = lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])
    rom = lambda x, Fm: oelbo.rom_operator(W, M, bc, x, Fm, st['g.logsigmas_y'])
    e2, _ = oelbo.elbo_supervised_freeX(
        dec, gp, st['gp.logsigmas_X'], rom, (st['q_z.supervised._mean'], st['q_z.supervised._logsigma']),
        (st['q_X.supervised._mean'], st['q_X.supervised._logsigma']), t(Xs), t(Y), t(F), t(eps_qz), t(eps_qX), log_field)
    if normalize:        # every term divided by its own batch size (generative.py:493-499,571-574)
        e1 = e1 / len(Xu)
        e2 = e2 / len(Xs)
    val = e1 + e2
    if l2_penalty is not None:      # generative.py:268-276: norms (not squared) of f's and the encoder's parameters
        pen = sum(torch.norm(v) for k, v in st.items() if k.startswith(('f.', 'encoder.')))
        val = val - l2_penalty * pen
    return val


def oracle_fixture_elbo(d, **kw):
    """oracle_elbo on a fixture's own inputs / state / injected noise -> (elbo float, {name: grad})."""
    n, nc, dz, Nu, bs, Ns = [int(v) for v in d['cfg']]
    st = state_of(d)
    Xu = np.asarray(d['Xu'])[np.asarray(d['perm'][:bs])]
    val = oracle_elbo(st, Xu, d['Xs'], d['Y'], d['F'], d['eps_enc'], d['eps_qz'], d['eps_qX'], nc, n // nc, **kw)
    (-val).backward()
    return float(val.item()), {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}


def _c32_codecs(st, masks, n=32):
    mk = masks or {}
    cfg = CODEC[n]
    enc_p = {k[8:]: v for k, v in st.items() if k.startswith('encoder.')}
    dec_p = {k[2:]: v for k, v in st.items() if k.startswith('f.')}
    enc = lambda x: ocodec.encoder_forward(enc_p, x, n, cfg['blocks'], cfg['growth'], cfg['f0'], mk.get('enc'))
    dec = {g: (lambda z, g=g: ocodec.decoder_forward(dec_p, z, 8, cfg['blocks'], cfg['growth'], cfg['f0'],
                                                     mk.get(g)))
           for g in ('dec_u', 'dec_s', 'dec_v')}
    return enc, dec


def oracle_vo_fixture_elbo(d, vo_mean, vo_vars, masks=None, lockx=False, holdoff=False):
    """fp64 oracle of GenerativeModel.elbo with the VO term (armortized unsupervised + supervised +
    virtual observables; generative.py:247-287, freeX :341-392 / :461-500, lockX :300-339 / :429-459)
    on vo_elbo(_lockx)_c32.npz's state, data and injected noise.  vo_mean / vo_vars: the VO posterior
    the kernels conditioned (VirtualObservablesEnsemble.mean / .vars, fp32); the VO target is
    reparametrize(mean, 0.5 log vars) (generative.py:311,356).  masks: the kernels' ReLU decisions per
    codec call {'enc', 'dec_u', 'dec_s', 'dec_v'}.  holdoff: the VO term keeps logL_x - KL only.
    Returns (elbo float, {name: grad of -elbo})."""
    n, nc, dz, Nu, bs, Ns, Nvo, Nmc = [int(v) for v in d['cfg']]
    st = state_of(d)
    t = lambda k: torch.as_tensor(np.asarray(d[k]), dtype=torch.float64)
    M, W, bc = t('M'), t('W'), torch.as_tensor(d['bc_dofs'])
    enc, dec = _c32_codecs(st, masks, n)
    gp = lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])
    rom = lambda x, F: oelbo.rom_operator(W, M, bc, x, F, st['g.logsigmas_y'])
    qz = lambda key: (st['q_z.%s._mean' % key], st['q_z.%s._logsigma' % key])
    qx = lambda key: (st['q_X.%s._mean' % key], st['q_X.%s._logsigma' % key])
    pre = 'epsh' if holdoff else 'eps'
    e = lambda i: t('%s%d' % (pre, i))
    Xu = t('Xu')[torch.as_tensor(d['perm'][:bs])]
    e1, _ = oelbo.elbo_unsupervised_armortized(enc, dec['dec_u'], Xu, e(0))
    if lockx:
        e2, _ = oelbo.elbo_supervised_lockX(dec['dec_s'], gp, rom, qz('supervised'), t('Xs'), t('Ys'), t('Fs'), e(1))
        i_qz, i_y = 2, 3
    else:
        e2, _ = oelbo.elbo_supervised_freeX(dec['dec_s'], gp, st['gp.logsigmas_X'], rom, qz('supervised'),
                                            qx('supervised'), t('Xs'), t('Ys'), t('Fs'), e(1), e(2))
        i_qz, i_y = 3, 5
    if holdoff:
        z = oelbo.reparam(*qz('vo'), e(i_qz))
        mx, lsx = dec['dec_v'](z)
        e3 = oelbo.dgll(t('Xv'), mx, 2 * lsx) - oelbo.kl_unit(qz('vo')[0], 2 * qz('vo')[1])
    else:
        vm = torch.as_tensor(np.asarray(vo_mean), dtype=torch.float64)
        vv = torch.as_tensor(np.asarray(vo_vars), dtype=torch.float64)
        y = vm + torch.sqrt(vv) * e(i_y)
        if lockx:
            e3, _ = oelbo.elbo_supervised_lockX(dec['dec_v'], gp, rom, qz('vo'), t('Xv'), y, t('Fv'), e(i_qz))
        else:
            e3, _ = oelbo.elbo_supervised_freeX(dec['dec_v'], gp, st['gp.logsigmas_X'], rom, qz('vo'), qx('vo'),
                                                t('Xv'), y, t('Fv'), e(i_qz), e(4))
    val = e1 + e2 + e3
    (-val).backward()
    return float(val.item()), {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}


def oracle_vo_updates(d, lockx=False, n_updates=2):
    """fp64 oracle of update_virtual_observables x n_updates (generative.py:182-222: MC predictive through
    the ROM with the fixture's injected draws; VirtualObservables.py:642-669 conditioning, :971-998
    precision update between updates) on vo_elbo(_lockx)_c32.npz.  Returns a list of dicts
    {Y_mean, Y_std, vo_var, mean, vars} per update and the final prec_beta."""
    n, nc, dz, Nu, bs, Ns, Nvo, Nmc = [int(v) for v in d['cfg']]
    st = {k: v.detach() for k, v in state_of(d).items()}
    t = lambda k: torch.as_tensor(np.asarray(d[k]), dtype=torch.float64)
    M, W, bc = t('M'), t('W'), torch.as_tensor(d['bc_dofs'])
    G, A = t('Gamma'), t('alpha')
    m = G.shape[1]
    infinite = torch.zeros(m, dtype=torch.bool)
    infinite[:(nc + 1) ** 2] = True             # CGR rows: infinite precision; flux rows learnable
    vo_var = oelbo.vo_mean_variances(torch.ones(m, dtype=torch.float64), Nvo, infinite)
    gp = (lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias'])) if lockx else None
    qkey = 'q_z.vo' if lockx else 'q_X.vo'
    out, beta = [], None
    for it in range(n_updates):
        ex = t('upd%d.eps_X' % it).view(Nvo, Nmc, -1)
        ey = t('upd%d.eps_y' % it).view(Nvo, Nmc, -1)
        Ym, Ys = oelbo.vo_predictive(W, M, bc, st[qkey + '._mean'], st[qkey + '._logsigma'], t('Fv'),
                                     st['g.logsigmas_y'], ex, ey, gp_linear=gp)
        if it > 0:
            beta = oelbo.vo_precision_beta(list(G), list(A), list(out[-1]['mean']), list(out[-1]['vars']))
            vo_var = oelbo.vo_mean_variances(beta, Nvo, infinite)
        res = [oelbo.vo_condition(G[i], A[i], Ym[i], 1 / Ys[i] ** 2, vo_var) for i in range(Nvo)]
        out.append(dict(Y_mean=Ym, Y_std=Ys, vo_var=vo_var.clone(), mean=torch.stack([r[0] for r in res]),
                        vars=torch.stack([r[1] for r in res])))
    return out, beta


def oracle_nonarm_fixture_elbo(d, masks=None):
    """fp64 oracle of elbo_unsupervised (generative.py:515-544: per-sample q_z['unsupervised'] rows, the
    KL of q_z['supervised'], sic :525) + supervised freeX on elbo_nonarm_c32.npz; masks {'dec_u',
    'dec_s'}.  Returns (elbo float, {name: grad of -elbo})."""
    n, nc, dz, Nu, Ns = [int(v) for v in d['cfg']]
    st = state_of(d)
    t = lambda k: torch.as_tensor(np.asarray(d[k]), dtype=torch.float64)
    _, dec = _c32_codecs(st, masks, n)
    qzs = (st['q_z.supervised._mean'], st['q_z.supervised._logsigma'])
    Zu = oelbo.reparam(st['q_z.unsupervised._mean'], st['q_z.unsupervised._logsigma'], t('eps_u'))
    mx, lsx = dec['dec_u'](Zu)
    e1 = oelbo.dgll(t('Xu'), mx, 2 * lsx) - oelbo.kl_unit(qzs[0], 2 * qzs[1])
    e2, _ = oelbo.elbo_supervised_freeX(
        dec['dec_s'], lambda z: torch.nn.functional.linear(z, st['gp.fc.weight'], st['gp.fc.bias']),
        st['gp.logsigmas_X'], lambda x, F: oelbo.rom_operator(t('W'), t('M'), torch.as_tensor(d['bc_dofs']), x, F,
                                                              st['g.logsigmas_y']),
        qzs, (st['q_X.supervised._mean'], st['q_X.supervised._logsigma']), t('Xs'), t('Y'), t('F'), t('eps_qz'),
        t('eps_qX'))
    val = e1 + e2
    (-val).backward()
    return float(val.item()), {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}


def tensor_rel(g, ref):
    """Per-tensor relative error max|g - ref| / max|ref| (no absolute floor)."""
    g = np.asarray(g, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-300))


# gradients that reach the loss without passing backward through a ReLU mask (the last decoder conv,
# the ROM / gp / q_X rows): a fp32 forward can flip a ReLU whose fp64 input is within rounding of 0
# (tens of near-ties among the ~10^7 activations of a C64 batch), which moves every gradient upstream
# of that pixel by its share; these tensors are immune to that
MASK_FREE = ('f.features.LastTransUp.conv3.', 'g.logsigmas_y', 'gp.', 'q_X.')


def check_grads(errs, tol_all=5e-3, tol_mask_free=1e-4, tol_median=2e-5, frac_tight=0.7, tight=1e-4):
    """Gradient parity of a whole model: every tensor within tol_all (per-tensor relative, no floor),
    mask-free tensors within tol_mask_free, the median tensor within tol_median and at least
    frac_tight of the tensors within ``tight`` (a systematic kernel error fails these broadly;
    isolated ReLU-tie flips do not).  Returns a printable report."""
    items = sorted(errs.items(), key=lambda kv: -kv[1])
    rep = '\n'.join('%-58s %.2e' % kv for kv in items)
    vals = np.array([e for _, e in items])
    assert vals.max() < tol_all, rep
    bad = {k: e for k, e in items if k.startswith(MASK_FREE) and e >= tol_mask_free}
    assert not bad, (bad, rep)
    assert np.median(vals) < tol_median, rep
    assert (vals < tight).mean() >= frac_tight, rep
    return rep
