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
