"""The ReLU branch decisions of the native fp32 kernels, read back from an ElboEngine's workspace
after its forward: for every BatchNorm+ReLU the consumer conv applies on load, mask =
(fmaf(x, sc, sh) > 0) with x the stored raw fp32 input and (sc, sh) the kernels' fp32 coefficients
from the fp64 batch sums, reproduced bit for bit (replica summation order and explicit FMAs,
conv.hip stat_finish / mean_invstd / phase 2), so a near-tie pixel takes the kernels' branch
exactly; for the encoder's FC ReLU, the stored pre-activation (head.hip hpre).  Test
infrastructure: fed to the fp64 oracle (oracle/codec.py masks) so that activations within rounding
of 0 take the same branch on both sides."""
from fractions import Fraction

import numpy as np
import torch

from gpi import _lib as L
from gpi.engine import N_TERMS


def _round_f32(q):
    """The float32 nearest to the Fraction q (ties to even): one rounding, as fmaf's."""
    f = np.float32(float(q))
    best = f
    for c in (np.nextafter(f, np.float32(-np.inf)), np.nextafter(f, np.float32(np.inf))):
        dc, db = abs(Fraction(float(c)) - q), abs(Fraction(float(best)) - q)
        if dc < db or (dc == db and (int(np.float32(c).view(np.int32)) & 1) == 0):
            best = c
    return np.float32(best)


def replica_sums(stats_r):
    """conv.hip stat_finish: the GPI_REPLICAS fp64 records [R, ..., 4] of a channel summed in the
    kernels' order -- per half h (replicas 8h..8h+7) the even and the odd replicas separately, the
    two halves added last."""
    R = stats_r.shape[0]
    assert R == 16
    halves = []
    for h in range(2):
        s0 = np.zeros(stats_r.shape[1:])
        s1 = np.zeros(stats_r.shape[1:])
        for r in range(0, 8, 2):
            s0 = s0 + stats_r[8 * h + r]
            s1 = s1 + stats_r[8 * h + r + 1]
        halves.append(s0 + s1)
    return halves[0] + halves[1]


def _coefs(stats, gamma, beta, n, eps=1e-5):
    """conv.hip mean_invstd + phase 2, every rounding as the kernels do it: mean = fl32(s/n),
    var = fma(-m, m, s2/n) in fp64, inv = fl32(1 / sqrt(var + eps)), sc = fl32(gamma inv),
    sh = fmaf(-fl32(mean gamma), inv, beta)."""
    C = stats.shape[0]
    sc = np.empty(C, np.float32)
    sh = np.empty(C, np.float32)
    e = np.float64(np.float32(eps))
    for c in range(C):
        m = np.float64(stats[c, 0]) / np.float64(n)
        s2n = np.float64(stats[c, 1]) / np.float64(n)
        var = float(Fraction(float(s2n)) - Fraction(float(m)) * Fraction(float(m)))   # one fp64 rounding
        var = max(var, 0.0)
        mean = np.float32(m)
        inv = np.float32(np.float64(1.0) / np.sqrt(np.float64(var) + e))
        g, b = np.float32(gamma[c]), np.float32(beta[c])
        sc[c] = np.float32(g * inv)
        p = np.float32(np.float64(mean) * np.float64(g))                                 # exact product, one rounding
        sh[c] = _round_f32(Fraction(float(b)) - Fraction(float(p)) * Fraction(float(inv)))
    return sc.astype(np.float64), sh.astype(np.float64)


def _program_masks(prog, ws_np, stats, P, rows, group, n_group):
    out = {}
    for op in prog.ops:
        if op.bn is None:
            continue
        src = op.src
        B_all = None
        base = src.off
        d = op.desc
        x = ws_np[base:base + (rows.stop) * src.per_sample].reshape(-1, src.C, src.H, src.W)[rows, op.c0:op.c0 + op.cin]
        st = stats[group, d.in_stat:d.in_stat + op.cin]
        sc, sh = _coefs(st, P[d.gamma_off:d.gamma_off + op.cin], P[d.beta_off:d.beta_off + op.cin],
                        float(n_group) * src.H * src.W)
        # fmaf(x, sc, sh) > 0: the fp64 product of two fp32 values is exact and one fp64 addition
        # keeps the sign of the exact sum (the kernels' single fp32 rounding keeps it too)
        y = x.astype(np.float64) * sc[None, :, None, None] + sh[None, :, None, None]
        out[op.bn] = torch.tensor(y > 0)
        del B_all
    return out


def engine_relu_masks(engine):
    """{'enc': {...}, 'dec_u': {...}, 'dec_s': {...}} after engine.forward (before the next
    forward / step epilogue clears the statistics)."""
    torch.cuda.synchronize()
    ws = engine.ws
    ws_np = ws.t_ws.cpu().numpy()
    P = engine.flat.P.detach().cpu().numpy()
    R, G = L.GPI_REPLICAS, L.GPI_MAX_GROUPS
    scr = ws.t_scr.cpu().numpy()
    o = N_TERMS * R
    stats = replica_sums(scr[o:o + R * G * ws.n_stats * 4].reshape(R, G, ws.n_stats, 4))
    masks = {}
    if engine.ep is not None and engine.B_u > 0:
        estats = stats      # the encoder context's statistics live in the same arena, group 0
        masks['enc'] = _program_masks(engine.ep, ws_np, estats, P, slice(0, engine.B_u), 0, engine.B_u)
        hp = ws_np[engine.hb['hpre']:engine.hb['hpre'] + engine.B_u * engine.ep.d_feat]
        masks['enc']['features.FC'] = torch.tensor(hp.reshape(engine.B_u, -1) > 0)
    g = 0
    if engine.B_u > 0:
        masks['dec_u'] = _program_masks(engine.dp, ws_np, stats, P, slice(0, engine.B_u), g, engine.B_u)
        g += 1
    if engine.N_s > 0:
        masks['dec_s'] = _program_masks(engine.dp, ws_np, stats, P, slice(engine.B_u, engine.B_u + engine.N_s), g,
                                        engine.N_s)
        g += 1
    if getattr(engine, 'N_vo', 0) > 0:       # the VO term's decoder batch: the third BN group
        r0 = engine.B_u + engine.N_s
        masks['dec_v'] = _program_masks(engine.dp, ws_np, stats, P, slice(r0, r0 + engine.N_vo), g, engine.N_vo)
    return masks


def codec_engine_masks(e, B):
    """The ReLU decisions of a standalone EncoderEngine / DecoderEngine (CNNEncoder / CNNDecoder module
    path) after its forward: {BN layer: mask} over the B samples (one BN group), plus the encoder FC's
    ('features.FC') for an encoder engine."""
    torch.cuda.synchronize()
    ws = e.ws
    R, G = L.GPI_REPLICAS, L.GPI_MAX_GROUPS
    scr = ws.t_scr.cpu().numpy()
    o = N_TERMS * R
    stats = replica_sums(scr[o:o + R * G * ws.n_stats * 4].reshape(R, G, ws.n_stats, 4))
    ws_np = ws.t_ws.cpu().numpy()
    masks = _program_masks(e.p, ws_np, stats, e.flat.P.detach().cpu().numpy(), slice(0, B), 0, B)
    if 'hpre' in getattr(e, 'hb', {}) and e.p.kind == 'encoder':
        hp = ws_np[e.hb['hpre']:e.hb['hpre'] + B * e.p.d_feat]
        masks['features.FC'] = torch.tensor(hp.reshape(B, -1) > 0)
    return masks
