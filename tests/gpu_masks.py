"""The ReLU branch decisions of the native fp32 kernels, read back from an ElboEngine's workspace
after its forward: for every BatchNorm+ReLU the consumer conv applies on load, mask = (x * sc + sh
> 0) with x the stored raw fp32 input and (sc, sh) the kernels' fp32 coefficients from the fp64
batch sums (conv.hip mean_invstd / phase 2); for the encoder's FC ReLU, the stored pre-activation
(head.hip hpre).  Test infrastructure: fed to the fp64 oracle (oracle/codec.py masks) so that
activations within rounding of 0 take the same branch on both sides."""
import numpy as np
import torch

from gpi import _lib as L
from gpi.engine import N_TERMS


def _coefs(stats, gamma, beta, n, eps=1e-5):
    """conv.hip mean_invstd + phase 2, in the kernels' precisions."""
    m = stats[:, 0] / n
    var = np.maximum(stats[:, 1] / n - m * m, 0.0)
    mean = m.astype(np.float32)
    inv = (1.0 / np.sqrt(var + np.float64(np.float32(eps)))).astype(np.float32)
    g = gamma.astype(np.float32)
    b = beta.astype(np.float32)
    sc = g * inv
    sh = b - (mean * g) * inv
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
    stats = scr[o:o + R * G * ws.n_stats * 4].reshape(R, G, ws.n_stats, 4).sum(0)
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
