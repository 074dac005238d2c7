"""Autograd bridge between the drop-in modules and the native engines.

Parameters are never handed to autograd individually: each native call
takes a 0-d *anchor* leaf so that autograd invokes our backward, which
writes the fp64 gradient of every parameter through the kernels and hands
it over in one flat buffer (FlatParameters.deliver).
"""
import torch

from . import _lib as L
from .engine import EncoderEngine, DecoderEngine, rom_call, ROM_NN
from .flat import FlatParameters


def anchor(module, device):
    a = getattr(module, '_gpi_anchor', None)
    if a is None or a.device != device:
        a = torch.zeros((), device=device, requires_grad=True)
        object.__setattr__(module, '_gpi_anchor', a)
    return a


def module_flat(module, device):
    """FlatParameters owning all of ``module``'s parameters (creates one if needed)."""
    flat = getattr(module, '_gpi_flat', None)
    if flat is None or flat.P.device != device or not all(flat.owns(p) for p in module.parameters()):
        flat = FlatParameters(list(module.named_parameters()), device)
        set_flat(module, flat)
    return flat


def set_flat(module, flat):
    for m in module.modules():
        object.__setattr__(m, '_gpi_flat', flat)
        object.__setattr__(m, '_gpi_engines', {})


def engine_for(module, key, build):
    cache = getattr(module, '_gpi_engines', None)
    if cache is None:
        cache = {}
        object.__setattr__(module, '_gpi_engines', cache)
    e = cache.get(key)
    if e is None:
        e = build()
        cache[key] = e
    return e


def _deliver(flat, scale=None):
    tmp = torch.empty_like(flat.G)
    L.check(L.lib().gpi_grad_finalize(L.ptr(flat.gacc), L.ptr(tmp), flat.numel, L.FINALIZE_ZERO, None,
                                      L.stream_handle()), 'grad finalize')
    if scale is not None:
        tmp.mul_(scale)
    flat.deliver(tmp)


class EncoderFunction(torch.autograd.Function):

    @staticmethod
    def forward(ctx, a, x, engine, dropout=None, seed=0):
        ctx.engine = engine
        return engine.forward(x, dropout, seed)

    @staticmethod
    def backward(ctx, dmu, dls):
        e = ctx.engine
        dmu = torch.zeros(e.B, e.dz, device=e.flat.P.device) if dmu is None else dmu.contiguous()
        dls = torch.zeros(e.B, e.dz, device=e.flat.P.device) if dls is None else dls.contiguous()
        e.backward(dmu, dls)
        _deliver(e.flat)
        return None, None, None, None, None


def _seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _take_injected(module):
    """Dropout2d channel scales a test injected for the next call (module._gpi_inject_dropout)."""
    d = getattr(module, '_gpi_inject_dropout', None)
    if d is not None:
        object.__setattr__(module, '_gpi_inject_dropout', None)
    return d


def encoder_forward(enc, x):
    L.require_device(x)
    if x.dim() < 4:
        x = x.unsqueeze(1)
    dev = x.device
    flat = module_flat(enc, dev)
    B = x.shape[0]
    e = engine_for(enc, ('enc', B, id(flat)), lambda: EncoderEngine(enc, flat, B))
    drop = _take_injected(enc)
    return EncoderFunction.apply(anchor(enc, dev), x, e, drop, _seed() if (e.p.drop_numel and drop is None) else 0)


class DecoderFunction(torch.autograd.Function):

    @staticmethod
    def forward(ctx, a, z, engine, dropout=None, seed=0):
        ctx.engine = engine
        return engine.forward(z.contiguous().float(), dropout, seed)

    @staticmethod
    def backward(ctx, dout):
        e = ctx.engine
        dz = e.backward(dout.contiguous())
        _deliver(e.flat)
        return None, dz, None, None, None


def decoder_forward(dec, z):
    L.require_device(z)
    dev = z.device
    flat = module_flat(dec, dev)
    B = z.shape[0]
    e = engine_for(dec, ('dec', B, id(flat)), lambda: DecoderEngine(dec, flat, B))
    drop = _take_injected(dec)
    return DecoderFunction.apply(anchor(dec, dev), z, e, drop, _seed() if (e.p.drop_numel and drop is None) else 0)


class RomOperatorFunction(torch.autograd.Function):
    """ReducedOrderModelOperator mean: effprop -> W solve(K(exp(effprop)+1e-8), F)."""

    @staticmethod
    def forward(ctx, x, F, nc, refine, input_kappa):
        x = x.contiguous().float()
        F = F.contiguous().float()
        n = nc * refine
        mu = torch.empty(x.shape[0], (n + 1) * (n - 1), device=x.device, dtype=torch.float32)
        uc = torch.empty(x.shape[0], ROM_NN(nc), device=x.device, dtype=torch.float32)
        rom_call(nc, refine, x, F, input_kappa, L.ROM_FORWARD, mu_y=mu, uc=uc)
        ctx.save_for_backward(x, F)
        ctx.cfg = (nc, refine, input_kappa)
        return mu, uc

    @staticmethod
    def backward(ctx, dmu, duc):
        x, F = ctx.saved_tensors
        nc, refine, input_kappa = ctx.cfg
        gx = torch.empty_like(x)
        rom_call(nc, refine, x, F, input_kappa, L.ROM_BACKWARD,
                 dmu=dmu.contiguous() if dmu is not None else None,
                 duc=duc.contiguous() if duc is not None else None, gx=gx)
        return gx, None, None, None, None
