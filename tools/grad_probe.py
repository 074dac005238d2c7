"""Native encoder/decoder gradients vs the fp64 oracle on white-noise inputs at several grid
sizes; prints the worst relative error per parameter and saves the input-gradient error map.
Diagnostic tool (runs on the GPU box): python tools/grad_probe.py 64 128 256"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bottleneck.Encoder import CNNEncoder  # noqa: E402
from bottleneck.Decoder import CNNDecoder  # noqa: E402
from oracle import codec as oc  # noqa: E402

BLOCKS = {32: [1, 1], 64: [1, 2, 1], 128: [1, 2, 2, 1], 256: [1, 2, 2, 2, 1]}


def rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def run(imsize, B=2, dz=64):
    blocks = BLOCKS[imsize]
    torch.manual_seed(0)
    enc = CNNEncoder(imsize, dz, blocks, 4, 6, drop_rate=0)
    gen = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for m in enc.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(1.0 + 0.3 * torch.randn(m.weight.shape, generator=gen))
                m.bias.copy_(0.2 * torch.randn(m.bias.shape, generator=gen))
    sd = {k: v.clone().double() for k, v in enc.state_dict().items()}
    X = torch.randn(B, imsize, imsize, generator=gen).double() * 0.8 + 0.4
    wm, ws = torch.randn(B, dz, generator=gen).double(), torch.randn(B, dz, generator=gen).double()
    enc = enc.cuda()
    Xc = X.float().cuda()
    mu, ls = enc(Xc)
    (torch.sum(mu * wm.float().cuda()) + torch.sum(ls * ws.float().cuda())).backward()
    p = {k: v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point() and 'running' not in k}
    Xo = X.clone().requires_grad_(True)
    mo, lo = oc.encoder_forward(p, Xo, imsize, blocks, 4, 6)
    (torch.sum(mo * wm) + torch.sum(lo * ws)).backward()
    print('== encoder %d: mu %.2e' % (imsize, rel(mu.detach().cpu().double(), mo.detach())))
    for k, q in enc.named_parameters():
        e = rel(q.grad.cpu().double(), p[k].grad)
        if e > 1e-4:
            print('   %-45s %.2e' % (k, e))


if __name__ == '__main__':
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    for s in sys.argv[1:]:
        run(int(s))
