"""Diagnostic: the fused epilogue + Adam launch vs the two-launch form on the C32 golden model, step by
step (eager, then captured): max abs / rel difference of every piece of step state.
usage: python tools/fused_adam_probe.py"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'generative-physics-informed-pde_amd')]
import torch  # noqa: E402
from test_gpu_parity import load, build_golden_model, cuda  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def diff(name, a, b):
    a, b = a.double(), b.double()
    d = (a - b).abs()
    i = int(d.argmax()) if d.numel() else 0
    print('%-10s max|d| %.3e at %d (a %.6e b %.6e)  n_diff %d / %d' % (name, float(d.max()) if d.numel() else 0, i,
                                                                     float(a.flatten()[i]), float(b.flatten()[i]),
                                                                     int((d > 0).sum()), d.numel()))


def main():
    d = load('elbo_c32.npz')
    for mode in ('eager', 'graph'):
        model_a, bs = build_golden_model(d)
        model_b = copy.deepcopy(model_a)
        Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
        two = FusedElboStep(model_a, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
        one = FusedElboStep(model_b, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
        two.fuse_adam = False
        if mode == 'graph':
            two.capture()
            one.capture()
        for it in range(3):
            two.step()
            one.step()
            torch.cuda.synchronize()
            print(mode, 'step', it, 'ctr', two.step_ctr.item(), one.step_ctr.item(), 'rng', two.rng_off.item(),
                  one.rng_off.item(), 'done', one.done_ctr.item())
            for n, a, b in (('P', two.flat.P, one.flat.P), ('m', two.m, one.m), ('v', two.v, one.v),
                            ('G', two.flat.G, one.flat.G), ('terms', two.last_terms, one.last_terms),
                            ('idx', two.idx, one.idx), ('gacc', two.flat.gacc, one.flat.gacc)):
                diff(n, a, b)


if __name__ == '__main__':
    main()
