"""Diagnostic: captured FusedElboStep in graph modes 'single' / 'streams', fused and two-launch
(epilogue, Adam) step tails, C32 golden model: which mutable-state tensors differ after each step."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import conftest  # noqa: E402,F401
from test_gpu_parity import load, cuda, build_golden_model  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def make(model, mode, fused, d, bs):
    os.environ['GPI_GRAPH_MODE'] = mode
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    s = FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    s.fuse_adam = fused
    s.capture()
    return s


def main():
    d = load('elbo_c32.npz')
    m0, bs = build_golden_model(d)
    arms = {}
    for mode in ('single', 'streams'):
        for fused in (True, False):
            arms[(mode, fused)] = make(copy.deepcopy(m0), mode, fused, d, bs)
    names = ['P', 'm', 'v', 'step_ctr', 'rng_off', 'idx', 'idx_next', 'done_ctr', 'handoff_flags', 'side_done']
    ref = arms[('single', True)]
    for it in range(4):
        for s in arms.values():
            s.step()
            torch.cuda.synchronize()
        for k, s in arms.items():
            if s is ref:
                continue
            diffs = []
            for i, (a, b) in enumerate(zip(ref._mutable_state(), s._mutable_state())):
                if a.shape != b.shape or not torch.equal(a, b):
                    nm = names[i] if i < len(names) else 'state%d' % i
                    dd = (a.double() - b.double()).abs().max().item() if a.shape == b.shape else -1
                    diffs.append('%s(%.3g)' % (nm, dd))
            print('step %d %-8s fused=%d: %s' % (it, k[0], k[1], ', '.join(diffs) or 'identical'), flush=True)
        print('   step_ctr', {('%s/%d' % k): int(s.step_ctr.item()) for k, s in arms.items()},
              'flags', {('%s/%d' % k): s.handoff_flags[:4].tolist() for k, s in arms.items()}, flush=True)


if __name__ == '__main__':
    main()
