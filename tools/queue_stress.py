"""Stress of the cross-stream flag hand-offs under hardware-queue sharing: many FusedElboStep objects
(each with its own side stream, plus the streams capture() creates) in one process, each captured and
replayed a few steps, interleaved; a flag wait that times out (its stream shares a hardware queue with
the producer behind it) sets the hand-off error word, which check_handoff() raises on.
usage: python tools/queue_stress.py MODE N_OBJECTS [N_EXTRA_STREAMS]"""
import copy
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import conftest  # noqa: E402,F401
from test_gpu_parity import load, cuda, build_golden_model  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    mode, n = sys.argv[1], int(sys.argv[2])
    extra = [torch.cuda.Stream() for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 0)]
    os.environ['GPI_GRAPH_MODE'] = mode
    d = load('elbo_c32.npz')
    m0, bs = build_golden_model(d)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    objs = []
    for i in range(n):
        s = FusedElboStep(copy.deepcopy(m0), Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
        s.fuse_adam = bool(i % 2 == 0)
        s.capture()
        objs.append(s)
    bad = 0
    for it in range(3):
        for i, s in enumerate(objs):
            t0 = time.time()
            s.step()
            torch.cuda.synchronize()
            dt = time.time() - t0
            try:
                s.check_handoff()
            except RuntimeError:
                bad += 1
                print('mode %s object %d step %d: flag wait timed out (%.2f s)' % (mode, i, it, dt), flush=True)
                s.handoff_flags[4].zero_()
    print('mode %s objects %d extra streams %d: %d timed-out steps of %d; graph modes %s' % (
        mode, n, len(extra), bad, 3 * n, [s.graph_mode for s in objs]), flush=True)


if __name__ == '__main__':
    main()
