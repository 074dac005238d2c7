"""Where the compile-time shape kernels and the generic ones disagree (debugging aid, GPU): one eager step of
the bench workload in two child processes (GPI_CONV_SHAPES=1 / 0), then every workspace buffer of the
encoder and decoder programs (forward values and S / gradient buffers), the BN statistics and the flat
gradient compared bit for bit; prints each differing region with its count and largest difference.
usage: python tools/shape_diff.py"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path[:0] = [%r, %r]
import numpy as np, torch
import bench
from gpi.train import FusedElboStep
dev = torch.device('cuda', 0)
model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
Xu, Xs, Y, F = data
step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
step.step_eager()
torch.cuda.synchronize()
e = step.engine
regs = []
for tag, prog, B in (('enc', e.ep, e.B_u), ('dec', e.dp, e.B)):
    for b in prog.buffers:
        if b.external:
            continue
        regs.append((tag + ':' + b.name, b.off, B * b.per_sample))
        if b.s_off is not None:
            regs.append((tag + ':S:' + b.name, b.s_off, B * b.per_sample))
ws = e.ws.t_ws.cpu().numpy()
np.savez(sys.argv[1], ws=ws, G=step.flat.G.cpu().numpy(), P=step.flat.P.cpu().numpy(),
         names=np.array([r[0] for r in regs]), offs=np.array([[r[1], r[2]] for r in regs], dtype=np.int64))
''' % (ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))


def run(on, path):
    env = dict(os.environ, GPI_CONV_SHAPES='1' if on else '0')
    r = subprocess.run([sys.executable, '-c', CHILD, path], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    return np.load(path)


def main():
    d = tempfile.mkdtemp()
    a, b = run(True, os.path.join(d, 'on.npz')), run(False, os.path.join(d, 'off.npz'))
    for (name, (off, n)) in zip(a['names'], a['offs']):
        x, y = a['ws'][off:off + n], b['ws'][off:off + n]
        bad = np.flatnonzero(x.view(np.uint32) != y.view(np.uint32))
        if bad.size:
            print('%-45s %9d of %9d differ, first at %d, max |diff| %.3e (max |ref| %.3e)' % (
                name, bad.size, n, bad[0], np.abs(x - y).max(), np.abs(y).max()))
        else:
            print('%-45s identical' % name)
    for k in ('G', 'P'):
        bad = np.flatnonzero(a[k].view(np.uint32) != b[k].view(np.uint32))
        print('%s: %d of %d differ' % (k, bad.size, a[k].size))


if __name__ == '__main__':
    main()
