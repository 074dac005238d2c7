"""Measurement of the FOM data-generation row on the GPU.

For each grid: draw N log-conductivity images with the device random-field sampler
(gpi_random_field), map them to DG0 cells, and solve the N FOM problems with one batched
gpi_fom_solve launch; HIP events on the launch stream time both.  The CPU baseline is the
host path the GPU one replaces (per-sample scipy sparse LU on the same stencil system,
DataLoader.assemble without device) on a bounded sample of the same fields.
Prints one JSON line per grid.

  python tools/fom_bench.py [--grids 64,128,256] [--out profiles/r01_fom_bench.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))

from gpi import fom                                     # noqa: E402
from physics.RandomField import NormalRandomFieldSampler  # noqa: E402
from physics.grid import StructuredGrid                 # noqa: E402

# grid -> (labelled samples solved, images drawn, correlation length, truncation)
CASES = {32: (1024, 20480, 0.15, None), 64: (2048, 20480, 0.04, 'adaptive'), 128: (512, 4096, 0.04, 'adaptive'),
         256: (128, 1024, 0.04, 'adaptive')}
HBM_PEAK = 8000.0   # GB/s (MI355X_MICROARCH.md)


def pixels_to_cells(X):
    """[N, n, n] images -> [N, 2 n^2] DG0 cells (physics/grid.py pixel_to_cells, on the device)."""
    sq = torch.flip(X, dims=[1]).reshape(X.shape[0], -1)
    return sq.repeat_interleave(2, dim=1).contiguous()


def timed(fn):
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    out = fn()
    b.record(st)
    torch.cuda.synchronize()
    return out, a.elapsed_time(b) * 1e-3


def run(n, cpu_sample):
    N, N_img, l, trunc = CASES[n]
    s = NormalRandomFieldSampler.FromImage(n, n, 0.4, 0.8, l, Truncation=trunc)
    s.sample_device(4, seed=1)                           # factors to the device, warm-up
    X, t_rf = timed(lambda: s.sample_device(N_img, seed=2))
    xd = pixels_to_cells(X[:N])
    rng = np.random.default_rng(n)
    U = rng.uniform(-0.5, 0.5, (N, 4))
    bc = torch.tensor(U, dtype=torch.float64, device='cuda')
    fom.fom_solve(xd[:8], bc[:8], n).check()             # warm-up
    res, t_fom = timed(lambda: fom.fom_solve(xd, bc, n))
    res.check()
    iters = res.iters.cpu().numpy()
    dy = (n + 1) * (n - 1)
    mg_min = int(os.environ.get('GPI_FOM_MG_MIN', '64'))
    mg = mg_min > 0 and n >= mg_min and n & (n - 1) == 0 and n >= 8
    # algorithmic bytes per fine node and iteration.  Jacobi-PCG: update pass reads u w p s x r dinv,
    # writes p s x r u; stencil pass reads u r + 2 conductances, writes w -> 17 doubles.  Multigrid-PCG
    # (fine level; the coarse levels add ~1/3): A p 4, x / r update 6, four red-black half sweeps 16,
    # residual 5, restriction 1, prolongation 2.5, (r, z) 2, p update 3 -> 40 doubles
    bpn = 320 if mg else 136
    bytes_alg = bpn * dy * float(iters.sum())
    cpu = None
    err = None
    if cpu_sample > 0:
        # CPU baseline: per-sample scipy sparse LU of the same system on a bounded sample
        g = StructuredGrid(n)
        xh = xd[:cpu_sample].cpu().numpy()
        t0 = time.perf_counter()
        Yh = np.stack([g.solve(np.exp(xh[k]), U[k]) for k in range(cpu_sample)])
        t_cpu = time.perf_counter() - t0
        err = float(np.abs(res.y[:cpu_sample].cpu().numpy() - Yh).max())
        cpu = {'value': cpu_sample / t_cpu, 'unit': 'samples/s', 'cores': 1, 'kind': 'port',
               'sample': '%d samples, scipy spsolve on the stencil system (host path)' % cpu_sample}
    return {
        'metric': 'FOM labels solved per second (%dx%d)' % (n, n), 'value': N / t_fom, 'unit': 'samples/s',
        'n_samples': N, 'ms': t_fom * 1e3, 'iters_mean': float(iters.mean()), 'iters_max': int(iters.max()),
        'dtype': 'f64', 'data': 'synthetic (device random field, l=%g, truncation %s)' % (l, trunc),
        'random_field': {'images': N_img, 'ms': t_rf * 1e3, 'images_per_s': N_img / t_rf},
        'solver': 'multigrid-preconditioned CG (V(1,1), red-black GS)' if mg else 'Jacobi-preconditioned CG',
        'roofline': {'bound': 'hbm', 'achieved': bytes_alg / t_fom / 1e9, 'peak': HBM_PEAK, 'unit': 'GB/s',
                     'frac': bytes_alg / t_fom / 1e9 / HBM_PEAK, 'bytes_per_node_iter': bpn},
        'cpu_baseline': cpu,
        'max_abs_diff_vs_cpu': err,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--grids', default='32,64,128,256')
    ap.add_argument('--cpu-sample', type=int, default=16)
    ap.add_argument('--out', default=None)
    ap.add_argument('--no-cpu', action='store_true')
    a = ap.parse_args()
    if a.no_cpu:
        a.cpu_sample = 0
    lines = []
    for n in [int(v) for v in a.grids.split(',')]:
        r = run(n, a.cpu_sample if n <= 128 or a.cpu_sample == 0 else max(2, a.cpu_sample // 8))
        print(json.dumps(r), flush=True)
        lines.append(json.dumps(r))
    if a.out:
        with open(a.out, 'w') as f:
            f.write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main()
