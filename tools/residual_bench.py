"""Throughput of the coarse-grained residual kernel (gpi_cgr_residual: CGR rows, optionally the flux rows
fused into the same pass) against the HBM roofline, with a CPU baseline -- the measured line for the
fixed-stencil residual that north_star names.

usage: python tools/residual_bench.py [out.json] [--quick] [--no-cpu]

Per field the kernel must read log kappa [n, n], y [(n+1)(n-1)], the 4 BC values and write
r [(nc+1)^2] (+ r_flux [2 nc^2]): algorithmic bytes = 4 (n^2 + (n+1)(n-1) + 4 + (nc+1)^2 [+ 2 nc^2]).
Fields resident in HBM, HIP events on the launch stream, 20 launches averaged (after one warm launch).
`traffic`: HBM bytes per launch from the PMC passes of tools/r05_residual_pmc.sh (FETCH_SIZE / WRITE_SIZE,
(2 FETCH + WRITE) x 1 KiB on gfx950), taken from profiles/*residual_traffic*.json only when the sha1 of
csrc/stencil.hip + csrc/common.h recorded there is the current one (else null).
CPU baseline ("port", oracle.fem): the reference path per field -- FE assembly of K from kappa plus the residual
W^T (K yhat - f), scipy.sparse -- on 16 single-threaded host processes (the step baseline's 16 cores), a bounded
sample of fields -- the reference assembles Gamma
with FEniCS per VO sample (physics/LinearElliptic.py:137-159) and evaluates Gamma y - alpha
(VirtualObservables.py:990), which is slower still.
"""
import ctypes as C
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402

PEAK = 8000.0          # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)
CONFIGS = ((64, 8, 4096), (128, 8, 1024), (256, 8, 256))


def stencil_sha():
    h = hashlib.sha1()
    for f in ('stencil.hip', 'common.h'):
        with open(os.path.join(ROOT, 'generative-physics-informed-pde_amd', 'csrc', f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


def traffic_entries():
    """{(grid, flux): traffic bytes per launch} from the newest sha-matched traffic file in profiles/."""
    sha = stencil_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*residual_traffic*.json')), reverse=True):
        try:
            t = json.load(open(f))
        except ValueError:
            continue
        if t.get('stencil_sha1') == sha:
            return {(e['grid'], e['flux']): e for e in t['entries']}, os.path.basename(f)
    return {}, None


def launch(lk, y, bc, nc, r, rf):
    d = L.ResidualDesc()
    d.n_fine, d.nc, d.n = lk.shape[-1], nc, lk.shape[0]
    d.logkappa, d.y, d.bc, d.r = lk.data_ptr(), y.data_ptr(), bc.data_ptr(), r.data_ptr()
    d.r_flux = rf.data_ptr() if rf is not None else None
    L.check(L.lib().gpi_cgr_residual(C.byref(d), L.stream_handle()), 'cgr residual')


_W = {}


def _cpu_init(n, nc):
    os.environ['OMP_NUM_THREADS'] = '1'
    from oracle import fem
    mf = fem.unit_square_mesh(n)
    _W['mf'], _W['W'] = mf, fem.prolongation_free(fem.unit_square_mesh(nc), mf)


def _cpu_fields(args):
    """CGR residuals of a chunk of fields in one worker (oracle.fem, scipy.sparse, one thread)."""
    from oracle import fem
    lk, y, bc = args
    mf, W = _W['mf'], _W['W']
    for f in range(lk.shape[0]):
        K, fe = fem.assemble_system(mf, np.exp(fem.image_to_cells(lk[f])), bc[f])
        _ = W.T @ (K @ y[f] - fe)
    return lk.shape[0]


def cpu_port(lk, y, bc, nc, workers):
    """The reference path per field -- FE assembly of K from kappa, then W^T (K yhat - f) (oracle.fem restates
    LinearElliptic.py:137-159 + VirtualObservables.py:990 with scipy.sparse) -- over `workers` host processes
    of one thread each, the fields split evenly; fields per second of wall time (pool warmed first)."""
    import concurrent.futures as cf
    import multiprocessing as mp
    n = lk.shape[-1]
    chunks = [(lk[i::workers], y[i::workers], bc[i::workers]) for i in range(workers)]
    with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context('spawn'), initializer=_cpu_init,
                                initargs=(n, nc)) as ex:
        list(ex.map(_cpu_fields, [(c[0][:1], c[1][:1], c[2][:1]) for c in chunks]))      # warm every worker
        t0 = time.perf_counter()
        done = sum(ex.map(_cpu_fields, chunks))
        return done / (time.perf_counter() - t0)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    out = args[0] if args else None
    quick = '--quick' in sys.argv
    dev = torch.device('cuda', 0)
    tr, tr_file = traffic_entries()
    res = []
    samples = {}
    for n, nc, N in CONFIGS:
        g = torch.Generator(device='cpu').manual_seed(n)
        lk = (0.8 * torch.randn(N, n, n, generator=g)).to(dev)
        y = torch.randn(N, (n + 1) * (n - 1), generator=g).to(dev)
        bc = (torch.rand(N, 4, generator=g) - 0.5).to(dev)
        r = torch.empty(N, (nc + 1) ** 2, device=dev)
        rf = torch.empty(N, 2 * nc * nc, device=dev)
        for flux in (False, True):
            launch(lk, y, bc, nc, r, rf if flux else None)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(20):
                launch(lk, y, bc, nc, r, rf if flux else None)
            t1.record()
            torch.cuda.synchronize()
            us = t0.elapsed_time(t1) * 1e3 / 20
            byt = 4.0 * N * (n * n + (n + 1) * (n - 1) + 4 + (nc + 1) ** 2 + (2 * nc * nc if flux else 0))
            gbs = byt / us / 1e3
            te = tr.get((n, flux))
            line = dict(metric='coarse-grained residual fields/sec (%d^2 grid, nc %d%s)' % (n, nc, ', + flux rows'
                                                                                        if flux else ''),
                        value=round(N / us * 1e6), unit='fields/s', higher_is_better=True,
                        grid=n, nc=nc, fields=N, flux=flux, us_per_launch=round(us, 2), dtype='f32',
                        data='synthetic', roofline=dict(bound='hbm', achieved=round(gbs, 1), peak=PEAK,
                                                        unit='GB/s', frac=round(gbs / PEAK, 4),
                                                        algorithmic_bytes=byt,
                                                        traffic=round(te['traffic_bytes']) if te else None,
                                                        traffic_file=tr_file if te else None),
                        cpu_baseline=None)
            res.append(line)
        if n <= 128:
            samples[n] = (lk[:512].cpu().numpy().astype(np.float64), y[:512].cpu().numpy().astype(np.float64),
                          bc[:512].cpu().numpy().astype(np.float64), nc)
    # CPU baselines after every GPU measurement (the worker pool stays off the host while kernels are timed)
    for n, (lk, y, bc, nc) in samples.items():
        if '--no-cpu' in sys.argv:
            continue
        # the same 16 host cores as the step's CPU baseline (bench.py), one single-threaded process each
        workers = 16
        ncpu = workers * ((2 if quick else 24) if n == 64 else (1 if quick else 3))
        fps = cpu_port(lk[:ncpu], y[:ncpu], bc[:ncpu], nc, workers)
        cpu = dict(value=round(fps, 2), unit='fields/s', cores=workers, kind='port',
                   sample='%d fields of the %d^2 batch, reference-path FE assembly + residual W^T (K yhat - f) '
                          '(oracle.fem, scipy.sparse), %d single-threaded host processes' % (ncpu, n, workers))
        for line in res:
            if line['grid'] == n:
                line['cpu_baseline'] = cpu
    for line in res:
        print(json.dumps(line), flush=True)
    if out:
        with open(out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
