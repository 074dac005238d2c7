"""Throughput of the coarse-grained residual kernel (gpi_cgr_residual: CGR rows, optionally the
flux rows) against the HBM roofline, with a CPU baseline.

usage: python tools/residual_bench.py [out.json]

Per field the kernel must read log kappa [n, n], y [(n+1)(n-1)], the 4 BC values and write
r [(nc+1)^2] (+ r_flux [2 nc^2]): algorithmic bytes = 4 (n^2 + (n+1)(n-1) + 4 + (nc+1)^2 [+ 2 nc^2]).
Fields resident in HBM, HIP events on the launch stream, 20 launches averaged.
CPU baseline ("port"): the same residual per field with scipy.sparse (K assembled once per field
from kappa, K_f yhat restricted by W^T) on one host core -- the reference assembles Gamma with
FEniCS per VO sample (physics/LinearElliptic.py:137-159) and evaluates Gamma y - alpha
(VirtualObservables.py:990), which is slower still.
"""
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
import ctypes as C  # noqa: E402

PEAK = 8000.0


def launch(lk, y, bc, nc, r, rf):
    d = L.ResidualDesc()
    d.n_fine, d.nc, d.n = lk.shape[-1], nc, lk.shape[0]
    d.logkappa, d.y, d.bc, d.r = lk.data_ptr(), y.data_ptr(), bc.data_ptr(), r.data_ptr()
    d.r_flux = rf.data_ptr() if rf is not None else None
    L.check(L.lib().gpi_cgr_residual(C.byref(d), L.stream_handle()), 'cgr residual')


def cpu_port(lk, y, bc, nc, n_fields):
    """scipy.sparse restatement of one CGR residual per field (oracle-style, 1 core)."""
    from oracle import fem
    n = lk.shape[-1]
    mf = fem.unit_square_mesh(n)
    mc = fem.unit_square_mesh(nc)
    W = fem.prolongation_free(mc, mf)
    t0 = time.perf_counter()
    for f in range(n_fields):
        K, fe = fem.assemble_system(mf, np.exp(fem.image_to_cells(lk[f])), bc[f])
        _ = W.T @ (K @ y[f] - fe)
    return (time.perf_counter() - t0) / n_fields


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    dev = torch.device('cuda', 0)
    res = []
    for n, nc, N in ((64, 8, 4096), (128, 8, 1024), (256, 8, 256)):
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
            res.append(dict(grid=n, nc=nc, fields=N, flux=flux, us_per_launch=round(us, 2),
                            fields_per_s=round(N / us * 1e6), bytes_per_launch=byt, achieved_GBs=round(gbs, 1),
                            peak_GBs=PEAK, frac=round(gbs / PEAK, 4)))
            print(json.dumps(res[-1]))
        if n <= 128:
            ncpu = 8 if n == 64 else 2
            s = cpu_port(lk[:ncpu].cpu().numpy().astype(np.float64), y[:ncpu].cpu().numpy().astype(np.float64),
                         bc[:ncpu].cpu().numpy().astype(np.float64), nc, ncpu)
            res.append(dict(grid=n, cpu_port_fields_per_s=round(1.0 / s, 2), cores=1,
                            sample='%d fields, scipy.sparse assembly + K yhat + W^T (oracle.fem), 1 core' % ncpu))
            print(json.dumps(res[-1]))
    if out:
        with open(out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
