"""Run the coarse-grained residual kernel alone (for rocprofv3 counter passes): n^2 grid, N fields,
flux rows on/off, `reps` launches.  usage: python tools/cgr_probe.py [n] [N] [flux 0/1] [reps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd')]
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    flux = len(sys.argv) > 3 and sys.argv[3] == '1'
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    nc = 8
    dev = torch.device('cuda', 0)
    g = torch.Generator(device='cpu').manual_seed(n)
    lk = (0.8 * torch.randn(N, n, n, generator=g)).to(dev)
    y = torch.randn(N, (n + 1) * (n - 1), generator=g).to(dev)
    bc = (torch.rand(N, 4, generator=g) - 0.5).to(dev)
    r = torch.empty(N, (nc + 1) ** 2, device=dev)
    rf = torch.empty(N, 2 * nc * nc, device=dev) if flux else None
    d = L.ResidualDesc(n_fine=n, nc=nc, n=N, logkappa=lk.data_ptr(), y=y.data_ptr(), bc=bc.data_ptr(),
                       r=r.data_ptr(), r_flux=rf.data_ptr() if flux else None)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    L.check(L.lib().gpi_cgr_residual(C.byref(d), L.stream_handle()), 'residual')
    t0.record()
    for _ in range(reps):
        L.check(L.lib().gpi_cgr_residual(C.byref(d), L.stream_handle()), 'residual')
    t1.record()
    torch.cuda.synchronize()
    print('cgr n=%d N=%d flux=%d: %.2f us/launch' % (n, N, flux, 1e3 * t0.elapsed_time(t1) / reps))


if __name__ == '__main__':
    main()
