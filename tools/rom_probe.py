"""Time the ELBO step's ROM launch (gpi_rom, LOGLIK mode, the C64 labeled batch) in isolation,
and the whole fused step, with HIP events on the launch stream.

usage: [GPI_LIB_VARIANT=nt64] python tools/rom_probe.py [reps]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def timed(fn, reps):
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    lib, st = L.lib(), L.stream_handle()
    rom_us = timed(lambda: L.check(lib.gpi_rom(C.byref(e.rom), st), 'rom'), reps)
    fwd = L.RomDesc.from_buffer_copy(e.rom)
    fwd.mode, fwd.mu_y = L.ROM_FORWARD, None
    uc = torch.empty(fwd.n, (fwd.nc + 1) ** 2, dtype=torch.float32, device=dev)
    fwd.uc = uc.data_ptr()
    solve_us = timed(lambda: L.check(lib.gpi_rom(C.byref(fwd), st), 'rom fwd'), reps)
    print('rom coarse solve only (FORWARD, no prolongation): %.1f us' % solve_us)
    if os.environ.get('GPI_LIB_VARIANT') == 'timing':
        import numpy as np
        f = lib.gpi_debug_rom_stamps
        f.restype, f.argtypes = C.c_int, [C.c_void_p]
        ph = np.zeros((256, 8), np.uint64)
        L.check(f(ph.ctypes.data), 'stamps')          # clear
        L.check(lib.gpi_rom(C.byref(e.rom), st), 'rom')
        torch.cuda.synchronize()
        L.check(f(ph.ctypes.data), 'stamps')
        p = ph[:e.rom.n][:, [0, 1, 6, 2, 7, 3, 4, 5]].astype(np.int64)
        names = ['load+assemble', 'cholesky', 'solves', 'prolong+loglik', 'loss sum', 'adjoint', 'dJ/dx']
        dd = np.diff(p, axis=1).mean(0)
        print('rom_kernel phases (cycles, mean over %d workgroups): %s; total %.0f' % (
            e.rom.n, ', '.join('%s %.0f' % (n, v) for n, v in zip(names, dd)), (p[:, 7] - p[:, 0]).mean()))
    step.capture()
    step_us = timed(step.step, reps)
    print('variant %s: rom %.1f us, step %.1f us (%.0f samples/s)' % (
        os.environ.get('GPI_LIB_VARIANT', 'default'), rom_us, step_us, (B_u + N_s) / step_us * 1e6))


if __name__ == '__main__':
    main()
