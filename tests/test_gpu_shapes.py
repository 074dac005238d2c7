"""Compile-time conv shapes on the GPU (csrc/conv_shapes.h, conv.hip fold_shape): every conv launch of the
bench step (C64, BASELINE config 2/3 per GPU) but the fused output conv runs a shape instantiation, and the
step's results are bit-identical to the generic kernels' (GPI_CONV_SHAPES=0 in a child process): folding
the geometry into constants changes the address arithmetic, never an operation on the data."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, PKG

pytestmark = pytest.mark.gpu

STEP = r'''
import sys
sys.path[:0] = [%r, %r]
import numpy as np, torch
import bench
from gpi.train import FusedElboStep
dev = torch.device('cuda', 0)
model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
Xu, Xs, Y, F = data
step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
for _ in range(2):
    step.step_eager()
torch.cuda.synchronize()
np.savez(sys.argv[1], P=step.flat.P.cpu().numpy(), G=step.flat.G.cpu().numpy())
''' % (ROOT, PKG)


def shape_info():
    from gpi import _lib as L
    info = (C.c_int64 * 4)()
    assert L.lib().gpi_conv_shape_info(info) == 0
    return list(info)


def run_step(tmp_path, name, shapes_on):
    out = str(tmp_path / name)
    env = dict(os.environ, GPI_CONV_SHAPES='1' if shapes_on else '0')
    r = subprocess.run([sys.executable, '-c', STEP, out], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(out)


def test_bench_step_launches_run_on_their_shapes(device):
    """One eager step of the bench workload: 45 conv launches (23 encoder + decoder forwards, 22 backwards
    incl. the fused output conv), every one on its compile-time shape (the fused output conv with its
    geometry folded, GPI_FUSE_FOLD)."""
    import bench
    from gpi.train import FusedElboStep
    model, data, (B_u, N_s), physics = bench.build('c64', device, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
    step.step_eager()
    torch.cuda.synchronize()
    n0 = shape_info()
    step.step_eager()
    torch.cuda.synchronize()
    n1 = shape_info()
    assert n1[0] > 0
    planned, matched = n1[1] - n0[1], n1[2] - n0[2]
    assert planned == 45 and matched == planned, (planned, matched)


def test_shape_kernels_bit_identical_to_generic(device, tmp_path):
    """Two eager steps (forward, backward, Adam) of the bench workload with the shape instantiations and
    with the generic kernels: parameters and the last gradient equal bit for bit."""
    a = run_step(tmp_path, 'on.npz', True)
    b = run_step(tmp_path, 'off.npz', False)
    for k in ('P', 'G'):
        assert a[k].shape == b[k].shape
        diff = np.flatnonzero(a[k].view(np.uint32) != b[k].view(np.uint32))
        assert diff.size == 0, (k, diff.size, np.abs(a[k] - b[k]).max())
