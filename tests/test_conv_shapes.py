"""Compile-time conv shapes without a GPU (csrc/conv_shapes.h, conv.hip fold_shape): the committed table is
exactly what tools/gen_conv_shapes.py plans from the engine's C64 program layouts today -- a stale table
would only send launches back to the generic kernels, silently -- and the host planner answers without a
device.  The GPU side (every launch of the bench step on its shape, bit-identical results) is
tests/test_gpu_shapes.py."""
import ctypes as C
import os
import subprocess
import sys

from conftest import ROOT, PKG

SHAPES_H = os.path.join(PKG, 'csrc', 'conv_shapes.h')


def test_committed_shape_table_is_current(tmp_path):
    out = str(tmp_path / 'conv_shapes.h')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'gen_conv_shapes.py'), '--out', out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert open(out).read() == open(SHAPES_H).read(), 'conv_shapes.h is stale: rerun tools/gen_conv_shapes.py'


def test_shape_table_entries_are_distinct():
    rows = [l.strip().rstrip('\\').strip().rstrip(',') for l in open(SHAPES_H) if l.strip().startswith('{')]
    n = int(next(l.split()[2] for l in open(SHAPES_H) if l.startswith('#define GPI_CONV_SHAPE_COUNT')))
    assert n == len(rows) > 0
    assert len(set(rows)) == len(rows)


def test_shape_info_counts_without_device():
    from gpi import _lib as L
    info = (C.c_int64 * 4)()
    assert L.lib().gpi_conv_shape_info(info) == 0
    assert info[0] == len([l for l in open(SHAPES_H) if l.strip().startswith('{')])
