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


def _define(name):
    for line in open(SHAPES_H):
        if line.startswith('#define ' + name + ' '):
            return line.split(None, 2)[2].strip()
    return None


def test_shape_parts_and_nofold_list_are_consistent():
    """The table's parts (one object of conv.hip each, GPI_CONV_SHAPE_PART) cover it in order, and the entries
    left to the generic kernels (GPI_CONV_SHAPE_NOFOLD) are entries of it."""
    n = int(_define('GPI_CONV_SHAPE_COUNT'))
    bounds = [int(v) for v in _define('GPI_CONV_SHAPE_BOUNDS').strip('{}').split(',')]
    assert len(bounds) == 5 and bounds[0] == 0 and bounds[-1] == n
    assert all(a <= b for a, b in zip(bounds, bounds[1:]))
    nofold = [int(v) for v in _define('GPI_CONV_SHAPE_NOFOLD').strip('{}').split(',')]
    assert all(v == -1 or 0 <= v < n for v in nofold)


def test_no_shape_instantiation_spills():
    """Every compile-time shape instantiation in the built objects fits its occupancy target without spilling
    (a regenerated table can move an entry that spills out of GPI_CONV_SHAPE_NOFOLD's list: this catches it).
    Needs the built objects (csrc/build/conv*.o); skipped without them."""
    import glob
    import pytest
    objs = sorted(glob.glob(os.path.join(PKG, 'csrc', 'build', 'conv*.o')))
    if not objs:
        pytest.skip('conv objects not built here')
    tool = os.path.join(ROOT, 'tools', 'kernel_resources.sh')
    bad = []
    for o in objs:
        r = subprocess.run(['bash', tool, o, 'conv_'], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-1000:]
        for line in r.stdout.splitlines():
            name, f = line.split()[0], line.split()
            # shape instantiations carry a non-negative last template argument (ELi<n>EE); -1 prints as Lin1
            if 'Lin1EE' not in name and int(f[f.index('spill') + 1]) > 0:
                bad.append(line)
    assert not bad, bad
