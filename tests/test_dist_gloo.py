"""Data-parallel path on CPU: two gloo ranks.

The native step's only cross-rank exchange is gpi.train.allreduce_shared: one
SUM all-reduce of the shared-parameter prefix of the flat gradient, with the
per-sample variational rows rank-owned.  These tests run that exchange over a
real process group (gloo, world_size 2, 127.0.0.1) on models built exactly as
bench.py builds them on every rank, and check the sum convention against the
oracle: the ELBO is a sum over samples, so the summed per-rank gradients of
the shared parameters equal the gradient over the union batch.
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, port):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)


def _build_model():
    from factories.model import ModelFactory
    fac = ModelFactory.FromIdentifier('highres32')
    fac.set('device', 'cpu')
    torch.manual_seed(0)                       # bench.py: identical shared parameters on every rank
    physics, model, _, encoder, _, _ = fac.setup()
    model.encoder = encoder
    N_s = 4

    class _T(object):
        def __init__(self, **t):
            self.t = t
            self.N = next(iter(t.values())).shape[0]

        def __bool__(self):
            return True

        def get(self, k, random_subset=None):
            return self.t[k]

    n = physics['fom'].grid.n
    X = torch.zeros(N_s, n, n)
    model.register_datasets({'supervised': _T(X=X, Y=torch.zeros(N_s, (n + 1) * (n - 1)),
                                              F_ROM_BC=torch.zeros(N_s, physics['rom'].grid.num_nodes)),
                             'unsupervised': _T(X=torch.zeros(8, n, n))}, None,
                            create_unsupervised_variational_approximation=False)
    return model


def _worker_allreduce(rank, port, q):
    try:
        _init(rank, port)
        from gpi.train import allreduce_shared
        model = _build_model()
        flat = model.native_flat()
        P0 = flat.P.clone()
        g = torch.Generator().manual_seed(100 + rank)
        G = torch.randn(flat.numel, generator=g)
        flat.G.copy_(G)
        allreduce_shared(flat)
        out = dict(rank=rank, n_shared=flat.n_shared, numel=flat.numel, P_shared=P0[:flat.n_shared].clone(),
                   G=flat.G.clone(), G_in=G, names=list(flat.names))
        q.put(out)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        q.put(dict(rank=rank, error=repr(e)))


def _run(fn):
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=fn, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert 'error' not in r, r
    return sorted(res, key=lambda r: r['rank'])


def test_allreduce_shared_prefix_sum_and_local_rows():
    a, b = _run(_worker_allreduce)
    n = a['n_shared']
    assert n == b['n_shared'] and 0 < n < a['numel'], 'shared prefix must exclude the per-sample q rows'
    # shared parameters come first and are identical on both ranks (seeded construction)
    shared_names = [x for x in a['names'] if x.startswith(('f.', 'g.', 'gp.', 'encoder.'))]
    assert a['names'][:len(shared_names)] == shared_names
    assert torch.equal(a['P_shared'], b['P_shared'])
    # SUM over ranks on the shared prefix, bit-identical on both ranks
    expect = a['G_in'][:n] + b['G_in'][:n]
    assert torch.allclose(a['G'][:n], expect, rtol=1e-6, atol=1e-6)
    assert torch.equal(a['G'][:n], b['G'][:n])
    # rank-owned rows (q_z / q_X of this rank's labeled samples) untouched
    assert torch.equal(a['G'][n:], a['G_in'][n:])
    assert torch.equal(b['G'][n:], b['G_in'][n:])


def _worker_sum_convention(rank, port, q):
    """Each rank takes half of a labeled batch through the oracle ROM likelihood;
    the all-reduced shared gradient must equal the union-batch gradient."""
    try:
        _init(rank, port)
        from oracle import elbo as oelbo
        from oracle import fem
        torch.manual_seed(7)
        nc = 4
        coarse, fine = fem.unit_square_mesh(nc), fem.unit_square_mesh(4 * nc)
        M = torch.tensor(fem.rom_stiffness_tensor(coarse), dtype=torch.float64)
        W = torch.tensor(fem.prolongation_free(coarse, fine), dtype=torch.float64)
        bc = torch.tensor(fem.dirichlet_split(coarse)[0])
        N, nT = 8, 2 * nc * nc
        X = torch.randn(N, nT, dtype=torch.float64) * 0.3
        F = torch.zeros(N, (nc + 1) ** 2, dtype=torch.float64)
        F[:, bc] = torch.rand(N, len(bc), dtype=torch.float64) - 0.5
        Y = torch.randn(N, W.shape[0], dtype=torch.float64) * 0.1
        ls = torch.full((W.shape[0],), 0.3, dtype=torch.float64, requires_grad=True)

        def loss(rows):
            mu, lsy = oelbo.rom_operator(W, M, bc, X[rows], F[rows], ls)
            return -oelbo.dgll(Y[rows], mu, 2 * lsy)

        lo, hi = rank * N // WORLD, (rank + 1) * N // WORLD
        g_local, = torch.autograd.grad(loss(slice(lo, hi)), ls)
        g_sum = g_local.clone()
        dist.all_reduce(g_sum, op=dist.ReduceOp.SUM)
        g_union, = torch.autograd.grad(loss(slice(0, N)), ls)
        q.put(dict(rank=rank, err=float((g_sum - g_union).abs().max()), scale=float(g_union.abs().max())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put(dict(rank=rank, error=repr(e)))


def test_sum_allreduce_equals_union_batch_gradient():
    for r in _run(_worker_sum_convention):
        assert r['err'] <= 1e-12 * max(1.0, r['scale']), r
