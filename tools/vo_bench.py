"""Virtual-observable update pipeline on the device vs a CPU port.

GenerativeModel.update_virtual_observables (generative.py:182-222) at the notebook's VO sizes
(example.ipynb: N_vo_max = 128, N_monte_carlo_vo = 128) on 32^2 (ROM 4x4) and 64^2 (ROM 8x8), with
CGR + flux query rows (m = (nc+1)^2 + 2 nc^2): q_X draws -> N_vo * N_mc coarse ROM solves -> MC moments
-> precision update -> batched fp64 conditioning.  Fields / BCs synthetic, parameters random-init.
CPU baseline ("port", 1 thread): the oracle's restatement of the same update (per VO sample: MC ROM
solves, torch.mean / torch.std, dense fp64 conditioning) on a bounded sample of VO samples.

usage: python tools/vo_bench.py [out.json]
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


class _DS(object):
    def __init__(self, **t):
        self.t = t
        self.N = next(iter(t.values())).shape[0]

    def __bool__(self):
        return True

    def get(self, k, random_subset=None):
        return self.t[k]


def run(ident, N_vo, N_mc, reps, dev):
    from factories.model import ModelFactory
    from bottleneck import VirtualObservables as VO
    from physics.BoundaryConditions import BoundaryCondition
    from physics.grid import pixel_to_cells
    fac = ModelFactory.FromIdentifier(ident)
    fac.set('device', 'cuda')
    torch.manual_seed(0)
    physics, model, _, encoder, _, _ = fac.setup()
    model = model.to(dev)
    n = physics['fom'].grid.n
    nc = physics['rom'].grid.n
    rng = np.random.default_rng(3)
    X = rng.normal(0.4, 0.8, (N_vo, n, n))
    U = rng.uniform(-0.5, 0.5, (N_vo, 4))
    F = np.stack([physics['rom'].grid.full_force(u) for u in U])
    QPE = VO.QuerryPointEnsemble([VO.QuerryPoint(physics['fom'], pixel_to_cells(x), BoundaryCondition(u))
                                  for x, u in zip(X, U)])
    QE = VO.QuerryEnsemble.FromQuerryPointEnsemble(QPE, physics, True, True, 0, 0, dtype=torch.float32, device=dev)
    ens = VO.VirtualObservablesEnsemble(QPE, QE, dtype=torch.float32, device=dev)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    model.register_datasets({'vo': _DS(X=t(X), Y=t(np.zeros((N_vo, (n + 1) * (n - 1)))), F_ROM_BC=t(F))}, ens)
    times, post = {}, {}
    for mode in ('dense', 'sparse'):            # same updates (same seeds) through both conditioning paths
        ens.sparse = mode == 'sparse'
        torch.manual_seed(1)
        model.update_virtual_observables(N_mc, step=0)
        model.update_virtual_observables(N_mc, step=1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(reps):
            model.update_virtual_observables(N_mc, step=it + 2)
        torch.cuda.synchronize()
        times[mode] = (time.perf_counter() - t0) / reps
        torch.manual_seed(2)
        model.update_virtual_observables(N_mc, step=reps + 2)
        post[mode] = (ens._mean64.clone(), ens._vars64.clone())
    dm = ((post['dense'][0] - post['sparse'][0]).abs().max() / post['dense'][0].abs().max()).item()
    dv = ((post['dense'][1] - post['sparse'][1]).abs().max() / post['dense'][1].abs().max()).item()
    dt = times['sparse']
    m = int(ens._QuerryEnsemble.gamma.shape[1])
    return dict(grid=n, nc=nc, N_vo=N_vo, N_mc=N_mc, m=m, ms_per_update=round(dt * 1e3, 3),
                vo_samples_per_s=round(N_vo / dt, 1), conditioning='column-sparse (SparsePlan r=%d)'
                % ens._plan.r, ms_per_update_dense=round(times['dense'] * 1e3, 3),
                sparse_vs_dense_rel_diff=dict(mean=dm, vars=dv)), (model, ens, X, U, F, physics)


def cpu_port(state, N_vo_cpu, N_mc):
    """oracle restatement, per VO sample (the reference's loop structure), 1 thread."""
    from oracle import elbo as oelbo, fem
    model, ens, X, U, F, physics = state
    torch.set_num_threads(1)
    nc = physics['rom'].grid.n
    n = physics['fom'].grid.n
    mc, mf = fem.unit_square_mesh(nc), fem.unit_square_mesh(n)
    M = torch.tensor(fem.rom_stiffness_tensor(mc))
    W = torch.tensor(fem.prolongation_free(mc, mf))
    bc = torch.tensor(fem.dirichlet_split(mc)[0])
    G = ens._QuerryEnsemble.gamma[:N_vo_cpu].cpu()
    A = ens._QuerryEnsemble.alpha[:N_vo_cpu].cpu()
    qx = model.q_X['vo']
    mu, ls = qx.mean.detach().cpu().double()[:N_vo_cpu], qx.logsigma.detach().cpu().double()[:N_vo_cpu]
    lsy = model.g.logsigmas_y.detach().cpu().double()
    Fd = torch.tensor(F[:N_vo_cpu])
    vo_var = torch.ones(G.shape[1], dtype=torch.float64)
    g = torch.Generator().manual_seed(0)
    t0 = time.perf_counter()
    ex = torch.randn(N_vo_cpu, N_mc, mu.shape[1], generator=g, dtype=torch.float64)
    ey = torch.randn(N_vo_cpu, N_mc, W.shape[0], generator=g, dtype=torch.float64)
    Ym, Ys = oelbo.vo_predictive(W, M, bc, mu, ls, Fd, lsy, ex, ey)
    for i in range(N_vo_cpu):
        oelbo.vo_condition(G[i], A[i], Ym[i], 1 / Ys[i] ** 2, vo_var)
    return (time.perf_counter() - t0) / N_vo_cpu


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    dev = torch.device('cuda', 0)
    res = []
    for ident, ncpu in (('highres32', 8), ('highres', 2)):
        r, state = run(ident, 128, 128, 10, dev)
        s = cpu_port(state, ncpu, 128)
        r.update(cpu_port_vo_samples_per_s=round(1.0 / s, 2), cpu_cores=1,
                 cpu_sample='%d VO samples x 128 MC (oracle restatement, fp64)' % ncpu,
                 speedup=round(r['vo_samples_per_s'] * s, 1))
        res.append(r)
        print(json.dumps(r))
    if out:
        with open(out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
