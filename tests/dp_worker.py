"""One rank of the data-parallel native step on a shared GPU (gloo process group): launched by
tests/test_gpu_dist.py through torch.distributed.run with 2 ranks.  Test infrastructure.

Each rank runs the NATIVE FusedElboStep on its shard of the elbo_c32 fixture: the unlabeled
pool is shared, every rank draws the same global permutation (shared subset seed) and takes
its B_u-slice; labeled samples (and their q_z / q_X rows) are split by index.  The rank
records the inputs it drew, its local gradient, the all-reduced gradient and the parameters
after one Adam update into <out>/rank<r>.npz."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B_U = 4          # per rank (global 8 of the fixture's pool of 16)
NS_RANK = 2      # labeled samples per rank (fixture: 4)
# BASELINE config 3's per-rank shape (C64 highres, droprate 0.2): B_u = 256 unlabeled of a shared pool of
# 1024 per rank + N_s = 32 rank-owned labeled samples
C64_BU, C64_NS, C64_POOL = 256, 32, 1024


def c64_data(world, rank):
    """Synthetic config-3 inputs: the shared unlabeled pool (same on every rank) and rank `rank`'s
    labeled fields, targets and ROM boundary forces (tests/test_gpu_dist.py regenerates them)."""
    n, nc = 64, 8
    rng = np.random.default_rng(7)
    Xu = rng.normal(0.3, 0.6, (C64_POOL * world, n, n)).astype(np.float32)
    rr = np.random.default_rng(100 + rank)
    Xs = rr.normal(0.3, 0.6, (C64_NS, n, n)).astype(np.float32)
    Y = rr.normal(0.0, 0.3, (C64_NS, (n + 1) * (n - 1))).astype(np.float32)
    F = np.zeros((C64_NS, (nc + 1) ** 2), dtype=np.float32)
    bnodes = [e for e in range((nc + 1) ** 2) if e % (nc + 1) in (0, nc)]
    F[:, bnodes] = rr.uniform(-0.5, 0.5, (C64_NS, len(bnodes)))
    return Xu, Xs, Y, F


def c64_model(world, rank):
    """The config-3 model (highres factory: C64 codec, Dropout2d 0.2, ROM 8x8; torch.manual_seed(0), so the
    shared parameters and q rows are identical on every rank) with rank `rank`'s datasets registered, and
    the step's device inputs (X_pool, X_s, Y, F)."""
    from factories.model import ModelFactory
    from test_gpu_c64 import _DS
    torch.manual_seed(0)
    fac = ModelFactory.FromIdentifier('highres')
    fac.set('device', 'cuda')
    physics_, model, _, encoder, _, _ = fac.setup()
    model.encoder = encoder.cuda()
    Xu, Xs, Y, F = c64_data(world, rank)
    cu = lambda a: torch.tensor(a, device='cuda')
    model.register_datasets({'supervised': _DS(X=cu(Xs), Y=cu(Y), F_ROM_BC=cu(F)),
                             'unsupervised': _DS(perm=None, X=cu(Xu))}, None,
                            create_unsupervised_variational_approximation=False)
    model.cuda()
    return model, (cu(Xu), cu(Xs), cu(Y), cu(F))


def run_c64_sync(out):
    """One SyncBN step of the NATIVE FusedElboStep at config 3's per-rank shape; records the inputs it
    drew, the kernels' ReLU decisions (for the fp64 union-batch oracle), the local and all-reduced
    gradients and the ELBO."""
    import ctypes as C
    from gpi.train import FusedElboStep
    from gpi import _lib as L
    from gpu_masks import engine_relu_masks
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('gloo')
    model, (Xu, Xs, Y, F) = c64_model(world, rank)
    step = FusedElboStep(model, Xu, C64_BU, Xs, Y, F, lr=1e-3, seed=50 + rank, subset_seed=9,
                         distributed=True, rank=rank, world=world, sync_bn=True)
    assert step.sync_bn and step.engine.bn_sync is not None
    e = step.engine
    rec = dict(idx=step.idx.cpu().numpy(), eps_z=e.eps_z().cpu().numpy(), eps_x=e.eps_x().cpu().numpy(),
               P0=step.flat.P.cpu().numpy())
    for key, dd in e.dropout_views().items():
        for nm, v in dd.items():
            rec['drop.%s.%s' % (key, nm)] = v.cpu().numpy()
    step._forward_backward(epilogue=False)
    masks = engine_relu_masks(e)            # before the epilogue clears the statistics
    for call, mm in masks.items():
        for nm, m in mm.items():
            rec['mask.%s.%s' % (call, nm)] = m.numpy()
    L.check(L.lib().gpi_step_epilogue(C.byref(step.epi), L.stream_handle()), 'step epilogue')
    torch.cuda.synchronize()
    rec['G_local'] = step.flat.G.cpu().numpy()
    step.allreduce()
    torch.cuda.synchronize()
    rec['G_red'] = step.flat.G.cpu().numpy()
    rec['n_shared'] = np.int64(step.flat.n_shared)
    rec['elbo'] = np.float64(step.elbo().item())
    names = [k for k, _ in model.named_parameters()]
    rec['names'] = np.array(names)
    rec['offsets'] = np.array([step.flat.name_offsets[k] for k in names])
    for k, p in model.named_parameters():
        rec['shape.' + k] = np.array(p.shape, dtype=np.int64)
    rec['counts'] = np.array(e.bn_global_counts['dec'] + [e.bn_global_counts['enc']])
    np.savez(os.path.join(out, 'rank%d.npz' % rank), **rec)
    dist.barrier()
    dist.destroy_process_group()


# labeled samples per rank of the 'sync_uneven' mode (the fixture's 4 split unevenly: the SyncBN
# statistics of the labeled decoder group then have per-rank counts 1 and 3)
NS_UNEVEN = (1, 3)


def shard_model(d, rank, B_u=B_U, ns=NS_RANK, lo=None):
    """The fixture model restricted to rank's labeled shard [lo, lo + ns) (default lo = rank * ns; state rows
    sliced accordingly)."""
    from test_gpu_parity import build_golden_model
    lo = rank * ns if lo is None else lo
    sl = slice(lo, lo + ns)
    e = dict(d)
    for k in ('Xs', 'Y', 'F'):
        e[k] = d[k][sl]
    for k in list(e):
        if k.startswith(('state.q_z.supervised', 'state.q_X.supervised')):
            e[k] = d[k][sl]
    e['cfg'] = np.array([int(d['cfg'][0]), int(d['cfg'][1]), int(d['cfg'][2]), int(d['cfg'][3]), B_u, ns])
    return build_golden_model(e)


def main(out, mode='replica'):
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    sync_bn = mode in ('sync', 'sync_uneven')    # SyncBN: BN statistics over both ranks' batches (eager: gloo)
    torch.cuda.set_device(0)                      # every rank on the one GPU of the box
    dist.init_process_group('gloo')
    from elbo_ref import load
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    if mode == 'sync_uneven':
        model, _ = shard_model(d, rank, ns=NS_UNEVEN[rank], lo=sum(NS_UNEVEN[:rank]))
    else:
        model, _ = shard_model(d, rank)
    ds = model._datasets['supervised']
    Xu = torch.tensor(d['Xu'], device='cuda')
    try:        # world > 1 without a shared subset seed: refused (ranks would draw different permutations)
        FusedElboStep(model, Xu, B_U, ds.get('X'), ds.get('Y'), ds.get('F_ROM_BC'), seed=50 + rank,
                      distributed=True, rank=rank, world=world)
        raise AssertionError('FusedElboStep accepted world > 1 without subset_seed')
    except ValueError:
        pass
    step = FusedElboStep(model, Xu, B_U, ds.get('X'), ds.get('Y'), ds.get('F_ROM_BC'), lr=1e-3, seed=50 + rank,
                         subset_seed=9, distributed=True, rank=rank, world=world, sync_bn=sync_bn)
    assert step.sync_bn == sync_bn
    e = step.engine
    rec = dict(idx=step.idx.cpu().numpy(), eps_z=e.eps_z().cpu().numpy(), eps_x=e.eps_x().cpu().numpy(),
               P0=step.flat.P.cpu().numpy())
    step.forward_backward()
    torch.cuda.synchronize()
    rec['G_local'] = step.flat.G.cpu().numpy()
    step.allreduce()
    torch.cuda.synchronize()
    rec['G_red'] = step.flat.G.cpu().numpy()
    step.update()
    torch.cuda.synchronize()
    rec['P1'] = step.flat.P.cpu().numpy()
    rec['n_shared'] = np.int64(step.flat.n_shared)
    rec['elbo'] = np.float64(step.elbo().item())
    names = [k for k, _ in model.named_parameters()]
    rec['names'] = np.array(names)
    rec['offsets'] = np.array([step.flat.name_offsets[k] for k in names])
    if sync_bn:
        rec['counts'] = np.array(e.bn_global_counts['dec'] + [e.bn_global_counts['enc']])
    np.savez(os.path.join(out, 'rank%d.npz' % rank), **rec)
    dist.barrier()
    dist.destroy_process_group()


def run_timeout(out):
    """Two eager data-parallel steps; in the second, rank 1's side-stream flag can never reach its target
    (set 2^30 below it), so rank 1's hand-off wait times out (~10 s).  Records whether each rank's
    parameters / Adam moments moved in that step, the all-reduced error slot and whether check_handoff
    raises."""
    from gpi.train import FusedElboStep
    from elbo_ref import load
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('gloo')
    d = load('elbo_c32.npz')
    model, _ = shard_model(d, rank)
    ds = model._datasets['supervised']
    Xu = torch.tensor(d['Xu'], device='cuda')
    step = FusedElboStep(model, Xu, B_U, ds.get('X'), ds.get('Y'), ds.get('F_ROM_BC'), lr=1e-3, seed=50 + rank,
                         subset_seed=9, distributed=True, rank=rank, world=world)
    rec = dict(handoff=np.array(step.handoff), err_slot=np.int64(step.flat.err_slot))
    step.step_eager()
    torch.cuda.synchronize()
    step.check_handoff()
    P0, m0, v0 = step.flat.P.clone(), step.m.clone(), step.v.clone()
    if rank == 1:
        step.handoff_flags[3] -= (1 << 30)
    step.step_eager()
    torch.cuda.synchronize()
    rec['err_word'] = np.int64(step.handoff_flags[4].item())
    rec['slot_sum'] = np.float64(step.flat.G[step.flat.err_slot].item()) if step.flat.err_slot >= 0 else np.nan
    rec['P_same'] = np.int64(torch.equal(step.flat.P, P0))
    rec['mv_same'] = np.int64(torch.equal(step.m, m0) and torch.equal(step.v, v0))
    try:
        step.check_handoff()
        rec['raised'] = np.int64(0)
    except RuntimeError:
        rec['raised'] = np.int64(1)
    np.savez(os.path.join(out, 'rank%d.npz' % rank), **rec)
    dist.barrier()
    dist.destroy_process_group()


def run_peer(out):
    """SyncBN through the one-shot peer exchange (gpi.peer, IPC-mapped buffers of the two ranks' processes on
    the box's GPU): three eager steps with bn_exchange='collective' (fold / gloo all-reduce / unfold), three
    eager steps with 'peer', and three captured-graph replays with 'peer' (the exchange kernels spinning on
    the other process's flags inside the graph), each from the same initial state; records the parameters."""
    from gpi.train import FusedElboStep
    from elbo_ref import load
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('gloo')
    d = load('elbo_c32.npz')
    rec = {}
    for tag, exch, cap in (('coll', 'collective', False), ('peer', 'peer', False), ('peer_graph', 'peer', True)):
        model, _ = shard_model(d, rank)
        ds = model._datasets['supervised']
        Xu = torch.tensor(d['Xu'], device='cuda')
        st = FusedElboStep(model, Xu, B_U, ds.get('X'), ds.get('Y'), ds.get('F_ROM_BC'), lr=1e-3, seed=50 + rank,
                           subset_seed=9, distributed=True, rank=rank, world=world, sync_bn=True, bn_exchange=exch)
        assert st.sync_bn and (st._peer is not None) == (exch == 'peer')
        if cap:
            st.capture()
        for _ in range(3):
            if cap:
                st.step()
            else:
                st.step_eager()
        torch.cuda.synchronize()
        st.check_handoff()
        rec[tag] = st.flat.P.cpu().numpy()
        rec[tag + '.elbo'] = np.float64(st.elbo().item())
        rec['n_shared'] = np.int64(st.flat.n_shared)
        if st._peer is not None:
            rec[tag + '.seq'] = np.int64(st._peer.seq.item())
        dist.barrier()
    np.savez(os.path.join(out, 'rank%d.npz' % rank), **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[2] == 'peer':
        run_peer(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == 'c64sync':
        run_c64_sync(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == 'timeout':
        run_timeout(sys.argv[1])
    else:
        main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else 'replica')
