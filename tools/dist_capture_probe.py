"""RCCL all-reduce captured in the fused step's graph: run with torch.distributed.run (nccl), compare
graph replays with eager steps of an identical copy (same seeds) -- parameters after 3 steps.
--sync-bn: SyncBN (every BN layer's batch sums all-reduced conv by conv, ~46 collectives per step) captured
into the step graph as well; the replays must equal the eager SyncBN steps bit for bit, and at world size 1
the SyncBN step must also agree with the replica-BN step to rounding (the same batch statistics).
--unroll K: the graph copy captures K steps per replay (FusedElboStep.capture(unroll=K), K all-reduces in one
graph) and takes its 3 steps by run(3).
usage: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/dist_capture_probe.py
       [--sync-bn] [--unroll K] [--config c32|c64]
--config c64: BASELINE config 3's per-rank shape (C64 highres codec, B_u = 256, N_s = 32, Dropout2d 0.2; 42 SyncBN
collectives per step) instead of the C32 golden fixture."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd'), os.path.join(ROOT, 'tests')]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    rank, world = dist.get_rank(), dist.get_world_size()
    from elbo_ref import load
    from test_gpu_parity import build_golden_model, cuda
    from gpi.train import FusedElboStep
    cfg = sys.argv[sys.argv.index('--config') + 1] if '--config' in sys.argv else 'c32'
    if cfg == 'c64':
        # BASELINE config 3's per-rank step (C64 highres, B_u = 256 of a shared pool, N_s = 32, Dropout2d 0.2)
        from dp_worker import c64_model, C64_BU
        ma, (Xu, Xs, Y, F) = c64_model(world, rank)
        args = (Xu, C64_BU, Xs, Y, F)
    else:
        d = load('elbo_c32.npz')
        ma, bs = build_golden_model(d)
        args = (cuda(d['Xu']), bs // world, cuda(d['Xs']), cuda(d['Y']), cuda(d['F']))
    mb = copy.deepcopy(ma)
    sync = '--sync-bn' in sys.argv
    mc = copy.deepcopy(ma) if sync and world == 1 else None
    kw = dict(lr=1e-3, seed=5 + rank, subset_seed=1, distributed=True, rank=rank, world=world, sync_bn=sync)
    eager = FusedElboStep(ma, *args, **kw)
    graph = FusedElboStep(mb, *args, **kw)
    assert eager.sync_bn == sync and graph.sync_bn == sync
    assert (graph.engine.bn_sync is not None) == sync
    n_coll = [0]
    if sync:     # count the codec's collectives of one captured step
        inner = graph.engine.bn_sync

        def counted(t):
            n_coll[0] += 1
            inner(t)
        graph.engine.bn_sync = counted
    unroll = int(sys.argv[sys.argv.index('--unroll') + 1]) if '--unroll' in sys.argv else 1
    graph.capture(unroll=unroll)
    assert not graph.split_graph
    n_per_step = n_coll[0] // 3          # two warm-up steps + the captured one
    print('rank %d: graph mode %s, %d step(s) per replay' % (rank, graph.graph_mode, graph.unroll), flush=True)
    for _ in range(3):
        eager.step_eager()
    if unroll > 1:
        graph.run(3)
    else:
        for _ in range(3):
            graph.step()
    torch.cuda.synchronize()
    graph.check_handoff()
    err = (graph.flat.P - eager.flat.P).abs().max().item()
    what = 'SyncBN (%d codec collectives per step, %s) + ' % (n_per_step, cfg) if sync else ''
    print('rank %d world %d: graph-captured %sall-reduce vs eager, max |dP| = %.3e' % (rank, world, what, err),
          flush=True)
    assert err < 1e-6
    if mc is not None:
        # one rank: SyncBN's statistics are the replica-BN ones (folded into replica 0, other order)
        ref = FusedElboStep(mc, *args, **dict(kw, sync_bn=False))
        for _ in range(3):
            ref.step_eager()
        torch.cuda.synchronize()
        dr = ((graph.flat.P - ref.flat.P).abs().max() / ref.flat.P.abs().max()).item()
        print('rank %d world 1: SyncBN vs replica-BN after 3 steps, max |dP| / max |P| = %.3e' % (rank, dr),
              flush=True)
        assert dr < 1e-5
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
