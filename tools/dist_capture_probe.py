"""RCCL all-reduce captured in the fused step's graph: run with torch.distributed.run (nccl), compare
graph replays with eager steps of an identical copy (same seeds) -- parameters after 3 steps.
usage: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/dist_capture_probe.py"""
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
    d = load('elbo_c32.npz')
    ma, bs = build_golden_model(d)
    mb = copy.deepcopy(ma)
    args = (cuda(d['Xu']), bs // world, cuda(d['Xs']), cuda(d['Y']), cuda(d['F']))
    kw = dict(lr=1e-3, seed=5 + rank, subset_seed=1, distributed=True, rank=rank, world=world)
    eager = FusedElboStep(ma, *args, **kw)
    graph = FusedElboStep(mb, *args, **kw)
    graph.capture()
    assert not graph.split_graph
    for _ in range(3):
        eager.step_eager()
        graph.step()
    torch.cuda.synchronize()
    err = (graph.flat.P - eager.flat.P).abs().max().item()
    print('rank %d world %d: graph-captured all-reduce vs eager, max |dP| = %.3e' % (rank, world, err), flush=True)
    assert err < 1e-6
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
