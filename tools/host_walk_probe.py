"""Host cost of launching the fused C64 step's graph: the time replay() takes on the host with an
idle GPU (synchronize after every replay, so no queue back-pressure can stretch the call), and the
wall time per step including the wait.  Run once per environment (DEBUG_HIP_FORCE_GRAPH_QUEUES,
GPI_GRAPH_MODE ...) to compare launch structures.
usage: python tools/host_walk_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
    step.capture()
    for _ in range(20):
        step.step()
    torch.cuda.synchronize()
    call, wall = 0.0, 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        step.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        call += t1 - t0
        wall += t2 - t0
    tag = ' '.join('%s=%s' % (k, os.environ[k]) for k in ('DEBUG_HIP_FORCE_GRAPH_QUEUES', 'GPI_GRAPH_MODE')
                   if k in os.environ) or 'defaults'
    print('%-40s host replay() %.4f ms, wall per synced step %.4f ms' % (tag, 1e3 * call / reps, 1e3 * wall / reps))


if __name__ == '__main__':
    main()
