"""Per-operator HIP-event profile of the C64 step's codec launches (bench.profile_kernels) with the
library the environment selects -- for timing experiments outside bench.py (e.g. the timing build's
GPI_DBG_SKIP work-skip switches, which bench.py refuses).  Results with skipped work are invalid;
timing only.  usage: GPI_PHASE_TIMING=1 GPI_DBG_SKIP=k python tools/skip_kprof.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    prof = bench.profile_kernels(step, reps=50)
    with open(sys.argv[1], 'w') as fh:
        json.dump([dict(op=n, ms=ms, bytes=b, flops=f) for n, ms, b, f in prof], fh, indent=1)


if __name__ == '__main__':
    main()
