"""Every codec launch of the C64 ELBO step (forward, backward, fused output conv), N times each in a
fixed order after one warm step -- the workload of the per-operator PMC passes
(tools/pmc_round.sh).  Writes the launch manifest (op, direction, launches, algorithmic bytes per
launch) to argv[1].  usage: python tools/pmc_all.py MANIFEST.json [N] [CONFIG]  (CONFIG: a bench.py
--config name, default c64)"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    config = sys.argv[3] if len(sys.argv) > 3 else 'c64'
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build(config, dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    st = L.stream_handle()
    manifest = []
    for name, kind, fn, d, ctx, B in bench.step_conv_launches(e):
        for _ in range(n):
            L.check(fn(C.byref(d), C.byref(ctx), st), name)
        manifest.append(dict(op=name, launches=n, algorithmic_bytes=bench.launch_bytes(kind, d, B)))
    torch.cuda.synchronize()
    with open(out, 'w') as fh:
        json.dump(dict(conv_hip_sha1=bench.conv_source_sha(), config=config, launches=manifest), fh, indent=1)


if __name__ == '__main__':
    main()
