"""Every codec operator of the C64 ELBO step, forward and backward, launched N times each in a
fixed order after one warm step -- the workload of the per-operator PMC passes
(tools/pmc_round.sh).  Writes the launch manifest (op, direction, launches, algorithmic bytes per
launch) to argv[1].  usage: python tools/pmc_all.py MANIFEST.json [N]"""
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
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    lib = L.lib()
    st = L.stream_handle()
    manifest = []
    for prog, descs, ctx, B in ((e.ep, e.enc_descs, e.ectx, e.B_u), (e.dp, e.dec_descs, e.dctx, e.B)):
        for i, op in enumerate(prog.ops):
            for fwd in (True, False):
                fn = lib.gpi_conv_forward if fwd else lib.gpi_conv_backward
                for _ in range(n):
                    L.check(fn(C.byref(descs[i]), C.byref(ctx), st), op.name)
                manifest.append(dict(op='%s.%s' % (op.name, 'fwd' if fwd else 'bwd'), launches=n,
                                     algorithmic_bytes=bench.conv_bytes(descs[i], B, fwd)))
    torch.cuda.synchronize()
    with open(out, 'w') as fh:
        json.dump(dict(conv_hip_sha1=bench.conv_source_sha(), launches=manifest), fh, indent=1)


if __name__ == '__main__':
    main()
