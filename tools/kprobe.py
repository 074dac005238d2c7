"""Run single codec operators of the C64 ELBO step in isolation (for rocprofv3 counter passes).

usage: python tools/kprobe.py OP_SUBSTRING [fwd|bwd] [reps]
e.g.   python tools/kprobe.py LastTransUp.conv1 bwd 50
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    pat = sys.argv[1]
    which = sys.argv[2] if len(sys.argv) > 2 else 'bwd'
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    lib = L.lib()
    st = L.stream_handle()
    for prog, descs, ctx in ((e.ep, e.enc_descs, e.ectx), (e.dp, e.dec_descs, e.dctx)):
        for i, op in enumerate(prog.ops):
            if pat not in op.name:
                continue
            fn = lib.gpi_conv_forward if which == 'fwd' else lib.gpi_conv_backward
            if prog is e.dp and i == e.n_dec_sep and e.n_dec_sep < len(e.dec_descs) and which != 'fwd':
                fn = lib.gpi_conv_loss_fused          # the decoder output conv runs fused in the step
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(reps):
                L.check(fn(C.byref(descs[i]), C.byref(ctx), st), op.name)
            t1.record()
            torch.cuda.synchronize()
            print('%s.%s  %.2f us/launch' % (op.name, which, 1e3 * t0.elapsed_time(t1) / reps))


if __name__ == '__main__':
    main()
