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
    found = []
    for prog, descs, ctx in ((e.ep, e.enc_descs, e.ectx), (e.dp, e.dec_descs, e.dctx)):
        for i, op in enumerate(prog.ops):
            fn = lib.gpi_conv_forward if which == 'fwd' else lib.gpi_conv_backward
            if prog is e.dp and i == e.n_dec_sep and e.n_dec_sep < len(e.dec_descs) and which != 'fwd':
                fn = lib.gpi_conv_loss_fused          # the decoder output conv runs fused in the step
            found.append((op.name, fn, descs[i], ctx))

    def timed(launches):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for name, fn, d, ctx in launches:            # warm
            L.check(fn(C.byref(d), C.byref(ctx), st), name)
        t0.record()
        for _ in range(reps):
            for name, fn, d, ctx in launches:
                L.check(fn(C.byref(d), C.byref(ctx), st), name)
        t1.record()
        torch.cuda.synchronize()
        return 1e3 * t0.elapsed_time(t1) / reps

    sel = [f for f in found if pat in f[0]]
    for f in sel:
        print('%s.%s  %.2f us/launch' % (f[0], which, timed([f])))
    # KPROBE_OTHER=substring: the selected op alone, the other alone, and the two alternating (a per-launch cost
    # that only the alternation shows -- cold instruction cache, evicted operands -- is the pair's excess)
    other = os.environ.get('KPROBE_OTHER')
    if other and sel:
        o = [f for f in found if other in f[0]][0]
        a, b, ab = timed([sel[0]]), timed([o]), timed([sel[0], o])
        print('alone %s %.2f  %s %.2f  alternating pair %.2f  excess %.2f us' % (sel[0][0], a, o[0], b, ab, ab - a - b))


if __name__ == '__main__':
    main()
