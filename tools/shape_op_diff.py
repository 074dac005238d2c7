"""One conv op of the bench step run with its compile-time shape kernel and with the generic kernel on the same
workspace state (debugging aid, GPU): the op's output region compared element by element, the differing
(sample, channel, row, column) positions summarised.
usage: python tools/shape_op_diff.py OP_SUBSTRING [fwd|bwd]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import bench  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    pat, which = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else 'fwd')
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    lib = L.lib()
    ws = e.ws.t_ws
    for prog, descs, ctx, B in ((e.ep, e.enc_descs, e.ectx, e.B_u), (e.dp, e.dec_descs, e.dctx, e.B)):
        for i, op in enumerate(prog.ops):
            if pat not in op.name:
                continue
            d = descs[i]
            fn = lib.gpi_conv_forward if which == 'fwd' else lib.gpi_conv_backward
            HW = d.h_out * d.w_out if which == 'fwd' else d.h_in * d.w_in
            off = d.out_off if which == 'fwd' else d.gin_off
            ctot = d.out_ctot if which == 'fwd' else d.in_ctot
            n = B * ctot * HW
            before = ws[off:off + n].clone()
            outs = []
            for on in ('1', '0'):
                ws[off:off + n].copy_(before)
                os.environ['GPI_CONV_SHAPES'] = on
                info0 = (C.c_int64 * 4)()
                lib.gpi_conv_shape_info(info0)
                L.check(fn(C.byref(d), C.byref(ctx), L.stream_handle()), op.name)
                torch.cuda.synchronize()
                info1 = (C.c_int64 * 4)()
                lib.gpi_conv_shape_info(info1)
                outs.append(ws[off:off + n].cpu().numpy().reshape(B, ctot, d.h_out if which == 'fwd' else d.h_in, -1))
                print('%s %s shapes=%s: matched %d' % (op.name, which, on, info1[2] - info0[2]))
            a, b = outs
            c0 = d.out_c0 if which == 'fwd' else d.in_c0
            nc = d.cout if which == 'fwd' else d.cin
            a, b = a[:, c0:c0 + nc], b[:, c0:c0 + nc]
            bad = np.argwhere(a != b)
            print('differ: %d of %d, max |diff| %.3e' % (len(bad), a.size, np.abs(a - b).max() if a.size else 0))
            if len(bad):
                for q in bad[:12]:
                    print('  at %s: shapes %r generic %r' % (tuple(q), a[tuple(q)], b[tuple(q)]))
                print('  nan in shapes %d, in generic %d' % (np.isnan(a).sum(), np.isnan(b).sum()))
                for ax, nm in enumerate(('sample', 'channel', 'row', 'col')):
                    u, cnt = np.unique(bad[:, ax], return_counts=True)
                    print('  %s: %s' % (nm, ' '.join('%d:%d' % (x, y) for x, y in list(zip(u, cnt))[:70])))
            return


if __name__ == '__main__':
    main()
