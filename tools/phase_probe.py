"""Per-phase timing of single codec operators (timing build of the library).

usage: GPI_PHASE_TIMING=1 python tools/phase_probe.py [OP_SUBSTRING ...] [--fwd]
Runs every matching operator of the C64 ELBO step once more after a warm step,
reads the s_memtime stamps each workgroup wrote at its phase boundaries and
prints mean cycles per phase, the mean workgroup lifetime, the kernel span on
the 100 MHz real-time clock and the mean number of workgroups in flight, the entry / exit
time distribution and, from the HW_ID / XCC_ID each workgroup records, the exit times by
workgroups per CU and by XCD.
Phases (backward): 0 entry | 1 bases | 2 loads landed + stats | 3 coefficients |
4 activations | 5 input gradient | 6 BN-backward sums + weight gradient | 7 slab row sums
(vop ops, weight gradient first: 5 weight gradient | 6 input gradient); inside phase 1:
12 weights issued | 13 gradient image issued | 14 BN operand image issued | 8 input image issued |
9 epilogue operands issued | 10 stat loads issued | 11 stats summed.
"""
import ctypes as C
import os
import sys

os.environ['GPI_PHASE_TIMING'] = '1'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import bench  # noqa: E402
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    fwd = '--fwd' in sys.argv
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F)
    step.step_eager()
    torch.cuda.synchronize()
    e = step.engine
    lib = L.lib()
    stamps = lib.gpi_debug_phase_stamps
    stamps.restype = C.c_int
    stamps.argtypes = [C.c_void_p, C.c_void_p]
    st = L.stream_handle()
    ph = np.zeros((4096, 16), np.uint64)
    rt = np.zeros((4096, 2), np.uint64)
    for prog, descs, ctx in ((e.ep, e.enc_descs, e.ectx), (e.dp, e.dec_descs, e.dctx)):
        for i, op in enumerate(prog.ops):
            if args and not any(a in op.name for a in args):
                continue
            info = (C.c_int32 * 8)()
            L.check(lib.gpi_conv_launch_info(C.byref(descs[i]), C.byref(ctx.groups), 1 if fwd else 0, info), 'info')
            nb = min(info[1], 4096)       # workgroups of the launch
            fn = lib.gpi_conv_forward if fwd else lib.gpi_conv_backward
            if prog is e.dp and i == e.n_dec_sep and e.n_dec_sep < len(e.dec_descs) and not fwd:
                fn = lib.gpi_conv_loss_fused          # the decoder output conv runs fused in the step
            torch.cuda.synchronize()
            L.check(stamps(ph.ctypes.data, rt.ctypes.data), 'stamps')     # clears the device stamps
            for _ in range(3):     # the last launch's stamps remain
                L.check(fn(C.byref(descs[i]), C.byref(ctx), st), op.name)
            torch.cuda.synchronize()
            L.check(stamps(ph.ctypes.data, rt.ctypes.data), 'stamps')
            p = ph[:nb].astype(np.int64)
            r = rt[:nb].astype(np.int64)
            d = np.diff(p, axis=1)
            used = [k for k in range(7) if (p[:, k + 1] != 0).all() and (p[:, k] != 0).all()]
            life = (r[:, 1] - r[:, 0]) * 10.0 / 1e3          # us
            span = (r[:, 1].max() - r[:, 0].min()) * 10.0 / 1e3
            inflight = life.sum() / span if span > 0 else 0
            print('%-44s %s blocks %5d  life %6.2f us  span %6.2f us  in-flight %5.1f' %
                  (op.name, 'fwd' if fwd else 'bwd', nb, life.mean(), span, inflight))
            print('    cycles/phase: ' + '  '.join('%d:%6.0f' % (k + 1, d[:, k].mean()) for k in used))
            if os.environ.get('GPI_PROBE_HALVES') and nb % 2 == 0:
                # split launches (role by block half: input gradient first, weight gradient second)
                for hname, sl in (('first half ', slice(0, nb // 2)), ('second half', slice(nb // 2, nb))):
                    print('    %s life %6.2f us  cycles/phase: %s' % (hname, life[sl].mean(), '  '.join(
                        '%d:%6.0f' % (k + 1, d[sl, k].mean()) for k in used)))
            if os.environ.get('GPI_PROBE_RAW'):
                base = p[:, 5]
                print('    raw (cycles after stamp 5): ' + '  '.join('%d:%6.0f' % (k, (p[:, k] - base).mean())
                                                                    for k in (12, 13, 14, 8, 9, 6, 7)))
            t0 = r[:, 0].min()
            ent = np.sort((r[:, 0] - t0) * 10.0 / 1e3)
            ext = np.sort((r[:, 1] - t0) * 10.0 / 1e3)
            q = lambda a, f: a[min(len(a) - 1, int(f * len(a)))]
            print('    entry us p10/p50/p90/max %5.2f %5.2f %5.2f %5.2f   exit p10/p50/p90/max %5.2f %5.2f %5.2f %5.2f' %
                  (q(ent, .1), q(ent, .5), q(ent, .9), ent[-1], q(ext, .1), q(ext, .5), q(ext, .9), ext[-1]))
            hw = ph[:nb, 15].astype(np.uint64)
            if (hw != 0).any():
                hid = (hw & np.uint64(0xffffffff)).astype(np.int64)
                xcc = ((hw >> np.uint64(32)) & np.uint64(0xf)).astype(np.int64)
                cu = (hid >> 8) & 15
                sh = (hid >> 12) & 1
                se = (hid >> 13) & 7
                key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
                ex = (r[:, 1] - t0) * 10.0 / 1e3
                lf = (r[:, 1] - r[:, 0]) * 10.0 / 1e3
                ukey, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
                per = cnt[inv]            # workgroups that ran on this workgroup's CU
                print('    CUs used %d; workgroups per CU: %s' %
                      (len(ukey), ' '.join('%d:%d' % (k, (cnt == k).sum()) for k in np.unique(cnt))))
                for k in np.unique(per):
                    m = per == k
                    print('      on CUs with %d wg: n %4d  life mean %5.2f  exit mean %5.2f max %5.2f' %
                          (k, m.sum(), lf[m].mean(), ex[m].mean(), ex[m].max()))
                print('    exit mean by XCC: ' + ' '.join('%d:%5.2f' % (x, ex[xcc == x].mean()) for x in np.unique(xcc)))
            sub = [1, 12, 13, 14, 8, 9, 10, 11, 2]     # phase-1 issue points (timing build, backward)
            if all((p[:, k] != 0).all() for k in sub):
                print('    phase-1 split: ' + '  '.join('%d->%d:%6.0f' % (sub[k], sub[k + 1],
                      (p[:, sub[k + 1]] - p[:, sub[k]]).mean()) for k in range(len(sub) - 1)))


if __name__ == '__main__':
    main()
