"""Launch geometry of every conv of the C64 ELBO step (host only, no GPU): rows per tile,
workgroups, LDS per workgroup, resident workgroups per CU (LDS / VGPR bound) and rounds on
256 CUs.  usage: python tools/conv_geometry.py [c64|c32|c128|c256]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd')]
from gpi import _lib as L  # noqa: E402
from gpi.engine import Workspace, groups_struct  # noqa: E402
from gpi.plan import encoder_program, decoder_program  # noqa: E402
import bench  # noqa: E402

CUS = 256
LDS_CU = 160 * 1024


def main(cfg='c64', vgpr_wgs=(6, 4)):
    from factories.model import ModelFactory
    fname, B_u, N_s, pool, field = bench.CONFIGS[cfg]
    fac = ModelFactory.FromIdentifier(fname)
    fac.set('device', 'cpu')
    _, model, _, enc, _, _ = fac.setup()
    lib = L.lib()
    for kind, prog, B, sizes in (('enc', encoder_program(**enc.native_config()), B_u, [B_u]),
                                 ('dec', decoder_program(**model.f.native_config()), B_u + N_s, [B_u, N_s])):
        ws = Workspace()
        descs = prog.layout(B, ws.ws, ws.stats, ws.parts, groups_struct(sizes), lambda n: 0)
        g = groups_struct(sizes)
        for i, op in enumerate(prog.ops):
            for fwd in (1, 0):
                info = (C.c_int32 * 8)()
                L.check(lib.gpi_conv_launch_info(C.byref(descs[i]), C.byref(g), fwd, info), op.name)
                th, nb, lds, cp, npx, P, PG = list(info)[:7]
                per_cu = min(LDS_CU // max(lds, 1), vgpr_wgs[1] if (op.k == 5 and not fwd) else vgpr_wgs[0])
                print('%s %-40s %s k%d s%d up%d %2d->%-2d %3dx%-3d th %3d npx %d P %3d PG %3d blocks %5d lds %6d  wg/cu %d  rounds %.2f' % (
                    kind, op.name, 'fwd' if fwd else 'bwd', op.k, op.stride, op.upsample, op.cin, op.cout,
                    op.dst.H, op.dst.W, th, npx, P, PG, nb, lds, per_cu, nb / (per_cu * CUS)))


if __name__ == '__main__':
    main(*sys.argv[1:2])
