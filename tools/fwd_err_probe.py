"""Forward / worst gradient relative error of the 128^2 and 256^2 codec cases (tests/test_gpu_parity._codec_case) for six seeds, under the
current environment (tile / channel-group A/B of the parity margins).  usage: TAG=x python tools/fwd_err_probe.py"""
import sys, os
sys.path[:0] = ['tests', '.', 'generative-physics-informed-pde_amd']
import test_gpu_parity as t
for imsize, blocks, B in [(128, [1, 2, 2, 1], 3), (256, [1, 2, 2, 2, 1], 2)]:
    out = []
    for seed in range(6):
        fwd, errs = t._codec_case(imsize, blocks, B, seed)
        out.append('%.3g/%.3g' % (fwd, max(errs.values())))
    print(os.environ.get('TAG', ''), imsize, ' '.join(out), flush=True)
