"""Critical-path probe of the fused C64 step (timing experiments only; variants skip work, so their
ELBO values are meaningless): ms per graph replay of the full step and of variants without the
side-stream ROM ('no_rom'), without the next-step noise draws ('no_noise'), or without both; and
schedule variants that do all the work: 'enc_reduce_main' (encoder slab reduction on the main stream),
'rom_first' (ROM captured before the decoder forward), 'subset_early' (next-step subset ahead of the ROM).
usage: python tools/critpath_probe.py VARIANT [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from gpi.train import FusedElboStep  # noqa: E402


def main():
    variant = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    dev = torch.device('cuda', 0)
    model, data, (B_u, N_s), physics = bench.build('c64', dev, seed=1)
    Xu, Xs, Y, F = data
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321, subset_seed=777)
    e = step.engine
    if variant in ('no_rom', 'no_side'):
        e.roms = []
        e.early_rom = False
    if variant in ('no_noise', 'no_side'):
        step._launch_noise = lambda *a, **k: None
    if variant == 'subset_early':
        step.subset_early = True
    if variant == 'rom_first':
        e.rom_first = True
    if variant == 'enc_reduce_main':
        e.enc_reduce = 'main'
    unroll = int(os.environ.get('GPI_UNROLL', '4'))     # as bench.py: steps per graph replay
    step.capture(unroll=unroll)
    step.run(32)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    step.run(steps)
    t1.record()
    torch.cuda.synchronize()
    print('%-10s %.4f ms/step' % (variant, t0.elapsed_time(t1) / steps))


if __name__ == '__main__':
    main()
