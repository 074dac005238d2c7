"""Per-launch floor of dependent kernels in one HIP graph on one stream (GPU time per node, HIP events around
replays): N tiny launches -- a one-thread kernel (gpi_rng_advance) and a 1024-workgroup fill of 1 MB -- the floor
under which a codec conv launch cannot go however little it computes.
usage: python tools/kernel_floor_probe.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'generative-physics-informed-pde_amd')]
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402


def per_node(body, n=64, reps=50):
    st = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        for _ in range(3):
            body()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            for _ in range(n):
                body()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        a.record(st)
        for _ in range(reps):
            g.replay()
        b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * n)


def main():
    lib = L.lib()
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    buf = torch.zeros(256 * 1024, dtype=torch.float32, device='cuda')
    res = dict(one_thread_us=per_node(lambda: L.check(lib.gpi_rng_advance(C.c_void_p(off.data_ptr()), C.c_uint64(1),
                                                                          L.stream_handle()), 'adv')),
               fill_1MB_1024wg_us=per_node(lambda: buf.fill_(1.0)))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
