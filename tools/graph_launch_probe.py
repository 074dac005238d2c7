"""Host cost of replaying a HIP graph, per node: graphs of N tiny kernel nodes (gpi_rng_advance,
one thread) on one stream, and on two streams with a fork / join, timed on the host around
replay() (no synchronize inside the timed loop, one every 8 replays so the queue cannot fill).
usage: python tools/graph_launch_probe.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))
import torch  # noqa: E402
from gpi import _lib as L  # noqa: E402


def build(n, two_streams):
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    lib = L.lib()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        if two_streams:
            side.wait_stream(main)
        for i in range(n):
            st = side if (two_streams and i % 4 == 3) else main
            with torch.cuda.stream(st):
                L.check(lib.gpi_rng_advance(C.c_void_p(off.data_ptr()), C.c_uint64(1), L.stream_handle()), 'adv')
        if two_streams:
            main.wait_stream(side)
    return g, off


def host_cost(g, reps=200):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    tot = 0.0
    for r in range(reps // 8):
        t0 = time.perf_counter()
        for _ in range(8):
            g.replay()
        tot += time.perf_counter() - t0
        torch.cuda.synchronize()
    return tot / (reps // 8 * 8)


def build_linear(n, stream):
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    lib = L.lib()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(g, stream=stream):
            for i in range(n):
                L.check(lib.gpi_rng_advance(C.c_void_p(off.data_ptr()), C.c_uint64(1), L.stream_handle()), 'adv')
    return g, off


def split_cost(reps=200):
    """The step's shape as single-stream graphs: main M1 (16) -> fork -> side S (16) | main M2 (32)
    -> join -> main M3 (2); events recorded / waited between the graph launches."""
    main, side = torch.cuda.Stream(), torch.cuda.Stream()
    m1, _ = build_linear(16, main)
    s1, _ = build_linear(16, side)
    m2, _ = build_linear(32, main)
    m3, _ = build_linear(2, main)
    e1, e2 = torch.cuda.Event(), torch.cuda.Event()

    def it():
        with torch.cuda.stream(main):
            m1.replay()
            e1.record(main)
        with torch.cuda.stream(side):
            side.wait_event(e1)
            s1.replay()
            e2.record(side)
        with torch.cuda.stream(main):
            m2.replay()
            main.wait_event(e2)
            m3.replay()
    for _ in range(5):
        it()
    torch.cuda.synchronize()
    tot = 0.0
    for r in range(reps // 8):
        t0 = time.perf_counter()
        for _ in range(8):
            it()
        tot += time.perf_counter() - t0
        torch.cuda.synchronize()
    return tot / (reps // 8 * 8)


def main():
    out = {}
    t = split_cost()
    out['split_66'] = round(t * 1e6, 1)
    print('split single-stream graphs, 66 nodes: %.1f us host per iteration' % (t * 1e6), flush=True)
    for two in (False, True):
        for n in (1, 16, 64):
            g, _ = build(n, two)
            t = host_cost(g)
            out['%s_%d' % ('two' if two else 'one', n)] = round(t * 1e6, 1)
            print('%s stream(s), %3d nodes: %.1f us host per replay' % ('two' if two else 'one', n, t * 1e6),
                  flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
