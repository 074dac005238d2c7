"""ELBO training-step throughput of the native MI355X path.

metric : ELBO-step samples/sec on 64x64 grids (BASELINE.json), whole job.
step   : random armortized subset + reparametrisation noise + ELBO forward
         (encoder, dense head, decoder with fused Gaussian log-lik, ROM solve
         with fused log-lik) + backward + [RCCL SUM all-reduce of the shared
         gradients] + Adam over every parameter  (training.py:405-417 without
         the PredictionEnsemble / monitoring extras).
work   : per GPU B_u = 256 unlabeled + N_s = 32 labeled 64x64 samples
         (highres codec, ROM 8x8, the factory's Dropout2d rate 0.2), weak
         scaling over GPUs.

Usage: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no
torch.distributed environment, this process starts ``torch.distributed.run
--nproc-per-node N`` as a CHILD (before it touches the GPU) and relays rank 0's
JSON line; under torchrun (WORLD_SIZE set) WORLD_SIZE must equal N.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'generative-physics-informed-pde_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# kernel arguments in device memory (ROCm 7's default here; measured 434k vs 347k samples/s without it, r01q):
# pinned so that a runtime with another default does not silently take the slow path
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F32_PEAK_TFS = 157.3       # MI355X fp32 peak, vector (v_pk_fma_f32) = matrix (v_mfma_f32_16x16x4_f32) (same table)
RIDGE_FLOP_PER_B = F32_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)   # 19.7 flop/B
# HBM traffic per launch of the heaviest operators, from two separate rocprofv3 PMC
# passes (FETCH_SIZE, WRITE_SIZE) over tools/kprobe.py: tools/profile_round.sh +
# tools/pmc_traffic.py.  Used for roofline.traffic when the dominant operator is listed.
# One file per bench configuration (the entry for an operator is used only when it was measured on this
# conv.hip / common.h and at this run's algorithmic bytes, i.e. the same shape).
TRAFFIC_FILES = {'c64': ['r06_traffic.json', 'r05_traffic.json'], 'c128': ['r06_traffic_c128.json', 'r05_traffic_c128.json'],
                 'c256': ['r06_traffic_c256.json', 'r05_traffic_c256.json'], 'c32': ['r05_traffic_c32.json']}


def traffic_json(config):
    """The newest existing PMC traffic file of a bench configuration (or None)."""
    for f in TRAFFIC_FILES.get(config, []):
        p = os.path.join(ROOT, 'profiles', f)
        if os.path.exists(p):
            return p
    return None

CONFIGS = {
    # name: (factory, B_u, N_s, pool, field params (mean, std, corrlength))
    'c64': ('highres', 256, 32, 1024, (0.4, 0.8, 0.04)),
    'c32': ('highres32', 64, 16, 256, (0.4, 0.8, 0.15)),
    'c128': ('highres128', 256, 32, 512, (0.4, 0.8, 0.04)),
    'c256': ('highres256', 128, 32, 256, (0.4, 0.8, 0.04)),
}


# BASELINE.json configs each bench configuration corresponds to (c64: 2 at N = 1, 3 at N = 8)
CONFIG_TAG = {'c32': '1', 'c64': '2/3', 'c128': '4', 'c256': '5'}


def make_data(fac, n, pool, N_s, field, seed, device, rank=0):
    """Unlabeled pool: the SAME on every rank (seed), each rank slices a shared global permutation
    of it; labeled samples (fields, FOM labels, ROM boundary forces): rank-owned (seed + 1 + rank)."""
    from physics.RandomField import NormalRandomFieldSampler
    from physics.grid import pixel_to_cells
    rfs = NormalRandomFieldSampler.FromImage(n, n, *field)
    Xu = rfs.sample(batch_size=pool, rng=np.random.default_rng(seed))
    rng = np.random.default_rng(seed + 1 + rank)
    Xs = rfs.sample(batch_size=N_s, rng=rng)
    U = rng.uniform(-0.5, 0.5, (N_s, 4))
    physics = fac._physics()
    fom, rom = physics['fom'].grid, physics['rom'].grid
    Y = np.stack([fom.solve(np.exp(pixel_to_cells(x)), u) for x, u in zip(Xs, U)])
    F = np.stack([rom.full_force(u) for u in U])
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=device).contiguous()
    return t(Xu), t(Xs), t(Y), t(F), U


def build(cfg_name, device, seed, rank=0, world=1):
    from factories.model import ModelFactory
    fname, B_u, N_s, pool, field = CONFIGS[cfg_name]
    pool *= world                              # global pool; per-GPU work fixed (weak scaling)
    fac = ModelFactory.FromIdentifier(fname)
    fac.set('device', 'cuda')
    torch.manual_seed(0)                       # identical shared parameters on every rank
    physics, model, _, encoder, dtype, _ = fac.setup()
    model = model.to(device)
    encoder = encoder.to(device)
    n = physics['fom'].grid.n
    Xu, Xs, Y, F, U = make_data(fac, n, pool, N_s, field, seed, device, rank)

    class _T(object):       # device-resident dataset views
        def __init__(self, **t):
            self.t = t
            self.N = next(iter(t.values())).shape[0]

        def __bool__(self):
            return True

        def get(self, k, random_subset=None):
            return self.t[k]

    model.encoder = encoder
    model.register_datasets({'supervised': _T(X=Xs, Y=Y, F_ROM_BC=F), 'unsupervised': _T(X=Xu)}, None,
                            create_unsupervised_variational_approximation=False)
    return model, (Xu, Xs, Y, F), (B_u, N_s), physics


def conv_bytes(d, B, fwd, fused=False):
    """Algorithmic HBM bytes of one conv launch (each tensor read / written once).  fused: the
    output conv's gpi_conv_loss_fused launch (input + target read, input gradient written; the
    loss gradient never leaves LDS)."""
    hwi, hwo = d.h_in * d.w_in, d.h_out * d.w_out
    loss = d.epilogue in (2, 3)                 # GPI_EPI_GAUSS_LOSS / GPI_EPI_GAUSS_EXP_LOSS
    if fused:
        return 4.0 * B * (d.cin * hwi * (3 if d.gin_accumulate else 2) + hwo)
    if fwd:
        b = B * d.cin * hwi
        if loss:
            b += B * (hwo + 2 * hwo + (d.cout * hwo if d.out_off >= 0 else 0))   # target, gradient, (mu, ls)
        else:
            b += B * d.cout * hwo
    else:
        b = B * (d.cin * hwi + (2 if d.gout_mode == 0 else 1) * d.cout * hwo)
        if d.gin_off >= 0:
            b += B * d.cin * hwi * (2 if d.gin_accumulate else 1)
    return 4.0 * b


def conv_flops(d, B, kind):
    """Algorithmic fp32 FLOPs of one conv launch: M = B * H_out * W_out * cout * cin * K^2 multiply-adds
    per pass (every (output pixel, tap, input channel, output channel) product once; the upsampling
    convs' taps run on the upsampled image), 2 flops each; forward one pass, backward the weight
    gradient plus the input gradient when there is one, the fused output conv all three (its halo-row
    forward recompute and the loss epilogue's few flops per pixel are not counted)."""
    m = float(B) * d.h_out * d.w_out * d.cout * d.cin * d.k * d.k
    if kind == 'fwd':
        return 2.0 * m
    if kind == 'fused':
        return 6.0 * m
    return 2.0 * m * (2 if d.gin_off >= 0 else 1)


def step_conv_launches(e):
    """The codec launches of one ELBO step of engine e, in step order per program:
    [(name, kind, entry point, desc, ctx, batch)] with kind 'fwd' / 'bwd', or 'fused' for the
    output conv's single forward + loss + backward launch (engine.n_dec_sep)."""
    import ctypes as C  # noqa: F401
    from gpi import _lib as L
    lib = L.lib()
    fns = {'fwd': lib.gpi_conv_forward, 'bwd': lib.gpi_conv_backward, 'fused': lib.gpi_conv_loss_fused}
    progs = []
    if e.ep is not None:
        progs.append((e.ep, e.enc_descs, e.ectx, e.B_u, len(e.enc_descs), 0, e.n_enc_conv))
    progs.append((e.dp, e.dec_descs, e.dctx, e.B, e.n_dec_sep, e.dec0, len(e.dec_descs)))
    out = []
    for prog, descs, ctx, B, n_sep, i0, i1 in progs:
        for i, op in enumerate(prog.ops):
            if i < i0 or i >= i1:          # not launched as a conv by the engine
                continue
            for kind in (('fused',) if i >= n_sep else ('fwd', 'bwd')):
                out.append(('%s.%s' % (op.name, kind), kind, fns[kind], descs[i], ctx, B))
    return out


def launch_bytes(kind, d, B):
    return conv_bytes(d, B, kind == 'fwd', fused=kind == 'fused')


def profile_kernels(step, reps=20):
    """Per-launch device time of every codec operator, measured with HIP events on
    the stream the kernels run on; returns [(name, ms, bytes, flops)].  The reps launches of an
    operator are captured into one HIP graph and timed as two replays of it: back to back on
    the device, so a slow host (eager launches through ctypes cost about as much as the
    smallest kernels) cannot stretch the measured time."""
    import ctypes as C
    from gpi import _lib as L
    out = []
    for name, kind, fn, d, ctx, B in step_conv_launches(step.engine):
        st = L.stream_handle()
        for _ in range(3):
            fn(C.byref(d), C.byref(ctx), st)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode='thread_local'):   # (rank 0 of a DP job: other
            cst = L.stream_handle()                                      # threads may touch the device)
            for _ in range(reps):
                fn(C.byref(d), C.byref(ctx), cst)
        g.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        g.replay()
        g.replay()
        t1.record()
        torch.cuda.synchronize()
        out.append((name, t0.elapsed_time(t1) / (2 * reps), launch_bytes(kind, d, B), conv_flops(d, B, kind)))
        del g
    return out


def log(msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    sys.stderr.write('[bench %.1fs] %s\n' % (time.perf_counter() - T_START, msg))
    sys.stderr.flush()


T_START = time.perf_counter()


def cgroup_cpus():
    """CPU quota of this process's cgroup (cpu.max / cfs quota), None when unlimited."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:
            q, p = fh.read().split()[:2]
            if q != 'max':
                return max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as fh:
            q = int(fh.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fh:
            p = int(fh.read())
        if q > 0:
            return max(1, q // p)
    except (OSError, ValueError):
        pass
    return None


def host_cpu():
    """(cores this process may run on, all host cores, CPU model string).  The usable cores are the
    affinity set capped by the cgroup CPU quota (a GPU box shows every CPU of the machine but grants
    one GPU's share: 256 torch threads there ran the step at 100 s instead of ~0.2 s, r02b)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = cgroup_cpus()
    if quota is not None:
        usable = min(usable, quota)
    env = os.environ.get('OMP_NUM_THREADS')
    if env and env.isdigit() and quota is None:
        usable = min(usable, int(env))
    model = 'unknown'
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return usable, os.cpu_count() or usable, model


def cpu_baseline(model, data, B_u, N_s, physics, warmup=10, steps=50, budget_s=45.0):
    """The oracle (CPU port of the reference step, torch fp32) timed on the host cores
    (BASELINE.md section 3): torch threads = every core this process may run on, 10 warm-up + 50
    timed steps of the same step shape; if the warm-up shows 50 steps would exceed budget_s, fewer
    timed steps (>= 5) and the sample says so."""
    from oracle import codec as ocodec
    from oracle import elbo as oelbo
    from oracle import fem
    threads, host_cores, cpu_model = host_cpu()
    torch.set_num_threads(threads)
    Xu, Xs, Y, F = [t.detach().cpu() for t in data]
    enc, dec = model.encoder, model.f
    ec, dc = enc.native_config(), dec.native_config()
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.named_parameters()}
    nc = physics['rom'].grid.n
    M = torch.tensor(fem.rom_stiffness_tensor(fem.unit_square_mesh(nc)), dtype=torch.float32)
    W = torch.tensor(physics['W'], dtype=torch.float32)
    bc = torch.tensor(physics['rom'].grid.constrained_dofs)
    pe = {k[8:]: v for k, v in params.items() if k.startswith('encoder.')}
    pd = {k[2:]: v for k, v in params.items() if k.startswith('f.')}
    opt = torch.optim.Adam(params.values(), lr=1e-2)
    from gpi.plan import encoder_program, decoder_program
    drop_e = encoder_program(**ec).ops if ec['drop_rate'] else []
    drop_d = decoder_program(**dc).ops if dc['drop_rate'] else []
    drop_e = [(op.name, op.cout) for op in drop_e if op.drop]
    drop_d = [(op.name, op.cout) for op in drop_d if op.drop]

    def masks(layers, B, p):       # Dropout2d in train mode, as every reference forward draws it
        return {n: torch.bernoulli(torch.full((B, c), 1 - p)) / (1 - p) for n, c in layers} if layers else None

    def one_step():
        opt.zero_grad()
        idx = torch.randperm(Xu.shape[0])[:B_u]
        X = Xu[idx]
        encf = lambda x: ocodec.encoder_forward(pe, x, ec['imsize'], ec['blocks'], ec['growth'], ec['init_features'],
                                                drops=masks(drop_e, x.shape[0], ec['drop_rate']))
        decf = lambda z: ocodec.decoder_forward(pd, z, dc['latent_img_size'], dc['blocks'], dc['growth'],
                                                dc['init_features'], drops=masks(drop_d, z.shape[0], dc['drop_rate']))
        e1, _ = oelbo.elbo_unsupervised_armortized(encf, decf, X, torch.randn(B_u, dec.dim_latent))
        gp = lambda z: torch.nn.functional.linear(z, params['gp.fc.weight'], params['gp.fc.bias'])
        rom = lambda x, Fm: oelbo.rom_operator(W, M, bc, x, Fm, params['g.logsigmas_y'])
        qz = (params['q_z.supervised._mean'], params['q_z.supervised._logsigma'])
        qx = (params['q_X.supervised._mean'], params['q_X.supervised._logsigma'])
        e2, _ = oelbo.elbo_supervised_freeX(decf, gp, params['gp.logsigmas_X'], rom, qz, qx, Xs, Y, F,
                                            torch.randn(N_s, dec.dim_latent), torch.randn(N_s, qx[0].shape[1]))
        (-(e1 + e2)).backward()
        opt.step()

    t0 = time.perf_counter()
    w = 0
    while w < warmup:
        one_step()
        w += 1
        if time.perf_counter() - t0 > budget_s / 3:       # a slow host: fewer warm-up steps
            break
    t_step = (time.perf_counter() - t0) / w
    log('cpu baseline: %d threads, %d warm-up steps, %.3f s/step' % (threads, w, t_step))
    warmup = w
    k = steps if t_step * steps <= budget_s else max(5, int(budget_s / t_step))
    t0 = time.perf_counter()
    for _ in range(k):
        one_step()
    dt = time.perf_counter() - t0
    note = '' if k == steps else ' (budget-capped from %d)' % steps
    return dict(value=round((B_u + N_s) * k / dt, 1), unit='samples/s', cores=threads, host_cores=host_cores,
                cpu_model=cpu_model, kind='port', ms_per_step=round(1e3 * dt / k, 2),
                sample='%d warm-up + %d timed steps%s of the same step (B_u=%d, N_s=%d) on CPU torch fp32 '
                       '(oracle port), torch threads = %d' % (warmup, k, note, B_u, N_s, threads))


def step_bytes(model, B_u, N_s, physics):
    """Algorithmic HBM bytes of one step: per unlabeled sample
    4 [6 (S_enc + S_dec) + 6 H W], per labeled sample 4 [6 S_dec + 6 H W] + 4 (d_y + n_c + 2 n_T),
    S = sum over BatchNorm layers of their input elements per sample."""
    from gpi.plan import encoder_program, decoder_program

    def S(prog):
        return sum(op.cin * op.src.H * op.src.W for op in prog.ops if op.bn is not None)
    s_enc = S(encoder_program(**model.encoder.native_config()))
    s_dec = S(decoder_program(**model.f.native_config()))
    n = physics['fom'].grid.n
    nc = physics['rom'].grid.n
    d_y, n_c, n_T = (n + 1) * (n - 1), (nc + 1) ** 2, 2 * nc * nc
    per_u = 4 * (6 * (s_enc + s_dec) + 6 * n * n)
    per_s = 4 * (6 * s_dec + 6 * n * n) + 4 * (d_y + n_c + 2 * n_T)
    return B_u * per_u + N_s * per_s, dict(S_enc=s_enc, S_dec=s_dec, per_unlabeled=per_u, per_labeled=per_s)


def conv_shape_info():
    """Compile-time conv shapes (csrc/conv_shapes.h): table entries, conv launches planned since load and how many
    of them ran a shape instantiation (the graph's launches are planned once, at capture)."""
    import ctypes as C
    from gpi import _lib as L
    info = (C.c_int64 * 4)()
    if L.lib().gpi_conv_shape_info(info) != 0:
        return None
    return {'table': int(info[0]), 'launches_planned': int(info[1]), 'on_shape': int(info[2])}


def conv_source_sha():
    """sha1 of csrc/conv.hip + csrc/common.h (+ csrc/conv_shapes.h, the compile-time shapes, from r06): the
    conv kernels' sources.  PMC traffic figures are only used for the code they were measured on."""
    import hashlib
    h = hashlib.sha1()
    for f in ('conv.hip', 'common.h', 'conv_shapes.h'):
        with open(os.path.join(PKG, 'csrc', f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """--gpus n > 1 without a torch.distributed environment: one process per GPU through
    torch.distributed.run, started as a child process of this one (which has not touched the GPU:
    no exec from a GPU-initialised process).  Rank 0's stdout (the JSON line) is relayed; the
    ranks' stderr goes straight through.  Returns the launcher's exit code."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
           '--master-addr', '127.0.0.1', '--master-port', str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    log('launching %d ranks: %s' % (n, ' '.join(cmd[1:])))
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')     # dmabuf IPC (RCCL across processes)
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout.splitlines():
        if line.startswith('{'):
            print(line)
            sys.stdout.flush()
        elif line.strip():
            sys.stderr.write(line + '\n')
    return proc.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=200)
    ap.add_argument('--config', default='c64', choices=sorted(CONFIGS))
    ap.add_argument('--no-graph', action='store_true')
    # 4 steps per replay: 0.5726 / 0.5728 vs 0.5768 / 0.5773 ms per step with 1 (r04l, one box)
    ap.add_argument('--unroll', type=int, default=int(os.environ.get('GPI_UNROLL', '4')),
                    help="steps per graph replay ('streams' graph mode; FusedElboStep.capture(unroll))")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--kprof', default=None, help='write the per-operator HIP-event profile (JSON) here')
    ap.add_argument('--sync-bn', action='store_true',
                    help='SyncBN: BN statistics over the union of the ranks\' batches (default replica-BN; at N = 1 '
                         'a one-rank process group, to time the exchange)')
    ap.add_argument('--bn-exchange', default='collective', choices=['collective', 'peer'],
                    help="SyncBN seams: 'collective' (fold / RCCL all-reduce / unfold) or 'peer' (one-shot exchange "
                         'through IPC-mapped buffers, one launch per seam)')
    args = ap.parse_args()
    dbg = sorted(k for k in os.environ if k.startswith('GPI_DBG_') or k == 'GPI_PHASE_TIMING')
    if dbg:
        raise SystemExit('bench.py refuses to report with %s set (timing build / switches that skip work)' % dbg)
    # any other GPI_* variable is a tuning knob (tiles, pixel blocking, role split, output-conv fusion,
    # graph all-reduce, an A/B build of the library): recorded in the JSON line
    tuning = {k: os.environ[k] for k in sorted(os.environ) if k.startswith('GPI_')}

    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if 'WORLD_SIZE' not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ['WORLD_SIZE']) != args.gpus:
        raise SystemExit('bench.py: WORLD_SIZE=%s differs from --gpus %d (refusing to report a line for a '
                         'different GPU count)' % (os.environ['WORLD_SIZE'], args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    distributed = world > 1 or args.sync_bn
    # GPI_BENCH_BACKEND=gloo: rehearsal of the N > 1 path with every rank on the visible GPU(s)
    # (ranks share a device; RCCL refuses that).  The driver's multi-GPU runs use RCCL ('nccl').
    backend = os.environ.get('GPI_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % torch.cuda.device_count()
    if distributed:
        torch.cuda.set_device(local)
        kw = {}
        if 'MASTER_ADDR' not in os.environ:          # --sync-bn at N = 1 without torchrun: a one-rank group
            import socket
            sk = socket.socket()
            sk.bind(('127.0.0.1', 0))
            kw = dict(init_method='tcp://127.0.0.1:%d' % sk.getsockname()[1], rank=0, world_size=1)
            sk.close()
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local), **kw)
        else:
            dist.init_process_group(backend, **kw)
    device = torch.device('cuda', local)
    torch.cuda.set_device(device)

    from gpi.train import FusedElboStep
    log('building %s (rank %d of %d)' % (args.config, rank, world))
    model, data, (B_u, N_s), physics = build(args.config, device, seed=1000, rank=rank, world=world)
    log('data ready')
    Xu, Xs, Y, F = data
    # shared subset seed: every rank draws the same global permutation and takes its slice
    # N > 1 over RCCL: the all-reduce is a node of the step's graph (GPI_GRAPH_ALLREDUCE=0: host-side
    # between two graphs, as with gloo)
    step = FusedElboStep(model, Xu, B_u, Xs, Y, F, lr=1e-2, seed=4321 + rank, subset_seed=777,
                         distributed=distributed, rank=rank, world=world,
                         graph_allreduce=os.environ.get('GPI_GRAPH_ALLREDUCE', '1') == '1', sync_bn=args.sync_bn,
                         bn_exchange=args.bn_exchange)
    if not args.no_graph and not (step.sync_bn and backend != 'nccl' and args.bn_exchange != 'peer'):
        step.capture(unroll=args.unroll)
    log('captured (graph mode %s, %d step(s) per replay); warm-up' % (step.graph_mode, step.unroll))
    step.run(args.warmup)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step.run(args.steps)
    t_enq = time.perf_counter()          # host time to enqueue the K steps (graph launches)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if distributed:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    elbo = float(step.elbo().item())
    if not math.isfinite(elbo):
        raise RuntimeError('non-finite ELBO %r' % elbo)
    step.engine.check_flag()
    step.check_handoff()                 # no cross-stream flag wait timed out

    roof = None
    cpu = None
    per_step = B_u + N_s
    ms_step = 1e3 * dt / args.steps
    sbytes, sparts = step_bytes(model, B_u, N_s, physics)
    log('timed %d steps: %.4f ms/step' % (args.steps, ms_step))
    if rank == 0 and not args.no_roofline:
        prof = profile_kernels(step)
        log('per-operator profile done')
        if args.kprof:
            with open(args.kprof, 'w') as fh:
                json.dump([dict(op=n, ms=m, bytes=b, gbs=b / (m * 1e-3) / 1e9, flops=f, tfs=f / (m * 1e-3) / 1e12)
                           for n, m, b, f in prof], fh, indent=1)
        name, ms, byts, flops = max(prof, key=lambda t: t[1])
        ach = byts / (ms * 1e-3) / 1e9
        ach_tf = flops / (ms * 1e-3) / 1e12
        ai = flops / byts
        traffic = None
        traffic_note = 'no PMC traffic file for %s' % args.config
        tjp = traffic_json(args.config)
        if tjp is not None:
            with open(tjp) as fh:
                tj = json.load(fh)
            if tj.get('conv_hip_sha1') != conv_source_sha():
                traffic_note = '%s measured on other conv.hip code: dropped' % os.path.basename(tjp)
            else:
                t = tj['ops'].get(name)
                if t is None:
                    traffic_note = '%s has no entry for %s' % (os.path.basename(tjp), name)
                elif abs(t.get('algorithmic_bytes', -1) - byts) > 0.5:
                    # the file's entry is this operator at another shape (e.g. the c64 record on a c128 run)
                    traffic_note = '%s measured on another workload shape: dropped' % os.path.basename(tjp)
                else:
                    traffic = round(t['traffic_bytes'])
                    traffic_note = '%s (PMC FETCH_SIZE / WRITE_SIZE passes)' % os.path.basename(tjp)
        step_ach = sbytes / (ms_step * 1e-3) / 1e9
        # the dominant launch's bound by its arithmetic intensity: above the fp32 ridge (19.7 flop/B) it is
        # compute-bound (the fused 5x5 output conv: 30 flop/B), priced against the fp32 peak; below it
        # the HBM roofline.  Both figures are recorded.
        hbm = dict(achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit='GB/s', frac=round(ach / HBM_PEAK_GBS, 4))
        cmp_ = dict(achieved=round(ach_tf, 2), peak=F32_PEAK_TFS, unit='TFLOP/s', frac=round(ach_tf / F32_PEAK_TFS, 4))
        main = cmp_ if ai >= RIDGE_FLOP_PER_B else hbm
        # bound: the contract's roofline name ('mfma' = the compute roofline, priced at the fp32 peak, which
        # the packed-VALU v_pk_fma_f32 and the fp32 MFMA share); limiter: what actually issues the flops
        roof = dict(bound='mfma' if ai >= RIDGE_FLOP_PER_B else 'hbm',
                    limiter=('fp32 compute (VALU v_pk_fma_f32 forward / input gradient, MFMA weight gradient)'
                             if ai >= RIDGE_FLOP_PER_B else 'HBM bandwidth'),
                    achieved=main['achieved'], peak=main['peak'],
                    unit=main['unit'], frac=main['frac'], traffic=traffic, traffic_source=traffic_note, kernel=name,
                    kernel_ms=round(ms, 5), bytes_per_launch=byts, flops_per_launch=flops,
                    arithmetic_intensity=round(ai, 2), ridge=round(RIDGE_FLOP_PER_B, 2), hbm=hbm, compute=cmp_,
                    codec_ms_sum=round(sum(t[1] for t in prof), 4),
                    step=dict(bytes=sbytes, achieved=round(step_ach, 1), frac=round(step_ach / HBM_PEAK_GBS, 4),
                              **sparts))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log('cpu baseline')
        cpu = cpu_baseline(model, data, B_u, N_s, physics)

    if rank == 0:
        value = world * per_step * args.steps / dt
        line = {
            'metric': 'ELBO training-step samples/sec (64x64 grids)' if args.config == 'c64' else
            'ELBO training-step samples/sec (%s)' % args.config,
            'value': round(value, 1), 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_step, 4), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': 'BASELINE config %s: %s grid, B_u=%d unlabeled + N_s=%d labeled per GPU, '
                                   'ROM %dx%d, fused native step' % (CONFIG_TAG[args.config], args.config, B_u, N_s,
                                                                     physics['rom'].grid.n, physics['rom'].grid.n),
                       'global_batch': world * per_step, 'grid': physics['fom'].grid.n,
                       'parallelism': 'dp%d' % world, 'graph': step.graph is not None,
                       'graph_mode': step.graph_mode if step.graph is not None else None,
                       'steps_per_replay': step.unroll,
                       'world': world, 'backend': backend if distributed else None,
                       'allreduce': None if not distributed else
                       ('host-side between graphs' if args.no_graph or getattr(step, 'split_graph', True) else 'in-graph'),
                       'bn': 'replica' if not getattr(step, 'sync_bn', False) else 'sync (%s exchange)' % step.bn_exchange},
            'elbo_last': elbo,
            'host_enqueue_ms_per_step': round(1e3 * (t_enq - t0) / args.steps, 4),
            'conv_shapes': conv_shape_info(),
            'roofline': roof,
            'cpu_baseline': cpu,
        }
        if tuning:
            line['tuning_env'] = tuning
        print(json.dumps(line))
    if distributed:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
