"""Data-parallel native step on the GPU: two gloo ranks share the box's
one GPU (RCCL refuses two ranks on one device; the driver's 8-GPU node runs the same code over
RCCL), each running the NATIVE FusedElboStep on its shard (tests/dp_worker.py).

Checks: both ranks drew the same global permutation and took disjoint slices of it; the
all-reduced shared-gradient prefix equals the SUM of the two single-process shard gradients
(module path GenerativeModel.elbo on each shard with the rank's own subset and noise); the
per-sample q rows stay rank-local (not communicated); after Adam the shared parameters are
identical on both ranks."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from elbo_ref import load, tensor_rel

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_native_step(device, tmp_path):
    from dp_worker import shard_model, B_U
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dp_worker.py'),
           str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rk = [dict(np.load(str(tmp_path / ('rank%d.npz' % i)))) for i in range(2)]
    # one global permutation, rank slices disjoint
    assert np.array_equal(rk[0]['idx'], rk[1]['idx'])
    idx = rk[0]['idx']
    assert len(set(idx.tolist())) == 2 * B_U
    ns = int(rk[0]['n_shared'])
    assert ns == int(rk[1]['n_shared'])
    # reference: each shard's gradient through the single-process module path
    d = load('elbo_c32.npz')
    shard_G = []
    for rank in range(2):
        model, _ = shard_model(d, rank)
        model._datasets['unsupervised'].perm = torch.tensor(idx[rank * B_U:(rank + 1) * B_U], device='cuda').long()
        eps = (torch.tensor(rk[rank]['eps_z'], device='cuda'), torch.tensor(rk[rank]['eps_x'], device='cuda'))
        with torch.no_grad():
            offs = rk[rank]['offsets']
            assert [k for k, _ in model.named_parameters()] == list(rk[rank]['names'])
            for (k, p), o in zip(model.named_parameters(), offs):
                p.copy_(torch.tensor(rk[rank]['P0'][o:o + p.numel()].reshape(p.shape)))
        elbo = model.elbo(step=0, armortized_bs=B_U, eps=eps)
        (-elbo).backward()
        assert abs(elbo.item() - float(rk[rank]['elbo'])) <= 1e-5 * abs(elbo.item())
        G = np.zeros_like(rk[rank]['G_local'])
        for (k, p), o in zip(model.named_parameters(), offs):
            G[o:o + p.numel()] = p.grad.cpu().numpy().ravel()
        shard_G.append(G)
        # the rank's local (pre-exchange) gradient is its shard's gradient
        assert tensor_rel(rk[rank]['G_local'], G) < 1e-5
    total = shard_G[0][:ns] + shard_G[1][:ns]
    for rank in range(2):
        # shared prefix: the SUM over the shards (the ELBO is a sum over samples, normalize=False)
        assert tensor_rel(rk[rank]['G_red'][:ns], total) < 1e-5
        # per-sample q rows: rank-local, untouched by the exchange
        assert np.array_equal(rk[rank]['G_red'][ns:], rk[rank]['G_local'][ns:])
    # replicated shared parameters stay identical after the update
    assert np.array_equal(rk[0]['P1'][:ns], rk[1]['P1'][:ns])
    assert np.array_equal(rk[0]['P0'][:ns], rk[1]['P0'][:ns])


@pytest.mark.parametrize('mode', ['sync', 'sync_uneven'])
def test_dp_two_ranks_sync_bn(device, tmp_path, mode):
    """SyncBN (FusedElboStep(sync_bn=True)): with every BN layer normalised over
    both ranks' batches, the all-reduced shared gradient of two gloo ranks equals the gradient of ONE
    process running the union batch (the reference's semantics at the global batch: train-mode BN over
    the whole codec call, codec.py:164-173), and each rank's q rows equal the union's rows of its
    labeled shard.  'sync_uneven': the labeled shards hold 1 and 3 samples, so the labeled decoder
    group's per-rank counts differ (each all-reduced BN sum is scaled by the rank's count over the global
    one).  Tolerance 5e-5 per tensor (fp32 sums in another order); the ELBO halves sum to the union ELBO
    within 1e-5."""
    from dp_worker import B_U, NS_RANK, NS_UNEVEN
    from test_gpu_parity import build_golden_model
    ns_r = list(NS_UNEVEN) if mode == 'sync_uneven' else [NS_RANK, NS_RANK]
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dp_worker.py'),
           str(tmp_path), mode]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rk = [dict(np.load(str(tmp_path / ('rank%d.npz' % i)))) for i in range(2)]
    assert list(rk[0]['counts']) == [2 * B_U, sum(ns_r), 2 * B_U]
    idx = rk[0]['idx']
    ns = int(rk[0]['n_shared'])
    d = load('elbo_c32.npz')
    e = dict(d)
    e['cfg'] = np.array([int(d['cfg'][0]), int(d['cfg'][1]), int(d['cfg'][2]), int(d['cfg'][3]), 2 * B_U,
                         sum(ns_r)])
    for k in ('Xs', 'Y', 'F'):
        e[k] = d[k][:sum(ns_r)]
    model, _ = build_golden_model(e)
    model._datasets['unsupervised'].perm = torch.tensor(idx[:2 * B_U], device='cuda').long()
    dz = rk[0]['eps_z'].shape[1]
    ez = np.concatenate([rk[0]['eps_z'][:B_U], rk[1]['eps_z'][:B_U], rk[0]['eps_z'][B_U:], rk[1]['eps_z'][B_U:]])
    ex = np.concatenate([rk[0]['eps_x'], rk[1]['eps_x']])
    assert ez.shape == (2 * B_U + sum(ns_r), dz)
    names = list(rk[0]['names'])
    # the union's q rows: rank 0's shard, then rank 1's (per-row sizes from the union parameter)
    row_parts = lambda p: [p.numel() // sum(ns_r) * n for n in ns_r]
    with torch.no_grad():       # the ranks' initial parameters (shared: identical; q rows: shard rows)
        for k, p in model.named_parameters():
            i = names.index(k)
            o = [int(rk[j]['offsets'][i]) for j in range(2)]
            if k.startswith(('q_z.', 'q_X.')):
                parts = [rk[j]['P0'][o[j]:o[j] + row_parts(p)[j]] for j in range(2)]
                p.copy_(torch.tensor(np.concatenate(parts).reshape(p.shape)))
            else:
                p.copy_(torch.tensor(rk[0]['P0'][o[0]:o[0] + p.numel()].reshape(p.shape)))
    elbo = model.elbo(step=0, armortized_bs=2 * B_U, eps=(torch.tensor(ez, device='cuda'),
                                                          torch.tensor(ex, device='cuda')))
    (-elbo).backward()
    tot = float(rk[0]['elbo']) + float(rk[1]['elbo'])
    assert abs(tot - elbo.item()) <= 1e-5 * abs(elbo.item()), (tot, elbo.item())
    errs = {}
    for k, p in model.named_parameters():
        i = names.index(k)
        g = p.grad.cpu().numpy().ravel()
        if k.startswith(('q_z.', 'q_X.')):
            rp = row_parts(p)
            for j in range(2):
                o, lo = int(rk[j]['offsets'][i]), sum(rp[:j])
                errs['%s[rank%d]' % (k, j)] = tensor_rel(rk[j]['G_red'][o:o + rp[j]], g[lo:lo + rp[j]])
        else:
            o = int(rk[0]['offsets'][i])
            assert o + p.numel() <= ns
            errs[k] = tensor_rel(rk[0]['G_red'][o:o + p.numel()], g)
            assert np.array_equal(rk[0]['G_red'][o:o + p.numel()], rk[1]['G_red'][o:o + p.numel()])
    bad = {k: v for k, v in errs.items() if v >= 5e-5}
    assert not bad, (bad, sorted(errs.items(), key=lambda kv: -kv[1])[:8])


def test_rccl_allreduce_captured_in_step_graph(device):
    """The RCCL (backend 'nccl') all-reduce of the shared gradients captured inside the fused step's
    HIP graph: replays equal eager steps bit for bit (world size 1 on this one-GPU box; the driver's
    8-GPU node runs the same capture across ranks)."""
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(),
           os.path.join(os.path.dirname(HERE), 'tools', 'dist_capture_probe.py')]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'max |dP| = 0.000e+00' in r.stdout, r.stdout[-2000:]


def test_rccl_allreduce_captured_unrolled(device):
    """The bench's N > 1 form: two steps per replay of the captured graphs ('streams' mode when the probe
    allows), i.e. two RCCL all-reduces inside one graph, and run(3) = one 2-step replay + one single step;
    equal to eager steps (world size 1 on this box)."""
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(),
           os.path.join(os.path.dirname(HERE), 'tools', 'dist_capture_probe.py'), '--unroll', '2']
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'max |dP| = 0.000e+00' in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize('cfg,n_coll', [('c32', 26), ('c64', 42)])
def test_rccl_sync_bn_captured_in_step_graph(device, cfg, n_coll):
    """SyncBN over RCCL inside the captured step (world size 1 on this box; the 8-GPU node runs the
    same graph across ranks): the per-conv collectives of the BN batch sums (26 at C32; 42 at C64, the
    graph an 8-GPU config-3 SyncBN bench captures: highres codec, B_u = 256, N_s = 32, Dropout2d 0.2) are
    graph nodes, the replays equal eager SyncBN steps bit for bit, and at one rank SyncBN agrees with
    replica-BN to rounding."""
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(),
           os.path.join(os.path.dirname(HERE), 'tools', 'dist_capture_probe.py'), '--sync-bn', '--config', cfg]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'max |dP| = 0.000e+00' in r.stdout, r.stdout[-2000:]
    n = int(r.stdout.split('SyncBN (')[1].split()[0])
    assert n == n_coll, r.stdout[-2000:]
    assert 'SyncBN vs replica-BN' in r.stdout, r.stdout[-2000:]


def test_dp_config3_sync_bn_vs_union_oracle(device, tmp_path):
    """BASELINE config 3 at its own global batch through the real DP code: 8 gloo ranks (config 3's
    world), each running the NATIVE FusedElboStep with SyncBN at config 3's per-rank shape (C64 highres,
    B_u = 256 of a shared pool + N_s = 32 rank-owned labeled samples, Dropout2d 0.2), against the fp64
    oracle of ONE process on the union batch (B_u = 2048, N_s = 256: train-mode BN over the whole codec
    call, codec.py:164-173) on the ranks' own subsets, noise and dropout scales, with the kernels' ReLU
    decisions (tests/gpu_masks.py).  The ranks' ELBOs sum to the union ELBO within 1e-5; the
    all-reduced shared gradient and each rank's q rows match the union gradient at 5e-5 per tensor.
    (The ranks share the box's one GPU over gloo; only the RCCL-over-xGMI wire itself stays for the
    8-GPU node.)"""
    from dp_worker import C64_BU, C64_NS, c64_data
    from elbo_ref import oracle_elbo
    from test_gpu_c64 import check_mask_audit
    from oracle import codec as ocodec
    world = 8
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % world,
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dp_worker.py'),
           str(tmp_path), 'c64sync']
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rk = [dict(np.load(str(tmp_path / ('rank%d.npz' % i)))) for i in range(world)]
    idx = rk[0]['idx']
    assert all(np.array_equal(x['idx'], idx) for x in rk)
    assert len(set(idx[:world * C64_BU].tolist())) == world * C64_BU
    # every BN group's global count: world x the per-rank batch
    assert list(rk[0]['counts']) == [world * C64_BU, world * C64_NS, world * C64_BU]
    ns = int(rk[0]['n_shared'])
    Xu, _, _, _ = c64_data(world, 0)
    data = [c64_data(world, j)[1:] for j in range(world)]
    cat = lambda parts: np.concatenate(parts, 0)
    Xs, Y, F = [cat([dd[i] for dd in data]) for i in range(3)]
    eps_enc = cat([x['eps_z'][:C64_BU] for x in rk])
    eps_qz = cat([x['eps_z'][C64_BU:] for x in rk])
    eps_qX = cat([x['eps_x'] for x in rk])
    drops = {'enc': {}, 'dec': {}}
    masks = {'enc': {}, 'dec_u': {}, 'dec_s': {}}
    for k in rk[0]:
        if k.startswith('drop.enc.'):
            drops['enc'][k[9:]] = torch.tensor(cat([x[k] for x in rk]), dtype=torch.float64)
        elif k.startswith('drop.dec.'):        # union decoder rows: every rank's unlabeled, then labeled
            drops['dec'][k[9:]] = torch.tensor(cat([x[k][:C64_BU] for x in rk] + [x[k][C64_BU:] for x in rk]),
                                               dtype=torch.float64)
        elif k.startswith('mask.'):
            call, nm = k[5:].split('.', 1)
            masks[call][nm] = torch.tensor(cat([x[k] for x in rk]))
    assert drops['enc'] and drops['dec'] and masks['enc'] and masks['dec_u'] and masks['dec_s']
    names = list(rk[0]['names'])
    st = {}
    for i, k in enumerate(names):
        shp = tuple(int(v) for v in rk[0]['shape.' + k])
        nel = int(np.prod(shp))
        if k.startswith(('q_z.', 'q_X.')):       # rank-owned rows: the union's rows in rank order
            a = cat([x['P0'][int(x['offsets'][i]):int(x['offsets'][i]) + nel].reshape(shp) for x in rk])
        else:
            o = int(rk[0]['offsets'][i])
            a = rk[0]['P0'][o:o + nel].reshape(shp)
        st[k] = torch.tensor(a, dtype=torch.float64, requires_grad=True)
    ocodec.MASK_AUDIT.clear()
    val = oracle_elbo(st, Xu[idx[:world * C64_BU]], Xs, Y, F, eps_enc, eps_qz, eps_qX, 8, 8, masks=masks,
                      drops=drops)
    check_mask_audit()
    (-val).backward()
    tot = sum(float(x['elbo']) for x in rk)
    assert abs(tot - val.item()) <= 1e-5 * abs(val.item()), (tot, val.item())
    errs = {}
    for i, k in enumerate(names):
        g = st[k].grad.numpy().ravel()
        if k.startswith(('q_z.', 'q_X.')):
            part = g.size // world
            for j, x in enumerate(rk):
                o = int(x['offsets'][i])
                errs['%s[rank%d]' % (k, j)] = tensor_rel(x['G_red'][o:o + part], g[j * part:(j + 1) * part])
        else:
            o = int(rk[0]['offsets'][i])
            assert o + g.size <= ns
            errs[k] = tensor_rel(rk[0]['G_red'][o:o + g.size], g)
            for x in rk[1:]:
                assert np.array_equal(x['G_red'][o:o + g.size], rk[0]['G_red'][o:o + g.size]), k
    bad = {k: v for k, v in errs.items() if not v < 5e-5}
    assert not bad, (bad, sorted(errs.items(), key=lambda kv: -kv[1])[:8])



def test_dp_hand_off_timeout_on_one_rank_stops_every_rank(device, tmp_path):
    """a hand-off wait that times out on ONE rank (its gradient may be incomplete) must not let
    the other ranks apply the all-reduced gradient.  Rank 1's side-stream flag is pushed out of reach in the
    second of two data-parallel steps: its wait times out (~10 s), its epilogue writes 1 into the flat
    gradient's error slot (inside the all-reduced shared prefix), the SUM carries it to rank 0, and BOTH ranks
    leave parameters and Adam moments untouched and raise (check_handoff)."""
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dp_worker.py'),
           str(tmp_path), 'timeout']
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rk = [dict(np.load(str(tmp_path / ('rank%d.npz' % i)))) for i in range(2)]
    if str(rk[0]['handoff']) != 'flags':
        pytest.skip('no flag hand-off in this configuration')
    for i in range(2):
        assert int(rk[i]['err_slot']) >= 0
        assert float(rk[i]['slot_sum']) == 1.0, i          # rank 1's timeout, summed over both ranks
        assert int(rk[i]['err_word']) == 1, i              # rank 1: its wait; rank 0: set by its Adam
        assert int(rk[i]['P_same']) == 1 and int(rk[i]['mv_same']) == 1, i
        assert int(rk[i]['raised']) == 1, i


def test_sync_bn_peer_exchange_two_ranks(device, tmp_path):
    """The throughput SyncBN exchange (gpi_bn_exchange GPI_BNX_PEER through the ranks' IPC-mapped buffers: one
    launch per BN seam, no collective call) with two ranks' processes on the box's GPU: three eager SyncBN steps
    equal the collective form's (fold / gloo all-reduce / unfold) bit for bit -- the two-rank sum a + b either
    way -- and three replays of the captured step graph (the exchange kernels spinning on the other process's
    flags inside the graph) equal the eager peer steps bit for bit; the ranks' replicated parameters stay
    identical.  (codec.py:164-173 at the union batch.)"""
    env = dict(os.environ)
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dp_worker.py'),
           str(tmp_path), 'peer']
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rk = [dict(np.load(str(tmp_path / ('rank%d.npz' % i)))) for i in range(2)]
    for i in range(2):
        assert np.array_equal(rk[i]['peer'], rk[i]['coll']), i
        assert np.array_equal(rk[i]['peer_graph'], rk[i]['peer']), i
        assert rk[i]['peer.elbo'] == rk[i]['coll.elbo']
        assert int(rk[i]['peer.seq']) > 0 and int(rk[i]['peer_graph.seq']) > 0
    ns = int(rk[0]['n_shared'])
    assert ns > 0 and np.array_equal(rk[0]['peer'][:ns], rk[1]['peer'][:ns])
