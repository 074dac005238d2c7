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
