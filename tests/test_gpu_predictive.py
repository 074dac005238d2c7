"""GPU parity of the monitoring / validation paths: the native
PredictionEnsemble.update (decoder-only ELBO + Adam on the validation q_z) and the batched
Analysis.eval_all_y, against the reference run recorded in pe_analysis_c32.npz
(injected noise).  Tolerances: q_z after 3 Adam steps 1e-4 relative, ELBO terms 2e-5,
predictive scores 1e-4."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


def cuda(a, dtype=torch.float32):
    return torch.tensor(np.asarray(a), dtype=dtype, device='cuda')


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


class _DS(object):
    label = 'validation'

    def __init__(self, **t):
        self.t = t
        self.N = next(iter(t.values())).shape[0]

    def __bool__(self):
        return True

    def get(self, key, random_subset=None):
        return self.t[key]


class _Writer(object):
    def __init__(self):
        self.d = {}

    def add_scalar(self, k, v, global_step=None):
        self.d[k] = float(v.detach()) if hasattr(v, "detach") else float(v)


def build(d):
    from bottleneck.Decoder import CNNDecoder
    from bottleneck.components import EffectivePropertyMap, ReducedOrderModelOperator
    from bottleneck.ROM import ROM
    from bottleneck.generative import GenerativeModel
    from physics.grid import StructuredGrid
    n, nc, dz, Nval, Nmc, iters = [int(v) for v in d['cfg']]
    dec = CNNDecoder(n, dz, (8, 8), 1, 4, [1, 1], False, 4, drop_rate=0.)
    rom = ROM(StructuredGrid(nc), n // nc)
    g = ReducedOrderModelOperator(rom, torch.tensor(d['W']), dtype=torch.float32, device='cuda')
    gp = EffectivePropertyMap(dz, 2 * nc * nc, dtype=torch.float32, device='cuda')
    model = GenerativeModel(f=dec.cuda(), g=g, gp=gp, dtype=torch.float32, device=torch.device('cuda'))
    model.load_state_dict({k[6:]: torch.tensor(v) for k, v in d.items() if k.startswith('state.')})
    model.cuda()
    ds = _DS(X=cuda(d['X']), Y=cuda(d['Y']), F_ROM_BC=cuda(d['F']))
    return model, ds


def test_prediction_ensemble_update(device):
    from bottleneck.components import PredictionEnsemble
    from lamp.optimization import LearningScheduleWrapper
    d = load('pe_analysis_c32.npz')
    model, ds = build(d)
    pe = PredictionEnsemble(model, ds, LearningScheduleWrapper.Dummy(), lr=1e-2, writer=_Writer())
    iters = int(d['cfg'][5])
    pe.update(numIter=iters, record=True, step=0, eps=[cuda(e) for e in d['pe_eps']])
    w = pe.writer.d
    for k in ('elbo', 'logL', 'KLD'):
        ref = float(d['pe_' + k])
        assert abs(w['PredictionEnsemble/' + k] - ref) <= 2e-5 * max(abs(ref), 1.0), (k, w, ref)
    assert rel(pe.q_z.mean.detach().cpu(), d['pe_mean']) < 1e-4
    assert rel(pe.q_z.logsigma.detach().cpu(), d['pe_logsigma']) < 1e-4


def test_prediction_ensemble_input_gradient_only(device, monkeypatch):
    """The PredictionEnsemble's codec backward without weight gradients (the default: no slab rows,
    reductions or dense weight GEMM) moves q_z exactly as the full backward does, and leaves the
    model's decoder untouched."""
    from bottleneck.components import PredictionEnsemble
    from lamp.optimization import LearningScheduleWrapper
    d = load('pe_analysis_c32.npz')
    out = {}
    for flag in ('1', '0'):
        monkeypatch.setenv('GPI_PE_SHARED_GRADS', flag)
        model, ds = build(d)
        before = [p.detach().clone() for p in model.f.parameters()]
        pe = PredictionEnsemble(model, ds, LearningScheduleWrapper.Dummy(), lr=1e-2, writer=_Writer())
        pe.update(numIter=3, record=True, step=0, eps=[cuda(e) for e in d['pe_eps']])
        torch.cuda.synchronize()
        assert all(torch.equal(a, b.detach()) for a, b in zip(before, model.f.parameters()))
        out[flag] = (pe.q_z.mean.detach().clone(), pe.q_z.logsigma.detach().clone(), dict(pe.writer.d))
    assert torch.equal(out['1'][0], out['0'][0]) and torch.equal(out['1'][1], out['0'][1])
    assert out['1'][2] == out['0'][2]


def test_analysis_eval_all_y(device):
    from bottleneck.components import Analysis, VariationalApproximation
    d = load('pe_analysis_c32.npz')
    model, ds = build(d)
    n, nc, dz, Nval, Nmc, iters = [int(v) for v in d['cfg']]
    q = VariationalApproximation(dz, Nval, ds.get('X'))
    q.init(cuda(d['q_mean']), cuda(d['q_logsigma']))
    an = Analysis(q, model, ds)
    logscore, r2, relerr = an.eval_all_y(Nmc, eps=(cuda(d['an_eps_z']), cuda(d['an_eps_x']), cuda(d['an_eps_y'])))
    assert abs(logscore - float(d['logscore'])) <= 1e-4 * abs(float(d['logscore']))
    assert abs(r2 - float(d['r2'])) <= 1e-4 * abs(float(d['r2']))
    assert abs(relerr - float(d['relerr'])) <= 1e-4 * abs(float(d['relerr']))


@pytest.mark.parametrize('captured', [False, True])
def test_concurrent_prediction_ensemble_matches_sequential(device, tmp_path, captured):
    """ConcurrentPredictionEnsemble (the PE group of iteration n on a second stream, concurrently with
    training step n+1) leaves the model parameters and the PE's q_z exactly as the sequential
    schedule (step n, then the PE group on theta_{n+1}; training.py:417-419) does over five iterations,
    eager and as HIP graphs; the BN running buffers get the same number of updates (their EMA order
    differs by one step, documented)."""
    import sys
    sys.path.insert(0, __file__.rsplit('/', 1)[0])
    from test_gpu_training import _setup
    from gpi.train import FusedElboStep
    from gpi.predictive import PredictionEnsembleEngine, ConcurrentPredictionEnsemble
    from bottleneck.components import VariationalApproximation
    out = {}
    for conc in (False, True):
        model, val = _setup(tmp_path / ('c' if conc else 's'), seed=0)
        ds_u, ds_s = model._datasets['unsupervised'], model._datasets['supervised']
        step = FusedElboStep(model, ds_u.get('X'), 32, ds_s.get('X'), ds_s.get('Y'), ds_s.get('F_ROM_BC'),
                             lr=1e-2, seed=3)
        Xv = val.get('X').contiguous().float()
        q = VariationalApproximation(model.dim_latent, Xv.shape[0], Xv).to('cuda')
        torch.manual_seed(9)
        pe = PredictionEnsembleEngine(model, q, Xv, lambda: 1e-2, running_stage=conc)
        if captured:
            step.capture()
        if conc:
            cpe = ConcurrentPredictionEnsemble(pe, 3)
            if captured:
                cpe.capture()
            for _ in range(5):
                cpe.before_step()
                step.step()
                cpe.after_step()
            cpe.catch_up()
        else:
            for _ in range(5):
                step.step()
                for i in range(3):
                    pe.update(sync=i == 0)
        torch.cuda.synchronize()
        out[conc] = (step.flat.P.clone(), pe.flat.P[pe.q_off:].clone(),
                     {n: b.clone() for n, b in model.f.named_buffers()})
    assert torch.equal(out[False][0], out[True][0])
    assert torch.equal(out[False][1], out[True][1])
    for n, b in out[False][2].items():
        c = out[True][2][n]
        if n.endswith('num_batches_tracked'):
            assert torch.equal(b, c), n
        else:
            assert torch.isfinite(c).all() and (c - b).abs().max() <= 0.25 * b.abs().max() + 0.05, n


def test_pe_running_stage_fold_exact(device):
    """ConcurrentPredictionEnsemble's BN running-statistics fold, pinned exactly: one PE
    group of 3 iterations with running_stage=True (the calls' EMA updates go to the zeroed staging
    buffers of the shadow decoder), folded as running = (1 - m)^3 running + staged, equals the same
    group run with running_stage=False (every call updates model.f's buffers directly) to fp32 rounding
    (2e-6 relative); num_batches_tracked equal, staging buffers zeroed by the fold, q_z identical.  A
    wrong decay exponent or momentum, or a missed zeroing, moves the buffers by >= 1e-2 relative."""
    from gpi.predictive import PredictionEnsembleEngine, ConcurrentPredictionEnsemble
    from bottleneck.components import VariationalApproximation
    d = load('pe_analysis_c32.npz')
    out = {}
    for stage in (False, True):
        model, ds = build(d)
        n, nc, dz, Nval, Nmc, iters = [int(v) for v in d['cfg']]
        q = VariationalApproximation(dz, Nval, ds.get('X')).to('cuda')
        q.init(cuda(d['q_mean']), cuda(d['q_logsigma']))
        before = {k: b.clone() for k, b in model.f.named_buffers()}
        torch.manual_seed(9)
        pe = PredictionEnsembleEngine(model, q, ds.get('X').contiguous().float(), lambda: 1e-2, running_stage=stage)
        for i in range(3):
            pe.update(sync=i == 0)
        if stage:
            cpe = ConcurrentPredictionEnsemble(pe, 3)
            cpe._fold()
            for b in cpe._fl_stage + cpe._nb_stage:
                assert not b.any()
        torch.cuda.synchronize()
        out[stage] = ({k: b.clone() for k, b in model.f.named_buffers()}, pe.flat.P[pe.q_off:].clone(), before)
    direct, staged = out[False][0], out[True][0]
    assert torch.equal(out[False][1], out[True][1])
    moved = 0
    for k, b in direct.items():
        c = staged[k]
        if k.endswith('num_batches_tracked'):
            assert torch.equal(b, c) and int(b) == int(out[False][2][k]) + 3, k
            continue
        err = ((c - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
        assert err < 2e-6, (k, err)
        moved += int(not torch.equal(b, out[False][2][k]))
    assert moved > 0
