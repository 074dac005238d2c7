"""The reference notebook's published run, end to end on the native path (statistical parity).

example.ipynb (cells 2-8) trains highres32 for 15,000 iterations and reports, after 250 final
PredictionEnsemble rounds, R^2 0.97996 and predictive log-score 2.3292 on the validation set
(example.ipynb:159-160, Analysis.eval_all_y with 1024 MC samples).  Configuration (cell 2):
dim_latent 16, ptype NDP, N_u = 1024 unlabeled with armortized batch 64, N_s = 128 labeled,
N_val = 128, N_vo = 0, lr 1e-2 for the model's Adam and the PredictionEnsemble's Adam, both under
MultiStepLR(milestones [250, 1500], factor sqrt(0.1)) stepped once per iteration
(training.py:452, components.py:385), 3 PE updates per iteration (training.py:419), monitoring
eval_all_y(64 MC) every 1000 iterations (training.py:421-428), final 250 x 3 PE updates +
eval_all_y(1024 MC) (training.py:457-460).  Data: factories/data.py highres32 (32x32 Gaussian
fields, mean 0.4, std 0.8, length 0.15, no truncation; FOM labels with random BCs), generated on
the device (DataFactory(device=...)); the reference's cdata/highres32.pt is not shipped, and the
RNG streams differ -- a statistical comparison, not a bitwise one.

Here: the fused native ELBO step (one HIP graph per iteration), the three PE updates in a second
graph, the schedulers' learning rates copied to the device when they change.

usage: python tools/notebook_run.py [iterations] [out.json]
"""
import json
import math
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'generative-physics-informed-pde_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

PUBLISHED = dict(r2_y=0.9799582958221436, logscore_y=2.329190492630005, it_s=35.57,
                 source='example.ipynb:112,159-160 (15,000 iterations, unnamed CUDA GPU, PyTorch 1.1)')


class _LrHandle(torch.optim.Optimizer):
    """The PE's learning rate as a torch optimizer for LearningScheduleWrapper (as FusedAdamSchedule)."""

    def __init__(self, lr):
        super().__init__([torch.zeros(1)], dict(lr=lr))

    def step(self, closure=None):
        return None


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 15000
    out = sys.argv[2] if len(sys.argv) > 2 else None
    torch.manual_seed(0)
    np.random.seed(0)
    dev = torch.device('cuda', 0)
    from factories.model import ModelFactory
    from factories.data import DataFactory
    from utils.data import DataSet
    from lamp.optimization import LearningScheduleWrapper
    from gpi.train import FusedElboStep
    from gpi.predictive import PredictionEnsembleEngine, ConcurrentPredictionEnsemble, predictive_y, predictive_scores
    from bottleneck.components import VariationalApproximation

    t_setup = time.perf_counter()
    fac = ModelFactory.FromIdentifier('highres32')
    fac.set('device', 'cuda')
    fac.set('dim_latent', 16)
    fac.set('ptype', 'NDP')
    physics, model, _, encoder, _, _ = fac.setup()
    tmp = tempfile.mkdtemp(prefix='nb32_')
    df = DataFactory.FromIdentifier('highres32', device=dev, seed=0, path=tmp + '/')
    dl, dlu = df.setup()
    N_s, N_val, N_u, bs = 128, 128, 1024, 64
    dl.assemble(physics, indices=range(N_s + N_val), device=dev)      # FOM labels on the GPU
    sup = DataSet(dl, np.arange(N_s), device=dev, label='supervised')
    val = DataSet(dl, np.arange(N_s, N_s + N_val), device=dev, label='validation')
    unsup = DataSet(dlu, np.arange(N_u), device=dev, label='unsupervised')
    model.encoder = encoder
    model.register_datasets({'supervised': sup, 'unsupervised': unsup}, None,
                            create_unsupervised_variational_approximation=False)
    Xu = unsup.get('X').contiguous().float()
    Xs, Ys, Fs = sup.get('X'), sup.get('Y'), sup.get('F_ROM_BC')
    Xv, Yv, Fv = val.get('X').contiguous().float(), val.get('Y').contiguous().float(), val.get('F_ROM_BC')

    sw = LearningScheduleWrapper.MultiStepLR([250, 1500], factor=math.sqrt(0.1))     # training.py:615
    step = FusedElboStep(model, Xu, bs, Xs, Ys, Fs, lr=1e-2, seed=1234)
    sw.register_optimizer(step.optimizer, 'training')
    q_val = VariationalApproximation(model.dim_latent, N_val, Xv).to(dev)
    pe_lr = _LrHandle(1e-2)
    sw.register_optimizer(pe_lr, 'validation')                                       # components.py:337
    pe = PredictionEnsembleEngine(model, q_val, Xv, lambda: pe_lr.param_groups[0]['lr'], running_stage=True)
    pe._sync_lr()
    step.capture()
    # the PE group of iteration n-1 runs concurrently with training step n (same parameters and q_z as
    # the sequential loop; gpi.predictive.ConcurrentPredictionEnsemble)
    cpe = ConcurrentPredictionEnsemble(pe, 3)
    cpe.capture()
    t_setup = time.perf_counter() - t_setup

    def monitor(n_mc):
        mean, std = predictive_y(model, q_val.mean, q_val.logsigma, Fv, n_mc)
        relerr, logscore, r2 = predictive_scores(Yv, mean, std)
        return dict(relerr_y=relerr, logscore_y=logscore, r2_y=r2)

    history = []
    t0 = time.perf_counter()
    for n in range(iters):
        cpe.before_step()
        step.step()
        cpe.after_step()
        if n % 1000 == 0 and n > 0:                               # training.py:421-428
            cpe.catch_up()                                        # PE(n) done: the reference's order
            m = monitor(64)
            m.update(iteration=n, elbo=float(step.elbo().item()), lr=step.optimizer.param_groups[0]['lr'])
            history.append(m)
            sys.stderr.write('[nb] %s\n' % json.dumps(m))
            sys.stderr.flush()
        sw.step('training')                                       # training.py:452
        sw.step('validation')                                     # components.py:385, once per update(3)
        step.sync_lr()
    cpe.catch_up()
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    # final: 250 rounds of 3 PE updates, then eval_all_y with 1024 MC samples (training.py:457-460)
    t1 = time.perf_counter()
    for _ in range(250):
        pe._sync_lr()
        cpe.graph.replay()
        cpe._fold()
        sw.step('validation')
    final = monitor(1024)
    torch.cuda.synchronize()
    t_final = time.perf_counter() - t1
    step.engine.check_flag()
    res = dict(metric='notebook run (example.ipynb) final validation scores', iterations=iters,
               r2_y=final['r2_y'], logscore_y=final['logscore_y'], relerr_y=final['relerr_y'],
               published=PUBLISHED, it_s=round(iters / t_train, 1), train_s=round(t_train, 2),
               final_s=round(t_final, 2), setup_s=round(t_setup, 2), elbo_last=float(step.elbo().item()),
               history=history, n_gpus=1, dtype='f32',
               data='device-generated highres32 fields + FOM labels (the reference cdata file is not shipped)',
               note='statistical parity only: RNG streams and data draws differ from the reference run')
    print(json.dumps(res))
    if out:
        with open(out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
