"""End-to-end training smoke: the reference's Trainer.run loop body
(training.py:403-455) driven through the drop-in modules on the native path, BASELINE config 1 sizes
(32x32, 16 labeled + 64 unlabeled), 50 steps:

    optimizer.zero_grad(); elbo = model.elbo(...); (-elbo).backward(); optimizer.step()
    PE.update(3); scheduler_wrapper.step('training', metric=elbo)

with ModelFactory('highres32').setup(), DataFactory device-side data generation (random fields +
FOM labels on the GPU), torch Adam over model.parameters(), LearningScheduleWrapper.MultiStepLR and
PredictionEnsemble; then the same with the fused graph-captured step.  The ELBO must rise (the
objective is maximised): mean of the last 10 steps above the mean of the first 10, all finite."""
import math
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_STEPS = 50


def _setup(tmp_path, seed=0):
    from factories.model import ModelFactory
    from factories.data import DataFactory
    from utils.data import DataSet
    torch.manual_seed(seed)
    fac = ModelFactory.FromIdentifier('highres32')
    fac.set('device', 'cuda')
    physics, model, _, encoder, dtype, device = fac.setup()
    df = DataFactory.FromIdentifier('highres32', device=device, seed=seed, path=str(tmp_path) + '/')
    dl, dlu = df.setup()
    dl.assemble(physics, indices=range(32), device=device)         # FOM labels on the GPU
    sup = DataSet(dl, np.arange(16), device=device, label='supervised')
    val = DataSet(dl, np.arange(16, 32), device=device, label='validation')
    unsup = DataSet(dlu, np.arange(64), device=device, label='unsupervised')
    model.encoder = encoder
    model.register_datasets({'supervised': sup, 'unsupervised': unsup}, None,
                            create_unsupervised_variational_approximation=False)
    return model, val


def test_trainer_loop_module_path(device, tmp_path):
    from lamp.optimization import LearningScheduleWrapper
    from bottleneck.components import PredictionEnsemble, Analysis
    model, val = _setup(tmp_path)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)                      # training.py:254
    sw = LearningScheduleWrapper.MultiStepLR([20, 40], factor=math.sqrt(0.1))  # training.py:615
    sw.register_optimizer(opt, 'training')
    pe = PredictionEnsemble(model, val, sw, lr=1e-2)
    elbos = []
    with warnings.catch_warnings():
        # the PredictionEnsemble's native q_z update reports its optimizer step to torch's scheduler
        # hook (no "lr_scheduler.step() before optimizer.step()" warning for the 'validation' schedule)
        warnings.filterwarnings('error', message='.*lr_scheduler.step.*')
        for n in range(N_STEPS):
            opt.zero_grad()
            elbo = model.elbo(step=n, armortized_bs=32)
            (-elbo).backward()
            opt.step()
            pe.update(3, step=n)
            sw.step('training', metric=elbo)
            elbos.append(elbo.item())
    assert all(math.isfinite(e) for e in elbos)
    assert np.mean(elbos[-10:]) > np.mean(elbos[:10]), elbos
    assert opt.param_groups[0]['lr'] == pytest.approx(1e-3, rel=1e-6)     # two milestones x sqrt(0.1)
    for _ in range(3):                                                     # training.py:457-460
        pe.update(3, step=N_STEPS)
    logscore, r2, relerr = Analysis(pe.q_z, model, val).eval_all_y(16)
    assert all(math.isfinite(float(v)) for v in (logscore, r2, relerr))


def test_trainer_loop_fused_step(device, tmp_path):
    from lamp.optimization import LearningScheduleWrapper
    from gpi.train import FusedElboStep
    model, _ = _setup(tmp_path, seed=1)
    ds_s, ds_u = model.datasets['supervised'], model.datasets['unsupervised']
    step = FusedElboStep(model, ds_u.get('X'), 32, ds_s.get('X'), ds_s.get('Y'), ds_s.get('F_ROM_BC'), lr=1e-2,
                         seed=3)
    sw = LearningScheduleWrapper.MultiStepLR([20, 40], factor=math.sqrt(0.1))
    sw.register_optimizer(step.optimizer, 'training')
    step.capture()
    elbos = []
    with warnings.catch_warnings():
        # the fused step reports its optimizer step to torch's scheduler hook (no "lr_scheduler.step()
        # before optimizer.step()" warning)
        warnings.filterwarnings('error', message='.*lr_scheduler.step.*')
        for n in range(N_STEPS):
            step.step()
            sw.step('training', metric=None)
            elbos.append(step.elbo())
    elbos = [float(e.item()) for e in elbos]
    assert all(math.isfinite(e) for e in elbos)
    assert np.mean(elbos[-10:]) > np.mean(elbos[:10]), elbos
    assert step.lr.item() == pytest.approx(1e-3, rel=1e-5)
    step.engine.check_flag()
