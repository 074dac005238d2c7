"""lamp.optimization -- LearningScheduleWrapper (reference lamp/optimization.py:5-94).

Keeps one torch LR scheduler per registered optimizer id and steps it every
``interval`` calls.  Same constructors (stepLR, MultiStepLR,
ReduceLROnPlateau, Dummy) and call signature ``step(id, N, N_max, interval,
metric)`` as the reference, so training.py drives it unchanged.
"""
import torch


class LearningScheduleWrapper(object):

    def __init__(self, create_scheduler, disable=False):
        self._factory = create_scheduler
        self._disable = disable
        self._entries = {}          # id -> [optimizer, scheduler, counter]

    # ------------------------------------------------------------ factories
    @classmethod
    def stepLR(cls, step_size, factor=0.1):
        return cls(lambda opt: torch.optim.lr_scheduler.StepLR(opt, step_size=step_size, gamma=factor))

    @classmethod
    def MultiStepLR(cls, milestones, factor, last_epoch=-1):
        assert factor < 1
        return cls(lambda opt: torch.optim.lr_scheduler.MultiStepLR(opt, milestones=milestones, gamma=factor,
                                                                    last_epoch=last_epoch))

    @classmethod
    def ReduceLROnPlateau(cls, patience, threshold=1e-3, factor=0.1, min_lr=1e-3, verbose=True, mode='max'):
        assert factor < 1
        return cls(lambda opt: torch.optim.lr_scheduler.ReduceLROnPlateau(
            opt, mode=mode, patience=patience, threshold=threshold, factor=factor, min_lr=min_lr))

    @classmethod
    def Dummy(cls):
        w = cls(lambda opt: None)
        w.lock()
        return w

    # ------------------------------------------------------------------ api
    def lock(self):
        self._disable = True

    def unlock(self):
        self._disable = False

    def register_optimizer(self, optimizer, id):
        self._entries[id] = [optimizer, self._factory(optimizer), 0]

    def set_learning_rate_manually(self, id, lr):
        for group in self._entries[id][0].param_groups:
            group['lr'] = lr

    def step(self, id, N=None, N_max=None, interval=1, metric=None):
        if id not in self._entries:
            raise ValueError('LearningScheduleWrapper does not have "{}" optimizer registered'.format(id))
        entry = self._entries[id]
        entry[2] += 1
        if self._disable:
            return
        if entry[2] % (interval or 1):
            return
        sched = entry[1]
        if isinstance(sched, torch.optim.lr_scheduler.ReduceLROnPlateau):
            if metric is None:
                raise ValueError('ReduceLROnPlateau requires metric')
            sched.step(metric)
        else:
            sched.step()
