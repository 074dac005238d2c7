"""Data factories (reference factories/data.py:1-101): identifier -> (dataloader, unsupervised dataloader).

``DataFactory.FromIdentifier('highres' | 'highres32' | 'highres128' | 'highres256').setup()`` loads
``cdata/<identifier>.pt`` / ``.ptu`` when present, else draws the images from the factory's
random-field sampler and saves them (factories/data.py:49-61).  ``device`` moves the draw (and,
through DataLoader.assemble(device=...), the FOM labels) onto the GPU; the host path draws with
numpy as before.  The unsupervised pool is locked against physics assembly (:67).
"""
import os

import numpy as np

from physics.RandomField import NormalRandomFieldSampler
from utils.data import DataLoader

DATAPATH = 'cdata/'


def ensure_file_extension(file, extension):
    return file if file.endswith(extension) else file + extension


class DataFactory(object):

    def __init__(self, config=None, device=None, seed=0, path=None):
        self.config = config
        self._forced_setup = False
        self._identifier = None
        self._device = device
        self._seed = int(seed)
        self._path = path

    @property
    def path(self):
        return self._check_path(self._path if self._path is not None else DATAPATH)

    def _check_path(self, path):
        if path[-1] != '/':
            raise ValueError('path must end with a backslash | path= {}'.format(path))
        return path

    @property
    def identifier(self):
        return self._identifier if self._identifier is not None else type(self).__name__

    @classmethod
    def FromIdentifier(cls, identifier, *args, **kwargs):
        factory_class = _FACTORIES.get(identifier)   # capitalisation has to match (:37-43)
        if factory_class is None:
            raise KeyError('DataFactory cannot provide factory for specified identifier {}'.format(identifier))
        return factory_class(*args, **kwargs)

    @classmethod
    def FromRandomFieldSampler(cls, rfs, N, N_unsupervised):
        raise NotImplementedError

    def _create_dataloader(self, N, identifier, extension, sub):
        file = ensure_file_extension(self.path + identifier, extension)
        if os.path.exists(file) and not self._forced_setup:
            return DataLoader.FromFile(file)
        print('Could not find {} to load dataset (or forced); creating from sampler... '.format(file))
        rng = np.random.default_rng((self._seed, sub))
        dl = DataLoader.FromSampler(self._rfs, N, rng=rng, device=self._device, seed=self._seed * 2 + sub)
        os.makedirs(os.path.dirname(file) or '.', exist_ok=True)
        dl.save(file)
        return dl

    def _create_dataloaders(self, rfs, N, N_unsupervised, identifier):
        dataloader = self._create_dataloader(N, identifier, '.pt', 0)
        dataloader_unsupervised = self._create_dataloader(N_unsupervised, identifier, '.ptu', 1)
        dataloader_unsupervised.lock_physics_assembly()
        return dataloader, dataloader_unsupervised

    def setup(self):
        return self._create_dataloaders(self._rfs, self._N, self._N_unsupervised, self.identifier)

    def force_setup(self):
        self._forced_setup = True
        return self.setup()


class highres(DataFactory):
    """64^2, 2048 labelled / 20480 unlabelled, l = 0.04, adaptive KL truncation (factories/data.py:80-89)."""

    def __init__(self, *args, **kwargs):
        super(highres, self).__init__(*args, **kwargs)
        self._N = 2 * 1024
        self._N_unsupervised = 2048 * 10
        self._rfs = NormalRandomFieldSampler.FromImage(64, 64, 0.4, 0.80, 0.04, Truncation='adaptive')


class highres32(DataFactory):
    """32^2, 1024 labelled / 20480 unlabelled, l = 0.15, full Cholesky (factories/data.py:91-100)."""

    def __init__(self, *args, **kwargs):
        super(highres32, self).__init__(*args, **kwargs)
        self._N = 1024
        self._N_unsupervised = 2048 * 10
        self._rfs = NormalRandomFieldSampler.FromImage(32, 32, 0.4, 0.80, 0.15, Truncation=None)


class highres128(DataFactory):
    """Beyond the reference's 8192-pixel cap (RandomField.py:43): separable sampler at 128^2."""

    def __init__(self, *args, **kwargs):
        super(highres128, self).__init__(*args, **kwargs)
        self._N = 1024
        self._N_unsupervised = 4096
        self._rfs = NormalRandomFieldSampler.FromImage(128, 128, 0.4, 0.80, 0.04, Truncation='adaptive')


class highres256(DataFactory):
    """Separable sampler at 256^2."""

    def __init__(self, *args, **kwargs):
        super(highres256, self).__init__(*args, **kwargs)
        self._N = 512
        self._N_unsupervised = 2048
        self._rfs = NormalRandomFieldSampler.FromImage(256, 256, 0.4, 0.80, 0.04, Truncation='adaptive')


_FACTORIES = {c.__name__: c for c in (highres, highres32, highres128, highres256)}
