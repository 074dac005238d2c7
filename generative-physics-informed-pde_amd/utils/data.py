"""Datasets (reference utils/data.py:8-459): images, labels, BCs, restrictions.

``DataLoader`` holds N log-conductivity images with their boundary
conditions and (after ``assemble``) the FOM labels Y on the fine free nodes
and the coarse F_ROM_BC vectors (utils/data.py:72-103; setup-side, float64,
structured-grid solves instead of FEniCS).  With ``device`` set, the images
are drawn and the labels solved on the GPU (gpi.fom: batched PCG on the
stencil, separable random-field sampler); otherwise on the host (scipy).  ``DataSet`` is a view
on a subset of indices with device-cached tensors and the reference's
``get(key, random_subset)`` semantics (utils/data.py:419-445).
"""
import numpy as np
import torch

from physics.BoundaryConditions import BoundaryConditionEnsemble
from physics.grid import pixel_to_cells


class DataLoader(object):

    def __init__(self, X, bce=None):
        self.X = np.asarray(X, dtype=np.float64)        # [N, py, px] log-conductivity images
        self.BCE = bce if bce is not None else BoundaryConditionEnsemble.FromFactory(self.X.shape[0])
        self.X_DG = None
        self.Y = None
        self.F_ROM_BC = None
        self.fom_iters = None
        self._lock_physics_assembly = False

    @classmethod
    def FromSampler(cls, sampler, N, rng=None, device=None, seed=0):
        """N images from ``sampler`` (utils/data.py:312-325) and N random NDP conditions.
        device: draw the images on the GPU (Philox stream ``seed``) instead of with ``rng``."""
        rng = rng or np.random
        if device is not None:
            X = sampler.sample_device(N, seed=seed, device=device).cpu().numpy()
        else:
            X = sampler.sample(batch_size=N, rng=rng)
        return cls(X, BoundaryConditionEnsemble.FromFactory(N, rng))

    def lock_physics_assembly(self):
        """Unsupervised pools are never assembled (utils/data.py:66-67,74-75)."""
        self._lock_physics_assembly = True

    @property
    def N(self):
        return self.X.shape[0]

    def assemble(self, physics, indices=None, solve=True, device=None, rtol=1e-13):
        """X_DG, FOM labels Y (free dofs) and F_ROM_BC for ``indices`` (default: all).
        device: solve on the GPU (one batched gpi_fom_solve launch) instead of per-sample scipy."""
        if self._lock_physics_assembly:
            raise RuntimeError('physics assembly is locked for this dataloader')
        fom, rom = physics['fom'], physics['rom']
        self.BCE.register_function_space('fom', fom)
        self.BCE.register_function_space('rom', rom)
        self.X_DG = pixel_to_cells(self.X)
        self.F_ROM_BC = self.BCE.FULL_F_WITH_APPLIED_BC('rom')
        if solve:
            idx = np.arange(self.N) if indices is None else np.asarray(list(indices), dtype=np.int64)
            Y = np.full((self.N, fom.dim_out), np.nan)
            if device is not None:
                import torch as _t
                from gpi import fom as gfom
                xd = _t.tensor(self.X_DG[idx], dtype=_t.float64, device=device)
                bc = _t.tensor(self.BCE.U[idx], dtype=_t.float64, device=device)
                res = gfom.fom_solve(xd, bc, fom.grid.n, rtol=rtol).check()
                Y[idx] = res.y.cpu().numpy()
                self.fom_iters = res.iters.cpu().numpy()
            else:
                for n in idx:
                    Y[n] = fom.grid.solve(np.exp(self.X_DG[n]), self.BCE[n].u)
            self.Y = Y
        return self

    def save(self, path):
        """torch.save of {'X': double [N, py, px], ...} (utils/data.py:284-291); the NDP
        encodings are stored beside the images so labels can be re-assembled identically."""
        if len(path.split('.')) == 1:
            raise ValueError(path)
        torch.save({'X': torch.tensor(self.X), 'U': torch.tensor(self.BCE.U)}, path)

    @classmethod
    def FromFile(cls, path):
        d = torch.load(path, weights_only=True, map_location='cpu')
        X = d['X'].numpy()
        if 'U' in d:
            return cls(X, BoundaryConditionEnsemble.FromEncoding(d['U'].numpy()))
        return cls(X)   # reference files hold {'X', 'hash'} only: fresh NDP conditions (utils/data.py:62-68)


class DataSet(object):

    VALID = ('X', 'X_DG', 'Y', 'F_ROM_BC', 'BCE')

    def __init__(self, dataloader, indices, dtype=torch.float32, device=None, label=''):
        self._dl = dataloader
        self.indices = np.asarray(indices, dtype=np.int64)
        self._dtype = dtype
        self._device = device
        self._cache = {}
        self.label = label

    @property
    def N(self):
        return self.indices.size

    def __len__(self):
        return self.N

    def __bool__(self):
        return self.N > 0

    def restrict(self, N):
        self.indices = self.indices[:N]
        self._cache = {}

    def get(self, key, random_subset=None):
        if key not in self.VALID:
            raise ValueError(key)
        if key not in self._cache:
            if key == 'BCE':
                q = self._dl.BCE[list(self.indices)]
            else:
                q = torch.tensor(getattr(self._dl, key)[self.indices])
                if key in ('X', 'Y', 'F_ROM_BC'):
                    q = q.to(dtype=self._dtype, device=self._device).contiguous()
            self._cache[key] = q
        if random_subset is None:
            return self._cache[key]
        perm = torch.randperm(self.N, dtype=torch.long, device=self._device)
        return self._cache[key][perm[0:random_subset]]

    def __repr__(self):
        return 'Virtual dataset with {} datapoints | {}'.format(self.N, self.label)
