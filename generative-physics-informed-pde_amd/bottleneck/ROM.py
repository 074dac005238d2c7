"""Coarse-grained model (reference bottleneck/ROM.py:5-104) on the native ROM kernel.

The reference keeps a dense FEniCS tensor M [n_c, n_c, n_T] and, per call,
forms K = M x^T, replaces the Dirichlet rows and runs a dense batched LU.
Here the operator is the closed-form stencil of the structured coarse mesh
(physics/grid.py) solved per sample in LDS by rom.hip; ``M`` is still
available (dense, built lazily) for callers that inspect it.
"""
import torch

from gpi import _lib as L
from gpi.native import RomOperatorFunction


class ROM(object):

    def __init__(self, grid, refine, dtype=torch.float32, device=None):
        self.grid = grid                 # physics.grid.StructuredGrid of the coarse mesh
        self.nc = grid.n
        self.refine = int(refine)
        self.dtype = dtype
        self.device = device
        self._bc_dofs = torch.tensor(grid.constrained_dofs, dtype=torch.long)
        self._free_dofs = torch.tensor(grid.free_dofs, dtype=torch.long)
        self._M = None

    @classmethod
    def FromPhysics(cls, physics, dtype=torch.float32, device=None):
        """physics: the 'rom' LinearEllipticPhysics (ROM.py:37-57); cap of 290 cells kept (ROM.py:43-44)."""
        if physics.grid.num_cells > 290:
            raise Exception('ROM exceeds intended maximum size')
        return cls(physics.grid, physics.refine_to_fom, dtype=dtype, device=device)

    @property
    def M(self):
        if self._M is None:
            self._M = torch.tensor(self.grid.rom_tensor(), dtype=self.dtype, device=self.device)
        return self._M

    @property
    def V_dim(self):
        return self.grid.num_nodes

    @property
    def Vc_dim(self):
        return self.grid.num_cells

    @property
    def dim_in(self):
        return self.Vc_dim

    @property
    def dim_out(self):
        return self.V_dim

    def __call__(self, X, F=None, ReturnStiffness=False):
        """Coarse solution u [N, n_c] of K(X) u = F with Dirichlet rows (X = conductivity)."""
        if F is None:
            raise DeprecationWarning
        if X.dim() < 2:
            X = X.unsqueeze(0)
        if F.dim() > 2:
            F = F.squeeze(2)
        _, uc = RomOperatorFunction.apply(X, F, self.nc, self.refine, True)
        if ReturnStiffness:
            return uc, self.GetStiffness(X)
        return uc

    def GetStiffness(self, x, DirichletBC=True):
        """Dense K [n_c, n_c, N] (inspection only; the solve never forms it)."""
        K = torch.matmul(self.M.to(x.device), x.t())
        if DirichletBC:
            K[self._bc_dofs] = 0
            K[self._bc_dofs, self._bc_dofs] = 1
        return K

    def __repr__(self):
        return 'ROM (native stencil, %dx%d coarse squares) | Maps: %d -> %d' % (self.nc, self.nc, self.Vc_dim,
                                                                                 self.V_dim)
