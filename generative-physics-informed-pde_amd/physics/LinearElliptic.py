"""Linear-elliptic physics -div(kappa grad u) = 0 on the structured unit-square mesh.

Replaces LinearEllipticPhysics (reference physics/LinearElliptic.py:8-159) and
the NDP factory (physics/LinearEllipticFactories.py:182-285): CG1 solution,
DG0 (per-triangle) conductivity, Dirichlet data on x=0 / x=1 linear in y,
homogeneous Neumann on y=0 / y=1, zero source.  Assembly is the closed-form
stencil of physics/grid.py instead of FEniCS.  Setup-side (host, float64).
"""
import numpy as np

from physics.grid import StructuredGrid


def GetFactory(id):
    """Reference quirk kept: 'ND' compares id.lower() == 'ND' and is unreachable
    (physics/LinearEllipticFactories.py:11)."""
    if id.lower() == 'ND':
        raise AssertionError('unreachable')
    if id.lower() == 'ndp':
        return 'NDP', 2
    raise NotImplementedError('physics type %r (only NDP is reachable in the reference)' % id)


class LinearEllipticPhysics(object):

    def __init__(self, identifier, physics_id, n, refine_to_fom=1):
        GetFactory(physics_id)
        self.identifier = identifier
        self.physics_id = 'NDP'
        self.grid = StructuredGrid(n)
        self.refine_to_fom = int(refine_to_fom)

    @property
    def free_dofs(self):
        return self.grid.free_dofs

    @property
    def constrained_dofs(self):
        return self.grid.constrained_dofs

    @property
    def tdim(self):
        return 2

    @property
    def dim_in(self):
        return self.grid.num_cells

    @property
    def dim_out(self):
        return self.grid.dim_out

    @property
    def dim_out_all(self):
        return self.grid.num_nodes

    def set_x(self, x):
        if np.any(np.asarray(x) <= 0):
            raise ValueError('Trying to set negative or zero material values')

    def assemble_system(self, x, bc, *, only_free_dofs=True):
        """(K_ff, f_eff) for conductivity x per cell (LinearElliptic.py:137-159)."""
        self.set_x(x)
        if not only_free_dofs:
            return self.grid.stiffness(x), np.zeros(self.grid.num_nodes)
        return self.grid.assemble_system(x, _bc_values(bc))

    def solve(self, x, bc, only_free_dofs=True, ReturnType='numpy'):
        self.set_x(x)
        y = self.grid.solve(x, _bc_values(bc))
        return y if only_free_dofs else self.grid.scatter(y, _bc_values(bc))

    def scatter_restricted_solution(self, y, bc, ReturnFunction=False):
        return self.grid.scatter(y, _bc_values(bc))


def _bc_values(bc):
    return bc.u if hasattr(bc, 'u') else np.asarray(bc, dtype=np.float64)
