"""Flux constraints (reference bottleneck/flux.py:7-158) on the native path.

The reference builds, per coarse cell, a FEniCS form summing kappa grad(u).n
over the fine facets lying on the cell's edges (ds on the Dirichlet edges,
'+'-restricted dS elsewhere) and assembles its derivative w.r.t. u for every
VO sample.  Here the rows come from the closed-form facet fluxes of the
structured P1 mesh (csrc/vo.hip, vo_query_flux; gpi_cgr_residual's r_flux for
the residual Gamma_fc y itself).

'+' side: DOLFIN's interior-facet assembler takes the first cell of the facet
as '+' and swaps the pair when the form carries cell domains with a larger
marker on the other side; FluxForm.append_dx attaches the cell function that
marks the fine cells of coarse cell k with 1 (flux.py:128-135), so '+' is the
fine cell inside coarse cell k: every row is the OUTWARD flux of its coarse
cell.  dS over the y=0 / y=1 boundary facets integrates nothing.  The
reduced alpha is the (negated) dot product with the zero-initialised
self.Gamma (flux.py:153-156), i.e. identically 0 -- kept.
"""
import numpy as np
import torch

from gpi import _lib as L
from gpi import vo as V


class FluxConstraintReducedOrderModel(object):

    def __init__(self, physics, bc=None):
        self._physics = physics
        self.n_fine = physics['fom'].grid.n
        self.nc = physics['rom'].grid.n
        self._initialized = False

    @property
    def initialized(self):
        return self._initialized

    @property
    def tdim(self):
        return 2

    @property
    def N(self):
        return 2 * self.nc * self.nc

    def create_measures(self):
        self._initialized = True

    def assemble_reduced(self, x, bc, device=None):
        """(Gamma_reduced [N, d_y], alpha_reduced [N]) for conductivity x per DG0 cell (fp64 device tensors)."""
        if not self._initialized:
            self.create_measures()
        dev = device if device is not None else torch.device('cuda')
        lx = torch.log(torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)).view(1, -1)
        u = torch.as_tensor(bc.u if hasattr(bc, 'u') else np.asarray(bc, dtype=np.float64),
                            dtype=torch.float64, device=dev).view(1, 4)
        g, a = V.vo_query(lx, u, self.n_fine, self.nc, L.VO_FLUX)
        return g[0], a[0]
