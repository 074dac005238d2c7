"""Structured-grid closed forms that replace the reference's FEniCS assembly.

The reference builds its linear-elliptic operators with FEniCS on a
``UnitSquareMesh(nx_rom, ny_rom)`` refined ``num_refines`` times
(factories/model.py:130-133) with CG1 trial/test functions and a DG0
conductivity (physics/LinearEllipticFactories.py:199-221).  On that mesh the
P1 stiffness of a right-isosceles triangle (right-angle vertex r, legs to a
and b) is kappa/2 * [[2,-1,-1],[-1,1,0],[-1,0,1]]: the hypotenuse couples
nothing, so the assembled operator is a 5-point stencil

    (K u)_p = sum_{q in N4(p)} c_pq (u_p - u_q),
    c_pq    = 1/2 * (kappa of the triangles having edge pq as a leg),

for every h.  This module holds those closed forms (setup-time, host side,
float64) and the node/pixel orderings shared with the HIP kernels:

  * node (i, j) -> id i + (n+1) j, coordinates (i/n, j/n);
  * free nodes: 1 <= i <= n-1 (x=0 / x=1 are Dirichlet), ordered by id,
    i.e. free index = j (n-1) + (i-1);  d_y = (n+1)(n-1);
  * square (i, j) is split into T_lr (cell 2q) and T_ul (cell 2q+1),
    q = i + n j ("right" diagonal);
  * image pixel (r, c), row 0 = top  <->  square (i=c, j=n-1-r)
    (bottleneck/utils.py:69-98).
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


class StructuredGrid(object):
    """n x n squares on the unit square."""

    def __init__(self, n):
        self.n = int(n)
        n = self.n
        self.num_nodes = (n + 1) ** 2
        ii, jj = np.meshgrid(np.arange(n + 1), np.arange(n + 1))  # [j, i]
        self.node_i = ii.ravel()
        self.node_j = jj.ravel()
        self.coords = np.stack([self.node_i / n, self.node_j / n], 1)
        dirichlet = (self.node_i == 0) | (self.node_i == n)
        self.constrained_dofs = np.where(dirichlet)[0]
        self.free_dofs = np.where(~dirichlet)[0]
        self.dim_out = self.free_dofs.size             # d_y
        self.num_cells = 2 * n * n

    # ---------------------------------------------------------------- BCs
    def dirichlet_values(self, u, nodes=None):
        """NDP boundary: left u0(1-y)+u1 y, right u2(1-y)+u3 y
        (physics/LinearEllipticFactories.py:269-273)."""
        if nodes is None:
            nodes = self.constrained_dofs
        u0, u1, u2, u3 = [float(v) for v in u]
        y = self.node_j[nodes] / self.n
        left = u0 * (1 - y) + u1 * y
        right = u2 * (1 - y) + u3 * y
        return np.where(self.node_i[nodes] == 0, left, right)

    def full_force(self, u):
        """FULL_F_WITH_APPLIED_BC row (physics/BoundaryConditions.py:132-147):
        zero source (NDP), Dirichlet values on constrained nodes."""
        F = np.zeros(self.num_nodes)
        F[self.constrained_dofs] = self.dirichlet_values(u)
        return F

    def scatter(self, y_free, u):
        """scatter_restricted_solution (physics/LinearElliptic.py:103-118)."""
        out = np.zeros(self.num_nodes)
        out[self.constrained_dofs] = self.dirichlet_values(u)
        out[self.free_dofs] = y_free
        return out

    # -------------------------------------------------------- conductances
    def cell_kappa_from_image(self, kappa_img):
        """Both triangles of a square take the pixel value."""
        n = self.n
        img = np.asarray(kappa_img, dtype=np.float64)
        sq = img[..., ::-1, :]                       # [j, i]
        c = np.repeat(sq.reshape(img.shape[:-2] + (n * n,)), 2, axis=-1)
        return c

    def edge_conductances(self, kappa_cells):
        """Per-triangle kappa [.., 2n^2] -> horizontal c_h [n+1, n] (edge
        (i,j)-(i+1,j) at [j, i]) and vertical c_v [n, n+1] (edge
        (i,j)-(i,j+1) at [j, i])."""
        n = self.n
        k = np.asarray(kappa_cells, dtype=np.float64).reshape(n, n, 2)  # [j, i, {lr, ul}]
        lr, ul = k[..., 0], k[..., 1]
        ch = np.zeros((n + 1, n))
        ch[:n, :] += 0.5 * lr          # bottom edge of square (i,j): leg of T_lr
        ch[1:, :] += 0.5 * ul          # top edge of square (i,j): leg of T_ul
        cv = np.zeros((n, n + 1))
        cv[:, 1:] += 0.5 * lr          # right edge of square (i,j): leg of T_lr
        cv[:, :n] += 0.5 * ul          # left edge of square (i,j): leg of T_ul
        return ch, cv

    def stiffness(self, kappa_cells):
        """Assembled (all-node) stiffness as scipy CSR."""
        n = self.n
        ch, cv = self.edge_conductances(kappa_cells)
        rows, cols, vals = [], [], []
        jj, ii = np.meshgrid(np.arange(n + 1), np.arange(n), indexing='ij')
        p = (ii + (n + 1) * jj).ravel()
        q = p + 1
        c = ch.ravel()
        rows += [p, q, p, q]; cols += [p, q, q, p]; vals += [c, c, -c, -c]
        jj, ii = np.meshgrid(np.arange(n), np.arange(n + 1), indexing='ij')
        p = (ii + (n + 1) * jj).ravel()
        q = p + (n + 1)
        c = cv.ravel()
        rows += [p, q, p, q]; cols += [p, q, q, p]; vals += [c, c, -c, -c]
        K = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                          shape=(self.num_nodes, self.num_nodes))
        return K.tocsr()

    def assemble_system(self, kappa_cells, u):
        """Dirichlet-reduced (K_ff, f_eff = -K_fc g)  (LinearElliptic.py:137-159)."""
        K = self.stiffness(kappa_cells)
        c, f = self.constrained_dofs, self.free_dofs
        g = self.dirichlet_values(u)
        Kff = K[f][:, f]
        feff = -(K[f][:, c] @ g)
        return Kff, feff

    def solve(self, kappa_cells, u):
        """FOM solve on free dofs (LinearElliptic.py:85-101)."""
        Kff, feff = self.assemble_system(kappa_cells, u)
        return spla.spsolve(Kff.tocsc(), feff)

    # ---------------------------------------------------------- ROM tensor
    def rom_tensor(self):
        """M[:, :, t] = stiffness of cell t at kappa = 1 (ROM.py:46-53), dense."""
        nn = self.num_nodes
        M = np.zeros((nn, nn, self.num_cells))
        for t in range(self.num_cells):
            e = np.zeros(self.num_cells)
            e[t] = 1.0
            M[:, :, t] = self.stiffness(e).toarray()
        return M

    # -------------------------------------------------------- prolongation
    def prolongation_from(self, coarse, only_free=True):
        """W[p, k] = coarse P1 basis k at fine node p (components.py:38-60)."""
        r = self.n // coarse.n
        assert r * coarse.n == self.n
        nodes = self.free_dofs if only_free else np.arange(self.num_nodes)
        W = np.zeros((nodes.size, coarse.num_nodes))
        for row, p in enumerate(nodes):
            for k, w in coarse_interp_weights(self.node_i[p], self.node_j[p], r, coarse.n):
                W[row, k] += w
        return W


def coarse_interp_weights(i, j, r, nc):
    """P1 interpolation of fine node (i, j) from the coarse "/" mesh
    (r = refinement factor).  Returns [(coarse node id, weight)] x3."""
    I = min(i // r, nc - 1)
    J = min(j // r, nc - 1)
    xi = (i - I * r) / r
    eta = (j - J * r) / r
    n00 = I + (nc + 1) * J
    n10 = n00 + 1
    n01 = n00 + (nc + 1)
    n11 = n01 + 1
    if xi >= eta:    # T_lr = {v0, v1, v3}
        return [(n00, 1 - xi), (n10, xi - eta), (n11, eta)]
    return [(n00, 1 - eta), (n01, eta - xi), (n11, xi)]


def pixel_to_cells(img):
    """DG0 cell values from an image (bottleneck/utils.py:127-132)."""
    img = np.asarray(img)
    n = img.shape[-1]
    sq = img[..., ::-1, :].reshape(img.shape[:-2] + (n * n,))
    return np.repeat(sq, 2, axis=-1)
