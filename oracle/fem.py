"""Generic P1 finite-element restatement of the reference's FEniCS setup.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  numpy float64.

This is deliberately the *generic* FE algorithm -- element matrices from
barycentric gradients, scatter-assembly, point location + barycentric
evaluation, facet integrals -- and NOT the closed-form 5-point stencils the
product kernels use, so that agreement between the two pins the stencil
derivation.

Mesh conventions (the build's ordering; DOLFIN's own numbering of a refined
mesh cannot be reproduced without DOLFIN, so parity is defined on this
ordering -- the reference's torch code is ordering-agnostic given consistent
M / W / F / Y):
  * ``UnitSquareMesh(n, n)`` with DOLFIN's default "right" diagonal
    (factories/model.py:132): square (i, j) has corners v0=(i,j), v1=(i+1,j),
    v2=(i,j+1), v3=(i+1,j+1) and is split into T_lr={v0,v1,v3} (cell 2q) and
    T_ul={v0,v2,v3} (cell 2q+1), q = i + n*j.
  * node (i, j) has id i + (n+1)*j and coordinates (i/n, j/n).
  * ``refine`` (fawkes/utils.py:9-14) splits every triangle into four by edge
    midpoints; ``refine_mesh`` below does exactly that on a generic triangle
    list and tests check it reproduces the structured mesh at n*2^r.
  * Dirichlet boundary = x=0 ("left") and x=1 ("right")
    (physics/LinearEllipticFactories.py:27-30,273); constrained dofs sorted by
    node id; free dofs = the rest, sorted by node id.
  * pixel (r, c) of an image (row 0 = top) <-> square (i=c, j=n-1-r); both
    triangles of the square take the pixel value (bottleneck/utils.py:69-98).
"""
import numpy as np

LOG2PI = 1.8378770664093453


# --------------------------------------------------------------------------
# meshes
# --------------------------------------------------------------------------
class TriMesh(object):
    """Plain triangle mesh: ``coords`` [nv, 2], ``cells`` [nc, 3]."""

    def __init__(self, coords, cells):
        self.coords = np.asarray(coords, dtype=np.float64)
        self.cells = np.asarray(cells, dtype=np.int64)

    @property
    def num_vertices(self):
        return self.coords.shape[0]

    @property
    def num_cells(self):
        return self.cells.shape[0]


def unit_square_mesh(n):
    """UnitSquareMesh(n, n), "right" diagonal (factories/model.py:132)."""
    xs = np.arange(n + 1) / n
    X, Y = np.meshgrid(xs, xs)              # [j, i]
    coords = np.stack([X.ravel(), Y.ravel()], 1)
    cells = []
    for j in range(n):
        for i in range(n):
            v0 = i + (n + 1) * j
            v1 = v0 + 1
            v2 = v0 + (n + 1)
            v3 = v2 + 1
            cells.append((v0, v1, v3))
            cells.append((v0, v2, v3))
    return TriMesh(coords, cells)


def refine_mesh(mesh):
    """Uniform red refinement: each triangle -> 4 via edge midpoints."""
    coords = [tuple(c) for c in mesh.coords]
    index = {c: k for k, c in enumerate(coords)}

    def vid(p):
        key = (round(p[0], 14), round(p[1], 14))
        if key not in index:
            index[key] = len(coords)
            coords.append(key)
        return index[key]

    # re-key existing vertices with the same rounding
    index = {(round(c[0], 14), round(c[1], 14)): k for k, c in enumerate(coords)}
    cells = []
    C = mesh.coords
    for a, b, c in mesh.cells:
        ab = vid(0.5 * (C[a] + C[b]))
        bc = vid(0.5 * (C[b] + C[c]))
        ca = vid(0.5 * (C[c] + C[a]))
        cells += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
    return TriMesh(np.array(coords), cells)


def same_triangulation(m1, m2, tol=1e-12):
    """True if two meshes have the same vertex set and the same triangles."""
    def key(m):
        tris = set()
        for cell in m.cells:
            pts = sorted((round(m.coords[v][0] / tol) * tol, round(m.coords[v][1] / tol) * tol)
                         for v in cell)
            tris.add(tuple(pts))
        return tris
    return key(m1) == key(m2)


# --------------------------------------------------------------------------
# P1 element algebra
# --------------------------------------------------------------------------
def barycentric_gradients(p):
    """p: [3,2] triangle vertices -> (area, grads [3,2])."""
    x0, y0 = p[0]
    x1, y1 = p[1]
    x2, y2 = p[2]
    det = (x1 - x0) * (y2 - y0) - (x2 - x0) * (y1 - y0)
    area = 0.5 * abs(det)
    grads = np.array([[y1 - y2, x2 - x1],
                      [y2 - y0, x0 - x2],
                      [y0 - y1, x1 - x0]]) / det
    return area, grads


def element_stiffness(p):
    """int_T grad(phi_a).grad(phi_b) dx for P1 on triangle p (kappa = 1)."""
    area, g = barycentric_gradients(p)
    return area * g @ g.T


def assemble_stiffness(mesh, kappa_cells):
    """a = kappa grad(u).grad(v) dx, CG1 x DG0 kappa (LinearEllipticFactories.py:219)."""
    nv = mesh.num_vertices
    K = np.zeros((nv, nv))
    for t, cell in enumerate(mesh.cells):
        Ke = element_stiffness(mesh.coords[cell]) * kappa_cells[t]
        K[np.ix_(cell, cell)] += Ke
    return K


def apply_stiffness(mesh, kappa_cells, u_full):
    """K u without forming K: vectorised element loop (same element algebra as
    assemble_stiffness), usable at 128^2 / 256^2 where a dense K does not fit."""
    P = mesh.coords[mesh.cells]                              # [nc, 3, 2]
    x0, y0 = P[:, 0, 0], P[:, 0, 1]
    x1, y1 = P[:, 1, 0], P[:, 1, 1]
    x2, y2 = P[:, 2, 0], P[:, 2, 1]
    det = (x1 - x0) * (y2 - y0) - (x2 - x0) * (y1 - y0)
    g = np.stack([np.stack([y1 - y2, x2 - x1], -1), np.stack([y2 - y0, x0 - x2], -1),
                  np.stack([y0 - y1, x1 - x0], -1)], 1) / det[:, None, None]
    Ke = (0.5 * np.abs(det) * np.asarray(kappa_cells, dtype=np.float64))[:, None, None] * np.einsum(
        'cad,cbd->cab', g, g)
    contrib = np.einsum('cab,cb->ca', Ke, np.asarray(u_full, dtype=np.float64)[mesh.cells])
    out = np.zeros(mesh.num_vertices)
    np.add.at(out, mesh.cells, contrib)
    return out


def rom_stiffness_tensor(mesh):
    """M[:, :, t] = d a / d kappa_t  (bottleneck/ROM.py:46-53)."""
    nv = mesh.num_vertices
    M = np.zeros((nv, nv, mesh.num_cells))
    for t, cell in enumerate(mesh.cells):
        M[np.ix_(cell, cell, [t])] += element_stiffness(mesh.coords[cell])[:, :, None]
    return M


# --------------------------------------------------------------------------
# boundary conditions (NDP factory, LinearEllipticFactories.py:239-281)
# --------------------------------------------------------------------------
def dirichlet_split(mesh, tol=1e-12):
    x = mesh.coords[:, 0]
    constrained = np.where((np.abs(x) < tol) | (np.abs(x - 1.0) < tol))[0]
    free = np.setdiff1d(np.arange(mesh.num_vertices), constrained)
    return constrained, free


def dirichlet_values(mesh, nodes, u):
    """left: u0(1-y)+u1 y ; right: u2(1-y)+u3 y."""
    u0, u1, u2, u3 = u
    x = mesh.coords[nodes, 0]
    y = mesh.coords[nodes, 1]
    left = u0 * (1 - y) + u1 * y
    right = u2 * (1 - y) + u3 * y
    return np.where(x < 0.5, left, right)


def assemble_system(mesh, kappa_cells, u_bc, f=None):
    """Dirichlet-reduced system (physics/LinearElliptic.py:137-159).

    Returns K_ff, f_eff = f_free - K_fc g.  The NDP source is 0.
    """
    K = assemble_stiffness(mesh, kappa_cells)
    c, fr = dirichlet_split(mesh)
    g = dirichlet_values(mesh, c, u_bc)
    if f is None:
        f = np.zeros(mesh.num_vertices)
    f_eff = f[fr] - K[np.ix_(fr, c)] @ g
    return K[np.ix_(fr, fr)], f_eff


def solve_fom(mesh, kappa_cells, u_bc):
    """FOM label y on free dofs (physics/LinearElliptic.py:85-101)."""
    K, f = assemble_system(mesh, kappa_cells, u_bc)
    return np.linalg.solve(K, f)


def fom_residual(mesh, kappa_cells, u_bc, y_free):
    """(K yhat)_free = K_ff y - f_eff with yhat = y on the free nodes, g on the Dirichlet nodes
    (the FOM residual of physics/LinearElliptic.py:137-159, f = 0), any mesh size."""
    c, fr = dirichlet_split(mesh)
    u = np.zeros(mesh.num_vertices)
    u[c] = dirichlet_values(mesh, c, u_bc)
    u[fr] = y_free
    return apply_stiffness(mesh, kappa_cells, u)[fr]


def full_solution(mesh, y_free, u_bc):
    """scatter_restricted_solution (physics/LinearElliptic.py:103-118)."""
    c, fr = dirichlet_split(mesh)
    out = np.zeros(mesh.num_vertices)
    out[c] = dirichlet_values(mesh, c, u_bc)
    out[fr] = y_free
    return out


def f_rom_bc(mesh_c, u_bc):
    """FULL_F_WITH_APPLIED_BC (physics/BoundaryConditions.py:132-147); f=0."""
    c, _ = dirichlet_split(mesh_c)
    F = np.zeros(mesh_c.num_vertices)
    F[c] = dirichlet_values(mesh_c, c, u_bc)
    return F


# --------------------------------------------------------------------------
# prolongation W (components.py:38-60, fawkes/utils.py:115-192)
# --------------------------------------------------------------------------
def _bary_tables(mesh):
    if getattr(mesh, '_bary', None) is None:
        P = mesh.coords[mesh.cells]                               # [nc, 3, 2]
        G = np.stack([barycentric_gradients(p)[1] for p in P])    # [nc, 3, 2]
        mesh._bary = (P, G)
    return mesh._bary


def locate(mesh, pt, tol=1e-12):
    """First cell containing pt (bounding-box-tree first collision semantics) and its barycentrics."""
    P, G = _bary_tables(mesh)
    d = pt[None, :] - P[:, 0, :]
    l1 = np.einsum('ck,ck->c', G[:, 1], d)
    l2 = np.einsum('ck,ck->c', G[:, 2], d)
    lam = np.stack([1.0 - l1 - l2, l1, l2], 1)
    hit = np.where(np.all(lam >= -tol, 1))[0]
    if hit.size == 0:
        raise ValueError('point outside mesh')
    return int(hit[0]), lam[hit[0]]


def prolongation(mesh_c, points):
    """W[p, k] = phi_k^coarse(point p) -> [n_points, n_c] (dense)."""
    W = np.zeros((len(points), mesh_c.num_vertices))
    for r, pt in enumerate(points):
        t, lam = locate(mesh_c, np.asarray(pt))
        W[r, mesh_c.cells[t]] = lam
    return W


def prolongation_free(mesh_c, mesh_f):
    _, fr = dirichlet_split(mesh_f)
    return prolongation(mesh_c, mesh_f.coords[fr])


# --------------------------------------------------------------------------
# images <-> DG0 cells (bottleneck/utils.py:69-132)
# --------------------------------------------------------------------------
def image_to_cells(img):
    """Pixel value -> both triangles of its square; img [..., n, n] (row 0 top)."""
    img = np.asarray(img)
    n = img.shape[-1]
    out = np.zeros(img.shape[:-2] + (2 * n * n,))
    for r in range(n):
        for c in range(n):
            q = c + n * (n - 1 - r)
            out[..., 2 * q] = img[..., r, c]
            out[..., 2 * q + 1] = img[..., r, c]
    return out


# --------------------------------------------------------------------------
# residual operators
# --------------------------------------------------------------------------
def cgr_query(mesh_f, W_free, kappa_cells, u_bc):
    """CoarseGrainedResidualSampler: Gamma = W^T K_ff, alpha = W^T f_eff
    (VirtualObservables.py:57-69,297-321)."""
    K, f = assemble_system(mesh_f, kappa_cells, u_bc)
    return W_free.T @ K, W_free.T @ f


def _coarse_cell_facets(mesh_c, k):
    cell = mesh_c.cells[k]
    return [(cell[a], cell[b]) for a, b in ((0, 1), (1, 2), (2, 0))]


def _on_segment(p, a, b, tol=1e-12):
    return np.linalg.norm(p - a) + np.linalg.norm(p - b) - np.linalg.norm(a - b) < tol


def flux_rows(mesh_c, mesh_f, kappa_cells):
    """FluxConstraintReducedOrderModel rows (bottleneck/flux.py:81-158).

    Row k: sum over fine facets lying on the boundary of coarse triangle k of
    |e| kappa_T grad(u)|_T . n_T.  Coarse facets on the Dirichlet boundary
    (x=0 / x=1) use ``ds`` (T = the adjacent fine cell, n outward);
    every other coarse facet uses ``dS`` with the '+' restriction
    (flux.py:31).  PARITY UNPINNED: DOLFIN picks '+' from its facet-cell
    connectivity, which is not reproducible here; this oracle takes '+' =
    the fine cell inside coarse cell k (outward flux).  ``dS`` over a
    top/bottom boundary facet has no neighbour and contributes nothing.
    Returns (Gamma_full [n_T, n_vf], alpha [n_T]); alpha is identically 0
    (flux.py:153 dots the zero-initialised self.Gamma).
    """
    nT = mesh_c.num_cells
    G = np.zeros((nT, mesh_f.num_vertices))
    Cf = mesh_f.coords
    # fine facet -> adjacent fine cells
    facet_cells = {}
    for t, cell in enumerate(mesh_f.cells):
        for a, b in ((0, 1), (1, 2), (2, 0)):
            key = tuple(sorted((cell[a], cell[b])))
            facet_cells.setdefault(key, []).append(t)
    cen_c = np.array([mesh_c.coords[c].mean(0) for c in mesh_c.cells])
    for k in range(nT):
        for va, vb in _coarse_cell_facets(mesh_c, k):
            A, B = mesh_c.coords[va], mesh_c.coords[vb]
            exterior = (abs(A[0] - B[0]) < 1e-12) and (abs(A[0]) < 1e-12 or abs(A[0] - 1) < 1e-12)
            for key, cells in facet_cells.items():
                mp = 0.5 * (Cf[key[0]] + Cf[key[1]])
                if not _on_segment(mp, A, B):
                    continue
                if len(cells) == 1 and not exterior:
                    continue     # dS over a boundary facet: no contribution
                # the fine cell inside coarse triangle k
                inside = None
                for t in cells:
                    ct = Cf[mesh_f.cells[t]].mean(0)
                    _, lam = _bary(mesh_c.coords[mesh_c.cells[k]], ct)
                    if np.all(lam >= -1e-12):
                        inside = t
                if inside is None:
                    continue
                p = Cf[mesh_f.cells[inside]]
                _, g = barycentric_gradients(p)
                e = Cf[key[1]] - Cf[key[0]]
                length = np.linalg.norm(e)
                nrm = np.array([e[1], -e[0]]) / length
                if nrm @ (mp - p.mean(0)) < 0:
                    nrm = -nrm
                G[k, mesh_f.cells[inside]] += length * kappa_cells[inside] * (g @ nrm)
    return G, np.zeros(nT)


def _bary(p, pt):
    _, g = barycentric_gradients(p)
    l1 = g[1] @ (pt - p[0])
    l2 = g[2] @ (pt - p[0])
    return None, np.array([1 - l1 - l2, l1, l2])


def flux_residual_structured(nc, r, kappa_lr, kappa_ul, y_free):
    """r_fc = Gamma_fc[:, free] y for every coarse triangle (bottleneck/flux.py:81-158, the rows of
    ``flux_rows`` above, alpha = 0), in closed form on the structured mesh and vectorised so that it
    runs at 128^2 / 256^2 where the generic facet search of ``flux_rows`` does not finish.  Pinned
    against ``flux_rows`` on small meshes (tests/test_physics_stencil.py).

    kappa_lr / kappa_ul: [n, n] conductivities of the fine T_lr / T_ul of square (i, j) at [j, i];
    y_free: fine free-node values (Dirichlet columns x = 0 / 1 enter as 0, the free-column
    restriction).  Per fine triangle with corner values u0 (i,j), u1 (i+1,j), u2 (i,j+1), u3
    (i+1,j+1), |e| kappa grad(u).n on its facets:
      T_lr: bottom kappa (u1 - u3), right kappa (u1 - u0), diagonal kappa (u0 - 2 u1 + u3);
      T_ul: left kappa (u2 - u3), top kappa (u2 - u0), diagonal kappa (u0 - 2 u2 + u3).
    Coarse T_lr rows take the bottom facets (not on y = 0: dS without a neighbour), right facets and
    diagonal of their coarse square; T_ul rows the left facets, top facets (not on y = 1) and
    diagonal."""
    n = nc * r
    u = np.zeros((n + 1, n + 1))
    u[:, 1:n] = np.asarray(y_free, dtype=np.float64).reshape(n + 1, n - 1)
    kl = np.asarray(kappa_lr, dtype=np.float64)
    ku = np.asarray(kappa_ul, dtype=np.float64)
    u0, u1, u2, u3 = u[:-1, :-1], u[:-1, 1:], u[1:, :-1], u[1:, 1:]          # [j, i] of square (i, j)
    rows = np.zeros((nc, nc, 2))                                            # [J, I, lr / ul]
    # T_lr bottom facets: fine row j = J r, summed over the r squares of each coarse column
    bot = (kl * (u1 - u3))[::r, :].reshape(nc, nc, r).sum(2)
    bot[0, :] = 0.0
    right = (kl * (u1 - u0))[:, r - 1::r].reshape(nc, r, nc).sum(1)
    a = np.arange(n)
    diag_sq = (a % r)[None, :] == (a % r)[:, None]                           # squares on the coarse diagonals
    dl = np.where(diag_sq, kl * (u0 - 2 * u1 + u3), 0.0).reshape(nc, r, nc, r).sum((1, 3))
    rows[:, :, 0] = bot + right + dl
    left = (ku * (u2 - u3))[:, ::r].reshape(nc, r, nc).sum(1)
    top = (ku * (u2 - u0))[r - 1::r, :].reshape(nc, nc, r).sum(2)
    top[-1, :] = 0.0
    du = np.where(diag_sq, ku * (u0 - 2 * u2 + u3), 0.0).reshape(nc, r, nc, r).sum((1, 3))
    rows[:, :, 1] = left + top + du
    return rows.reshape(-1)            # coarse cell 2 (I + nc J) + {0: T_lr, 1: T_ul}


def image_to_square_kappa(img):
    """Pixel image (row 0 = top) -> [n, n] per-square values at [j, i] (both triangles)."""
    img = np.asarray(img, dtype=np.float64)
    return img[..., ::-1, :]
