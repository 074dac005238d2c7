"""Host index lists of the column-sparse VO conditioning (gpi/vo.py sparse_index_lists, the
bookkeeping behind include/gpi.h gpi_vo_sparse): the sums the device kernels run over them
(csrc/vo.hip vo_lambda_sparse_kernel, vo_rhs_sparse_kernel, vo_columns_sparse_kernel,
vo_precision_sparse_kernel), restated here in numpy, reproduce the dense forms of
VirtualObservables.py:642-669,971-998 (Lambda = Gamma C Gamma^T + diag(v), Gamma g - alpha,
Gamma_i^T Lambda^-1 Gamma_i, Gamma^2 vars) on random column-sparse Gamma, including empty rows
and columns.  CPU only."""
import numpy as np
import pytest

from gpi.vo import sparse_index_lists


def pattern(G):
    """What gpi_vo_pattern returns: per column the ascending rows nonzero in any sample."""
    N, m, dy = G.shape
    nz = (G != 0).any(axis=0)
    r = max(int(nz.sum(0).max()), 1)
    rows = -np.ones((dy, r), dtype=np.int32)
    for i in range(dy):
        a = np.nonzero(nz[:, i])[0]
        rows[i, :len(a)] = a
    return rows


def random_sparse(rng, N, m, dy, k):
    G = np.zeros((N, m, dy))
    for i in range(dy):
        if i % 7 == 3:
            continue                                      # empty column
        a = rng.choice(m - 1, size=rng.integers(1, k + 1), replace=False)   # row m-1 stays empty
        G[:, a, i] = rng.normal(size=(N, len(a)))
    return G


@pytest.mark.parametrize('N,m,dy,k', [(3, 9, 40, 4), (2, 25, 200, 11), (1, 5, 3, 4)])
def test_sparse_lists_reproduce_dense_forms(N, m, dy, k):
    rng = np.random.default_rng(m * dy)
    G = random_sparse(rng, N, m, dy, k)
    rows = pattern(G)
    r = rows.shape[1]
    li = sparse_index_lists(rows, m)
    vals = np.where(rows[None] >= 0, np.take_along_axis(G, np.maximum(rows.T, 0)[None].repeat(N, 0), axis=1)
                    .transpose(0, 2, 1), 0.0)                                  # [N, dy, r]
    prec = rng.uniform(0.5, 3.0, (N, dy))
    vv = rng.uniform(0.1, 1.0, m)
    g = rng.normal(size=(N, dy))
    alpha = rng.normal(size=(N, m))
    mu = rng.normal(size=(N, dy))
    va = rng.uniform(0.1, 1.0, (N, dy))
    # all diagonals present, entries a >= b, ascending, contributions grouped by entry
    ab = li['pair_ab']
    assert np.all(np.diff(ab) > 0) and np.all(ab // m >= ab % m)
    assert set(range(0, m * m, m + 1)) <= set(ab.tolist())
    for j in range(N):
        v = vals[j].reshape(-1)
        # Lambda
        lam = np.zeros((m, m))
        for p in range(len(ab)):
            acc = 0.0
            for e in range(li['pair_ptr'][p], li['pair_ptr'][p + 1]):
                src = int(li['pair_src'][e])
                i, st = divmod(src, r * r)
                s, t = divmod(st, r)
                acc += v[i * r + s] / prec[j, i] * v[i * r + t]
            a, b = divmod(int(ab[p]), m)
            if a == b:
                acc += vv[a]
            lam[a, b] = lam[b, a] = acc
        ref = G[j] @ np.diag(1.0 / prec[j]) @ G[j].T + np.diag(vv)
        np.testing.assert_allclose(lam, ref, rtol=1e-12, atol=1e-12)
        # Gamma g - alpha and the precision terms by rows
        bvec = np.zeros(m)
        s1 = np.zeros(m)
        s2 = np.zeros(m)
        for a in range(m):
            for e in range(li['row_ptr'][a], li['row_ptr'][a + 1]):
                src = int(li['row_src'][e])
                i = src // r
                bvec[a] += v[src] * g[j, i]
                s1[a] += v[src] * mu[j, i]
                s2[a] += v[src] ** 2 * va[j, i]
        np.testing.assert_allclose(bvec - alpha[j], G[j] @ g[j] - alpha[j], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(s1, G[j] @ mu[j], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(s2, (G[j] ** 2) @ va[j], rtol=1e-12, atol=1e-12)
        # column quadratic forms from the slots vs |L^-1 Gamma_i|^2
        inv = np.linalg.inv(ref)
        Lc = np.linalg.cholesky(ref)
        qd = (np.linalg.solve(Lc, G[j]) ** 2).sum(0)
        for i in range(dy):
            q = 0.0
            for s in range(r):
                if rows[i, s] < 0:
                    continue
                off = sum(vals[j, i, t] * inv[rows[i, s], rows[i, t]] for t in range(s) if rows[i, t] >= 0)
                q += vals[j, i, s] * (2.0 * off + vals[j, i, s] * inv[rows[i, s], rows[i, s]])
            assert abs(q - qd[i]) <= 1e-10 * max(1.0, abs(qd[i]))
