"""Independent numpy oracles for the benchmark problem.

* `box_model`: direct, vectorised element-by-element model of the whole
  problem on a small global mesh (any geometry perturbation): RHS b = M f,
  BC, u = b, y = A u.  Reproduces the reference's published norms
  (`src/test_output.py:19`, `examples/mat_comp-16.json`).
* `kron_norms`: O(n) closed form of ||u|| and the action-mode ||y|| for the
  unperturbed box from 1D matrices (valid at any size, e.g. the 19.2 G / 32 G
  DoF published runs).
* `cg_model`: unpreconditioned CG on the oracle operator.

This file deliberately shares no code with the package except the 1D
quadrature tables (themselves unit-tested against closed forms).
"""

from __future__ import annotations

import numpy as np

from benchmark_dolfinx_amd.fem.quadrature import OperatorTables

KAPPA = 2.0


def f_source(x, y, z):
    return 1000.0 * np.exp(-((x - 0.5) ** 2 + (y - 0.5) ** 2) / 0.02)


def _ref_grad_tables(t: OperatorTables):
    """gradref[a, q, d] for a in nd^3 (lexicographic), q in nq^3."""
    B, D = t.B, t.Dd
    g0 = np.einsum("xi,yj,zk->xyzijk", D, B, B)
    g1 = np.einsum("xi,yj,zk->xyzijk", B, D, B)
    g2 = np.einsum("xi,yj,zk->xyzijk", B, B, D)
    nq, nd = t.nq, t.nd
    g = np.stack([g0, g1, g2], axis=-1).reshape(nq ** 3, nd ** 3, 3)
    val = np.einsum("xi,yj,zk->xyzijk", B, B, B).reshape(nq ** 3, nd ** 3)
    return np.transpose(g, (1, 0, 2)), val.T  # (a, q, 3), (a, q)


def box_model(ncells, degree, qmode=1, use_gauss=False, vertices=None, kappa_cells=None):
    """Return dict(u, y, b, bc, N) on the global lattice (z fastest).
    kappa_cells: optional per-cell coefficient (nx, ny, nz); default KAPPA."""
    t = OperatorTables(degree, qmode, use_gauss)
    nx, ny, nz = ncells
    P = degree
    N = (nx * P + 1, ny * P + 1, nz * P + 1)
    if vertices is None:
        vx, vy, vz = np.meshgrid(np.arange(nx + 1) / nx, np.arange(ny + 1) / ny,
                                 np.arange(nz + 1) / nz, indexing="ij")
        vertices = np.stack([vx, vy, vz], axis=-1)
    cx, cy, cz = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    cx, cy, cz = cx.ravel(), cy.ravel(), cz.ravel()
    C = cx.size
    # cell vertices (C, 8, 3), TP order v = 4a + 2b + c
    cv = np.empty((C, 8, 3))
    for a in range(2):
        for b in range(2):
            for c in range(2):
                cv[:, 4 * a + 2 * b + c] = vertices[cx + a, cy + b, cz + c]
    dphi = t.geometry_dphi()  # (3, Q, 8)
    J = np.einsum("cvi,jqv->cqij", cv, dphi)
    det = np.linalg.det(J)
    Jinv = np.linalg.inv(J)
    w3 = t.weights3d()
    # G = w det J^-1 J^-T
    G = np.einsum("cqid,cqjd->cqij", Jinv, Jinv) * (w3[None, :] * det)[..., None, None]
    # dof map
    nd = t.nd
    li = np.arange(nd)
    I = (cx[:, None] * P + li[None, :])
    Jd = (cy[:, None] * P + li[None, :])
    K = (cz[:, None] * P + li[None, :])
    dofs = ((I[:, :, None, None] * N[1] + Jd[:, None, :, None]) * N[2]
            + K[:, None, None, :]).reshape(C, nd ** 3)
    # node coordinates (trilinear map of GLL nodes)
    xn = t.nodes
    Nl = np.array([1 - xn, xn])  # (2, nd)
    shp = np.einsum("ai,bj,ck->abcijk", Nl, Nl, Nl).reshape(8, nd ** 3)
    xphys = np.einsum("cvd,va->cad", cv, shp)
    fvals = np.zeros(int(np.prod(N)))
    fvals[dofs.ravel()] = f_source(xphys[..., 0], xphys[..., 1], xphys[..., 2]).ravel()
    gref, val = _ref_grad_tables(t)
    # RHS b = M f
    fe = fvals[dofs]
    fq = np.einsum("aq,ca->cq", val, fe) * (w3[None, :] * det)
    be = np.einsum("aq,cq->ca", val, fq)
    b = np.zeros_like(fvals)
    np.add.at(b, dofs.ravel(), be.ravel())
    # BC
    ix, iy, iz = np.meshgrid(np.arange(N[0]), np.arange(N[1]), np.arange(N[2]), indexing="ij")
    bc = ((ix == 0) | (ix == N[0] - 1) | (iy == 0) | (iy == N[1] - 1)
          | (iz == 0) | (iz == N[2] - 1)).ravel()
    b[bc] = 0.0
    u = b.copy()

    kap = (np.full(C, KAPPA) if kappa_cells is None
           else np.asarray(kappa_cells, dtype=np.float64).reshape(-1))

    def apply(x):
        xe = np.where(bc[dofs], 0.0, x[dofs])
        gu = np.einsum("aqd,ca->cqd", gref, xe)
        Fq = kap[:, None, None] * np.einsum("cqde,cqe->cqd", G, gu)
        ye = np.einsum("aqd,cqd->ca", gref, Fq)
        ye = np.where(bc[dofs], 0.0, ye)
        y = np.zeros_like(x)
        np.add.at(y, dofs.ravel(), ye.ravel())
        y[bc] = x[bc]
        return y

    y = apply(u)
    return dict(u=u, y=y, b=b, bc=bc, N=N, apply=apply, f=fvals, dofs=dofs)


def cg_model(apply, b, nreps):
    """Reference CG (src/cg.hpp:89-169) with rtol = 0, x0 = 0."""
    x = np.zeros_like(b)
    y = apply(x)
    r = b - y
    p = r.copy()
    rnorm = p @ r
    for _ in range(nreps):
        y = apply(p)
        alpha = rnorm / (p @ y)
        x = x + alpha * p
        r = r - alpha * y
        rnew = r @ r
        beta = rnew / rnorm
        rnorm = rnew
        p = beta * p + r
    return x


def _mats_1d(n, t: OperatorTables):
    """1D assembled mass and stiffness on [0, 1] with n uniform cells."""
    P = t.degree
    Nn = n * P + 1
    M = np.zeros((Nn, Nn))
    K = np.zeros((Nn, Nn))
    h = 1.0 / n
    Me = t.B.T @ np.diag(t.qwts * h) @ t.B
    Ke = t.Dd.T @ np.diag(t.qwts / h) @ t.Dd
    for c in range(n):
        s = slice(c * P, c * P + P + 1)
        M[s, s] += Me
        K[s, s] += Ke
    x = np.concatenate([(c + t.nodes[:-1]) * h for c in range(n)] + [np.array([1.0])])
    return M, K, x


def kron_norms(ncells, degree, qmode=1, use_gauss=False):
    """Closed-form (||u||, ||y_action||) on the unperturbed box (Appendix A.3)."""
    t = OperatorTables(degree, qmode, use_gauss)
    mats = [_mats_1d(n, t) for n in ncells]
    g = lambda s: np.exp(-((s - 0.5) ** 2) / 0.02)  # noqa: E731
    m = []
    for d, (M, K, x) in enumerate(mats):
        vec = g(x) if d < 2 else np.ones_like(x)
        mv = M @ vec
        mv[0] = 0.0
        mv[-1] = 0.0
        m.append(mv)
    unorm = 1000.0 * np.prod([np.linalg.norm(v) for v in m])
    # y = kappa * sum_a kron_d (a==d ? K~ u~ : M~ u~), interior only
    terms = []
    for a in range(3):
        fac = []
        for d, (M, K, x) in enumerate(mats):
            ui = m[d][1:-1]
            A = (K if a == d else M)[1:-1, 1:-1]
            fac.append(A @ ui)
        terms.append(fac)
    ysq = 0.0
    for a in range(3):
        for bb in range(3):
            prod = 1.0
            for d in range(3):
                prod *= terms[a][d] @ terms[bb][d]
            ysq += prod
    ynorm = KAPPA * 1000.0 * np.sqrt(ysq)
    return unorm, ynorm
