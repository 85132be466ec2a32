"""1D quadrature rules and Lagrange tables on [0, 1].

Replaces the Basix calls the reference makes when it builds the operator
(`src/laplacian.hpp:125-212`: `make_quadrature`, `create_element(interval)`,
`compute_interpolation_operator`, `tabulate`).  Everything here is small,
host-side and computed once in float64; kernels receive the tables as
constants.

Conventions (reference semantics):

* element nodes: GLL points with ``P + 1`` nodes (GLL-warped == GLL on an
  interval);
* quadrature: ``nq = P + 1 + qmode`` points, GLL (default) or Gauss-Legendre
  (``--use_gauss``), tensor product with the last index fastest;
* ``phi0[q, i] = l_i(x_q)``  (element-0 Lagrange basis at the quadrature
  points, the interpolation operator to the element whose nodes are the
  quadrature points, `src/laplacian.hpp:179-185`);
* ``dphi1[q, j] = l^quad_j'(x_q)`` (derivative of the quadrature-node
  Lagrange basis at the quadrature points, `src/laplacian.hpp:201`).
"""

from __future__ import annotations

import functools

import numpy as np
from numpy.polynomial import legendre as npleg


def _legendre(n: int, x: np.ndarray) -> np.ndarray:
    c = np.zeros(n + 1)
    c[n] = 1.0
    return npleg.legval(x, c)


@functools.lru_cache(maxsize=None)
def gll(n: int) -> tuple[np.ndarray, np.ndarray]:
    """Gauss-Lobatto-Legendre points and weights with ``n >= 2`` points on [0, 1].

    Interior points are the roots of P'_{n-1}, polished by Newton in float64;
    weights are ``2 / (n (n-1) P_{n-1}(xi)^2)`` on [-1, 1], halved for [0, 1].
    """
    if n < 2:
        raise ValueError("GLL needs at least 2 points")
    c = np.zeros(n)
    c[n - 1] = 1.0
    dc = npleg.legder(c)
    interior = np.sort(np.real(npleg.legroots(dc))) if n > 2 else np.zeros(0)
    # Newton polish on P'_{n-1}(x) = 0
    d2c = npleg.legder(dc)
    for _ in range(5):
        if interior.size == 0:
            break
        f = npleg.legval(interior, dc)
        fp = npleg.legval(interior, d2c)
        interior = interior - f / fp
    xi = np.concatenate([[-1.0], interior, [1.0]])
    pn = _legendre(n - 1, xi)
    w = 2.0 / (n * (n - 1) * pn * pn)
    return 0.5 * (xi + 1.0), 0.5 * w


@functools.lru_cache(maxsize=None)
def gauss_legendre(n: int) -> tuple[np.ndarray, np.ndarray]:
    """Gauss-Legendre (Gauss-Jacobi alpha=0) points and weights on [0, 1]."""
    xi, w = npleg.leggauss(n)
    # Newton polish of the roots of P_n
    c = np.zeros(n + 1)
    c[n] = 1.0
    dc = npleg.legder(c)
    for _ in range(3):
        xi = xi - npleg.legval(xi, c) / npleg.legval(xi, dc)
    pd = npleg.legval(xi, dc)
    w = 2.0 / ((1.0 - xi * xi) * pd * pd)
    return 0.5 * (xi + 1.0), 0.5 * w


def lagrange_tables(nodes: np.ndarray, x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Values and first derivatives of the Lagrange basis on ``nodes`` at ``x``.

    Returns ``(V, D)`` with ``V[q, i] = l_i(x_q)`` and ``D[q, i] = l_i'(x_q)``.
    Barycentric-free product formula; exact at nodes.
    """
    nodes = np.asarray(nodes, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    n = nodes.size
    V = np.ones((x.size, n))
    D = np.zeros((x.size, n))
    for i in range(n):
        others = [m for m in range(n) if m != i]
        denom = np.prod([nodes[i] - nodes[m] for m in others])
        for q, xq in enumerate(x):
            terms = [xq - nodes[m] for m in others]
            V[q, i] = np.prod(terms) / denom
            s = 0.0
            for a in range(len(others)):
                s += np.prod([terms[b] for b in range(len(others)) if b != a])
            D[q, i] = s / denom
    return V, D


class OperatorTables:
    """All 1D data a degree-P / qmode operator needs.

    Attributes:
        degree, qmode, use_gauss, nd (=P+1), nq (=P+1+qmode)
        nodes: GLL element nodes on [0, 1] (nd,)
        qpts, qwts: 1D quadrature (nq,)
        phi0: (nq, nd) interpolation matrix, entries below 5 eps set to 0
        dphi1: (nq, nq) derivative of the quadrature-node Lagrange basis
        is_identity: phi0 == I (collocated fast path)
        B, Dd: (nq, nd) value/derivative tables of the element basis at the
            quadrature points (Dd = dphi1 @ phi0), used by assembly / oracles
    """

    def __init__(self, degree: int, qmode: int = 1, use_gauss: bool = False,
                 eps: float = np.finfo(np.float64).eps):
        if not 1 <= degree <= 7:
            raise ValueError(f"Unsupported degree {degree} (1..7)")
        if qmode not in (0, 1):
            raise ValueError("Invalid qmode.")
        self.degree = degree
        self.qmode = qmode
        self.use_gauss = use_gauss
        self.nd = degree + 1
        self.nq = degree + 1 + qmode
        self.nodes, _ = gll(self.nd)
        if use_gauss:
            self.qpts, self.qwts = gauss_legendre(self.nq)
        else:
            self.qpts, self.qwts = gll(self.nq)
        phi0, Dd = lagrange_tables(self.nodes, self.qpts)
        phi0 = phi0.copy()
        phi0[np.abs(phi0) < 5 * eps] = 0.0
        self.phi0 = phi0
        _, self.dphi1 = lagrange_tables(self.qpts, self.qpts)
        self.is_identity = (phi0.shape[0] == phi0.shape[1]
                            and np.array_equal(phi0, np.eye(phi0.shape[0])))
        if qmode == 0 and not self.is_identity:
            # reference: src/laplacian.hpp:197-198
            raise RuntimeError("Expecting identity matrix for qmode=0")
        self.B = phi0
        self.Dd = self.dphi1 @ phi0

    def geometry_dphi(self) -> np.ndarray:
        """Trilinear coordinate-element gradients at the 3D quadrature points.

        Shape (3, nq^3, 8): d N_v / d X_d at point q, vertex v in TP order
        v = 4*a + 2*b + c for vertex offsets (a, b, c) in x, y, z.
        """
        nq = self.nq
        t = self.qpts
        out = np.zeros((3, nq ** 3, 8))
        for qx in range(nq):
            for qy in range(nq):
                for qz in range(nq):
                    q = (qx * nq + qy) * nq + qz
                    X = (t[qx], t[qy], t[qz])
                    for a in range(2):
                        for b in range(2):
                            for c in range(2):
                                v = 4 * a + 2 * b + c
                                fx = X[0] if a else 1 - X[0]
                                fy = X[1] if b else 1 - X[1]
                                fz = X[2] if c else 1 - X[2]
                                sx = 1 if a else -1
                                sy = 1 if b else -1
                                sz = 1 if c else -1
                                out[0, q, v] = sx * fy * fz
                                out[1, q, v] = fx * sy * fz
                                out[2, q, v] = fx * fy * sz
        return out

    def weights3d(self) -> np.ndarray:
        w = self.qwts
        return np.einsum("i,j,k->ijk", w, w, w).reshape(-1)
