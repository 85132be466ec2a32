"""Host FEM numerics (replaces Basix: src/laplacian.hpp:125-212)."""

import numpy as np
import pytest

from benchmark_dolfinx_amd.fem.quadrature import (OperatorTables, gauss_legendre, gll,
                                                   lagrange_tables)


@pytest.mark.parametrize("n", range(2, 11))
def test_gll_exactness(n):
    x, w = gll(n)
    assert x[0] == 0.0 and x[-1] == 1.0
    assert np.all(np.diff(x) > 0)
    for k in range(0, 2 * n - 2):  # exact up to degree 2n-3
        assert abs(w @ x ** k - 1.0 / (k + 1)) < 1e-14, k


@pytest.mark.parametrize("n", range(1, 11))
def test_gauss_exactness(n):
    x, w = gauss_legendre(n)
    assert np.all((x > 0) & (x < 1))
    for k in range(0, 2 * n):  # exact up to degree 2n-1
        assert abs(w @ x ** k - 1.0 / (k + 1)) < 1e-14, k


def test_gll_known_values():
    x, w = gll(3)
    assert np.allclose(x, [0, 0.5, 1]) and np.allclose(w, [1 / 6, 2 / 3, 1 / 6])
    x, w = gll(4)
    s = 0.5 / np.sqrt(5)
    assert np.allclose(x, [0, 0.5 - s, 0.5 + s, 1]) and np.allclose(w, [1 / 12, 5 / 12, 5 / 12, 1 / 12])


@pytest.mark.parametrize("n", range(2, 9))
def test_lagrange_partition_of_unity(n):
    nodes, _ = gll(n)
    xs = np.linspace(0, 1, 13)
    V, D = lagrange_tables(nodes, xs)
    assert np.allclose(V.sum(1), 1.0, atol=1e-13)
    assert np.allclose(D.sum(1), 0.0, atol=1e-10)
    Vn, _ = lagrange_tables(nodes, nodes)
    assert np.allclose(Vn, np.eye(n), atol=1e-14)
    # derivative of x^k is reproduced
    for k in range(n):
        assert np.allclose(D @ nodes ** k, k * xs ** max(k - 1, 0) if k else 0.0, atol=1e-9)


@pytest.mark.parametrize("P", range(1, 8))
@pytest.mark.parametrize("qmode", [0, 1])
@pytest.mark.parametrize("gauss", [False, True])
def test_operator_tables(P, qmode, gauss):
    if gauss and qmode == 0:
        # reference quirk Q5: src/laplacian.hpp:197-198
        with pytest.raises(RuntimeError, match="identity"):
            OperatorTables(P, qmode, gauss)
        return
    t = OperatorTables(P, qmode, gauss)
    assert t.nd == P + 1 and t.nq == P + 1 + qmode
    assert t.phi0.shape == (t.nq, t.nd) and t.dphi1.shape == (t.nq, t.nq)
    assert t.is_identity == (qmode == 0 and not gauss)
    assert np.allclose(t.phi0.sum(1), 1.0, atol=1e-13)
    assert np.allclose(t.dphi1.sum(1), 0.0, atol=1e-10)
    assert np.allclose(t.Dd, t.dphi1 @ t.phi0)
    # Dd differentiates the element nodes' coordinate exactly
    assert np.allclose(t.Dd @ t.nodes, 1.0, atol=1e-11)
    assert abs(t.weights3d().sum() - 1.0) < 1e-13


def test_invalid_degree():
    with pytest.raises(ValueError):
        OperatorTables(8)
    with pytest.raises(ValueError):
        OperatorTables(3, 2)


def test_geometry_dphi_affine():
    t = OperatorTables(2, 1)
    d = t.geometry_dphi()
    assert d.shape == (3, t.nq ** 3, 8)
    assert np.allclose(d.sum(-1), 0.0)
    # unit cube vertices: J = I
    v = np.array([[a, b, c] for a in (0, 1) for b in (0, 1) for c in (0, 1)], float)
    J = np.einsum("vi,jqv->qij", v, d)
    assert np.allclose(J, np.eye(3)[None])
