"""Host-side checks of the Kronecker-core tables (fused5): the 1D
matrices M = B^T W B, K = Dd^T W Dd, C = Dd^T W B packed by the HIP library's
host entry points match numpy, and the Kronecker sum they define reproduces
the dense element stiffness matrix of an affine cell (no GPU needed: the
packers are host code in libbdx_hip.so)."""

import ctypes

import numpy as np
import pytest

from benchmark_dolfinx_amd.fem.quadrature import OperatorTables
from benchmark_dolfinx_amd.ops.native import ptr


def _lib():
    try:
        from benchmark_dolfinx_amd.ops import native
        return native.hip()
    except Exception as e:  # pragma: no cover - no HIP runtime in this environment
        pytest.skip(f"libbdx_hip.so not loadable here: {e}")


def _mats(tab):
    t = OperatorTables(*tab)
    B, Dd, w = t.phi0, t.Dd, t.qwts
    return t, B.T @ np.diag(w) @ B, Dd.T @ np.diag(w) @ Dd, Dd.T @ np.diag(w) @ B


@pytest.mark.parametrize("suf,npdt", [("f64", np.float64), ("f32", np.float32)])
@pytest.mark.parametrize("P", [3, 4, 5, 6, 7])
@pytest.mark.parametrize("qmode,gauss", [(0, False), (1, False), (1, True)])
def test_fused5_tables(P, qmode, gauss, suf, npdt):
    lib = _lib()
    t, M, K, C = _mats((P, qmode, gauss))
    nd, nq = P + 1, t.phi0.shape[0]
    fn = getattr(lib, f"bdx_fused5_tables_{suf}_p{P}")
    phi0 = np.ascontiguousarray(t.phi0, dtype=np.float64)
    Dd = np.ascontiguousarray(t.Dd, dtype=np.float64)
    w = np.ascontiguousarray(t.qwts, dtype=np.float64)
    n = fn(nd, nq, ptr(phi0), ptr(Dd), ptr(w), None)
    assert n >= 256
    out = np.zeros(n, dtype=npdt)
    assert fn(nd, nq, ptr(phi0), ptr(Dd), ptr(w), ptr(out)) == n
    blk = out[:256].reshape(4, 8, 8).astype(np.float64)
    tol = 1e-14 if npdt == np.float64 else 1e-6
    for b, ref in enumerate((M, K, C, C.T)):
        np.testing.assert_allclose(blk[b, :nd, :nd], ref, atol=tol * np.abs(ref).max())
        assert not blk[b, nd:, :].any() and not blk[b, :, nd:].any()
    ty, tz = ctypes.c_int(0), ctypes.c_int(0)
    for code in (1, 2):
        assert getattr(lib, f"bdx_fused5_tile_p{P}_{suf}")(code, ctypes.byref(ty),
                                                           ctypes.byref(tz)) == 0
        assert ty.value >= 1 and tz.value >= 1


@pytest.mark.parametrize("P", [2, 3, 5])
@pytest.mark.parametrize("qmode,gauss", [(0, False), (1, False), (1, True)])
def test_kronecker_sum_is_the_affine_stiffness(P, qmode, gauss):
    """A_e = sum over the 9 (G_ab, x.y.z) Kronecker blocks equals the dense
    quadrature stiffness matrix of a sheared parallelepiped cell."""
    t, M, K, C = _mats((P, qmode, gauss))
    B, Dd, w = t.phi0, t.Dd, t.qwts
    J = np.array([[0.9, 0.2, 0.1], [0.05, 1.1, 0.3], [0.0, 0.15, 0.8]])
    Ji = np.linalg.inv(J)
    G = 2.0 * abs(np.linalg.det(J)) * Ji @ Ji.T
    # dense: grad phi_(ijk) at (qx,qy,qz) via the tensor tables
    k3 = lambda a, b, c: np.einsum("ai,bj,ck->abcijk", a, b, c).reshape(len(w) ** 3, -1)
    g = [k3(Dd, B, B), k3(B, Dd, B), k3(B, B, Dd)]
    W3 = np.einsum("a,b,c->abc", w, w, w).ravel()
    A = sum(G[a, b] * g[a].T @ (W3[:, None] * g[b]) for a in range(3) for b in range(3))
    kr = lambda x, y, z: np.kron(np.kron(x, y), z)
    Ak = (G[0, 0] * kr(K, M, M) + G[1, 1] * kr(M, K, M) + G[2, 2] * kr(M, M, K)
          + G[1, 2] * (kr(M, C, C.T) + kr(M, C.T, C)) + G[0, 1] * (kr(C, C.T, M) + kr(C.T, C, M))
          + G[0, 2] * (kr(C, M, C.T) + kr(C.T, M, C)))
    np.testing.assert_allclose(Ak, A, atol=1e-12 * np.abs(A).max())


@pytest.mark.parametrize("P", [3, 6])
def test_fused5_pass_schedule(P):
    """numpy emulation of lap_fused5.h's x -> z -> y pass schedule (the
    y-factor groups zM, zK, zCt, zC) reproduces the Kronecker-sum action."""
    t, M, K, C = _mats((P, 1, False))
    Ct = C.T
    rng = np.random.default_rng(0)
    nd = P + 1
    u = rng.standard_normal((nd, nd, nd))  # u[i][j][k] (x, y, z)
    G = rng.standard_normal((3, 3))
    G = G @ G.T
    ax = lambda Mat, v, a: np.moveaxis(np.tensordot(Mat, v, axes=([1], [a])), 0, a)
    # x pass
    ak, am, ac, at = (ax(X, u, 0) for X in (K, M, C, Ct))
    # z pass (axis 2)
    zM = (G[0, 0] * ax(M, ak, 2) + G[2, 2] * ax(K, am, 2) + G[0, 2] * ax(Ct, ac, 2)
          + G[0, 2] * ax(C, at, 2))
    zK = G[1, 1] * ax(M, am, 2)
    zCt = G[0, 1] * ax(M, ac, 2) + G[1, 2] * ax(C, am, 2)
    zC = G[0, 1] * ax(M, at, 2) + G[1, 2] * ax(Ct, am, 2)
    # y pass (axis 1)
    ye = ax(M, zM, 1) + ax(K, zK, 1) + ax(Ct, zCt, 1) + ax(C, zC, 1)
    kr = lambda x, y, z: np.kron(np.kron(x, y), z)
    Ak = (G[0, 0] * kr(K, M, M) + G[1, 1] * kr(M, K, M) + G[2, 2] * kr(M, M, K)
          + G[1, 2] * (kr(M, C, Ct) + kr(M, Ct, C)) + G[0, 1] * (kr(C, Ct, M) + kr(Ct, C, M))
          + G[0, 2] * (kr(C, M, Ct) + kr(Ct, M, C)))
    np.testing.assert_allclose(ye.ravel(), Ak @ u.ravel(), atol=1e-12 * np.abs(Ak).max())
