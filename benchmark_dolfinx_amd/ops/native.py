"""ctypes bindings of the in-tree native libraries.

The libraries expose a plain C ABI (raw pointers + sizes + a HIP stream), so
kernels take torch tensors' ``data_ptr()`` directly and run on torch's
current HIP stream.  ``torch`` must be imported before the HIP library is
loaded so that both share one HIP runtime (same SONAME ``libamdhip64.so.7``).

On a machine with a GPU the HIP library is mandatory: `hip()` raises if it
cannot be built or loaded (no silent CPU fallback).
"""

from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from . import build as _build

_lock = threading.Lock()
_host = None
_hip = None
_loaded = {}

vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_int64
f64 = ctypes.c_double
f32 = ctypes.c_float


def ptr(x) -> int:
    """Raw data pointer of a torch tensor or numpy array (None -> 0).

    The caller must keep `x` (or its base) alive for the duration of the
    native call: never pass a temporary such as ``ptr(np.asarray(...))``.
    """
    if x is None:
        return 0
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"], "native call needs a contiguous array"
        return x.ctypes.data
    assert x.is_contiguous(), "native call needs a contiguous tensor"
    return x.data_ptr()


def _declare(lib, name, argtypes, restype=None):
    fn = getattr(lib, name)
    fn.argtypes = argtypes
    fn.restype = restype
    return fn


def host():
    """The host runtime library (built on first use)."""
    global _host
    with _lock:
        if _host is None:
            # BDX_HOST_LIB: an alternative build (the ASan/UBSan library)
            path = os.environ.get("BDX_HOST_LIB") or _build.build_host()
            lib = ctypes.CDLL(str(path))
            _loaded["host"] = str(path)
            for suf, ft in (("f64", f64), ("f32", f32)):
                _declare(lib, f"bdx_cpu_stiffness_{suf}",
                         [vp, i32, vp, vp, vp, vp, vp, i32, vp, ft, vp, vp, vp, vp, vp])
                _declare(lib, f"bdx_cpu_stiffness_g_{suf}",
                         [vp, i32, vp, vp, vp, vp, vp, i32, vp, vp, ft, vp, vp, vp, vp, vp])
                _declare(lib, f"bdx_cpu_geometry_{suf}", [vp, i32, vp, vp, vp, vp])
                _declare(lib, f"bdx_cpu_dofmap_{suf}",
                         [i32, i32, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, ft, vp,
                          vp, vp])
                _declare(lib, f"bdx_cpu_dofmap_geometry_{suf}", [i32, i32, vp, vp, i32, vp, vp, vp])
                _declare(lib, f"bdx_cpu_mass_{suf}",
                         [vp, i32, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp])
                _declare(lib, f"bdx_cpu_csr_{suf}",
                         [vp, i32, vp, vp, vp, vp, vp, ft, vp, vp, vp, vp, i32], i64)
                _declare(lib, f"bdx_cpu_spmv_{suf}", [i64, vp, vp, vp, vp, vp, vp, i32])
                _declare(lib, f"bdx_cpu_interp_f_{suf}", [vp, vp, vp, vp])
            _host = lib
    return _host


def hip_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def hip():
    """The HIP kernel library (gfx950).  Raises if unavailable."""
    global _hip
    with _lock:
        if _hip is None:
            import torch  # noqa: F401  (shares the HIP runtime; see module doc)
            override = os.environ.get("BDX_HIP_LIB")  # A/B experiments: a variant .so
            path = override if override else _build.build_hip()
            lib = ctypes.CDLL(str(path), mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)
            _loaded["hip"] = str(path)
            from . import hip_api
            hip_api.declare(lib)
            _hip = lib
    return _hip


def build_flags() -> dict:
    """Build facts of the loaded HIP library that decide whether a timing is
    valid: the arch, the library file, and whether it is the production build
    (the in-tree libbdx_hip.so, built with no extra flags) rather than an
    A/B variant (BDX_HIP_LIB) or a bounds-checked debug build (BDX_DEBUG)."""
    lib = hip()
    fn = lib.bdx_build_debug
    fn.restype = ctypes.c_int
    debug = int(fn())
    path = _loaded.get("hip", "")
    production = os.path.abspath(path) == os.path.abspath(str(_build.HIP_SO))
    return {"arch": _build.HIP_ARCH, "hiplib": os.path.basename(path), "debug": debug,
            "production": production, "valid": production and not debug}


def loaded_libraries() -> list[str]:
    out = []
    if _host is not None:
        out.append(_loaded.get("host", str(_build.HOST_SO)))
    if _hip is not None:
        out.append(_loaded.get("hip", str(_build.HIP_SO)))
    return out
