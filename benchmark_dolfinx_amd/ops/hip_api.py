"""ctypes signatures of libbdx_hip.so (see csrc/hip/*.hip)."""

from __future__ import annotations

import ctypes

vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_int64
f64 = ctypes.c_double
f32 = ctypes.c_float


def _d(lib, name, argtypes, restype=i32):
    fn = getattr(lib, name)
    fn.argtypes = argtypes
    fn.restype = restype


def declare(lib) -> None:
    _d(lib, "bdx_hip_partials_size", [])
    _d(lib, "bdx_device_info", [i32, ctypes.c_char_p, i32])
    for suf in ("f64", "f32"):
        ft = f64 if suf == "f64" else f32
        _d(lib, f"bdx_dot_{suf}", [i64, i64, i64, i64, i64, vp, vp, vp, vp, i32, vp])
        _d(lib, f"bdx_cg_update_{suf}",
           [i64, i64, i64, i64, i64, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp])
        _d(lib, f"bdx_p_update_{suf}", [i64, i64, i64, i64, i64, vp, vp, vp, i32, i32, vp])
        _d(lib, f"bdx_axpy_{suf}", [i64, i64, i64, i64, i64, vp, f64, vp, vp, vp])
        _d(lib, f"bdx_box_copy_{suf}", [i32, vp, i64, i64, vp, i32, i64, vp, vp])
        _d(lib, f"bdx_box_copy_lat_{suf}", [i32, vp, vp, vp, i32, i64, vp, vp])
        _d(lib, f"bdx_layout_convert_{suf}", [i32, vp, vp, vp, vp])
        _d(lib, f"bdx_v1_apply_{suf}",
           [i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, f64, vp, vp, vp, vp, vp, vp])
        _d(lib, f"bdx_geometry_{suf}", [vp, i32, vp, vp, vp, vp, vp, vp, vp])
        _d(lib, f"bdx_dofmap_apply_{suf}",
           [i32, i32, i32, i32, vp, vp, i32, i64, vp, vp, vp, vp, vp, f64, vp, vp, vp, vp, vp, vp,
            vp, i32, i32, i32, i32, vp, vp, vp])
        _d(lib, f"bdx_dofmap_cg_update_{suf}", [i64, vp, vp, vp, vp, i32, i32, vp, vp, vp])
        _d(lib, f"bdx_dofmap_xflush_{suf}", [i64, vp, vp, vp, i32, i32, vp])
        _d(lib, f"bdx_dofmap_geometry_{suf}", [i32, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp])
        _d(lib, f"bdx_spmv_{suf}", [i64, vp, vp, vp, vp, vp, vp, i32, vp])
        for P in range(1, 8):
            name = f"bdx_fused_apply_{suf}_p{P}"
            if hasattr(lib, name):
                _d(lib, name, [i32, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                               vp, vp, vp, vp, f64, vp, vp, i32, i32, i32, i32, vp])
        for P, v in [(P, v) for P in range(1, 8) for v in (2, 3)]:
            if hasattr(lib, f"bdx_fused{v}_segments_{suf}_p{P}"):
                _d(lib, f"bdx_fused{v}_segments_{suf}_p{P}", [i32, i32, i32, i32])
        for P, v in [(P, v) for P in range(1, 8) for v in (2, 3, 4, 5)]:
            name = f"bdx_fused{v}_apply_{suf}_p{P}"
            if hasattr(lib, name):
                _d(lib, name, [i32, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                               vp, vp, f64, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp])
        _d(lib, f"bdx_fused_finalize_{suf}", [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp])
        _d(lib, f"bdx_cg_update_iface_{suf}", [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32,
                                                vp, i32, i32, i32, vp, vp])
        _d(lib, f"bdx_xflush_{suf}", [vp, vp, vp, vp, vp, i32, i32, vp])
        _d(lib, f"bdx_fused_tables_{suf}", [i32, i32, vp, vp, vp])
        _d(lib, f"bdx_fused3_tables_{suf}", [i32, i32, vp, vp, vp])
        for P in range(1, 8):
            if hasattr(lib, f"bdx_fused5_tables_{suf}_p{P}"):
                _d(lib, f"bdx_fused5_tables_{suf}_p{P}", [i32, i32, vp, vp, vp, vp])
                _d(lib, f"bdx_fused5_tile_p{P}_{suf}", [i32, vp, vp])
                _d(lib, f"bdx_fused5_segments_{suf}_p{P}", [i32, i32, i32])
    _d(lib, "bdx_fused_tile", [i32, vp, vp])
    # native CG runtime (runtime.hip)
    _d(lib, "bdx_rt_nccl_unique_id", [vp])
    _d(lib, "bdx_rt_rccl_selftest", [vp, i32, vp])
    _d(lib, "bdx_rt_create", [i32, vp, vp, vp, f64, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32,
                              i64, vp, vp, vp], vp)
    _d(lib, "bdx_rt_create_dofmap", [i32, vp, vp, i64, f64, vp, vp, vp, vp, i32, i32, i32, i64,
                                     vp], vp)
    _d(lib, "bdx_dofmap_nblocks", [i32, i32])
    _d(lib, "bdx_dofmap_set_mfma", [i32])
    _d(lib, "bdx_dofmap_uses_mfma", [i32, i32])
    _d(lib, "bdx_rt_tiled", [vp])
    _d(lib, "bdx_rt_connect", [vp, vp, i32])
    _d(lib, "bdx_rt_comm_count", [vp])
    _d(lib, "bdx_rt_overlap", [vp])
    _d(lib, "bdx_rt_comm_priority", [vp, vp])
    _d(lib, "bdx_rt_preflight", [vp, f64, vp])
    _d(lib, "bdx_rt_overlap_probe", [vp, i64, vp, i32, vp])
    _d(lib, "bdx_rt_bind_x", [vp, vp])
    _d(lib, "bdx_rt_wait", [vp])
    _d(lib, "bdx_rt_profile", [vp, ctypes.c_long, vp, i32])
    _d(lib, "bdx_rt_reset", [vp])
    _d(lib, "bdx_rt_iterate", [vp, ctypes.c_long])
    _d(lib, "bdx_rt_iterate_timed", [vp, ctypes.c_long, vp])
    _d(lib, "bdx_rt_state", [vp, vp, vp])
    _d(lib, "bdx_rt_destroy", [vp], None)
    _d(lib, "bdx_rt_release_group", [i64], None)
    _d(lib, "bdx_reduce_partials", [vp, i32, vp, i32, vp])
    _d(lib, "bdx_dofmap_mark_writers", [vp, i32, vp, i32, vp, i32, vp, i64, vp])
    del ft
