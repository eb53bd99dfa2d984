"""ctypes declarations of the C ABIs (include/gpusolve_hip.h, include/gpusolve_driver.h, and the
diagnostics library's include/gpusolve_diag.h, which only tools/ and tests/ load).

The shared libraries are built in-tree by gpu-solve_amd/Makefile (``__graft_entry__.build()``).
There is no fallback: if a library is missing, loading raises ``ImportError`` naming the build step.
"""
import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # gpu-solve_amd/
LIB_DIR = os.path.join(PKG_ROOT, "lib")
BIN_DIR = os.path.join(PKG_ROOT, "bin")
KERNEL_LIB = os.path.join(LIB_DIR, "libgpusolve_hip.so")
DIAG_LIB = os.path.join(LIB_DIR, "libgpusolve_diag.so")  # tools/ and tests/ only (include/gpusolve_diag.h)
DRIVER_LIB = os.path.join(LIB_DIR, "libgpusolve_driver.so")
EXECUTABLE = os.path.join(BIN_DIR, "GpuSolve-hip")

GS_LINEAR, GS_NONLINEAR, GS_NEWTON = 0, 1, 2
GS_NEWTON_B = 3  # NEWTON with the precomputed linearisation factor B (include/gpusolve_hip.h)
GS_NEWTON_G = 4  # GS_NEWTON_B whose factor field holds gamma everywhere (the first Newton iteration)
GS_EINVAL = 100001

dptr = C.POINTER(C.c_double)
i64 = C.c_int64


class gs_stencil(C.Structure):
    _fields_ = [("s", C.c_double * 7), ("ox", C.c_int * 7), ("oy", C.c_int * 7), ("oz", C.c_int * 7)]


class gs_level(C.Structure):
    _fields_ = [("nx", i64), ("ny", i64), ("nz", i64), ("ldy", i64), ("ldz", i64), ("z0", i64), ("h", C.c_double)]


class gs_coarse_level(C.Structure):
    _fields_ = [("v", C.c_void_p), ("v_alt", C.c_void_p), ("f", C.c_void_p), ("r", C.c_void_p),
                ("rest_v", C.c_void_p), ("newton_v", C.c_void_p), ("geom", gs_level), ("v_zero", C.c_int)]


class gs_params(C.Structure):
    _fields_ = [("maxiter", i64), ("tol", C.c_double), ("dims", i64 * 3), ("mode", C.c_int), ("pre", i64),
                ("post", i64), ("omega", C.c_double), ("gamma", C.c_double), ("stencil", gs_stencil)]


# name -> (restype, argtypes); void* is used for device pointers and streams
KERNEL_API = {
    "gs_field_layout": (C.c_int, [i64, i64, i64, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]),
    "gs_rhs_init": (C.c_int, [C.POINTER(gs_level), C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_void_p]),
    "gs_jacobi_sweep": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double, C.c_double,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_jacobi_sweep_norm": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double, C.c_double,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_jacobi_sweep2_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level)]),
    "gs_jacobi_sweep2_supported_mode": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double, C.c_double,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "gs_jacobi_sweep2_norm": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                        C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                        C.c_int, C.c_void_p, C.c_void_p]),
    "gs_jacobi_sweep2_num_partials": (i64, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2_kernel": (C.c_char_p, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2_prolong_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2_prolong": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double, C.c_double,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(gs_level), C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "gs_jacobi_sweep2_prolong_ws_elems": (i64, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2_prolong_ws": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                              C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(gs_level),
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, i64,
                                              C.c_void_p]),
    "gs_residual": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double, C.c_void_p,
                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_residual_num_partials": (i64, [C.POINTER(gs_stencil), C.POINTER(gs_level)]),
    "gs_sumsq_finish": (C.c_int, [C.c_void_p, i64, C.c_void_p, C.c_int, C.c_void_p]),
    "gs_restrict": (C.c_int, [C.c_void_p, C.POINTER(gs_level), C.c_void_p, C.POINTER(gs_level), C.c_void_p]),
    "gs_residual_restrict": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.POINTER(gs_level), C.c_void_p]),
    "gs_residual_restrict_slab_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level)]),
    "gs_residual_restrict_slab": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.POINTER(gs_level), C.c_int, C.c_void_p]),
    "gs_tiled_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_smooth2_restrict_tiled": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                            C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.POINTER(gs_level), C.c_void_p]),
    "gs_prolong_smooth2_tiled": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int, C.c_double,
                                           C.c_double, C.c_void_p, C.c_void_p, C.POINTER(gs_level), C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_restrict2": (C.c_int, [C.c_void_p, C.POINTER(gs_level), C.c_void_p, C.c_void_p, C.POINTER(gs_level),
                               C.c_void_p]),
    "gs_interpolate": (C.c_int, [C.c_void_p, C.POINTER(gs_level), C.c_void_p, C.POINTER(gs_level), C.c_void_p]),
    "gs_prolong_add": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(gs_level), C.c_void_p, C.POINTER(gs_level),
                                 C.c_void_p]),
    "gs_apply_op": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                              C.c_void_p]),
    "gs_apply_op_add": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                                  C.c_void_p]),
    "gs_newton_F": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_newton_F_update_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level)]),
    "gs_newton_F_update_restrict_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.POINTER(gs_level)]),
    "gs_newton_F_update_restrict": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.POINTER(gs_level), C.c_void_p]),
    "gs_newton_F_update_restrict_bfac": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.POINTER(gs_level), C.c_void_p, C.c_void_p]),
    "gs_newton_bfac": (C.c_int, [C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_newton_F_update": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_fill": (C.c_int, [C.c_void_p, C.c_double, i64, C.c_void_p]),
    "gs_copy": (C.c_int, [C.c_void_p, C.c_void_p, i64, C.c_void_p]),
    "gs_axpy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_double, i64, C.c_void_p]),
    "gs_coarse_cycle_max_levels": (C.c_int, []),
    "gs_coarse_cycle": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_coarse_level), C.c_int, C.c_int, C.c_double,
                                  C.c_double, C.c_int, C.c_int, C.c_void_p]),
    "gs_strerror": (C.c_char_p, [C.c_int]),
    "gs_build_info": (C.c_char_p, []),
}

DRIVER_API = {
    "gs_parse_config": (C.c_int, [C.c_char_p, C.POINTER(gs_params)]),
    "gs_grid_create": (C.c_void_p, [C.POINTER(gs_params)]),
    "gs_grid_destroy": (None, [C.c_void_p]),
    "gs_grid_solve": (C.c_int, [C.c_void_p, C.c_int, dptr, C.c_int, C.POINTER(C.c_int)]),
    "gs_grid_vcycle": (C.c_int, [C.c_void_p, dptr]),
    "gs_grid_jacobi": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "gs_grid_residual_norm": (C.c_int, [C.c_void_p, C.c_int, dptr]),
    "gs_grid_num_levels": (C.c_int, [C.c_void_p]),
    "gs_grid_level_fused": (C.c_int, [C.c_void_p, C.c_int]),
    "gs_grid_level": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(gs_level)]),
    "gs_grid_field": (C.c_void_p, [C.c_void_p, C.c_int, C.c_int]),
    "gs_grid_stream": (C.c_void_p, [C.c_void_p]),
    "gs_grid_download": (C.c_int, [C.c_void_p, C.c_int, C.c_int, dptr]),
    "gs_grid_upload": (C.c_int, [C.c_void_p, C.c_int, C.c_int, dptr]),
    "gs_grid_sync": (C.c_int, [C.c_void_p]),
    "gs_grid_comm_stats": (C.c_int, [C.c_void_p, dptr, C.POINTER(C.c_int64)]),
    "gs_grid_comm_stats_max": (C.c_int, [C.c_void_p, dptr]),
    "gs_grid_metrics": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int, dptr, C.c_int]),
    "gs_dump_write": (C.c_int, [dptr, i64, i64, i64, C.c_char_p]),
    "gs_grid_dump": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p]),
    "gs_grid_time_jacobi": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]),
    "gs_grid_time_vcycles": (C.c_int, [C.c_void_p, C.c_int, dptr, dptr]),
    "gs_zslab_plan": (C.c_int, [C.POINTER(i64), C.c_int, i64, C.c_int, C.POINTER(C.c_int), C.POINTER(i64),
                                C.POINTER(i64)]),
    "gs_zslab_schedule": (C.c_int, [C.POINTER(gs_params), C.c_int, C.c_int, i64, C.c_char_p, i64, C.POINTER(i64)]),
    "gs_rccl_unique_id": (C.c_int, [C.POINTER(C.c_ubyte)]),
    "gs_uid_publish": (C.c_int, [C.c_char_p, C.POINTER(C.c_ubyte)]),
    "gs_uid_default_path": (C.c_int, [C.c_char_p, C.c_int]),
    "gs_uid_await": (C.c_int, [C.c_char_p, C.c_double, C.POINTER(C.c_ubyte)]),
    "gs_grid_create_rccl": (C.c_void_p, [C.POINTER(gs_params), C.c_int, C.c_int, C.POINTER(C.c_ubyte)]),
    "gs_grid_create_rccl_ctas": (C.c_void_p, [C.POINTER(gs_params), C.c_int, C.c_int, C.POINTER(C.c_ubyte), C.c_int]),
    "gs_grid_comm_ctas": (C.c_int, [C.c_void_p]),
    "gs_rccl_channels_per_peer_hint": (C.c_int, [C.c_int]),
    "gs_zslab_loopback_run": (C.c_int, [C.POINTER(gs_params), C.c_int, i64, C.c_int, C.c_int, dptr, C.c_int,
                                        C.POINTER(C.c_int), dptr]),
    "gs_debug_bounded_wait": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_char_p, C.c_int]),
    "gs_debug_loopback_abort": (C.c_int, [C.c_int, C.c_int]),
    "gs_last_error": (C.c_char_p, []),
}

# libgpusolve_diag.so (include/gpusolve_diag.h): tuning variants, bandwidth probes, k_prr — not the product
DIAG_API = {
    "gs_smooth2_restrict_zero_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.POINTER(gs_level),
                                                     C.c_int]),
    "gs_smooth2_restrict_zero": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.POINTER(gs_level), C.c_void_p]),
    "gs_jacobi_sweep2_restrict_supported": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level),
                                                      C.POINTER(gs_level), C.c_int]),
    "gs_jacobi_sweep2_restrict": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.POINTER(gs_level), C.c_void_p]),
    "gs_jacobi_sweep2_restrict_num_partials": (i64, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.POINTER(gs_level)]),
    "gs_debug_num_variants": (C.c_int, []),
    "gs_debug_variant_name": (C.c_char_p, [C.c_int]),
    "gs_debug_sweep_variant": (C.c_int, [C.c_int, C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_debug_div_check": (C.c_int, [C.c_void_p, i64, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_debug_nb_quot": (C.c_int, [C.c_void_p, C.c_void_p, i64, C.c_void_p, C.c_void_p]),
    "gs_debug_num_pair_variants": (C.c_int, []),
    "gs_debug_pair_variant_name": (C.c_char_p, [C.c_int]),
    "gs_debug_pair_timestamps": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "gs_debug_pair_reverse": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "gs_debug_pair_blocks": (i64, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_int]),
    "gs_debug_pair_shape": (C.c_int, [C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "gs_debug_pair_variant": (C.c_int, [C.c_int, C.POINTER(gs_stencil), C.POINTER(gs_level), C.c_double, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "gs_debug_stream_triad": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, i64, C.c_void_p]),
    "gs_debug_phase_probe": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_debug_march": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(gs_level), C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_debug_bw": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, i64, C.c_void_p,
                              C.c_void_p]),
}

_cache = {}


def _load(path, api):
    if path in _cache:
        return _cache[path]
    if not os.path.exists(path):
        raise ImportError(f"{path} is not built: run `make -C gpu-solve_amd` (or __graft_entry__.build())")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (res, args) in api.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _cache[path] = lib
    return lib


def kernels():
    """The thin C-ABI launcher library (libgpusolve_hip.so)."""
    return _load(KERNEL_LIB, KERNEL_API)


def diag():
    """The diagnostics library (libgpusolve_diag.so): measurement and tuning code, never the product path."""
    kernels()
    return _load(DIAG_LIB, DIAG_API)


def driver():
    """The host driver library (libgpusolve_driver.so); loads the kernel library first."""
    kernels()
    return _load(DRIVER_LIB, DRIVER_API)
