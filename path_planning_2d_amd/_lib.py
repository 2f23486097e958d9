"""ctypes binding of ``libpp2_hip.so`` (the C ABI declared in include/pp2.h).

The shared library is built in-tree (``path_planning_2d_amd/libpp2_hip.so``,
see ``csrc/Makefile`` / ``__graft_entry__.build()``).  There is no fallback:
if the library is missing or fails to load, importing the product API raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# PP2_LIBRARY points at a diagnostic build of the same ABI (tools/micro/).
# include/pp2.h PP2_ABI_VERSION (tests/test_abi.py checks the two agree)
PP2_ABI_VERSION = 3
LIB_PATH = os.environ.get("PP2_LIBRARY") or os.path.join(PKG_DIR, "libpp2_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "pp2.h")

RCCL_ID_BYTES = 128

PP2_OK = 0
STATUS_NAMES = {0: "PP2_OK", 1: "PP2_EINVAL", 2: "PP2_EHIP", 3: "PP2_EIO",
                4: "PP2_ENOMEM", 5: "PP2_ESTATE", 6: "PP2_ERCCL"}


class Pp2Error(RuntimeError):
    def __init__(self, status: int, fn: str, message: str):
        self.status = status
        super().__init__(f"{fn}: {STATUS_NAMES.get(status, status)}: {message}")


_vp = C.c_void_p
_u8p = C.POINTER(C.c_uint8)
_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int)
_u32p = C.POINTER(C.c_uint32)
_f64p = C.POINTER(C.c_double)

# name -> argtypes (all return int status unless listed in _RESTYPES)
SIGNATURES = {
    "pp2_abi_version": [],
    "pp2_status_string": [C.c_int],
    "pp2_last_error": [],
    "pp2_device_count": [_i32p],
    "pp2_create": [C.POINTER(_vp), C.c_int, C.c_uint32, C.c_uint32, _u8p,
                   C.c_int32, C.c_int32, C.c_float],
    "pp2_create_shard": [C.POINTER(_vp), C.c_int, C.c_uint32, C.c_uint32,
                         C.c_uint32, C.c_uint32, _u8p, C.c_int32, C.c_int32,
                         C.c_float],
    "pp2_destroy": [_vp],
    "pp2_set_stream": [_vp, _vp],
    "pp2_synchronize": [_vp],
    "pp2_get_geometry": [_vp, _u32p, _u32p, _u32p, _u32p],
    "pp2_set_cells_per_lane": [_vp, C.c_int],
    "pp2_set_tuning": [_vp, C.c_int, C.c_int],
    "pp2_comm_rounds": [_vp, C.POINTER(C.c_int), C.POINTER(C.c_longlong), _f32p, C.c_int],
    "pp2_model_generate": [_vp],
    "pp2_model_download": [_vp, _f32p, _f32p, _f32p, _f32p],
    "pp2_model_upload": [_vp, _f32p, _f32p, _f32p, _f32p],
    "pp2_model_save": [_vp, C.c_char_p],
    "pp2_model_load": [_vp, C.c_char_p],
    "pp2_model_dict_info": [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pp2_loop_steps_per_launch": [_vp, C.POINTER(C.c_int)],
    "pp2_resident_tiling": [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pp2_resident_launches": [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pp2_resident_status": [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pp2_belief_set": [_vp, _f32p],
    "pp2_belief_get": [_vp, _f32p],
    "pp2_belief_update": [_vp, C.c_uint8, C.c_uint8],
    "pp2_belief_get_raw": [_vp, _f32p, _f32p],
    "pp2_belief_mass": [_vp, _f32p],
    "pp2_mdp_reset": [_vp],
    "pp2_mdp_sweep": [_vp, C.c_int],
    "pp2_mdp_solve": [_vp, C.c_int, _i32p, _f64p],
    "pp2_mdp_get": [_vp, _f32p, _u8p],
    "pp2_loop_step": [_vp, C.c_uint8, C.c_uint8],
    # trajectories go in as bytes objects (c_char_p: a pointer to their
    # buffer, no per-call ctypes array objects -- ~8 us of host time per call)
    "pp2_loop_run": [_vp, C.c_int, C.c_char_p, C.c_char_p],
    "pp2_fib_reset": [_vp],
    "pp2_fib_sweep": [_vp, C.c_int],
    "pp2_fib_solve": [_vp, C.c_int, _i32p, _f32p],
    "pp2_fib_get": [_vp, _f32p],
    "pp2_fib_set": [_vp, _f32p],
    "pp2_fib_save": [_vp, C.c_char_p],
    "pp2_fib_load": [_vp, C.c_char_p],
    "pp2_pbvi_belief_set": [_vp, _f32p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)],
    "pp2_pbvi_set_beliefs": [_vp, C.c_uint32, _f32p],
    "pp2_pbvi_get_beliefs": [_vp, _f32p],
    "pp2_pbvi_backup": [_vp, C.c_int],
    "pp2_pbvi_solve": [_vp, _f32p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)],
    "pp2_pbvi_info": [_vp, _u32p, _i32p],
    "pp2_pbvi_get": [_vp, _f32p, _u8p],
    "pp2_pbvi_set": [_vp, C.c_uint32, _f32p, _u8p],
    "pp2_pbvi_evaluate": [_vp, C.c_int, _f32p, _f32p, _u8p],
    "pp2_pbvi_save": [_vp, C.c_char_p],
    "pp2_pbvi_load": [_vp, C.c_char_p, C.c_uint32],
    "pp2_planner_default_params": [_vp],
    "pp2_planner_create": [C.POINTER(_vp), _vp, _vp],
    "pp2_planner_destroy": [_vp],
    "pp2_planner_step": [_vp, C.c_uint8, C.c_uint8, _f32p, _u8p, _f32p],
    "pp2_planner_reset": [_vp],
    "pp2_planner_info": [_vp, _vp],
    "pp2_curand_uniforms": [C.c_uint64, C.c_int, _f32p, _f32p],
    "pp2_rollout_create": [C.POINTER(_vp), _vp, C.c_int, C.c_int],
    "pp2_rollout_destroy": [_vp],
    "pp2_rollout_set_root": [_vp, _f32p],
    "pp2_rollout_run": [_vp, _u8p, _u8p],
    "pp2_rollout_results": [_vp, _f32p, _f32p, _f32p, _f32p],
    "pp2_rollout_get_belief": [_vp, C.c_int, _f32p],
    "pp2_shard_group_create": [C.POINTER(_vp), C.POINTER(_vp), C.c_int],
    "pp2_shard_group_destroy": [_vp],
    "pp2_shard_group_loop_step": [_vp, C.c_uint8, C.c_uint8],
    "pp2_shard_group_loop_run": [_vp, C.c_int, C.c_char_p, C.c_char_p],
    "pp2_shard_group_belief_update": [_vp, C.c_uint8, C.c_uint8],
    "pp2_shard_group_mdp_sweep": [_vp, C.c_int],
    "pp2_shard_group_mdp_solve": [_vp, C.c_int, _i32p, _f64p],
    "pp2_shard_group_fib_sweep": [_vp, C.c_int],
    "pp2_shard_group_synchronize": [_vp],
    "pp2_rccl_unique_id": [_u8p],
    "pp2_shard_comm_init": [_vp, _u8p, C.c_int, C.c_int],
}
_RESTYPES = {"pp2_status_string": C.c_char_p, "pp2_last_error": C.c_char_p}

_lib = None


def load() -> C.CDLL:
    """Load the in-tree library (raises if it is missing -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C "
            f"{os.path.join(PKG_DIR, 'csrc')}` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None and os.environ.get("PP2_ALLOW_PARTIAL_ABI") == "1":
            continue  # diagnostic only: an older build (A/B timing) lacks newer entry points
        if fn is None:
            raise ImportError(f"{LIB_PATH} does not export {name}")
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, C.c_int)
    partial = os.environ.get("PP2_ALLOW_PARTIAL_ABI") == "1"
    if getattr(lib, "pp2_abi_version", None) is not None:
        ver = lib.pp2_abi_version()
    elif partial:
        ver = 0  # a diagnostic build older than the version symbol
    else:
        raise ImportError(f"{LIB_PATH} does not export pp2_abi_version")
    if ver != PP2_ABI_VERSION:
        if not partial:
            raise ImportError(f"{LIB_PATH} has ABI version {ver}, this package expects "
                              f"{PP2_ABI_VERSION} (rebuild the library)")
        import warnings
        warnings.warn(f"PP2_ALLOW_PARTIAL_ABI: {LIB_PATH} has ABI version {ver}, "
                      f"expected {PP2_ABI_VERSION}")
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    st = getattr(lib, name)(*args)
    if st != PP2_OK:
        msg = lib.pp2_last_error()
        raise Pp2Error(st, name, msg.decode() if msg else "")


def exported_symbols():
    return list(SIGNATURES)
