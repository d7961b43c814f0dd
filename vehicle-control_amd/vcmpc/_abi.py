"""ctypes binding of ``libvcmpc.so`` (the C ABI declared in ``include/vcmpc.h``).

This is the "thin ctypes C-ABI shim" of the north star: struct mirrors of
``vc_params`` and typed prototypes of every ``vc_*`` entry point.  There is no
CPU fallback anywhere in the package -- if the shared library is missing or was
built for a different ABI, importing the solver raises.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_NAME = "libvcmpc.so"
LIB_PATH = os.environ.get("VCMPC_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME))
ABI_VERSION = 13
VC_MAX_OBSTACLES = 16
OBS_MARGIN_MIN = 0.05  # VC_OBS_MARGIN_MIN (csrc/vc_kernels.hpp)

VC_MODEL_KINEMATIC, VC_MODEL_DYNAMIC, VC_MODEL_CASCADED = 0, 1, 2
VC_F64, VC_F32 = 0, 1
VC_HOST_PTRS, VC_DEVICE_PTRS = 0, 1
VC_TYRE_FIALA, VC_TYRE_LINEAR = 0, 1
VC_SOLVED, VC_MAX_ITER, VC_NONFINITE, VC_OUT_OF_DOMAIN = 0, 1, 2, 3
VC_OK, VC_E_ARG, VC_E_HIP, VC_E_UNSUPPORTED = 0, -1, -2, -3

STATUS_NAMES = {VC_SOLVED: "solved", VC_MAX_ITER: "max_iter", VC_NONFINITE: "nonfinite",
                VC_OUT_OF_DOMAIN: "out_of_domain"}


class vc_kin_car(C.Structure):
    _fields_ = [("l", C.c_double)]


class vc_dyn_car(C.Structure):
    _fields_ = [(k, C.c_double) for k in (
        "l", "m", "Izz", "a", "b", "h", "eps", "Peng",
        "Xdf", "Xdr", "Xbf", "Xbr", "Caf", "Car",
        "Cd", "muf", "mur", "theta", "phi", "Av2", "Frr")] + [("tyre", C.c_int32), ("pad_", C.c_int32)]


class vc_kin_mpc(C.Structure):
    _fields_ = [(k, C.c_double) for k in (
        "w_time", "w_ey", "w_epsi", "w_v", "w_w", "w_a", "w_dev", "w_b",
        "a_min", "a_max", "w_min", "w_max",
        "v_min", "v_max", "delta_min", "delta_max", "ey_min", "ey_max", "w_obs")]


class vc_dyn_mpc(C.Structure):
    _fields_ = [(k, C.c_double) for k in (
        "w_time", "w_speed", "w_ey", "w_epsi", "w_w", "w_Fx", "w_dev", "w_b", "w_slip",
        "w_min", "w_max", "Ux_min", "max_speed", "delta_min", "delta_max", "ey_min", "ey_max",
        "fx_scale", "trust_Fx")] + [("sqp_iters", C.c_int32), ("pad_", C.c_int32), ("w_obs", C.c_double)]


class vc_qp(C.Structure):
    _fields_ = [("prox", C.c_double), ("tol", C.c_double), ("trust_a", C.c_double), ("trust_w", C.c_double),
                ("max_iter", C.c_int32), ("polish", C.c_int32), ("solver", C.c_int32), ("kin_sqp", C.c_int32),
                ("shift", C.c_int32), ("ms", C.c_int32), ("elastic", C.c_double)]


class vc_obstacles(C.Structure):
    _fields_ = [("n", C.c_int32), ("inside", C.c_int32), ("margin_min", C.c_double),
                ("s", C.c_double * VC_MAX_OBSTACLES), ("ey", C.c_double * VC_MAX_OBSTACLES),
                ("radius", C.c_double * VC_MAX_OBSTACLES)]


class vc_casc_mpc(C.Structure):
    _fields_ = [("horizon_pm", C.c_int32), ("pad_", C.c_int32)] + [(k, C.c_double) for k in (
        "ds_pm", "w_dev_pm", "w_Fy", "w_switch", "V_min", "ey_min_pm", "ey_max_pm")]


class vc_params(C.Structure):
    _fields_ = [("kin_car", vc_kin_car), ("dyn_car", vc_dyn_car), ("kin_mpc", vc_kin_mpc), ("qp", vc_qp),
                ("dyn_mpc", vc_dyn_mpc), ("obs", vc_obstacles), ("casc", vc_casc_mpc)]


class VcError(RuntimeError):
    """Raised for a negative ``vc_*`` return code (API or HIP error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"vcmpc error {code}: {msg}")
        self.code = code


_vp = C.c_void_p
_i32p = C.POINTER(C.c_int32)

# name -> (restype, argtypes); every symbol include/vcmpc.h declares
PROTOTYPES = {
    "vc_abi_version": (C.c_int, []),
    "vc_params_sizeof": (C.c_int, []),
    "vc_create": (_vp, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(vc_params)]),
    "vc_destroy": (None, [_vp]),
    "vc_last_error": (C.c_char_p, [_vp]),
    "vc_set_stream": (C.c_int, [_vp, _vp]),
    "vc_synchronize": (C.c_int, [_vp]),
    "vc_set_obstacles": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double]),
    "vc_solve": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_solve_diag": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_solve_from": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_solve_debug": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_debug_stride": (C.c_int, []),
    "vc_debug_qp_fault": (C.c_int, [_vp, C.c_int, C.c_int]),
    "vc_debug_rcp": (C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int]),
    "vc_rollout": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_linearize": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_condense": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_plant_step": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, _vp, C.c_int]),
    "vc_spatial_step": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, C.c_int]),
    "vc_ode": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_int, _vp, C.c_int]),
    "vc_track_set": (C.c_int, [_vp, C.c_int, C.c_double, C.c_double, _vp]),
    "vc_track_k": (C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int]),
    "vc_horizon": (C.c_int, [_vp, C.c_int, _vp, _vp, C.c_double, _vp, _vp, C.c_int]),
    "vc_drive": (C.c_int, [_vp, C.c_int, _vp, _vp, C.c_double, _vp, C.c_int]),
    "vc_simulate": (C.c_int, [_vp, C.c_int, C.c_int, C.c_double, C.c_double, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int]),
}

_LIB = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load ``libvcmpc.so`` once, bind every prototype and check the ABI."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # SONAME as /opt/rocm's).  Loading torch first makes the dynamic loader bind
    # libvcmpc.so to that copy; loaded the other way round, two runtimes coexist
    # and torch's device discovery fails.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise ImportError(
            f"{p} not found: build it with `make -C vehicle-control_amd/csrc` "
            "(or __graft_entry__.build()); vcmpc has no CPU fallback")
    lib = C.CDLL(p)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)  # AttributeError = missing export
        fn.restype = res
        fn.argtypes = args
    if lib.vc_abi_version() != ABI_VERSION:
        raise ImportError(f"{p}: ABI version {lib.vc_abi_version()} != {ABI_VERSION}")
    if lib.vc_params_sizeof() != C.sizeof(vc_params):
        raise ImportError(f"{p}: sizeof(vc_params) {lib.vc_params_sizeof()} != ctypes {C.sizeof(vc_params)}")
    if path is None:
        _LIB = lib
    return lib


def check(lib, ctx, code: int) -> None:
    if code != VC_OK:
        msg = lib.vc_last_error(ctx)
        raise VcError(code, msg.decode() if msg else "")
