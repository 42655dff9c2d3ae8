"""ctypes binding of librbhip.so (include/rbhip.h).

There is no fallback: if the library is missing, or no HIP device is
present, every compute entry raises.  Build it with
`python -c "import __graft_entry__ as g; g.build()"` (or `make -C
rigidbody-simulation_amd/csrc`).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RBHIP_LIB_PATH: a diagnostic build of the same library (A/B runs)
LIB_PATH = os.environ.get("RBHIP_LIB_PATH") or os.path.join(HERE, "librbhip.so")

RB_OK = 0
ERRNAMES = {-22: "EINVAL", -12: "ENOMEM", -19: "ENODEV", -75: "EOVERFLOW", -95: "EUNSUPPORTED",
            -33: "EDOM"}
RB_BODY_SPHERE, RB_BODY_BOX = 0, 1
RB_F64, RB_F32 = 0, 1
RB_NORMAL_ORIENTED, RB_NORMAL_RAW = 0, 1
RB_CK_PLANE_SPHERE, RB_CK_PLANE_BOX0, RB_CK_SPHERE_SPHERE = 0, 1, 16
RB_CK_SPHERE_BOX, RB_CK_BOX_BOX0, RB_CK_BOX_EDGE = 17, 32, 40
RB_LAW_MUJOCO, RB_LAW_BALLS = 0, 1


class RbError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        self.code = code
        super().__init__(f"{where} failed: {ERRNAMES.get(code, code)}: {msg}")


class SceneDesc(C.Structure):
    _fields_ = [("n_bodies", C.c_int64), ("n_planes", C.c_int32), ("dtype", C.c_int32),
                ("normal_convention", C.c_int32), ("device", C.c_int32), ("rank", C.c_int32),
                ("world_size", C.c_int32), ("max_partners", C.c_int32),
                ("bucket_capacity", C.c_int32), ("kind", C.c_void_p), ("mass", C.c_void_p),
                ("inertia", C.c_void_p), ("size", C.c_void_p), ("planes", C.c_void_p),
                ("gravity", C.c_double * 3)]


# every symbol include/rbhip.h declares, with its ctypes signature
_P, _I64, _I32, _D = C.c_void_p, C.c_int64, C.c_int32, C.c_double
SIGNATURES = {
    "rb_world_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SceneDesc)]),
    "rb_world_destroy": (None, [_P]),
    "rb_last_error": (C.c_char_p, []),
    "rb_version": (C.c_char_p, []),
    "rb_set_stream": (C.c_int, [_P, _P]),
    "rb_set_state": (C.c_int, [_P, _P, _P]),
    "rb_get_state": (C.c_int, [_P, _P, _P]),
    "rb_set_xfrc": (C.c_int, [_P, _P]),
    "rb_step": (C.c_int, [_P, _I64, _D, _D, _D, _D]),
    "rb_step_async": (C.c_int, [_P, _I64, _D, _D, _D, _D]),
    "rb_sync": (C.c_int, [_P]),
    "rb_shard_step": (C.c_int, [_P, _D, _D, _D, _D]),
    "rb_shard_exchange_done": (C.c_int, [_P]),
    "rb_gpos_buffer": (C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(_I64), C.POINTER(_I32)]),
    "rb_gquat_buffer": (C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(_I64), C.POINTER(_I32)]),
    "rb_comm_unique_id": (C.c_int, [_P, _I32]),
    "rb_shard_comm_init": (C.c_int, [_P, _P, _I32]),
    "rb_shard_run": (C.c_int, [_P, _I64, _D, _D, _D, _D]),
    "rb_p2p_handles": (C.c_int, [_P, _P, _I64, C.POINTER(_I64)]),
    "rb_p2p_connect": (C.c_int, [_P, _P, _I64]),
    "rb_p2p_halo": (C.c_int, [_P, _I32]),
    "rb_record_contacts": (C.c_int, [_P, C.c_int]),
    "rb_get_contacts": (C.c_int, [_P, _P, _P, _P, _P, _I64, C.POINTER(_I64)]),
    "rb_kat_impulse": (C.c_int, [_I32, _I32, _I64, _P, _P]),
    "rb_kat_inertia": (C.c_int, [_I32, _I32, _I64, _P, _P]),
    "rb_kat_apply": (C.c_int, [_I32, _I32, _I64, _P, _P]),
    "rb_kat_pair_impulse": (C.c_int, [_I32, _I32, _I64, _P, _P]),
    "rb_kat_narrow": (C.c_int, [_I32, _I32, _I64, _P, _P]),
    "rb_set_contact_law": (C.c_int, [_P, _I32, _D]),
    "rb_query": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64)]),
    "rb_kernel_timing": (C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(_I64)]),
    "rb_tile_config": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_double, _I64]),
    "rb_world_stats": (C.c_int, [_P, C.POINTER(_I64), _I32]),
}

# rb_world_stats indices (include/rbhip.h RB_STAT_*)
STAT_NAMES = ["graphs", "form", "box_opt_chunks", "box_rollbacks", "refits", "table_grows", "buckets",
              "max_partners", "io_skipped", "io_uploads", "tile_runs", "tile_steps", "tile_rollbacks",
              "tile_builds", "tile_why", "tile_slots", "tile_cols", "tile_on", "hashed_form"]
FORM_NAMES = {0: "rb::step_kernel_one", 1: "rb::step_kernel_coop", 2: "rb::step_kernel_wide",
              3: "rb::step_kernel_coop_help", 4: "rb::step_kernel_wide_help", 5: "rb::tile_step_kernel"}

_lib = None


def load(path: str = LIB_PATH):
    """Load librbhip.so (raises if absent: the product path has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"librbhip.so not built at {path}: run __graft_entry__.build() "
                           "(the HIP path has no CPU fallback)")
    # One HIP runtime per process: torch wheels bundle their own libamdhip64 /
    # libhsa-runtime64 (same sonames as /opt/rocm's).  Loaded first, torch's
    # copies also serve this library; loaded after ours, torch would bring a
    # second HSA runtime that finds no GPU (torch.cuda.is_available() False,
    # measured on MI355X), breaking torch interop (rbhip.shard buffers).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int, where: str):
    if rc != RB_OK:
        msg = _lib.rb_last_error().decode() if _lib is not None else ""
        raise RbError(rc, where, msg)


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)
