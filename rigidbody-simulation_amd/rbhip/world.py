"""World: a scene resident on one MI355X, stepped by librbhip.so.

Host side of the drop-in boundary.  It replaces the MuJoCo model/data pair
the reference step functions mutate (collision.py:56, time_integeration.py:13,
multi_sphere_bounce.py:42) with explicit arrays; the state crosses the
boundary in the reference's own layout (qpos stride 7, qvel stride 6).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from .scenes import Scene

COMM_ID_BYTES = 128      # ncclUniqueId (rccl.h NCCL_UNIQUE_ID_BYTES)


class World:
    def __init__(self, scene: Scene, device: int = 0, dtype: str = "f64", rank: int = 0,
                 world_size: int = 1, max_partners: int = 16, bucket_capacity: int = 0,
                 normal_convention: Optional[str] = None, law: str = "mujoco", tol: float = 0.01):
        """law: "mujoco" — the per-body Gauss-Seidel law of collision.py /
        multi_sphere_bounce.py; "balls" — the two-ball law of
        ball_collision.py:73-125 (tol: its contact tolerance, :102)."""
        L = _lib.load()
        self.scene = scene
        self.dtype = dtype
        self.rank, self.world_size = rank, world_size
        nc = normal_convention or scene.normal_convention
        self._kind = np.ascontiguousarray(scene.kind, np.int32)
        self._mass = np.ascontiguousarray(scene.mass, np.float64)
        self._inertia = np.ascontiguousarray(scene.inertia, np.float64)
        self._size = np.ascontiguousarray(scene.size, np.float64)
        self._planes = np.ascontiguousarray(scene.planes, np.float64)
        d = _lib.SceneDesc()
        d.n_bodies = scene.n
        d.n_planes = self._planes.shape[0]
        d.dtype = _lib.RB_F64 if dtype == "f64" else _lib.RB_F32
        d.normal_convention = _lib.RB_NORMAL_RAW if nc == "raw" else _lib.RB_NORMAL_ORIENTED
        d.device, d.rank, d.world_size = device, rank, world_size
        d.max_partners, d.bucket_capacity = max_partners, bucket_capacity
        d.kind, d.mass = _lib.ptr(self._kind), _lib.ptr(self._mass)
        d.inertia, d.size = _lib.ptr(self._inertia), _lib.ptr(self._size)
        d.planes = _lib.ptr(self._planes) if d.n_planes else None
        for k in range(3):
            d.gravity[k] = float(scene.gravity[k])
        h = C.c_void_p()
        _lib.check(L.rb_world_create(C.byref(h), C.byref(d)), "rb_world_create")
        self._h = h
        self._L = L
        # records per body (rb_world_create): 4 per plane, 1 per sphere
        # partner, up to 4 per partner in scenes with boxes; max_partners can
        # grow in a guarded chunk (16 -> 32), so contacts() recomputes it
        self._n_planes = d.n_planes
        self._any_box = bool(np.any(self._kind != 0))
        self.maxrec = self._maxrec(max_partners)
        n_owned, bpb = C.c_int64(), C.c_int64()
        _lib.check(L.rb_query(h, C.byref(n_owned), C.byref(bpb)), "rb_query")
        self.n_owned = n_owned.value
        self.bytes_per_body_step = bpb.value
        S = -(-scene.n // world_size)
        self.lo = S * rank
        self.hi = min(self.lo + S, scene.n)
        self.law = "mujoco"
        if law != "mujoco":
            self.set_contact_law(law, tol)
        self.set_state(scene.qpos0, scene.qvel0)

    def _maxrec(self, max_partners: int) -> int:
        return 4 * self._n_planes + (4 if self._any_box else 1) * max_partners

    def set_contact_law(self, law: str, tol: float = 0.01):
        """Switch between the default law and the two-ball law (rb_set_contact_law)."""
        code = {"mujoco": _lib.RB_LAW_MUJOCO, "balls": _lib.RB_LAW_BALLS}[law]
        _lib.check(self._L.rb_set_contact_law(self._h, code, float(tol)), "rb_set_contact_law")
        self.law, self.tol = law, float(tol)

    # ---- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.rb_world_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- state --------------------------------------------------------------
    def set_state(self, qpos, qvel):
        q = np.ascontiguousarray(qpos, np.float64).reshape(self.scene.n, 7)
        v = np.ascontiguousarray(qvel, np.float64).reshape(self.scene.n, 6)
        _lib.check(self._L.rb_set_state(self._h, _lib.ptr(q), _lib.ptr(v)), "rb_set_state")

    def get_state(self, qpos=None, qvel=None):
        """Returns global (N,7)/(N,6) arrays; only this shard's rows are filled."""
        q = np.zeros((self.scene.n, 7)) if qpos is None else qpos
        v = np.zeros((self.scene.n, 6)) if qvel is None else qvel
        _lib.check(self._L.rb_get_state(self._h, _lib.ptr(q), _lib.ptr(v)), "rb_get_state")
        return q, v

    def set_xfrc(self, xfrc):
        x = None if xfrc is None else np.ascontiguousarray(xfrc, np.float64).reshape(self.scene.n, 6)
        _lib.check(self._L.rb_set_xfrc(self._h, _lib.ptr(x)), "rb_set_xfrc")

    def set_stream(self, stream_handle: int):
        """Enqueue all later work on this hipStream_t (0 = HIP's null stream,
        which is torch's default stream)."""
        _lib.check(self._L.rb_set_stream(self._h, C.c_void_p(stream_handle or None)), "rb_set_stream")

    # ---- stepping -----------------------------------------------------------
    def _params(self, dt, restitution, friction, threshold):
        sc = self.scene
        return (sc.dt if dt is None else dt, sc.restitution if restitution is None else restitution,
                sc.friction if friction is None else friction,
                sc.threshold if threshold is None else threshold)

    def step(self, nsteps: int = 1, dt=None, restitution=None, friction=None, threshold=None):
        p = self._params(dt, restitution, friction, threshold)
        _lib.check(self._L.rb_step(self._h, int(nsteps), *p), "rb_step")

    def step_async(self, nsteps: int = 1, dt=None, restitution=None, friction=None, threshold=None):
        p = self._params(dt, restitution, friction, threshold)
        _lib.check(self._L.rb_step_async(self._h, int(nsteps), *p), "rb_step_async")

    def sync(self):
        _lib.check(self._L.rb_sync(self._h), "rb_sync")

    # ---- sharded stepping ---------------------------------------------------
    def shard_step(self, dt=None, restitution=None, friction=None, threshold=None):
        p = self._params(dt, restitution, friction, threshold)
        _lib.check(self._L.rb_shard_step(self._h, *p), "rb_shard_step")

    def shard_exchange_done(self):
        _lib.check(self._L.rb_shard_exchange_done(self._h), "rb_shard_exchange_done")

    def gpos_buffer(self):
        """(device pointer, elements per shard, bytes per element) of the
        replicated [P][S][4] position buffer."""
        p, n, b = C.c_void_p(), C.c_int64(), C.c_int32()
        _lib.check(self._L.rb_gpos_buffer(self._h, C.byref(p), C.byref(n), C.byref(b)), "rb_gpos_buffer")
        return p.value, n.value, b.value

    def gquat_buffer(self):
        """(device pointer, elements per shard, bytes per element) of the
        replicated [P][S][4] orientation buffer the same exchange fills in
        box worlds; (None, 0, esz) for sphere-only worlds."""
        p, n, b = C.c_void_p(), C.c_int64(), C.c_int32()
        _lib.check(self._L.rb_gquat_buffer(self._h, C.byref(p), C.byref(n), C.byref(b)), "rb_gquat_buffer")
        return p.value, n.value, b.value

    # ---- in-library exchange (RCCL communicator owned by the world) ---------
    @staticmethod
    def comm_unique_id() -> bytes:
        """A new communicator id (rank 0 makes it, every rank joins with it)."""
        L = _lib.load()
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _lib.check(L.rb_comm_unique_id(buf, COMM_ID_BYTES), "rb_comm_unique_id")
        return buf.raw

    def shard_comm_init(self, uid: bytes):
        """Join the world's ranks in one RCCL communicator (blocks until all have)."""
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"communicator id must be {COMM_ID_BYTES} bytes")
        _lib.check(self._L.rb_shard_comm_init(self._h, C.c_char_p(uid), COMM_ID_BYTES), "rb_shard_comm_init")

    def p2p_handles(self) -> bytes:
        """This rank's IPC handles for the peer-to-peer exchange."""
        n = C.c_int64()
        _lib.check(self._L.rb_p2p_handles(self._h, None, 0, C.byref(n)), "rb_p2p_handles")
        buf = C.create_string_buffer(n.value)
        _lib.check(self._L.rb_p2p_handles(self._h, buf, n.value, C.byref(n)), "rb_p2p_handles")
        return buf.raw

    def p2p_connect(self, all_handles: bytes):
        """Map every peer's buffers (all ranks' handles concatenated in rank
        order); collective: no rank may step before all have connected."""
        _lib.check(self._L.rb_p2p_connect(self._h, C.c_char_p(all_handles), len(all_handles)), "rb_p2p_connect")

    def p2p_halo(self, enable: bool = True):
        """Halo mode of the peer-to-peer exchange (push only the bodies a peer
        can reach); collective, after p2p_connect."""
        _lib.check(self._L.rb_p2p_halo(self._h, 1 if enable else 0), "rb_p2p_halo")

    def shard_run(self, nsteps: int = 1, dt=None, restitution=None, friction=None, threshold=None):
        """nsteps sharded steps with the in-library exchange (enqueued only)."""
        p = self._params(dt, restitution, friction, threshold)
        _lib.check(self._L.rb_shard_run(self._h, int(nsteps), *p), "rb_shard_run")

    # ---- parity support -----------------------------------------------------
    def record_contacts(self, enable: bool = True):
        _lib.check(self._L.rb_record_contacts(self._h, int(bool(enable))), "rb_record_contacts")

    def contacts(self):
        """Contact list of the most recent step, CSR over owned bodies:
        (counts, partner, kind, dist)."""
        n = self.n_owned
        self.maxrec = self._maxrec(self.stats()["max_partners"])   # (the library may have grown it)
        cap = max(1, n * self.maxrec)
        cnt = np.zeros(n, np.int32)
        par = np.zeros(cap, np.int32)
        kin = np.zeros(cap, np.int32)
        dis = np.zeros(cap)
        tot = C.c_int64()
        _lib.check(self._L.rb_get_contacts(self._h, _lib.ptr(cnt), _lib.ptr(par), _lib.ptr(kin),
                                           _lib.ptr(dis), cap, C.byref(tot)), "rb_get_contacts")
        t = tot.value
        return cnt, par[:t], kin[:t], dis[:t]

    def stats(self) -> dict:
        """Counters of the world (rb_world_stats, include/rbhip.h RB_STAT_*):
        the step kernel form, tile-form runs and roll-backs, refits, ..."""
        n = len(_lib.STAT_NAMES)
        buf = (C.c_int64 * n)()
        rc = self._L.rb_world_stats(self._h, buf, n)
        if rc < 0:
            _lib.check(rc, "rb_world_stats")
        return {k: int(buf[i]) for i, k in enumerate(_lib.STAT_NAMES[:rc])}

    def kernel_timing(self, enable: bool):
        """Toggle per-launch HIP-event timing of the step kernel; returns the
        (average ms, launches) collected since it was last enabled."""
        avg, n = C.c_double(), C.c_int64()
        _lib.check(self._L.rb_kernel_timing(self._h, int(bool(enable)), C.byref(avg), C.byref(n)),
                   "rb_kernel_timing")
        return avg.value, n.value


def kat_impulse(inp: np.ndarray, dtype: str = "f64", device: int = 0) -> np.ndarray:
    """Device known-answer entry: a1 (collision.py:7-48) then a2
    (physics_utils.py:25-49) per row of inp[:, 24] -> out[:, 10]."""
    L = _lib.load()
    inp = np.ascontiguousarray(inp, np.float64).reshape(-1, 24)
    out = np.zeros((inp.shape[0], 10))
    _lib.check(L.rb_kat_impulse(device, _lib.RB_F64 if dtype == "f64" else _lib.RB_F32, inp.shape[0],
                                _lib.ptr(inp), _lib.ptr(out)), "rb_kat_impulse")
    return out


def kat_inertia(inp: np.ndarray, dtype: str = "f64", device: int = 0) -> np.ndarray:
    """Device known-answer entry: compute_inertia_tensor_world (collision.py:51-53)
    and its inverse per row of inp[:, 7] -> out[:, 18]."""
    L = _lib.load()
    inp = np.ascontiguousarray(inp, np.float64).reshape(-1, 7)
    out = np.zeros((inp.shape[0], 18))
    _lib.check(L.rb_kat_inertia(device, _lib.RB_F64 if dtype == "f64" else _lib.RB_F32, inp.shape[0],
                                _lib.ptr(inp), _lib.ptr(out)), "rb_kat_inertia")
    return out


def kat_apply(inp: np.ndarray, dtype: str = "f64", device: int = 0) -> np.ndarray:
    """Device entry for apply_impulse_friction (physics_utils.py:25-49) with
    given impulses, per row of inp[:, 26] -> out[:, 6] = v', w'."""
    L = _lib.load()
    inp = np.ascontiguousarray(inp, np.float64).reshape(-1, 26)
    out = np.zeros((inp.shape[0], 6))
    _lib.check(L.rb_kat_apply(device, _lib.RB_F64 if dtype == "f64" else _lib.RB_F32, inp.shape[0],
                              _lib.ptr(inp), _lib.ptr(out)), "rb_kat_apply")
    return out


def kat_pair_impulse(inp: np.ndarray, dtype: str = "f64", device: int = 0) -> np.ndarray:
    """Device known-answer entry: compute_collision_impulse (ball_collision.py:53-68)
    per row of inp[:, 27] = m, e, mu, v, w, r, n, I_inv(9) -> out[:, 3]."""
    L = _lib.load()
    inp = np.ascontiguousarray(inp, np.float64).reshape(-1, 27)
    out = np.zeros((inp.shape[0], 3))
    _lib.check(L.rb_kat_pair_impulse(device, _lib.RB_F64 if dtype == "f64" else _lib.RB_F32, inp.shape[0],
                                     _lib.ptr(inp), _lib.ptr(out)), "rb_kat_pair_impulse")
    return out


def kat_narrow(inp: np.ndarray, dtype: str = "f64", device: int = 0) -> np.ndarray:
    """Device entry for the box-involved narrowphase (rb_boxes.hpp; SURVEY
    §8f row 4) per row of inp[:, 22] = kind1, kind2, c1, q1, s1, c2, q2, s2
    -> out[:, 33] = count, then per contact dist, pos[3], frame[3], kind."""
    L = _lib.load()
    inp = np.ascontiguousarray(inp, np.float64).reshape(-1, 22)
    out = np.zeros((inp.shape[0], 33))
    _lib.check(L.rb_kat_narrow(device, _lib.RB_F64 if dtype == "f64" else _lib.RB_F32, inp.shape[0],
                               _lib.ptr(inp), _lib.ptr(out)), "rb_kat_narrow")
    return out
