"""Body-range sharding of one scene over the GPUs of a node.

Rank r owns bodies [r*S, r*S + S), S = ceil(N / P).  The exchange buffer
holds (x, y, z, bounding radius) per body in global id order ([P][S][4]);
two such buffers alternate step by step inside the library.  Worlds with box
bodies exchange a second [P][S][4] buffer, the orientations (w, x, y, z):
a box's contacts depend on its orientation (rb_gquat_buffer).  Each step is Jacobi
across bodies (multi_sphere_bounce.py:43-46: one contact pass, then every
body updated from step-start data), and the reference treats a contact
partner as static (collision.py:27), so a rank needs only the step-start
POSITIONS of other ranks' bodies.  Per step:

    step kernel             owned bodies: contacts + impulses + integrate;
                            new positions land in this rank's slice of the
                            replicated [P][S][4] position buffer
    all-gather              RCCL over xGMI, in place on that buffer
    remote insert           publish the other ranks' positions to the
                            broadphase of the next step

Transports:
    "p2p"    (default on an nccl process group) every rank reads the other
             ranks' fresh slices straight from their buffers over xGMI (IPC
             mappings, handles exchanged once through torch.distributed),
             signalled by device flags: rb_shard_run replays K steps from
             one captured HIP graph (SURVEY §7 hard part 4).  For large
             shards (halo="auto": >= HALO_MIN_SHARD bodies per rank) the
             halo mode instead pushes to each peer only the bodies within
             one cell of the peer's own bodies' cell bounds;
    "rccl"   the library owns an RCCL
             communicator (id broadcast once through torch.distributed) and
             runs all three per step itself: rb_shard_run replays K steps
             from one captured HIP graph, no host work per step;
    "nccl"   rb_shard_step, torch.distributed.all_gather_into_tensor on the
             library's buffer and stream, rb_shard_exchange_done (three host
             calls per step);
    "host"   the same through host memory, for gloo groups (several ranks
             sharing one GPU in tests).

Contacts are generated from identical global positions with global body
ids in a canonical order, so fp64 results are bit-identical for any P.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional

import numpy as np

from ._lib import RbError
from .scenes import Scene
from .world import World

# shard size from which the peer-to-peer exchange pushes halos instead of
# reading whole slices: a halo step costs two kernels and two one-way flag
# latencies, a full read (P-1) x S x 32 B over xGMI (~28 us for 65,536 fp64
# bodies from 7 peers at ~75 GB/s per link)
HALO_MIN_SHARD = 16384


class _DeviceBuffer:
    """__cuda_array_interface__ view of library-owned device memory, so torch
    can wrap it without a copy (torch.as_tensor consumes the interface)."""

    def __init__(self, ptr: int, n: int, esz: int):
        self.__cuda_array_interface__ = {
            "shape": (n,), "typestr": "<f8" if esz == 8 else "<f4", "data": (ptr, False),
            "version": 2, "strides": None, "stream": None}


def _wrap(world: World, torch, which: str):
    ptr, shard_elems, esz = getattr(world, which)()
    if not ptr:
        return None, 0
    total = shard_elems * world.world_size
    t = torch.as_tensor(_DeviceBuffer(ptr, total, esz), device=f"cuda:{torch.cuda.current_device()}")
    return t, shard_elems


def wrap_gpos(world: World, torch):
    """Torch view of the buffer the pending exchange fills (call between
    shard_step and shard_exchange_done)."""
    return _wrap(world, torch, "gpos_buffer")


def wrap_gquat(world: World, torch):
    """Torch view of the orientation buffer the pending exchange fills in
    box worlds (None, 0 in sphere-only worlds)."""
    return _wrap(world, torch, "gquat_buffer")


class ShardedWorld:
    """One rank's shard of a scene; `step` runs the exchange each step.

    transport: "p2p" (peer-to-peer reads over IPC mappings, graph-replayed;
    the default when the process group backend is nccl), "rccl" (in-library
    RCCL all-gather, graph-replayed), "nccl" (torch.distributed all-gather
    per step) or "host" (stage through host memory, for gloo process groups,
    e.g. several ranks sharing one GPU in tests).

    `world_factory(rank, world_size)` may supply the per-rank stepper (any
    object with the World shard interface and an `exchange_buffer(torch)`
    method returning (tensor, shard_elems)); by default it is a HIP World on
    `device`."""

    def __init__(self, scene: Scene, dtype: str = "f64", device: Optional[int] = None,
                 group=None, transport: Optional[str] = None, world_factory=None, halo="auto",
                 **world_kw):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.P = dist.get_world_size(group)
            backend = dist.get_backend(group)
        else:
            self.rank, self.P, backend = 0, 1, None
        self.transport = (transport or os.environ.get("RBHIP_SHARD_TRANSPORT") or
                          ("p2p" if backend == "nccl" and world_factory is None else
                           "nccl" if backend == "nccl" else "host"))
        self._views = {}
        if world_factory is not None:
            self.world = world_factory(self.rank, self.P)
        else:
            if device is None:
                device = torch.cuda.current_device()
            torch.cuda.set_device(device)
            self.world = World(scene, device=device, dtype=dtype, rank=self.rank, world_size=self.P,
                               **world_kw)
            self.stream = torch.cuda.current_stream(device)
            self.world.set_stream(self.stream.cuda_stream)
        self.halo = False
        if self.transport == "p2p":
            self._connect_p2p()
        if self.transport == "p2p":
            env = os.environ.get("RBHIP_P2P_HALO")
            h = {"1": True, "0": False}.get(env, halo) if env else halo
            if h == "auto":
                h = -(-scene.n // self.P) >= HALO_MIN_SHARD
            if h:
                self.world.p2p_halo(True)
                self.halo = True
        if self.transport == "rccl":
            # rank 0 of the group makes the communicator id, every rank joins;
            # without RCCL in this process every rank takes the torch path
            uid = [None]
            if self.rank == 0:
                try:
                    uid[0] = World.comm_unique_id()
                except RbError as e:
                    warnings.warn(f"in-library RCCL exchange unavailable ({e}); using torch.distributed")
            if self.P > 1:
                src = dist.get_global_rank(group, 0) if group is not None else 0
                dist.broadcast_object_list(uid, src=src, group=group)
            if uid[0] is None:
                self.transport = "nccl"
            else:
                self.world.shard_comm_init(uid[0])

    def _connect_p2p(self):
        """Exchange IPC handles once and map every peer's buffers; on any
        failure (on every rank alike) fall back to the RCCL transport."""
        dist, torch = self.dist, self.torch
        try:
            mine = self.world.p2p_handles()
        except RbError as e:
            mine = None
            warnings.warn(f"peer-to-peer exchange unavailable ({e})")
        blobs = [mine]
        if self.P > 1:
            blobs = [None] * self.P
            dist.all_gather_object(blobs, mine, group=self.group)
        ok = all(b is not None for b in blobs)
        connected = False
        if ok:
            try:
                self.world.p2p_connect(b"".join(blobs))
                connected = True
            except RbError as e:
                ok = False
                warnings.warn(f"peer-to-peer exchange unavailable ({e})")
        if self.P > 1:
            dev = f"cuda:{torch.cuda.current_device()}" if dist.get_backend(self.group) == "nccl" else "cpu"
            t = torch.tensor([1 if ok else 0], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            ok = bool(t.item())
        if not ok:
            if connected:
                raise RuntimeError("peer-to-peer exchange connected on some ranks only")
            self.transport = "rccl"
        if self.P > 1:
            dist.barrier(group=self.group)   # every rank connected before any steps

    def _buffers(self):
        """[(whole buffer, this rank's slice)] of the pending exchange: the
        positions, and in box worlds the orientations; the alternating
        buffers' views are built once."""
        if hasattr(self.world, "exchange_buffer"):
            buf, n = self.world.exchange_buffer(self.torch)
            return [(buf, buf[self.rank * n:(self.rank + 1) * n])]
        out = []
        for which, wrap in (("gpos_buffer", wrap_gpos), ("gquat_buffer", wrap_gquat)):
            ptr = getattr(self.world, which)()[0]
            if not ptr:
                continue
            v = self._views.get(ptr)
            if v is None:
                buf, n = wrap(self.world, self.torch)
                v = self._views[ptr] = (buf, buf[self.rank * n:(self.rank + 1) * n])
            out.append(v)
        return out

    def _exchange(self):
        for buf, mine in self._buffers():
            n = mine.numel()
            if self.transport == "nccl":
                # in place: the input is this rank's chunk of the output buffer
                self.dist.all_gather_into_tensor(buf, mine, group=self.group)
            else:
                cpu = mine.to("cpu")
                out = self.torch.empty(self.P * n, dtype=cpu.dtype)
                self.dist.all_gather_into_tensor(out, cpu, group=self.group)
                buf.copy_(out.to(buf.device))

    def step(self, nsteps: int = 1, **params):
        if self.transport in ("p2p", "rccl"):
            self.world.shard_run(nsteps, **params)
            return
        if self.P == 1:
            self.world.step_async(nsteps, **params)
            return
        for _ in range(nsteps):
            self.world.shard_step(**params)
            self._exchange()
            self.world.shard_exchange_done()

    def sync(self):
        self.world.sync()

    def gather_state(self):
        """Full (qpos, qvel) on every rank (host all-gather of owned rows)."""
        q, v = self.world.get_state()
        if self.P == 1:
            return q, v
        # each rank contributes its own rows [r*S, r*S + S) (padded to S):
        # an all-gather moves the words unchanged (a sum would turn -0.0
        # into +0.0), so the result is bit-identical to one World's state
        n = q.shape[0]
        S = -(-n // self.P)
        lo, hi = min(self.rank * S, n), min(self.rank * S + S, n)
        mine = np.zeros((S, 13))
        mine[:hi - lo, :7], mine[:hi - lo, 7:] = q[lo:hi], v[lo:hi]
        t = self.torch.from_numpy(mine)
        if self.dist.get_backend(self.group) == "nccl":
            t = t.to(f"cuda:{self.torch.cuda.current_device()}")
        parts = [self.torch.empty_like(t) for _ in range(self.P)]
        self.dist.all_gather(parts, t, group=self.group)
        a = self.torch.cat(parts).cpu().numpy()[:n]
        return a[:, :7].copy(), a[:, 7:].copy()
