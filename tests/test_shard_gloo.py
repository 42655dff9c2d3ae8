"""Body-range sharding over torch.distributed (gloo, world_size 2 and 3) on
CPU: the real ShardedWorld exchange logic (the library's [P][S][4] snapshot
layout — x, y, z, bounding radius per body in global id order — in-rank
slice, all-gather, publish), with the per-rank stepper emulated by the
oracle (test-only stand-in for librbhip's rb_shard_step /
rb_shard_exchange_done).  Result must be bit-identical to one rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


class OracleShardStepper:
    """Emulates one rank of the library's sharded world on the CPU: it keeps
    the full AoS state, steps it with the oracle, keeps only its own rows,
    and takes other ranks' positions from the replicated buffer."""

    def __init__(self, scene, rank, P):
        from oracle import oracle as O
        self.O, self.sc, self.rank, self.P = O, scene, rank, P
        self.osc = O.OracleScene(scene)
        self.S = -(-scene.n // P)
        self.lo, self.hi = rank * self.S, min(rank * self.S + self.S, scene.n)
        self.q = scene.qpos0.copy()
        self.v = scene.qvel0.copy()
        # rb_internal.hpp Snap<T>{x, y, z, r}, [P][S][4] (rb_gpos_buffer)
        self.buf = torch.zeros(P * self.S * 4, dtype=torch.float64)
        g = self.buf.view(P, self.S, 4)
        for b in range(scene.n):
            g[b // self.S, b % self.S, 0:3] = torch.from_numpy(self.q[b, 0:3])
            g[b // self.S, b % self.S, 3] = float(scene.size[b, 0])

    def exchange_buffer(self, torch_mod):
        return self.buf, 4 * self.S

    def shard_step(self, **params):
        q, v = self.O.step(self.osc, self.q, self.v, 1)
        self.q[self.lo:self.hi], self.v[self.lo:self.hi] = q[self.lo:self.hi], v[self.lo:self.hi]
        g = self.buf.view(self.P, self.S, 4)
        g[self.rank, : self.hi - self.lo, 0:3] = torch.from_numpy(self.q[self.lo:self.hi, 0:3].copy())

    def shard_exchange_done(self):
        g = self.buf.view(self.P, self.S, 4).numpy()
        for b in range(self.sc.n):
            if not (self.lo <= b < self.hi):
                self.q[b, 0:3] = g[b // self.S, b % self.S, 0:3]

    def sync(self):
        pass

    def get_state(self):
        q = np.zeros_like(self.q)
        v = np.zeros_like(self.v)
        q[self.lo:self.hi], v[self.lo:self.hi] = self.q[self.lo:self.hi], self.v[self.lo:self.hi]
        return q, v


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, P, port, steps, out):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    from rbhip import scenes
    from rbhip.shard import ShardedWorld
    sc = scenes.flat_spheres(9, 7, seed=3)             # N = 63: not a multiple of 2
    sw = ShardedWorld(sc, world_factory=lambda r, p: OracleShardStepper(sc, r, p))
    assert sw.transport == "host" and sw.P == P
    sw.step(steps)
    q, v = sw.gather_state()
    if rank == 0:
        np.save(out, np.concatenate([q, v], axis=1))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("P", [2, 3])
def test_sharded_exchange_is_p_invariant(tmp_path, oracle, P):
    from rbhip import scenes
    steps = 60
    sc = scenes.flat_spheres(9, 7, seed=3)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, steps)
    out = str(tmp_path / "state.npy")
    mp.start_processes(_worker, args=(P, _free_port(), steps, out), nprocs=P, start_method="spawn")
    got = np.load(out)
    # compared as 64-bit words: the gather must keep the sign of zeros
    assert np.array_equal(got[:, :7].view(np.uint64), q1.view(np.uint64))
    assert np.array_equal(got[:, 7:].view(np.uint64), v1.view(np.uint64))


def test_tiled_scene_ownership():
    """bench.py's weak-scaling world: rank r's contiguous id range is the r-th
    x-slab of the tiled ground."""
    from rbhip import scenes
    sc = scenes.tiled(scenes.flat_spheres, 4, 8, 6, seed=0)
    assert sc.n == 4 * 8 * 6
    S = sc.n // 4
    for r in range(4):
        xs = sc.qpos0[r * S:(r + 1) * S, 0]
        if r > 0:
            assert xs.min() > sc.qpos0[(r - 1) * S:r * S, 0].max()


def test_strong_scene_ownership():
    """bench.py's default (strong scaling): the one C3 scene split by body-id
    range; ids run row-major, so rank r's range is the r-th y-slab of
    256 / P grid rows."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from rbhip import scenes
    for P in (1, 2, 4, 8):
        sc, desc = bench.make_scene("c3", P, "strong")
        assert sc.n == 65536 and np.array_equal(sc.qpos0, scenes.make("c3").qpos0)
        S = -(-sc.n // P)
        for r in range(1, P):
            assert sc.qpos0[r * S:(r + 1) * S, 1].min() > sc.qpos0[(r - 1) * S:r * S, 1].max()
        assert ("strong" in desc) == (P > 1)
    sc, desc = bench.make_scene("c4", 8, "weak")
    assert sc.n == 8 * 65536 and "weak" in desc
