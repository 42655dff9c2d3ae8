"""The exactness argument of the XCD-resident K-step blocks (csrc/rb_xblock.hip,
DESIGN §4.2), checked on the CPU with the oracle (no GPU).

A block copies each slab of the scene plus a ghost band of width
    W = K reach + 2 (K - 1) V dt
(reach = twice the largest radius, V bounds every body's speed over the K
steps), steps the copy K times on its own and keeps only the slab's bodies.
The reference step is Jacobi across bodies (multi_sphere_bounce.py:43 one
contact pass, :46-90 per-body updates from step-start data), so a body's
state after K steps depends only on bodies within W of it at the start.
Here the oracle steps the WHOLE scene K steps and, separately, every slab's
copy (the subset of bodies within the band, ids kept in ascending order, as
the kernel compacts them) K steps: the owned bodies must come out
bit-identical, and the speed bound must hold — the same check the kernel
makes.  Also: with no band at all (each slab stepped alone) owned bodies
near the cuts differ, as evidence that the band is what makes it exact."""
from dataclasses import replace

import numpy as np
import pytest

from rbhip import scenes

G = 8


def _sub(sc, ids):
    return replace(sc, name=sc.name + "_sub", kind=sc.kind[ids], mass=sc.mass[ids], inertia=sc.inertia[ids],
                   size=sc.size[ids], qpos0=sc.qpos0[ids], qvel0=sc.qvel0[ids], names=None)


def _block_check(oracle, sc, q, v, K, valpha=1.5, vbeta=0.5, shrink=0.0):
    """Step (q, v) K steps whole and slab by slab; returns (owned bodies
    differing, speed bound held)."""
    osc = oracle.OracleScene(sc)
    qk, vk = oracle.step(osc, q, v, K)
    reach = 2 * float(np.max(sc.size[:, 0]))
    vmax = float(np.linalg.norm(v[:, :3], axis=1).max())
    gdt = float(np.linalg.norm(sc.gravity)) * sc.dt
    V = valpha * vmax + vbeta + K * gdt
    W = K * reach + 2 * (K - 1) * V * sc.dt + 1e-3 * reach - shrink
    # the speed bound over the K steps (every body: the union of the groups' checks)
    held = True
    qs, vs = q, v
    for _ in range(K):
        qs, vs = oracle.step(osc, qs, vs, 1)
        held &= bool(np.linalg.norm(vs[:, :3], axis=1).max() <= V)
    ext = q[:, :2].max(0) - q[:, :2].min(0)
    axis = 1 if ext[1] > ext[0] else 0
    u = q[:, axis]
    cut = [-np.inf] + [0.5 * (np.sort(u)[len(u) * g // G - 1] + np.sort(u)[len(u) * g // G]) for g in range(1, G)] + [np.inf]
    bad = 0
    for g in range(G):
        own = (u >= cut[g]) & (u < cut[g + 1])
        lo, hi = (cut[g] - W if g else -np.inf), (cut[g + 1] + W if g < G - 1 else np.inf)
        ids = np.flatnonzero((u >= lo) & (u < hi))          # ascending: the kernel's compaction order
        sub = _sub(sc, ids)
        q1, v1 = oracle.step(oracle.OracleScene(sub), q[ids], v[ids], K)
        mine = own[ids]
        bad += int((~(np.all(q1[mine].view(np.uint64) == qk[ids[mine]].view(np.uint64), axis=1) &
                      np.all(v1[mine].view(np.uint64) == vk[ids[mine]].view(np.uint64), axis=1))).sum())
    return bad, held


@pytest.mark.parametrize("K", [2, 6])
def test_slab_copies_with_band_are_exact(oracle, K):
    """A C3-like scene (96 x 96 spheres, the bench's seeded generator) from
    step 25 (bodies landing, bouncing, colliding), blocks of K steps."""
    sc = scenes.flat_spheres(96, 96, seed=0)
    osc = oracle.OracleScene(sc)
    q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 25)
    bad, held = _block_check(oracle, sc, q, v, K)
    assert held, "the speed bound failed (the kernel would roll the chunk back)"
    assert bad == 0, f"{bad} owned bodies differ from the whole-scene run"


def test_band_matters(oracle):
    """Without the band (W = 0: each slab stepped alone) owned bodies near
    the slab edges come out wrong — the band is what makes the blocks exact."""
    sc = scenes.flat_spheres(96, 96, seed=0)
    osc = oracle.OracleScene(sc)
    q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 60)
    K = 6
    reach = 2 * float(np.max(sc.size[:, 0]))
    vmax = float(np.linalg.norm(v[:, :3], axis=1).max())
    V = 1.5 * vmax + 0.5 + K * float(np.linalg.norm(sc.gravity)) * sc.dt
    W = K * reach + 2 * (K - 1) * V * sc.dt + 1e-3 * reach
    bad, _ = _block_check(oracle, sc, q, v, K, shrink=W)
    assert bad > 0


def test_sharded_copies_with_pushed_ghosts_are_exact(oracle):
    """The sharded blocks' argument (rb_p2p.hip xs_push_kernel):
    rank r owns ids [rS, rS + S); a peer pushes every body within W of r's
    bounding box (x and y) — the ghosts; each of r's 8 groups copies its
    slab of r's bodies plus every own body or ghost within W along the slab
    axis.  Stepped K steps by the oracle, every rank's owned bodies match
    the whole scene bit for bit (C3-like scene in 4 row slabs of 96 x 24)."""
    sc = scenes.flat_spheres(96, 96, seed=0)
    osc = oracle.OracleScene(sc)
    q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 25)
    K, P = 6, 4
    qk, vk = oracle.step(osc, q, v, K)
    n = sc.n
    S = -(-n // P)
    reach = 2 * float(np.max(sc.size[:, 0]))
    vmax = float(np.linalg.norm(v[:, :3], axis=1).max())
    V = 1.5 * vmax + 0.5 + K * float(np.linalg.norm(sc.gravity)) * sc.dt
    W = K * reach + 2 * (K - 1) * V * sc.dt + 1e-3 * reach
    bad = 0
    for r in range(P):
        own = np.arange(r * S, min(n, r * S + S))
        lo, hi = q[own, :2].min(0), q[own, :2].max(0)
        others = np.setdiff1d(np.arange(n), own)
        near = np.all((q[others, :2] >= lo - W) & (q[others, :2] <= hi + W), axis=1)
        ghosts = others[near]
        ext = hi - lo
        axis = 1 if ext[1] > ext[0] else 0
        u = np.sort(q[own, axis])
        cut = [-np.inf] + [0.5 * (u[len(u) * g // G - 1] + u[len(u) * g // G]) for g in range(1, G)] + [np.inf]
        pool = np.union1d(own, ghosts)
        for g in range(G):
            a, b = (cut[g] - W if g else -np.inf), (cut[g + 1] + W if g < G - 1 else np.inf)
            ids = pool[(q[pool, axis] >= a) & (q[pool, axis] < b)]
            mine = np.isin(ids, own) & (q[ids, axis] >= cut[g]) & (q[ids, axis] < cut[g + 1])
            q1, v1 = oracle.step(oracle.OracleScene(_sub(sc, ids)), q[ids], v[ids], K)
            bad += int((~(np.all(q1[mine].view(np.uint64) == qk[ids[mine]].view(np.uint64), axis=1) &
                          np.all(v1[mine].view(np.uint64) == vk[ids[mine]].view(np.uint64), axis=1))).sum())
    assert bad == 0
