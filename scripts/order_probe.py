"""Diagnostic: how much does the body-id order (= the memory order of the
state and snapshots, and which bodies share a wave) cost the step kernel?
Runs C3-shaped flat scenes with the same bodies renumbered row-major (the
bench scene), in 8x8 tiles (a wave = an 8x8 patch), in Morton order and in a
random order, and prints ms/step (HIP events, graph-replayed steps after a
warm-up).  Renumbering changes the Gauss-Seidel contact order, so these are
different (equally valid) scenes: a measurement of layout, not the bench."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
from dataclasses import replace
import numpy as np
import torch
import rbhip
from rbhip import scenes


def permuted(sc, order):
    return replace(sc, kind=sc.kind[order], mass=sc.mass[order], inertia=sc.inertia[order], size=sc.size[order],
                   qpos0=sc.qpos0[order], qvel0=sc.qvel0[order])


def orders(nx, ny):
    n = nx * ny
    iy, ix = np.divmod(np.arange(n), nx)
    yield "row-major", np.arange(n)
    for t in (8, 16):
        yield f"tile{t}", np.lexsort((ix % t, iy % t, ix // t, iy // t))
    m = np.zeros(n, np.int64)
    for b in range(16):
        m |= ((ix >> b) & 1) << (2 * b) | ((iy >> b) & 1) << (2 * b + 1)
    yield "morton", np.argsort(m, kind="stable")
    yield "random", np.random.default_rng(1).permutation(n)


def time_scene(sc, warm, K):
    with rbhip.World(sc) as w:
        w.set_stream(torch.cuda.current_stream().cuda_stream)
        w.step(warm)
        w.step(K)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); w.step_async(K); e1.record(); w.sync()
        return e0.elapsed_time(e1) / K * 1e3


nx = int(os.environ.get("NX", "256")); ny = int(os.environ.get("NY", "256"))
warm = int(os.environ.get("WARM", "50")); K = int(os.environ.get("K", "400"))
base = scenes.flat_spheres(nx, ny, seed=0)
print(f"| order | N | us/step (steps {warm + K + 1}-{warm + 2 * K}) |")
print("|---|---|---|")
for name, o in orders(nx, ny):
    us = time_scene(permuted(base, o), warm, K)
    print(f"| {name} | {base.n} | {us:.2f} |", flush=True)
