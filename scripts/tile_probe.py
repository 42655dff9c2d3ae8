"""CPU probe for the K-step tile design: how far bodies move per
step in the bench window, and how deep the ghost band must be.

For block starts in the bench window it reports, per K:
  * the largest 3-D displacement of any body over the block (the skin S the
    block's neighbour lists need);
  * per tile (T x T m columns, band W): loaded bodies / owned bodies and the
    smallest hop count of an owned body from the band's outer layer over the
    neighbour-list graph (pairs within reach + 2S at the block start) —
    the block is exact for K steps when that count is >= K.

    python scripts/tile_probe.py --config c3 --start 450 --steps 64
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))

from oracle import oracle as O  # noqa: E402
from rbhip import scenes  # noqa: E402


def hops(pos, edges_i, edges_j, n, src_mask, kmax):
    h = np.where(src_mask, 0, kmax + 1).astype(np.int32)
    for _ in range(kmax):
        m = np.minimum(h[edges_i], h[edges_j])
        nh = h.copy()
        np.minimum.at(nh, edges_i, h[edges_j] + 1)
        np.minimum.at(nh, edges_j, h[edges_i] + 1)
        if np.array_equal(nh, h):
            break
        h = nh
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--start", type=int, default=450)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--tile", type=float, nargs="+", default=[4.8])
    ap.add_argument("--band", type=float, nargs="+", default=[0.6, 0.9, 1.2])
    ap.add_argument("--k", type=int, nargs="+", default=[4, 8, 16])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    sc = scenes.make(a.config)
    osc = O.OracleScene(sc)
    O.set_threads(a.threads)
    q, v = sc.qpos0.copy(), sc.qvel0.copy()
    if a.start:
        q, v = O.step(osc, q, v, a.start)
    traj = [q[:, :3].copy()]
    vel = [v.copy()]
    for _ in range(a.steps):
        q, v = O.step(osc, q, v, 1)
        traj.append(q[:, :3].copy())
        vel.append(v.copy())
    traj = np.array(traj)
    reach = 2 * float(sc.size[:, 0].max())
    spd = np.linalg.norm(np.array(vel)[:, :, :3], axis=2)
    print(f"{a.config}: steps {a.start}..{a.start + a.steps}; reach {reach}; max |v| {spd.max():.3f} m/s "
          f"(p99.9 {np.quantile(spd, 0.999):.3f}); max step disp {np.linalg.norm(np.diff(traj, axis=0), axis=2).max():.4f} m")
    for K in a.k:
        for b0 in range(0, a.steps - K + 1, max(K, a.steps // 4)):
            x0 = traj[b0]
            # per-body, per-axis displacement bounds over the block (the real
            # kernel predicts them from the velocity and checks them after)
            Sa = np.abs(traj[b0:b0 + K + 1] - x0[None]).max(axis=0) * 1.1 + 1e-4   # [N,3]
            Smax = Sa.max(axis=0)
            tree = cKDTree(x0)
            pairs = tree.query_pairs(reach + 2 * np.linalg.norm(Smax), output_type="ndarray")
            dd = np.abs(x0[pairs[:, 0]] - x0[pairs[:, 1]])
            keep = np.all(dd < reach + Sa[pairs[:, 0]] + Sa[pairs[:, 1]], axis=1)
            keep &= np.linalg.norm(dd, axis=1) < reach + np.linalg.norm(Sa[pairs[:, 0]], axis=1) + np.linalg.norm(Sa[pairs[:, 1]], axis=1)
            pairs = pairs[keep]
            deg = np.bincount(pairs.ravel(), minlength=sc.n)
            for T in a.tile:
                for W in a.band:
                    lo = x0[:, :2].min(0)
                    tix = np.floor((x0[:, :2] - lo) / T).astype(int)
                    ntx, nty = tix.max(0) + 1
                    worst, rho_l, rho_o, maxload = 10 ** 9, 0, 0, 0
                    for tx in range(ntx):
                        for ty in range(nty):
                            r0 = lo + np.array([tx, ty]) * T
                            r1 = r0 + T
                            own = np.all((x0[:, :2] >= r0) & (x0[:, :2] < r1), axis=1)
                            if not own.any():
                                continue
                            L0, L1 = r0 - W, r1 + W
                            ld = np.all((x0[:, :2] >= L0) & (x0[:, :2] < L1), axis=1)
                            idx = np.flatnonzero(ld)
                            loc = -np.ones(sc.n, np.int64)
                            loc[idx] = np.arange(idx.size)
                            e = pairs[ld[pairs[:, 0]] & ld[pairs[:, 1]]]
                            xy = x0[idx, :2]
                            sb = Sa[idx]
                            bx = np.minimum(xy[:, 0] - L0[0], L1[0] - xy[:, 0]) < reach + sb[:, 0] + Smax[0]
                            by = np.minimum(xy[:, 1] - L0[1], L1[1] - xy[:, 1]) < reach + sb[:, 1] + Smax[1]
                            h = hops(xy, loc[e[:, 0]], loc[e[:, 1]], idx.size, bx | by, K)
                            worst = min(worst, int(h[own[idx]].min()))
                            rho_l += idx.size
                            rho_o += int(own.sum())
                            maxload = max(maxload, idx.size)
                    print(f"  K={K:2d} block@{a.start + b0}: Smax={Smax.round(4)} mean deg {deg.mean():.2f} max {deg.max()} | "
                          f"T={T} W={W}: min hop {worst} ({'ok' if worst >= K else 'FAIL'}), "
                          f"loaded/owned {rho_l / rho_o:.2f}, max loaded {maxload}", flush=True)

if __name__ == "__main__":
    main()
