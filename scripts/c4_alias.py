"""Diagnostic (CPU, oracle): the world's linear bucket layout under drift.
The layout's period split (rb_capi.hip fit_period: lg bits over x, y, z,
scored by colliding groups) is fitted to the positions at rb_set_state.
Here: the split chosen at t = 0 for C4, and at later steps the ids a body's
eight buckets hold under that split (aliased cells included) against the
true ids of its eight cells, and against the split refitted then.

    python scripts/c4_alias.py [--steps 451,651,851,1801]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
sys.path.insert(0, ROOT)
GB = (3, 3, 2)


def groups(q, inv_cs):
    c = np.floor(q[:, :3] * inv_cs).astype(np.int64)
    return c, c >> np.array(GB)


def collisions(occ, l):
    """fit_period's score: groups a search reads (occupied + neighbours) that
    share a bucket run with another, one of them occupied."""
    occ = np.unique(occ, axis=0)
    nb = np.array([[dx, dy, dz] for dz in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)])
    q = np.unique((occ[:, None, :] + nb[None]).reshape(-1, 3), axis=0) if len(occ) <= 8192 else occ
    occ_set = {tuple(r) for r in occ}
    isocc = np.array([tuple(r) in occ_set for r in q])
    idx = (q[:, 0] & ((1 << l[0]) - 1)) | ((q[:, 1] & ((1 << l[1]) - 1)) << l[0]) | \
          ((q[:, 2] & ((1 << l[2]) - 1)) << (l[0] + l[1]))
    order = np.lexsort((~isocc, idx))
    idx, isocc = idx[order], isocc[order]
    u, start, cnt = np.unique(idx, return_index=True, return_counts=True)
    anyocc = np.maximum.reduceat(isocc.astype(np.int64), start) > 0
    return int(((cnt - 1) * anyocc).sum())


def best_split(q, inv_cs, lg):
    c, g = groups(q, inv_cs)
    occ = np.unique(g, axis=0)
    lo, hi = q[:, :3].min(0) * inv_cs, q[:, :3].max(0) * inv_cs
    need = (np.floor(hi) - np.floor(lo) + 2) / np.array([1 << b for b in GB])
    best = None
    for lx in range(0, min(lg, 15) + 1):
        for ly in range(0, min(lg - lx, 15) + 1):
            lz = lg - lx - ly
            if lz > 15:
                continue
            l = (lx, ly, lz)
            coll = collisions(occ, l)
            fold = max(need[d] / (1 << l[d]) for d in range(3))
            nf = sum(need[d] > (1 << l[d]) for d in range(3))
            key = (int(coll), int(nf), float(fold))
            if best is None or key < best[0]:
                best = (key, l)
    return tuple(int(x) for x in best[1]), best[0]


def bucket_of(c, l):
    g = c >> np.array(GB)
    sc = (g[:, 0] & ((1 << l[0]) - 1)) | ((g[:, 1] & ((1 << l[1]) - 1)) << l[0]) | \
         ((g[:, 2] & ((1 << l[2]) - 1)) << (l[0] + l[1]))
    inn = (c[:, 0] & 7) | ((c[:, 1] & 7) << 3) | ((c[:, 2] & 3) << 6)
    return (sc << 8) | inn


def per_body(q, inv_cs, l):
    c = np.floor(q[:, :3] * inv_cs).astype(np.int64)
    s = np.where(q[:, :3] * inv_cs - c < 0.5, -1, 1)
    b0 = bucket_of(c, l)
    ub, cnt = np.unique(b0, return_counts=True)
    tot = np.zeros(len(q), np.int64)
    seen = []
    for m in range(8):
        off = np.stack([(m & 1) * s[:, 0], ((m >> 1) & 1) * s[:, 1], ((m >> 2) & 1) * s[:, 2]], 1)
        bk = bucket_of(c + off, l)
        dup = np.zeros(len(q), bool)
        for prev in seen:
            dup |= prev == bk
        seen.append(bk)
        i = np.minimum(np.searchsorted(ub, bk), len(ub) - 1)
        tot += np.where((ub[i] == bk) & ~dup, cnt[i], 0)
    return tot, int(cnt.max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="451,651,851,1801")
    a = ap.parse_args()
    from oracle import oracle as O
    from rbhip import scenes
    O.build()
    O.set_threads(8)
    sc = scenes.make("c4")
    rmax = float(np.max(sc.size[:, 0]))
    inv_cs = 1.0 / (4.0 * rmax * 1.001)
    H = 1 << int(np.ceil(np.log2(32 * sc.n)))
    lg = int(np.log2(H)) - sum(GB)
    l0, key0 = best_split(sc.qpos0, inv_cs, lg)
    print(json.dumps({"H": H, "lg": lg, "split_t0": l0, "score_t0": key0}), flush=True)
    osc = O.OracleScene(sc, max_partners=32)
    q, v, done = sc.qpos0, sc.qvel0, 0
    for t in [int(x) for x in a.steps.split(",")]:
        q, v = O.step(osc, q, v, t - done)
        done = t
        ids0, mb0 = per_body(q, inv_cs, l0)
        lt, keyt = best_split(q, inv_cs, lg)
        idst, mbt = per_body(q, inv_cs, lt)
        nw = sc.n // 64
        w0 = ids0[:nw * 64].reshape(nw, 64).max(1)
        wt = idst[:nw * 64].reshape(nw, 64).max(1)
        ext = (q[:, :3].max(0) - q[:, :3].min(0)).round(1).tolist()
        print(json.dumps({"step": t, "extent_m": ext,
                          "t0_split": {"ids_per_body_mean": float(ids0.mean()), "max": int(ids0.max()),
                                       "wave_max_mean": float(w0.mean()), "max_bucket": mb0,
                                       "buckets_over_30": None},
                          "refit_split": {"l": lt, "score": keyt, "ids_per_body_mean": float(idst.mean()),
                                          "max": int(idst.max()), "wave_max_mean": float(wt.mean()),
                                          "max_bucket": mbt}}), flush=True)


if __name__ == "__main__":
    main()
