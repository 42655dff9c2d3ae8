"""Diagnostic (CPU, oracle): how crowded C4's neighbourhoods get, in the
wide search's units (rb_grid.hpp search_buckets_wide).  For each body, the
2x2x2 nearest cells of the world's grid (cell = 4 rmax x 1.001); a bucket's
head carries 6 ids, the rest are read in batches of 12 (the rare path).
Per window step: the bodies' head candidates and extra ids, and the rare
path's dependent batches per body — per bucket (round 3: each bucket's
extra ids in their own batches) and across buckets (round 4) — as the
max over each 64-body wave, whose slowest lane sets its time.

    python scripts/c4_crowding.py [--steps 261,451,651,851,1201,1801]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
sys.path.insert(0, ROOT)


def stats_at(q, rmax):
    cs = 4.0 * rmax * 1.001
    c = np.floor(q[:, :3] / cs).astype(np.int64)
    fr = q[:, :3] / cs - c
    s = np.where(fr < 0.5, -1, 1)
    key = lambda a: (a[:, 0] + (1 << 20)) * (1 << 42) + (a[:, 1] + (1 << 20)) * (1 << 21) + (a[:, 2] + (1 << 20))
    k0 = key(c)
    uk, cnt = np.unique(k0, return_counts=True)
    n = q.shape[0]
    head = np.zeros(n, np.int64)
    extra = np.zeros(n, np.int64)
    per_bucket = np.zeros(n, np.int64)
    for m in range(8):
        off = np.stack([(m & 1) * s[:, 0], ((m >> 1) & 1) * s[:, 1], ((m >> 2) & 1) * s[:, 2]], 1)
        kk = key(c + off)
        idx = np.searchsorted(uk, kk)
        idx = np.minimum(idx, uk.size - 1)
        ct = np.where(uk[idx] == kk, cnt[idx], 0)
        head += np.minimum(ct, 6)
        ex = np.maximum(ct - 6, 0)
        extra += ex
        per_bucket += -(-ex // 12)
    head -= 1                                     # the body itself
    flat = -(-extra // 12)
    hb = np.maximum(1, -(-head // 12))
    nw = n // 64
    wave = lambda a: a[:nw * 64].reshape(nw, 64).max(1)
    return {"head_cand_mean": float(head.mean()), "head_cand_max": int(head.max()),
            "extra_ids_mean": float(extra.mean()), "extra_ids_p99": float(np.percentile(extra, 99)),
            "extra_ids_max": int(extra.max()),
            "max_bodies_per_cell": int(cnt.max()),
            "wave_batches_r3_mean": float(wave(hb + per_bucket).mean()),
            "wave_batches_r4_mean": float(wave(hb + flat).mean()),
            "wave_batches_r3_max": int(wave(hb + per_bucket).max()),
            "wave_batches_r4_max": int(wave(hb + flat).max()),
            "waves_with_rare_path": int((wave(extra) > 0).sum()), "waves": nw}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", default="261,451,651,851,1201,1801")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    from oracle import oracle as O
    from rbhip import scenes
    O.build()
    O.set_threads(a.threads)
    sc = scenes.make(a.config)
    osc = O.OracleScene(sc, max_partners=32)    # (C4's pile-ups pass 16 partners)
    rmax = float(np.max(sc.size[:, 0]))
    q, v, done = sc.qpos0, sc.qvel0, 0
    for t in [int(x) for x in a.steps.split(",")]:
        q, v = O.step(osc, q, v, t - done)
        done = t
        print(json.dumps({"config": a.config, "step": t, **stats_at(q, rmax)}), flush=True)


if __name__ == "__main__":
    main()
