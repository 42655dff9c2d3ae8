"""Time the K-step tile blocks against the per-step kernels (one GPU).

    python scripts/tile_time.py [--config c3] [--warmup 450] [--steps 400] [--k 8] [--band 0] [--owned 256]

For each mode: a fresh World, `warmup` steps, `steps` untimed steps (the
per-step path captures its graph there), then `steps` timed steps (host wall
clock around one synchronous rb_step), with the world's counters
(blocks, redos, fallbacks).  Checks that both modes end bit-identical.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))

import rbhip  # noqa: E402
from rbhip import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warmup", type=int, default=450)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--band", type=float, default=0.0)
    ap.add_argument("--owned", type=int, default=0)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--modes", default="0,1")
    a = ap.parse_args()
    if a.config.startswith("flat:"):                 # flat:NXxNY (C3's layout, e.g. one 8-GPU slab: flat:256x32)
        nx, ny = (int(v) for v in a.config[5:].split("x"))
        sc = scenes.flat_spheres(nx, ny)
    else:
        sc = scenes.make(a.config)
    res = {}
    for mode in [int(m) for m in a.modes.split(",")]:
        with rbhip.World(sc, dtype=a.dtype) as w:
            w.tile_config(mode, a.k, a.band, a.owned)
            w.step(a.warmup)
            w.step(a.steps)                   # capture the per-step graph outside the timed region
            s0 = w.stats()
            t0 = time.perf_counter()
            w.step(a.steps)
            el = time.perf_counter() - t0
            s1 = w.stats()
            q, v = w.get_state()
        d = {k: s1[k] - s0[k] for k in ("tile_blocks", "tile_redo_taint", "tile_redo_bound", "tile_restart",
                                         "tile_fallback", "tile_steps")}
        res[mode] = (q, v)
        print(json.dumps({"config": a.config, "dtype": a.dtype, "tile_mode": mode, "bodies": sc.n,
                          "timed_steps": [a.warmup + a.steps + 1, a.warmup + 2 * a.steps], "us_per_step": el / a.steps * 1e6,
                          "body_steps_per_s": sc.n * a.steps / el, "tiles": s1["tiles"], "tile_kmax": s1["tile_kmax"],
                          "tile_size_m": s1["tile_size_um"] * 1e-6, **d}), flush=True)
    if len(res) == 2:
        (q0, v0), (q1, v1) = res.values()
        same = np.array_equal(q0.view(np.uint64), q1.view(np.uint64)) and np.array_equal(v0.view(np.uint64),
                                                                                       v1.view(np.uint64))
        print(json.dumps({"bit_identical_modes": bool(same)}), flush=True)
        if not same:
            sys.exit(3)


if __name__ == "__main__":
    main()
