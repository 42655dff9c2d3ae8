"""Host cost of the reference-surface per-frame entry and drift of C4.

    python scripts/frame_cost.py [--config c3] [--frames 20]

1. custom_step_multi_sphere's per-frame path (rbhip.adapter.step_model, as
   multi_sphere_bounce.py:42 is called once per frame): every call uploads
   the state (rb_set_state), runs one step and downloads the state.  Timed
   per call and split into set_state / step / get_state, on the scene's
   65,536 bodies, with the positions moving between calls (fit_period's
   group-box cache) and with the same positions.
2. C4 drift: the wall clock of 200 steps at steps 261-460
   and at 1,801-2,000 of one world (the layout period is fitted once, from
   the initial positions).
One JSON line per measurement.
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
from rbhip import adapter, scenes  # noqa: E402


def timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return time.perf_counter() - t0, r


def frame_cost(cfg: str, frames: int):
    sc = scenes.make(cfg)
    model, data = adapter.load_scene_model(sc)
    p = dict(dt=sc.dt, restitution=sc.restitution, friction=sc.friction, threshold=sc.threshold)
    adapter.step_model(model, data, 1, **p)          # world creation, first fit, graph-free single step
    tot = []
    for _ in range(frames):
        t, _ = timed(lambda: adapter.step_model(model, data, 1, **p))
        tot.append(t)
    w = adapter.world_for(model, "oriented", "mujoco", 0.01, sc.restitution, sc.friction)
    qi, vi = adapter.state_index(model)
    parts = {"set_state": [], "step": [], "get_state": [], "set_state_same": []}
    for _ in range(frames):
        q, v = np.asarray(data.qpos)[qi], np.asarray(data.qvel)[vi]
        t, _ = timed(lambda: w.set_state(q, v)); parts["set_state"].append(t)
        t, _ = timed(lambda: w.step(1, **p)); parts["step"].append(t)
        t, (q2, v2) = timed(lambda: w.get_state()); parts["get_state"].append(t)
        data.qpos[qi], data.qvel[vi] = q2, v2
        t, _ = timed(lambda: w.set_state(q2, v2)); parts["set_state_same"].append(t)
    print(json.dumps({"what": "per-frame host cost (adapter.step_model, 1 step per call)", "config": cfg,
                      "bodies": sc.n, "frames": frames, "ms_per_call_median": 1e3 * float(np.median(tot)),
                      **{f"{k}_ms_median": 1e3 * float(np.median(v)) for k, v in parts.items()}}), flush=True)


def c4_drift():
    # C4 needs max_partners >= 28 after ~550 steps (sliding rows run into
    # each other: up to 28 sphere partners, the oracle with max_partners=64)
    sc = scenes.make("c4")
    out = {}
    with rbhip.World(sc, max_partners=32) as w:
        w.step(260)
        w.step(200)                                  # graph capture outside the timed windows
        w.step(1)
        w.sync()
        c = 461
        for lo in (461, 1801):
            w.step(lo - c)
            w.sync()
            t, _ = timed(lambda: w.step(200))
            out[f"steps_{lo}_{lo + 199}_us_per_step"] = t / 200 * 1e6
            c = lo + 200
    a, b = out["steps_461_660_us_per_step"], out["steps_1801_2000_us_per_step"]
    print(json.dumps({"what": "C4 drift: wall clock per step of 200-step windows (one world, max_partners 32)", **out,
                      "late_over_early": b / a}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--skip-drift", action="store_true")
    a = ap.parse_args()
    frame_cost(a.config, a.frames)
    if not a.skip_drift:
        c4_drift()


if __name__ == "__main__":
    main()
