"""Per-phase cycles of the tile-block kernel (diagnostic build
librbhip_stamps.so, RB_TILE_STAMPS=1): load bins, load records, lists,
K steps, write-back, summed over the stepping workgroups of the timed steps.

    python scripts/tile_stamps.py [--config c3] [--warmup 450] [--steps 400] [--k 8] [--band 0] [--owned 0]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))

from rbhip import _lib, scenes  # noqa: E402

L = _lib.load(os.path.join(ROOT, "rigidbody-simulation_amd", "rbhip", "librbhip_stamps.so"))
import rbhip  # noqa: E402

L.rb_diag_tile_stamps.argtypes = [C.c_void_p, C.c_int]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warmup", type=int, default=450)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--band", type=float, default=0.0)
    ap.add_argument("--owned", type=int, default=0)
    a = ap.parse_args()
    sc = scenes.make(a.config)
    buf = (C.c_ulonglong * 16)()
    with rbhip.World(sc) as w:
        w.tile_config(1, a.k, a.band, a.owned)
        w.step(a.warmup)
        L.rb_diag_tile_stamps(buf, 1)
        s0 = w.stats()
        t0 = time.perf_counter()
        w.step(a.steps)
        el = time.perf_counter() - t0
        s1 = w.stats()
        L.rb_diag_tile_stamps(buf, 0)
    n = max(buf[8], 1)
    names = ["", "load bins", "load records", "lists", "steps", "write"]
    out = {"config": a.config, "us_per_step": el / a.steps * 1e6, "wg_blocks": buf[8],
           "mean_k_run": buf[9] / n, "mean_stepped": buf[10] / n, "mean_outer": buf[11] / n,
           "cycles_per_wg": {names[k]: buf[k] / n for k in range(1, 6)},
           "active_lanes_per_wg_step": buf[14] / max(buf[9], 1), "active_waves_per_wg_step": buf[15] / max(buf[9], 1),
           "lists_split": {"columns": buf[12] / n, "scan": buf[13] / n, "sort": (buf[3] - 0) / n},
           "tile": {k: s1[k] - s0[k] for k in ("tile_blocks", "tile_redo_taint", "tile_redo_bound", "tile_restart",
                                                "tile_fallback", "tile_steps")}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
