"""Diagnostic: per-phase stamps of the tile kernel (build/tile_stamps.so,
built with EXTRA=-DRB_TILE_STAMPS=1).  Steps a scene in the tile form, then
one more single-step run, and prints per phase the median / p90 / max of the
workgroups' core-clock cycles, and the launch's start spread and span from
the constant 100 MHz clock.  Not part of the product.

    python scripts/tile_stamps.py [--config c3] [--warm 400] [--lib build/tile_stamps.so]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))

PHASES = ["column tables", "window starts", "loads + gravity/planes", "window to LDS + far + search", "(empty: the id order is selected in the solves)",
          "partner solves + integrate", "place + barrier", "bin scan + offsets", "record stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warm", type=int, default=400)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "tile_stamps.so"))
    a = ap.parse_args()
    import numpy as np
    os.environ["RBHIP_TILE"] = "1"
    from rbhip import _lib, scenes
    import rbhip.world as W
    L = _lib.load(a.lib)
    L.rb_diag_tile_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    sc = scenes.make(a.config)
    with W.World(sc, max_partners=32 if a.config == "c4" else 16) as w:
        for _ in range(a.warm // 50):                # (chunks: a rollback's backoff ends between them)
            w.step(50)
        for _ in range(20):                          # a 2-step run that committed in the tile form
            s0 = w.stats()                           # (the stamps: its second step's)
            w.step(2)
            st = w.stats()
            if st["tile_steps"] == s0["tile_steps"] + 2 and st["tile_rollbacks"] == s0["tile_rollbacks"]:
                break
            print("  (single step not committed in the tile form:", {k: st[k] for k in st if k.startswith("tile")}, ")")
        else:
            sys.exit("no committed 2-step tile run")
        nb = st["tile_slots"]
        buf = np.zeros((nb, 12), np.uint64)
        rc = L.rb_diag_tile_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb)
        assert rc == 0, rc
    s = buf.astype(np.int64)
    live = s[:, 9] > 0
    print(f"{a.config}: {nb} slots ({int(live.sum())} ran to the end), stats {st}")
    for k, name in enumerate(PHASES):
        d = s[live, k + 1] - s[live, k]
        d = d[(d >= 0) & (d < 10**8)]
        if d.size:
            print(f"  {k}->{k + 1} {name:22s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8.0f}")
    tot = s[live, 9] - s[live, 0]
    print(f"  total per workgroup: median {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max()} cycles")
    r0, r1 = s[live, 10], s[live, 11]
    t0 = r0.min()
    print(f"  100 MHz clock: starts spread over {(r0.max() - t0) / 100:.2f} us, last end {(r1.max() - t0) / 100:.2f} us "
          f"after the first start; median workgroup {np.median(r1 - r0) / 100:.2f} us")


if __name__ == "__main__":
    main()
