"""Diagnostic: per-step stamps of the resident kernel (diag/res_stamps.so,
built with EXTRA=-DRB_RES_STAMPS=1).  Steps a scene in the resident form,
then one more window of K steps, and prints from the constant 100 MHz clock:
the launch's start spread, each workgroup's setup, and per step the time to
the imports' arrival, the cell sort, the solve and the publication (median /
p90 / max over the slots), relative to the launch's first start.  Not part of the
product.

    python scripts/res_stamps.py [--config c2] [--warm 40] [--k 16] [--lib diag/res_stamps.so]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
NST = 40


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--lib", default=os.path.join(ROOT, "diag", "res_stamps.so"))
    a = ap.parse_args()
    import numpy as np
    os.environ["RBHIP_RESIDENT"] = "1"
    os.environ["RBHIP_TILE"] = "0"
    from rbhip import _lib, scenes
    import rbhip.world as W
    L = _lib.load(a.lib)
    L.rb_diag_res_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    sc = scenes.make(a.config) if ":" not in a.config else scenes.flat_spheres(*map(int, a.config.split(":")[1:]))
    with W.World(sc) as w:
        w.step(a.warm)
        for _ in range(20):
            s0 = w.stats()
            w.step(a.k)
            st = w.stats()
            if st["res_steps"] == s0["res_steps"] + a.k and st["res_rollbacks"] == s0["res_rollbacks"]:
                break
            print("  (window not committed:", {k: st[k] for k in st if k.startswith("res")}, ")")
        else:
            sys.exit("no committed resident window")
        nb = st["res_slots"]
        buf = np.zeros((nb, NST), np.uint64)
        rc = L.rb_diag_res_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb)
        assert rc == 0, rc
    s = buf.astype(np.int64)
    live = s[:, 2] > 0
    s = s[live]
    t0 = s[:, 0].min()
    us = lambda v: (v - t0) / 100.0                      # noqa: E731
    q = lambda v: f"{np.median(v):8.2f} {np.percentile(v, 90):8.2f} {v.max():8.2f}"   # noqa: E731
    print(f"{a.config}: {nb} slots, {int(live.sum())} with bodies; K = {a.k}; stats {st}")
    print(f"  (us after the first start: median p90 max)")
    print(f"  start                  {q(us(s[:, 0]))}")
    print(f"  setup done (bin lists)  {q(us(s[:, 1]))}")
    n = min(a.k, 8)
    for t in range(n):
        c = 4 + 4 * t
        print(f"  step {t}: imports in {q(us(s[:, c]))} | sorted {q(us(s[:, c + 1]))} | "
              f"solved {q(us(s[:, c + 2]))} | published {q(us(s[:, c + 3]))}")
    print(f"  end                    {q(us(s[:, 2]))}")
    # per phase (median over slots of each slot's own interval), steps 1 .. n-2
    ph = {"wait + import": [], "cell sort": [], "solve": [], "export + publish": []}
    for t in range(1, n - 1):
        c = 4 + 4 * t
        ph["wait + import"].append(np.median(s[:, c] - s[:, c - 1]) / 100.0)
        ph["cell sort"].append(np.median(s[:, c + 1] - s[:, c]) / 100.0)
        ph["solve"].append(np.median(s[:, c + 2] - s[:, c + 1]) / 100.0)
        ph["export + publish"].append(np.median(s[:, c + 3] - s[:, c + 2]) / 100.0)
    for k, v in ph.items():
        print(f"  phase {k:18s} median over slots, per step: {np.round(v, 2).tolist()}")
    d = np.diff(np.median(us(s[:, 7:4 + 4 * n:4]), axis=0))
    print(f"  per step (median publication to publication): {np.round(d, 2).tolist()}")


if __name__ == "__main__":
    main()
