"""Diagnostic: where a step of the XCD-resident blocks goes.
Loads the stamp build of the library (`make -C rigidbody-simulation_amd/csrc
OUT=../../build/xbstamps.so OBJDIR=build_xbstamps EXTRA=-DRB_XB_STAMPS=1`),
steps a scene to `--start`, then one launch of K steps, and prints the body
code's phase spans (s_memtime cycles, wave 0 of each workgroup, the launch's
last step: rb_kernels.hip STAMP) and the launch's own phases
(rb_diag_xb_stamps, us).  Phases: 0 start, 1 own loads issued, 8 heads back,
9 head candidates tested, 10 rare path done, 2 search done, 3 forces,
4 solves done, 5 claim + snapshot store, 6 end."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "xbstamps.so"))
    ap.add_argument("--config", default="c3")
    ap.add_argument("--start", type=int, default=25)
    ap.add_argument("--k", type=int, default=8)
    a = ap.parse_args()
    os.environ["RBHIP_XB"] = "1"
    os.environ["RBHIP_XB_K"] = str(a.k)
    from rbhip import _lib, scenes
    import rbhip.world as W
    L = _lib.load(a.lib)
    L.rb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    sc = scenes.flat_spheres(256, 32, seed=0) if a.config == "slab8k" else scenes.make(a.config)
    with W.World(sc) as w:
        w.step(a.start)
        w.step(a.k)
        st = w.stats()
        buf = np.zeros((256, 16), np.uint64)
        L.rb_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), 256)
        xb = np.zeros((512, 8), np.uint64)
        wpg = ctypes.c_int32(0)
        _lib.check(L.rb_diag_xb_stamps(w._h, xb.ctypes.data_as(ctypes.c_void_p), 512, ctypes.byref(wpg)), "stamps")
    nwg = 8 * wpg.value
    b = buf[:nwg].astype(np.int64)
    phases = [(0, 1, "own loads"), (1, 8, "heads"), (8, 9, "head cands"), (9, 10, "rare path"),
              (10, 2, "search tail"), (2, 3, "forces"), (3, 4, "solves"), (4, 5, "claim+snap"), (5, 6, "quat+store")]
    out = {"config": a.config, "K": a.k, "xb_steps": st["xb_steps"], "xb_fallbacks": st["xb_fallbacks"],
           "step_cycles_median": int(np.median(b[:, 6] - b[:, 0])), "step_cycles_max": int((b[:, 6] - b[:, 0]).max())}
    for lo, hi, nm in phases:
        d = b[:, hi] - b[:, lo]
        out[nm] = [int(np.median(d)), int(d.max())]
    x = xb[:nwg].astype(np.int64)
    d = np.diff(x, axis=1) / 100.0
    names = ["bound", "counts", "map", "copy", "step0", "steps1..", "commit"]
    out["launch_us_median"] = {nm: round(float(np.median(d[:, j])), 2) for j, nm in enumerate(names)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
