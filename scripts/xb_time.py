"""Per-step time of the XCD-resident K-step blocks against the per-step
kernels: a scene stepped from t = 0 to step `start`, then
`steps` steps timed (HIP events on the world's stream around one async call,
then rb_sync), for each K.  Also checks the final states bit for bit.

    python scripts/xb_time.py [--config c3] [--start 25] [--steps 20] [--ks 0,2,4,6,8,12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--start", type=int, default=25)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="0,2,4,6,8,12")
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    import numpy as np
    import torch
    import rbhip
    from rbhip import scenes
    rbhip.load()
    # slab8k: one rank's 256 x 32 slab of C3 at 8 GPUs (8,192 bodies)
    sc = scenes.flat_spheres(256, 32, seed=0) if a.config == "slab8k" else scenes.make(a.config)
    rows, ref = [], None
    for k in [int(x) for x in a.ks.split(",")]:
        os.environ["RBHIP_XB"] = "1" if k > 0 else "0"
        if k > 0:
            os.environ["RBHIP_XB_K"] = str(k)
        w = rbhip.World(sc, dtype=a.dtype)
        w.set_stream(torch.cuda.current_stream().cuda_stream)
        w.step(a.start)
        w.step_async(a.steps)            # capture
        w.sync()
        times = []
        for rep in range(a.reps):           # successive windows after the first (capture) call
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            w.step_async(a.steps)
            e1.record()
            w.sync()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            times.append((e0.elapsed_time(e1) / a.steps * 1e3, wall / a.steps * 1e6))
        st = w.stats()
        phases = None
        if k > 0 and st["xb_steps"] > 0:
            # the last launch's phase stamps (rb_diag_xb_stamps): median
            # workgroup's time per phase, us
            import ctypes
            buf = np.zeros((512, 8), np.uint64)
            wpg = ctypes.c_int32(0)
            rbhip._lib.check(w._L.rb_diag_xb_stamps(w._h, buf.ctypes.data_as(ctypes.c_void_p), 512, ctypes.byref(wpg)),
                             "rb_diag_xb_stamps")
            b = buf[:8 * wpg.value].astype(np.int64)
            d = np.diff(b, axis=1) / 100.0
            names = ["bound", "counts", "map", "copy", "step0", "steps1..", "commit"]
            phases = {nm: round(float(np.median(d[:, j])), 2) for j, nm in enumerate(names)}
            phases["span"] = round(float((b[:, 7].max() - b[:, 0].min()) / 100.0), 2)
        q, v = w.get_state()
        w.close()
        if ref is None:
            ref = (q, v)
        same = bool(np.array_equal(q.view(np.uint64), ref[0].view(np.uint64)) and
                    np.array_equal(v.view(np.uint64), ref[1].view(np.uint64)))
        dev = sorted(t[0] for t in times)
        wall = sorted(t[1] for t in times)
        rows.append({"K": k, "us_per_step_events_min": dev[0], "us_per_step_events_med": dev[len(dev) // 2],
                     "us_per_step_wall_med": wall[len(wall) // 2], "same_as_first": same,
                     "xb_steps": st["xb_steps"], "xb_fallbacks": st["xb_fallbacks"], "form": st["form"],
                     "phases_us": phases})
        print(json.dumps(rows[-1]), flush=True)
    os.environ.pop("RBHIP_XB", None)
    os.environ.pop("RBHIP_XB_K", None)


if __name__ == "__main__":
    main()
