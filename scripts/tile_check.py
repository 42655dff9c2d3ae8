"""Diagnostic: the cell-ordered tile form against the hashed-cell forms on
the GPU — bit identity of the state (uint64 words) after each chunk, the
tile counters, and the time per step of both (HIP events around K
graph-replayed steps on torch's stream).  Not part of the product.

    python scripts/tile_check.py [--configs c3,c2,c4,flat:1024:1024,incl:512:512] [--chunks 5,20,20,100] [--time 200]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def world(sc, tile, **kw):
    import rbhip
    os.environ["RBHIP_TILE"] = "1" if tile else "0"
    try:
        return rbhip.World(sc, **kw)
    finally:
        del os.environ["RBHIP_TILE"]


def same(a, b):
    import numpy as np
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c2,c4")
    ap.add_argument("--chunks", default="5,20,20,100,1,1,300")
    ap.add_argument("--time", type=int, default=200)
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rbhip import scenes
    chunks = [int(c) for c in a.chunks.split(",")]
    for cfg in a.configs.split(","):
        # "flat:NX:NY" / "incl:NX:NY": scenes.flat_spheres / incline_spheres(NX, NY)
        if ":" in cfg:
            kind, nx, ny = cfg.split(":")
            sc = {"flat": scenes.flat_spheres, "incl": scenes.incline_spheres}[kind](int(nx), int(ny))
        else:
            sc = scenes.make(cfg)
        kw = {"max_partners": 32} if cfg == "c4" or cfg.startswith("incl") else {}
        wt, wh = world(sc, True, dtype=a.dtype, **kw), world(sc, False, dtype=a.dtype, **kw)
        done = 0
        ok = True
        for n in chunks:
            wt.step_async(n)
            wh.step_async(n)
            done += n
            wt.sync()
            wh.sync()
            qt, vt = wt.get_state()
            qh, vh = wh.get_state()
            eq = same(qt, qh) and same(vt, vh)
            ok &= eq
            if not eq:
                bad = np.flatnonzero(~(np.all(qt.view(np.uint64) == qh.view(np.uint64), axis=1)))
                print(f"{cfg}: DIFFER after {done} steps: {bad.size} bodies, first {bad[:8].tolist()}, "
                      f"max |dq| {np.abs(qt - qh).max():.3e}", flush=True)
                break
        st = wt.stats()
        print(f"{cfg}: {'bit-identical' if ok else 'MISMATCH'} after {done} steps; tile stats "
              f"{ {k: st[k] for k in st if k.startswith('tile') or k == 'form'} }", flush=True)
        if a.time:
            res = {}
            for name, w in (("tile", wt), ("hashed", wh)):
                w.step(a.time)                     # capture the K-step graph
                w.sync()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s = torch.cuda.current_stream().cuda_stream
                w.set_stream(s)
                w.step(a.time)
                w.sync()
                e0.record()
                t0 = time.perf_counter()
                w.step_async(a.time)
                e1.record()
                w.sync()
                torch.cuda.synchronize()
                res[name] = (e0.elapsed_time(e1) * 1e3 / a.time, (time.perf_counter() - t0) * 1e6 / a.time)
            st = wt.stats()
            print(f"{cfg}: us/step device (wall): tile {res['tile'][0]:.2f} ({res['tile'][1]:.2f})  "
                  f"hashed {res['hashed'][0]:.2f} ({res['hashed'][1]:.2f}); tile rollbacks {st['tile_rollbacks']} "
                  f"why {st['tile_why']} slots {st['tile_slots']} cols {st['tile_cols']}", flush=True)
        wt.close()
        wh.close()


if __name__ == "__main__":
    main()
