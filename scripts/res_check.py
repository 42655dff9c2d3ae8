"""Diagnostic: the resident form (rb_resident.hip) against the hashed-cell
forms on the GPU — bit identity of the state (uint64 words) after each
chunk, the resident counters, and the time per step of both (HIP events
around K graph-replayed steps on torch's stream).  Not part of the product.

    python scripts/res_check.py [--configs c3,c2] [--chunks 5,20,20,100,1,1,300] [--time 200,20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def world(sc, resident, **kw):
    import rbhip
    env = {"RBHIP_RESIDENT": "1" if resident else "0", "RBHIP_TILE": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return rbhip.World(sc, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def same(a, b):
    import numpy as np
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c2")
    ap.add_argument("--chunks", default="5,20,20,100,1,1,300")
    ap.add_argument("--time", default="200,20")
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rbhip import scenes
    chunks = [int(c) for c in a.chunks.split(",") if c]
    for cfg in a.configs.split(","):
        if ":" in cfg:
            kind, nx, ny = cfg.split(":")
            sc = {"flat": scenes.flat_spheres, "incl": scenes.incline_spheres}[kind](int(nx), int(ny))
        else:
            sc = scenes.make(cfg)
        kw = {"max_partners": 32} if cfg == "c4" or cfg.startswith("incl") else {}
        wr, wh = world(sc, True, dtype=a.dtype, **kw), world(sc, False, dtype=a.dtype, **kw)
        done = 0
        ok = True
        for n in chunks:
            wr.step_async(n)
            wh.step_async(n)
            done += n
            wr.sync()
            wh.sync()
            qt, vt = wr.get_state()
            qh, vh = wh.get_state()
            eq = same(qt, qh) and same(vt, vh)
            ok &= eq
            st = wr.stats()
            print(f"{cfg}: after {done} steps {'identical' if eq else 'DIFFER'}; "
                  f"{ {k: st[k] for k in st if k.startswith('res') or k == 'form'} }", flush=True)
            if not eq:
                bad = np.flatnonzero(~(np.all(qt.view(np.uint64) == qh.view(np.uint64), axis=1)))
                print(f"{cfg}: DIFFER after {done} steps: {bad.size} bodies, first {bad[:8].tolist()}, "
                      f"max |dq| {np.abs(qt - qh).max():.3e}", flush=True)
                break
        print(f"{cfg}: {'bit-identical' if ok else 'MISMATCH'} after {done} steps", flush=True)
        for K in [int(k) for k in a.time.split(",") if k]:
            res = {}
            rb0 = wr.stats()["res_rollbacks"]
            for name, w in (("resident", wr), ("hashed", wh)):
                w.step(K)                          # capture the K-step graph
                w.sync()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s = torch.cuda.current_stream().cuda_stream
                w.set_stream(s)
                w.step(K)
                w.sync()
                e0.record()
                t0 = time.perf_counter()
                w.step_async(K)
                e1.record()
                w.sync()
                torch.cuda.synchronize()
                res[name] = (e0.elapsed_time(e1) * 1e3 / K, (time.perf_counter() - t0) * 1e6 / K)
            st = wr.stats()
            valid = "valid" if st["res_rollbacks"] == rb0 and st["form"] == 6 else "INVALID (roll-backs in the timed runs)"
            print(f"{cfg}: K={K} [{valid}] us/step device (wall): resident {res['resident'][0]:.2f} ({res['resident'][1]:.2f})  "
                  f"hashed {res['hashed'][0]:.2f} ({res['hashed'][1]:.2f}); "
                  f"{ {k: st[k] for k in st if k.startswith('res')} }", flush=True)
        qt, vt = wr.get_state()
        qh, vh = wh.get_state()
        print(f"{cfg}: final {'bit-identical' if same(qt, qh) and same(vt, vh) else 'MISMATCH'}", flush=True)
        wr.close()
        wh.close()


if __name__ == "__main__":
    main()
