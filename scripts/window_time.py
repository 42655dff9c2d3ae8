"""Diagnostic: per-step device time of a window of graph-replayed steps
(HIP events around K steps after W warm steps, scene from rbhip.scenes) for
the library given — A/Bs of library builds, one build per process.  Not
part of the product.

    python scripts/window_time.py [--lib PATH] --config c3 --warm 45 --steps 20 [--reps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "rigidbody-simulation_amd", "rbhip", "librbhip.so"))
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warm", type=int, default=45)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    assert a.warm >= a.steps, "warm >= steps (the last K warm steps capture the graph)"
    import torch
    torch.cuda.init()
    from rbhip import _lib, scenes
    _lib.load(a.lib)
    import rbhip
    sc = scenes.make(a.config)
    kw = {"max_partners": 32} if a.config == "c4" else {}
    out = []
    for r in range(a.reps):
        with rbhip.World(sc, **kw) as w:
            w.set_stream(torch.cuda.current_stream().cuda_stream)
            # the last K warm steps capture the K-step graph the window replays
            w.step(a.warm - a.steps)
            w.step(a.steps)
            w.sync()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            w.step_async(a.steps)
            e1.record()
            w.sync()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3 / a.steps)
            form = _lib.FORM_NAMES.get(w.stats()["form"])
    print(f"{os.path.basename(a.lib)} {a.config} steps {a.warm + 1}-{a.warm + a.steps}: "
          f"{' '.join(f'{t:.2f}' for t in out)} us/step ({form})", flush=True)


if __name__ == "__main__":
    main()
