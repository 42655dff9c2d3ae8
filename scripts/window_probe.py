"""Diagnostic: C3's per-step device time window by window (50-step graph
replays, HIP events) in the hashed forms and in the tile form, from t = 0 to
step 850.  Not part of the product.

    python scripts/window_probe.py [--config c3] [--steps 850]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=850)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import rbhip
    from rbhip import scenes
    sc = scenes.make(a.config)
    rows = {}
    for name, tile in (("hashed", "0"), ("tile", "1")):
        os.environ["RBHIP_TILE"] = tile
        with rbhip.World(sc) as w:
            del os.environ["RBHIP_TILE"]
            w.set_stream(torch.cuda.current_stream().cuda_stream)
            w.step(2)                               # (steps 1-2: table / bins built; the first
                                                    # 50-step window below also captures its graph)
            done, out = 2, []
            while done + 50 <= a.steps:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                w.step_async(50)
                e1.record()
                w.sync()
                torch.cuda.synchronize()
                out.append((done + 1, done + 50, e0.elapsed_time(e1) * 1e3 / 50))
                done += 50
            rows[name] = out
    for (lo, hi, h), (_, _, t) in zip(rows["hashed"], rows["tile"]):
        print(f"{a.config} steps {lo:4d}-{hi:4d}: hashed {h:6.2f} us  tile {t:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
