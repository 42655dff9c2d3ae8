"""Diagnostic: per-step device time (HIP events around K graph-replayed
steps, after 260 warm steps) of C2 and of the 8,192-sphere slab (256 x 32:
one C3 rank's shape at P = 8), for the library given (default: the
in-tree one; a diagnostic build is swapped in by the caller).  Not part of
the product.

    python scripts/slab_time.py [--lib PATH] [--K 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "rigidbody-simulation_amd", "rbhip", "librbhip.so"))
    ap.add_argument("--K", type=int, default=200)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from rbhip import _lib, scenes
    _lib.load(a.lib)
    import rbhip
    for name, sc in (("c2", scenes.make("c2")), ("slab8192", scenes.flat_spheres(256, 32))):
        with rbhip.World(sc) as w:
            w.set_stream(torch.cuda.current_stream().cuda_stream)
            w.step(260)
            w.step(a.K)
            w.sync()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            w.step_async(a.K)
            e1.record()
            w.sync()
            torch.cuda.synchronize()
            form = _lib.FORM_NAMES.get(w.stats()["form"])
            print(f"{os.path.basename(a.lib)} {name}: {e0.elapsed_time(e1) * 1e3 / a.K:.2f} us/step ({form})", flush=True)


if __name__ == "__main__":
    main()
