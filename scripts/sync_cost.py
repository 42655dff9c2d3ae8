"""Diagnostic: host-side costs around a graph-replayed run (the driver's
bench shape: K = 20 steps between two syncs) — the enqueue call, rb_sync on
an idle stream, torch.cuda.synchronize, and the whole timed region against
its HIP-event device time.  Not part of the product.

    python scripts/sync_cost.py [--config c3] [--steps 20] [--reps 50]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    import rbhip
    from rbhip import scenes
    sc = scenes.make(a.config)
    K = a.steps
    with rbhip.World(sc) as w:
        w.set_stream(torch.cuda.current_stream().cuda_stream)
        w.step(5)
        w.step(K)                                   # capture
        w.sync(); torch.cuda.synchronize()
        enq, syn, tsyn, region, dev = [], [], [], [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            w.step_async(K)
            e1.record()
            t1 = time.perf_counter()
            w.sync()
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            enq.append(t1 - t0); region.append(t3 - t0); dev.append(e0.elapsed_time(e1) * 1e-3)
            # an idle sync and an idle device sync
            s0 = time.perf_counter(); w.sync(); s1 = time.perf_counter(); torch.cuda.synchronize(); s2 = time.perf_counter()
            syn.append(s1 - s0); tsyn.append(s2 - s1)
        us = lambda v: f"{np.median(v) * 1e6:8.1f} us"
        print(f"{a.config}, K = {K}: enqueue {us(enq)}; region {us(region)} = {np.median(region) / K * 1e6:.2f} us/step; "
              f"device {us(dev)} = {np.median(dev) / K * 1e6:.2f} us/step; idle rb_sync {us(syn)}; idle torch sync {us(tsyn)}")


if __name__ == "__main__":
    main()
