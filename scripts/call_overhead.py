"""Diagnostic: where the driver's bench shape (K = 20 graph-replayed C3 steps
per timed call) spends the wall time that is not step-kernel time.  Repeats
the bench's N = 1 timed region (event, rb_step_async, event, rb_sync,
torch.cuda.synchronize) and times each host call; prints medians.  Not part
of the product.

    python scripts/call_overhead.py [--K 20] [--reps 40]   (RBHIP_GRAPH_MIN_STEPS: eager below)
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from rbhip import _lib
    if a.lib:
        _lib.load(a.lib)
    import rbhip
    from rbhip import scenes
    with rbhip.World(scenes.make("c3")) as w:
        w.set_stream(torch.cuda.current_stream().cuda_stream)
        w.step(a.K)
        w.sync()
        rows = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            t1 = time.perf_counter()
            w.step_async(a.K)
            t2 = time.perf_counter()
            e1.record()
            t3 = time.perf_counter()
            w.sync()
            t4 = time.perf_counter()
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0, e0.elapsed_time(e1) * 1e-3))
        med = [statistics.median(r[k] for r in rows) * 1e6 for k in range(7)]
        print(f"{os.path.basename(a.lib or 'librbhip.so')} K={a.K} graph_min={os.environ.get('RBHIP_GRAPH_MIN_STEPS', 'default')}: median us: ev0.record {med[0]:.1f}, rb_step_async {med[1]:.1f}, ev1.record {med[2]:.1f}, "
              f"rb_sync {med[3]:.1f}, torch sync {med[4]:.1f}; wall {med[5]:.1f} ({med[5] / a.K:.2f} per step), "
              f"events {med[6]:.1f} ({med[6] / a.K:.2f} per step)", flush=True)


if __name__ == "__main__":
    main()
