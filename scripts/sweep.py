"""Throughput sweep (1 GPU): body-steps/s and algorithmic HBM GB/s of the
step kernel for the BASELINE configs and large flat scenes.  Prints a
markdown table (used for DESIGN.md).  Timing: HIP events around K
graph-replayed steps; `form` is the step form that ran (rbhip stats: 5 is
the cell-ordered tile form, the default above 65,536 bodies; RBHIP_TILE=0
for the hashed-cell forms throughout)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
import torch
import rbhip
from rbhip import scenes

cases = [("c2", lambda: scenes.make("c2")), ("c3", lambda: scenes.make("c3")), ("c4", lambda: scenes.make("c4")),
         ("c5", lambda: scenes.make("c5")), ("flat 272x272", lambda: scenes.flat_spheres(272, 272)),
         ("flat 362x362", lambda: scenes.flat_spheres(362, 362)),
         ("flat 512x512", lambda: scenes.flat_spheres(512, 512)),
         ("flat 1024x1024", lambda: scenes.flat_spheres(1024, 1024)),
         ("flat 2048x2048", lambda: scenes.flat_spheres(2048, 2048))]
only = os.environ.get("ONLY")
print("| scene | N | dtype | form | steps | ms/step | body-steps/s | algorithmic GB/s | frac of 8 TB/s |")
print("|---|---|---|---|---|---|---|---|---|")
for name, mk in cases:
    if only and name not in only.split(","):
        continue
    sc = mk()
    for dt in ("f64", "f32"):
        K = 200 if sc.n <= 300000 else 50
        with rbhip.World(sc, dtype=dt) as w:
            w.set_stream(torch.cuda.current_stream().cuda_stream)
            w.step(60)
            w.step(K)          # graph capture
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); w.step_async(K); e1.record(); w.sync()
            ms = e0.elapsed_time(e1) / K
            gbs = w.bytes_per_body_step * sc.n / (ms * 1e-3) / 1e9
            form = w.stats()["form"]
        print(f"| {name} | {sc.n} | {dt} | {form} | {K} | {ms:.4f} | {sc.n / ms * 1e3:.3e} | {gbs:.0f} | {gbs / 8000:.3f} |", flush=True)
