"""Diagnostic for DESIGN §6 (strong-scaling budget): the step kernel's own
time on each rank of a P-way body-range sharding of one scene (CFG, default
c3), P = 1, 2, 4, 8, all ranks in this process on one GPU, serialised on
one stream.  The ranks exchange their fresh slices with device copies
between rb_shard_step and rb_shard_exchange_done (the host transport's
role), so every kernel sees the true scene; the step-kernel launches are
timed with HIP events.  Prints the slowest rank's average (the strong-
scaling critical path without the exchange).  Not part of the product."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
import numpy as np
import torch
torch.cuda.init()
import rbhip
from rbhip import scenes
from rbhip.shard import wrap_gpos

sc = scenes.make(os.environ.get("CFG", "c3"))
WARM, K = int(os.environ.get("WARM", "450")), int(os.environ.get("K", "200"))
stream = torch.cuda.current_stream().cuda_stream
print(f"| P | owned bodies per rank | form | step kernel us, slowest rank (steps {WARM + 1}-{WARM + K}) | mean over ranks |")
print("|---|---|---|---|---|")
for P in [int(v) for v in os.environ.get("PS", "1,2,4,8").split(",")]:
    ws = [rbhip.World(sc, rank=r, world_size=P) for r in range(P)]
    for w in ws:
        w.set_stream(stream)

    def step_all():
        for w in ws:
            w.shard_step()
        if P > 1:
            views = [wrap_gpos(w, torch) for w in ws]
            S = views[0][1]
            for r in range(P):
                src = views[r][0][r * S:(r + 1) * S]
                for q in range(P):
                    if q != r:
                        views[q][0][r * S:(r + 1) * S].copy_(src)
        for w in ws:
            w.shard_exchange_done()

    for _ in range(WARM):
        step_all()
    for w in ws:
        w.kernel_timing(True)
    for _ in range(K):
        step_all()
    us = [w.kernel_timing(False)[0] * 1e3 for w in ws]
    n = ws[0].n_owned
    form = "coop" if n <= 20480 else "wide" if n <= 65536 else "one"
    print(f"| {P} | {n} | {form} | {max(us):.2f} | {np.mean(us):.2f} |", flush=True)
    for w in ws:
        w.close()
