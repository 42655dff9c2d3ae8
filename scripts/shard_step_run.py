"""Step P body-range shards of one scene in ONE process on one GPU (host-driven
exchange: shard_step, device copies of the position slices, exchange_done),
so that rocprofv3 PMC passes see exactly the step kernel each rank of a
P-GPU strong-scaling run launches (same shard size, same table contents).

    python scripts/shard_step_run.py --config c3 --P 8 [--warmup 50] [--steps 100] [--dtype f64]

Used by profiles/collect_pmc.py (keys <config>_<dtype>_p<P>).
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    import torch
    import rbhip
    from rbhip import scenes
    from rbhip.shard import wrap_gpos
    sc = scenes.make(a.config)
    worlds = [rbhip.World(sc, rank=r, world_size=a.P, dtype=a.dtype) for r in range(a.P)]
    for _ in range(a.warmup + a.steps):
        for w in worlds:
            w.shard_step()
        for w in worlds:
            w.sync()
        bufs = [wrap_gpos(w, torch) for w in worlds]
        n = bufs[0][1]
        for r, (buf, _) in enumerate(bufs):
            for o, (obuf, _) in enumerate(bufs):
                if o != r:
                    buf[o * n:(o + 1) * n].copy_(obuf[o * n:(o + 1) * n])
        torch.cuda.synchronize()
        for w in worlds:
            w.shard_exchange_done()
    st = worlds[0].stats()
    print(f"{a.config} P={a.P}: {a.warmup + a.steps} steps, {worlds[0].n_owned} bodies per rank, "
          f"kernel {rbhip._lib.FORM_NAMES.get(st['form'])}", flush=True)
    for w in worlds:
        w.close()


if __name__ == "__main__":
    main()
