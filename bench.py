"""Benchmark: body-steps/s of the rigid-body hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--dtype f64]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

Workload (BASELINE.json configs[1], the metric's single-GPU config): C2 —
4,096 spheres r 0.1 on flat ground, e 0.8, mu 0.3, dt 0.01, fp64, seeded
synthetic initial conditions (rbhip.scenes.flat_spheres).  A "step" is one
reference step of the whole scene (contacts, impulses, integration).  With
N ranks the scene is N such 64x64 patches side by side on one shared ground
(weak scaling: 4,096 bodies per GPU); rank r owns patch r and the ranks
all-gather positions over RCCL every step.

value = total bodies x K / (max over ranks of the timed region), with the
state resident in HBM.  roofline: algorithmic HBM bytes of the step kernel
(248 B per sphere body-step in fp64) x owned bodies / its
average launch duration.  One rank: HIP events recorded on the world's
stream (torch's current stream) around the timed region, which is exactly K
graph-replayed step-kernel launches, / K.  Several ranks: an event pair
around each step-kernel launch over a second run of K steps.
cpu_baseline: the oracle (C restatement of the reference arithmetic) on rank 0
at N=1 over the full C2 scene for 2,000 steps, on the GPU's host-core share
(OMP_NUM_THREADS, 16 on the GPU box) and on one core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=2000)
    return ap.parse_args()


def make_scene(cfg: str, P: int):
    from rbhip import scenes
    if cfg == "c2":
        return scenes.tiled(scenes.flat_spheres, P, 64, 64, seed=0), "c2: 4096 spheres/GPU, flat ground"
    if cfg == "c3":
        return scenes.tiled(scenes.flat_spheres, P, 256, 256, seed=0), "c3: 65536 spheres/GPU, flat ground"
    if cfg == "c4":
        return scenes.tiled(scenes.incline_spheres, P, 256, 256, seed=0), "c4: 65536 spheres/GPU, 0.7 rad incline"
    return scenes.tiled(scenes.incline_cubes, P, 128, 128, seed=0), "c5: 16384 cubes/GPU, 0.7 rad incline"


def cpu_baseline(cfg: str, steps: int):
    """Oracle (C restatement of the reference arithmetic) on the single-GPU
    scene, on all of this GPU's host-core share (OpenMP over bodies) and on
    one core; returns the cpu_baseline dict."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    sc, _ = make_scene(cfg, 1)
    osc = O.OracleScene(sc)
    cores = int(os.environ.get("OMP_NUM_THREADS", "16"))
    rates = {}
    for th in (cores, 1):
        O.set_threads(th)
        t0 = time.perf_counter()
        O.step(osc, sc.qpos0, sc.qvel0, steps)
        rates[th] = (sc.n * steps / (time.perf_counter() - t0), time.perf_counter() - t0)
    return {"value": rates[cores][0], "unit": "body-steps/s", "cores": cores, "kind": "port",
            "value_1core": rates[1][0],
            "sample": f"oracle/rb_oracle.c (C restatement of collision.py/physics_utils.py/"
                      f"multi_sphere_bounce.py arithmetic, bit-identical to the GPU path) on the full {cfg} "
                      f"scene, {sc.n} bodies x {steps} steps from t=0: {cores} OpenMP threads "
                      f"{rates[cores][1]:.1f} s, 1 thread {rates[1][1]:.1f} s"}


def traffic_from_profiles(cfg: str, dtype: str):
    """HBM bytes per step-kernel launch from the committed PMC summary
    (profiles/pmc_traffic.json, written by profiles/collect_pmc.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(f"{cfg}_{dtype}", {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    P = max(world_size, 1)
    # RBHIP_BENCH_BACKEND=gloo (with RBHIP_SHARD_TRANSPORT=p2p) rehearses the
    # multi-rank path with several ranks sharing the visible GPUs; its
    # numbers are not measurements
    backend = os.environ.get("RBHIP_BENCH_BACKEND", "nccl")
    device = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(device)
    if P > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
        else:
            dist.init_process_group(backend)
    from rbhip.shard import ShardedWorld

    scene, desc = make_scene(args.config, P)
    sw = ShardedWorld(scene, dtype=args.dtype, device=device)
    w = sw.world

    def barrier_sync():
        torch.cuda.synchronize()
        if P > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # warmup (also builds and caches the K-step graphs)
    sw.step(args.warmup)
    sw.sync()
    sw.step(args.steps)              # capture the K-step graph outside the timed region
    sw.sync()
    barrier_sync()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()                      # the library enqueues on torch's current stream
    sw.step(args.steps)
    ev1.record()
    sw.sync()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1)
    if P > 1:
        t = torch.tensor([elapsed], device=f"cuda:{device}" if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # roofline: average step-kernel launch duration.  One rank: the timed
    # region is exactly K back-to-back step-kernel launches (graph replay),
    # so HIP events around it / K.  Several ranks: a step also runs the
    # exchange, so time each step-kernel launch with its own event pair.
    if P == 1:
        avg_ms, launches, timing = region_ms / args.steps, args.steps, "HIP events around the timed region / K"
    else:
        w.kernel_timing(True)
        sw.step(args.steps)
        sw.sync()
        avg_ms, launches = w.kernel_timing(False)
        timing = "HIP event pair around each step-kernel launch (second run of K steps)"
    bytes_per_launch = w.bytes_per_body_step * w.n_owned
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = traffic_from_profiles(args.config, args.dtype)

    value = scene.n * args.steps / elapsed
    line = {
        "metric": "body-steps/sec (N spheres x steps/s)",
        "value": value,
        "unit": "body-steps/s",
        "n_gpus": P,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded rbhip.scenes, SURVEY 8d)",
        "config": {"workload": desc, "bodies_total": scene.n, "bodies_per_gpu": w.n_owned,
                   "parallelism": f"body-range shards x{P}" + (f", {sw.transport} position exchange, graph-replayed" if P > 1 else ""),
                   "dt": scene.dt, "restitution": scene.restitution, "friction": scene.friction},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("rb::step_kernel_coop" if w.n_owned <= int(os.environ.get("RBHIP_COOP_MAX_BODIES", "32768"))
                                else "rb::step_kernel_one"),
                     "avg_launch_ms": avg_ms, "launches_timed": launches,
                     "timing": timing,
                     "algorithmic_bytes_per_launch": bytes_per_launch},
    }
    if rank == 0 and P == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_steps)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if P > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
