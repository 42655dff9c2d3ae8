"""Benchmark: body-steps/s of the rigid-body hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--dtype f64]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

Workload: C3 (BASELINE.json configs[2]) in fp64 — 65,536 spheres r 0.1 on
flat ground, e 0.8, mu 0.3, dt 0.01, seeded synthetic initial conditions
(rbhip.scenes.flat_spheres).  That is the scene the north-star
target is quoted on ("≥1M body-steps/sec on a 65 536-sphere scene at
1×MI355X with ≥3.5× at 8 GPUs"); `--config c2` runs configs[1] (4,096
spheres), c4 / c5 the incline and cube scenes.  A "step" is one reference
step of the whole scene (contacts, impulses, integration).  With N ranks
the scene is N such 256x256 patches side by side on one shared ground (weak
scaling: 65,536 bodies per GPU); rank r owns patch r, and the ranks exchange
positions inside the library every step (peer-to-peer over xGMI: halo
pushes for shards this large).

N > 1 is validated: after the warmup and again after the timed region, every
rank's bodies must be bit-identical to one World of the whole scene stepped
the same number of steps on rank 0's GPU.  A transport that fails the first
check (or times out) is replaced by the next (p2p halo -> p2p full reads
-> rccl); one that fails the second makes the run exit non-zero instead of
printing a number.

value = total bodies x K / (max over ranks of the timed region), with the
state resident in HBM.  roofline: algorithmic HBM bytes of the step kernel
(248 B per sphere body-step in fp64) x owned bodies / its
average launch duration.  One rank: HIP events recorded on the world's
stream (torch's current stream) around the timed region, which is exactly K
graph-replayed step-kernel launches, / K.  Several ranks: an event pair
around each step-kernel launch over a second run of K steps.
cpu_baseline: the oracle (C restatement of the reference arithmetic) on rank 0
at N=1 over the full single-GPU scene for --cpu-steps steps from t = 0, on
the GPU's host-core share (OMP_NUM_THREADS, 16 on the GPU box) and on one
core.
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
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=200)
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


class SingleWorldCheck:
    """N > 1: compare every rank's bodies, bit for bit, with one World of the
    whole scene stepped on rank 0's GPU (collective: every rank calls it
    with the same step count)."""

    def __init__(self, scene, dtype, device, rank, P):
        self.scene, self.dtype, self.device, self.rank, self.P = scene, dtype, device, rank, P
        self.ref, self.done = None, 0

    def __call__(self, sw, steps_total) -> bool:
        import numpy as np
        import torch
        import torch.distributed as dist
        ok = 1
        try:
            sw.sync()
        except Exception as e:          # an exchange timeout or a device error
            print(f"bench: rank {self.rank}: {e}", file=sys.stderr, flush=True)
            ok = 0
        dev = f"cuda:{self.device}" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([ok], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if not int(t.item()):
            return False
        q, v = sw.gather_state()
        same = 1
        if self.rank == 0:
            import rbhip
            if self.ref is None:
                self.ref = rbhip.World(self.scene, device=self.device, dtype=self.dtype)
            self.ref.step(steps_total - self.done)
            self.done = steps_total
            q1, v1 = self.ref.get_state()
            same = int(np.array_equal(q, q1) and np.array_equal(v, v1))
            if not same:
                bad = np.flatnonzero(~(np.all(q == q1, axis=1) & np.all(v == v1, axis=1)))
                print(f"bench: {bad.size} bodies differ from the single World after {steps_total} steps "
                      f"(first ids {bad[:8].tolist()})", file=sys.stderr, flush=True)
        t = torch.tensor([same], device=dev)
        dist.broadcast(t, src=0)
        return bool(int(t.item()))


def step_kernel_name(n_owned: int) -> str:
    """The step kernel form the library picks for n_owned bodies
    (rb_capi.hip launch_one: coop <= 20,480 < wide <= 65,536 < one)."""
    if n_owned <= int(os.environ.get("RBHIP_COOP_MAX_BODIES", "20480")):
        return "rb::step_kernel_coop"
    if n_owned <= int(os.environ.get("RBHIP_WIDE_MAX_BODIES", "65536")):
        return "rb::step_kernel_wide"
    return "rb::step_kernel_one"


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
    check = SingleWorldCheck(scene, args.dtype, device, rank, P) if P > 1 else None
    # (transport, halo): the library's default (peer-to-peer, halo for large
    # shards), then peer-to-peer full reads, then RCCL
    transports = [(None, "auto"), ("p2p", False), ("rccl", "auto")] if P > 1 else [(None, "auto")]
    for k, (tr, halo) in enumerate(transports):
        sw = ShardedWorld(scene, dtype=args.dtype, device=device, transport=tr, halo=halo)
        # warmup (also builds and caches the K-step graphs)
        sw.step(args.warmup)
        if check is None or check(sw, args.warmup):
            break
        name = sw.transport + (" (halo)" if sw.halo else "")
        sw.world.close()
        if k + 1 == len(transports):
            raise SystemExit(f"bench: every transport failed validation (last: {name})")
        if rank == 0:
            print(f"bench: {name} exchange failed validation; falling back to {transports[k + 1][0]}"
                  f"{'' if transports[k + 1][1] else ' (full reads)'}", file=sys.stderr, flush=True)
    w = sw.world
    sw.sync()

    def barrier_sync():
        torch.cuda.synchronize()
        if P > 1:
            dist.barrier()
        torch.cuda.synchronize()

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
        if not check(sw, args.warmup + 2 * args.steps):
            raise SystemExit("bench: the sharded run diverged from the single-World run during the timed steps")

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
                   "parallelism": f"body-range shards x{P}" + (
                       f", {sw.transport}{' halo' if sw.halo else ''} position exchange, graph-replayed" if P > 1 else ""),
                   "dt": scene.dt, "restitution": scene.restitution, "friction": scene.friction,
                   **({"validated": f"bit-identical to one World of the whole scene after {args.warmup} and "
                                    f"{args.warmup + 2 * args.steps} steps"} if P > 1 else {})},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": step_kernel_name(w.n_owned),
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
