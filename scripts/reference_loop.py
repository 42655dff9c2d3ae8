"""The reference's own N-body step loop, timed on this container's CPU (the
"reference's NumPy/CPU loop" the north-star puts the GPU numbers next to).

Runs multi_sphere_bounce.py:42-92's body loop through the golden harness of
tests/golden/make_golden.py (`nbody_step`: the reference's own
compute_inertia_tensor_world, compute_collision_impulse_friction and
apply_impulse_friction from /root/reference/src/physics, line for line with
SURVEY D1/D2 fixed; contacts from the harness's restated mj_forward, since
MuJoCo is not installable offline) on configs[1] (C2: 4,096 spheres on flat
ground) for a fixed number of steps from t = 0, and writes body-steps/s with
the host's core count and CPU model to a JSON file.  The mj_forward stub's
own time is reported apart (MuJoCo would run that part in C).  The reference
cannot travel to the GPU box, so bench.py quotes the committed JSON.

    python scripts/reference_loop.py [--steps 20] [--config c2] [--out profiles/r05/reference_loop_c2.json]
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "reference_loop_c2.json"))
    a = ap.parse_args()
    import numpy as np
    import make_golden as G
    from rbhip import scenes
    G.install_stub()
    sys.path.insert(0, a.reference)
    from src.physics import collision as ref_collision
    from src.physics import physics_utils as ref_utils

    class Ref:
        compute_collision_impulse_friction = staticmethod(ref_collision.compute_collision_impulse_friction)
        apply_impulse_friction = staticmethod(ref_utils.apply_impulse_friction)
        compute_inertia_tensor_world = staticmethod(ref_collision.compute_inertia_tensor_world)

    sc = scenes.make(a.config)
    model = G.Model(sc)
    data = G.Data(model)
    # the harness's mj_forward, timed on its own
    fwd = G.mj_forward
    t_fwd = [0.0]

    def timed_forward(m, d):
        t0 = time.perf_counter()
        fwd(m, d)
        t_fwd[0] += time.perf_counter() - t0

    G.mj_forward = timed_forward
    t0 = time.perf_counter()
    for _ in range(a.steps):
        G.nbody_step(Ref, model, data, sc.dt, sc.restitution, sc.friction, sc.threshold, sc.normal_convention)
    el = time.perf_counter() - t0
    G.mj_forward = fwd
    body_steps = sc.n * a.steps
    rec = {
        "what": "the reference's own N-body step loop (multi_sphere_bounce.py:42-92 body loop, D1/D2 fixed) "
                "calling its collision.py / physics_utils.py functions, through tests/golden/make_golden.py's "
                "harness; contacts from the harness's restated mj_forward",
        "config": a.config, "bodies": sc.n, "steps": a.steps, "from_step": 0,
        "seconds": el, "mj_forward_seconds": t_fwd[0],
        "body_steps_per_s": body_steps / el,
        "body_steps_per_s_excluding_mj_forward": body_steps / max(el - t_fwd[0], 1e-12),
        "cores": 1, "nproc": os.cpu_count(), "cpu_model": cpu_model(),
        "python": platform.python_version(), "numpy": np.__version__,
        "script": "scripts/reference_loop.py",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
