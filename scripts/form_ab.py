"""A/B of the per-step kernel forms on one scene family (env knobs read at
world creation), graph-replayed steps 261-460 after a warm run.

    python scripts/form_ab.py [incline_cubes|flat_spheres] [sizes, e.g. 32,64,128]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
import rbhip  # noqa: E402
from rbhip import scenes  # noqa: E402

fam = sys.argv[1] if len(sys.argv) > 1 else "incline_cubes"
sizes = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "32,64,96,128").split(",")]
forms = {"help": {}, "coop": {"RBHIP_HELP_MAX_BODIES": "0"}, "wide": {"RBHIP_COOP_MAX_BODIES": "0"}}
for n in sizes:
    sc = getattr(scenes, fam)(n, n)
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for name, env in forms.items():
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            with rbhip.World(sc) as w:
                w.step(60)
                w.step(200)
                w.sync()
                t0 = time.perf_counter()
                w.step(200)
                us = (time.perf_counter() - t0) / 200 * 1e6
                form = rbhip._lib.FORM_NAMES.get(w.stats()["form"])
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            print(f"{fam} N={sc.n:6d} round {rnd} {name:5s} {form:28s} {us:7.2f} us/step", flush=True)
