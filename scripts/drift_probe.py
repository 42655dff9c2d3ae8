"""C4 drift: step a world to 2,000 steps in chunks, printing after each the
wall clock and the layout counters (refits, table growth)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
import rbhip  # noqa: E402
from rbhip import scenes  # noqa: E402

chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 200
sc = scenes.make("c4")
with rbhip.World(sc, max_partners=32) as w:
    for c in range(0, 2000, chunk):
        t0 = time.perf_counter()
        try:
            w.step(chunk)
        except rbhip.RbError as e:
            print(f"steps {c}-{c + chunk}: {e}", flush=True)
            break
        st = w.stats()
        print(f"steps {c + 1}-{c + chunk}: {1e6 * (time.perf_counter() - t0) / chunk:.1f} us/step, refits {st['refits']}"
              f" grows {st['table_grows']} buckets {st['buckets']}", flush=True)
