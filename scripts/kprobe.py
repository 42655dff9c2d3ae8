"""Diagnostic driver for rocprofv3 --pmc runs: run the step kernel of one
library build (LIB env, default in-tree) on a flat-sphere scene of NX*NY
bodies for STEPS steps.  Not part of the product."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
from rbhip import _lib, scenes
import rbhip.world as W
lib = os.environ.get("LIB")
if lib:
    _lib.load(lib)
nx = int(os.environ.get("NX", "1024")); ny = int(os.environ.get("NY", "1024"))
cfg = os.environ.get("CFG", "flat")
sc = scenes.flat_spheres(nx, ny, seed=0) if cfg == "flat" else scenes.incline_spheres(nx, ny, seed=0)
with W.World(sc, dtype=os.environ.get("DTYPE", "f64")) as w:
    w.step(int(os.environ.get("WARM", "60")))
    w.step(int(os.environ.get("STEPS", "20")))
print("ok")
