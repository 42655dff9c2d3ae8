"""Diagnostic: time the step kernel (graph replay, or GRAPH=0: HIP events per launch) for several
builds (VARIANTS: ";"-separated extra compiler flags) and runtime settings
(ENVS: ";"-separated entries of ","-separated NAME=VALUE applied before each world is created), over
several flat-sphere scene sizes, interleaved in one process.  Not part of the
product; results go to stdout."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
CSRC = os.path.join(ROOT, "rigidbody-simulation_amd", "csrc")
variants = os.environ.get("VARIANTS", "").split(";")
envs = os.environ.get("ENVS", "").split(";")
sizes = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("SIZES", "64x64,256x256,1024x1024").split(",")]
paths = {}
# PREBUILT=1: use build/ablate<k>.so made beforehand (BUILD_ONLY=1 makes them
# and exits), so the GPU box does not compile
os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
for k, v in enumerate(variants if not os.environ.get("LIBS") else []):
    out = os.path.join(ROOT, "build", f"ablate{k}.so")
    if os.environ.get("PREBUILT") != "1":
        subprocess.run(f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off "
                       f"{v} -o {out} rb_kernels.hip rb_balls.hip rb_p2p.hip rb_capi.hip", shell=True,
                       check=True, cwd=CSRC)
    paths[v] = out
if os.environ.get("BUILD_ONLY") == "1":
    sys.exit(0)
# LIBS: ";"-separated library paths to compare instead of VARIANTS builds
if os.environ.get("LIBS"):
    variants = os.environ["LIBS"].split(";")
    paths = {v: os.path.join(ROOT, v) for v in variants}
import torch  # noqa: E402  (initialise torch's HIP context before the library's)
torch.cuda.init()
from rbhip import _lib, scenes
import rbhip.world as W


def run_one(sc):
    """Average step-kernel time (ms) of one world of scene sc."""
    with W.World(sc) as w:
        if os.environ.get("GRAPH", "1") == "1":
            # K graph-replayed steps between HIP events on torch's stream
            w.set_stream(torch.cuda.current_stream().cuda_stream)
            w.step(int(os.environ.get("WARM", "60")))
            w.step(200)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); w.step(200); e1.record(); torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 200
        w.step(60)
        w.kernel_timing(True)
        w.step(100)
        return w.kernel_timing(False)[0]


res = {}
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for v in variants:
        _lib._lib = None
        _lib.load(paths[v])
        for env in envs:
            # an ENVS entry may set several variables: NAME=VALUE,NAME=VALUE
            assigns = [a.split("=") for a in env.split(",")] if env else []
            for name, val in assigns:
                os.environ[name] = val
            for nx, ny in sizes:
                kind = os.environ.get("SCENE", "flat")
                sc = (scenes.incline_spheres(nx, ny, seed=0) if kind == "incline"
                      else scenes.incline_cubes(nx, ny, seed=0) if kind == "cubes"
                      else scenes.flat_spheres(nx, ny, seed=0))
                try:
                    avg = run_one(sc)
                except _lib.RbError as e:        # a diagnostic build may produce garbage
                    print(f"{v} {env} N={nx * ny}: {e}", flush=True)
                    continue
                res.setdefault((v, env, nx * ny), []).append(avg)
            for name, _ in assigns:
                del os.environ[name]
for (v, env, n), t in sorted(res.items(), key=lambda kv: (kv[0][2], kv[0][0], kv[0][1])):
    print(f"N={n:8d} {v:20s} {env:34s} kernel ms {min(t):.4f} -> {n / min(t) / 1e6:7.2f} G body-steps/s")
