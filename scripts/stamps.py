"""Diagnostic: per-phase cycle stamps of the step kernel (RB_STAMPS build).
Phases: 0 start | 1 after table clear | 2 after broadphase search |
3 after state load + gravity | 4 after contact solves | 5 after position
store + insert | 6 end.  Prints the median / p90 over workgroups."""
import ctypes, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
CSRC = os.path.join(ROOT, "rigidbody-simulation_amd", "csrc")
extra = os.environ.get("EXTRA_FLAGS", "")
# a prebuilt stamps library (built on the CPU host, shipped with the tree) or build one here
LIB = os.environ.get("STAMP_LIB", "/tmp/libstamp.so")
if not os.path.exists(LIB):
    subprocess.run(f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off "
                   f"-DRB_STAMPS=1 {extra} -o {LIB} rb_kernels.hip rb_balls.hip rb_p2p.hip rb_capi.hip", shell=True,
                   check=True, cwd=CSRC)
from rbhip import _lib, scenes
import rbhip.world as W
L = _lib.load(LIB)
L.rb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
sizes = [(64, 64, 300), (256, 256, 60), (1024, 1024, 60)]
if os.environ.get("STAMP_SIZES"):        # e.g. "64x64,128x64,256x256"
    sizes = [(int(a), int(b), 300) for a, b in (t.split("x") for t in os.environ["STAMP_SIZES"].split(","))]
for nx, ny, warm in sizes:
    if nx * ny * (8 if nx * ny <= 20480 else 1) > 64 * (1 << 16): continue
    sc = scenes.flat_spheres(nx, ny, seed=0)
    G = 8 if sc.n <= int(os.environ.get("RBHIP_COOP_MAX_BODIES", "20480")) else 1
    nb = (sc.n * G + 63) // 64
    with W.World(sc) as w:
        w.step(warm)
        w.step(1)
        buf = np.zeros((nb, 16), np.uint64)
        L.rb_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb)
    d = np.diff(buf[:, :7].astype(np.int64), axis=1)
    tot = (buf[:, 6].astype(np.int64) - buf[:, 0].astype(np.int64))
    span = buf[:, 6].max() - buf[:, 0].min()
    print(f"N={sc.n}: kernel span {int(span)} cyc; per-block total median {int(np.median(tot))} p90 {int(np.percentile(tot, 90))}")
    names = ["clear", "search", "load+grav", "solves", "pos+insert", "quat+store"]
    for k, nm in enumerate(names):
        print(f"   {nm:12s} median {int(np.median(d[:, k])):8d}  p90 {int(np.percentile(d[:, k], 90)):8d}")
    if G == 1:  # one-lane search sub-phases
        sub = [(1, 8, "snap+heads issue"), (8, 9, "heads+batch1"), (9, 10, "later batches"), (10, 2, "tail")]
        for a, b_, nm in sub:
            dd = buf[:, b_].astype(np.int64) - buf[:, a].astype(np.int64)
            print(f"     {nm:16s} median {int(np.median(dd)):8d}  p90 {int(np.percentile(dd, 90)):8d}")
    if G > 1:   # cooperative search sub-phases
        sub = [(1, 8, "snap+cell"), (8, 9, "invI"), (9, 10, "bucket+test"), (10, 11, "place+sync"), (11, 2, "sort+sync")]
        for a, b_, nm in sub:
            dd = buf[:, b_].astype(np.int64) - buf[:, a].astype(np.int64)
            print(f"     {nm:12s} median {int(np.median(dd)):8d}  p90 {int(np.percentile(dd, 90)):8d}")
