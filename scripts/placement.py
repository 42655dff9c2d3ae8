"""Diagnostic: where the step kernel's waves run (RB_STAMPS build: block 0..N's
first wave records HW_ID and XCC_ID).  Counts waves per (XCC, SE, SH, CU,
SIMD): more than one wave on a SIMD while others idle would double that
SIMD's VALU time.  Not part of the product."""
import ctypes, os, sys
from collections import Counter
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
from rbhip import _lib, scenes
import rbhip.world as W
L = _lib.load(os.environ.get("STAMP_LIB", os.path.join(ROOT, "build", "stamp.so")))
L.rb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
for nx, ny in [(256, 256), (256, 128), (128, 64)]:
    sc = scenes.flat_spheres(nx, ny, seed=0)
    G = 8 if sc.n <= 20480 else 1
    nb = (sc.n * G + 63) // 64
    with W.World(sc) as w:
        w.step(60)
        w.step(1)
        buf = np.zeros((nb, 16), np.uint64)
        L.rb_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb)
    hw = buf[:, 15].astype(np.int64)
    xcc = buf[:, 14].astype(np.int64) & 0xF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    per_simd = Counter(zip(xcc, se, sh, cu, simd))
    per_cu = Counter(zip(xcc, se, sh, cu))
    print(f"N={sc.n}: {nb} blocks on {len(per_cu)} CUs, {len(per_simd)} SIMDs; "
          f"waves per SIMD {sorted(Counter(per_simd.values()).items())}; blocks per CU {sorted(Counter(per_cu.values()).items())}; "
          f"per XCC {sorted(Counter(xcc.tolist()).items())}", flush=True)
