"""Diagnostic: per-phase cycle stamps of the step kernel in C4's pile-up
phase (RB_STAMPS build, e.g. `make -C rigidbody-simulation_amd/csrc
OUT=../../build/stamps.so OBJDIR=build_stamps EXTRA=-DRB_STAMPS=1`).
C4 (65,536 spheres on the incline) is stepped from t = 0 to `--warm` steps
(max_partners 32, the bench's c4 world), then one recorded launch; prints
the phase spans of the slowest blocks and the median, and how many blocks
are slow.  Phases (rb_kernels.hip STAMP): 0 start, 1 own loads issued,
8 heads back, 9 head candidates tested, 10 rare path done, 2 search done,
3 forces, 4 solves done, 5 claim + snapshot store, 6 end."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "stamps.so"))
    ap.add_argument("--warm", type=int, default=700)
    ap.add_argument("--config", default="c4")
    a = ap.parse_args()
    from rbhip import _lib, scenes
    import rbhip.world as W
    L = _lib.load(a.lib)
    L.rb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    sc = scenes.make(a.config)
    nb = (sc.n + 63) // 64
    with W.World(sc, max_partners=32) as w:
        w.step(a.warm)
        w.record_contacts(True)
        w.step(1)
        cnt, par, kin, _ = w.contacts()
        buf = np.zeros((nb, 16), np.uint64)
        L.rb_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb)
    b = buf.astype(np.int64)
    tot = b[:, 6] - b[:, 0]
    order = np.argsort(tot)[::-1]
    phases = [(0, 1, "own loads"), (1, 8, "heads"), (8, 9, "head cands"), (9, 10, "rare path"),
              (10, 2, "search tail"), (2, 3, "forces"), (3, 4, "solves"), (4, 5, "claim+snap"), (5, 6, "quat+store")]
    nss = np.bincount(np.repeat(np.arange(sc.n), cnt), weights=(kin == 16), minlength=sc.n)
    per_block = nss.reshape(-1, 64).max(1) if sc.n % 64 == 0 else None
    print(f"{a.config} after {a.warm} steps: kernel span {int(b[:, 6].max() - b[:, 0].min())} cycles; "
          f"block total median {int(np.median(tot))} p99 {int(np.percentile(tot, 99))} max {int(tot.max())}; "
          f"blocks over 2x median {int((tot > 2 * np.median(tot)).sum())} of {nb}; "
          f"sphere partners per body max {int(nss.max())} mean {nss.mean():.2f}")
    # s_memrealtime (100 MHz, one clock for the chip) at the first and last
    # stamp: when blocks start and end relative to the first start, in us
    st, en = (b[:, 12] - b[:, 12].min()) / 100.0, (b[:, 13] - b[:, 12].min()) / 100.0
    q = lambda a: " ".join(f"{np.percentile(a, x):.2f}" for x in (0, 10, 50, 90, 99, 100))
    print(f"  block start us (p0 p10 p50 p90 p99 max): {q(st)}")
    print(f"  block end   us (p0 p10 p50 p90 p99 max): {q(en)}")
    print(f"  block length us (median): {np.median(en - st):.2f}; cycles per us (memtime / realtime): "
          f"{np.median(tot / np.maximum(en - st, 1e-3)):.0f}")
    for label, rows in (("median", None), ("slowest", order[:5])):
        for lo, hi, nm in phases:
            d = b[:, hi] - b[:, lo]
            if rows is None:
                print(f"  {label:8s} {nm:12s} {int(np.median(d)):8d}")
            else:
                print(f"  {label:8s} {nm:12s} " + " ".join(f"{int(d[r]):8d}" for r in rows))
    if per_block is not None:
        print("  slowest blocks' max sphere partners:", [int(per_block[r]) for r in order[:5]])


if __name__ == "__main__":
    main()
