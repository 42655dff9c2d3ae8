"""Derived PMC figures from scripts/pmc_r02.sh summaries:
wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY are
disjoint parts of SQ_WAVE_CYCLES, MI355X_MICROARCH.md PMC table), VALU-issue
share, L2 hit rate, HBM bytes per launch (FETCH_SIZE x2 upper / x1 lower
bound + WRITE_SIZE, KB units).  Usage: pmc_derive.py DIR [SIZE...]"""
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_r02"
sizes = sys.argv[2:] or ["64x64", "256x256", "1024x1024"]
print("| scene | waves | wait (s_waitcnt) | issue-stalled | issuing | VALU issuing | L2 hit | "
      "HBM bytes / launch (lower-upper) |")
print("|---|---|---|---|---|---|---|---|")
for sz in sizes:
    v = {}
    with open(os.path.join(root, f"summary_{sz}.txt")) as f:
        for line in f:
            k, x = line.split()
            v[k] = float(x)
    wc = v["SQ_WAVE_CYCLES"]
    hit = v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
    lo = (v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    hi = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    nx, ny = (int(t) for t in sz.split("x"))
    print(f"| flat {nx}x{ny} ({nx * ny} bodies) | {int(v['SQ_WAVES'])} | {v['SQ_WAIT_ANY'] / wc:.0%} | "
          f"{v['SQ_WAIT_INST_ANY'] / wc:.0%} | {v['SQ_ACTIVE_INST_ANY'] / wc:.0%} | "
          f"{v['SQ_ACTIVE_INST_VALU'] / wc:.0%} | {hit:.0%} | {lo / 1e6:.1f}-{hi / 1e6:.1f} MB |")
