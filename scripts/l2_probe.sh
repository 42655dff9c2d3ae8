#!/bin/bash
# Diagnostic: scripts/l2_probe.hip (L2 contents across a kernel boundary).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/l2
for s in 0 1; do
  timeout -k 10 60 build/l2_probe $s 200
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/l2/s$s -o run -- build/l2_probe $s 40 > /dev/null 2>&1
  python3 - gpurun_out/l2/s$s <<'PY'
import csv, glob, sys, collections
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
acc = collections.defaultdict(list)
for r in rows:
    acc[(r["Kernel_Name"][:12], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"  {k:12s} {c:20s} mean {sum(v)/len(v):12.0f} over {len(v)} dispatches")
PY
done
